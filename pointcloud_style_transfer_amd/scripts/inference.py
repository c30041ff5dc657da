"""Inference entry point -- drop-in for the reference's `scripts/inference.py`
(`DiffusionInference`, `process_file`, same CLI flags `:176-185`).

Differences from the reference, all deliberate:
  * the checkpoint is read with `utils.checkpoint.safe_load` (weights_only=True with the
    pickled `config.config.Config` allow-listed) -- never an unpickling load;
  * there is no CPU fallback: the compute path is the HIP library, so a machine without a
    GPU, or `--device cpu`, raises instead of silently switching device (the reference
    falls back to the CPU at `:65`; BASELINE configs[0] is that CPU plumbing run, which this
    build serves on the GPU instead).
Keyword-only addition: `precision=` on DiffusionInference and the `--precision {fp32,bf16}`
flag (default "fp32", the checkpoint's parity mode; "bf16" runs the noise MLP on the bf16 MFMA
kernel -- the mode bench.py measures).
Kept quirks: EMA weights are copied into the trainable parameters only and the BN buffers
stay at their init values (Q9, `:98-113`); `.txt` delimiters differ for source (',') and
reference (' ') (`:151-152`).
"""
from __future__ import annotations

import argparse
import os
import sys
import time
from typing import Tuple

import numpy as np
import torch
import torch.nn as nn

from ..config.config import Config
from ..data.preprocessing import PointCloudPreprocessor
from ..models.diffusion_model import DiffusionProcess, PointCloudDiffusionModel
from ..utils.checkpoint import safe_load
from ..utils.logger import Logger


class PointCloudVisualizer:
    """`PointCloudVisualizer.visualize_comparison` (inference.py:20-60); needs matplotlib."""

    @staticmethod
    def visualize_comparison(original, reconstructed, reference, title="Comparison", save_path=None):
        try:
            import matplotlib

            matplotlib.use("Agg")
            import matplotlib.pyplot as plt
        except ImportError:
            print("Warning: matplotlib not available, skipping visualization")
            return
        fig = plt.figure(figsize=(18, 6))
        for k, (pts, name, cmap) in enumerate([(original, "Original (Simulation)", "viridis"),
                                               (reconstructed, "Transferred", "plasma"),
                                               (reference, "Reference (Real)", "coolwarm")]):
            ax = fig.add_subplot(1, 3, k + 1, projection="3d")
            if len(pts) > 8000:
                pts = pts[np.random.choice(len(pts), 8000, replace=False)]
            ax.scatter(pts[:, 0], pts[:, 1], pts[:, 2], c=pts[:, 2], cmap=cmap, s=0.5)
            ax.set_title(name)
            ax.view_init(elev=20, azim=120)
        plt.suptitle(title, fontsize=16)
        if save_path:
            plt.savefig(save_path, dpi=200, bbox_inches="tight")
            plt.close()
        else:
            plt.show()


class DiffusionInference:
    """`DiffusionInference` (inference.py:62-171)."""

    def __init__(self, checkpoint_path: str, device: str = "cuda", *, precision: str = None):
        if precision not in (None, "fp32", "bf16"):
            raise ValueError(f"precision must be 'fp32' or 'bf16', got {precision!r}")
        dev = torch.device(device)
        if dev.type != "cuda":
            raise RuntimeError(f"DiffusionInference runs on the MI355X HIP path only; device "
                               f"{device!r} is not supported (use 'cuda' or 'cuda:N')")
        if not torch.cuda.is_available():
            raise RuntimeError("DiffusionInference runs on the MI355X HIP path; no GPU is visible")
        self.device = dev
        parts = os.path.normpath(checkpoint_path).split(os.sep)
        experiment_name = parts[-2] if len(parts) >= 2 else "default_inference"
        self.logger = Logger(name="Inference", log_dir="logs/inference",
                             experiment_name=experiment_name, file_output=True)
        self.config, self.model = self.load_model(checkpoint_path)
        if precision is not None:  # None keeps the checkpoint's (a reference pickle: "fp32")
            self.config.precision = precision
        self.diffusion_process = DiffusionProcess(self.config, device=str(self.device))
        self.preprocessor = PointCloudPreprocessor(total_points=self.config.total_points,
                                                   global_points=self.config.global_points)

    def load_model(self, checkpoint_path: str) -> Tuple[Config, nn.Module]:
        if not os.path.exists(checkpoint_path):
            raise FileNotFoundError(f"Checkpoint not found: {checkpoint_path}")
        ckpt = safe_load(checkpoint_path, map_location="cpu")
        config = ckpt["config"]
        model = PointCloudDiffusionModel(config)
        ema = ckpt.get("ema_state_dict")
        if ema:
            shadow = ema["shadow_params"]
            trainable = [p for p in model.parameters() if p.requires_grad]
            if len(shadow) == len(trainable):
                with torch.no_grad():
                    for p, s in zip(trainable, shadow):
                        p.copy_(s)
            else:
                self.logger.error("EMA weights mismatch. Falling back to standard weights.")
                model.load_state_dict(ckpt["model_state_dict"])
        else:
            self.logger.warning("EMA weights not found, loading standard model weights.")
            model.load_state_dict(ckpt["model_state_dict"])
        model.to(self.device).eval()
        return config, model

    @torch.no_grad()
    def transfer_style_hierarchical(self, source_points: np.ndarray, reference_points: np.ndarray,
                                    num_steps: int, guidance_scale: float) -> np.ndarray:
        t0 = time.time()
        src_n, src_params = self.preprocessor.normalize_point_cloud(source_points)
        ref_n, _ = self.preprocessor.normalize_point_cloud(reference_points)
        src = torch.from_numpy(src_n).float().to(self.device).unsqueeze(0)
        ref = torch.from_numpy(ref_n).float().to(self.device).unsqueeze(0)
        out = self.diffusion_process.guided_sample_loop(model=self.model, source_points=src,
                                                        condition_points=ref,
                                                        num_inference_steps=num_steps,
                                                        guidance_scale=guidance_scale)
        res = self.preprocessor.denormalize_point_cloud(out.squeeze(0).cpu().numpy(), src_params)
        self.logger.info(f"Hierarchical style transfer finished in {time.time() - t0:.2f}s")
        return res

    def process_file(self, source_path: str, reference_path: str, output_path: str,
                     visualize: bool, num_steps: int, guidance_scale: float):
        sim = np.loadtxt(source_path, delimiter=",") if source_path.endswith(".txt") else np.load(source_path)
        real = np.loadtxt(reference_path, delimiter=" ") if reference_path.endswith(".txt") else np.load(reference_path)
        out = self.transfer_style_hierarchical(sim, real, num_steps, guidance_scale)
        d = os.path.dirname(output_path)
        if d:
            os.makedirs(d, exist_ok=True)
        np.save(output_path, out.astype(np.float32))
        self.logger.info(f"Transferred point cloud saved to: {output_path}")
        if visualize:
            PointCloudVisualizer.visualize_comparison(sim, out, real, "Hierarchical Style Transfer Result",
                                                      os.path.splitext(output_path)[0] + ".png")
        return out


def main(argv=None):
    p = argparse.ArgumentParser(description="Hierarchical Point Cloud Style Transfer Inference")
    p.add_argument("--checkpoint", type=str, required=True)
    p.add_argument("--source", type=str, required=True)
    p.add_argument("--reference", type=str, required=True)
    p.add_argument("--output", type=str, required=True)
    p.add_argument("--device", type=str, default="cuda")
    p.add_argument("--visualize", action="store_true")
    p.add_argument("--num_steps", type=int, default=50)
    p.add_argument("--guidance_scale", type=float, default=7.5)
    p.add_argument("--precision", choices=["fp32", "bf16"], default=None,
                   help="noise-MLP arithmetic: fp32 (exact, the default of a reference "
                        "checkpoint) or bf16 (the bf16 MFMA kernel bench.py measures)")
    args = p.parse_args(argv)
    try:
        eng = DiffusionInference(args.checkpoint, args.device, precision=args.precision)
        eng.process_file(args.source, args.reference, args.output, args.visualize,
                         args.num_steps, args.guidance_scale)
        print("Inference completed successfully!")
    except Exception as e:  # noqa: BLE001 -- same reporting as inference.py:193-197
        print(f"Inference failed: {e}")
        import traceback

        traceback.print_exc()
        sys.exit(1)


if __name__ == "__main__":
    main()
