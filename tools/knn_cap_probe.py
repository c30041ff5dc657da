"""Experiment: the kNN build at many clouds (configs[4]'s per-GPU share: 32 clouds x 2 CFG rows,
120k points, 30k coarse rows) with the build launches capped at K work-groups per cloud row
(pcst_knn3_build's max_wg).  Prints the mean build and query time per call for each cap.
A development tool (tools/ only)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointcloud_style_transfer_amd import _hip  # noqa: E402


def main():
    rows, N, M = 64, 120000, 30000
    rng = np.random.default_rng(0)
    orig = torch.from_numpy(rng.standard_normal((rows, N, 3)).astype(np.float32)).cuda()
    idx = torch.from_numpy(np.stack([np.sort(rng.choice(N, M, replace=False))
                                     for _ in range(rows)]).astype(np.int64)).cuda()
    coarse = torch.from_numpy(rng.standard_normal((rows, M, 3)).astype(np.float32)).cuda()
    ws = _hip.knn_workspace(rows, N, M, device=orig.device)
    ref = None
    for per_row in (0, 4, 8, 16, 32, 64):
        cap = per_row * rows
        tb, tq = [], []
        for rep in range(6):
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record()
            h = _hip.knn3_build(orig, idx, ws, 0, cap)
            e1.record()
            out = _hip.knn3_query(coarse, h)
            e2.record()
            torch.cuda.synchronize()
            if rep:
                tb.append(e0.elapsed_time(e1))
                tq.append(e1.elapsed_time(e2))
        if ref is None:
            ref = out.clone()
        same = bool(torch.equal(out, ref))
        print(f"max_wg {per_row:3d}/row: build {1e3 * np.mean(tb):8.1f} us  query {1e3 * np.mean(tq):8.1f} us"
              f"  bit-identical {same}", flush=True)


if __name__ == "__main__":
    main()
