"""Timing probe for the fused residual-block kernels (csrc/train_mlp.hip resblock2_kernel) built
with -DPCST_X_RB2_STAMPS=1: wave 0 of tiles 0 and ntiles / 2 writes s_memtime stamps over the
first h row of its tile (start, A rows landed, after chunks 0 / 1 / 7 / 15, end).  Prints the
launch time (HIP events) and the stamp deltas in core cycles, forward and backward.

    PCST_LIB=pointcloud_style_transfer_amd/libpcst_hip_v_stamps.so python tools/rb_probe.py
"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    from pointcloud_style_transfer_amd import _hip
    M = int(os.environ.get("RB_PROBE_M", 327680))
    half = torch.float16
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(M, 256, device=dev, generator=g).to(half)
    w1 = (torch.randn(512, 256, device=dev, generator=g) * 0.06).to(half)
    w2 = (torch.randn(256, 512, device=dev, generator=g) * 0.04).to(half)
    b1 = torch.randn(512, device=dev, generator=g) * 0.1
    b2 = torch.randn(256, device=dev, generator=g) * 0.1
    w2t, w1t = w2.t().contiguous(), w1.t().contiguous()
    hm = torch.relu(x.float()).to(half).repeat(1, 2)
    ntiles = (M + 255) // 256
    res = {"M": M}

    def stamps(hbuf):
        out = {}
        for t in (0, 1):  # work-groups 0 and 1 (persistent kernel: stamps at the work-group's first tile)
            s = hbuf[t * 256].view(torch.int64)[:15].tolist()
            # chunk 9: [12] start (chunk 8's barrier), [8] first product issued, [9] epilogue
            # done, [10] second product issued, [11] DMA waited, [13]... see the kernel
            c9 = {"first": s[8] - s[13], "epi": s[9] - s[8], "second": s[10] - s[9],
                  "vmwait": s[11] - s[10], "barrier": s[12] - s[11]}
            d = [s[i + 1] - s[i] for i in range(6)]
            out[f"tile{t}"] = {"wg": s[7], "prologue": d[0], "chunk0": d[1], "chunk1": d[2],
                               "chunks2_7": d[3], "chunks8_15": d[4], "epilogue": d[5],
                               "total": s[6] - s[0], "chunk9": c9, "epi_tile0": s[14] - s[5]}
        return out

    for name in ("fwd", "bwd"):
        times = []
        for it in range(6):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if name == "fwd":
                h, xo = _hip.resblock_fwd16(x, w1, b1, w2, b2, seed=7, p=0.1)
            else:
                # dz (the kernel's "h" output) carries the stamps
                h, xo, dd = _hip.resblock_bwd16(x, w2t, w1t, hm, x,
                                                seed=9, p=0.1, dropout_copy=True)
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) * 1e3)
        res[name] = {"us": [round(t, 1) for t in times[2:]], "stamps": stamps(h)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
