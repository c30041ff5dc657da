"""K sweep of the bf16 GEMM (EP_BF16, O=512, M=240000): per-slice vs fixed per-tile cost."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pointcloud_style_transfer_amd import _hip  # noqa: E402

print("lib", os.environ.get("PCST_LIB", "default"))

M, O = 240000, int(os.environ.get("O", 512))
for K in (64, 128, 256, 512, 1024):
    A = torch.randn(M, K, device="cuda").bfloat16()
    W = torch.randn(O, K, device="cuda").bfloat16()
    for ep in (_hip.EP_BF16, _hip.EP_F32):
        f = lambda: _hip.gemm_ex(A, W, None, relu=True, epilogue=ep)  # noqa: E731
        f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            f()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 10 * 1e3
        print(f"K={K} ep={ep} us={us:.1f} TF={2*M*K*O/us/1e6:.0f}", flush=True)
