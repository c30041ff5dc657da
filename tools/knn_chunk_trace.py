"""Experiment: per-chunk timing of the rows-layout kNN query (an experiment build with
-DPCST_KNN_CHUNK_TRACE, loaded through PCST_LIB).

    make -C pointcloud_style_transfer_amd/csrc OUT=../libpcst_hip_v_ktrace.so BUILD=build_v_ktrace \\
        "XDEF=-DPCST_KNN_CHUNK_TRACE"
    PCST_LIB=$PWD/pointcloud_style_transfer_amd/libpcst_hip_v_ktrace.so python tools/knn_chunk_trace.py

One query of the bench's first step (noise cloud 120k, CFG x2, 30k device-drawn coarse points per
row): every chunk's (start, end) in 10 ns ticks, its wave, its lanes still open after pass 1,
whether pass 2 ran and its outliers.  Prints the launch span, chunk durations, start / end
distributions, chunks per wave, and durations split by pass 2 / outliers.
A development tool (tools/ only)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import knobs  # noqa: E402

knobs.apply()
from pointcloud_style_transfer_amd import _hip  # noqa: E402
from pointcloud_style_transfer_amd.synthetic import standard_normal  # noqa: E402


def rows_obound_offset(C, copies, N, M):
    """Byte offset of the rows workspace's obound array (knn.hip carve_knn_rows; white-box)."""
    B = C * copies
    Cmax = min(max(4096, 16 * M), 1024 * 4096 - 1)
    maxch = -(-N // 64) + 8 * (Cmax // 64) + 1
    off = 0
    for nbytes in (C * 64 * 72, C * 8 * 4, C * N * 16, C * N * 8, C * maxch * 8, B * N * 16,
                   B * N * 16, B * M * 16, B * N * 4):
        off = (off + 255) & ~255
        off += nbytes
    return (off + 255) & ~255


def main():
    dev = torch.device("cuda", 0)
    N, M = 120000, 30000
    x = torch.from_numpy(standard_normal(3000, (1, N, 3))).to(dev)
    ws = _hip.knn_rows_workspace(1, 2, N, M, dev)
    coarse = torch.randn(2, M, 3, device=dev)
    off = rows_obound_offset(1, 2, N, M)
    for rep in range(3):
        xc, xi = _hip.voxel_downsample(x, M, seed=rep, copies=2)
        h = _hip.knn3_rows_build(x, M, 2, ws)
        _hip.knn3_rows_refs(h, xi)
        for b in range(2):  # no stale records (chunks of known rows only are not recorded)
            o = off + (b * N + 4096) * 4
            ws[o:o + 16384 * 16].zero_()
        _hip.knn3_rows_query(coarse, h)
        torch.cuda.synchronize()
    st = _hip.knn_rows_stats(h)
    nch = st["chunks"][0]
    tr = []
    for b in range(2):
        o = off + (b * N + 4096) * 4
        tr.append(ws[o:o + nch * 16].view(torch.int32).view(nch, 4).cpu().numpy().astype(np.int64))
    tr = np.concatenate(tr)
    t0, t1 = tr[:, 0] & 0xFFFFFFFF, tr[:, 1] & 0xFFFFFFFF
    good = (t1 > t0) & (t1 - t0 < 100000)
    base = t0[good].min()
    s, e = (t0 - base) / 100.0, (t1 - base) / 100.0   # us
    d = e - s
    info = tr[:, 3]
    open1, p2, rows, vol = info & 0x7F, (info >> 7) & 1, (info >> 8) & 0xFF, info >> 16
    outl = tr[:, 2] >> 16
    wave = tr[:, 2] & 0xFFFF
    ok = good
    print(f"chunks {nch} per row, recorded {ok.sum()}, outliers {st['outliers']}")
    q = lambda a: " ".join(f"{np.percentile(a, p):.1f}" for p in (10, 50, 90, 99, 100))  # noqa: E731
    print("duration p10/50/90/99/max:", q(d[ok]))
    print("start    p10/50/90/99/max:", q(s[ok]))
    print("end      p10/50/90/99/max:", q(e[ok]))
    waves, cnt = np.unique(wave[ok], return_counts=True)
    print("waves used", len(waves), "chunks per wave histogram", np.bincount(cnt)[:8].tolist())
    print(f"pass 2 ran in {p2[ok].mean():.3f} of chunks; mean dur with / without pass 2: "
          f"{d[ok & (p2 > 0)].mean():.1f} / {d[ok & (p2 == 0)].mean():.1f}")
    print(f"chunks with outliers {np.mean(outl[ok] > 0):.3f}")
    print("mean open lanes after pass 1:", open1[ok].mean())
    for lo, hi in ((1, 16), (16, 32), (32, 48), (48, 64), (64, 65)):
        m = ok & (rows >= lo) & (rows < hi)
        if m.any():
            print(f"rows [{lo},{hi}): n {m.sum()}, dur mean {d[m].mean():.1f} p90 {np.percentile(d[m], 90):.1f}, "
                  f"pass2 {p2[m].mean():.2f}, box vol mean {vol[m].mean():.0f}")
    for lo, hi in ((0, 40), (40, 80), (80, 150), (150, 250), (250, 65536)):
        m = ok & (vol >= lo) & (vol < hi)
        if m.any():
            print(f"box vol [{lo},{hi}): n {m.sum()}, dur mean {d[m].mean():.1f} p90 {np.percentile(d[m], 90):.1f}, "
                  f"pass2 {p2[m].mean():.2f}, rows mean {rows[m].mean():.0f}")
    long = ok & (d >= np.percentile(d[ok], 95))
    print(f"the longest 5 %: rows mean {rows[long].mean():.0f}, vol mean {vol[long].mean():.0f}, "
          f"pass2 {p2[long].mean():.2f}, open1 mean {open1[long].mean():.1f}, start mean {s[long].mean():.1f}")
    order = np.argsort(np.where(ok, np.arange(len(ok)) % nch, 1 << 30))
    pos = (np.arange(len(ok)) % nch)
    for lo in range(0, nch, nch // 8):
        m = ok & (pos >= lo) & (pos < lo + nch // 8)
        print(f"  items [{lo},{lo + nch // 8}): dur mean {d[m].mean():.1f}, pass2 {p2[m].mean():.2f}")
    lastw = wave[np.argmax(np.where(ok, e, -1))]
    sel = ok & (wave == lastw)
    print("slowest wave's chunks (start, dur):", list(zip(np.round(s[sel], 1), np.round(d[sel], 1))))
    tot = d[ok].sum()
    print(f"sum of chunk durations {tot:.0f} wave-us = {tot / len(waves):.1f} us per used wave")


if __name__ == "__main__":
    main()
