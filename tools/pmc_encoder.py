"""HBM bytes per launch of the encoder kernels (FPS, ball query) from rocprofv3 --pmc
FETCH_SIZE / WRITE_SIZE passes over `bench.py`, split by launch shape (grid size: B = 1 and
B = 32 clouds), corrected as MI355X_MICROARCH.md's HBM section prescribes (FETCH_SIZE x2 on
gfx950, WRITE_SIZE as read).  Writes profiles/encoder_traffic.json, which bench.py reads for
`encoder_rooflines.*.counters`.

usage: python tools/pmc_encoder.py RUN_DIR [OUT_JSON]"""
import csv
import json
import os
import sys
from collections import defaultdict

# (name, kernel substring, fixed tag or None: tag by grid size).  FPS at one cloud runs the
# multi-CU kernel (geometry.hip fps_multi_kernel), at 32 clouds the culled one.
KERNELS = [("fps", "fps_multi_kernel", "b1"), ("fps", "fps_cull_kernel<30>", "b32"),
           ("ball_query", "ball_query_split_kernel", None)]


def main():
    run = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "encoder_traffic.json")
    acc = defaultdict(list)
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        with open(os.path.join(run, f"pmc_{c}", "pmc_counter_collection.csv")) as f:
            for r in csv.DictReader(f):
                for name, sub, tag in KERNELS:
                    if sub in r["Kernel_Name"]:
                        acc[(name, tag, int(r["Grid_Size"]), c)].append(float(r["Counter_Value"]))
    grids = sorted({(n, t or "", g) for n, t, g, _ in acc})
    rec = {"source": run, "correction": "FETCH_SIZE x2 (gfx950 wide-read tally), WRITE_SIZE x1",
           "unit": "bytes per launch", "bytes_per_launch": {}, "launches": {}}
    for name, t, g in grids:
        f = acc.get((name, t or None, g, "FETCH_SIZE"), [])
        w = acc.get((name, t or None, g, "WRITE_SIZE"), [])
        if not f or not w:
            continue
        # grid = threads; ball query runs 16 waves per cloud-chunk: its smaller grid is the
        # B = 1 launch, the larger B = 32
        tag = t or ("b1" if g == min(gg for nn, tt, gg in grids if nn == name and not tt) else "b32")
        key = f"{name}_{tag}"
        rec["bytes_per_launch"][key] = round(2.0 * 1024 * sum(f) / len(f) + 1024 * sum(w) / len(w))
        rec["launches"][key] = {"grid": g, "n": len(f)}
    with open(out, "w") as fh:
        json.dump(rec, fh, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
