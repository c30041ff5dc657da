"""Per-step breakdown of the trainer from a rocprofv3 kernel trace (tools/r4_check.sh trainprof):

    python tools/train_timeline.py gpurun_out/TAG/tprof/run_kernel_trace.csv [--anchor amp_update_scale]

Steps are delimited by the anchor kernel (one per optimizer step).  Prints, per queue, the busy
time per step and the kernels grouped by family, averaged over the steps after the first."""
import argparse
import collections
import csv
import re


def family(name):
    n = name.replace("void ", "").replace("pcst::", "")
    n = re.sub(r"\(.*", "", n)
    return n[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--anchor", default="amp_update_scale")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    ks = []
    for r in csv.DictReader(open(a.trace)):
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), family(r["Kernel_Name"]),
                   r.get("Queue_Id") or "?"))
    ks.sort()
    anchors = [i for i, k in enumerate(ks) if a.anchor in k[2]]
    steps = list(zip(anchors, anchors[1:]))[1:]  # skip the first (warm-up) interval
    if not steps:
        print("not enough steps")
        return
    walls, per_q, fam = [], collections.Counter(), collections.Counter()
    for s0, s1 in steps:
        t0, t1 = ks[s0][1], ks[s1][1]
        walls.append((t1 - t0) / 1e3)
        for st, en, n, q in ks[s0 + 1:s1 + 1]:
            per_q[q] += (en - st) / 1e3
            fam[n] += (en - st) / 1e3
    ns = len(steps)
    print(f"{ns} steps: wall mean {sum(walls) / ns:.1f} us (min {min(walls):.1f}, max {max(walls):.1f})")
    for q, v in per_q.most_common():
        print(f"  queue {q}: busy {v / ns:.1f} us/step")
    print("kernel families, us per step:")
    for n, v in fam.most_common(a.top):
        print(f"  {v / ns:9.1f}  {n}")


if __name__ == "__main__":
    main()
