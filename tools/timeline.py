"""Per-step timeline of the sampling loop from a rocprofv3 kernel trace:

    python tools/timeline.py gpurun_out/TAG/prof/run_kernel_trace.csv [--anchor noise_mlp] [--last 20]

Steps are delimited by the anchor kernel (one noise-MLP launch per step).  For the last N steps
prints each dispatch's offset from the step's first dispatch, duration and queue, then a summary:
step wall (anchor to anchor), busy time on the loop queue, gaps, and per-kernel mean durations."""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--anchor", default="noise_mlp")
    ap.add_argument("--last", type=int, default=20)
    ap.add_argument("--show", type=int, default=2, help="steps printed in full")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = []
    for r in rows:
        name = r.get("Kernel_Name") or r.get("KernelName") or r.get("Name")
        st = int(r.get("Start_Timestamp") or r.get("BeginNs"))
        en = int(r.get("End_Timestamp") or r.get("EndNs"))
        q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
        short = name.split("(")[0].replace("void ", "").replace("pcst::", "")
        ks.append((st, en, short, q))
    ks.sort()
    anchors = [i for i, k in enumerate(ks) if a.anchor in k[2]]
    anchors = anchors[-(a.last + 1):]
    # step j = the dispatches from anchor j up to anchor j+1: the post-MLP part of one step, then
    # the pre-MLP part of the next
    per = collections.defaultdict(list)
    walls = []
    for j in range(len(anchors) - 1):
        i0, i1 = anchors[j], anchors[j + 1]
        walls.append((ks[i1][0] - ks[i0][0]) / 1e3)
        for k in ks[i0:i1]:
            per[k[2]].append((k[1] - k[0]) / 1e3)
        if j < a.show:
            t0 = ks[i0][0]
            print(f"--- step {j}: anchor to anchor {walls[-1]:.1f} us")
            for k in ks[i0:i1 + 1]:
                print(f"  {(k[0] - t0) / 1e3:8.1f} +{(k[1] - k[0]) / 1e3:7.1f}  q{k[3]:>3}  {k[2][:70]}")
    n = len(walls)
    print(f"\n{n} steps: wall mean {sum(walls) / n:.1f} us, min {min(walls):.1f}, max {max(walls):.1f}")
    tot = 0.0
    for name, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        tot += sum(v) / n
        print(f"  {name[:60]:60s} {len(v) / n:5.2f}/step  mean {sum(v) / len(v):7.2f} us  "
              f"per step {sum(v) / n:7.2f} us")
    print(f"  sum of kernel time per step {tot:.1f} us (overlapping streams counted twice)")


if __name__ == "__main__":
    main()
