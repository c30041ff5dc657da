#!/bin/bash
# Chamfer forward timing per mode (1 exhaustive, 3 hybrid, 2 grid) over the noise of a predicted
# x0 against its lidar-like target (tools/bench_chamfer.py); the trainer's clouds span this range.
set -u
OUT=gpurun_out/${1:-cdsweep}; mkdir -p "$OUT"
for n in 0.02 0.2 1 4; do
  for m in 1 3 2; do
    timeout -k 10 120 python tools/bench_chamfer.py --kind lidar --noise $n --mode $m --reps 5 >> "$OUT/sweep.jsonl" || exit 1
    tail -1 "$OUT/sweep.jsonl"
  done
done
