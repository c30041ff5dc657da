set -u
for S in 20 300; do
for cfg in "seq 0" "side 0" "side_lo 0" "side 65536" "side_lo 65536" "side_lo 98304"; do
  set -- $cfg
  PCST_KNN_BUILD_LDS_PAD=$2 timeout -k 10 200 python tools/overlap_probe.py --mode $1 --steps $S 2>/dev/null | tail -1 || exit 1
done
done
