#!/bin/bash
# Round-5 GPU check: tools/r5_check.sh TAG [STAGES...]  (round 4's stages plus timeline)
#   tests=EXPR   pytest -m gpu -k EXPR (tests=all: the whole GPU suite)
#   smoke        __graft_entry__.smoke()
#   bench        the driver's invocation (bench.py --gpus 1 --steps 20 --warmup 5)
#   prof         rocprofv3 kernel trace + stats of the driver's window (tools/kstats.py summary)
#   pmc          noise-MLP counters over the driver's window: one SQ pass (MFMA count, MFMA-busy
#                cycles, LDS waits), FETCH_SIZE and WRITE_SIZE passes (tools/pmc_summary.py)
#   b32          the 32-cloud bench (configs[4]'s per-GPU share)
#   train        tools/bench_train.py (configs[2]) plain
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
TAG=$1; shift; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BENCH="bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-encoder --no-other-precision --no-extra"
for st in "$@"; do
  case $st in
    tests=*)
      K=${st#tests=}
      if [ "$K" = all ]; then SEL=(); else SEL=(-k "$K"); fi
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
          "${SEL[@]}" > "$OUT/pytest.log" 2>&1
      rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" "$OUT/pytest.log" | head; tail -1 "$OUT/pytest.log"
      if [ $rc -ne 0 ]; then exit $rc; fi ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
      rc=$?; tail -1 "$OUT/smoke.log"; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    bench)
      timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
      rc=$?; echo "bench rc=$rc"; if [ $rc -ne 0 ]; then tail -3 "$OUT/bench.err"; exit $rc; fi
      python -c "import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]);print('bench', d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['avg_launch_ms'])" ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
          python $BENCH > "$OUT/pbench.json" 2> "$OUT/pbench.err"
      rc=$?; echo "prof rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "$OUT/pbench.err"; exit $rc; fi
      python tools/kstats.py "$OUT/prof/run_kernel_stats.csv" 25 | tee "$OUT/kernel_top.txt" ;;
    pmc)
      # counter passes serialise every queue's dispatches: the single-stream step layout (no
      # cross-stream flag waits, which would spin to their poll bound), 10 steps
      PB="tools/bench_knobs.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline --no-encoder --no-other-precision --no-extra"
      PCST_KNN_OVERLAP=0 timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS \
          SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/p1" -o pmc -- \
          python $PB > "$OUT/p1.log" 2>&1
      rc=$?; echo "pmc sq rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "$OUT/p1.log"; exit $rc; fi
      for C in FETCH_SIZE WRITE_SIZE; do
        PCST_KNN_OVERLAP=0 timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o pmc -- \
            python $PB > "$OUT/pmc_$C.log" 2>&1
        rc=$?; echo "pmc $C rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "$OUT/pmc_$C.log"; exit $rc; fi
      done
      python tools/pmc_sq.py "$OUT" noise_mlp | tee "$OUT/noise_mlp_sq_counters.txt"
      python tools/pmc_summary.py "$OUT" noise_mlp --json "$OUT/noise_mlp_traffic.json" | tail -4 ;;
    b32)
      timeout -k 10 300 python bench.py --gpus 1 --clouds-per-gpu 32 --steps 20 --warmup 3 --no-cpu-baseline \
          --no-encoder --no-other-precision --no-extra > "$OUT/bench_b32.json" 2> "$OUT/bench_b32.err"
      rc=$?; echo "b32 rc=$rc"; if [ $rc -ne 0 ]; then tail -3 "$OUT/bench_b32.err"; exit $rc; fi
      python -c "import json;d=json.loads(open('$OUT/bench_b32.json').read().strip().splitlines()[-1]);print('b32', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])" ;;
    train)
      timeout -k 10 300 python tools/bench_train.py > "$OUT/train.json" 2> "$OUT/train.err"
      rc=$?; echo "train rc=$rc"; if [ $rc -ne 0 ]; then tail -3 "$OUT/train.err"; exit $rc; fi
      tail -c 600 "$OUT/train.json"; echo ;;
    trainpmc)
      TB="tools/bench_train.py --steps 3 --warmup 1"
      timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
          SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d "$OUT/psq" -o pmc -- \
          python $TB > "$OUT/psq.log" 2>&1
      rc=$?; echo "trainpmc sq rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "$OUT/psq.log"; exit $rc; fi
      for C in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o pmc -- \
            python $TB > "$OUT/tpmc_$C.log" 2>&1
        rc=$?; echo "trainpmc $C rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "$OUT/tpmc_$C.log"; exit $rc; fi
      done
      python tools/pmc_summary.py "$OUT" gemm_bf | head -30 | tee "$OUT/train_traffic.txt"
      for k in "gemm_bf_kernel<1" "gemm_bf_kernel<3" "gemm_bf_kernel<6" "gemm_bf_kernel<7" wgrad_ex_kernel; do
        echo "== $k"; python tools/pmc_sq.py "$OUT" "$k"
      done | tee "$OUT/train_sq.txt" ;;
    trainprof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tprof" -o run -- \
          python tools/bench_train.py --steps 4 --warmup 2 > "$OUT/tprof.json" 2> "$OUT/tprof.err"
      rc=$?; echo "trainprof rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "$OUT/tprof.err"; exit $rc; fi
      python tools/kstats.py "$OUT/tprof/run_kernel_stats.csv" 40 | tee "$OUT/train_kernel_top.txt"; python tools/kstats.py "$OUT/tprof/run_kernel_stats.csv" 400 > "$OUT/train_kernel_all.txt" ;;
    split=*)
      # split=G: the 32-cloud step as G concurrent groups (tools/split_probe.py)
      timeout -k 10 500 python tools/split_probe.py --clouds 32 --groups ${st#split=} > "$OUT/split.json" 2> "$OUT/split.err"
      rc=$?; echo "split rc=$rc"; cat "$OUT/split.json"; if [ $rc -ne 0 ]; then tail -5 "$OUT/split.err"; exit $rc; fi ;;
    trainpmc2)
      # the fused residual-block kernels: LDS, MFMA and wait counters (one SQ pass)
      TB="tools/bench_train.py --steps 3 --warmup 1"
      timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS \
          SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d "$OUT/psq2" -o pmc -- \
          python $TB > "$OUT/psq2.log" 2>&1
      rc=$?; echo "trainpmc2 rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "$OUT/psq2.log"; exit $rc; fi
      for k in "resblock3_kernel" "resblock_kernel<true" "wgrad_ex_kernel<unsigned short, unsigned short"; do
        echo "== $k"; python tools/pmc_sq.py "$OUT" "$k" psq2
      done | tee "$OUT/train_sq2.txt" ;;
    trainab=*)
      # trainab=v_a,v_b: bench_train.py with the product library and each experiment library
      # pointcloud_style_transfer_amd/libpcst_hip_<v>.so, two alternating passes
      VS=${st#trainab=}
      for pass in 1 2; do
        for v in prod ${VS//,/ }; do
          # v_name: experiment library; NAME=VAL: the product library with that knob (tools/knobs.py)
          lib=$PWD/pointcloud_style_transfer_amd/libpcst_hip.so; kv=PCST_NONE=1
          case $v in prod) ;; *=*) kv=$v ;; *) lib=$PWD/pointcloud_style_transfer_amd/libpcst_hip_$v.so ;; esac
          env "$kv" PCST_LIB=$lib timeout -k 10 300 python tools/bench_train.py > "$OUT/train_$v.$pass.json" 2> "$OUT/train_$v.$pass.err"
          rc=$?; if [ $rc -ne 0 ]; then tail -3 "$OUT/train_$v.$pass.err"; exit $rc; fi
          python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['final_loss'])" "$OUT/train_$v.$pass.json" "$v.$pass"
        done
      done ;;
    b32prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/b32prof" -o run -- \
          python bench.py --gpus 1 --clouds-per-gpu 32 --steps 10 --warmup 3 --no-cpu-baseline --no-encoder --no-extra \
          --no-other-precision --no-extra > "$OUT/b32prof.json" 2> "$OUT/b32prof.err"
      rc=$?; echo "b32prof rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "$OUT/b32prof.err"; exit $rc; fi
      python tools/kstats.py "$OUT/b32prof/run_kernel_stats.csv" 25 | tee "$OUT/b32_kernel_top.txt" ;;
    benchlib=*)
      # benchlib=v_a,v_b: the driver-window bench (and the 32-cloud bench) with each library, two passes
      VS=${st#benchlib=}
      for pass in 1 2; do
        for v in prod ${VS//,/ }; do
          if [ "$v" = prod ]; then lib=$PWD/pointcloud_style_transfer_amd/libpcst_hip.so; else lib=$PWD/pointcloud_style_transfer_amd/libpcst_hip_$v.so; fi
          PCST_LIB=$lib timeout -k 10 200 python tools/bench_knobs.py ${BENCH#bench.py } > "$OUT/bench_$v.$pass.json" 2> "$OUT/bench_$v.$pass.err"
          rc=$?; if [ $rc -ne 0 ]; then tail -3 "$OUT/bench_$v.$pass.err"; exit $rc; fi
          PCST_LIB=$lib timeout -k 10 200 python tools/bench_knobs.py --gpus 1 --clouds-per-gpu 32 --steps 10 --warmup 3 \
              --no-cpu-baseline --no-encoder --no-other-precision --no-extra > "$OUT/b32_$v.$pass.json" 2> "$OUT/b32_$v.$pass.err"
          rc=$?; if [ $rc -ne 0 ]; then tail -3 "$OUT/b32_$v.$pass.err"; exit $rc; fi
          python -c "import json,sys; f=lambda p: json.loads(open(p).read().strip().splitlines()[-1]); a=f(sys.argv[1]); b=f(sys.argv[2]); print(sys.argv[3], 'b1', a['value'], a['ms_per_step'], a['roofline']['avg_launch_ms'], 'b32', b['ms_per_step'])" "$OUT/bench_$v.$pass.json" "$OUT/b32_$v.$pass.json" "$v.$pass"
        done
      done ;;
    benchknob=*)
      # benchknob=NAME=VAL,...: the driver-window bench (and the 32-cloud bench) with the product
      # library plain and with each knob (tools/knobs.py through tools/bench_knobs.py), two passes
      VS=${st#benchknob=}
      for pass in 1 2; do
        for v in prod ${VS//,/ }; do
          kv=PCST_NONE=1; if [ "$v" != prod ]; then kv=$v; fi
          env "$kv" timeout -k 10 200 python tools/bench_knobs.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
              --no-encoder --no-other-precision --no-extra > "$OUT/bench_$v.$pass.json" 2> "$OUT/bench_$v.$pass.err"
          rc=$?; if [ $rc -ne 0 ]; then tail -3 "$OUT/bench_$v.$pass.err"; exit $rc; fi
          env "$kv" timeout -k 10 200 python tools/bench_knobs.py --gpus 1 --clouds-per-gpu 32 --steps 10 --warmup 3 \
              --no-cpu-baseline --no-encoder --no-other-precision --no-extra > "$OUT/b32_$v.$pass.json" 2> "$OUT/b32_$v.$pass.err"
          rc=$?; if [ $rc -ne 0 ]; then tail -3 "$OUT/b32_$v.$pass.err"; exit $rc; fi
          python -c "import json,sys; f=lambda p: json.loads(open(p).read().strip().splitlines()[-1]); a=f(sys.argv[1]); b=f(sys.argv[2]); print(sys.argv[3], 'b1', a['value'], a['ms_per_step'], a['roofline']['avg_launch_ms'], 'b32', b['ms_per_step'])" "$OUT/bench_$v.$pass.json" "$OUT/b32_$v.$pass.json" "$v.$pass"
        done
      done ;;
    proflib=*)
      # proflib=v_a,v_b: kernel stats of the driver-window bench with each library (kNN / voxel rows)
      VS=${st#proflib=}
      for v in prod ${VS//,/ }; do
        lib=$PWD/pointcloud_style_transfer_amd/libpcst_hip.so
        if [ "$v" != prod ]; then lib=$PWD/pointcloud_style_transfer_amd/libpcst_hip_$v.so; fi
        PCST_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$v" -o run -- \
            python tools/bench_knobs.py ${BENCH#bench.py } > "$OUT/pbench_$v.json" 2> "$OUT/pbench_$v.err"
        rc=$?; if [ $rc -ne 0 ]; then tail -5 "$OUT/pbench_$v.err"; exit $rc; fi
        echo "== $v"; python tools/kstats.py "$OUT/prof_$v/run_kernel_stats.csv" 12 | tee "$OUT/kernel_top_$v.txt"
      done ;;
    timeline)
      python tools/timeline.py "$OUT/prof/run_kernel_trace.csv" --last 18 --show 2 | tee "$OUT/driver_window_timeline.txt" | tail -40 ;;
    fpsab=*)
      # fpsab=v_a,v_b: tools/fps_ab.py with the product library and each experiment library
      VS=${st#fpsab=}
      for v in prod ${VS//,/ }; do
        lib=$PWD/pointcloud_style_transfer_amd/libpcst_hip.so
        if [ "$v" != prod ]; then lib=$PWD/pointcloud_style_transfer_amd/libpcst_hip_$v.so; fi
        PCST_LIB=$lib timeout -k 10 120 python tools/fps_ab.py > "$OUT/fps_$v.txt" 2>&1
        rc=$?; cat "$OUT/fps_$v.txt"; if [ $rc -ne 0 ]; then exit $rc; fi
      done ;;
    knnab=*)
      # knnab=v_a,v_b: tools/knn_check.py result hashes with the product library and each experiment library
      VS=${st#knnab=}
      for v in prod ${VS//,/ }; do
        lib=$PWD/pointcloud_style_transfer_amd/libpcst_hip.so
        if [ "$v" != prod ]; then lib=$PWD/pointcloud_style_transfer_amd/libpcst_hip_$v.so; fi
        PCST_LIB=$lib timeout -k 10 120 python tools/knn_check.py > "$OUT/knn_$v.txt" 2>&1
        rc=$?; grep -v amdgpu.ids "$OUT/knn_$v.txt"; if [ $rc -ne 0 ]; then exit $rc; fi
      done ;;
    eventab)
      # the driver-window bench with MLP events on every timed step vs every 4th (two alternating passes)
      for pass in 1 2; do
        for e in 1 4; do
          timeout -k 10 200 python bench.py ${BENCH#bench.py } --event-every $e > "$OUT/bench_ev$e.$pass.json" 2> "$OUT/bench_ev$e.$pass.err"
          rc=$?; if [ $rc -ne 0 ]; then tail -3 "$OUT/bench_ev$e.$pass.err"; exit $rc; fi
          python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('events every', sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" "$OUT/bench_ev$e.$pass.json" "$e.$pass"
        done
      done ;;
    graphab)
      # configs[4]'s batch32 leg (eager and graph) with GRAPH_FORK_BUILD on and off, two alternating passes
      for pass in 1 2; do
        for v in prod PCST_GRAPH_FORK_BUILD=0; do
          kv=PCST_NONE=1; if [ "$v" != prod ]; then kv=$v; fi
          env "$kv" timeout -k 10 300 python tools/bench_knobs.py --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline \
              --no-encoder --no-other-precision > "$OUT/graph_$v.$pass.json" 2> "$OUT/graph_$v.$pass.err"
          rc=$?; if [ $rc -ne 0 ]; then tail -3 "$OUT/graph_$v.$pass.err"; exit $rc; fi
          python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); b=d['batch32']; print(sys.argv[2], 'eager', b['eager']['ms_per_step'], 'graph', b['graph']['ms_per_step'], 'train', d['train_step']['ms_per_step'])" "$OUT/graph_$v.$pass.json" "$v.$pass"
        done
      done ;;
    loop1000)
      timeout -k 10 600 python -u tools/loop1000_probe.py > "$OUT/loop1000.jsonl" 2> "$OUT/loop1000.err"
      rc=$?; echo "loop1000 rc=$rc"; cat "$OUT/loop1000.jsonl"; if [ $rc -ne 0 ]; then tail -3 "$OUT/loop1000.err"; exit $rc; fi ;;
    *) echo "unknown stage $st"; exit 2 ;;
  esac
done
