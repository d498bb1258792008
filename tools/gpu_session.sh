#!/bin/bash
# One GPU session on the MI355X box: tests, smoke, benches, A/B runs and rocprofv3 profiles.
# Every GPU step has its own time limit; the session stops at the first failing step
# (fault / abort / timeout), so nothing runs on a GPU in a bad state.
#
#   bash tools/gpu_session.sh [OUT=dir] step...       (default steps: test smoke serve kbench prof)
#
# steps:
#   test          pytest -m gpu (whole GPU tier)          smoke      __graft_entry__.smoke()
#   serve         headline bench (Iris /predict)           serve_wide F=256 /predict, K=1000 and K=2, f32 and bf16
#   resident      resident SMALL-path kernel: its GPU tests (tests/test_resident.py)
#   serve_res     the driver's serve command, resident kernel on / off, interleaved x3 (RES_ROUNDS)
#   marker        rocprofv3 --marker-trace of serve / serve_wide with the roctx stage ranges on
#   serve_ab      serve with kernel-argument batches on/off, interleaved x2 (box variance is large)
#   serve_idle    serve with the idle-engine fast path on (8 rows) / off, interleaved x2
#   serve_abenv   serve with AB_VAR set to each of AB_VALS, interleaved x2
#   serve_compl   serve with COMPLS completer threads (default "1 2"), interleaved x2
#   dispatch_ab   serve with source-affinity vs per-connection round-robin dispatch (DISPATCHES), N=1 and N=2 (p2p), x2
#   serve_pin     serve with the rank pinned to physical cores (server / load generator apart) vs unpinned, x2
#   serve_spin    serve with busy-polling IO threads / spinning batcher+completer (SPINS="0 50"), interleaved x2
#   selfl         bench.py --gpus 2 self-launched (p2p on one device) + the refusal without p2p
#   dptrain       fused DP training: GPU comm tests, N=1 / N=2 (p2p) benches, fused vs unfused, kernel traces
#   kbench        gemv / gemm / train / train_softmax benches
#   prof          rocprofv3 --kernel-trace --stats of every bench mode (incl. serve and serve_wide)
#   pmc_gemm      hardware counters of the gemm bench (tools/pmc_profile.sh)
#   gemm_ws       W-stationary persistent gemm_softmax kernel vs the 32x32 kernel (tests, A/B x2, kernel stats)
#   split_big     class-split kernel vs tiles kernel at B = 256 / 1024 / 2048, interleaved x2
#   gemm_xcd      XCD-local vs agent-scope split merge in the tiles kernels (MLAPI_GEMM_XCD=1/0), B = 1024 / 8192
#   split_xcd     XCD-local vs agent-scope split merge (MLAPI_SPLIT_XCD=1/0), B = 32..2048, x2 + kernel stats
#   threads       IO-thread / load-generator-thread split sweep, THREADS="io:cl ..." (default "10:4 8:6 6:6"), x2
#   gdw           softmax G+dW kernel: its GPU tests + tools/softmax_train_sweep.py timings
#   serve_ab_old  interleaved x3 serve bench: ab_old/ (previous build) vs the working tree
#   serve_ab3     interleaved x2: ab_old/ vs the working tree vs the working tree with AB_ENV (e.g. MLAPI_KERNARG_HOST=1)
#   gemm_ab       interleaved x3 gemm bench: ab_old/mlapi_amd (stashed previous build) vs the working tree
#   prev_ab       interleaved x3: the previous build copied to ab_prev/ vs the working tree (PREV_ARGS)
#   wide_trace    WIDE kernel timeline + rocprofv3 phase split (tools/wide_trace.py, tools/wide_probe.py)
#   bench_abenv   any bench mode (BENCH_ARGS) with AB_VAR set to each of AB_VALS, interleaved x2
#   serve_lgsplit IO threads x load-generator threads (SPLITS="io:lg ...", LGARGS), interleaved
#   serve_n2res   two ranks on one GPU: resident on / off x placement
#   serve_wide64  serve_wide at f64 for K = 2 / 40 / 1000
#   faults        resident-path fault injection tests + the 17-32-row wide host-merge test
#   steer         paired + shuffled phases, io_steer 0 / 1 x SPLITS (default "8:8 8:5 8:6"), interleaved x RES_ROUNDS
#   shuf_env      paired + shuffled phases with AB_VAR set to each of AB_VALS (SPLITS), interleaved x RES_ROUNDS
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
export TMPDIR=/tmp
O=gpurun_out
if [[ "${1:-}" == OUT=* ]]; then O="${1#OUT=}"; shift; fi
mkdir -p "$O"
O=$(cd "$O" && pwd)
stop() { echo "STOP: $1 failed with rc=$2"; tail -20 "$3"; exit "$2"; }
run() {  # run <name> <limit_s> <cmd...>: output to $O/<name>.log
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  [ $rc -eq 0 ] || stop "$name" $rc "$O/$name.log"
  tail -2 "$O/$name.log" | cut -c1-600
}
prof() {  # prof <name> <limit_s> <bench args...>
  local name=$1 lim=$2; shift 2
  (cd /tmp && timeout -k 10 "$lim" rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$name" -o "$name" \
     -- python3 "$R/bench.py" "$@" > "$O/prof_$name.log" 2>&1)
  local rc=$?
  [ $rc -eq 0 ] || stop "prof_$name" $rc "$O/prof_$name.log"
  trim
  tail -1 "$O/prof_$name.log" | cut -c1-300
}
trim() {  # gpurun copies gpurun_out/ back only below 64 MiB: keep the --stats summaries, drop big traces
  find "$O" -name '*_trace.csv' -size +6M -delete
}
steps="${*:-test smoke serve kbench prof}"
for s in $steps; do
  case $s in
    test) run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    smoke) run smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    serve) run bench_serve 300 python -u bench.py --steps 200 --warmup 20 ;;
    resident) run pytest_resident 400 python -u -m pytest tests/test_resident.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    serve_resv)  # resident-path variants, interleaved x RES_ROUNDS: off, spin 5 / 2 us, 1 poll in flight, sleep 3 us
      for r in $(seq 1 "${RES_ROUNDS:-2}"); do
        MLAPI_RESIDENT=off run "resv_off_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
        run "resv_spin5_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
        MLAPI_IO_RING_SPIN_US=2 run "resv_spin2_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
        MLAPI_RESIDENT_DEPTH=1 run "resv_d1_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
        MLAPI_IO_RING_SLEEP_US=3 run "resv_sleep3_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
      done ;;
    serve_resx)  # resident-path experiments: polling cost with rows on the queue (shadow), IO / loadgen splits
      for r in $(seq 1 "${RES_ROUNDS:-2}"); do
        MLAPI_RESIDENT=off run "resx_off_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
        MLAPI_RESIDENT_SHADOW=1 MLAPI_RESIDENT_IDLE_POLLS=1000000000 run "resx_shadow_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
        run "resx_on_io6_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --io-threads 6 --client-threads 4
        run "resx_on_io8_lg6_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --io-threads 8 --client-threads 6
        run "resx_on_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
      done ;;
    serve_lgspin)  # load-generator spin (MLAPI_LOADGEN_SPIN_US) x resident path x IO threads, interleaved
      for r in $(seq 1 "${RES_ROUNDS:-2}"); do
        MLAPI_RESIDENT=off run "lgs_off_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
        MLAPI_RESIDENT=off MLAPI_LOADGEN_SPIN_US=50 run "lgs_off_spin_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
        run "lgs_on_io6_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --io-threads 6 --client-threads 4
        MLAPI_LOADGEN_SPIN_US=50 run "lgs_on_io6_spin_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --io-threads 6 --client-threads 4
        MLAPI_LOADGEN_SPIN_US=50 run "lgs_on_io8_spin_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --io-threads 8 --client-threads 4
        MLAPI_LOADGEN_SPIN_US=50 run "lgs_on_io10_spin_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
      done ;;
    serve_numa)  # NUMA-node placement of the rank + load generator (--pin numa) x resident path, interleaved
      for r in $(seq 1 "${RES_ROUNDS:-2}"); do
        MLAPI_RESIDENT=off run "numa_off_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --pin numa
        run "numa_on_io8_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --pin numa --io-threads 8 --client-threads 4
        MLAPI_LOADGEN_SPIN_US=50 run "numa_on_io8_spin_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --pin numa --io-threads 8 --client-threads 4
        run "numa_on_io10_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --pin numa
        run "nonuma_on_io8_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --io-threads 8 --client-threads 4
        MLAPI_RESIDENT=off run "nonuma_off_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
      done ;;
    serve_lgsplit)  # IO threads x load-generator threads (SPLITS="io:lg ...", LGARGS: extra bench args), interleaved
      for r in $(seq 1 "${RES_ROUNDS:-2}"); do
        for sp in ${SPLITS:-8:4 8:5 7:5 8:6 7:6}; do
          run "lgsplit_${sp/:/_}_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --io-threads ${sp%%:*} --client-threads ${sp##*:} ${LGARGS:-}
        done
      done ;;
    faults)
      run pytest_faults 400 python -u -m pytest tests/test_resident.py tests/test_wide_gpu.py -m gpu -x -v -p no:cacheprovider \
        --timeout 120 --timeout-method thread -k "fault or metrics or host_merge_17" ;;
    steer)  # SO_INCOMING_CPU connection steering off / on, paired and shuffled clients
      for r in $(seq 1 "${RES_ROUNDS:-2}"); do
        for sp in ${SPLITS:-8:8 8:5 8:6}; do
          for st in 0 1; do
            MLAPI_IO_STEER=$st run "steer${st}_${sp/:/_}_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 \
              --io-threads ${sp%%:*} --client-threads ${sp##*:} ${LGARGS:-}
          done
        done
      done ;;
    shuf_env)
      for r in $(seq 1 "${RES_ROUNDS:-2}"); do
        for sp in ${SPLITS:-8:8}; do
          for v in ${AB_VALS}; do
            export "$AB_VAR=$v"
            run "env_${v}_${sp/:/_}_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 \
              --io-threads ${sp%%:*} --client-threads ${sp##*:} ${LGARGS:-}
            unset "$AB_VAR"
          done
        done
      done ;;
    serve_n2res)  # two ranks on the one GPU (P2P data plane): resident on / off x placement, interleaved
      for r in $(seq 1 "${RES_ROUNDS:-2}"); do
        for pin in auto on; do
          for m in on off; do
            MLAPI_COMM=p2p MLAPI_RESIDENT=$m run "n2_${m}_${pin}_r$r" 300 python -u bench.py --gpus 2 --steps 20 --warmup 3 --pin $pin
          done
        done
      done ;;
    serve_res)  # the driver's exact command with the resident kernel on / off, interleaved
      for r in $(seq 1 "${RES_ROUNDS:-3}"); do
        for m in on off; do
          MLAPI_RESIDENT=$m run "serve_res${m}_r$r" 300 python -u bench.py --gpus 1 --steps 20 --warmup 5
        done
      done ;;
    serve_wide64)  # wide models at the default f64 (sklearn's dtype): every body byte-compared (rel_tol 0)
      for k in 2 40 1000; do
        run "bench_serve_wide_k${k}_f64" 300 python -u bench.py --mode serve_wide --wide-classes $k --wide-dtype f64 --steps 20 --warmup 5
      done ;;
    serve_wide)
      for dt in f32 bf16; do
        run bench_serve_wide_k1000_$dt 300 python -u bench.py --mode serve_wide --wide-classes 1000 --wide-dtype $dt --steps 40 --warmup 5
        run bench_serve_wide_k2_$dt 300 python -u bench.py --mode serve_wide --wide-classes 2 --wide-dtype $dt --steps 40 --warmup 5
      done ;;
    prof_wide)  # kernel durations of the served wide batches (class-split + host merge, BAR-staged rows)
      for dt in bf16 f32; do
        prof "serve_wide_k1000_$dt" 300 --mode serve_wide --wide-dtype $dt --steps 10 --warmup 2 --reqs-per-conn 256
      done ;;
    prof_direct)  # wide batches dispatched into the engine's HSA queue: mlapi_gemv_* / mlapi_split_* in the trace
      prof serve_wide_k2_bf16_direct 300 --mode serve_wide --wide-classes 2 --wide-dtype bf16 --steps 10 --warmup 2 --reqs-per-conn 256
      prof serve_wide_k40_f32_direct 300 --mode serve_wide --wide-classes 40 --wide-dtype f32 --steps 10 --warmup 2 --reqs-per-conn 256
      run bench_serve_wide_k40_f32 300 python -u bench.py --mode serve_wide --wide-classes 40 --wide-dtype f32 --steps 40 --warmup 5
      MLAPI_DIRECT_WIDE=0 run bench_serve_wide_k40_f32_hip 300 python -u bench.py --mode serve_wide --wide-classes 40 --wide-dtype f32 --steps 40 --warmup 5
      run bench_serve_wide_k40_f32_r2 300 python -u bench.py --mode serve_wide --wide-classes 40 --wide-dtype f32 --steps 40 --warmup 5
      MLAPI_DIRECT_WIDE=0 run bench_serve_wide_k40_f32_hip_r2 300 python -u bench.py --mode serve_wide --wide-classes 40 --wide-dtype f32 --steps 40 --warmup 5
      ;;
    marker)  # roctx ranges of every serving stage (MLAPI_ROCTX=1) + kernel trace: rocprofv3 --marker-trace
      (cd /tmp && MLAPI_ROCTX=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv \
         -d "$O/prof_marker_serve" -o serve -- python3 "$R/bench.py" --steps 5 --warmup 1 --reqs-per-conn 256 --c1-requests 500 \
         > "$O/prof_marker_serve.log" 2>&1) || stop marker $? "$O/prof_marker_serve.log"
      (cd /tmp && MLAPI_ROCTX=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv \
         -d "$O/prof_marker_serve_wide" -o serve_wide -- python3 "$R/bench.py" --mode serve_wide --steps 3 --warmup 1 \
         --reqs-per-conn 128 --c1-requests 300 > "$O/prof_marker_serve_wide.log" 2>&1) || stop marker_wide $? "$O/prof_marker_serve_wide.log"
      trim
      tail -1 "$O/prof_marker_serve.log" | cut -c1-200 ;;
    serve_ab)
      for r in 1 2; do
        for m in 1 0; do
          MLAPI_INLINE_ARGS=$m run "serve_inline${m}_r$r" 300 python -u bench.py --steps 100 --warmup 10
        done
      done ;;
    serve_idle)
      for r in 1 2; do
        for m in 8 0; do
          MLAPI_IDLE_INLINE_ROWS=$m run "serve_idle${m}_r$r" 300 python -u bench.py --steps 60 --warmup 5
        done
      done ;;
    serve_abenv)  # generic interleaved A/B: AB_VAR=<env var> AB_VALS="<v1> <v2> ..."
      for r in 1 2; do
        for v in $AB_VALS; do
          env "$AB_VAR=$v" timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 > "$O/serve_${AB_VAR}_${v}_r$r.log" 2>&1 \
            || stop "serve_${AB_VAR}_${v}_r$r" $? "$O/serve_${AB_VAR}_${v}_r$r.log"
          tail -1 "$O/serve_${AB_VAR}_${v}_r$r.log" | cut -c1-300
        done
      done ;;
    serve_compl)
      for r in 1 2; do
        for c in ${COMPLS:-1 2}; do
          MLAPI_COMPLETERS=$c run "serve_compl${c}_r$r" 300 python -u bench.py --steps 60 --warmup 5
        done
      done ;;
    dispatch_ab)  # connection dispatch (DISPATCHES, default "source acceptor"), interleaved x2 (N=1 and p2p N=2)
      for r in 1 2; do
        for d in ${DISPATCHES:-source acceptor}; do
          run "serve_dispatch_${d}_r$r" 300 python -u bench.py --steps 60 --warmup 5 --dispatch $d
          MLAPI_COMM=p2p run "serve_dispatch_${d}_n2_r$r" 300 python -u bench.py --gpus 2 --steps 30 --warmup 3 --dispatch $d
        done
      done ;;
    serve_pin)
      for r in 1 2; do
        for p in on off; do
          run "serve_pin${p}_r$r" 300 python -u bench.py --steps 60 --warmup 5 --pin $p
        done
      done ;;
    serve_spin)
      for r in 1 2; do
        for sp in ${SPINS:-0 50}; do
          MLAPI_SPIN_US=$sp MLAPI_IO_SPIN_US=$sp run "serve_spin${sp}_r$r" 300 python -u bench.py --steps 60 --warmup 5
        done
      done ;;
    selfl)  # bench.py --gpus N self-launch on the 1-GPU box: p2p shares the device; plain RCCL must refuse
      MLAPI_COMM=p2p run bench_selflaunch_p2p_n2 300 python -u bench.py --gpus 2 --steps 20 --warmup 3
      MLAPI_COMM=p2p run bench_selflaunch_p2p_train_n2 300 python -u bench.py --gpus 2 --mode train --steps 50 --warmup 5
      timeout -k 10 120 python -u bench.py --gpus 2 --steps 3 --warmup 1 > "$O/bench_selflaunch_rccl_n2_refused.log" 2>&1
      rc=$?; echo "rccl n2 on 1 GPU: rc=$rc (expected 2)"; [ $rc -eq 2 ] || stop selfl_refuse $rc "$O/bench_selflaunch_rccl_n2_refused.log" ;;
    dptrain)  # fused DP training step: GPU tests, benches at N=1 / N=2 (p2p on one device), kernel traces
      run pytest_dp 600 python -u -m pytest tests/test_comm_gpu.py -x -v -p no:cacheprovider --timeout 240 --timeout-method thread
      for m in train train_softmax; do
        run "bench_${m}_n1" 300 python -u bench.py --mode $m --steps 100 --warmup 10
        MLAPI_DP_FUSED=0 run "bench_${m}_n1_unfused" 300 python -u bench.py --mode $m --steps 100 --warmup 10
        MLAPI_COMM=p2p run "bench_${m}_n2" 300 python -u bench.py --gpus 2 --mode $m --steps 100 --warmup 10
        prof "${m}_n1" 300 --mode $m --steps 20 --warmup 2
      done ;;
    p2pmode)  # fused DP exchange protocol variants (MLAPI_P2P_MODE bits), interleaved x2, N=1 and N=2
      for r in 1 2; do
        for md in 0 1 2 3; do
          MLAPI_P2P_MODE=$md run "tsm_mode${md}_r$r" 300 python -u bench.py --mode train_softmax --steps 100 --warmup 10
          MLAPI_P2P_MODE=$md MLAPI_COMM=p2p run "tsm_mode${md}_n2_r$r" 300 python -u bench.py --gpus 2 --mode train_softmax --steps 100 --warmup 10
        done
        MLAPI_DP_FUSED=0 run "tsm_unfused_r$r" 300 python -u bench.py --mode train_softmax --steps 100 --warmup 10
      done ;;
    split)  # class-split multiclass kernel: GPU tests, graph-replay timings vs the tiles kernel, rocprofv3
      run pytest_split 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "linear_split or gemm"
      for B in 1 8 32; do
        run "gemm_tiles_b$B" 120 python -u bench.py --mode gemm --batch $B --steps 2000 --warmup 50
        run "gemm_split_b$B" 120 python -u bench.py --mode gemm --batch $B --steps 2000 --warmup 50 --gemm-kernel split
      done
      run gemm_split_f32_b256 120 python -u bench.py --mode gemm --batch 256 --steps 1000 --warmup 50 --gemm-dtype f32
      run gemm_split_f32_b1024 120 python -u bench.py --mode gemm --batch 1024 --steps 1000 --warmup 50 --gemm-dtype f32
      prof gemm_split_b8 120 --mode gemm --batch 8 --steps 200 --warmup 5 --gemm-kernel split --launch eager
      prof gemm_tiles_b8 120 --mode gemm --batch 8 --steps 200 --warmup 5 --launch eager ;;
    splitprobe)  # phase cost of the class-split kernel: full / no merge / no ticket (kernel durations)
      for pr in 0 1 2; do
        MLAPI_SPLIT_PROBE=$pr prof "split_probe${pr}_b8" 120 --mode gemm --batch 8 --steps 300 --warmup 5 --gemm-kernel split --launch eager
        MLAPI_SPLIT_PROBE=$pr prof "split_probe${pr}_b1" 120 --mode gemm --batch 1 --steps 300 --warmup 5 --gemm-kernel split --launch eager
      done
      prof "tiles_b1" 120 --mode gemm --batch 1 --steps 300 --warmup 5 --launch eager ;;
    kbench)  # kernel benches; the training modes in steady state (200 warm-up steps: the GPU's clock ramp)
      for m in gemv gemm; do run "bench_$m" 300 python -u bench.py --mode $m --steps 100 --warmup 10; done
      for m in train train_softmax; do run "bench_$m" 300 python -u bench.py --mode $m --steps 500 --warmup 200; done
      run bench_train_softmax_f1024 300 python -u bench.py --mode train_softmax --softmax-features 1024 --steps 100 --warmup 20 ;;
    driver)  # the driver's exact headline command
      run bench_driver 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 ;;
    prof)
      for m in gemv gemm train train_softmax; do prof "$m" 300 --mode $m --steps 20 --warmup 2; done
      prof serve 300 --steps 20 --warmup 2 --reqs-per-conn 512
      prof serve_wide 300 --mode serve_wide --steps 10 --warmup 2 --reqs-per-conn 256 ;;
    pmc_big)  # every counter group (one pass each) for the big kernels: gemm_softmax32 (B = 262,144),
              # softmax_grad_dw (F = 256), softmax_rows MODE 5 + gdw_gemm_dma (F = 1024)
      PMC_BENCHES="gemm_big:--mode gemm --batch 262144 --steps 5 --warmup 1|tsm256:--mode train_softmax --steps 5 --warmup 1|tsm1024:--mode train_softmax --softmax-features 1024 --steps 5 --warmup 1" \
        run pmc_big 1200 bash tools/pmc_profile.sh ;;
    pmc_gemm) PMC_BENCHES="gemm:--mode gemm --steps 5 --warmup 1|gemm_big:--mode gemm --batch 262144 --steps 5 --warmup 1" run pmc_gemm 600 bash tools/pmc_profile.sh ;;
    gemm_ws)  # W-stationary persistent kernel vs the 32x32 kernel: tests, interleaved benches, kernel stats
      MLAPI_GEMM_WS=1 run pytest_gemm 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "gemm or softmax"
      for r in 1 2; do
        for kk in t32 ws; do
          run "gemm_${kk}_b262144_r$r" 120 python -u bench.py --mode gemm --batch 262144 --steps 200 --warmup 10 --gemm-kernel $kk
          run "gemm_${kk}_b65536_r$r" 120 python -u bench.py --mode gemm --batch 65536 --steps 500 --warmup 10 --gemm-kernel $kk
        done
      done
      for r in 1 2; do
        run "bench_train_softmax_t32_r$r" 300 python -u bench.py --mode train_softmax --steps 100 --warmup 10
        MLAPI_GEMM_WS=1 run "bench_train_softmax_ws_r$r" 300 python -u bench.py --mode train_softmax --steps 100 --warmup 10
      done
      prof gemm_ws_b262144 120 --mode gemm --batch 262144 --steps 20 --warmup 2 --gemm-kernel ws
      prof gemm_t32_b262144 120 --mode gemm --batch 262144 --steps 20 --warmup 2 --gemm-kernel t32
      MLAPI_GEMM_WS=1 prof train_softmax_ws 300 --mode train_softmax --steps 20 --warmup 2 ;;
    split_xcd)  # XCD-local vs agent-scope split merge (linear_split.h): tests, interleaved benches, kernel stats
      run pytest_split_xcd 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "linear_split"
      for r in 1 2; do
        for x in 1 0; do
          for B in 32 256 1024 2048; do
            MLAPI_SPLIT_XCD=$x run "gemm_split_xcd${x}_b${B}_r$r" 120 python -u bench.py --mode gemm --batch $B --steps 2000 --warmup 50 --gemm-kernel split
          done
        done
        run "gemm_tiles_b1024_r$r" 120 python -u bench.py --mode gemm --batch 1024 --steps 2000 --warmup 50
      done
      for x in 1 0; do
        MLAPI_SPLIT_XCD=$x prof "split_xcd${x}_b1024" 120 --mode gemm --batch 1024 --steps 300 --warmup 5 --gemm-kernel split --launch eager
        MLAPI_SPLIT_XCD=$x prof "split_xcd${x}_b32" 120 --mode gemm --batch 32 --steps 300 --warmup 5 --gemm-kernel split --launch eager
      done ;;
    gemm_xcd)  # XCD-local vs agent-scope split merge in the tiles kernels (MLAPI_GEMM_XCD=1/0), x2 + kernel stats
      run pytest_gemm_xcd 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "gemm or softmax or rowstat or train"
      for r in 1 2; do
        for x in 1 0; do
          for B in 1024 8192; do
            MLAPI_GEMM_XCD=$x run "gemm_xcd${x}_b${B}_r$r" 120 python -u bench.py --mode gemm --batch $B --steps 2000 --warmup 50
          done
        done
      done
      for x in 1 0; do
        MLAPI_GEMM_XCD=$x prof "gemm_xcd${x}_b1024" 120 --mode gemm --batch 1024 --steps 300 --warmup 5 --launch eager
      done ;;
    split_big)  # class-split kernel vs the tiles kernel at medium batches (B=1024 is BASELINE config 3)
      for r in 1 2; do
        for B in 256 1024 2048; do
          run "gemm_tiles_b${B}_r$r" 120 python -u bench.py --mode gemm --batch $B --steps 2000 --warmup 50
          run "gemm_split_b${B}_r$r" 120 python -u bench.py --mode gemm --batch $B --steps 2000 --warmup 50 --gemm-kernel split
        done
      done ;;
    threads)
      for r in 1 2; do
        for tc in ${THREADS:-10:4 8:6 6:6}; do
          run "sweep_io${tc%%:*}_cl${tc##*:}_r$r" 300 python -u bench.py --steps 60 --warmup 5 \
            --io-threads "${tc%%:*}" --client-threads "${tc##*:}" --c1-requests 1000
        done
      done ;;
    gdw)
      run pytest_gdw 240 python -u -m pytest tests/test_kernels_gpu.py -k "softmax_grad" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
      run gdw_sweep 180 python -u tools/softmax_train_sweep.py ;;
    serve_ab_old)  # interleaved x3 serve bench: ab_old/ (previous build + its bench.py) vs the working tree
      for r in 1 2 3; do
        run "serve_old_r$r" 300 python -c "import sys, runpy; sys.path.insert(0, 'ab_old'); sys.argv = ['bench.py'] + sys.argv[1:]; runpy.run_path('ab_old/bench.py', run_name='__main__')" \
          --steps 100 --warmup 10 ${EXTRA:-}
        run "serve_new_r$r" 300 python -u bench.py --steps 100 --warmup 10 ${EXTRA:-}
      done ;;
    serve_ab3)  # interleaved x2: ab_old/ (previous build) vs the working tree vs the working tree with AB_ENV set
      for r in 1 2; do
        run "serve_old_r$r" 300 python -c "import sys, runpy; sys.path.insert(0, 'ab_old'); sys.argv = ['bench.py'] + sys.argv[1:]; runpy.run_path('ab_old/bench.py', run_name='__main__')" \
          --steps 100 --warmup 10
        run "serve_new_r$r" 300 python -u bench.py --steps 100 --warmup 10
        env ${AB_ENV:-MLAPI_NOTHING=1} timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 > "$O/serve_newenv_r$r.log" 2>&1 \
          || stop "serve_newenv_r$r" $? "$O/serve_newenv_r$r.log"
        tail -1 "$O/serve_newenv_r$r.log" | cut -c1-200
      done ;;
    wide_trace)  # WIDE kernel: in-kernel timeline (tools/wide_trace.py) + rocprofv3 phase durations (tools/wide_probe.py)
      run wide_trace 180 python3 -u tools/wide_trace.py 256 1000 200
      run wide_probe_prof 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/wide_prof" -o prof -- python3 tools/wide_probe.py
      python3 tools/wide_probe_summary.py "$(find "$O/wide_prof" -name '*kernel_trace.csv' -print -quit)" > "$O/wide_probe_summary.txt" 2>&1
      cat "$O/wide_trace.log" "$O/wide_probe_summary.txt" ;;
    bench_abenv)  # AB_VAR=<env var> AB_VALS="<v1> <v2>" BENCH_ARGS="<bench args>": interleaved x2
      for r in 1 2; do
        for v in $AB_VALS; do
          env "$AB_VAR=$v" timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > "$O/bench_${AB_VAR}_${v}_r$r.log" 2>&1 \
            || stop "bench_${AB_VAR}_${v}_r$r" $? "$O/bench_${AB_VAR}_${v}_r$r.log"
          grep '^{' "$O/bench_${AB_VAR}_${v}_r$r.log" | cut -c1-240
        done
      done ;;
    prev_ab)  # interleaved x3: the previous build copied to ab_prev/ vs the working tree, same bench args (PREV_ARGS)
      for r in 1 2 3; do
        run "prev_old_r$r" 300 python -c "import sys, runpy; sys.path.insert(0, 'ab_prev'); sys.argv = ['bench.py'] + sys.argv[1:]; runpy.run_path('bench.py', run_name='__main__')" ${PREV_ARGS}
        run "prev_new_r$r" 300 python -u bench.py ${PREV_ARGS}
      done ;;
    gemm_ab)
      for r in 1 2 3; do
        run "gemm_old_r$r" 120 python -c "import sys, runpy; sys.path.insert(0, 'ab_old'); sys.argv = ['bench.py'] + sys.argv[1:]; runpy.run_path('bench.py', run_name='__main__')" \
          --mode gemm --steps 2000 --warmup 100 ${EXTRA:-}
        run "gemm_new_r$r" 120 python -u bench.py --mode gemm --steps 2000 --warmup 100 ${EXTRA:-}
      done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "SESSION DONE"
