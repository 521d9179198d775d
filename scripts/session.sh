#!/bin/bash
# One GPU-box session of named steps (STEPS="a,b,c"). Every GPU step runs under
# its own time limit; the session stops at the first step that faults, aborts
# or times out (any exit code other than 0/1). Logs: gpurun_out/<step>.log,
# rocprofv3 output: gpurun_out/prof_<step>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"; local t0=$SECONDS
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc wall=$((SECONDS - t0))s"; tail -n 3 "gpurun_out/$name.log" | cut -c1-1500
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
kt() {  # name timeout bench-args...: kernel trace + stats of a bench command
  local name=$1 t=$2; shift 2
  step "$name" "$t" rocprofv3 --kernel-trace --stats -f csv -d "gpurun_out/prof_$name" -o run -- python3 bench.py "$@"
}
pmc() {  # name counters... -- bench-args...
  local name=$1; shift
  local ctrs=()
  while [ "$1" != "--" ]; do ctrs+=("$1"); shift; done; shift
  step "$name" 120 rocprofv3 --pmc "${ctrs[@]}" --kernel-include-regex k_rx -f csv -d "gpurun_out/prof_$name" -o run -- python3 bench.py "$@"
}
pmcv() {  # tag bench-args...: the three PMC passes of one variant, one batch per launch
  local tag=$1; shift
  local a="--steps 40 --warmup 4 --no-cpu --no-timing --streams 1 --fuse 1"
  pmc "pmc_fetch_$tag" FETCH_SIZE -- $a "$@" &&
  pmc "pmc_write_$tag" WRITE_SIZE -- $a "$@" &&
  pmc "pmc_ea_$tag" TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -- $a "$@"
}
var() {  # 200-step run of one variant (fused launches, the default layout)
  local n; n=$(echo "$*" | tr -d ' -' | cut -c1-48)
  step "var_$n" 300 python bench.py --steps 200 --warmup 20 --no-cpu "$@"
}
DRV="--gpus 1 --steps 20 --warmup 5"
IFS=, read -ra ST <<< "${STEPS:-tests,smoke,bench}"
for s in "${ST[@]}"; do
  case $s in
    tests) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    tests_sel) step pytest_sel 600 python -u -m pytest $SEL -m gpu -x -v --timeout 120 --timeout-method thread ;;
    tests_flow) step pytest_flow 600 python -u -m pytest tests/test_flow.py tests/test_flow_imp.py -m gpu -x -v --timeout 120 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 300 python bench.py $DRV ;;
    bench_s1) step bench_s1 300 python bench.py $DRV --streams 1 --fuse 1 --no-cpu ;;
    bench_long) step bench_long 300 python bench.py --steps 200 --warmup 20 --no-cpu ;;
    bench_long_s1) step bench_long_s1 300 python bench.py --steps 200 --warmup 20 --no-cpu --streams 1 --fuse 1 ;;
    kt_drv) kt kt_drv 300 $DRV --no-cpu ;;
    kt_drv_s1) kt kt_drv_s1 300 $DRV --no-cpu --streams 1 --fuse 1 ;;
    kt_long) kt kt_long 300 --steps 200 --warmup 20 --no-cpu ;;
    kt_w40) kt kt_w40 300 --gpus 1 --steps 20 --warmup 40 --no-cpu ;;
    kt_notime) kt kt_notime 300 $DRV --no-cpu --no-timing ;;
    kt_nopf) kt kt_nopf 300 $DRV --no-cpu --prefault 0 ;;
    kt_nopf_s1) kt kt_nopf_s1 300 $DRV --no-cpu --prefault 0 --streams 1 ;;
    kt_notime_s1) kt kt_notime_s1 300 $DRV --no-cpu --no-timing --streams 1 ;;
    kt_w40_s1) kt kt_w40_s1 300 --gpus 1 --steps 20 --warmup 40 --no-cpu --streams 1 ;;
    diag) for k in 1 2 3; do FCGPU_BENCH_DIAG=1 step "diag$k" 300 python bench.py $DRV --no-cpu; done ;;
    bench2) step bench2 300 python bench.py $DRV --no-cpu ;;
    bench3) step bench3 300 python bench.py $DRV --no-cpu ;;
    # PMC per batch: one batch per launch (--fuse 1)
    pmc) pmc pmc_fetch FETCH_SIZE -- --steps 40 --warmup 4 --no-cpu --no-timing --streams 1 --fuse 1
         pmc pmc_write WRITE_SIZE -- --steps 40 --warmup 4 --no-cpu --no-timing --streams 1 --fuse 1
         pmc pmc_ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -- --steps 40 --warmup 4 --no-cpu --no-timing --streams 1 --fuse 1 ;;
    bench_s2) step bench_s2 300 python bench.py $DRV --streams 2 --fuse 1 --no-cpu ;;
    bench_long_s2) step bench_long_s2 300 python bench.py --steps 200 --warmup 20 --no-cpu --streams 2 --fuse 1 ;;
    kt_drv_s2) kt kt_drv_s2 300 $DRV --no-cpu --streams 2 --fuse 1 ;;
    pmc_var) pmc pmc_fetch_fb128 FETCH_SIZE -- --steps 40 --warmup 4 --no-cpu --no-timing --streams 1 --fuse 1 --frame-bytes 128
             pmc pmc_fetch_fb1500 FETCH_SIZE -- --steps 40 --warmup 4 --no-cpu --no-timing --streams 1 --fuse 1 --frame-bytes 1500
             pmc pmc_fetch_c3 FETCH_SIZE -- --steps 40 --warmup 4 --no-cpu --no-timing --streams 1 --fuse 1 --workload c3
             pmc pmc_fetch_c4flow FETCH_SIZE -- --steps 40 --warmup 4 --no-cpu --no-timing --workload c4 --flow-capacity 2000000
             pmc pmc_ea_c4flow TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -- --steps 40 --warmup 4 --no-cpu --no-timing --workload c4 --flow-capacity 2000000
             pmc pmc_write_c4flow WRITE_SIZE -- --steps 40 --warmup 4 --no-cpu --no-timing --workload c4 --flow-capacity 2000000 ;;
    crcvar) for v in "--classify lbcrc" "--workload c4 --classify lbcrc"; do
                n=$(echo "$v" | tr -d ' -' | cut -c1-40)
                step "var_$n" 300 python bench.py --steps 200 --warmup 20 --no-cpu $v
              done ;;
    flowvar) for v in "--flow-capacity 1" "--workload c3 --flow-capacity 20000" "--workload c4 --flow-capacity 2000000" \
                      "--partition global" "--classify ipclass16" "--workload c4 --classify ipclass16"; do
                n=$(echo "$v" | tr -d ' -' | cut -c1-40)
                step "var_$n" 300 python bench.py --steps 200 --warmup 20 --no-cpu $v
              done ;;
    sweep) for fb in 64 128 256 512 1024 1500; do
             step "sweep_$fb" 300 python bench.py --steps 200 --warmup 20 --no-cpu --frame-bytes $fb
             step "sweep_s2_$fb" 300 python bench.py --steps 200 --warmup 20 --no-cpu --frame-bytes $fb --streams 2 --fuse 1
           done ;;
    variants) for v in "--workload c3" "--workload c4" "--workload c5" "--classify ipclass16" \
                       "--workload c4 --classify ipclass16" "--flow-capacity 1" "--workload c3 --flow-capacity 20000" \
                       "--workload c4 --flow-capacity 2000000" "--partition global" "--no-perm" "--shard strong"; do
                n=$(echo "$v" | tr -d ' -' | cut -c1-40)
                step "var_$n" 300 python bench.py --steps 200 --warmup 20 --no-cpu $v
              done ;;
    host) step host_rate 600 python scripts/host_rate.py ;;
    host_q16) GPU_MAX_HW_QUEUES=16 step host_rate_q16 600 python scripts/host_rate.py ;;
    kgather) step kgather 180 ./scripts/kgather 64 ;;
    khg) for a in "16384 64 0 0" "16384 32 0 16" "16384 48 0 16" "262144 64 0 0" "262144 32 0 16" "262144 48 0 16"; do
           n=$(echo "$a" | tr ' ' _)
           step "khg_$n" 120 ./scripts/khostgather $a
         done ;;
    kt_flow) kt kt_flow_c2 300 --steps 200 --warmup 20 --no-cpu --flow-capacity 1 &&
             kt kt_flow_c3 300 --steps 200 --warmup 20 --no-cpu --workload c3 --flow-capacity 20000 &&
             kt kt_flow_c4 300 --steps 200 --warmup 20 --no-cpu --workload c4 --flow-capacity 2000000 ;;
    latency) step latency 120 python scripts/latency_probe.py ;;
    crossover) step crossover 1000 python -u scripts/crossover.py ;;
    crossover3) step crossover 600 python -u scripts/crossover.py --threads 8,16 &&
                step crossover_b 600 python -u scripts/crossover.py --threads 8,16 &&
                step crossover_c 600 python -u scripts/crossover.py --threads 8,16 ;;
    crossover2) step crossover_b 600 python -u scripts/crossover.py --threads 8,16 &&
                step crossover_c 600 python -u scripts/crossover.py --threads 8,16 ;;
    crossover16) step crossover16 600 python -u scripts/crossover.py --threads 8,16 --no-cpu ;;
    mock_ab) step mock_ab 600 bash scripts/mock_ab_box.sh ;;
    # the element's host-side ceiling (mock GPU library, zero-copy staging as on
    # the box at >= 4 threads), pushed for 2 s, beside the real element
    mock_timed) step mock_timed 600 bash -c 'for r in 1 2; do for t in 1 8 12 16; do MOCK_ZEROCOPY=1 timeout -k 5 60 scripts/mock/base/element_bench $t auto 0 || exit $?; timeout -k 5 120 python scripts/element_threads.py $t || exit $?; done; done' ;;
    el_sweep) step el_sweep 900 bash scripts/el_sweep.sh 3 ;;
    el_sweep2) BATCHES="4096 8192 16384" SLOTS_LIST=2 step el_sweep2 900 bash scripts/el_sweep.sh 3 16 8 4 ;;
    # the job's 16-CPU cgroup quota is shared with the HIP runtime's own threads
    el_quota) step el_quota 900 bash -c 'for r in 1 2 3; do for t in 16 15 14 12; do timeout -k 5 120 python scripts/element_threads.py $t || exit $?; done; done' ;;
    # the flow re-shard kernels: GPU tests, rates, kernel trace
    exchange) step pytest_exchange 600 python -u -m pytest tests/test_exchange.py tests/test_dist.py -m gpu -x -v --timeout 120 --timeout-method thread &&
              step exchange_rate 300 python scripts/exchange_rate.py &&
              step kt_exchange 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_kt_exchange -o run -- python3 scripts/exchange_rate.py --reps 20 ;;
    # CPU time the element's process takes (user + sys vs wall) and the job
    # cgroup's CFS throttling around 8- and 16-thread runs
    el_cpu) step el_cpu 600 bash -c 'cat /sys/fs/cgroup/cpu.max 2>/dev/null; for t in 8 12 16; do cat /sys/fs/cgroup/cpu.stat 2>/dev/null | tr "\n" " "; echo; timeout -k 5 120 python scripts/element_threads.py $t || exit $?; done; cat /sys/fs/cgroup/cpu.stat 2>/dev/null | tr "\n" " "; echo' ;;
    # SLOTS 2 vs 3 at 12 / 16 threads, pushed for 2 s, three interleaved rounds
    el_slots) step el_slots 900 bash -c 'for r in 1 2 3; do for t in 12 16; do for sl in 2 3; do timeout -k 5 120 python scripts/element_threads.py $t 0 auto $sl || exit $?; done; done; done' ;;
    # compact records packed 8 B apart (in-tree) against 16 B (scripts/mock/align16)
    el_align) ALT=scripts/mock/align16/libfcclick.so step el_align 900 bash scripts/el_ab_lib.sh 3 ;;
    # 4-B descriptors (in-tree) against 8-B (scripts/mock/desc8)
    el_desc) ALT=scripts/mock/desc8/libfcclick.so step el_desc 900 bash scripts/el_ab_lib.sh 3 ;;
    # 8-B IPv4 annotations (in-tree) against 16-B (scripts/mock/anno16)
    el_anno) ALT=scripts/mock/anno16/libfcclick.so step el_anno 900 bash scripts/el_ab_lib.sh 3 ;;
    # the element's defaults at 1-16 threads, two interleaved rounds
    el_default) step el_default 600 bash -c 'for r in 1 2; do for t in 1 2 4 8 12 16; do timeout -k 5 120 python scripts/element_threads.py $t || exit $?; done; done' ;;
    # the element at 16 threads (default BATCH/ZEROCOPY/SLOTS): rate, then a kernel trace
    el16) step el16 300 python scripts/element_threads.py 16 &&
          step el16_s3 300 python scripts/element_threads.py 16 0 auto 3 &&
          step el16_b8k 300 python scripts/element_threads.py 16 8192 auto 2 &&
          step el8 300 python scripts/element_threads.py 8 &&
          step kt_el16 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_kt_el16 -o run -- python3 scripts/element_threads.py 16 ;;
    dist2) step dist2 300 python bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 --no-cpu ;;
    # the driver's 8-rank command shape, rehearsed on one GPU (gloo: RCCL needs a GPU per rank)
    dist8) step dist8_weak 900 python bench.py --gpus 8 --backend gloo --steps 20 --warmup 5 --no-cpu &&
           step dist8_strong 900 python bench.py --gpus 8 --backend gloo --shard strong --steps 20 --warmup 5 --no-cpu ;;
    # round 5: every variant on the final kernel sources, 200 steps
    r5var) var && var --workload c3 && var --workload c3 --layout split && var --workload c4 &&
           var --workload c5 && var --workload c5 --layout split && var --classify ipclass16 &&
           var --workload c4 --classify ipclass16 && var --classify ipclass16 --program-jit 0 &&
           var --classify lbcrc && var --l4 udp && var --rewrite && var --partition global && var --no-perm &&
           var --errors 0.01 && var --shard strong && var --flow-capacity 1 &&
           var --workload c3 --flow-capacity 20000 && var --workload c4 --flow-capacity 2000000 &&
           var --workload c4 --flow-capacity 2000000 --flow-manager imp --flow-timeout 1 &&
           var --classify lbtable && var --classify haship ;;
    r5flowvar) var --flow-capacity 1 && var --workload c3 --flow-capacity 20000 &&
               var --workload c4 --flow-capacity 2000000 &&
               var --workload c4 --flow-capacity 2000000 --flow-manager imp --flow-timeout 1 && var ;;
    r5sweep) for fb in 128 256 512 1024 1500; do var --frame-bytes $fb && var --frame-bytes $fb --layout split || exit $?; done ;;
    # round 5: PMC traffic of the variants (profiles/pmc_traffic.json, scripts/pmc_traffic.py)
    r5pmc) pmcv c2 && pmcv c3 --workload c3 && pmcv c3split --workload c3 --layout split &&
           pmcv c5 --workload c5 && pmcv c5split --workload c5 --layout split ;;
    r5pmc2) pmcv c4 --workload c4 && pmcv c4flow --workload c4 --flow-capacity 2000000 &&
            pmcv ipc16 --classify ipclass16 && pmcv l4udp --l4 udp && pmcv rewrite --rewrite &&
            pmcv fb1500 --frame-bytes 1500 && pmcv fb1500split --frame-bytes 1500 --layout split ;;
    # round 5: the flow re-shard inside the bench (N = 1 on the GPU, the 8-rank command shape over gloo)
    reshard) step reshard1 300 python bench.py --flow-reshard --workload c4 --steps 50 --warmup 5 --no-cpu &&
             step reshard8 900 python bench.py --gpus 8 --backend gloo --flow-reshard --workload c4 --steps 5 --warmup 1 --no-cpu ;;
    xbuild) step pytest_xbuild 600 python -u -m pytest tests/test_exchange.py tests/test_bench_dist.py tests/test_dist.py -m gpu -x -v --timeout 120 --timeout-method thread &&
            step exchange_rate 300 python scripts/exchange_rate.py &&
            step kt_exchange 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_kt_exchange -o run -- python3 scripts/exchange_rate.py --reps 20 ;;
    xrate) step exchange_rate 300 python scripts/exchange_rate.py --reps 30 &&
           step kt_exchange 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_kt_exchange -o run -- python3 scripts/exchange_rate.py --reps 20 ;;
    # LB_MODE cst_hash_agg (CLS_LB_TABLE) beside the headline's LB_MODE hash
    r5lbt) var && var --classify lbtable && var --workload c4 --classify lbtable &&
           var --workload c5 --layout split --classify lbtable && var --classify lbcrc ;;
    # A/B of the library in fastclick_amd/lib/ab/libfcgpu_old.so against the tree's, interleaved
    autoab) for k in 1 2; do
              for w in "--workload c5" "--workload c5 --layout split" "--workload c2"; do
                n=$(echo "$w" | tr -d ' -' | cut -c1-40)
                FCGPU_LIB=fastclick_amd/lib/ab/libfcgpu_old.so step "ab_old_${n}_$k" 300 python bench.py --steps 200 --warmup 20 --no-cpu $w &&
                step "ab_new_${n}_$k" 300 python bench.py --steps 200 --warmup 20 --no-cpu $w || exit $?
              done
            done ;;
    # the same A/B over the variants in $ABV ("|"-separated bench options)
    abv) IFS='|' read -ra VV <<< "$ABV"
         for k in 1 2; do
           for w in "${VV[@]}"; do
             n=$(echo "$w" | tr -d ' -' | cut -c1-40)
             FCGPU_LIB=fastclick_amd/lib/ab/libfcgpu_old.so step "ab_old_${n}_$k" 300 python bench.py --steps 200 --warmup 20 --no-cpu $w &&
             step "ab_new_${n}_$k" 300 python bench.py --steps 200 --warmup 20 --no-cpu $w || exit $?
           done
         done ;;
    # round 6: the fixed-capacity re-shard (no host sync per step) against the counted one, interleaved;
    # a forced-overflow run (every step replayed); the 8-rank command shape over gloo
    r6reshard) for k in 1 2; do
                 step "reshard1_fixed_$k" 300 python bench.py --flow-reshard --workload c4 --steps 50 --warmup 5 --no-cpu &&
                 step "reshard1_counted_$k" 300 python bench.py --flow-reshard --workload c4 --steps 50 --warmup 5 --no-cpu --reshard-exchange counted || exit $?
               done &&
               step reshard1_overflow 300 python bench.py --flow-reshard --workload c4 --steps 20 --warmup 2 --no-cpu --reshard-slack 0.5 &&
               step reshard8_fixed 900 python bench.py --gpus 8 --backend gloo --flow-reshard --workload c4 --steps 5 --warmup 1 --no-cpu ;;
    # round 6: the build's scan inside k_xbtile (lib/ab/libfcgpu_old.so: the three-launch build), interleaved
    r6xbuild) for k in 1 2; do
                FCGPU_LIB=fastclick_amd/lib/ab/libfcgpu_old.so step "xrate_old_$k" 300 python scripts/exchange_rate.py --reps 30 &&
                step "xrate_new_$k" 300 python scripts/exchange_rate.py --reps 30 || exit $?
              done ;;
    # round 6: the fixed re-shard's host time per stage and its kernel trace
    r6reshost) FCGPU_RESHARD_HOST=1 step reshard1_fixed_host 300 python bench.py --flow-reshard --workload c4 --steps 50 --warmup 5 --no-cpu &&
               kt kt_reshard_fixed 300 --flow-reshard --workload c4 --steps 10 --warmup 2 --no-cpu ;;
    # round 6: the final re-shard rates (fixed and counted interleaved, host times, overflow, 8-rank shape)
    r6reshard2) for k in 1 2 3; do
                  FCGPU_RESHARD_HOST=1 step "reshard1_fixed_f$k" 300 python bench.py --flow-reshard --workload c4 --steps 50 --warmup 5 --no-cpu &&
                  step "reshard1_counted_f$k" 300 python bench.py --flow-reshard --workload c4 --steps 50 --warmup 5 --no-cpu --reshard-exchange counted || exit $?
                done &&
                step reshard1_overflow_f 300 python bench.py --flow-reshard --workload c4 --steps 20 --warmup 2 --no-cpu --reshard-slack 0.5 &&
                step reshard8_fixed_f 900 python bench.py --gpus 8 --backend gloo --flow-reshard --workload c4 --steps 5 --warmup 1 --no-cpu ;;
    # round 6: k_xbuild's copy loop, 4 / 8 chunks in flight per lane, plain / non-temporal source loads
    r6xcopy) for k in 1 2; do
               for v in 4 8 4nt 8nt; do
                 FCGPU_XBUILD=$v step "xcopy_${v}_$k" 300 python scripts/exchange_rate.py --reps 30 || exit $?
               done
             done ;;
    # round 6: the wire layouts' own ceiling (bare window gather vs k_rx, same box)
    r6gather) step gather_bound 600 python scripts/gather_bound.py ;;
    r6hwq) for r in 1 2; do for c in 4:4 8:8 16:16 4:8; do
             ns=${c%%:*}; hq=${c##*:}
             FCGPU_AGG_STREAMS=$ns GPU_MAX_HW_QUEUES=$hq step hwq_s${ns}_q${hq}_$r 120 python scripts/element_threads.py 16 || exit 1
           done; done ;;
    r6agg) for r in 1 2 3; do for a in 4 8 2; do
             FCGPU_AGG_LAUNCH=$a step agg${a}_$r 300 python scripts/crossover.py --chains base,udp --threads 16 --no-cpu || exit 1
           done; done ;;
    r6prog) for r in 1 2 3; do
              FCCLICK_LIB=fastclick_amd/lib/ab/libfcclick_prev.so step pg_prev_$r 300 python scripts/crossover.py --chains prog16 --threads 8,16 --no-cpu || exit 1
              step pg_new_$r 300 python scripts/crossover.py --chains prog16 --threads 8,16 --no-cpu || exit 1
            done ;;
    r6fbatch) for r in 1 2; do
                step fb_flow_$r 300 python scripts/element_batch_sweep.py flow20k 16 auto,4096,16384,32768,65536 || exit 1
                step fb_base_$r 300 python scripts/element_batch_sweep.py base 16 auto,4096,16384 || exit 1
              done ;;
    r6elab) for r in 1 2 3; do
              FCCLICK_LIB=fastclick_amd/lib/ab/libfcclick_old.so step el_old_$r 300 python scripts/crossover.py --chains base,udp --threads 8,16 --no-cpu || exit 1
              step el_new_$r 300 python scripts/crossover.py --chains base,udp --threads 8,16 --no-cpu || exit 1
            done &&
            for r in 1 2; do step el_cpu_$r 300 python scripts/crossover.py --chains base,udp --threads 16 --no-gpu || exit 1; done ;;
    r6cbatch) for r in 1 2; do for t in 1 2 3; do for b in 16384 8192 4096; do
                step cb_t${t}_b${b}_$r 120 python scripts/element_threads.py $t $b false || exit 1
              done; done; done ;;
    r6stages) for r in 1 2; do for st in 1 0; do
                FCGPU_RESHARD_STAGES=$st step reshard_st${st}_$r 300 python bench.py --flow-reshard --workload c4 --steps 50 --warmup 5 --no-cpu || exit 1
              done; done &&
              FCGPU_RESHARD_STAGES=0 FCGPU_RESHARD_HOST=1 step reshard_host 300 python bench.py --flow-reshard --workload c4 --steps 50 --warmup 5 --no-cpu ;;
    r6cache) for r in 1 2; do for nb in 1 2 3 16; do
               step cache_nb${nb}_$r 300 python bench.py --nbuf $nb --steps 200 --warmup 20 --no-cpu || exit 1
               step cache20_nb${nb}_$r 300 python bench.py --nbuf $nb --no-cpu || exit 1
             done; done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
exit 0
