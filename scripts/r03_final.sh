#!/bin/bash
# Round 3 evidence session (profiles/r03_final/): every GPU step under its own
# time limit, stopping at the first step that faults, aborts or times out.
#   STEPS=a,b,c bash scripts/r03_final.sh      (default: all, in this order)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 "gpurun_out/$name.log" | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
kt() {  # name timeout bench-args...
  local name=$1 t=$2; shift 2
  step "$name" "$t" rocprofv3 --kernel-trace --stats -f csv -d "gpurun_out/prof_$name" -o run -- python3 bench.py "$@"
}
pmc() {  # name counters... -- bench-args...
  local name=$1; shift
  local ctrs=()
  while [ "$1" != "--" ]; do ctrs+=("$1"); shift; done; shift
  echo "== $name"; timeout -s KILL 120 rocprofv3 --pmc "${ctrs[@]}" --kernel-include-regex k_rx -f csv \
      -d "gpurun_out/$name" -o run -- python3 bench.py "$@" > "gpurun_out/$name.log" 2>&1 || { echo "stopping after $name"; exit 3; }
}
DRV="--gpus 1 --steps 20 --warmup 5"
V="--steps 200 --warmup 20 --no-cpu"
ONE="--steps 40 --warmup 4 --no-cpu --no-timing --streams 1 --fuse 1"
IFS=, read -ra ST <<< "${STEPS:-tests,smoke,bench,variants,strong,sweep,kt,pmc,host,dist}"
for s in "${ST[@]}"; do
  case $s in
    tests) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 300 python bench.py $DRV
           step bench2 300 python bench.py $DRV --no-cpu
           step bench3 300 python bench.py $DRV --no-cpu
           step bench_long 300 python bench.py --steps 200 --warmup 20 --no-cpu ;;
    variants)
      for v in "--workload c3" "--workload c4" "--workload c5" "--classify ipclass16" "--classify ipclass16 --program-jit 0" \
               "--workload c4 --classify ipclass16" "--classify lbcrc" "--flow-capacity 1" \
               "--workload c3 --flow-capacity 20000" "--workload c4 --flow-capacity 2000000" \
               "--workload c4 --flow-capacity 2000000 --flow-manager imp --flow-timeout 1" \
               "--partition global" "--no-perm" "--errors 0.01" "--workload c4 --errors 0.01" \
               "--l4 udp" "--rewrite" "--nbuf 1"; do
        n=$(echo "$v" | tr -d ' -' | cut -c1-48)
        step "var_$n" 300 python bench.py $V $v
      done ;;
    strong)
      for p in 1048576 524288 262144 131072; do
        step "strong_drv_$p" 300 python bench.py $DRV --no-cpu --shard strong --packets $p
        step "strong_long_$p" 300 python bench.py $V --shard strong --packets $p
      done ;;
    sweep) for fb in 64 128 256 512 1024 1500; do step "sweep_$fb" 300 python bench.py $V --frame-bytes $fb; done ;;
    kt) kt kt_drv 300 $DRV --no-cpu
        kt kt_long 300 --steps 200 --warmup 20 --no-cpu
        kt kt_strong131k 300 $DRV --no-cpu --shard strong --packets 131072 ;;
    pmc) pmc pmc_fetch FETCH_SIZE -- $ONE
         pmc pmc_write WRITE_SIZE -- $ONE
         pmc pmc_ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_DRAM_sum -- $ONE
         pmc pmc_fetch_strong131k FETCH_SIZE -- $ONE --shard strong --packets 131072
         for w in c3 c5; do
           pmc pmc_ea_$w TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_DRAM_sum -- $ONE --workload $w
         done
         pmc pmc_ea_c4flow TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_DRAM_sum -- \
             --steps 40 --warmup 4 --no-cpu --no-timing --workload c4 --flow-capacity 2000000 ;;
    host) step host_rate 600 python scripts/host_rate.py
          step host_threads 600 python scripts/host_rate.py threads
          step host_span 300 python scripts/host_rate.py span ;;
    dist) step dist2 300 python bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 --no-cpu
          step dist2_strong 300 python bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 --no-cpu --shard strong ;;
    latency) step latency 120 python scripts/latency_probe.py
             step kargs 60 ./scripts/kargs ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
exit 0
