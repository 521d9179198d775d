set -o pipefail
mkdir -p gpurun_out/impvar
B="python bench.py --steps 200 --warmup 20 --no-cpu"
run() { name=$1; shift; timeout -k 10 180 $B "$@" > gpurun_out/impvar/$name.json 2> gpurun_out/impvar/$name.err || { echo "FAIL $name"; exit 1; }; tail -c 600 gpurun_out/impvar/$name.json; echo; }
run c4_hmp --workload c4 --flow-capacity 2000000
run c4_imp --workload c4 --flow-capacity 2000000 --flow-manager imp
run c4_imp_to --workload c4 --flow-capacity 2000000 --flow-manager imp --flow-timeout 1
run c2_imp_to --workload c2 --flow-capacity 65536 --flow-manager imp --flow-timeout 1
run c3_imp_to --workload c3 --flow-capacity 65536 --flow-manager imp --flow-timeout 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/impvar/prof -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 10 --no-cpu --workload c4 --flow-capacity 2000000 --flow-manager imp --flow-timeout 1 > $GRAFT_REPO_ROOT/gpurun_out/impvar/prof.log 2>&1
