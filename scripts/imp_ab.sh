#!/bin/bash
# IMP lastseen stamping A/B, one box, interleaved rounds:
# HMP against IMP with TIMEOUT (FCGPU_LASTSEEN packet / run / check) at 1,
# 10k and 1M flows; 200-step bench runs, k_rx time per 1M batch from each
# line's roofline.kernel_ms. Logs: gpurun_out/imp_ab/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/imp_ab
mkdir -p "$out"
ROUNDS=${ROUNDS:-2}
declare -A W=([f1]="--flow-capacity 16" [f10k]="--workload c3 --flow-capacity 20000"
              [f1m]="--workload c4 --flow-capacity 2000000")
for r in $(seq 1 "$ROUNDS"); do
  for w in f1 f10k f1m; do
    for v in hmp packet run check; do
      if [ $v = hmp ]; then args="${W[$w]}"; ls=run
      else args="${W[$w]} --flow-manager imp --flow-timeout 1"; ls=$v; fi
      log="$out/r${r}_${w}_${v}.log"
      FCGPU_LASTSEEN=$ls timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 --no-cpu $args > "$log" 2>&1
      rc=$?
      k=$(grep -o '"kernel_ms": [0-9.]*' "$log" | head -1 | cut -d' ' -f2)
      echo "round $r $w $v rc=$rc k_rx_ms=$k"
      if [ $rc -ne 0 ]; then echo "stopping (rc=$rc)"; tail -5 "$log"; exit $rc; fi
    done
  done
done
