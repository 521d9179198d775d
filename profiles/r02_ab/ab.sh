# A/B on one box: the round's flow-table variants, old (ab_old/) vs current
set -o pipefail
mkdir -p gpurun_out/ab
for v in "--flow-capacity 1" "--workload c4 --flow-capacity 2000000"; do
  n=$(echo "$v" | tr -d ' -' | cut -c1-40)
  for side in old new old new; do
    if [ $side = old ]; then d=ab_old; x="--streams 1"; else d=.; x="--streams 1 --fuse 1"; fi
    (cd $d && timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu $x $v) > gpurun_out/ab/${side}_$n.json 2>/dev/null || exit 1
    python -c "import json; l=json.loads(open('gpurun_out/ab/${side}_$n.json').read().strip().splitlines()[-1]); print('$side $n', l['value'], l['roofline']['kernel_ms'])"
  done
done
