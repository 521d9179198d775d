# exchange_rate.py for the builds in fastclick_amd/lib/ab/ (base, old) and the tree's, interleaved
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for k in 1 2; do
  for v in base old; do
    FCGPU_LIB=fastclick_amd/lib/ab/libfcgpu_$v.so timeout -k 10 300 python scripts/exchange_rate.py --reps 30 > gpurun_out/xab_${v}_$k.log 2>&1 || exit $?
  done
  timeout -k 10 300 python scripts/exchange_rate.py --reps 30 > gpurun_out/xab_new_$k.log 2>&1 || exit $?
  echo "round $k done"
done
