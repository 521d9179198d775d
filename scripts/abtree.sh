# interleaved 200-step runs: the side tree's build (ab_tree/, another commit),
# the same with FCGPU_LIB=ab_tree/fastclick_amd/lib/libfcgpu_pad.so, and this tree
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for k in 1 2 3; do
  (cd ab_tree && timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu > ../gpurun_out/abt_old_$k.log 2>&1) || exit $?
  if [ -f ab_tree/fastclick_amd/lib/libfcgpu_pad.so ]; then
    (cd ab_tree && FCGPU_LIB=fastclick_amd/lib/libfcgpu_pad.so timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu > ../gpurun_out/abt_pad_$k.log 2>&1) || exit $?
  fi
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu > gpurun_out/abt_new_$k.log 2>&1 || exit $?
  echo "round $k done"
done
