cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for k in 1 2 3; do
  for v in "" "--streams 2" "--streams 2 --fuse 10"; do
    n=$(echo "x$v" | tr -d ' -')
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu $v > gpurun_out/s2f_${n}_$k.log 2>&1 || exit $?
    echo "[$v] $(grep -o '"value": [0-9.]*' gpurun_out/s2f_${n}_$k.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s2f_${n}_$k.log) $(grep -o '"batches_per_launch": [0-9]*' gpurun_out/s2f_${n}_$k.log)"
  done
done
