# bench.py over several library builds of the same ABI, interleaved:
#   LIBS="old tpw1024 tpw512" ARGS="--partition global --fuse 1" bash scripts/libab.sh
# (fastclick_amd/lib/ab/libfcgpu_<name>.so; "tree" = the in-tree build)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for k in 1 2; do
  for v in $LIBS; do
    lib=fastclick_amd/lib/ab/libfcgpu_$v.so
    [ "$v" = tree ] && lib=fastclick_amd/lib/libfcgpu.so
    IFS='|' read -ra AA <<< "$ARGS"
    for a in "${AA[@]}"; do
      n=$(echo "$a" | tr -d ' -' | cut -c1-40)
      FCGPU_LIB=$lib timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu $a > gpurun_out/lab_${v}_${n}_$k.log 2>&1 || exit $?
    done
  done
  echo "round $k done"
done
