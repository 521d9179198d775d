#!/bin/bash
# round 3, session 4: the element's host threads vs CPU placement (NUMA node of
# the GPU, SMT siblings, CCDs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
{ lscpu; echo; numactl --hardware 2>&1; echo; cat /sys/fs/cgroup/cpuset.cpus.effective 2>&1; echo;
  for d in /sys/class/drm/card*/device; do echo "$d numa_node=$(cat $d/numa_node 2>/dev/null) local_cpulist=$(cat $d/local_cpulist 2>/dev/null)"; done;
  rocm-smi --showtoponuma 2>&1 | head -30; } > gpurun_out/topo.txt 2>&1
NODE=$(for d in /sys/class/drm/card*/device; do n=$(cat $d/numa_node 2>/dev/null); [ -n "$n" ] && [ "$n" -ge 0 ] && echo $n && break; done)
echo "gpu numa node: $NODE" >> gpurun_out/topo.txt
LOCAL=$(cat /sys/devices/system/node/node${NODE:-0}/cpulist 2>/dev/null)
echo "local cpus: $LOCAL" >> gpurun_out/topo.txt
for t in 1 4 8; do
  timeout -k 10 120 python scripts/element_threads.py $t > /tmp/x.json 2>&1 && echo "free $(cat /tmp/x.json)" >> gpurun_out/el_place.log || exit $?
done
# the node's first cores, one thread per physical core (no SMT siblings assumed: lowest-numbered CPUs)
FIRST=$(python3 -c "
import sys
s='$LOCAL'.split(',')[0]
a,b=(s.split('-')+[s])[:2]
print(f'{a}-{int(a)+15}')")
echo "pinned set: $FIRST" >> gpurun_out/topo.txt
for t in 1 4 8 16; do
  timeout -k 10 120 taskset -c $FIRST python scripts/element_threads.py $t > /tmp/x.json 2>&1 && echo "node_local $(cat /tmp/x.json)" >> gpurun_out/el_place.log || exit $?
done
