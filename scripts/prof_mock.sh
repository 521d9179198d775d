#!/bin/bash
# gprof of the element's host work over the mock library (no GPU touched):
# scripts/prof_mock.sh [THREADS] -> gpurun_out/prof_mock_<T>.txt. Profiling aid.
set -e
cd "$(dirname "$0")/.."
T=${1:-1}
export MOCK_ZEROCOPY=${MOCK_ZEROCOPY:-1}     # the batch size the element runs at on the shared queue (BATCH auto)
D=${TMPDIR:-/tmp}/prof_mock
mkdir -p $D gpurun_out
sed 's/    run("Pass", &floor, err);/    if (getenv("FLOOR")) run("Pass", \&floor, err);/' scripts/mock_element_bench.cc > $D/eb.cc
g++ -O2 -g -pg -std=c++17 -Iinclude -Ifastclick_amd/csrc/host scripts/mock_fcgpu.cc \
    fastclick_amd/csrc/host/fcclick_capi.cc fastclick_amd/csrc/host/pcap_reader.cc $D/eb.cc -o $D/eb_pg -lpthread
(cd $D && ./eb_pg $T auto 0 && gprof -b ./eb_pg gmon.out > flat.txt) 
head -30 $D/flat.txt | cut -c1-200 > gpurun_out/prof_mock_$T.txt
g++ -O3 -std=c++17 -Iinclude -Ifastclick_amd/csrc/host scripts/mock_fcgpu.cc \
    fastclick_amd/csrc/host/fcclick_capi.cc fastclick_amd/csrc/host/pcap_reader.cc scripts/mock_element_bench.cc \
    -o $D/eb -lpthread
for t in 1 16; do $D/eb $t auto 0; done >> gpurun_out/prof_mock_$T.txt
