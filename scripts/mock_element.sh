#!/bin/bash
# Build the element harness against scripts/mock_fcgpu.cc (no GPU) and time its
# host-side work: scripts/mock_element.sh [THREADS [BATCH]]. Profiling aid only.
set -e
cd "$(dirname "$0")/.."
M=${MOCK_DIR:-/tmp/mock}
mkdir -p $M
g++ -O3 -std=c++17 -fPIC -shared -Iinclude scripts/mock_fcgpu.cc -Wl,-soname,libfcgpu_mock.so -o $M/libfcgpu_mock.so
g++ -O3 -std=c++17 -fPIC -shared -Iinclude fastclick_amd/csrc/host/fcclick_capi.cc fastclick_amd/csrc/host/pcap_reader.cc \
    $M/libfcgpu_mock.so -Wl,-rpath,$M -o $M/libfcclick_mock.so
g++ -O3 -std=c++17 -Iinclude scripts/mock_element_bench.cc $M/libfcclick_mock.so -Wl,-rpath,$M -o $M/element_bench
[ -n "$NO_RUN" ] || $M/element_bench "${1:-1}" "${2:-16384}"
