#!/bin/bash
# Development A/B builds of the LP kernel: tools/build_variants.sh name "-DFLAG ..." [name "-D..."]...
# Compiles lp_hyper.hip with the flags and links it with the other objects of the default build
# into sqlp_amd/libtwosd_hip_<name>.so (select with TWOSD_LIB=<name>).
set -e
cd "$(dirname "$0")/../sqlp_amd/csrc"
make -s build/api.hip.o build/pool_sort.hip.o build/sampler.hip.o build/dvs_kernel.hip.o build/cut_kernel.hip.o build/vkey.hip.o build/pool_gpu.hip.o build/host_basis.cpp.o
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -Wall -Wno-unused-function -Wno-unused-value -Wno-unused-result"
OTHERS="build/api.hip.o build/pool_sort.hip.o build/sampler.hip.o build/dvs_kernel.hip.o build/cut_kernel.hip.o build/vkey.hip.o build/pool_gpu.hip.o build/host_basis.cpp.o"
mkdir -p build_v
pids=()
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  ( /opt/rocm/bin/hipcc $FL $flags -c lp_hyper.hip -o build_v/lp_hyper_$name.o &&
    /opt/rocm/bin/hipcc $FL -shared -pthread -o ../libtwosd_hip_$name.so $OTHERS build_v/lp_hyper_$name.o ) &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
exit $rc
