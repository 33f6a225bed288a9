#!/bin/bash
# Development A/B builds: tools/build_variants.sh [-f source.hip] name "-DFLAG ..." [name "-D..."]...
# Compiles the source (default lp_hyper.hip) with the flags and links it with the other objects of
# the default build into sqlp_amd/libtwosd_hip_<name>.so (select with TWOSD_LIB=<name>).
set -e
cd "$(dirname "$0")/../sqlp_amd/csrc"
SRC=lp_hyper.hip
if [ "$1" = "-f" ]; then SRC=$2; shift 2; fi
ALL="api.hip lp_hyper.hip pool_sort.hip sampler.hip dvs_kernel.hip cut_kernel.hip vkey.hip pool_gpu.hip"
OTHERS="build/host_basis.cpp.o"
for f in $ALL; do [ "$f" = "$SRC" ] || OTHERS="$OTHERS build/$f.o"; done
make -s $OTHERS
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -Wall -Wno-unused-function -Wno-unused-value -Wno-unused-result"
mkdir -p build_v
pids=()
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  ( /opt/rocm/bin/hipcc $FL $flags -c $SRC -o build_v/${SRC%.hip}_$name.o &&
    /opt/rocm/bin/hipcc $FL -shared -pthread -o ../libtwosd_hip_$name.so $OTHERS build_v/${SRC%.hip}_$name.o ) &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
exit $rc
