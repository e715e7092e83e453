#!/bin/bash
# A/B builds of the NTT switches: lib/ab_<name>.so with ntt.hip compiled under
# the given -D flags and every other object from the regular build.
# usage: build_ab.sh name "-DFHE_ASM_ADD=0 ..." [name2 "flags2" ...]
set -e
cd "$(dirname "$0")/../fhe-sorting_amd"
make -s -j8 lib/libfhesort.so >/dev/null
OBJS=$(ls build/device/kernels.o build/device/encode.o build/engine/engine.o build/host/*.o build/algo/*.o build/wire/*.o build/capi/*.o)
while [ $# -ge 2 ]; do
  mkdir -p build/ab
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-function $2 -c csrc/device/ntt.hip -o build/ab/ntt_$1.o 2>/dev/null
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/ab_$1.so build/ab/ntt_$1.o $OBJS -L/opt/rocm/lib -lrccl -lamdhip64 -Wl,-rpath,/opt/rocm/lib
  echo "lib/ab_$1.so: $2"
  shift 2
done
