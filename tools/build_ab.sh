#!/bin/bash
# Build A/B diagnostic libraries against the current C-ABI object:
#   tools/build_ab.sh name:-DFLAG ... [rev:<git-rev>]
# (flags that change results, -DPECH_AB_NOLDS / -DPECH_AB_NOLOAD, need -DPECH_DIAG too)
# "rev:<rev>" builds build/lib_<rev>.so from the kernel source at that git
# revision (e.g. the previous release) for before/after comparisons.
set -e
cd "$(dirname "$0")/.."
make -s build/crc32c_api.o build/crc32c_async.o build/crc32c_cpu.o build/crc32c_msgr.o
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function"
for spec in "$@"; do
  name=${spec%%:*}; arg=${spec#*:}
  if [ "$name" = rev ]; then
    mkdir -p build/rev_$arg
    git show "$arg":pech_amd/csrc/crc32c_kernels.hip > build/rev_$arg/crc32c_kernels.hip
    $HIPCC $FLAGS -Ipech_amd/csrc -c build/rev_$arg/crc32c_kernels.hip -o build/k_rev_$arg.o
    $HIPCC $FLAGS -shared -o build/lib_$arg.so build/k_rev_$arg.o build/crc32c_api.o build/crc32c_async.o \
      build/crc32c_cpu.o build/crc32c_msgr.o
    echo "build/lib_$arg.so"
  else
    make -s variant V="$name" D="$arg"
    echo "build/lib_$name.so"
  fi
done
