#!/bin/bash
# Build A/B diagnostic libraries against the current C-ABI object:
#   tools/build_ab.sh name:-DFLAG ... [rev:<git-rev>]
# (flags that change results, -DPECH_AB_NOLDS / -DPECH_AB_NOLOAD, need -DPECH_DIAG too)
# "rev:<rev>" builds build/lib_<rev>.so from the kernel source at that git
# revision (e.g. the previous release) for before/after comparisons.
# "tree:<rev>" builds the WHOLE library (kernels and C-ABI) of that revision
# in a temp tree -> build/lib_tree_<rev>.so: for revisions whose kernel
# arguments differ from the current host code's (same-box A/B of releases).
set -e
cd "$(dirname "$0")/.."
make -s build/crc32c_api.o build/crc32c_async.o build/crc32c_cpu.o build/crc32c_msgr.o
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function"
for spec in "$@"; do
  name=${spec%%:*}; arg=${spec#*:}
  if [ "$name" = tree ]; then
    t=$(mktemp -d)
    git archive "$arg" pech_amd include Makefile | tar -x -C "$t"
    make -s -C "$t" pech_amd/libpech_crc32c.so
    cp "$t/pech_amd/libpech_crc32c.so" build/lib_tree_$arg.so
    rm -rf "$t"
    echo "build/lib_tree_$arg.so"
  elif [ "$name" = rev ]; then
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
