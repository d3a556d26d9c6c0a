#!/bin/bash
# Per-wave timing stamps (PECH_STAMPS builds) for c3 and c2, then A/B libs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in ${STAMP_LIBS:-build/lib_stamps.so}; do
  for cfg in ${STAMP_CONFIGS:-c3 c2}; do
    o=gpurun_out/stamps_$(basename $lib .so)_$cfg.txt
    PECH_CRC32C_LIB=$lib timeout -k 10 120 python tools/wave_stamps.py $cfg > $o 2>&1 \
      || { echo "stamps $lib $cfg rc=$?"; cat $o; exit 1; }
    echo "== $lib $cfg"; grep -v amdgpu.ids $o
  done
done
AB_LIBS="${AB_LIBS:-}" AB_CONFIGS="${AB_CONFIGS:-c3}" bash tools/gpu_perf.sh
