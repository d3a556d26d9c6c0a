#!/bin/bash
# Small launches: neighbouring live shares per workgroup (release) against strided (build/lib_strided.so) and the no-atomic
# diagnostic (build/lib_noatomic.so: out[] XORs dropped, wrong CRCs): parity, launch_sizes, curve, bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for L in build/lib_dbg.so pech_amd/libpech_crc32c.so; do
  PECH_CRC32C_LIB=$L timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flat.py \
    tests/test_gpu_parity.py tests/test_gpu_bounds.py tests/test_async.py > gpurun_out/t_deal.log 2>&1 || { tail -30 gpurun_out/t_deal.log; exit 1; }
  echo "$L: $(tail -1 gpurun_out/t_deal.log) oob=$(grep -c 'PECH OOB' gpurun_out/t_deal.log)"
  grep -q "PECH OOB" gpurun_out/t_deal.log && exit 1
done
for L in ${DLIBS:-pech_amd/libpech_crc32c.so build/lib_strided.so build/lib_noatomic.so}; do
  echo "== $L"
  LS_NOCHECK=1 PECH_CRC32C_LIB=$L timeout -k 10 300 python tools/launch_sizes.py 1x4m 2x4m 3x4m 4x4m 7x4m 8x4m 8x4100000 10x3m \
    12x2731k 100x300k 64x500k 16x4m 24x4m 2>&1 | grep -v amdgpu || exit 1
done
LIBS="${CLIBS:-pech_amd/libpech_crc32c.so build/lib_strided.so}" REPS=2 bash tools/gpu_ab_curve.sh 2>&1 | grep -v amdgpu | tail -4
