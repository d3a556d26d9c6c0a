#!/bin/bash
# A/B of the release library against ${B} (default build/lib_split64.so: v0.31 split threshold 64 rows): parity on the release and
# bounds-checked builds, odd launch sizes (tools/launch_sizes.py), bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for L in build/lib_dbg.so pech_amd/libpech_crc32c.so; do
  PECH_CRC32C_LIB=$L timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flat.py \
    tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_bounds.py > gpurun_out/t_split.log 2>&1 || { tail -30 gpurun_out/t_split.log; exit 1; }
  echo "$L: $(tail -1 gpurun_out/t_split.log) oob=$(grep -c 'PECH OOB' gpurun_out/t_split.log)"
  grep -q "PECH OOB" gpurun_out/t_split.log && exit 1
done
for L in pech_amd/libpech_crc32c.so ${B:-build/lib_split64.so}; do
  echo "== $L"
  PECH_CRC32C_LIB=$L timeout -k 10 300 python tools/launch_sizes.py ${SIZES:-8x4m 7x4m 8x4000k 8x4100000 8x3900000 10x3m 12x2731k 32x1m 100x300k 64x500k 1x4m 3x4m 16x4m 24x4m 48x4100000 200x1300k} 2>&1 | grep -v amdgpu || exit 1
done
SKIP_TESTS=1 AB_LIBS="pech_amd/libpech_crc32c.so ${B:-build/lib_split64.so}" AB_CONFIGS="${CFGS:-c3 c4 c4-64k c2-odd}" PASSES=2 \
  bash tools/gpu_round.sh > gpurun_out/round_split.txt 2>&1 || { tail -5 gpurun_out/round_split.txt; exit 1; }
grep "^lib" gpurun_out/round_split.txt
