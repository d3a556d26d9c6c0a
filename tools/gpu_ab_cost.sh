#!/bin/bash
# v0.31 candidate: cost-weighted static shares for mixed batches, against equal rows (build/lib_nocost.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for L in build/lib_dbg.so pech_amd/libpech_crc32c.so; do
  PECH_CRC32C_LIB=$L timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_fuzz.py tests/test_gpu_bounds.py > gpurun_out/t_cost.log 2>&1 || { tail -30 gpurun_out/t_cost.log; exit 1; }
  echo "$L: $(tail -1 gpurun_out/t_cost.log) oob=$(grep -c 'PECH OOB' gpurun_out/t_cost.log)"
  grep -q "PECH OOB" gpurun_out/t_cost.log && exit 1
done
SKIP_TESTS=1 STAMP_CONFIGS="c4" AB_LIBS="pech_amd/libpech_crc32c.so build/lib_nocost.so" AB_CONFIGS="c4 c4-64k c2-odd" PASSES=3 \
  bash tools/gpu_round.sh > gpurun_out/round_cost.txt 2>&1 || { tail -5 gpurun_out/round_cost.txt; exit 1; }
grep -v "amdgpu\|^xcc" gpurun_out/round_cost.txt
