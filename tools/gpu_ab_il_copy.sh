#!/bin/bash
# fused copy with interleaved rows (build/lib_il.so, -DPECH_IL_COPY=1) vs the release
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop() { echo "stopping after rc=$1 ($2)"; exit "$1"; }
PECH_CRC32C_LIB=build/lib_dbg_il.so timeout -k 10 300 python -u -m pytest tests/test_copy.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_copy_dbg.log 2>&1 || { tail -30 gpurun_out/pytest_copy_dbg.log; stop $? dbg; }
echo "dbg: $(tail -1 gpurun_out/pytest_copy_dbg.log) oob=$(grep -c 'PECH OOB' gpurun_out/pytest_copy_dbg.log)"
grep -q "PECH OOB" gpurun_out/pytest_copy_dbg.log && stop 1 oob
PECH_CRC32C_LIB=build/lib_il.so timeout -k 10 300 python -u -m pytest tests/test_copy.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_copy.log 2>&1 || { tail -30 gpurun_out/pytest_copy.log; stop $? rel; }
echo "il release: $(tail -1 gpurun_out/pytest_copy.log)"
SKIP_TESTS=1 AB_EXTRA="--op copy" AB_LIBS="build/lib_il.so pech_amd/libpech_crc32c.so build/lib_il.so pech_amd/libpech_crc32c.so" \
  AB_CONFIGS="c3 c4-1m" bash tools/gpu_round.sh
