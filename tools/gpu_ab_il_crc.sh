#!/bin/bash
# CRC-only kernel with interleaved rows (build/lib_ilcrc.so, -DPECH_IL_CRC=1) vs the release (slices + pool)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop() { echo "stopping after rc=$1 ($2)"; exit "$1"; }
PECH_CRC32C_LIB=build/lib_dbg_ilcrc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_ilcrc_dbg.log 2>&1 || { tail -30 gpurun_out/pytest_ilcrc_dbg.log; stop $? dbg; }
echo "dbg: $(tail -1 gpurun_out/pytest_ilcrc_dbg.log) oob=$(grep -c 'PECH OOB' gpurun_out/pytest_ilcrc_dbg.log)"
grep -q "PECH OOB" gpurun_out/pytest_ilcrc_dbg.log && stop 1 oob
SKIP_TESTS=1 AB_LIBS="build/lib_ilcrc.so pech_amd/libpech_crc32c.so build/lib_ilcrc.so pech_amd/libpech_crc32c.so" \
  AB_CONFIGS="c3 c4-1m c4-4m" bash tools/gpu_round.sh
