#!/bin/bash
# A/B one kernel variant: bounds-checked parity (build/lib_dbg$V.so), release
# parity (build/lib_$V.so), then bench A/B against the default library.
# Usage: V=name AB_CONFIGS="c3 c2" bash tools/gpu_ab_variant.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PECH_CRC32C_LIB=build/lib_dbg$V.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_dbg$V.log 2>&1 || { tail -20 gpurun_out/pytest_dbg$V.log; exit 1; }
echo "dbg: $(tail -1 gpurun_out/pytest_dbg$V.log) oob=$(grep -c 'PECH OOB' gpurun_out/pytest_dbg$V.log)"
grep -q "PECH OOB" gpurun_out/pytest_dbg$V.log && exit 1
PECH_CRC32C_LIB=build/lib_$V.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_$V.log 2>&1 || { tail -20 gpurun_out/pytest_$V.log; exit 1; }
echo "release: $(tail -1 gpurun_out/pytest_$V.log)"
SKIP_TESTS=1 AB_LIBS="pech_amd/libpech_crc32c.so build/lib_$V.so pech_amd/libpech_crc32c.so build/lib_$V.so" \
  AB_CONFIGS="${AB_CONFIGS:-c3 c2 c4}" bash tools/gpu_round.sh
