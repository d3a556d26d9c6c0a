#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PECH_CRC32C_LIB=build/lib_sf.so timeout -k 10 300 python -u -m pytest tests/test_copy.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sf.log 2>&1 || { tail -20 gpurun_out/pytest_sf.log; exit 1; }
echo "sf parity: $(tail -1 gpurun_out/pytest_sf.log)"
SKIP_TESTS=1 AB_EXTRA="--op copy --api planned" AB_LIBS="build/lib_sf.so pech_amd/libpech_crc32c.so build/lib_sf.so pech_amd/libpech_crc32c.so" \
  AB_CONFIGS="c3 c2" bash tools/gpu_round.sh
