#!/bin/bash
# direct kernel with workgroup-interleaved positions (build/lib_wgi.so, -DPECH_DIRECT_WGI) vs the release
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop() { echo "stopping after rc=$1 ($2)"; exit "$1"; }
PECH_CRC32C_LIB=build/lib_dbg_wgi.so timeout -k 10 300 python -u -m pytest tests/test_gpu_direct.py tests/test_gpu_bounds.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_wgi_dbg.log 2>&1 || { tail -30 gpurun_out/pytest_wgi_dbg.log; stop $? dbg; }
echo "dbg: $(tail -1 gpurun_out/pytest_wgi_dbg.log) oob=$(grep -c 'PECH OOB' gpurun_out/pytest_wgi_dbg.log)"
grep -q "PECH OOB" gpurun_out/pytest_wgi_dbg.log && stop 1 oob
SKIP_TESTS=1 AB_LIBS="build/lib_wgi.so pech_amd/libpech_crc32c.so build/lib_wgi.so pech_amd/libpech_crc32c.so" \
  AB_CONFIGS="c2 c2-odd c4-4k" bash tools/gpu_round.sh
