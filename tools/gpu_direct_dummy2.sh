#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SKIP_TESTS=1 AB_LIBS="pech_amd/libpech_crc32c.so build/lib_clampdup.so pech_amd/libpech_crc32c.so build/lib_clampdup.so pech_amd/libpech_crc32c.so build/lib_clampdup.so" \
  AB_CONFIGS="c2-odd" bash tools/gpu_round.sh || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_direct.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_direct.log 2>&1 || { tail -30 gpurun_out/pytest_direct.log; exit 1; }
echo "direct: $(tail -1 gpurun_out/pytest_direct.log)"
CFGS="c2-odd" bash tools/gpu_prof.sh
