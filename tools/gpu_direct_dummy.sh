#!/bin/bash
# direct kernel: past-end ring loads from the constants table (release) vs the v0.18 clamp (lib_clampdup)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop() { echo "stopping after rc=$1 ($2)"; exit "$1"; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_rel.log 2>&1 || { tail -30 gpurun_out/pytest_rel.log; stop $? rel; }
echo "rel: $(tail -1 gpurun_out/pytest_rel.log)"
SKIP_TESTS=1 AB_LIBS="pech_amd/libpech_crc32c.so build/lib_clampdup.so pech_amd/libpech_crc32c.so build/lib_clampdup.so" \
  AB_CONFIGS="c2-odd c2" bash tools/gpu_round.sh || exit 1
CFGS="c2-odd" bash tools/gpu_prof.sh
