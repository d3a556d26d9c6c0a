#!/bin/bash
# Debug-build parity first (OOB loads print instead of faulting); only if
# clean, the release build's smoke + parity + bench + A/B perf.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PECH_CRC32C_LIB=build/lib_dbg.so timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_dbg.log 2>&1
rc=$?; echo "debug pytest rc=$rc oob=$(grep -c 'PECH OOB' gpurun_out/pytest_dbg.log)"; tail -2 gpurun_out/pytest_dbg.log
if [ $rc -ne 0 ] || grep -q "PECH OOB" gpurun_out/pytest_dbg.log; then echo "debug run not clean: stopping"; exit 1; fi
bash tools/gpu_check.sh || exit $?
AB_LIBS="${AB_LIBS:-}" AB_CONFIGS="${AB_CONFIGS:-c3}" PROF_CONFIGS="${PROF_CONFIGS:-}" bash tools/gpu_perf.sh
