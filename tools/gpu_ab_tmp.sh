#!/bin/bash
# scratch GPU session (round 3): GPU tests on the current build, then A/B prof
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
AB_LIBS="build/lib_v15.so pech_amd/libpech_crc32c.so" AB_CONFIGS="${CFGS:-c2-odd c4 c2-odd c4}" AB_STEPS=40 bash tools/gpu_ab_prof.sh || exit $?
[ -n "$SKIP_COPY" ] || AB_LIBS="build/lib_v15.so pech_amd/libpech_crc32c.so" AB_CONFIGS="c3 c2" AB_STEPS=20 AB_EXTRA="--op copy" bash tools/gpu_ab_prof.sh
