#!/bin/bash
# Validation session: parity tests against the bounds-checked debug build
# first (violations print "PECH OOB" and are redirected instead of faulting),
# then against the release build.  Stops at the first fault/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PECH_CRC32C_LIB=build/libdbg.so timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_dbg.log 2>&1
rc=$?; echo "debug pytest rc=$rc"; grep -c "PECH OOB" gpurun_out/pytest_dbg.log; grep -m5 "PECH OOB" gpurun_out/pytest_dbg.log; tail -3 gpurun_out/pytest_dbg.log
if [ $rc -ne 0 ] || grep -q "PECH OOB" gpurun_out/pytest_dbg.log; then echo "debug run not clean: stopping"; exit 1; fi
exit 0
