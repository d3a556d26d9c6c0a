#!/bin/bash
# One GPU-box session: smoke, GPU parity tests, a short bench.  Every GPU step
# has its own time limit; a fault/timeout/abort stops the script (no retries).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
BENCH_ARGS=${BENCH_ARGS:-"--steps 20 --cpu-seconds 5"}
ok_or_stop() { # rc 0 = pass, 1 = test failures (no fault) -> continue; else stop
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after rc=$1 ($2)"; exit "$1"; fi
}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; ok_or_stop $rc smoke
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; ok_or_stop $rc pytest
timeout -k 10 300 python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
exit $rc
