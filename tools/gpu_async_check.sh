#!/bin/bash
# Async layer / adapter check on the GPU box: their GPU tests (release and the
# fault-injection test build), the messenger CPU sweep, the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop() { echo "stopping after rc=$1 ($2)"; exit "$1"; }
timeout -k 10 400 python -u -m pytest tests/test_async.py tests/test_faults.py tests/test_abi.py tests/test_cpu_path.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_async.log 2>&1 || { tail -30 gpurun_out/pytest_async.log; stop $? async; }
echo "async: $(tail -1 gpurun_out/pytest_async.log)"
bash tools/gpu_msgr_cpu.sh > gpurun_out/msgr_cpu_sweep.txt 2>&1 || { tail -5 gpurun_out/msgr_cpu_sweep.txt; stop 1 msgr; }
tail -25 gpurun_out/msgr_cpu_sweep.txt
[ -n "$BENCH" ] && { timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; stop $? bench; }; tail -1 gpurun_out/bench_default.log; }
exit 0
