#!/bin/bash
# The driver's round-end commands, as it runs them (GPU box): the GPU suite,
# smoke, the default bench line at the driver's steps.  Time limits of our own.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/drv_pytest.log 2>&1 || { tail -30 gpurun_out/drv_pytest.log; exit 1; }
tail -1 gpurun_out/drv_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/drv_smoke.log 2>&1 || { cat gpurun_out/drv_smoke.log; exit 1; }
tail -1 gpurun_out/drv_smoke.log
t0=$(date +%s.%N)
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/drv_bench.log 2> gpurun_out/drv_bench.err || { tail -20 gpurun_out/drv_bench.err; exit 1; }
echo "bench wall $(python3 -c "import sys; print(round($(date +%s.%N) - $t0, 1))") s"
tail -1 gpurun_out/drv_bench.log
