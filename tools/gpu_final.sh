#!/bin/bash
# Round-end rehearsal on the GPU box: smoke, the bounds-checked build over the
# GPU tests (no "PECH OOB"), the default bench line exactly as the driver runs
# it, then the rocprofv3 passes (tools/gpu_prof.sh).  Each GPU step has its own
# time limit; a fault, timeout or abort stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop() { echo "stopping after rc=$1 ($2)"; exit "$1"; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || stop $? smoke
echo "smoke ok"
PECH_CRC32C_LIB=build/lib_dbg.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_dbg.log 2>&1 || { tail -30 gpurun_out/pytest_dbg.log; stop $? dbg; }
echo "dbg: $(tail -1 gpurun_out/pytest_dbg.log) oob=$(grep -c 'PECH OOB' gpurun_out/pytest_dbg.log)"
grep -q "PECH OOB" gpurun_out/pytest_dbg.log && stop 1 oob
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; stop $? bench; }
tail -1 gpurun_out/bench_default.log
CFGS="${CFGS:-c3 c2 c4}" bash tools/gpu_prof.sh
