#!/bin/bash
# Round-3 state check on a fresh box: smoke, the GPU suite on the release and
# the bounds-checked builds, the default bench line, then rocprofv3 passes
# (tools/gpu_prof.sh) for CFGS.  Each GPU step has its own limit; the first
# failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop() { echo "stopping after rc=$1 ($2)"; exit "$1"; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || stop $? smoke
echo "smoke ok"
[ -n "$PROBE" ] && { timeout -k 10 180 build/sched_probe 10 $PROBE > gpurun_out/probe_$PROBE.json 2>&1 || stop $? probe; cat gpurun_out/probe_$PROBE.json; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_rel.log 2>&1 || { tail -30 gpurun_out/pytest_rel.log; stop $? rel; }
echo "rel: $(tail -1 gpurun_out/pytest_rel.log)"
PECH_CRC32C_LIB=build/lib_dbg.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_dbg.log 2>&1 || { tail -30 gpurun_out/pytest_dbg.log; stop $? dbg; }
echo "dbg: $(tail -1 gpurun_out/pytest_dbg.log) oob=$(grep -c 'PECH OOB' gpurun_out/pytest_dbg.log)"
grep -q "PECH OOB" gpurun_out/pytest_dbg.log && stop 1 oob
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; stop $? bench; }
tail -1 gpurun_out/bench_default.log
CFGS="${CFGS:-c3 c2 c4 c2-odd}" bash tools/gpu_prof.sh
