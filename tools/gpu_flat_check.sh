#!/bin/bash
# Round-5 session: targeted GPU tests (TARGETS), the GPU suite on the release
# and the bounds-checked builds, then the flat / planned A/B on c3
# (`--flat-max`) and the launch curve of each.  Each GPU step time-limited;
# the first failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop() { echo "stopping after rc=$1 ($2)"; exit "$1"; }
T="python -u -m pytest -x -q --timeout 150 --timeout-method thread"
if [ -n "${TARGETS:-}" ]; then
  timeout -k 10 400 $T $TARGETS > gpurun_out/targets.log 2>&1 || { rc=$?; tail -40 gpurun_out/targets.log; stop $rc targets; }
  echo "targets: $(tail -1 gpurun_out/targets.log)"
fi
if [ -z "${SKIP_SUITE:-}" ]; then
  timeout -k 10 500 $T tests -m gpu > gpurun_out/pytest_rel.log 2>&1 || { rc=$?; tail -40 gpurun_out/pytest_rel.log; stop $rc rel; }
  echo "rel: $(tail -1 gpurun_out/pytest_rel.log)"
  PECH_CRC32C_LIB=build/lib_dbg.so timeout -k 10 500 $T tests -m gpu > gpurun_out/pytest_dbg.log 2>&1 \
    || { rc=$?; tail -40 gpurun_out/pytest_dbg.log; stop $rc dbg; }
  echo "dbg: $(tail -1 gpurun_out/pytest_dbg.log) oob=$(grep -c 'PECH OOB' gpurun_out/pytest_dbg.log)"
  grep -q "PECH OOB" gpurun_out/pytest_dbg.log && stop 1 oob
fi
for pass in 1 2; do
for fm in ${FLAT_MAXES:-256 0}; do
  for cfg in ${CFGS:-c3}; do
    o=gpurun_out/ab_${cfg}_fm$fm.log
    timeout -k 10 200 python bench.py --config $cfg --steps 30 --no-cpu-baseline --no-host-path --sustain-seconds 2 \
      --flat-max $fm ${AB_EXTRA:-} > $o 2>&1 || { rc=$?; tail -5 $o; stop $rc bench; }
    echo "$cfg flat-max $fm: $(tail -1 $o | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], r["kernel"], r["frac"], r["avg_launch_us"], d["serial"]["value"], d.get("sustained",{}).get("value"))')"
  done
done
done
for fm in ${FLAT_MAXES:-256 0}; do
  timeout -k 10 200 python bench.py --curve-only --flat-max $fm > gpurun_out/curve_fm$fm.log 2>&1 || { rc=$?; tail -5 gpurun_out/curve_fm$fm.log; stop $rc curve; }
  echo "curve flat-max $fm: $(tail -1 gpurun_out/curve_fm$fm.log)"
done
exit 0
