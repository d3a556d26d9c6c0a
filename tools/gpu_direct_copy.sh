#!/bin/bash
# the one-launch direct fused copy: parity (bounds-checked, release), then C2 copy small vs planned
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop() { echo "stopping after rc=$1 ($2)"; exit "$1"; }
PECH_CRC32C_LIB=build/lib_dbg.so timeout -k 10 300 python -u -m pytest tests/test_copy.py tests/test_abi.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_dcopy_dbg.log 2>&1 || { tail -30 gpurun_out/pytest_dcopy_dbg.log; stop $? dbg; }
echo "dbg: $(tail -1 gpurun_out/pytest_dcopy_dbg.log) oob=$(grep -c 'PECH OOB' gpurun_out/pytest_dcopy_dbg.log)"
grep -q "PECH OOB" gpurun_out/pytest_dcopy_dbg.log && stop 1 oob
timeout -k 10 300 python -u -m pytest tests/test_copy.py tests/test_abi.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_dcopy.log 2>&1 || { tail -30 gpurun_out/pytest_dcopy.log; stop $? rel; }
echo "rel: $(tail -1 gpurun_out/pytest_dcopy.log)"
for rep in 1 2; do for api in small planned; do
  timeout -k 10 240 python bench.py --config c2 --op copy --api $api --steps 30 --no-cpu-baseline --no-host-path > gpurun_out/dcopy_$api.log 2>&1 \
    || { tail -5 gpurun_out/dcopy_$api.log; stop $? "bench $api"; }
  echo "c2 copy $api: $(tail -1 gpurun_out/dcopy_$api.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], r["kernel"], r["avg_launch_us"], r["frac"], d["serial"]["value"])')"
done; done
