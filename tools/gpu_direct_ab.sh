#!/bin/bash
# Direct-kernel check (GPU box): its parity tests, then bench lines of the
# small-buffer configs on the direct (small) and planned entry points.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_direct.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_direct.log 2>&1 || { tail -n 30 gpurun_out/t_direct.log; exit 1; }
tail -n 1 gpurun_out/t_direct.log
for rep in $(seq 1 ${REPS:-2}); do
for cfg in ${CFGS:-c2 c2-odd}; do for api in ${APIS:-small planned}; do
  o=gpurun_out/b_${cfg}_${api}_$rep.log
  timeout -k 10 200 python bench.py --config $cfg --api $api --steps 30 --no-cpu-baseline --no-host-path --sustain-seconds 2 > $o 2>&1 || { tail -n 5 $o; exit 1; }
  echo "$cfg $api rep$rep $(tail -n 1 $o | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("value", d["value"], "us", r["avg_launch_us"], "frac", r["frac"], "serial", d["serial"]["value"])')"
done; done; done
