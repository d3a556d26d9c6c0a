mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_direct.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_direct.log 2>&1 || { tail -n 30 gpurun_out/t_direct.log; exit 1; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { tail -n 30 gpurun_out/t_gpu.log; exit 1; }
for cfg in c2 c2-odd; do for api in small planned small planned; do
  timeout -k 10 200 python bench.py --config $cfg --api $api --steps 30 --no-cpu-baseline --no-host-path --sustain-seconds 2 > gpurun_out/b_${cfg}_$api.log 2>&1 || { tail -n 5 gpurun_out/b_${cfg}_$api.log; exit 1; }
  echo "$cfg $api $(tail -n 1 gpurun_out/b_${cfg}_$api.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("value", d["value"], "us", r["avg_launch_us"], "frac", r["frac"], "serial", d["serial"]["value"])')"
done; done
SIZES="4096 16384 65536" bash tools/gpu_msgr_cpu.sh > gpurun_out/msgr_direct.txt 2>&1 && PECH_ASYNC_PLANNED=1 SIZES="4096 16384 65536" bash tools/gpu_msgr_cpu.sh > gpurun_out/msgr_planned.txt 2>&1
