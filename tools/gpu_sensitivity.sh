cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for d in random zeros ones; do for c in c3 c2; do
  timeout -k 10 200 python3 bench.py --config $c --data $d --no-host-path --cpu-seconds 2 --sustain-seconds 3 > gpurun_out/sens_${c}_$d.log 2>&1 || exit 3
  tail -1 gpurun_out/sens_${c}_$d.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c $d', d['value'], d['serial']['value'], r['avg_launch_us'], r['frac'], d['sustained']['value'], d['cpu_baseline']['sample'][-40:])"
done; done
timeout -k 10 200 python3 bench.py --config c3 --op copy --no-host-path --cpu-seconds 2 --sustain-seconds 3 > gpurun_out/copy_c3.log 2>&1 || exit 4
tail -1 gpurun_out/copy_c3.log
