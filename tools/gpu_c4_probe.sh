cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for c in c4 c2-1g c3; do
  PECH_CRC32C_LIB=build/lib_stamps.so timeout -k 10 120 python tools/wave_stamps.py $c > gpurun_out/stamps_$c.txt 2>&1 || exit 2
  grep -E "span|busy us|end   us|prologue|xcc|slot" gpurun_out/stamps_$c.txt
done
for c in c2-1g c4 c3; do
  timeout -k 10 150 python3 bench.py --config $c --steps 30 --no-cpu-baseline --no-host-path --sustain-seconds 2 > gpurun_out/b_$c.log 2>&1 || exit 3
  grep '^{' gpurun_out/b_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$c', d['value'], d['serial']['value'], r['avg_launch_us'], r['frac'])"
done
