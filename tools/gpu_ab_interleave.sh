cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for pass in 1 2; do for lib in build/lib_HEAD.so pech_amd/libpech_crc32c.so; do for c in c2 c4 c3; do
 PECH_CRC32C_LIB=$lib timeout -k 10 150 python3 bench.py --config $c --steps 30 --no-cpu-baseline --no-host-path --sustain-seconds 2 > gpurun_out/ab_$c.log 2>&1 || exit 3
 tail -1 gpurun_out/ab_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$lib $c', d['value'], d['serial']['value'], r['avg_launch_us'], r['frac'], d['sustained']['value'])"
done; done; done
