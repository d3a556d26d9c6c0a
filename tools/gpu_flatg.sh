#!/bin/bash
# flatg A/B on one box (GPU): the flat tests on the bounds-checked build, wave stamps of flatg against plan + main,
# then bench lines (LIBS: library builds, FMS: flat limits) with --flat-max 4096 (flatg) against the default (plan + main) and the 64 KiB launch curve both ways
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop() { echo "stopping after rc=$1 ($2)"; exit "$1"; }
if [ -z "${SKIP_DBG:-}" ]; then
PECH_CRC32C_LIB=build/lib_dbg.so timeout -k 10 400 python -u -m pytest tests/test_gpu_flat.py tests/test_gpu_bounds.py -x -q \
  --timeout 150 --timeout-method thread > gpurun_out/flatg_dbg.log 2>&1 || { tail -30 gpurun_out/flatg_dbg.log; stop 1 dbg; }
echo "dbg: $(tail -1 gpurun_out/flatg_dbg.log) oob=$(grep -c 'PECH OOB' gpurun_out/flatg_dbg.log)"
grep -q "PECH OOB" gpurun_out/flatg_dbg.log && { grep "PECH OOB" gpurun_out/flatg_dbg.log | head; stop 1 oob; }
fi
for sl in ${STAMP_LIBS:-build/lib_stamps.so}; do
for cfg in ${STAMPS:-4096x64k 512x64k}; do
  for fm in ${STAMP_FMS:-4096 0}; do
    PECH_FLAT_MAX=$fm PECH_CRC32C_LIB=$sl timeout -k 10 120 python tools/wave_stamps.py $cfg \
      > gpurun_out/stamps_flatg_$(basename $sl .so)_${cfg}_$fm.txt 2>&1 || stop $? "stamps $cfg"
    echo "== $(basename $sl) $cfg flat_max=$fm"; grep -v "amdgpu.ids\|^xcc\|histogram" gpurun_out/stamps_flatg_$(basename $sl .so)_${cfg}_$fm.txt
  done
done
done
for pass in 1 2; do
  for lib in ${LIBS:-pech_amd/libpech_crc32c.so}; do
  for fm in ${FMS:-4096 256}; do
    for cfg in ${CFGS:-c4-64k}; do
      o=gpurun_out/flatg_${cfg}_$fm.log
      PECH_CRC32C_LIB=$lib timeout -k 10 240 python bench.py --config $cfg --steps 30 --no-cpu-baseline --no-host-path --flat-max $fm > $o 2>&1 \
        || { tail -5 $o; stop 1 "bench $cfg $fm"; }
      echo "$(basename $lib) flat_max $fm $cfg: $(tail -1 $o | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], r["kernel"], r["avg_launch_us"], "serial", d["serial"]["value"], d["serial"]["ms_per_step"], "sustained", d["sustained"]["value"])')"
    done
    PECH_CRC32C_LIB=$lib timeout -k 10 120 python bench.py --curve-only --flat-max $fm > gpurun_out/flatg_curve_$fm.json 2>&1 || stop 1 "curve $fm"
    tail -1 gpurun_out/flatg_curve_$fm.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['launch_curve']['by_buffer_size_then_MiB']['64KiB']; print('$(basename $lib) curve 64KiB flat_max $fm main/step us:', [(c[m]['main_us'], c[m]['step_us']) for m in ('4','32','128','256','1024')])"
  done
  done
done
exit 0
