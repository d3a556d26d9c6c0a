#!/bin/bash
# Two-stream bench `value` A/B (GPU box): for each config, libraries
# alternated REPS times; prints value, per-launch main us and serial value.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
for cfg in ${AB_CONFIGS:-c4}; do
  for lib in ${AB_LIBS:-pech_amd/libpech_crc32c.so}; do
    o=gpurun_out/abv_$(basename $lib .so)_${cfg}_$rep.log
    PECH_CRC32C_LIB=$lib timeout -k 10 240 python bench.py --config $cfg --steps ${AB_STEPS:-30} --no-cpu-baseline \
      --no-host-path --sustain-seconds ${AB_SUSTAIN:-3} ${AB_EXTRA:-} > $o 2>&1 || { tail -5 $o; exit 1; }
    echo "$(basename $lib) $cfg rep$rep: $(tail -1 $o | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("value", d["value"], "main_us", r["avg_launch_us"], "frac", r["frac"], "serial", d["serial"]["value"], "sustained", d.get("sustained",{}).get("value"))')"
  done
done
done
exit 0
