#!/bin/bash
# A/B of kernel builds and environments on the launch-size curve
# (bench.py --curve-only), interleaved, REPS times:
#   LIBS="pech_amd/libpech_crc32c.so build/lib_x.so" ENVS="- PECH_RPW_MIN=128" bash tools/gpu_ab_curve.sh
# (ENVS: space-separated variants, each a comma-separated VAR=value list, "-" = none)
# Optional STAMPS="build/lib_stamps.so build/lib_stamps_x.so" CFGS="8x4m 64x4m": wave stamps per build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -f gpurun_out/ab_curve.jsonl
for rep in $(seq 1 ${REPS:-2}); do
  for L in ${LIBS:-pech_amd/libpech_crc32c.so}; do
    for ev in ${ENVS:--}; do
      envs=""; [ "$ev" != - ] && envs=${ev//,/ }
      env $envs PECH_CRC32C_LIB=$L timeout -k 10 120 python bench.py --curve-only ${CURVE_EXTRA:-} > gpurun_out/curve_tmp.json 2>&1 \
        || { cat gpurun_out/curve_tmp.json; exit 1; }
      tail -1 gpurun_out/curve_tmp.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d['env']='$ev'; print(json.dumps(d))" >> gpurun_out/ab_curve.jsonl
    done
  done
done
python3 - <<'PY'
import json
rows = [json.loads(l) for l in open("gpurun_out/ab_curve.jsonl")]
for r in rows:
    c = r["launch_curve"]["by_buffer_size_then_MiB"]
    print(r["lib"].split("/")[-1], r.get("env"), {b: [c[b][m]["main_us"] for m in ("4", "32", "128", "256", "1024")] for b in c})
PY
for L in $STAMPS; do
  for c in ${CFGS:-8x4m 64x4m}; do
    echo "== $L $c"
    PECH_CRC32C_LIB=$L timeout -k 10 120 python tools/wave_stamps.py $c 2>&1 | grep -v amdgpu.ids | head -12
  done
done
