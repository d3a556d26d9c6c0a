#!/bin/bash
# A/B of kernel builds on the launch-size curve (bench.py --curve-only), each
# library twice, interleaved: LIBS="pech_amd/libpech_crc32c.so build/lib_x.so" bash tools/gpu_ab_curve.sh
# Optional STAMPS="build/lib_stamps.so build/lib_stamps_x.so" CFGS="8x4m 64x4m": wave stamps per build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for L in $LIBS; do
    PECH_CRC32C_LIB=$L timeout -k 10 120 python bench.py --curve-only > gpurun_out/curve_tmp.json 2>&1 || { cat gpurun_out/curve_tmp.json; exit 1; }
    tail -1 gpurun_out/curve_tmp.json >> gpurun_out/ab_curve.jsonl
  done
done
python3 - <<'PY'
import json
rows = [json.loads(l) for l in open("gpurun_out/ab_curve.jsonl")]
for r in rows:
    c = r["launch_curve"]["by_buffer_size_then_MiB"]
    print(r["lib"].split("/")[-1], {b: [c[b][m]["main_us"] for m in ("4", "32", "128", "256", "1024")] for b in c})
PY
for L in $STAMPS; do
  for c in ${CFGS:-8x4m 64x4m}; do
    echo "== $L $c"
    PECH_CRC32C_LIB=$L timeout -k 10 120 python tools/wave_stamps.py $c 2>&1 | grep -v amdgpu.ids | head -12
  done
done
