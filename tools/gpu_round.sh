#!/bin/bash
# THE GPU-box session runner for validation and A/B measurements (every GPU
# step has its own time limit; the first failure ends the script).  Sections,
# each on when its variable is set:
#   (default)       the GPU suite on the bounds-checked build (OOB loads print instead of faulting), then on the
#                   release build; SKIP_TESTS=1 skips both, TEST_ENV adds environment to both
#   STAMP_CONFIGS   per-wave stamps of a -DPECH_STAMPS build (STAMP_LIB, default build/lib_stamps.so) for these
#                   tools/wave_stamps.py shapes (c3, c4, 8x4m, 512x64k, ...; PECH_FLAT_MAX in TEST_ENV picks a path)
#   CURVE=1         the launch-size curve (bench.py --curve-only) of every AB_LIBS build, CURVE_REPS times
#   AB_CONFIGS      bench lines over library builds (AB_LIBS), configs, environments (AB_ENVS: space-separated
#                   variants, each a comma-separated VAR=value list, "-" = none) and extra bench flags (AB_EXTRA:
#                   e.g. "--op copy", "--data zeros", "--single-thread --devices 0,0,0,0,0,0,0,0",
#                   "--sustain-seconds 4"), PASSES interleaved passes; columns: value (2-stream pass) GiB/s,
#                   per-launch GB/s, roofline frac, per-launch us, serial (1-stream) GiB/s, sustained GiB/s
#   RANKS           bench.py under torchrun with that many ranks sharing the GPU over gloo (the N > 1 driver's
#                   rehearsal on a one-GPU box; space-separated list, e.g. "2 4")
# Library builds for A/B: tools/build_ab.sh (variants, kernel-only revisions, whole trees of older releases).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stop() { echo "stopping after rc=$1 ($2)"; exit "$1"; }
if [ -z "${SKIP_TESTS:-}" ]; then
env ${TEST_ENV:-} PECH_CRC32C_LIB=build/lib_dbg.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 \
  --timeout-method thread > gpurun_out/pytest_dbg.log 2>&1 || { tail -30 gpurun_out/pytest_dbg.log; stop $? dbg; }
echo "dbg: $(tail -1 gpurun_out/pytest_dbg.log) oob=$(grep -c 'PECH OOB' gpurun_out/pytest_dbg.log)"
grep -q "PECH OOB" gpurun_out/pytest_dbg.log && stop 1 oob
env ${TEST_ENV:-} timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; stop $? pytest; }
echo "release: $(tail -1 gpurun_out/pytest_gpu.log)"
fi
for cfg in ${STAMP_CONFIGS:-}; do
  env ${TEST_ENV:-} PECH_CRC32C_LIB=${STAMP_LIB:-build/lib_stamps.so} timeout -k 10 120 python tools/wave_stamps.py $cfg \
    > gpurun_out/stamps_$cfg.txt 2>&1 || stop $? "stamps $cfg"
  grep -v "amdgpu.ids\|^xcc\|histogram" gpurun_out/stamps_$cfg.txt
done
if [ -n "${CURVE:-}" ]; then
  rm -f gpurun_out/ab_curve.jsonl
  for rep in $(seq 1 ${CURVE_REPS:-2}); do
    for L in ${AB_LIBS:-pech_amd/libpech_crc32c.so}; do
      PECH_CRC32C_LIB=$L timeout -k 10 120 python bench.py --curve-only > gpurun_out/curve_tmp.json 2>&1 \
        || { cat gpurun_out/curve_tmp.json; stop 1 "curve $L"; }
      tail -1 gpurun_out/curve_tmp.json >> gpurun_out/ab_curve.jsonl
    done
  done
  python3 - <<'PY'
import json
for l in open("gpurun_out/ab_curve.jsonl"):
    d = json.loads(l)
    c = d["launch_curve"]["by_buffer_size_then_MiB"]
    print(d["lib"].split("/")[-1], "main_us / step_us:",
          {b: [(c[b][m]["main_us"], c[b][m]["step_us"]) for m in ("4", "32", "128", "256", "1024")] for b in c})
PY
fi
for pass in $(seq 1 ${PASSES:-1}); do
for ev in ${AB_ENVS:--}; do
for lib in ${AB_LIBS:-pech_amd/libpech_crc32c.so}; do
  for cfg in ${AB_CONFIGS:-}; do
    o=gpurun_out/ab_$(basename $lib .so)_${ev//[=,]/_}_$cfg.log
    envs=""; [ "$ev" != - ] && envs=${ev//,/ }
    env $envs PECH_CRC32C_LIB=$lib timeout -k 10 240 python bench.py --config $cfg --steps 30 --no-cpu-baseline --no-host-path \
      ${AB_EXTRA:-} > $o 2>&1 || { tail -5 $o; stop $? "bench $lib $cfg"; }
    echo "$(basename $lib) $ev $cfg: $(tail -1 $o | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], r["achieved"], r["frac"], r["avg_launch_us"], d.get("serial", {}).get("value"), d.get("sustained", {}).get("value"), "host_issue", d["host_issue"]["issue_us_per_step"])')"
  done
done
done
done
for n in ${RANKS:-}; do
  PECH_BENCH_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 10 --warmup 3 \
    > gpurun_out/dist_rehearsal_n$n.log 2>&1 || { tail -20 gpurun_out/dist_rehearsal_n$n.log; stop $? "ranks $n"; }
  echo "ranks $n: $(tail -1 gpurun_out/dist_rehearsal_n$n.log | cut -c1-300)"
done
exit 0
