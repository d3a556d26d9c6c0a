#!/bin/bash
# The messenger side on the GPU box (build/msgr_sim bench), one script for the
# three measurements DESIGN §6.4-§6.7 quote:
#   WHAT=cpu  throughput mode: <BYTES_PER_PASS> of <SIZES> payloads per pass in crc32c_pages memory, flush every
#             64, epoll completion; MODES 0 async DMA, 1 async zero-copy, 2 the adapter, 3 the drop-in's host
#             routine -> gpurun_out/msgr_cpu.jsonl and a table (GiB/s, payloads/s, thread / process CPU us per
#             payload, latency p50/p99)
#   WHAT=lat  one payload in flight, 300 in sequence (<size> 1 <MODE> 300; MODE 2 the adapter, 3 the host
#             routine), over ENVS variants (space-separated, each a comma-separated VAR=value list, "-" = none;
#             PECH_CRC32C_MSGR_HOST_MAX=0 -- every payload on the GPU -- unless a variant sets it)
#   WHAT=prof the same lone payloads under rocprofv3's kernel and memory-copy traces, and with the runtime's
#             copies on blit kernels (HSA_ENABLE_SDMA=0)
# Every step time-limited; the first failure ends the script.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
mkdir -p gpurun_out
case "${WHAT:-cpu}" in
cpu)
  : > gpurun_out/msgr_cpu.jsonl
  for size in ${SIZES:-4096 16384 65536 262144 1048576 4194304}; do
    count=$(( ${BYTES_PER_PASS:-268435456} / size )); [ $count -gt 16384 ] && count=16384
    for mode in ${MODES:-0 1 2 3}; do
      timeout -k 10 120 build/msgr_sim bench $size $count $mode ${PASSES:-3} >> gpurun_out/msgr_cpu.jsonl \
        || { echo "msgr_sim rc=$? size $size mode $mode"; exit 1; }
    done
  done
  python3 - <<'PY'
import json
rows = [json.loads(l) for l in open("gpurun_out/msgr_cpu.jsonl")]
print("%9s %-15s %9s %12s %10s %10s %9s %9s" % ("bytes", "mode", "GiB/s", "payloads/s", "thr us/p", "proc us/p", "lat p50",
                                              "lat p99"))
for r in rows:
    print("%9d %-15s %9.2f %12.0f %10.3f %10.3f %9.1f %9.1f" % (r["payload_bytes"], r["mode"], r["GiBps"],
          r["payloads_per_s"], r["thread_cpu_us_per_payload"], r["process_cpu_us_per_payload"], r["latency_us_p50"],
          r["latency_us_p99"]))
PY
  ;;
lat)
  for rep in $(seq 1 ${REPS:-2}); do
    for size in ${SIZES:-65536 1048576 4194304}; do
      for ev in ${ENVS:-PECH_ASYNC_NOTIFY=3 PECH_ASYNC_NOTIFY=0}; do
        envs=""; [ "$ev" != - ] && envs=${ev//,/ }
        r=$(env PECH_CRC32C_MSGR_HOST_MAX=0 $envs timeout -k 10 120 build/msgr_sim bench $size 1 ${MODE:-2} 300) \
          || { echo "rc=$? $r"; exit 1; }
        echo "size $size mode ${MODE:-2} $ev: $(echo "$r" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["latency_us_p50"], d["latency_us_p99"], d["thread_cpu_us_per_payload"], d["process_cpu_us_per_payload"], "bad", d["bad"])')"
      done
    done
  done
  ;;
prof)
  for size in ${SIZES:-65536 1048576}; do
    PECH_CRC32C_MSGR_HOST_MAX=0 timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats \
      -d "$R/gpurun_out/latprof_$size" -o run --output-format csv -- build/msgr_sim bench $size 1 2 300 \
      > gpurun_out/latprof_$size.log 2>&1 || { tail -20 gpurun_out/latprof_$size.log; exit 1; }
    for sd in 1 0; do
      r=$(HSA_ENABLE_SDMA=$sd PECH_CRC32C_MSGR_HOST_MAX=0 timeout -k 10 120 build/msgr_sim bench $size 1 2 300) \
        || { echo "rc=$? $r"; exit 1; }
      echo "size $size sdma $sd: $(echo "$r" | tail -1)"
    done
  done
  ;;
*)
  echo "WHAT=cpu|lat|prof"; exit 2;;
esac
