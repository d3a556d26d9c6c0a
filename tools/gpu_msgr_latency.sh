#!/bin/bash
# One payload in flight (build/msgr_sim bench <size> 1 2 300: the adapter with
# every payload on the GPU): latency p50/p99, calling-thread and process CPU
# per payload, over env variants (ENVS: space-separated, each a comma-separated
# VAR=value list, "-" = none; default: the async layer's notify modes 3 and 0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
for size in ${SIZES:-65536 1048576 4194304}; do
  for ev in ${ENVS:-PECH_ASYNC_NOTIFY=3 PECH_ASYNC_NOTIFY=0}; do
    envs=""; [ "$ev" != - ] && envs=${ev//,/ }
    r=$(env $envs PECH_CRC32C_MSGR_HOST_MAX=0 timeout -k 10 120 build/msgr_sim bench $size 1 2 300) || { echo "rc=$? $r"; exit 1; }
    echo "size $size $ev: $(echo "$r" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["latency_us_p50"], d["latency_us_p99"], d["thread_cpu_us_per_payload"], d["process_cpu_us_per_payload"], "bad", d["bad"])')"
  done
done
done
