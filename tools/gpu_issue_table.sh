#!/bin/bash
# pech's model on one GPU box: one host thread issuing 8 shards (--single-thread
# --devices 0 x 8) at 256 MiB (c4-4m: 64 x 4 MiB) and 1 GiB (c3) per shard;
# the host_issue field: the thread's issue time per step of 8 launches beside
# the kernel time per launch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in ${CFGS:-c4-4m c3}; do
  timeout -k 10 300 python bench.py --single-thread --devices 0,0,0,0,0,0,0,0 --config $cfg --steps ${STEPS:-20} --warmup 3 \
    --no-cpu-baseline --no-host-path --sustain-seconds 0 > gpurun_out/issue_$cfg.log 2>&1 || { tail -20 gpurun_out/issue_$cfg.log; exit 1; }
  tail -1 gpurun_out/issue_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', json.dumps(d['host_issue']), 'value', d['value'], 'shards_checked', d.get('shards_checked'))"
done
