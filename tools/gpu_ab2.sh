#!/bin/bash
# bench A/B over extra bench.py arguments (BENCH_VARIANTS, ';'-separated) x configs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=';' read -ra VARS <<< "${BENCH_VARIANTS:---streams 1}"
i=0
for v in "${VARS[@]}"; do
  for cfg in ${AB_CONFIGS:-c3}; do
    o=gpurun_out/ab2_${i}_$cfg.log
    timeout -k 10 240 python bench.py --config $cfg --steps 30 --no-cpu-baseline --no-host-path $v > $o 2>&1 \
      || { echo "bench '$v' $cfg rc=$?"; tail -5 $o; exit 1; }
    echo "[$v] $cfg: $(tail -1 $o | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["achieved"], d["roofline"]["frac"], d["ms_per_step"], d["roofline"]["avg_launch_us"])')"
  done
  i=$((i+1))
done
