#!/bin/bash
# Rehearse bench.py's N>1 path (torchrun, barrier, MAX-over-ranks timing) on a
# 1-GPU box: ranks share the GPU over gloo (PECH_BENCH_BACKEND=gloo).  The
# per-rank numbers are not scaling data (ranks contend for one GPU's HBM);
# only the launch, rendezvous and the JSON line are checked.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for n in ${RANKS:-2 4}; do
  PECH_BENCH_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 10 --warmup 3 \
    > gpurun_out/dist_rehearsal_n$n.log 2>&1 || { rc=$?; tail -20 gpurun_out/dist_rehearsal_n$n.log; echo "stop rc=$rc n=$n"; exit $rc; }
  echo "n=$n: $(tail -1 gpurun_out/dist_rehearsal_n$n.log | cut -c1-300)"
done
