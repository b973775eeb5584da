#!/bin/bash
# Reference vs strict policy with real HIP workers: 4 slots on the one
# MI355X (BENCH_GPU_IDS), QUEUES=predict,track, KEYS_PER_POD=1 -- the
# multi-queue inflation the reference policy keeps and the
# strict policy removes.  4 workers on one device, not a scaling point.
set -o pipefail
OUT=gpurun_out/r4_policy
mkdir -p $OUT
for policy in reference strict; do
  BENCH_GPU_IDS=0,0,0,0 KIOSK_BENCH_OUT=$OUT/$policy timeout -k 10 420 \
      python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
      --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 \
      --steps 8 --warmup 1 --queues predict,track --policy $policy \
      > $OUT/$policy.json 2> $OUT/$policy.err \
      || { tail -30 $OUT/$policy.err; exit 1; }
  cat $OUT/$policy.json
done
