#!/bin/bash
# BASELINE config 3 with real HIP workers on the one MI355X of a gpurun box:
# QUEUES=predict,track, MAX_PODS=8, KEYS_PER_POD=1, lambda = 2/s, 60 s on /
# 60 s off.  All 8 slots are the same device (BENCH_GPU_IDS): 8 workers on
# one GPU, NOT a scaling point.  RCCL refuses 8 ranks on one device, so the
# node communicator falls back to shared memory (reported as such).
set -o pipefail
OUT=gpurun_out/r4_config3
mkdir -p $OUT
BENCH_GPU_IDS=0,0,0,0,0,0,0,0 KIOSK_BENCH_OUT=$OUT \
    timeout -k 10 560 python bench.py --gpus 8 --steps 2 --warmup 0 \
    --queues predict,track --kpp 1 --on 60 --off 60 --budget-s 520 \
    > $OUT/bench.json 2> $OUT/bench.err
