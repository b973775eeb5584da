#!/bin/bash
# Config 3 (tools/gpu_r4_config3.sh) under the strict policy: the same 8
# HIP workers on the one MI355X, QUEUES=predict,track, 60 s on / 60 s off.
# Strict sums the queues before clipping, so the multi-queue inflation of
# the reference policy (profiles/r4_config3) should vanish.
set -o pipefail
OUT=gpurun_out/r4_config3_strict
mkdir -p $OUT
BENCH_GPU_IDS=0,0,0,0,0,0,0,0 KIOSK_BENCH_OUT=$OUT \
    timeout -k 10 560 python bench.py --gpus 8 --steps 2 --warmup 0 \
    --queues predict,track --kpp 1 --on 60 --off 60 --budget-s 520 \
    --policy strict > $OUT/bench.json 2> $OUT/bench.err \
    || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
