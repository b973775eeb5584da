#!/bin/bash
# Excess-standby retirement: config 3 under strict (where drained workers
# recycle mid-burst), then the driver's N=1 command (unchanged expected).
set -o pipefail
OUT=gpurun_out/r4_retire
mkdir -p $OUT
BENCH_GPU_IDS=0,0,0,0,0,0,0,0 KIOSK_BENCH_OUT=$OUT/c3 \
    timeout -k 10 560 python bench.py --gpus 8 --steps 2 --warmup 0 \
    --queues predict,track --kpp 1 --on 60 --off 60 --budget-s 520 \
    --policy strict > $OUT/c3_strict.json 2> $OUT/c3_strict.err \
    || { tail -30 $OUT/c3_strict.err; exit 1; }
cat $OUT/c3_strict.json
KIOSK_BENCH_OUT=$OUT/n1 timeout -k 10 560 python bench.py --gpus 1 \
    --steps 20 --warmup 5 > $OUT/bench_n1.json 2> $OUT/bench_n1.err \
    || { tail -30 $OUT/bench_n1.err; exit 1; }
cat $OUT/bench_n1.json
