#!/bin/bash
# Round 4 defaults on one MI355X: can the zygote pre-register RCCL
# (tools/rccl_zygote_probe.py, with and without), then the driver's exact
# headline command with the shipped defaults.
set -o pipefail
OUT=gpurun_out/r4_defaults
mkdir -p $OUT
timeout -k 10 120 python tools/rccl_zygote_probe.py > $OUT/zygote_probe.jsonl \
    2> $OUT/zygote_probe.err || exit 1
timeout -k 10 120 python tools/rccl_zygote_probe.py --preload \
    >> $OUT/zygote_probe.jsonl 2>> $OUT/zygote_probe.err || exit 1
KIOSK_BENCH_OUT=$OUT/bench timeout -k 10 560 python bench.py --gpus 1 \
    --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
