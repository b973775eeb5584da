#!/bin/bash
# Demand-sized deep-idle pool on one MI355X: the driver's N=1 command (the
# one slot is the worker's: nothing should change), then the N=4 launch
# path with every slot on the one device (BENCH_GPU_IDS) to read the
# standby hold.
set -o pipefail
OUT=gpurun_out/r4_sized
mkdir -p $OUT
KIOSK_BENCH_OUT=$OUT/n1 timeout -k 10 560 python bench.py --gpus 1 \
    --steps 20 --warmup 5 > $OUT/bench_n1.json 2> $OUT/bench_n1.err \
    || { tail -30 $OUT/bench_n1.err; exit 1; }
cat $OUT/bench_n1.json
BENCH_GPU_IDS=0,0,0,0 KIOSK_BENCH_OUT=$OUT/n4 timeout -k 10 400 \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 4 \
    --steps 8 --warmup 2 > $OUT/bench_n4.json 2> $OUT/bench_n4.err \
    || { tail -30 $OUT/bench_n4.err; exit 1; }
cat $OUT/bench_n4.json
