#!/bin/bash
# Torch-free and PyTorch workers on the same box under the driver's N=1
# command, then the PyTorch worker on the N=4 launch path with every slot
# on the one device (4 torch standbys and workers sharing it).
set -o pipefail
OUT=gpurun_out/r4_torch_default
mkdir -p $OUT
KIOSK_BENCH_OUT=$OUT/native timeout -k 10 560 python bench.py --gpus 1 \
    --steps 20 --warmup 5 > $OUT/native_n1.json 2> $OUT/native_n1.err \
    || { tail -30 $OUT/native_n1.err; exit 1; }
cat $OUT/native_n1.json
export WORKER_ENGINE=kiosk_autoscaler_amd.models.torch_kiosk:TorchKioskEngine
KIOSK_BENCH_OUT=$OUT/torch timeout -k 10 560 python bench.py --gpus 1 \
    --steps 20 --warmup 5 > $OUT/torch_n1.json 2> $OUT/torch_n1.err \
    || { tail -30 $OUT/torch_n1.err; exit 1; }
cat $OUT/torch_n1.json
BENCH_GPU_IDS=0,0,0,0 KIOSK_BENCH_OUT=$OUT/torch_n4 timeout -k 10 400 \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 4 \
    --steps 8 --warmup 2 > $OUT/torch_n4.json 2> $OUT/torch_n4.err \
    || { tail -30 $OUT/torch_n4.err; exit 1; }
cat $OUT/torch_n4.json
