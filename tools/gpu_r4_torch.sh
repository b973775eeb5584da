#!/bin/bash
# VERDICT r3 next-step 3 on one MI355X: the PyTorch-ROCm worker on the
# hand-written kernels (models/torch_kiosk.py) under the driver's headline
# command, deep-idle default and resident device pool; the bench's cold
# cycle is its zygote cold spawn (cold_spawn_actuation_s).
set -o pipefail
OUT=gpurun_out/r4_torch
mkdir -p $OUT
export WORKER_ENGINE=kiosk_autoscaler_amd.models.torch_kiosk:TorchKioskEngine
KIOSK_BENCH_OUT=$OUT/deep timeout -k 10 560 python bench.py --gpus 1 \
    --steps 20 --warmup 5 > $OUT/deep_idle.json 2> $OUT/deep_idle.err || exit 1
POOL_IDLE_RELEASE_S=0 KIOSK_BENCH_OUT=$OUT/device timeout -k 10 560 \
    python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/device.json \
    2> $OUT/device.err
