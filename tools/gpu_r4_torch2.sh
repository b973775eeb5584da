#!/bin/bash
# The PyTorch worker after the serving-path and build fixes: its GPU tests,
# then the driver's command on the deep-idle default (the prebuilt events
# carry the engine build's stages).
set -o pipefail
OUT=gpurun_out/r4_torch2
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 \
    --timeout-method thread tests/test_torch_kiosk.py > $OUT/tests.log 2>&1 \
    || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
export WORKER_ENGINE=kiosk_autoscaler_amd.models.torch_kiosk:TorchKioskEngine
KIOSK_BENCH_OUT=$OUT/deep timeout -k 10 560 python bench.py --gpus 1 \
    --steps 20 --warmup 5 > $OUT/deep_idle.json 2> $OUT/deep_idle.err \
    || { tail -30 $OUT/deep_idle.err; exit 1; }
cat $OUT/deep_idle.json
