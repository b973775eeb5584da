#!/bin/bash
# The PyTorch engine's standby boot with ROCm's comgr (prefer_rocm_comgr)
# and no torch kernel on the boot path, its GPU tests, then the driver's
# command on the deep-idle default with that engine.
set -o pipefail
OUT=${OUT:-gpurun_out/r4_comgr2}
mkdir -p $OUT
timeout -k 10 300 python3 tools/torch_boot_probe.py --repeat 3 > $OUT/boot_worker_order.jsonl 2> $OUT/boot_worker_order.err \
    || { tail -20 $OUT/boot_worker_order.err; exit 1; }
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_torch_kiosk.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -n 1 $OUT/tests.log
export WORKER_ENGINE=kiosk_autoscaler_amd.models.torch_kiosk:TorchKioskEngine
KIOSK_BENCH_OUT=$OUT/deep timeout -k 10 560 python bench.py --gpus 1 \
    --steps 20 --warmup 5 > $OUT/deep_idle.json 2> $OUT/deep_idle.err \
    || { tail -30 $OUT/deep_idle.err; exit 1; }
cat $OUT/deep_idle.json
