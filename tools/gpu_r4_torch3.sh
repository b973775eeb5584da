#!/bin/bash
# The two GPU tests fixed after r4_final, then the PyTorch engine under the
# driver's command on the deep-idle default (engine build now ~3 ms).
set -o pipefail
OUT=gpurun_out/r4_torch3
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread \
    "tests/test_gpu_kernels.py::test_fence_warmup_and_preinit" \
    "tests/test_plugin_engine.py::test_gpu_torch_engine_plugin_serves_on_mi355x" \
    > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
export WORKER_ENGINE=kiosk_autoscaler_amd.models.torch_kiosk:TorchKioskEngine
KIOSK_BENCH_OUT=$OUT/deep timeout -k 10 560 python bench.py --gpus 1 \
    --steps 20 --warmup 5 > $OUT/deep_idle.json 2> $OUT/deep_idle.err \
    || { tail -30 $OUT/deep_idle.err; exit 1; }
cat $OUT/deep_idle.json
