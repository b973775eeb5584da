#!/bin/bash
# Round-4 validation on one MI355X: the torch boot probe (torch's bundled
# HIP runtime vs the image's), the whole GPU suite, smoke(), and the
# driver's exact bench command with the defaults.
set -o pipefail
OUT=${OUT:-gpurun_out/r4_final}
mkdir -p $OUT
timeout -k 10 200 python tools/torch_boot_probe.py --repeat 2 \
    > $OUT/boot.jsonl 2> $OUT/boot.err || { tail -20 $OUT/boot.err; exit 1; }
cat $OUT/boot.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 \
    --timeout-method thread > $OUT/gpu_tests.log 2>&1 \
    || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" \
    > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
KIOSK_BENCH_OUT=$OUT/bench timeout -k 10 560 python bench.py --gpus 1 \
    --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err \
    || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
