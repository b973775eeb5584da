#!/bin/bash
# The PyTorch engine's GPU tests and its boot breakdown with the preinit
# stream reused and the arena from hipMalloc + DLPack.
set -o pipefail
OUT=gpurun_out/r4_alloc4
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 180 \
    --timeout-method thread tests/test_torch_kiosk.py > $OUT/tests.log 2>&1 \
    || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python tools/torch_boot_probe.py --repeat 2 \
    > $OUT/boot.jsonl 2> $OUT/boot.err || { tail -20 $OUT/boot.err; exit 1; }
cat $OUT/boot.jsonl
