#!/bin/bash
# Round-4 validation on one MI355X: the whole GPU suite, smoke(), and the
# driver's exact bench command with the defaults.
set -o pipefail
OUT=${OUT:-gpurun_out/r4_final}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 240 \
    --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
tail -3 $OUT/gpu_tests.log
# a test failure still lets smoke and the bench run; a timeout, an abort
# or a crash does not
case $rc in 0|1) ;; *) echo "pytest rc=$rc"; exit $rc ;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" \
    > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
KIOSK_BENCH_OUT=$OUT/bench timeout -k 10 560 python bench.py --gpus 1 \
    --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err \
    || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
exit $rc
