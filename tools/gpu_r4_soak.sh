#!/bin/bash
# VERDICT r3 next-step 1 "done when", on one MI355X: the round-3 soak (80
# fast 0 -> 1 -> 0 cycles, a resident device pool, WORKER_MAX_RECYCLES=25
# so the worker retires three times and each replacement standby builds a
# new RCCL generation) -- no scale-up more than 50 ms after its tick.
set -o pipefail
OUT=${OUT:-gpurun_out/r4_soak}
mkdir -p $OUT
POOL_IDLE_RELEASE_S=0 WORKER_MAX_RECYCLES=25 KIOSK_BENCH_OUT=$OUT \
  timeout -k 10 480 python bench.py --gpus 1 \
  --steps 80 --warmup 2 --interval 0.2 --on 0.5 --service-ms 100 \
  --cold-cycles 0 --pod-start-s 0 --budget-s 450 \
  > $OUT/soak.json 2> $OUT/soak.err || { tail -30 $OUT/soak.err; exit 1; }
python tools/soak_actuation.py $OUT/bench_events_n1.jsonl > $OUT/actuation.json
cat $OUT/actuation.json
