# Soak on one MI355X: 80 fast scale 0 -> 1 -> 0 cycles (INTERVAL=0.2,
# 0.5 s bursts, 0.1 s of GPU work per key) with WORKER_MAX_RECYCLES=25, so
# the recycled worker retires three times: each retirement is shrunk out of
# the RCCL node communicator and the slot's fresh standby joins a new
# generation.  Checks: every key served, no error, idle-HBM drift between
# the first and last idle samples (idle_node_hbm_drift_mib), generations.
set -o pipefail
OUT=${OUT:-gpurun_out/soak}
mkdir -p $OUT
WORKER_MAX_RECYCLES=25 timeout -k 10 480 python bench.py --gpus 1 \
  --steps 80 --warmup 2 --interval 0.2 --on 0.5 --service-ms 100 \
  --cold-cycles 0 --pod-start-s 0 --budget-s 450 \
  > $OUT/soak.json 2> $OUT/soak.err || { tail -30 $OUT/soak.err; exit 1; }
cp gpurun_out/bench_events_n1.jsonl $OUT/soak_events.jsonl 2>/dev/null
tail -2 $OUT/soak.err
cat $OUT/soak.json
