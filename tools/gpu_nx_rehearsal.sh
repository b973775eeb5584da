# The driver's N>1 launch path (torchrun, one bench rank per GPU, gloo
# barrier + max-reduce, rank-0 JSON) on a 1-GPU box, N = 2 then 4:
# BENCH_GPU_IDS puts every worker slot on the one device, so RCCL refuses
# the node communicator (duplicate GPU) and the fence falls back to the
# shared-memory transport (FENCE_FALLBACK).  Each N under its own limit.
set -o pipefail
OUT=${OUT:-gpurun_out/nx}
mkdir -p $OUT
run() {
  n=$1; ids=$2; port=$3
  BENCH_GPU_IDS=$ids timeout -k 10 400 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus $n --steps ${STEPS:-8} \
    --warmup ${WARMUP:-2} > $OUT/bench_n$n.json 2> $OUT/bench_n$n.err \
    || { tail -30 $OUT/bench_n$n.err; return 1; }
  cp gpurun_out/bench_detail_n$n.json $OUT/ 2>/dev/null
  tail -3 $OUT/bench_n$n.err
  cat $OUT/bench_n$n.json
}
run 2 0,0 29511 && run 4 0,0,0,0 29512
