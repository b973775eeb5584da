# The driver's N>1 launch path (torchrun, one bench rank per GPU, gloo
# barrier + max-reduce, rank-0 JSON) on a 1-GPU box: BENCH_GPU_IDS=0,0 puts
# both worker slots on the one device, so RCCL refuses the node communicator
# (duplicate GPU) and the fence falls back to the store transport.
set -o pipefail
OUT=gpurun_out/n2
mkdir -p $OUT
export BENCH_GPU_IDS=0,0
timeout -k 10 560 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --steps ${STEPS:-8} --warmup ${WARMUP:-2} \
  > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cp gpurun_out/bench_detail_n2.json $OUT/ 2>/dev/null
tail -4 $OUT/bench.err
cat $OUT/bench.json
