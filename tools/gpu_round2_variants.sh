# Round-2 MI355X bench set: the driver's default command, then labelled
# variants (each its own bounded run; stop at the first failure).
#   bash tools/gpu_round2_variants.sh A   -> default + strict + 2 queues + idle-interval
#   bash tools/gpu_round2_variants.sh B   -> job KEYS_PER_POD=4 + 60 s-burst long form
#   bash tools/gpu_round2_variants.sh C   -> PyTorch plug-in engine (WORKER_ENGINE)
#   bash tools/gpu_round2_variants.sh D   -> INTERVAL=0.1 (reference loop, fast cadence)
#   bash tools/gpu_round2_variants.sh E   -> POOL_IDLE_RELEASE_S=3 (no GPU held when idle)
#   bash tools/gpu_round2_variants.sh F   -> WARM_POOL_MODE=context (no HBM held)
#   bash tools/gpu_round2_variants.sh G   -> configs 3/5 shapes: strict, 2 queues, jobs KPP=4
set -o pipefail
OUT=${OUT:-gpurun_out/r2_variants}
mkdir -p $OUT
run() {
  tag=$1; limit=$2; shift 2
  echo "== $tag: bench.py $*"
  timeout -k 10 $limit python bench.py "$@" > $OUT/$tag.json 2> $OUT/$tag.err
  rc=$?
  cp gpurun_out/bench_detail_n1.json $OUT/${tag}_detail.json 2>/dev/null
  tail -1 $OUT/$tag.err
  head -c 400 $OUT/$tag.json; echo
  return $rc
}
if [ "$1" = "A" ]; then
  run default 560 --gpus 1 --steps 20 --warmup 5 && \
  run strict 200 --gpus 1 --steps 10 --warmup 1 --policy strict --budget-s 180 && \
  run two_queues 200 --gpus 1 --steps 10 --warmup 1 --queues predict,track --budget-s 180 && \
  run idle_interval_0.1 200 --gpus 1 --steps 10 --warmup 1 --idle-interval 0.1 --budget-s 180
elif [ "$1" = "G" ]; then
  run strict 200 --gpus 1 --steps 10 --warmup 1 --policy strict --budget-s 180 && \
  run two_queues 200 --gpus 1 --steps 10 --warmup 1 --queues predict,track --budget-s 180 && \
  run job_kpp4_strict 260 --gpus 1 --steps 6 --warmup 1 --resource-type job --kpp 4 --on 8 --lam-per-gpu 1.0 --policy strict --budget-s 240 && \
  run job_kpp4_reference 260 --gpus 1 --steps 6 --warmup 1 --resource-type job --kpp 4 --on 8 --lam-per-gpu 1.0 --budget-s 240 --drain-timeout 20
elif [ "$1" = "D" ]; then
  # the reference's own loop at INTERVAL=0.1: only viable with a ~1 ms
  # actuator (with a pod start the same policy thrashes: see the
  # reference_sim_pod_start_* context fields)
  run interval_0.1 200 --gpus 1 --steps 20 --warmup 2 --interval 0.1 --budget-s 180
elif [ "$1" = "E" ]; then
  # deep idle: standbys exit after 3 s without demand (no GPU held between
  # bursts), every scale-up is then a cold spawn
  POOL_IDLE_RELEASE_S=3 run pool_idle_release_3s 200 --gpus 1 --steps 10 --warmup 1 --budget-s 180 --cold-cycles 0
elif [ "$1" = "F" ]; then
  # standbys with a HIP context and no HBM (WARM_POOL_MODE=context)
  run context_norecycle 200 --gpus 1 --steps 10 --warmup 1 --budget-s 180 --pool-mode context --no-recycle --cold-cycles 0
elif [ "$1" = "C" ]; then
  # a user's PyTorch model as the engine (WORKER_ENGINE plug-in): the same
  # standby / recycle / cache path, torch imported by the standby at boot
  WORKER_ENGINE=kiosk_autoscaler_amd.models.torch_engine:TorchMlpEngine \
    run torch_plugin 260 --gpus 1 --steps 8 --warmup 1 --budget-s 240
else
  run job_kpp4_strict 260 --gpus 1 --steps 6 --warmup 1 --resource-type job --kpp 4 --on 8 --lam-per-gpu 1.0 --policy strict --budget-s 240 && \
  run job_kpp4_reference 260 --gpus 1 --steps 6 --warmup 1 --resource-type job --kpp 4 --on 8 --lam-per-gpu 1.0 --budget-s 240 --drain-timeout 20 && \
  run longform_60s_bursts 400 --gpus 1 --steps 2 --warmup 0 --on 60 --budget-s 380 && \
  run import_norecycle 200 --gpus 1 --steps 8 --warmup 2 --budget-s 180 --pool-mode import --no-recycle --cold-cycles 0
fi
