# Round-3 MI355X bench set: what the standby pool holds vs what it costs.
#   bash tools/gpu_round3_tiers.sh A -> default (driver command, short) +
#        ENGINE_IDLE_RELEASE_S=5 with 6 s idle gaps (engine tier)
#   bash tools/gpu_round3_tiers.sh B -> context + recycle (node comm over
#        shm) + deep idle (POOL_IDLE_RELEASE_S=3)
#   bash tools/gpu_round3_tiers.sh C -> torch plug-in: warm pool, context,
#        cold spawn
#   bash tools/gpu_round3_tiers.sh D -> deep idle, built-in and torch engine
#        (node generation deferred until the woken worker is READY)
#   bash tools/gpu_round3_tiers.sh E -> deep idle woken by arrivals
#        (POOL_WAKE_POLL_S): release after 3 s and after 1 s, built-in and
#        torch engine
#   bash tools/gpu_round3_tiers.sh F -> deep idle woken POOL_WAKE_LEAD_S
#        before the tick, released 0.5 s after the scale-down: the driver's
#        command (20 + 5 steps), then the torch plug-in
#   bash tools/gpu_round3_tiers.sh G -> config-4 shape (60 s Poisson bursts,
#        60 s off), resident pool vs arrival-woken deep idle
#   bash tools/gpu_round3_tiers.sh H -> engine tier (ENGINE_IDLE_RELEASE_S=5,
#        6 s idle gaps) with the arrival-driven engine rebuild
#   bash tools/gpu_round3_tiers.sh I -> deep idle that keeps RCCL (release
#        60 s, 65 s idle gaps): wake, READY, then the RCCL generation
set -o pipefail
OUT=${OUT:-gpurun_out/r3_tiers}
mkdir -p $OUT
run() {
  tag=$1; limit=$2; shift 2
  echo "== $tag: bench.py $*"
  timeout -k 10 $limit python bench.py "$@" > $OUT/$tag.json 2> $OUT/$tag.err
  rc=$?
  cp gpurun_out/bench_detail_n1.json $OUT/${tag}_detail.json 2>/dev/null
  cp gpurun_out/bench_events_n1.jsonl $OUT/${tag}_events.jsonl 2>/dev/null
  tail -1 $OUT/$tag.err
  head -c 600 $OUT/$tag.json; echo
  return $rc
}
if [ "$1" = "A" ]; then
  run default 300 --gpus 1 --steps 8 --warmup 2 --budget-s 250 && \
  ENGINE_IDLE_RELEASE_S=5 run engine_release_5s 300 --gpus 1 --steps 8 --warmup 1 --off 6 --budget-s 270 --cold-cycles 0
elif [ "$1" = "B" ]; then
  run context_recycle 260 --gpus 1 --steps 10 --warmup 1 --budget-s 230 --pool-mode context --cold-cycles 0 && \
  POOL_IDLE_RELEASE_S=3 run pool_idle_release_3s 260 --gpus 1 --steps 10 --warmup 1 --budget-s 230 --cold-cycles 0
elif [ "$1" = "C" ]; then
  WORKER_ENGINE=kiosk_autoscaler_amd.models.torch_engine:TorchMlpEngine \
    run torch_device 260 --gpus 1 --steps 6 --warmup 1 --budget-s 230 && \
  WORKER_ENGINE=kiosk_autoscaler_amd.models.torch_engine:TorchMlpEngine \
    run torch_context 260 --gpus 1 --steps 6 --warmup 1 --budget-s 230 --pool-mode context --cold-cycles 0 && \
  WORKER_ENGINE=kiosk_autoscaler_amd.models.torch_engine:TorchMlpEngine POOL_IDLE_RELEASE_S=3 \
    run torch_deep_idle 260 --gpus 1 --steps 6 --warmup 1 --budget-s 230 --cold-cycles 0
elif [ "$1" = "D" ]; then
  POOL_IDLE_RELEASE_S=3 run deep_idle_v2 260 --gpus 1 --steps 10 --warmup 1 --budget-s 230 --cold-cycles 0 && \
  WORKER_ENGINE=kiosk_autoscaler_amd.models.torch_engine:TorchMlpEngine POOL_IDLE_RELEASE_S=3 \
    run torch_deep_idle_v2 260 --gpus 1 --steps 6 --warmup 1 --budget-s 230 --cold-cycles 0
elif [ "$1" = "E" ]; then
  POOL_IDLE_RELEASE_S=3 run deep_idle_wake_3s 260 --gpus 1 --steps 10 --warmup 1 --budget-s 230 --cold-cycles 0 && \
  POOL_IDLE_RELEASE_S=1 run deep_idle_wake_1s 260 --gpus 1 --steps 10 --warmup 1 --budget-s 230 --cold-cycles 0 && \
  WORKER_ENGINE=kiosk_autoscaler_amd.models.torch_engine:TorchMlpEngine POOL_IDLE_RELEASE_S=1 \
    run torch_deep_idle_wake_1s 260 --gpus 1 --steps 6 --warmup 1 --budget-s 230 --cold-cycles 0
elif [ "$1" = "F" ]; then
  POOL_IDLE_RELEASE_S=0.5 run deep_idle_lead 330 --gpus 1 --steps 20 --warmup 5 && \
  WORKER_ENGINE=kiosk_autoscaler_amd.models.torch_engine:TorchMlpEngine POOL_IDLE_RELEASE_S=0.5 \
    run torch_deep_idle_lead 260 --gpus 1 --steps 8 --warmup 1 --budget-s 230 --cold-cycles 0
elif [ "$1" = "G" ]; then
  run config4_resident 420 --gpus 1 --steps 2 --warmup 0 --on 60 --off 60 --budget-s 400 --cold-cycles 0 && \
  POOL_IDLE_RELEASE_S=0.5 run config4_deep_idle_wake 420 --gpus 1 --steps 2 --warmup 0 --on 60 --off 60 --budget-s 400 --cold-cycles 0
elif [ "$1" = "H" ]; then
  ENGINE_IDLE_RELEASE_S=5 run engine_release_5s_rebuild 300 --gpus 1 --steps 8 --warmup 1 --off 6 --budget-s 270 --cold-cycles 0
elif [ "$1" = "I" ]; then
  POOL_IDLE_RELEASE_S=60 run deep_idle_rccl_60s 420 --gpus 1 --steps 3 --warmup 0 --off 65 --budget-s 400 --cold-cycles 0
fi
