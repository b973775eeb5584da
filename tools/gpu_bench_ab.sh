#!/bin/bash
# One GPU call: the driver's bench command once per engine (or any env
# variant), each under its own time limit; JSON lines + detail/event files
# under gpurun_out/$TAG/<variant>/.
#   tools/gpu_bench_ab.sh TAG STEPS WARMUP VARIANT=ENV[,ENV..] ...
# e.g. tools/gpu_bench_ab.sh r5_ab 20 5 torch=WORKER_ENGINE=torch-kiosk \
#          builtin=WORKER_ENGINE=builtin
set -o pipefail
tag=$1; steps=$2; warmup=$3; shift 3
mkdir -p gpurun_out/$tag
for spec in "$@"; do
  name=${spec%%=*}; envs=${spec#*=}
  out=gpurun_out/$tag/$name
  mkdir -p $out
  ( IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done
    export KIOSK_BENCH_OUT=$out
    timeout -k 10 560 python -u bench.py --gpus 1 --steps $steps \
      --warmup $warmup --budget-s 520 > $out/bench.json 2> $out/bench.err ) || {
    echo "variant $name failed: $?"; tail -5 $out/bench.err; exit 1; }
  tail -c 3000 $out/bench.json | tail -1 | cut -c1-600
done
