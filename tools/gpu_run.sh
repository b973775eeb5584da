#!/bin/bash
# Every GPU call of the project through one parametrised script (VERDICT r4
# item 8: it replaces ~40 one-off tools/gpu_*.sh wrappers; the profiles/
# READMEs of earlier rounds still name those, tools/README.md maps them).
#
#   tools/gpu_run.sh tests  TAG                    GPU test suite
#   tools/gpu_run.sh bench  TAG STEPS WARMUP [NAME=ENV[,ENV..] ...]
#                                                  the driver's bench command
#                                                  once per env variant
#   tools/gpu_run.sh round  TAG STEPS WARMUP [...] tests, then bench
#   tools/gpu_run.sh args   TAG STEPS WARMUP NAME -- BENCH_ARGS..
#                                                  the driver's bench command
#                                                  plus bench arguments (the
#                                                  opt-in modes), one variant
#   tools/gpu_run.sh slots  TAG N STEPS -- BENCH_ARGS..
#                                                  N worker slots on the one
#                                                  device (BENCH_GPU_IDS)
#   tools/gpu_run.sh torchrun TAG N STEPS WARMUP   the N>1 launch path
#   tools/gpu_run.sh stats  TAG -- CMD..           rocprofv3 kernel trace +
#                                                  stats of CMD
#   tools/gpu_run.sh pmc    TAG 'COUNTERS' -- CMD.. one PMC pass of CMD
#   tools/gpu_run.sh probe  TAG SECONDS -- CMD..   CMD under a time limit
#
# Output under gpurun_out/TAG.  Every GPU step runs under its own time
# limit; a step that faults, aborts, segfaults or times out ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
recipe=$1; tag=$2; shift 2
out=gpurun_out/$tag
mkdir -p "$out"

fatal() {   # exit codes after which nothing more may touch the GPU
  case $1 in 0|1) return 1;; *) return 0;; esac
}

run_tests() {
  timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > "$out/pytest.log" 2>&1
  local rc=$?
  tail -4 "$out/pytest.log"
  echo "pytest rc $rc"
  return $rc
}

run_bench() {   # STEPS WARMUP [NAME=ENV[,ENV..] ...]
  local steps=$1 warmup=$2; shift 2
  [ $# -eq 0 ] && set -- default=
  for spec in "$@"; do
    local name=${spec%%=*} envs=${spec#*=} dir=$out/${spec%%=*}
    mkdir -p "$dir"
    ( IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done
      export KIOSK_BENCH_OUT=$dir
      timeout -k 10 560 python -u bench.py --gpus 1 --steps "$steps" \
        --warmup "$warmup" --budget-s 520 > "$dir/bench.json" \
        2> "$dir/bench.err" )
    local rc=$?
    if [ $rc -ne 0 ]; then
      echo "variant $name ended with $rc"; tail -5 "$dir/bench.err"
      return $rc
    fi
    tail -1 "$dir/bench.json" | cut -c1-400
  done
}

case $recipe in
  tests)
    run_tests ;;
  bench)
    run_bench "$@" ;;
  round)
    steps=$1; warmup=$2; shift 2
    run_tests; rc=$?
    fatal $rc && { echo "stopping after the GPU tests ($rc)"; exit $rc; }
    run_bench "$steps" "$warmup" "$@" ;;
  args)
    steps=$1; warmup=$2; name=$3; shift 4    # (the -- separator)
    dir=$out/$name; mkdir -p "$dir"
    KIOSK_BENCH_OUT=$dir timeout -k 10 560 python -u bench.py --gpus 1 \
      --steps "$steps" --warmup "$warmup" --budget-s 520 "$@" \
      > "$dir/bench.json" 2> "$dir/bench.err" \
      || { rc=$?; tail -30 "$dir/bench.err"; exit $rc; }
    tail -1 "$dir/bench.json" | cut -c1-400 ;;
  slots)
    n=$1; steps=$2; shift 3            # (the -- separator)
    ids=$(python3 -c "print(','.join(['0'] * $n))")
    BENCH_GPU_IDS=$ids KIOSK_BENCH_OUT=$out timeout -k 10 1000 \
      python -u bench.py --gpus "$n" --steps "$steps" --warmup 0 \
      --budget-s 960 "$@" > "$out/bench.json" 2> "$out/bench.err" \
      || { rc=$?; tail -30 "$out/bench.err"; exit $rc; }
    tail -1 "$out/bench.json" | cut -c1-600 ;;
  torchrun)
    n=$1; steps=$2; warmup=$3
    ids=$(python3 -c "print(','.join(['0'] * $n))")
    BENCH_GPU_IDS=$ids KIOSK_BENCH_OUT=$out timeout -k 10 500 \
      python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
      --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus "$n" \
      --steps "$steps" --warmup "$warmup" > "$out/bench.json" \
      2> "$out/bench.err" || { rc=$?; tail -30 "$out/bench.err"; exit $rc; }
    tail -1 "$out/bench.json" | cut -c1-600 ;;
  stats)
    shift                              # --
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$PWD/$out/prof" -o run -- "$@" > "$out/run.log" 2>&1
    rc=$?
    f=$(find "$out/prof" -name '*kernel_stats.csv' | head -1)
    [ -n "$f" ] && cp "$f" "$out/kernel_stats.csv" && head -20 "$out/kernel_stats.csv"
    find "$out/prof" \( -name '*.db' -o -name '*.csv' -size +15M \) -delete
    tail -3 "$out/run.log"
    exit $rc ;;
  pmc)
    counters=$1; shift 2               # COUNTERS --
    timeout -s KILL 90 rocprofv3 --pmc $counters --kernel-trace --stats \
      --output-format csv -d "$PWD/$out/pmc" -o run -- "$@" \
      > "$out/pmc.log" 2>&1
    rc=$?
    python3 tools/pmc_summary.py "$out/pmc" > "$out/summary.jsonl" 2>/dev/null
    tail -3 "$out/pmc.log"
    exit $rc ;;
  probe)
    secs=$1; shift 2                   # SECONDS --
    timeout -k 10 "$secs" "$@" > "$out/probe.out" 2> "$out/probe.err"
    rc=$?
    tail -20 "$out/probe.out"; tail -5 "$out/probe.err"
    exit $rc ;;
  *)
    echo "unknown recipe $recipe"; exit 2 ;;
esac
