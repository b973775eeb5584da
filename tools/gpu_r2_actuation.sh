# Engine-cache GPU tests, then short benches of the standby modes.
set -o pipefail
OUT=gpurun_out/r2_actuation
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py tests/test_faults.py tests/test_hbm_sizing.py -m gpu -x -q --timeout 150 --timeout-method thread -k "cache or recycled or hbm or elementwise" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
run() {
  tag=$1; shift
  timeout -k 10 220 python bench.py "$@" > $OUT/$tag.json 2> $OUT/$tag.err || return 1
  cp gpurun_out/bench_detail_n1.json $OUT/${tag}_detail.json
  python3 -c "import json,sys; d=json.loads(open('$OUT/$tag.json').read().strip().splitlines()[-1]); print('$tag', {k: d.get(k) for k in ('value','vs_baseline','actuation_mean_s','gpu_idle_pct','baseline_gpu_idle_pct','standby_gpu_s','gpu_alive_s','cold_spawn_actuation_s')})"
}
run device_recycle --gpus 1 --steps 8 --warmup 2 --budget-s 200 && \
run import_norecycle --gpus 1 --steps 8 --warmup 2 --budget-s 200 --pool-mode import --no-recycle --cold-cycles 0
