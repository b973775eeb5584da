# Fence-yield check: GPU tests, then the default bench (2 timed bursts) with
# FENCE_YIELD_MS at $1 (default 250; 0 = the old behaviour).
set -o pipefail
mkdir -p gpurun_out/fy
Y=${1:-250}
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/fy/gpu_tests.log 2>&1 && \
FENCE_YIELD_MS=$Y timeout -k 10 500 python bench.py --steps 2 --warmup 1 > gpurun_out/fy/bench_y$Y.json 2> gpurun_out/fy/bench_y$Y.err && \
cp gpurun_out/bench_events_n1.jsonl gpurun_out/fy/events_y$Y.jsonl
rc=$?
tail -2 gpurun_out/fy/gpu_tests.log; cat gpurun_out/fy/bench_y$Y.json
exit $rc
