# Fence-yield by short chunks (no pause): default bench, 2 timed bursts.
set -o pipefail
mkdir -p gpurun_out/fy
FENCE_YIELD_MS=0 FENCE_YIELD_CHUNK_MS=${1:-2} timeout -k 10 500 python bench.py --steps 2 --warmup 1 > gpurun_out/fy/bench_chunk.json 2> gpurun_out/fy/bench_chunk.err && \
cp gpurun_out/bench_events_n1.jsonl gpurun_out/fy/events_chunk.jsonl
rc=$?
cat gpurun_out/fy/bench_chunk.json
exit $rc
