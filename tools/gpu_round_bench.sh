# One GPU call: worker lifecycle profile (kernel + roctx marker trace),
# headline bench (reference policy) and the IDLE_INTERVAL variant.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r1d
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d gpurun_out/r1d/prof_worker -o worker -- python3 tools/profile_worker.py > gpurun_out/r1d/profile_worker.json 2> gpurun_out/r1d/profile_worker.err && \
timeout -k 10 900 python bench.py --steps 3 --warmup 1 > gpurun_out/r1d/bench.json 2> gpurun_out/r1d/bench.err && \
cp gpurun_out/bench_detail_n1.json gpurun_out/r1d/bench_detail_n1.json && \
bash tools/run_bench_variants.sh idle_fastpoll
rc=$?
cat gpurun_out/r1d/profile_worker.json gpurun_out/r1d/bench.json
find gpurun_out/r1d/prof_worker -name '*stats*' | head
exit $rc
