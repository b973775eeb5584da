# One GPU call: the driver's default `python bench.py` (N=1) exactly as the
# round end runs it, with its detail JSON kept.
set -o pipefail
mkdir -p gpurun_out/r1h
timeout -k 10 900 python bench.py > gpurun_out/r1h/bench.json 2> gpurun_out/r1h/bench.err && \
cp gpurun_out/bench_detail_n1.json gpurun_out/r1h/bench_detail_n1.json
rc=$?
cat gpurun_out/r1h/bench.json
exit $rc
