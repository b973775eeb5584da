set -o pipefail
mkdir -p gpurun_out/r1c
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/r1c/gpu_tests.log 2>&1 && \
timeout -k 10 300 python tools/bench_gemm.py > gpurun_out/r1c/bench_gemm.jsonl 2> gpurun_out/r1c/bench_gemm.err && \
bash tools/run_bench_variants.sh job_kpp4 two_queues
rc=$?
tail -5 gpurun_out/r1c/gpu_tests.log
cat gpurun_out/r1c/bench_gemm.jsonl
exit $rc
