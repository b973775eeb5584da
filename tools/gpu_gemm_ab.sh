# GEMM kernel A/B on one box: numerics tests for every variant, then the
# TFLOP/s table (tools/bench_gemm.py) into gpurun_out/gemm_ab/.
set -o pipefail
mkdir -p gpurun_out/gemm_ab
timeout -k 10 240 python -m pytest tests/test_gpu_kernels.py -x -q > gpurun_out/gemm_ab/tests.log 2>&1 && \
timeout -k 10 300 python tools/bench_gemm.py --rounds 7 > gpurun_out/gemm_ab/bench.jsonl 2> gpurun_out/gemm_ab/bench.err
rc=$?
tail -3 gpurun_out/gemm_ab/tests.log
cat gpurun_out/gemm_ab/bench.jsonl
exit $rc
