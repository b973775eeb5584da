# 4-wave GEMM: GPU kernel tests + GEMM microbenchmark (one process each)
set -o pipefail
mkdir -p gpurun_out/w4
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > gpurun_out/w4/tests.log 2>&1 && \
timeout -k 10 300 python tools/bench_gemm.py --rounds 7 --shapes ${SHAPES:-2048x16384x4096,2048x4096x16384,4096x4096x4096,8192x8192x8192} > gpurun_out/w4/bench.jsonl 2> gpurun_out/w4/bench.err
rc=$?
tail -3 gpurun_out/w4/tests.log; cat gpurun_out/w4/bench.jsonl
exit $rc
