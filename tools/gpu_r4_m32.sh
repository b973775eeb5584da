#!/bin/bash
# The 4-wave GEMM on v_mfma_f32_32x32x16_bf16 (gemm_set_mfma32): its GPU
# numerics tests, then an interleaved A/B against the 16x16x32 kernel at
# the worker's shapes and 8192^3.
set -o pipefail
OUT=gpurun_out/r4_m32
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 \
    --timeout-method thread tests/test_gpu_kernels.py -k "mfma32" \
    > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python tools/bench_gemm.py --mfma32 --rounds 7 \
    --shapes 2048x16384x4096,2048x4096x16384,8192x8192x8192 \
    --only native_gelu_auto,native_gelu_auto_m32,native256w4,native256w4_m32,native256w4_gelu,native256w4_gelu_m32,native256splitk,native256splitk_m32,torch \
    > $OUT/bench.jsonl 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.jsonl
