# Tile-row group size of the 4-wave 256x256 GEMM: time (A/B in one process,
# against hipBLASLt) and L2 fetch per group size (rocprofv3 --pmc, kernel
# trace + stats only), each step under its own time limit.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r3_group_m}
mkdir -p $OUT
timeout -k 10 300 python3 tools/bench_gemm.py --rounds 7 --group-m 1,2,8 \
  --shapes 2048x16384x4096,8192x8192x8192,2048x4096x16384 \
  --only native256w4,native256w4_gelu,native256w4_gm1,native256w4_gm2,native256w4_gm8,native256w4_gelu_gm1,native256w4_gelu_gm2,native256w4_gelu_gm8,torch,torch_gelu \
  > $OUT/bench.jsonl 2> $OUT/bench.err && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace --stats \
  --output-format csv -d $OUT/fetch -o f -- \
  python3 tools/gemm_fetch_probe.py > $OUT/fetch.log 2>&1 && \
python3 tools/gemm_fetch_probe.py --summarize $OUT/fetch > $OUT/fetch_summary.jsonl
