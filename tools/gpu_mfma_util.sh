# MFMA busy-over-active of the production forward, hipBLASLt at the same
# shapes and the warm-start calibration kernel (every SIMD issuing
# back-to-back MFMAs): one counter group per rocprofv3 run (kernel trace +
# stats only beside --pmc), each under its own time limit.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r3_mfma_util}
mkdir -p $OUT
run() {
  name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --stats \
    --output-format csv -d $OUT/$name -o fwd -- \
    python3 tools/forward_pmc.py > $OUT/$name.log 2>&1
}
run a SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE && \
run b SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE
rc=$?
python3 tools/pmc_summary.py $OUT/a $OUT/b > $OUT/summary.jsonl
grep -h "calib\|forward" $OUT/*.log
exit $rc
