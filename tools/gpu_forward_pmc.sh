# PMC counters of the production forward (ours) and hipBLASLt at the same
# shapes: one counter group per rocprofv3 run (no runtime/sys trace beside
# --pmc), each under its own time limit; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_fwd
mkdir -p $OUT
run() {
  name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --stats \
    --output-format csv -d $OUT/$name -o fwd -- \
    python3 tools/forward_pmc.py > $OUT/$name.log 2>&1
}
run a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE && \
run b SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE && \
run c FETCH_SIZE GRBM_GUI_ACTIVE && \
run d WRITE_SIZE TCC_HIT_sum && \
run e TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
rc=$?
python3 tools/pmc_summary.py $OUT/a $OUT/b $OUT/c $OUT/d $OUT/e > $OUT/summary.jsonl
tail -2 $OUT/*.log
exit $rc
