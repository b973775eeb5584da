#!/bin/bash
# Counters of the 4-wave GEMM on 16x16x32 vs 32x32x16 MFMAs (same launch,
# gemm_set_mfma32): MFMA busy, LDS bank conflicts, LDS waits.  Counters in
# their own runs, kernel trace + stats only.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4_m32_pmc
mkdir -p $OUT
ARGS="--shapes 8192x8192x8192,2048x16384x4096 --variants 256w4 --mfma32"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/a -o gemm -- python3 tools/gemm_pmc.py $ARGS > $OUT/a.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/b -o gemm -- python3 tools/gemm_pmc.py $ARGS > $OUT/b.log 2>&1 && \
python tools/pmc_summary.py $OUT/a $OUT/b > $OUT/summary.jsonl
rc=$?
cat $OUT/summary.jsonl | cut -c1-600
exit $rc
