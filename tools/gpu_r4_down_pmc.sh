#!/bin/bash
# Counters of the worker's two production GEMMs (down-projection split-K
# partials + reduce, up-projection 4-wave): MFMA busy, LDS conflicts.  In
# their own runs, kernel trace + stats only.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4_down_pmc
mkdir -p $OUT
ARGS="--shapes 2048x4096x16384,2048x16384x4096 --variants auto --iters 20"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/a -o gemm -- python3 tools/gemm_pmc.py $ARGS > $OUT/a.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/b -o gemm -- python3 tools/gemm_pmc.py $ARGS > $OUT/b.log 2>&1 && \
python tools/pmc_summary.py $OUT/a $OUT/b > $OUT/summary.jsonl
rc=$?
cat $OUT/summary.jsonl | cut -c1-600
exit $rc
