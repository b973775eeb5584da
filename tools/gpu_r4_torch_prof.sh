#!/bin/bash
# rocprofv3 kernel trace of the PyTorch-ROCm engine's lifecycle
# (tools/profile_torch_engine.py): an unprofiled timing run, then the
# kernel trace + stats.
set -o pipefail
OUT=${OUT:-gpurun_out/r4_torch_prof}
mkdir -p $OUT
timeout -k 10 120 python tools/profile_torch_engine.py > $OUT/unprofiled.json \
    2> $OUT/unprofiled.err || { tail -20 $OUT/unprofiled.err; exit 1; }
cat $OUT/unprofiled.json
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- \
    python3 tools/profile_torch_engine.py > $OUT/profiled.json \
    2> $OUT/profiled.err || { tail -20 $OUT/profiled.err; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
head -20 $OUT/kernel_stats.csv
