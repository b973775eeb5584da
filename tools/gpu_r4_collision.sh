#!/bin/bash
# Round 4: does an RCCL generation's one-time load still stall a worker's
# launches once every kernel launch goes through a resolved handle?
# (kernels/launch.hpp; profiles/r4_collision)
set -o pipefail
OUT=gpurun_out/r4_collision_fix
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q \
    --timeout 120 --timeout-method thread -m gpu > $OUT/gpu_kernels.log 2>&1 || exit 1
timeout -k 10 400 python tools/rccl_collision_probe.py --seconds 3 \
    --modes none:ready,inproc:ready,inproc:build,inproc:forward \
    --out $OUT/probe.jsonl || exit 1
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --stats \
    --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- \
    python3 tools/rccl_collision_probe.py --child --collider inproc \
    --work ready --seconds 2 > $OUT/prof_stdout.log 2>&1
