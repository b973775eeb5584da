#!/bin/bash
# Round 4 check on one MI355X: kernel + PyTorch-engine numerics, the RCCL
# collision probe on the fixed READY path (profiles/r4_collision), a
# rocprofv3 hip-trace of it, and a short headline bench with the defaults.
set -o pipefail
OUT=gpurun_out/r4_check
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py \
    tests/test_torch_kiosk.py -x -v -m gpu --timeout 240 \
    --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python tools/rccl_collision_probe.py --seconds 3 \
    --modes none:ready,inproc:ready,inproc:build,inproc:forward \
    --out $OUT/probe.jsonl || exit 1
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --stats \
    --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- \
    python3 tools/rccl_collision_probe.py --child --collider inproc \
    --work ready --seconds 2 > $OUT/prof_stdout.log 2>&1 || exit 1
KIOSK_BENCH_OUT=$OUT/bench timeout -k 10 420 python bench.py --steps 6 \
    --warmup 1 > $OUT/bench.json 2> $OUT/bench.err
