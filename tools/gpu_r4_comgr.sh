#!/bin/bash
# ROCm's comgr under torch's HIP runtime (ops/native.py prefer_rocm_comgr):
# first-stream cost per runtime, the PyTorch standby's boot stages, and the
# torch engine's GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/r4_comgr
mkdir -p "$out"
timeout -k 10 200 python3 tools/first_stream_probe.py --kinds native,torch,torch_rocm_comgr \
  --variants default --repeat 4 > "$out/first_stream.jsonl" 2> "$out/first_stream.err" && \
timeout -k 10 300 python3 tools/torch_boot_probe.py --repeat 3 > "$out/boot.jsonl" 2> "$out/boot.err" && \
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_torch_kiosk.py > "$out/tests.log" 2>&1
rc=$?
tail -n 5 "$out/tests.log"
exit $rc
