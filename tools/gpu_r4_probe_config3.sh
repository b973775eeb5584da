#!/bin/bash
# Torch vs torch-free standby boot breakdown, then BASELINE config 3 with 8
# HIP workers on the one MI355X (tools/gpu_r4_config3.sh).
set -o pipefail
mkdir -p gpurun_out/r4_boot
timeout -k 10 240 python tools/torch_boot_probe.py --repeat 3 \
    > gpurun_out/r4_boot/probe.jsonl 2> gpurun_out/r4_boot/probe.err \
    || { tail -20 gpurun_out/r4_boot/probe.err; exit 1; }
cat gpurun_out/r4_boot/probe.jsonl
bash tools/gpu_r4_config3.sh
