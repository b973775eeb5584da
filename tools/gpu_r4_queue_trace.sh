#!/bin/bash
# Which HSA calls make the first hardware queue cost ~85 ms in torch's
# bundled runtime and ~15 ms in the image's ROCm 7.2 (profiles/r4_boot)?
# One standby boot per runtime under rocprofv3 --hsa-trace --hip-trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
out=gpurun_out/r4_queue
mkdir -p "$out"
for kind in torch native; do
  timeout -k 10 180 rocprofv3 --hsa-trace --hip-trace --output-format csv -d "$out/$kind" -o q \
    -- python3 tools/torch_boot_probe.py --child "$kind" --model 1024x4096x2 \
    > "$out/$kind.log" 2>&1 || { echo "rocprofv3 $kind failed: $?"; exit 1; }
  for t in hsa_api hip_api; do
    f=$(ls "$out/$kind"/*"${t}_trace.csv" 2>/dev/null | head -n 1 || true)
    if [ -n "$f" ]; then
      python3 tools/hip_trace_longest.py "$f" --top 30 --hold-ms 1e9 \
        > "$out/${kind}_${t}_longest.txt"
    fi
  done
done
find "$out" \( -name '*.db' -o -name '*.csv' -size +15M \) -delete
ls -R "$out" | head -n 40 || true
echo done
