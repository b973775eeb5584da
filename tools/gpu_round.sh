#!/bin/bash
# The round's standard GPU call: the GPU test suite, then the driver's bench
# command (tools/gpu_bench_ab.sh variants).  A GPU step that faults, aborts,
# segfaults or times out ends the call (no further GPU work after it).
#   tools/gpu_round.sh TAG [STEPS WARMUP [VARIANT=ENV ...]]
set -o pipefail
tag=$1; steps=${2:-20}; warmup=${3:-5}; shift 3 2>/dev/null
mkdir -p gpurun_out/$tag
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/$tag/pytest.log 2>&1
rc=$?
tail -4 gpurun_out/$tag/pytest.log
echo "pytest rc $rc"
case $rc in 0|1) ;; *) echo "stopping: GPU test step ended with $rc"; exit $rc;; esac
[ $# -eq 0 ] && set -- default=
exec tools/gpu_bench_ab.sh $tag $steps $warmup "$@"
