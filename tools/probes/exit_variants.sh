#!/bin/bash
# Exit-teardown variants of tools/probes/exit_probe.py, one environment per
# tag, each case in 3 fresh processes:
#
#   bash tools/probes/exit_variants.sh OUTDIR CASES TAG=ENV[,ENV..] ...
#
# e.g. exit_variants.sh r6_exit ctx,torch_engine_rccl default= svm0=HSA_USE_SVM=0
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/${1:-r6_exit}; cases=${2:-ctx,engine_rccl,torch_engine_rccl}
shift 2
[ $# -eq 0 ] && set -- default= svm0=HSA_USE_SVM=0
mkdir -p "$out"
for spec in "$@"; do
  tag=${spec%%=*} envs=${spec#*=}
  ( IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done
    EXIT_PROBE_SLIM=1 EXIT_PROBE_TAG=$tag timeout -k 10 240 \
      python tools/probes/exit_probe.py "$cases" >> "$out/exit.jsonl" \
      2>> "$out/exit.err" ) || exit $?
done
