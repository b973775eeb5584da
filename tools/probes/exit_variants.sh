set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/r6_exit; mkdir -p $out
for tag in default svm0; do
  envs=""
  [ $tag = svm0 ] && envs="HSA_USE_SVM=0"
  env $envs EXIT_PROBE_SLIM=1 EXIT_PROBE_TAG=$tag timeout -k 10 240 python tools/probes/exit_probe.py ctx,engine_rccl,torch_engine_rccl >> $out/exit.jsonl 2>> $out/exit.err || exit $?
done
