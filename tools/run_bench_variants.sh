# Bench variants beyond the headline (docs/BENCHMARKS.md).  Usage:
#   bash tools/run_bench_variants.sh [name ...]   (default: all)
set -o pipefail
mkdir -p gpurun_out/variants
run() { name=$1; shift; timeout -k 10 600 python bench.py --gpus 1 "$@" > gpurun_out/variants/$name.json 2> gpurun_out/variants/$name.err && cp gpurun_out/bench_detail_n1.json gpurun_out/variants/${name}_detail.json; }
variant() {
  case $1 in
    strict) run strict --steps 3 --warmup 1 --policy strict ;;
    idle_fastpoll) run idle_fastpoll --steps 3 --warmup 1 --idle-interval 0.1 ;;
    # reference floor division strands < KEYS_PER_POD residual keys in job
    # mode, so the job variant runs the strict policy
    job_kpp4) run job_kpp4 --steps 2 --warmup 1 --resource-type job --kpp 4 --lam-per-gpu 1.0 --policy strict ;;
    two_queues) run two_queues --steps 3 --warmup 1 --queues predict,track ;;
    *) echo "unknown variant $1"; return 2 ;;
  esac
}
names=${*:-strict idle_fastpoll job_kpp4 two_queues}
rc=0
for n in $names; do variant $n || { rc=$?; break; }; done
echo "variants rc=$rc"
for f in gpurun_out/variants/*.json; do case $f in *_detail.json) ;; *) echo "$f"; cat $f; echo;; esac; done
exit $rc
