# Tighter headline (8 stratified phases) + config-3/5 shaped variants, 60 s bursts.
set -o pipefail
mkdir -p gpurun_out/headline_long
run() { name=$1; shift; timeout -k 10 1500 python bench.py "$@" > gpurun_out/headline_long/$name.json 2> gpurun_out/headline_long/$name.err && cp gpurun_out/bench_detail_n1.json gpurun_out/headline_long/${name}_detail.json; }
run default_k8 --steps 8 --warmup 1 && \
run two_queues --queues predict,track && \
run job_kpp4_strict --resource-type job --kpp 4 --lam-per-gpu 1.0 --policy strict
rc=$?
for f in gpurun_out/headline_long/*.json; do case $f in *_detail.json) ;; *) echo "$f"; cat $f;; esac; done
exit $rc
