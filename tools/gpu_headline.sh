# Headline (default flags = BASELINE config 4 shape) + the IDLE_INTERVAL and
# strict variants, all with 60 s bursts.
set -o pipefail
mkdir -p gpurun_out/headline
run() { name=$1; shift; timeout -k 10 900 python bench.py "$@" > gpurun_out/headline/$name.json 2> gpurun_out/headline/$name.err && cp gpurun_out/bench_detail_n1.json gpurun_out/headline/${name}_detail.json; }
run default && run idle_interval_0.1 --idle-interval 0.1 && run strict --policy strict
rc=$?
for f in gpurun_out/headline/*.json; do case $f in *_detail.json) ;; *) echo "$f"; cat $f;; esac; done
exit $rc
