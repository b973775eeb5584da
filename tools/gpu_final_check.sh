# Round-end rehearsal on one MI355X: the GPU test suite, smoke(), and the
# driver's exact bench command; each step bounded, stop at the first failure.
set -o pipefail
OUT=${OUT:-gpurun_out/final}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 580 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cp gpurun_out/bench_detail_n1.json $OUT/
tail -2 $OUT/bench.err
cat $OUT/bench.json
