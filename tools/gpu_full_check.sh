# Round-end rehearsal: GPU test suite, graft smoke(), a short default bench.
set -o pipefail
mkdir -p gpurun_out/full
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/full/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > gpurun_out/full/smoke.log 2>&1 && \
timeout -k 10 900 python bench.py --steps 2 --warmup 1 > gpurun_out/full/bench.json 2> gpurun_out/full/bench.err
rc=$?
tail -3 gpurun_out/full/gpu_tests.log; tail -2 gpurun_out/full/smoke.log; cat gpurun_out/full/bench.json
exit $rc
