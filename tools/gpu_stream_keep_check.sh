# The GPU suite + smoke on the current tree, then the worker start-up profile
# (assign -> READY stages of a fresh device standby).  Each step bounded.
set -o pipefail
OUT=gpurun_out/keep
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python tools/profile_worker.py > $OUT/profile_worker.json 2> $OUT/profile_worker.err || { tail -20 $OUT/profile_worker.err; exit 1; }
cat $OUT/profile_worker.json
