set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r1g
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d gpurun_out/r1g/prof_worker -o worker -- python3 tools/profile_worker.py > gpurun_out/r1g/profile_worker.json 2> gpurun_out/r1g/profile_worker.err && \
timeout -k 10 300 python tools/profile_worker.py > gpurun_out/r1g/profile_worker_unprofiled.json 2>> gpurun_out/r1g/profile_worker.err
rc=$?
cat gpurun_out/r1g/profile_worker_unprofiled.json
exit $rc
