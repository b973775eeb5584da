# rocprofv3 kernel trace + stats of one worker lifecycle on the final
# round-3 tree (standby preinit -> engine -> warm-start -> graph -> keys),
# then the same run unprofiled for host-side stage times.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r3_worker}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats \
  --output-format csv -d $OUT/prof -o worker -- \
  python3 tools/profile_worker.py > $OUT/profile_worker.json \
  2> $OUT/profile_worker.err && \
timeout -k 10 300 python tools/profile_worker.py \
  > $OUT/profile_worker_unprofiled.json 2>> $OUT/profile_worker.err
rc=$?
find $OUT/prof -name '*stats.csv' | head -5
cat $OUT/profile_worker_unprofiled.json
exit $rc
