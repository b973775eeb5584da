# A/B of 4-wave GEMM schedule variants (standalone builds of
# tools/gemm_ablate.hip, build/gemm_ab_<name>), interleaved over rounds so
# box drift hits every variant alike.  One JSON line per run.
#   SHAPES="M N K [EPI SPLITS];..."  (EPI 0 none, 1 bias+GELU, 2 bias+residual;
#   SPLITS >= 2: split-K partials + reduce)     ROUNDS=3
set -o pipefail
OUT=${OUT:-gpurun_out/gemm_ab}
mkdir -p $OUT
out=$OUT/ab.jsonl
: > $out
IFS=';' read -ra LIST <<< "${SHAPES:-8192 8192 8192;2048 16384 4096;4096 4096 4096}"
for round in $(seq 1 ${ROUNDS:-3}); do
  for spec in "${LIST[@]}"; do
    set -- $spec
    for b in build/gemm_ab_*; do
      name=$(basename $b)
      line=$(timeout -k 5 60 ./$b $1 $2 $3 4 ${4:-0} ${5:-1}) || exit 1
      echo "{\"variant\": \"$name\", \"round\": $round, \"run\": $line}" >> $out
    done
  done
done
cat $out | wc -l
