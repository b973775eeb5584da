# A/B of 4-wave GEMM schedule variants (standalone builds of
# tools/gemm_ablate.hip, build/gemm_ab_<name>), interleaved over rounds so
# box drift hits every variant alike.  One JSON line per run.
set -o pipefail
OUT=${OUT:-gpurun_out/gemm_ab}
mkdir -p $OUT
out=$OUT/ab.jsonl
: > $out
for round in 1 2 3; do
  for shape in "8192 8192 8192" "2048 16384 4096" "4096 4096 4096"; do
    for b in build/gemm_ab_*; do
      name=$(basename $b)
      line=$(timeout -k 5 60 ./$b $shape 4) || exit 1
      echo "{\"variant\": \"$name\", \"round\": $round, \"run\": $line}" >> $out
    done
  done
done
cat $out | wc -l
