# 4-wave ring GEMM variants / ablations (diagnostic builds of
# tools/gemm_ablate.hip: build/gemm_ablate_<ablate bits>)
set -o pipefail
mkdir -p gpurun_out/ablate
out=gpurun_out/ablate/ablate.jsonl
: > $out
for shape in "8192 8192 8192" "2048 16384 4096"; do
  timeout -k 5 60 ./build/gemm_ablate_0 $shape 8 >> $out || exit 1
  for b in build/gemm_ablate_*; do
    timeout -k 5 60 ./$b $shape 4 >> $out || exit 1
  done
done
cat $out
