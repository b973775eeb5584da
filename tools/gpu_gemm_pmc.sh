# PMC counters for the GEMM kernels (counters in their own run, kernel trace
# + stats only: no runtime/sys trace alongside --pmc).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --kernel-trace --stats --output-format csv -d gpurun_out/pmc/a -o gemm -- python3 tools/gemm_pmc.py --shapes ${PMC_SHAPES:-2048x16384x4096,2048x4096x16384} --variants ${PMC_VARIANTS:-256,256x128,128} > gpurun_out/pmc/a.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --stats --output-format csv -d gpurun_out/pmc/b -o gemm -- python3 tools/gemm_pmc.py --shapes ${PMC_SHAPES:-2048x16384x4096,2048x4096x16384} --variants ${PMC_VARIANTS:-256,256x128,128} > gpurun_out/pmc/b.log 2>&1
rc=$?
tail -3 gpurun_out/pmc/a.log gpurun_out/pmc/b.log
find gpurun_out/pmc -name '*.csv' | head -20
exit $rc
