mkdir -p gpurun_out/r4_stream
export AMD_COMGR_CACHE=1 AMD_COMGR_CACHE_DIR=/tmp/cc AMD_COMGR_TIME_STATISTICS=1 AMD_COMGR_EMIT_VERBOSE_LOGS=1 AMD_COMGR_REDIRECT_LOGS=stderr
for k in torch torch native native; do
  timeout -k 10 60 python3 tools/first_stream_probe.py --child $k > gpurun_out/r4_stream/verbose_$k.$RANDOM.log 2>&1 || exit 1
done
ls -la /tmp/cc > gpurun_out/r4_stream/cache_ls.txt
