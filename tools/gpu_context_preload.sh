# WARM_POOL_MODE=context with and without the code-object preload: standby
# HBM (probe) and actuation (bench), one box.  Each step bounded.
set -o pipefail
OUT=gpurun_out/ctxpre
mkdir -p $OUT
timeout -k 10 120 python tools/standby_hbm_probe.py > $OUT/hbm_probe.jsonl 2> $OUT/hbm_probe.err || { tail -20 $OUT/hbm_probe.err; exit 1; }
cat $OUT/hbm_probe.jsonl
for pre in 1 0; do
  CONTEXT_PRELOAD=$pre timeout -k 10 240 python bench.py --steps 8 --warmup 1 \
    --pool-mode context --no-recycle --cold-cycles 0 \
    > $OUT/context_pre$pre.json 2> $OUT/context_pre$pre.err || { tail -20 $OUT/context_pre$pre.err; exit 1; }
  python -c "import json,sys;d=json.loads(open('$OUT/context_pre$pre.json').read().splitlines()[-1]);print('preload=$pre',{k:d.get(k) for k in ('value','vs_baseline','actuation_mean_s','gpu_idle_pct','baseline_gpu_idle_pct','standby_pool_boot_hbm_mib','idle_node_hbm_mib','keys_done','keys')})"
done
