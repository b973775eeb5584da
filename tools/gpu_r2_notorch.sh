set -o pipefail
OUT=gpurun_out/r2_notorch
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "faults or hbm or node or recycled or cache" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 220 python bench.py --gpus 1 --steps 8 --warmup 2 --budget-s 200 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cp gpurun_out/bench_detail_n1.json gpurun_out/bench_events_n1.jsonl $OUT/
grep -m3 "services up\|warmup 0" $OUT/bench.err
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('value','vs_baseline','actuation_mean_s','gpu_idle_pct','baseline_gpu_idle_pct','cold_spawn_actuation_s','cold_spawn_latency_s','wall_s')}, d['fence'])"
python3 - <<'PY'
import json
ev=[json.loads(l) for l in open('gpurun_out/r2_notorch/bench_events_n1.jsonl')]
for e in ev:
    if e['ev'] in ('standby_ready',) and not e.get('recycled'):
        print('standby boot_s', round(e['boot_s'],3), 'preinit', e.get('preinit'))
PY
