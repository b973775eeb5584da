"""Per-epoch membership-fence timeline from a bench event log.

    python tools/fence_timeline.py gpurun_out/bench_events_n1.jsonl

For each epoch: manager send -> rank-0 report (``start_to_rank_ms``),
manager send -> ``fence_done`` (what the bench's ``fence_wall_ms_mean``
averages), the rank's own communicator init and wall time, and the
forward-pass pauses the serving loop took for fences (FENCE_YIELD_MS).
"""
import json
import sys


def timeline(path):
    events = [json.loads(line) for line in open(path) if line.strip()]
    start = {e['epoch']: e['t'] for e in events if e.get('ev') == 'fence_start'}
    rank0 = {e['epoch']: e for e in events
             if e.get('ev') == 'fence_rank' and e.get('rank', 0) == 0}
    done = {e['epoch']: e for e in events if e.get('ev') == 'fence_done'}
    rows = []
    for epoch in sorted(start):
        r, d = rank0.get(epoch), done.get(epoch)
        rows.append({
            'epoch': epoch,
            'start_to_rank_ms': (r['t'] - start[epoch]) / 1e6 if r else None,
            'start_to_done_ms': (d['t'] - start[epoch]) / 1e6 if d else None,
            'init_ms': r.get('init_ms') if r else None,
            'rank_wall_ms': r.get('wall_ms') if r else None,
            'mode': r.get('mode') if r else None,
        })
    paused = [e['paused_ms'] for e in events
              if e.get('ev') == 'key_done' and e.get('paused_ms')]
    return rows, paused


def main(argv):
    rows, paused = timeline(argv[1])
    for row in rows:
        print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v)
                          for k, v in row.items()}))
    done = [r['start_to_done_ms'] for r in rows
            if r['start_to_done_ms'] is not None]
    print(json.dumps({
        'epochs': len(rows),
        'start_to_done_ms_mean': round(sum(done) / len(done), 1)
        if done else None,
        'start_to_done_ms_max': round(max(done), 1) if done else None,
        'keys_paused': len(paused),
        'paused_ms_total': round(sum(paused), 1)}))


if __name__ == '__main__':
    main(sys.argv)
