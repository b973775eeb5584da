#!/usr/bin/env python3
"""Tick -> READY of every scale-up in a bench event log (JSONL): for each
``scale`` event that raised the target (the autoscaler's stamp right after
its PATCH), the time to the next ``worker_ready`` (the worker's own READY
stamp; the benchmark's ``actuation_s``) and the manager's assign ->
READY.  Prints a JSON summary: count, median,
p99, max, and the scale-ups above ``--limit-ms`` (none above
50 ms in the soak)."""
import argparse
import json
import sys


def main(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument('events')
    parser.add_argument('--limit-ms', type=float, default=50.0)
    args = parser.parse_args(argv)
    events = [json.loads(l) for l in open(args.events) if l.strip()]
    events.sort(key=lambda e: e.get('t', 0))
    rows = []
    for i, e in enumerate(events):
        if e.get('ev') != 'scale' or e.get('desired', 0) <= e.get('current',
                                                                   0):
            continue
        ready = next((u for u in events[i + 1:]
                      if u.get('ev') == 'worker_ready'), None)
        up = next((u for u in events[i + 1:] if u.get('ev') == 'worker_up'),
                  None)
        if ready is None:
            continue
        rows.append({'t': e['t'],
                     'tick_to_ready_ms': (ready['t'] - e['t']) / 1e6,
                     'assign_to_ready_ms': (1e3 * float(up.get('ready_s') or 0)
                                            if up else None),
                     'from_pool': up.get('from_pool') if up else None})
    lat = sorted(r['tick_to_ready_ms'] for r in rows)

    def pct(q):
        return round(lat[min(len(lat) - 1, int(q * len(lat)))], 3) \
            if lat else None
    over = [r for r in rows if r['tick_to_ready_ms'] > args.limit_ms]
    print(json.dumps({'scale_ups': len(rows), 'median_ms': pct(0.5),
                      'p99_ms': pct(0.99), 'max_ms': pct(1.0),
                      'limit_ms': args.limit_ms, 'over_limit': len(over),
                      'over': over[:10]}))
    return 0


if __name__ == '__main__':
    sys.exit(main())
