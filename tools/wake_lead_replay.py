#!/usr/bin/env python3
"""Replay woken-standby boot times against wake-lead estimators
(``gpumgr/pool.py:wake_lead``).

Input: bench event logs (``bench_events_n1.jsonl``) or a JSON file of boot
sequences (``{"runs": [[boot_s, ...], ...]}``, as
``profiles/r5_boot/woken_boots.json``).  For every woken boot after the
first of its run, the lead each estimator would have set from the boots
before it is compared with the boot: lateness (boot - lead, when positive)
is READY after the tick, hold (lead - boot) is a standby waiting for it.

    python tools/wake_lead_replay.py profiles/r5_boot/woken_boots.json
    python tools/wake_lead_replay.py --dump OUT.json EVENTS.jsonl [...]
"""
import argparse
import json
import sys

CAP_S = 0.75


def boots_of(path):
    """Spawn -> booted+prebuilt of each fresh standby a wake started in one
    event log: after the pool first parked (the pool's first boot and cold
    spawns are not wakes)."""
    out = []
    events = []
    with open(path) as fh:
        for line in fh:
            try:
                events.append(json.loads(line))
            except ValueError:
                continue
    parked = False
    retired = set()     # (logs of 184647d..: a retired worker's report)
    for ev in sorted(events, key=lambda e: e.get('t', 0)):
        if ev.get('ev') == 'pool_parked':
            parked = True
        elif ev.get('ev') == 'worker_retired':
            retired.add(ev.get('pid'))
        elif parked and ev.get('ev') == 'standby_ready' and \
                ev.get('boot_s') and not ev.get('recycled') and \
                ev.get('pid') not in retired:
            out.append(float(ev['boot_s']))
    return out


def slowest(window):
    def est(hist):
        return max(hist[-window:])
    return est


def second_slowest(window, min_samples=4):
    def est(hist):
        recent = sorted(hist[-window:])
        return recent[-2] if len(recent) >= min_samples else recent[-1]
    return est


def spread_margin(k=1.5, floor=0.01, hi=0.06, window=16):
    """gpumgr/pool.py ``wake_lead`` since round 6: second slowest of the
    window plus ``floor + k * (second slowest - median)``, clamped."""
    def est(hist):
        recent = sorted(hist[-window:])
        if len(recent) < 4:
            return recent[-1] + 0.05
        sized, median = recent[-2], recent[len(recent) // 2]
        return sized + min(hi, max(floor, floor + k * (sized - median)))
    return est


ESTIMATORS = {
    'slowest of 8': slowest(8),
    'slowest of 16': slowest(16),
    'second slowest of 8': second_slowest(8),
    'second slowest of 16': second_slowest(16),
}


def replay(runs, est, margin):
    late = hold = 0.0
    n = lates = 0
    for boots in runs:
        for i in range(1, len(boots)):
            lead = min(CAP_S, est(boots[:i]) + margin)
            late += max(0.0, boots[i] - lead)
            hold += max(0.0, lead - boots[i])
            lates += boots[i] > lead
            n += 1
    return {'late_ms_per_wake': round(late / n * 1e3, 2) if n else None,
            'hold_ms_per_wake': round(hold / n * 1e3, 1) if n else None,
            'late_wakes': lates, 'wakes': n}


def main(argv=None):
    parser = argparse.ArgumentParser(description=__doc__)
    parser.add_argument('inputs', nargs='+')
    parser.add_argument('--dump', default='')
    parser.add_argument('--min-boots', type=int, default=10)
    args = parser.parse_args(argv)
    runs = []
    for path in args.inputs:
        if path.endswith('.json'):
            with open(path) as fh:
                runs.extend(json.load(fh)['runs'])
        else:
            boots = boots_of(path)
            if len(boots) >= args.min_boots:
                runs.append(boots)
    if args.dump:
        with open(args.dump, 'w') as fh:
            json.dump({'runs': runs}, fh)
    print('%d runs, %d woken boots' % (len(runs), sum(map(len, runs))))
    for k in (1.0, 1.5, 2.0, 3.0):
        row = replay(runs, spread_margin(k), 0.0)
        print('second slowest of 16 + spread margin (k=%g): late %5.2f '
              'ms/wake (%d of %d), hold %5.1f ms/wake' % (
                  k, row['late_ms_per_wake'], row['late_wakes'],
                  row['wakes'], row['hold_ms_per_wake']))
    for name, est in ESTIMATORS.items():
        for margin in (0.03, 0.04, 0.05):
            row = replay(runs, est, margin)
            print('%-22s + %2.0f ms: late %5.2f ms/wake (%d of %d), hold '
                  '%5.1f ms/wake' % (name, margin * 1e3,
                                     row['late_ms_per_wake'],
                                     row['late_wakes'], row['wakes'],
                                     row['hold_ms_per_wake']))
    return 0


if __name__ == '__main__':
    sys.exit(main())
