#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--hip-trace`` CSV: the longest HIP API calls
(thread, function, ms) and, for each call of another thread that lasted
longer than ``--hold-ms``, which calls of the main thread overlapped it.

Used for profiles/r4_collision: which HIP call of a worker waits while
RCCL registers its fat binary / loads its code object on another thread.
"""
import argparse
import collections
import csv
import sys


def main(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument('trace')
    parser.add_argument('--top', type=int, default=15)
    parser.add_argument('--hold-ms', type=float, default=200.0)
    args = parser.parse_args(argv)
    rows = list(csv.DictReader(open(args.trace)))
    for r in rows:
        r['t0'] = int(r['Start_Timestamp'])
        r['t1'] = int(r['End_Timestamp'])
        r['ms'] = (r['t1'] - r['t0']) / 1e6
    main_tid = collections.Counter(r['Thread_Id'] for r in rows) \
        .most_common(1)[0][0]
    print('calls %d, main thread %s' % (len(rows), main_tid))
    print('\nlongest calls:')
    for r in sorted(rows, key=lambda r: -r['ms'])[:args.top]:
        print('  %9.2f ms  %-7s %s%s' % (
            r['ms'], r['Thread_Id'], r['Function'],
            '  (main)' if r['Thread_Id'] == main_tid else ''))
    holds = [r for r in rows if r['Thread_Id'] != main_tid and
             r['ms'] >= args.hold_ms]
    for h in holds:
        print('\nwhile %s held %.1f ms on thread %s, the main thread ran:'
              % (h['Function'], h['ms'], h['Thread_Id']))
        by = collections.defaultdict(list)
        for r in rows:
            if r['Thread_Id'] == main_tid and r['t0'] < h['t1'] and \
                    r['t1'] > h['t0']:
                by[r['Function']].append(r['ms'])
        for name, ms in sorted(by.items(), key=lambda kv: -max(kv[1])):
            print('  %-28s n=%-4d max %9.2f ms' % (name, len(ms), max(ms)))
    return 0


if __name__ == '__main__':
    sys.exit(main())
