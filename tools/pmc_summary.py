#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (one or more passes) per kernel.

Usage: python tools/pmc_summary.py gpurun_out/pmc/a gpurun_out/pmc/b
Prints one JSON line per kernel with the mean of each counter per dispatch
and derived ratios: MFMA busy over active (SQ_VALU_MFMA_BUSY_CYCLES, the
SIMD-cycles the matrix pipes were busy -- 16 per v_mfma_f32_16x16x32_bf16,
its issue interval -- summed over the 1024 SIMDs, over 1024 x the kernel's
cycles = GRBM_GUI_ACTIVE / 8, the counter summing the 8 XCDs: checked with
the warm-start kernel, whose own s_memtime / s_memrealtime stamps give the
shader clock, profiles/r3_mfma_util/), the shader clock that implies when
the kernel trace gives durations, LDS bank-conflict share, and the
wave-cycle split (parked / issue-stalled / issuing).
"""
import collections
import csv
import glob
import json
import os
import sys


def load_pass(d):
    """kernel -> counter -> mean per dispatch, for one rocprofv3 run."""
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    counts = collections.defaultdict(lambda: collections.defaultdict(set))
    for path in glob.glob(os.path.join(d, '**', '*counter_collection*.csv'),
                          recursive=True):
        with open(path) as handle:
            for row in csv.DictReader(handle):
                name = row.get('Kernel_Name', '')
                counter = row.get('Counter_Name', '')
                value = float(row.get('Counter_Value', 0) or 0)
                dispatch = row.get('Dispatch_Id', '')
                sums[name][counter] += value
                counts[name][counter].add(dispatch)
    return {name: {c: v / max(1, len(counts[name][c]))
                   for c, v in by_counter.items()}
            for name, by_counter in sums.items()}


def load(dirs):
    """Per kernel, each counter averaged over the passes that collected it.
    (Round 2 summed a counter collected in several passes -- GRBM_GUI_ACTIVE
    rides along in most -- over dispatch ids that repeat from pass to pass,
    inflating it by the number of passes.)"""
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for name, counters in load_pass(d).items():
            for c, v in counters.items():
                acc[name][c].append(v)
    return {name: {c: sum(v) / len(v) for c, v in by_counter.items()}
            for name, by_counter in acc.items()}


SIMDS = 1024          # 256 CUs x 4
GRBM_INSTANCES = 8    # GRBM_GUI_ACTIVE summed over the 8 XCDs


def durations(dirs):
    """Kernel name -> mean duration (ns) from the kernel-trace stats."""
    out = {}
    for d in dirs:
        for path in glob.glob(os.path.join(d, '**', '*kernel_stats.csv'),
                              recursive=True):
            with open(path) as handle:
                for row in csv.DictReader(handle):
                    try:
                        out[row['Name']] = float(row['AverageNs'])
                    except (KeyError, ValueError):
                        pass
    return out


def derive(c, duration_ns=None):
    d = {}
    if c.get('GRBM_GUI_ACTIVE') and 'SQ_VALU_MFMA_BUSY_CYCLES' in c:
        cycles = c['GRBM_GUI_ACTIVE'] / GRBM_INSTANCES
        d['kernel_cycles'] = cycles
        d['mfma_busy_over_active'] = c['SQ_VALU_MFMA_BUSY_CYCLES'] / (
            SIMDS * cycles)
        if duration_ns:
            d['shader_clock_ghz'] = cycles / duration_ns
    if c.get('SQ_LDS_IDX_ACTIVE'):
        d['lds_conflict_share'] = c.get('SQ_LDS_BANK_CONFLICT', 0) / \
            c['SQ_LDS_IDX_ACTIVE']
    total = sum(c.get(k, 0) for k in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY',
                                      'SQ_ACTIVE_INST_ANY'))
    if total:
        for k in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY'):
            d[k.lower() + '_share'] = c.get(k, 0) / total
    return d


def main():
    data = load(sys.argv[1:])
    times = durations(sys.argv[1:])
    for name, counters in sorted(data.items()):
        short = name.replace('kiosk::(anonymous namespace)::', '')
        short = short.replace('void ', '').split('(')[0]
        row = {'kernel': short}
        row.update({k: round(v, 1) for k, v in sorted(counters.items())})
        row.update({k: round(v, 4) for k, v in
                    derive(counters, times.get(name)).items()})
        print(json.dumps(row))


if __name__ == '__main__':
    main()
