#!/usr/bin/env python3
"""Per-kernel register / LDS / occupancy report for every gfx950 kernel
(hipcc -Rpass-analysis=kernel-resource-usage), as a markdown table.

    python tools/resource_usage.py > profiles/kernel_resource_usage.md
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ('VGPRs', 'AGPRs', 'SGPRs', 'ScratchSize [bytes/lane]',
          'Occupancy [waves/SIMD]', 'LDS Size [bytes/block]',
          'SGPRs Spill', 'VGPRs Spill')


def demangle(names):
    try:
        out = subprocess.run(['c++filt'], input='\n'.join(names),
                             stdout=subprocess.PIPE, text=True).stdout
        return out.splitlines()
    except OSError:
        return names


def main():
    rows = []
    for src in sorted(glob.glob(os.path.join(ROOT, 'csrc', 'kernels',
                                             '*.hip'))):
        with tempfile.TemporaryDirectory() as tmp:
            proc = subprocess.run(
                ['hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17',
                 '-I' + os.path.join(ROOT, 'csrc'), '-c', src, '-o',
                 os.path.join(tmp, 'k.o'),
                 '-Rpass-analysis=kernel-resource-usage'],
                stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        current = None
        for line in proc.stdout.splitlines():
            m = re.search(r'Function Name: (\S+)', line)
            if m:
                current = {'file': os.path.basename(src), 'name': m.group(1)}
                rows.append(current)
                continue
            for field in FIELDS:
                m = re.search(re.escape(field) + r': (\d+)', line)
                if m and current is not None:
                    current[field] = m.group(1)
    names = demangle([r['name'] for r in rows])
    print('| file | kernel | ' + ' | '.join(FIELDS) + ' |')
    print('|' + '---|' * (2 + len(FIELDS)))
    for row, name in zip(rows, names):
        short = name.replace('kiosk::(anonymous namespace)::', '')
        short = re.sub(r'\(.*\)$', '', short)
        print('| %s | `%s` | %s |' % (row['file'], short, ' | '.join(
            row.get(f, '') for f in FIELDS)))


if __name__ == '__main__':
    sys.exit(main())
