"""Kernel timeline of a rocprofv3 --kernel-trace run: per kernel its mean duration, and the
idle gap on the GPU before each launch (end of the previous kernel -> start of this one).
    python tools/trace_gaps.py <dir with *kernel_trace.csv> [--last K] [--match REGEX]
--last K: only the last K launches of the matching kernels' timeline (the timed loop).
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dir')
    ap.add_argument('--last', type=int, default=0)
    ap.add_argument('--match', default='nw_|fwd_r2c|rows_kernel|cols_kernel|k_')
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.dir, '**', '*kernel_trace.csv'), recursive=True)
    if not files:
        raise SystemExit(f'no kernel_trace.csv under {a.dir}')
    rows = []
    with open(files[0]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    rows.sort()
    pat = re.compile(a.match)
    rows = [r for r in rows if pat.search(r[2])]
    if a.last:
        rows = rows[-a.last:]
    per = {}
    for i, (s, e, k) in enumerate(rows):
        short = k.split('(')[0].split('<')[0].replace('void ', '').replace('nw::(anonymous namespace)::', '')
        d = per.setdefault(short, {'dur_us': [], 'gap_before_us': []})
        d['dur_us'].append((e - s) / 1e3)
        if i:
            d['gap_before_us'].append((s - rows[i - 1][1]) / 1e3)
    span = (rows[-1][1] - rows[0][0]) / 1e3 if rows else 0.0
    out = {'trace': os.path.relpath(files[0]), 'launches': len(rows), 'span_us': round(span, 1), 'kernels': {}}
    for k, d in per.items():
        out['kernels'][k] = {'launches': len(d['dur_us']),
                             'mean_dur_us': round(statistics.mean(d['dur_us']), 2),
                             'min_dur_us': round(min(d['dur_us']), 2), 'max_dur_us': round(max(d['dur_us']), 2),
                             'mean_gap_before_us': round(statistics.mean(d['gap_before_us']), 2)
                             if d['gap_before_us'] else None}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
