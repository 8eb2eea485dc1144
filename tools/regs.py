#!/usr/bin/env python3
"""Per-kernel VGPR / scratch / occupancy table of one HIP source (gfx950), from
clang's -Rpass-analysis=kernel-resource-usage remarks.
    python tools/regs.py ninwavelets_amd/csrc/nw_large.hip [filter]"""
import os
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ''
cmd = ['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++20', '-fno-slp-vectorize', *os.environ.get('DEFS', '').split(),
       '--cuda-device-only', '-c', src, '-o', '/tmp/_regs.co', '-Rpass-analysis=kernel-resource-usage']
err = subprocess.run(cmd, capture_output=True, text=True, cwd=None).stderr
rows, cur = [], None
for line in err.splitlines():
    m = re.search(r'Function Name: (\S+)', line)
    if m:
        cur = {'name': m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r'remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|SGPRs): (\d+)', line)
    if m and cur is not None:
        cur[m.group(1).split()[0]] = int(m.group(2))
dm = subprocess.run(['c++filt'], input='\n'.join(r['name'] for r in rows), capture_output=True, text=True).stdout.splitlines()
for r, d in zip(rows, dm):
    if flt in d:
        print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('ScratchSize', '?'):>4} scratch occ {r.get('Occupancy', '?')}  {d[:150]}")
if 'error' in err:
    print(err[-3000:])
