#!/bin/bash
# C4 signals per launch (bench --chunk): 512 vs 1024 vs 2048, interleaved twice
set -u
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/chunk; mkdir -p $R
for rep in 1 2; do for c in 512 1024 2048; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --chunk $c > $R/c$c-$rep.json 2> $R/c$c-$rep.log || { tail -3 $R/c$c-$rep.log; exit 1; }
  python3 -c "import json; d=json.load(open('$R/c$c-$rep.json')); r=d['roofline']; print('chunk $c rep$rep value=%.4e ms/step=%.2f kernel %.4f ms frac=%.4f' % (d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac']))"
done; done
