#!/bin/bash
# C5 cols-pass ablations (diagnostic variants give wrong results: timing only) + fp64 lines
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
R=gpurun_out/ab3; mkdir -p $R
run() {  # variant cfg tag extra-args
  local v=$1 cfg=$2 tag=$3; shift 3
  lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
  NINWAVE_LIB=$lib timeout -k 10 200 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline "$@" > $R/$v-$cfg-$tag.json 2> $R/$v-$cfg-$tag.log || { tail -3 $R/$v-$cfg-$tag.log; exit 1; }
  python3 -c "import json; d=json.load(open('$R/$v-$cfg-$tag.json')); r=d['roofline']; x=d.get('roofline_rows',{}); print('%-15s %s %s value=%.4e ms/step=%.2f %s %.4f ms frac=%.4f rows=%s' % ('$v', '$cfg', '$tag', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac'], x.get('avg_launch_ms')))"
}
for rep in 1 2; do
  for v in ${VARIANTS:-base colsblk colsnostore colsblknostore}; do run $v c5 r$rep; done
done
run base c4 f64 --dtype float64 --epochs 16
run base c5 f64 --dtype float64
