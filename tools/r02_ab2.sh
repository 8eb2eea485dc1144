#!/bin/bash
# parity (large + fused subsets), then A/B: C5 rows XD (base vs noxrows), C3/C4 tiles and pad16
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
R=gpurun_out/ab2; mkdir -p $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_shapes.py tests/test_gpu_large.py tests/test_gpu_dedup.py -x -q --timeout 200 --timeout-method thread > $R/pt.log 2>&1; rc=$?; tail -3 $R/pt.log; [ $rc -ne 0 ] && exit $rc
run() {  # variant cfg tag extra-args
  local v=$1 cfg=$2 tag=$3; shift 3
  lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
  NINWAVE_LIB=$lib timeout -k 10 200 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline "$@" > $R/$v-$cfg-$tag.json 2> $R/$v-$cfg-$tag.log || { tail -3 $R/$v-$cfg-$tag.log; exit 1; }
  python3 -c "import json; d=json.load(open('$R/$v-$cfg-$tag.json')); r=d['roofline']; x=d.get('roofline_rows',{}); print('%-8s %s %s value=%.4e ms/step=%.2f %s %.4f ms frac=%.4f rows=%s' % ('$v', '$cfg', '$tag', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac'], x.get('avg_launch_ms')))"
}
for rep in 1 2; do
  for v in base noxrows; do run $v c5 r$rep; done
done
for rep in 1 2; do
  for v in base pad16 tf16 tf32; do run $v c3 r$rep; run $v c4 r$rep --epochs 128; done
done
