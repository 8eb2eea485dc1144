#!/bin/bash
# fp64 rows XD and C4 group-size A/B (parity of the rx64 build on fp64 two-pass tests first)
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
R=gpurun_out/ab8; mkdir -p $R
NINWAVE_LIB=$PWD/ninwavelets_amd/libninwave_rx64.so timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_bench_shapes.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "float64 or f64 or reference or c5" > $R/pt.log 2>&1; rc=$?; tail -3 $R/pt.log; [ $rc -ne 0 ] && exit $rc
NINWAVE_LIB=$PWD/ninwavelets_amd/libninwave_g16.so timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_shapes.py -x -q --timeout 200 --timeout-method thread > $R/pt16.log 2>&1; rc=$?; tail -3 $R/pt16.log; [ $rc -ne 0 ] && exit $rc
run() {
  local v=$1 cfg=$2 tag=$3; shift 3
  lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
  NINWAVE_LIB=$lib timeout -k 10 200 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline "$@" > $R/$v-$cfg-$tag.json 2> $R/$v-$cfg-$tag.log || { tail -3 $R/$v-$cfg-$tag.log; exit 1; }
  python3 -c "import json; d=json.load(open('$R/$v-$cfg-$tag.json')); r=d['roofline']; x=d.get('roofline_rows',{}); print('%-6s %s %s value=%.4e ms/step=%.2f %s %.4f ms frac=%.4f rows=%s' % ('$v', '$cfg', '$tag', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac'], x.get('avg_launch_ms')))"
}
for rep in 1 2; do
  for v in base rx64; do run $v c5 f64r$rep --dtype float64; done
  for v in base g16 g4; do run $v c4 r$rep; run $v c3 r$rep; done
done
