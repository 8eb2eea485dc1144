#!/bin/bash
# fp64 twiddle bases from the LDS split table vs global table loads
set -u
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/split; mkdir -p $R
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_bench_shapes.py tests/test_gpu_chirp.py tests/test_gpu_dedup.py -x -q --timeout 200 --timeout-method thread -k "float64 or f64 or reference or c5" > $R/pt.log 2>&1; rc=$?; tail -3 $R/pt.log; [ $rc -ne 0 ] && exit $rc
run() {
  local v=$1 cfg=$2 tag=$3; shift 3
  lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
  NINWAVE_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline "$@" > $R/$v-$cfg-$tag.json 2> $R/$v-$cfg-$tag.log || { tail -3 $R/$v-$cfg-$tag.log; exit 1; }
  python3 -c "import json; d=json.load(open('$R/$v-$cfg-$tag.json')); r=d['roofline']; x=d.get('roofline_rows',{}); print('%-8s %s %s value=%.4e ms/step=%.2f %s %.4f ms frac=%.4f rows=%s' % ('$v', '$cfg', '$tag', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac'], x.get('avg_launch_ms')))"
}
for rep in 1 2; do for v in base nosplit; do
  run $v c4 f64r$rep --dtype float64 --epochs 16
  run $v c4 f64n4096r$rep --dtype float64 --epochs 16 --samples 4096
  run $v c5 f64r$rep --dtype float64
done; done
