#!/bin/bash
# fp64 n = 16384: E = 16 (1024 threads) with LDS-DMA of X vs E = 32
set -u
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/ab10; mkdir -p $R
NINWAVE_LIB=$PWD/ninwavelets_amd/libninwave_f64e16.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_shapes.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "float64 and (16384 or reference or interpolate)" > $R/pt.log 2>&1; rc=$?; tail -2 $R/pt.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do for v in base f64e16; do
  lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
  NINWAVE_LIB=$lib timeout -k 10 200 python bench.py --config c4 --dtype float64 --epochs 16 --steps 3 --warmup 1 --no-cpu-baseline > $R/$v-$rep.json 2> $R/$v-$rep.log || { tail -3 $R/$v-$rep.log; exit 1; }
  python3 -c "import json; d=json.load(open('$R/$v-$rep.json')); r=d['roofline']; print('%-7s rep$rep value=%.4e %.4f ms frac=%.4f' % ('$v', d['value'], r['avg_launch_ms'], r['frac']))"
done; done
