#!/bin/bash
# fp64 chirp-z: E = 8 (4 waves/SIMD, no scratch) vs E = 16 (2 waves/SIMD)
set -u
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/e64; mkdir -p $R
NINWAVE_LIB=$PWD/ninwavelets_amd/libninwave_e64_8.so timeout -k 10 600 python -u -m pytest tests/test_gpu_chirp.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "float64" > $R/pt.log 2>&1; rc=$?; tail -3 $R/pt.log; [ $rc -ne 0 ] && exit $rc
run() {
  local v=$1 tag=$2; shift 2
  lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
  NINWAVE_LIB=$lib timeout -k 10 200 python bench.py --config c3 --epochs 32 --dtype float64 --steps 3 --warmup 1 --no-cpu-baseline "$@" > $R/$v-$tag.json 2> $R/$v-$tag.log || { tail -3 $R/$v-$tag.log; exit 1; }
  python3 -c "import json; d=json.load(open('$R/$v-$tag.json')); r=d['roofline']; print('%-6s %-10s value=%.4e ms/step=%.2f %s %.4f ms' % ('$v', '$tag', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms']))"
}
for rep in 1 2; do for v in base e64_8; do
  run $v p1201-$rep --samples 1201; run $v c1201-$rep --samples 1201 --output cwt; run $v p2049-$rep --samples 2049; run $v p4097-$rep --samples 4097 --epochs 8
done; done
