#!/bin/bash
# signal-pair kernel X by LDS-DMA: parity (fp32 suites), then C3 / pair sizes A/B
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
R=gpurun_out/ab7; mkdir -p $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_shapes.py tests/test_gpu_dedup.py tests/test_gpu_scales.py -x -q --timeout 200 --timeout-method thread > $R/pt.log 2>&1; rc=$?; tail -3 $R/pt.log; [ $rc -ne 0 ] && exit $rc
run() {
  local v=$1 cfg=$2 tag=$3; shift 3
  lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
  NINWAVE_LIB=$lib timeout -k 10 200 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline "$@" > $R/$v-$cfg-$tag.json 2> $R/$v-$cfg-$tag.log || { tail -3 $R/$v-$cfg-$tag.log; exit 1; }
  python3 -c "import json; d=json.load(open('$R/$v-$cfg-$tag.json')); r=d['roofline']; print('%-6s %s %s value=%.4e ms/step=%.2f %s %.4f ms frac=%.4f' % ('$v', '$cfg', '$tag', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac']))"
}
for rep in 1 2; do
  for v in base nopxd; do run $v c3 r$rep; run $v c3 cwt$rep --output cwt --epochs 128; done
done
for v in base nopxd; do for n in 1024 2048; do run $v c3 n${n} --samples $n --epochs 128; done; done
