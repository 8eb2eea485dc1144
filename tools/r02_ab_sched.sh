#!/bin/bash
# fused kernels built with the max-ILP machine scheduler (-mllvm -amdgpu-sched-strategy=max-ilp)
# vs the default scheduler: C4 and C3, interleaved twice on one box
set -u
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/absched; mkdir -p $R
NINWAVE_LIB=$PWD/ninwavelets_amd/libninwave_ilp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_shapes.py -m gpu -x -q --timeout 200 --timeout-method thread > $R/pt.log 2>&1; rc=$?; tail -1 $R/pt.log; [ $rc -ne 0 ] && exit $rc
for cfg in c4 c3; do for rep in 1 2; do for v in base ilp; do
  lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
  NINWAVE_LIB=$lib timeout -k 10 200 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline > $R/$cfg-$v-$rep.json 2> $R/$cfg-$v-$rep.log || { tail -3 $R/$cfg-$v-$rep.log; exit 1; }
  python3 -c "import json; d=json.load(open('$R/$cfg-$v-$rep.json')); r=d['roofline']; print('%s %-5s rep$rep value=%.4e %.4f ms frac=%.4f' % ('$cfg', '$v', d['value'], r['avg_launch_ms'], r['frac']))"
done; done; done
