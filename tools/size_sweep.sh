#!/bin/bash
# fused-kernel frac over every supported size / output / dtype (diagnostic):
#   tools/size_sweep.sh [lib-variant]   -> gpurun_out/sweep/*.json
set -u
v=${1:-base}
lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
mkdir -p gpurun_out/sweep
for dt in ${DTYPES:-float32 float64}; do
  for n in 1024 2048 4096 8192 16384; do
    for o in cwt power; do
      ep=$(( 2 * 16384 / n )); [ $ep -lt 2 ] && ep=2
      NINWAVE_LIB=$lib timeout -k 10 200 python bench.py --config c3 --samples $n --output $o --dtype $dt \
        --epochs $ep --chunk 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sweep/$dt-$n-$o.json 2> gpurun_out/sweep/$dt-$n-$o.log || { tail -3 gpurun_out/sweep/$dt-$n-$o.log; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/sweep/$dt-$n-$o.json')); r=d['roofline']; print('%-8s %6d %-6s %-6s ms=%.3f GB/s=%.0f frac=%.3f' % ('$dt', $n, '$o', r['kernel'], r['avg_launch_ms'], r['achieved'], r['frac']))"
    done
  done
done
