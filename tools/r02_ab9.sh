#!/bin/bash
# fp64 XCD tile shapes: timing + one FETCH_SIZE pass each
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
R=gpurun_out/ab9; mkdir -p $R
NINWAVE_LIB=$PWD/ninwavelets_amd/libninwave_t16x2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_shapes.py -x -q --timeout 200 --timeout-method thread -k float64 > $R/pt.log 2>&1; rc=$?; tail -2 $R/pt.log; [ $rc -ne 0 ] && exit $rc
run() {
  local v=$1 cfg=$2 tag=$3; shift 3
  lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
  NINWAVE_LIB=$lib timeout -k 10 200 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline "$@" > $R/$v-$cfg-$tag.json 2> $R/$v-$cfg-$tag.log || { tail -3 $R/$v-$cfg-$tag.log; exit 1; }
  python3 -c "import json; d=json.load(open('$R/$v-$cfg-$tag.json')); r=d['roofline']; print('%-6s %s %s value=%.4e ms/step=%.2f %s %.4f ms frac=%.4f' % ('$v', '$cfg', '$tag', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac']))"
}
for rep in 1 2; do
  for v in base t16x2 t4x8 t32x1 t2x16; do run $v c4 f64r$rep --dtype float64 --epochs 16; done
done
for v in base t16x2 t4x8 t32x1 t2x16; do
  lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
  NINWAVE_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-include-regex nw_fused --pmc FETCH_SIZE -d $R/pmc_$v -o pmc --output-format csv -- python3 bench.py --config c4 --dtype float64 --epochs 16 --steps 1 --warmup 1 --no-cpu-baseline > $R/pmc_$v.log 2>&1 || { tail -3 $R/pmc_$v.log; exit 1; }
  python3 -c "
import csv,glob
v=[float(r['Counter_Value']) for f in glob.glob('$R/pmc_$v/**/*counter_collection.csv',recursive=True) for r in csv.DictReader(open(f))]
print('$v fetch GB/launch (2*FETCH_SIZE KiB)', round(2*sum(v)/len(v)*1024/1e9,3))"
done
