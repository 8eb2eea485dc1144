#!/bin/bash
# own forward R2C kernel: full GPU suite, then C4 / C3 / C2 A/B against rocFFT's R2C + copy
set -u
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/fwdab; mkdir -p $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $R/pt.log 2>&1; rc=$?; tail -3 $R/pt.log; [ $rc -ne 0 ] && exit $rc
run() {
  local v=$1 cfg=$2 tag=$3; shift 3
  lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
  NINWAVE_LIB=$lib timeout -k 10 200 python bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline "$@" > $R/$v-$cfg-$tag.json 2> $R/$v-$cfg-$tag.log || { tail -3 $R/$v-$cfg-$tag.log; exit 1; }
  python3 -c "import json; d=json.load(open('$R/$v-$cfg-$tag.json')); r=d['roofline']; st=d['stage_ms_per_step']; print('%-6s %s %s value=%.4e ms/step=%.3f kernel %.4f ms frac=%.4f fwd=%.3f copy=%.3f' % ('$v', '$cfg', '$tag', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], st['ms_forward'], st['ms_copy']))"
}
for rep in 1 2; do for v in base noown; do run $v c4 r$rep; run $v c3 r$rep; run $v c2 r$rep; run $v c4 f64r$rep --dtype float64 --epochs 16; done; done
