#!/bin/bash
# hybrid chirp-z (wide rows via rocFFT, the rest on chip) vs whole-wavelet rocFFT fallback
set -u
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/hyb; mkdir -p $R
run() {
  local v=$1 tag=$2; shift 2
  lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
  NINWAVE_LIB=$lib timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline "$@" > $R/$v-$tag.json 2> $R/$v-$tag.log || { tail -3 $R/$v-$tag.log; exit 1; }
  python3 -c "import json; d=json.load(open('$R/$v-$tag.json')); r=d['roofline']; st=d['stage_ms_per_step']; print('%-6s %-12s value=%.4e ms/step=%.2f engine=%s %s chirp=%.2f mul=%.2f inv=%.2f epi=%.2f exp=%.2f' % ('$v', '$tag', d['value'], d['ms_per_step'], d['config']['engine'], r['kernel'], st['ms_fused'], st['ms_multiply'], st['ms_inverse'], st['ms_epilogue'], st['ms_expand']))"
}
for v in base nohyb; do
  run $v f64p4097 --samples 4097 --dtype float64 --epochs 8
  run $v f64c4097 --samples 4097 --dtype float64 --epochs 8 --output cwt
  run $v f32p10001 --samples 10001 --epochs 8
  run $v f64p5001 --samples 5001 --dtype float64 --epochs 8
done
