#!/bin/bash
# chirp-z form: parity (chirp + bench-shape MNE tests), then N = 1201 / 4097 power and cwt A/B
set -u
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/chirpab; mkdir -p $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_chirp.py tests/test_gpu_bench_shapes.py -x -q --timeout 200 --timeout-method thread -k "chirp or mne or c2_morlet or interpolate" > $R/pt.log 2>&1; rc=$?; tail -3 $R/pt.log; [ $rc -ne 0 ] && exit $rc
run() {
  local v=$1 tag=$2; shift 2
  lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
  NINWAVE_LIB=$lib timeout -k 10 200 python bench.py --config c3 --epochs 64 --steps 3 --warmup 1 --no-cpu-baseline "$@" > $R/$v-$tag.json 2> $R/$v-$tag.log || { tail -3 $R/$v-$tag.log; exit 1; }
  python3 -c "import json; d=json.load(open('$R/$v-$tag.json')); r=d['roofline']; print('%-8s %-10s value=%.4e ms/step=%.2f %s %.4f ms' % ('$v', '$tag', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms']))"
}
for rep in 1 2; do for v in base oldchirp inconly; do
  run $v p1201-$rep --samples 1201; run $v c1201-$rep --samples 1201 --output cwt; run $v p4097-$rep --samples 4097
done; done
timeout -k 10 300 python bench.py --config c2 --steps 5 --warmup 2 > $R/bench_c2.json 2> $R/bench_c2.log; rc=$?; cat $R/bench_c2.json; exit $rc
