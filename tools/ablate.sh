#!/bin/bash
# time the fused kernel of each library variant (diagnostic): tools/ablate.sh v1 v2 ...
set -u
mkdir -p gpurun_out/ablate
for v in "$@"; do
  lib=ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=ninwavelets_amd/libninwave.so
  NINWAVE_LIB=$PWD/$lib timeout -k 10 200 python bench.py --epochs ${EPOCHS:-32} --steps 3 --warmup 1 --no-cpu-baseline ${BARGS:-} > gpurun_out/ablate/$v.json 2> gpurun_out/ablate/$v.log
  rc=$?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ablate/$v.json')); r=d['roofline']; print('%-12s value=%.3e  kernel_ms=%.3f  GB/s=%.0f frac=%.3f' % ('$v', d['value'], r['avg_launch_ms'], r['achieved'], r['frac']))" || { echo "$v rc=$rc"; tail -3 gpurun_out/ablate/$v.log; }
  if [ $rc -ne 0 ]; then exit $rc; fi
done
