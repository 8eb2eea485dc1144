#!/bin/bash
# power partials on the signal-pair kernel (base) vs the single-signal kernel (libninwave_single.so)
set -u
export PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=$PWD NS="1024 2048 4096"
R=gpurun_out/pairpsum; mkdir -p $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_bench_shapes.py tests/test_gpu_parity.py tests/test_gpu_dedup.py tests/test_gpu_scales.py tests/test_gpu_multi.py > $R/pt.log 2>&1; rc=$?; tail -2 $R/pt.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in base single; do
    lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
    NINWAVE_LIB=$lib timeout -k 10 300 python tools/r02_psum_ab.py $v || exit 1
  done
done
