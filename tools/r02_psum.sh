#!/bin/bash
# fused epoch power partials: reduction tests, then power_mean A/B against power + accumulate
set -u
export PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=$PWD
R=gpurun_out/psum; mkdir -p $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_bench_shapes.py::test_power_mean_fused_partials tests/test_gpu_bench_shapes.py::test_itc_fused_partials tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_dedup.py tests/test_gpu_scales.py > $R/pt.log 2>&1; rc=$?; tail -3 $R/pt.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in base nopsum; do
    lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
    NINWAVE_LIB=$lib timeout -k 10 200 python tools/r02_psum_ab.py $v || exit 1
  done
done
