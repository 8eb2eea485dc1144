#!/bin/bash
# power partials at E = 32 (n = 8192, 16384): 2 waves/SIMD (base), 3 waves/SIMD with spills
# (w3), and the per-signal chunk path (e16)
set -u
export PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=$PWD NS="8192 16384"
R=gpurun_out/psum32; mkdir -p $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_bench_shapes.py tests/test_gpu_parity.py tests/test_gpu_dedup.py tests/test_gpu_scales.py > $R/pt.log 2>&1; rc=$?; tail -2 $R/pt.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in base w3 e16; do
    lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
    NINWAVE_LIB=$lib timeout -k 10 300 python tools/r02_psum_ab.py $v || exit 1
  done
done
