#!/bin/bash
# ITC partials: rsqrt (base) vs hypot + divisions (libninwave_hyp.so) vs the chunk path (nopsum)
set -u
export PYTHONDONTWRITEBYTECODE=1 PYTHONPATH=$PWD
R=gpurun_out/itc; mkdir -p $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_bench_shapes.py::test_itc_fused_partials tests/test_gpu_parity.py -k "itc or epoch or reduction" > $R/pt.log 2>&1; rc=$?; tail -2 $R/pt.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in base hyp nopsum; do
    lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
    NINWAVE_LIB=$lib timeout -k 10 200 python tools/r02_psum_ab.py $v || exit 1
  done
done
