#!/bin/bash
# r3 candidate (fp64 Morse rows with x^3, 8-B packed fp32 |y|^2 / |y| stores): parity, then A/B
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
R=gpurun_out/c4; mkdir -p $R
NINWAVE_LIB=$PWD/ninwavelets_amd/libninwave_r3.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_bench_shapes.py tests/test_gpu_dedup.py tests/test_gpu_chirp.py tests/test_gpu_scales.py tests/test_gpu_multi.py -x -q --timeout 300 --timeout-method thread > $R/pytest.log 2>&1; rc=$?; tail -3 $R/pytest.log; [ $rc -ne 0 ] && exit $rc
tools/ab.sh $R/c5f64 2 "--config c5 --dtype float64 --steps 2 --warmup 1" base r3 || exit 1
tools/ab.sh $R/c3 2 "--config c3 --steps 3 --warmup 1" base r3 r3nopp || exit 1
tools/ab.sh $R/n1k 2 "--config c3 --samples 1024 --steps 3 --warmup 1" base r3 r3nopp || exit 1
tools/ab.sh $R/n16k 1 "--config c4 --output power --epochs 128 --steps 3 --warmup 1" base r3 r3nopp || exit 1
tools/ab.sh $R/f64red 1 "--config c3 --dtype float64 --epochs 32 --output power --steps 3 --warmup 1" base r3 || exit 1
NINWAVE_LIB=$PWD/ninwavelets_amd/libninwave_r3.so timeout -k 10 300 python tools/reduce_rate.py > $R/reduce.txt 2>&1; rc=$?; cat $R/reduce.txt; [ $rc -ne 0 ] && exit $rc
exit 0
