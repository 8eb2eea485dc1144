#!/bin/bash
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
R=gpurun_out/c6; mkdir -p $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_shapes.py tests/test_gpu_parity.py tests/test_gpu_dedup.py -x -q --timeout 300 --timeout-method thread > $R/pytest.log 2>&1; rc=$?; tail -3 $R/pytest.log; [ $rc -ne 0 ] && exit $rc
DTYPES="float64" NS="1024 2048 4096 8192 16384" timeout -k 10 300 python tools/reduce_rate.py r3 > $R/reduce64.txt 2>&1; rc=$?; cat $R/reduce64.txt; [ $rc -ne 0 ] && exit $rc
DTYPES="float32" NS="4096 8192 16384" timeout -k 10 300 python tools/reduce_rate.py r3 > $R/reduce32.txt 2>&1; rc=$?; cat $R/reduce32.txt; [ $rc -ne 0 ] && exit $rc
exit 0
