#!/bin/bash
# round-2 check on the box: GPU tests, smoke, default bench (+ --gpus 1 launcher path)
set -u
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/r02a; mkdir -p $R
nproc > $R/nproc.txt; python -c "import os; print(os.cpu_count(), len(os.sched_getaffinity(0)))" >> $R/nproc.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -ra > $R/pytest_gpu.log 2>&1; rc=$?; tail -5 $R/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.log 2>&1; rc=$?; tail -1 $R/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps 10 --warmup 3 > $R/bench.json 2> $R/bench.log; rc=$?; cat $R/bench.json; [ $rc -ne 0 ] && exit $rc
exit 0
