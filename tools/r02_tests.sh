#!/bin/bash
# GPU tests only (full -m gpu suite), log under gpurun_out/r02t/
set -u
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/r02t; mkdir -p $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -ra ${PYARGS:-} > $R/pytest_gpu.log 2>&1; rc=$?; tail -8 $R/pytest_gpu.log; exit $rc
