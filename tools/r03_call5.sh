#!/bin/bash
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
R=gpurun_out/c5; mkdir -p $R
for v in base r3b; do
  lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
  NINWAVE_LIB=$lib DTYPES="float64" NS="1024 2048 4096" timeout -k 10 300 python tools/reduce_rate.py $v > $R/reduce_$v.txt 2>&1; rc=$?; cat $R/reduce_$v.txt; [ $rc -ne 0 ] && exit $rc
done
exit 0
