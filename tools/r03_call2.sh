#!/bin/bash
# fp64 C4 diagnosis: phase stamps with / without stores, and A/B of W-load / twiddle-load ablations
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
R=gpurun_out/c2; mkdir -p $R
tools/ab.sh $R/ab 2 "--config c4 --dtype float64 --epochs 32 --steps 3 --warmup 1" base nowload nowloadtw tws16 || exit 1
for v in stamps stampsns; do
  for dt in float64 float32; do
    NINWAVE_LIB=$PWD/ninwavelets_amd/libninwave_$v.so DTYPE=$dt timeout -k 10 200 python tools/stamps.py > $R/$v-$dt.txt 2>&1 || { tail -5 $R/$v-$dt.txt; exit 1; }
    echo "== $v $dt"; cat $R/$v-$dt.txt
  done
done
exit 0
