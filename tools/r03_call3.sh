#!/bin/bash
# ablations: C5 fp64/fp32 W evaluation cost (rowsnow), C3 pair kernel (nostore/noexch/notw), fp64 C4 power vs cwt
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
R=gpurun_out/c3; mkdir -p $R
tools/ab.sh $R/c5f64 1 "--config c5 --dtype float64 --steps 2 --warmup 1" base rowsnow || exit 1
tools/ab.sh $R/c5 1 "--config c5 --steps 3 --warmup 1" base rowsnow || exit 1
tools/ab.sh $R/c3 2 "--config c3 --epochs 128 --steps 3 --warmup 1" base nostore noexch notw || exit 1
tools/ab.sh $R/c4 1 "--config c4 --epochs 128 --steps 3 --warmup 1" base nostore noexch notw || exit 1
tools/ab.sh $R/f64pow 1 "--config c4 --dtype float64 --output power --epochs 32 --steps 3 --warmup 1" base nostore || exit 1
exit 0
