#!/bin/bash
# Interleaved same-box A/B of library variants on one bench command (box-to-box spread is
# +-3..4 %, so only same-box deltas are quoted).  Variants are libninwave_<name>.so built
# with `make -C ninwavelets_amd/csrc VARIANT=<name> DEFS="-D..."`; "base" = libninwave.so.
#   tools/ab.sh <outdir> <reps> "<bench args>" base v1 v2 ...
# Prints one line per run: variant, rep, value, avg launch ms of the dominant kernel, frac.
set -u
export PYTHONDONTWRITEBYTECODE=1
R=$1; REPS=$2; BARGS=$3; shift 3
mkdir -p $R
for rep in $(seq 1 $REPS); do for v in "$@"; do
  lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
  NINWAVE_LIB=$lib timeout -k 10 300 python bench.py $BARGS --no-cpu-baseline --legs none > $R/$v-$rep.json 2> $R/$v-$rep.log || { echo "FAIL $v rep$rep"; tail -5 $R/$v-$rep.log; exit 1; }
  python3 - "$R/$v-$rep.json" "$v" "$rep" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d['roofline']; rr = d.get('roofline_rows') or {}
extra = f" rows {rr['avg_launch_ms']:.4f} ms {rr['frac']:.4f}" if rr else ''
print(f"{sys.argv[2]:<12} rep{sys.argv[3]} value={d['value']:.4e} step={d['ms_per_step']:.2f} ms "
      f"{r['kernel']} {r['avg_launch_ms']:.4f} ms frac={r['frac']:.4f}{extra}", flush=True)
PY
done; done
