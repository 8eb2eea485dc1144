#!/bin/bash
# Interleaved same-box A/B of environment settings on one bench command (tools/ab.sh's output
# format): tools/abenv.sh <outdir> <reps> "<bench args>" "NAME=VAL ..." "NAME=VAL ..." ...
# e.g. tools/abenv.sh out 2 "--config c5" "NW_LARGE_PIPE=0" "NW_LARGE_PIPE=1"
set -u
export PYTHONDONTWRITEBYTECODE=1
R=$1; REPS=$2; BARGS=$3; shift 3
mkdir -p $R
for rep in $(seq 1 $REPS); do i=0; for v in "$@"; do i=$((i+1))
  env $v timeout -k 10 300 python bench.py $BARGS --no-cpu-baseline --legs none > $R/v$i-$rep.json 2> $R/v$i-$rep.log || { echo "FAIL $v rep$rep"; tail -5 $R/v$i-$rep.log; exit 1; }
  python3 - "$R/v$i-$rep.json" "$v" "$rep" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d['roofline']; rr = d.get('roofline_rows') or {}
extra = f" rows {rr['avg_launch_ms']:.4f} ms {rr['frac']:.4f}" if rr else ''
print(f"{sys.argv[2]:<22} rep{sys.argv[3]} value={d['value']:.4e} step={d['ms_per_step']:.2f} ms "
      f"{r['kernel']} {r['avg_launch_ms']:.4f} ms frac={r['frac']:.4f}{extra}", flush=True)
PY
done; done
