#!/bin/bash
# Copy a tools/record.sh run (gpurun_out/rec/, merged back from the GPU box) into the
# tracked record under profiles/: bench lines, kernel-trace --stats summaries, PMC summaries
# (tied to the engine-source hash).  Raw counter csvs stay in gpurun_out/.  Host-side only.
set -eu
R=${1:-gpurun_out/rec}
P=profiles
ROUND=${ROUND:-r05}
for c in ${CFGS:-c4 c2 c3 c5 c5f64 c4f64}; do
  [ -s $R/bench_$c.json ] || { echo "no bench line for $c"; continue; }
  cp $R/bench_$c.json $P/${ROUND}_bench_$c.json
  st=$(find $R/prof_$c -name '*kernel_stats.csv' | head -1)
  [ -n "$st" ] && cp "$st" $P/${ROUND}_${c}_kernel_stats.csv
  for j in $R/pmc_${c}_*.json; do
    [ -e "$j" ] || continue
    k=${j#$R/pmc_${c}_}
    case $c in c4f64) dst=$P/pmc_c4_f64_$k ;; c5f64) dst=$P/pmc_c5_f64_$k ;; *) dst=$P/pmc_${c}_$k ;; esac
    cp "$j" "$dst"
  done
  echo "collected $c"
done
