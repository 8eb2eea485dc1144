#!/bin/bash
# PMC passes of k_expand_rows at C5 Shannon, its summary, the C5 Shannon bench line with
# the traffic, and rocFFT-engine bench lines at MNE-style non-power-of-two lengths.
set -u
R=gpurun_out/shan
mkdir -p $R
KREGEX=k_expand_rows ./tools/prof_counters.sh $R/pmc --config c5 --wavelet shannon --steps 2 --warmup 1 --no-cpu-baseline || exit $?
python3 tools/pmc_summary.py $R/pmc $R/pmc_c5_k_expand_rows.json k_expand_rows '{"chunk": 1, "n": 16777216, "freqs": 512, "out": "cwt", "dtype": "float32"}' || exit $?
cp $R/pmc_c5_k_expand_rows.json profiles/ && timeout -k 10 300 python bench.py --config c5 --wavelet shannon > $R/bench_c5_shannon.json 2> $R/bench_c5_shannon.log || exit $?
cat $R/bench_c5_shannon.json
for n in 1201 4097; do
  timeout -k 10 300 python bench.py --config c3 --samples $n --epochs 64 > $R/bench_c3_n$n.json 2> $R/bench_c3_n$n.log || { tail -5 $R/bench_c3_n$n.log; exit 1; }
  cat $R/bench_c3_n$n.json
done
