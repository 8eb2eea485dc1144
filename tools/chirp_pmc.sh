#!/bin/bash
# PMC passes of nw_chirp_kernel at the C3 shape with n = 1201, its summary, then the bench
# line that reads it back (traffic field)
set -u
R=gpurun_out/chirp_pmc
mkdir -p $R
KREGEX=nw_chirp_kernel ./tools/prof_counters.sh $R/pmc --config c3 --samples 1201 --epochs 64 --steps 2 --warmup 1 --no-cpu-baseline || exit $?
python3 tools/pmc_summary.py $R/pmc $R/pmc_c3_nw_chirp_kernel.json nw_chirp_kernel '{"chunk": 1024, "n": 1201, "freqs": 256, "out": "power", "dtype": "float32"}' || exit $?
cp $R/pmc_c3_nw_chirp_kernel.json profiles/ && timeout -k 10 300 python bench.py --config c3 --samples 1201 --epochs 64 > $R/bench.json 2> $R/bench.log || exit $?
cat $R/bench.json
