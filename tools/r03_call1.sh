#!/bin/bash
# Round-3 first GPU call: the new GPU tests (multi-rank bench path, torch-free drop-in,
# multi-device reductions), fp64 C4 A/B (twiddle split table / W registers), fp64 C5 rows PMC.
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
R=gpurun_out/c1; mkdir -p $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_ranks.py tests/test_gpu_torchfree.py tests/test_gpu_multi.py tests/test_dist_gpu.py tests/test_gpu_bench_shapes.py -x -v --timeout 500 --timeout-method thread > $R/pytest.log 2>&1; rc=$?; tail -3 $R/pytest.log; [ $rc -ne 0 ] && exit $rc
tools/ab.sh $R/ab64 2 "--config c4 --dtype float64 --epochs 32 --steps 3 --warmup 1" base tws16 tws16wk8 tws16wk4 nostore || exit 1
KREGEX="rows_kernel|cols_kernel" ./tools/prof_counters.sh $R/pmc_c5f64 --config c5 --dtype float64 --steps 1 --warmup 1 --no-cpu-baseline || exit 1
for k in rows_kernel cols_kernel; do python3 tools/pmc_summary.py $R/pmc_c5f64 $R/pmc_c5_f64_$k.json $k '{"chunk": 1, "n": 16777216, "freqs": 512, "out": "cwt", "dtype": "float64", "scales_per_launch": 16}' > /dev/null || exit 1; done
exit 0
