#!/bin/bash
# Repeated-row execution on the box: its parity tests, the full GPU suite, the C5 Shannon
# bench lines (fp32, fp64) and a rocprofv3 kernel-trace summary of the fp32 one.
set -u
R=gpurun_out/dedup
mkdir -p $R
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_dedup.py -x -q --timeout 120 --timeout-method thread > $R/pytest_dedup.log 2>&1
rc=$?; echo "dedup tests rc=$rc"; tail -5 $R/pytest_dedup.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -3 $R/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for dt in float32 float64; do
  timeout -k 10 400 python bench.py --config c5 --wavelet shannon --dtype $dt > $R/bench_c5_shannon_$dt.json 2> $R/bench_c5_shannon_$dt.log
  rc=$?; echo "bench c5 shannon $dt rc=$rc"; cat $R/bench_c5_shannon_$dt.json; [ $rc -ne 0 ] && { tail -5 $R/bench_c5_shannon_$dt.log; exit $rc; }
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/prof_c5_shannon -o run --output-format csv -- python3 bench.py --config c5 --wavelet shannon --steps 2 --warmup 1 --no-cpu-baseline > $R/prof_c5_shannon.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
