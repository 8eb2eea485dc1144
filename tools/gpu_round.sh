#!/bin/bash
# one GPU round: parity tests -> bench -> rocprof kernel trace (stops on any crash/timeout)
set -u
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 300 -ra > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; cat gpurun_out/smoke.log | tail -5
if [ $rc -gt 1 ]; then exit $rc; fi
for eng in ${ENGINES:-rocfft}; do
  timeout -k 10 400 python bench.py --steps ${STEPS:-2} --warmup 1 --engine $eng > gpurun_out/bench_$eng.json 2> gpurun_out/bench_$eng.log
  rc=$?; echo "bench $eng rc=$rc"; cat gpurun_out/bench_$eng.json; tail -3 gpurun_out/bench_$eng.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
if [ -n "${PROF:-}" ]; then
  export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --engine $PROF > gpurun_out/prof_bench.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof_bench.log; find gpurun_out/prof -name '*stats*' | head
fi
