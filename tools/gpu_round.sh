#!/bin/bash
# One GPU round on the box: parity tests -> smoke -> bench lines -> rocprofv3 kernel
# trace + PMC passes of the default bench; summaries land in gpurun_out/round/.
# Stops at the first crash/timeout (exit codes > 1).
set -u
mkdir -p gpurun_out/round
export PYTHONDONTWRITEBYTECODE=1
R=gpurun_out/round
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 300 -ra > $R/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 $R/pytest_gpu.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 $R/smoke.log
  if [ $rc -gt 1 ]; then exit $rc; fi
fi
for cfg in ${CONFIGS:-c4}; do
  for eng in ${ENGINES:-auto}; do
    timeout -k 10 400 python bench.py --config $cfg --engine $eng ${BENCH_ARGS:-} > $R/bench_${cfg}_$eng.json 2> $R/bench_${cfg}_$eng.log
    rc=$?; echo "bench $cfg $eng rc=$rc"; cat $R/bench_${cfg}_$eng.json
    if [ $rc -ne 0 ]; then tail -5 $R/bench_${cfg}_$eng.log; exit $rc; fi
  done
done
if [ -n "${PROF:-}" ]; then
  export TMPDIR=/tmp
  for cfg in ${PROF_CONFIGS:-c4}; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/prof_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > $R/prof_$cfg.log 2>&1
    rc=$?; echo "rocprof $cfg rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $R/prof_$cfg.log; exit $rc; fi
    ./tools/prof_counters.sh $R/pmc_$cfg --config $cfg --steps 2 --warmup 1 --no-cpu-baseline || exit $?
  done
fi
