# Refresh the round's measurement record for configs $CONFIGS (default c4 c3): bench line
# (with the CPU baselines), rocprofv3 kernel-trace --stats, PMC passes -> gpurun_out/refresh/
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
R=gpurun_out/refresh
mkdir -p $R
for cfg in ${CONFIGS:-c4 c3}; do
  timeout -k 10 400 python bench.py --config $cfg ${BARGS:-} > $R/bench_$cfg.json 2> $R/bench_$cfg.log
  rc=$?; echo "bench $cfg rc=$rc"; cat $R/bench_$cfg.json; [ $rc -ne 0 ] && { tail -5 $R/bench_$cfg.log; exit $rc; }
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/prof_$cfg -o run --output-format csv -- python3 bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline ${BARGS:-} > $R/prof_$cfg.log 2>&1
  rc=$?; echo "rocprof $cfg rc=$rc"; [ $rc -ne 0 ] && { tail -5 $R/prof_$cfg.log; exit $rc; }
  if [ -z "${NO_PMC:-}" ]; then
    ./tools/prof_counters.sh $R/pmc_$cfg --config $cfg --steps 2 --warmup 1 --no-cpu-baseline ${BARGS:-} || exit $?
  fi
done
exit 0
