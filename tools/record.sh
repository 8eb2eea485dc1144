#!/bin/bash
# Measurement record of the current build: GPU tests, smoke, bench lines, rocprofv3
# kernel-trace --stats and PMC passes (traffic tied to the engine-source hash) for C4, C3,
# C5 (fp32, fp64), C2 and the fp64 C4 shape.  Output under $REC (default gpurun_out/rec/); stops at the first
# failure; tools/collect.sh copies it into profiles/.  CFGS selects configs, SKIP_TESTS=1 the tests.
# (C2, one 0.2 ms launch per step, runs 400 steps after 40 warmups as its default-line leg does:
# shorter runs sit inside the clock ramp, profiles/r06_c2_steps_ab.txt)
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
R=${REC:-gpurun_out/rec}; mkdir -p $R
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $R/pytest_gpu.log 2>&1; rc=$?; tail -2 $R/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $R/smoke.log 2>&1; rc=$?; tail -1 $R/smoke.log; [ $rc -ne 0 ] && exit $rc
fi
# name | bench args (bench line) | pmc args | kernel for the PMC summary | summary config json
record() {
  local name=$1 bargs=$2 pargs=$3 kern=$4 cfgjson=$5
  timeout -k 10 400 python bench.py $bargs > $R/bench_$name.json 2> $R/bench_$name.log; rc=$?
  cat $R/bench_$name.json; [ $rc -ne 0 ] && { tail -3 $R/bench_$name.log; return $rc; }
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/prof_$name -o run --output-format csv -- python3 bench.py $pargs --no-cpu-baseline > $R/prof_$name.log 2>&1; rc=$?
  echo "rocprof $name rc=$rc"; [ $rc -ne 0 ] && { tail -3 $R/prof_$name.log; return $rc; }
  KREGEX="${kern// /|}" ./tools/prof_counters.sh $R/pmc_$name $pargs --no-cpu-baseline || return $?
  for k in $kern; do
    python3 tools/pmc_summary.py $R/pmc_$name $R/pmc_${name}_$k.json $k "$cfgjson" > /dev/null || return $?
    python3 -c "import json; d=json.load(open('$R/pmc_${name}_$k.json')); print('$name $k traffic', d.get('hbm_bytes_per_launch'), 'ms', round(d['profiled_avg_duration_ms'],4), 'clk', round(d.get('effective_clock_ghz',0),3))"
  done
}
CFGS=${CFGS:-c4 c2 c3 c5 c5f64 c4f64}
for c in $CFGS; do
  case $c in
    c4) record c4 "--steps 10 --warmup 3" "--config c4 --steps 2 --warmup 1 --legs none" "nw_fused_kernel" '{"chunk": 512, "n": 16384, "freqs": 256, "out": "cwt", "dtype": "float32"}' || exit $? ;;
    c2) record c2 "--config c2 --steps 400 --warmup 40" "--config c2 --steps 400 --warmup 40" "nw_fused_kernel" '{"chunk": 64, "n": 16384, "freqs": 128, "out": "cwt", "dtype": "float32"}' || exit $? ;;
    c3) record c3 "--config c3 --steps 5 --warmup 2" "--config c3 --steps 2 --warmup 1" "nw_fused_pair_kernel" '{"chunk": 1024, "n": 4096, "freqs": 256, "out": "power", "dtype": "float32"}' || exit $? ;;
    c5) record c5 "--config c5 --steps 3 --warmup 1" "--config c5 --steps 1 --warmup 1" "cols_kernel rows_kernel" '{"chunk": 1, "n": 16777216, "freqs": 512, "out": "cwt", "dtype": "float32", "scales_per_launch": 64}' || exit $? ;;
    c5f64) record c5f64 "--config c5 --dtype float64 --steps 3 --warmup 1" "--config c5 --dtype float64 --steps 1 --warmup 1" "cols_kernel rows_kernel" '{"chunk": 1, "n": 16777216, "freqs": 512, "out": "cwt", "dtype": "float64", "scales_per_launch": 32}' || exit $? ;;
    c4f64) record c4f64 "--config c4 --dtype float64 --steps 3 --warmup 1" "--config c4 --dtype float64 --epochs 16 --steps 2 --warmup 1" "nw_fused_kernel" '{"chunk": 512, "n": 16384, "freqs": 256, "out": "cwt", "dtype": "float64"}' || exit $? ;;
  esac
done
exit 0
