# end-of-round measurement record: C3 with PMC, C2 / C5 bench + kernel trace, fp64 lines
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
CONFIGS=c3 bash tools/refresh_profiles.sh || exit $?
CONFIGS="c2 c5" NO_PMC=1 bash tools/refresh_profiles.sh || exit $?
R=gpurun_out/refresh
timeout -k 10 300 python bench.py --config c5 --dtype float64 --steps 2 --warmup 1 --no-cpu-baseline > $R/bench_c5_f64.json 2> $R/bench_c5_f64.log || exit $?
timeout -k 10 300 python bench.py --config c4 --dtype float64 --epochs 16 --steps 2 --warmup 1 --no-cpu-baseline > $R/bench_n16384_f64.json 2> $R/bench_n16384_f64.log || exit $?
echo done
