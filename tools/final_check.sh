# round-end check, as the driver runs it: GPU tests, smoke, default bench; plus the fp64 C5 line
set -u
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/final/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/final/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.log; rc=$?; cat gpurun_out/final/bench.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config c5 --dtype float64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/final/bench_c5_f64.json 2> gpurun_out/final/bench_c5_f64.log; rc=$?; cat gpurun_out/final/bench_c5_f64.json; exit $rc
