# fp64 engine round: parity of the fp64 fused paths, then C5 / C4-shape fp64 benches
# (fused engine, and the rocFFT engine for comparison)
set -u
mkdir -p gpurun_out/f64
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_large.py -x -v --timeout 200 --timeout-method thread -k "fp64" > gpurun_out/f64/pytest_large.log 2>&1
rc=$?; tail -4 gpurun_out/f64/pytest_large.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 250 --timeout-method thread -k "c5_scale" > gpurun_out/f64/pytest_c5.log 2>&1
rc=$?; tail -4 gpurun_out/f64/pytest_c5.log; [ $rc -ne 0 ] && exit $rc
for eng in auto rocfft; do
timeout -k 10 400 python bench.py --config c5 --dtype float64 --engine $eng --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/f64/bench_c5_f64_$eng.json 2> gpurun_out/f64/bench_c5_f64_$eng.log
rc=$?; cat gpurun_out/f64/bench_c5_f64_$eng.json; [ $rc -ne 0 ] && { tail -5 gpurun_out/f64/bench_c5_f64_$eng.log; exit $rc; }
timeout -k 10 300 python bench.py --config c4 --dtype float64 --engine $eng --epochs 16 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/f64/bench_c4_f64_$eng.json 2> gpurun_out/f64/bench_c4_f64_$eng.log
rc=$?; cat gpurun_out/f64/bench_c4_f64_$eng.json; [ $rc -ne 0 ] && { tail -5 gpurun_out/f64/bench_c4_f64_$eng.log; exit $rc; }
done
exit 0
