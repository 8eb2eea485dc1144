set -u
export PYTHONDONTWRITEBYTECODE=1
DTYPES=float64 bash tools/size_sweep.sh > gpurun_out/sweep_f64.txt 2>&1; rc=$?; cat gpurun_out/sweep_f64.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -x -q --timeout 200 --timeout-method thread -k "float64 or fp64 or golden" > gpurun_out/pt_f64.log 2>&1; rc=$?; tail -3 gpurun_out/pt_f64.log; exit $rc
