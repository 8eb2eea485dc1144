set -u
export PYTHONDONTWRITEBYTECODE=1
DTYPES=float64 bash tools/size_sweep.sh e32 > gpurun_out/sweep_f64_e32.txt 2>&1; rc=$?; cat gpurun_out/sweep_f64_e32.txt; [ $rc -ne 0 ] && exit $rc
NINWAVE_LIB=$PWD/ninwavelets_amd/libninwave_e32.so timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "fp64_16384 or sampled" > gpurun_out/pt_e32.log 2>&1; rc=$?; tail -3 gpurun_out/pt_e32.log; exit $rc
