set -u
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/f64r
NINWAVE_LIB=$PWD/ninwavelets_amd/libninwave_n2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py -x -q --timeout 200 --timeout-method thread -k "fp64" > gpurun_out/f64r/pt_n2.log 2>&1; rc=$?; tail -2 gpurun_out/f64r/pt_n2.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="base n2" bash tools/f64_c5_rows.sh
