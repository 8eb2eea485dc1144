set -u
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/f64r
for v in ${VARIANTS:-base r16}; do
  lib=ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=ninwavelets_amd/libninwave.so
  NINWAVE_LIB=$PWD/$lib timeout -k 10 300 python bench.py --config c5 --dtype float64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/f64r/$v.json 2> gpurun_out/f64r/$v.log || { tail -3 gpurun_out/f64r/$v.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/f64r/$v.json')); s=d['stage_ms_per_step']; print('$v', round(d['ms_per_step'],1), s['ms_rows'], s['ms_fused'])"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py -x -q --timeout 200 --timeout-method thread -k "fp64" > gpurun_out/f64r/pt.log 2>&1; rc=$?; tail -2 gpurun_out/f64r/pt.log; exit $rc
