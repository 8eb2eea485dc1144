# signal-pair fused kernel (fp32, E = 16): parity, then kernel time vs variants (diagnostic)
set -u
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/pair
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "float32 or fp32 or sampled or engines or epoch or tensors or sharding" > gpurun_out/pair/pt.log 2>&1; rc=$?; tail -3 gpurun_out/pair/pt.log; [ $rc -ne 0 ] && exit $rc
for v in ${VARIANTS:-base p3 nopair}; do
  lib=ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=ninwavelets_amd/libninwave.so
  for n in 1024 2048 4096; do for o in cwt power; do
    ep=$(( 2 * 16384 / n ))
    NINWAVE_LIB=$PWD/$lib timeout -k 10 200 python bench.py --config c3 --samples $n --output $o --epochs $ep --chunk 256 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pair/$v-$n-$o.json 2> gpurun_out/pair/$v-$n-$o.log || { tail -3 gpurun_out/pair/$v-$n-$o.log; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/pair/$v-$n-$o.json')); r=d['roofline']; print('%-7s %6d %-6s ms=%.4f frac=%.3f' % ('$v', $n, '$o', r['avg_launch_ms'], r['frac']))"
  done; done
  NINWAVE_LIB=$PWD/$lib timeout -k 10 200 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pair/$v-c3.json 2> gpurun_out/pair/$v-c3.log || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/pair/$v-c3.json')); r=d['roofline']; print('%-7s C3 value=%.4e ms/step=%.2f kernel=%.4f frac=%.4f' % ('$v', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac']))"
done
