# signals per fused launch (bench --chunk) at C4 / C3 (diagnostic)
set -u
mkdir -p gpurun_out/chunk
for cfg in c4 c3; do
  for ch in 256 512 1024; do
    timeout -k 10 300 python bench.py --config $cfg --chunk $ch --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/chunk/${cfg}_$ch.json 2> gpurun_out/chunk/${cfg}_$ch.log
    rc=$?
    python3 -c "import json; d=json.load(open('gpurun_out/chunk/${cfg}_$ch.json')); r=d['roofline']; print('%s chunk=%-5s value=%.4e ms/step=%.2f kernel_ms=%.4f frac=%.4f' % ('$cfg', '$ch', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac']))" || { echo "$cfg $ch rc=$rc"; tail -3 gpurun_out/chunk/${cfg}_$ch.log; }
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
