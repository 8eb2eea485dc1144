# C5 two-pass: scales per launch pair (B size) x B store policy (diagnostic)
set -u
mkdir -p gpurun_out/mall
for v in base bnt; do
  lib=ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=ninwavelets_amd/libninwave.so
  for fc in 16 2 1; do
    NW_LARGE_FCHUNK=$fc NINWAVE_LIB=$PWD/$lib timeout -k 10 300 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/mall/${v}_$fc.json 2> gpurun_out/mall/${v}_$fc.log
    rc=$?
    python3 -c "import json; d=json.load(open('gpurun_out/mall/${v}_$fc.json')); s=d['stage_ms_per_step']; print('%-4s fc=%-3s ms/step=%.1f rows=%.1f cols=%.1f' % ('$v', '$fc', d['ms_per_step'], s['ms_rows'], s['ms_fused']))" || { echo "$v $fc rc=$rc"; tail -3 gpurun_out/mall/${v}_$fc.log; }
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
