#!/bin/bash
# A/B of LDS layouts (variants built with make VARIANT=...): parity subset on the default
# library, then kernel time for C4 / C3 per variant (interleaved twice), then one PMC pass
# (LDS conflict counters) per variant and config.
set -u
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
R=gpurun_out/ldsab; mkdir -p $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_shapes.py tests/test_gpu_large.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "${PTK:-not c5_all}" > $R/pt.log 2>&1; rc=$?; tail -3 $R/pt.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
for v in ${VARIANTS:-base old}; do
  lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
  for cfg in ${CFGS:-c4 c3}; do
    NINWAVE_LIB=$lib timeout -k 10 200 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline ${BARGS:-} > $R/$v-$cfg-$rep.json 2> $R/$v-$cfg-$rep.log || { tail -3 $R/$v-$cfg-$rep.log; exit 1; }
    python3 -c "import json; d=json.load(open('$R/$v-$cfg-$rep.json')); r=d['roofline']; print('%-6s %s rep$rep value=%.4e ms/step=%.2f kernel=%s %.4f ms frac=%.4f' % ('$v', '$cfg', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac']))"
  done
done
done
[ -n "${NOPMC:-}" ] && exit 0
for v in ${VARIANTS:-base old}; do
  lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
  for cfg in ${CFGS:-c4 c3}; do
    NINWAVE_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-include-regex "nw_fused" --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES -d $R/pmc_${v}_$cfg -o pmc --output-format csv -- python3 bench.py --config $cfg --steps 1 --warmup 1 --no-cpu-baseline --epochs 64 > $R/pmc_$v-$cfg.log 2>&1 || { tail -3 $R/pmc_$v-$cfg.log; exit 1; }
    python3 - "$R/pmc_${v}_$cfg" "$v" "$cfg" <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for row in csv.DictReader(open(f)):
        d[row['Counter_Name']].append(float(row['Counter_Value']))
m = {k: sum(v) / len(v) for k, v in d.items()}
print(sys.argv[2], sys.argv[3], 'conflict/lds_active=%.3f wait_lds/wave_cycles=%.3f valu/wave=%.3f' % (
    m.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, m.get('SQ_ACTIVE_INST_LDS', 1)),
    m.get('SQ_WAIT_INST_LDS', 0) / max(1, m.get('SQ_WAVE_CYCLES', 1)),
    m.get('SQ_ACTIVE_INST_VALU', 0) / max(1, m.get('SQ_WAVE_CYCLES', 1))), {k: round(v) for k, v in m.items()})
PY
    rm -rf $R/pmc_${v}_$cfg
  done
done
