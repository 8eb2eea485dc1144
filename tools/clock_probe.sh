#!/bin/bash
# effective shader clock of the fused kernel per library variant (diagnostic):
#   tools/clock_probe.sh v1 v2 ...   (GRBM_GUI_ACTIVE / 8 XCDs / kernel duration)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/clock
for v in "$@"; do
  lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
  export NINWAVE_LIB=$lib
  timeout -k 10 300 rocprofv3 --kernel-include-regex nw_fused --pmc GRBM_GUI_ACTIVE -d gpurun_out/clock/$v -o pmc --output-format csv -- python3 bench.py --epochs ${EPOCHS:-32} --steps 2 --warmup 1 --no-cpu-baseline ${BARGS:-} > gpurun_out/clock/$v.log 2>&1 || exit $?
  python3 - "$v" <<'PY'
import csv, sys, glob
v = sys.argv[1]
f = glob.glob(f'gpurun_out/clock/{v}/**/pmc_counter_collection.csv', recursive=True) + glob.glob(f'gpurun_out/clock/{v}/pmc_counter_collection.csv')
rows = [r for r in csv.DictReader(open(f[0])) if 'nw_fused' in r['Kernel_Name']]
g = sum(float(r['Counter_Value']) for r in rows) / len(rows)
d = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in rows) / len(rows)
print(f'{v:10s} kernel {d/1e6:.3f} ms  clock {g/8/d:.3f} GHz')
PY
done
