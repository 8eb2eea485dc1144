#!/bin/bash
# per-variant PMC snapshot of the fused kernel (diagnostic): clock, VALU/LDS/VMEM counts
#   tools/pmc_probe.sh v1 v2 ...   (BARGS / EPOCHS as tools/ablate.sh)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcp
for v in "$@"; do
  lib=$PWD/ninwavelets_amd/libninwave_$v.so; [ "$v" = base ] && lib=$PWD/ninwavelets_amd/libninwave.so
  export NINWAVE_LIB=$lib
  for grp in "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY"; do
    tag=$(echo $grp | cut -c1-4)
    timeout -k 10 300 rocprofv3 --kernel-include-regex nw_fused --pmc $grp -d gpurun_out/pmcp/$v-$tag -o pmc --output-format csv -- python3 bench.py --epochs ${EPOCHS:-32} --steps 2 --warmup 1 --no-cpu-baseline ${BARGS:-} > gpurun_out/pmcp/$v-$tag.log 2>&1 || exit $?
  done
  python3 - "$v" <<'PY'
import csv, sys, glob, collections
v = sys.argv[1]
vals = collections.defaultdict(list); durs = []
for f in glob.glob(f'gpurun_out/pmcp/{v}-*/**/pmc_counter_collection.csv', recursive=True) + glob.glob(f'gpurun_out/pmcp/{v}-*/pmc_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        if 'nw_fused' in r['Kernel_Name']:
            vals[r['Counter_Name']].append(float(r['Counter_Value'])); durs.append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
m = {k: sum(x) / len(x) for k, x in vals.items()}
d = sum(durs) / len(durs)
clk = m['GRBM_GUI_ACTIVE'] / 8 / d
wc = m['SQ_WAVE_CYCLES']
print(f"{v:8s} {d/1e6:.3f} ms clk {clk:.2f} GHz VALU {m['SQ_INSTS_VALU']/1e6:.0f}M busy {m['SQ_INSTS_VALU']*2/(d*clk*1024):.2f} LDS {m['SQ_INSTS_LDS']/1e6:.1f}M WR {m['SQ_INSTS_VMEM_WR']/1e6:.2f}M RD {m['SQ_INSTS_VMEM_RD']/1e6:.2f}M SALU {m['SQ_INSTS_SALU']/1e6:.0f}M | wait {m['SQ_WAIT_ANY']/wc:.2f} waitinst {m['SQ_WAIT_INST_ANY']/wc:.2f} activeVALU {m['SQ_ACTIVE_INST_VALU']/wc:.2f} activeANY {m['SQ_ACTIVE_INST_ANY']/wc:.2f} waves/CU {wc*4/(d*clk)/256:.1f}")
PY
done
