#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, kernel-trace only, no other tracing)
# usage: tools/prof_counters.sh <outdir> <bench args...>
set -u
out=$1; shift
export TMPDIR=/tmp
mkdir -p $out
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-include-regex "${KREGEX:-nw_fused|k1_multiply|cols_kernel|rows_kernel}" --pmc $grp -d $out/p$i -o pmc --output-format csv -- python3 bench.py "$@" > $out/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/p$i.log; exit $rc; fi
done <<'GROUPS'
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
GROUPS
