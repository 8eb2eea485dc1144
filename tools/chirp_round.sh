#!/bin/bash
# chirp-z form on the box: the GPU suite, then bench lines at MNE-style lengths (C3 shape,
# 64 epochs x 64 ch x 256 freqs power) and a rocprofv3 kernel-trace summary of the 1201 one
set -u
R=gpurun_out/chirp
mkdir -p $R
export PYTHONDONTWRITEBYTECODE=1
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/pt_all.log 2>&1
rc=$?; tail -3 $R/pt_all.log; [ $rc -ne 0 ] && exit $rc
fi
for n in ${LENGTHS:-1201 4097}; do
  timeout -k 10 300 python bench.py --config c3 --samples $n --epochs 64 ${BARGS:-} > $R/bench_c3_n$n.json 2> $R/bench_c3_n$n.log || { tail -5 $R/bench_c3_n$n.log; exit 1; }
  python3 -c "import json; d=json.load(open('$R/bench_c3_n$n.json')); r=d['roofline']; print('n=$n', d['config']['engine'], 'value=%.3e ms/step=%.2f kernel=%s ms=%.3f frac=%.3f' % (d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac']), d['stage_ms_per_step'])"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/prof_1201 -o run --output-format csv -- python3 bench.py --config c3 --samples 1201 --epochs 64 --steps 2 --warmup 1 --no-cpu-baseline > $R/prof_1201.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
