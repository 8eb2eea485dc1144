set -u
mkdir -p gpurun_out/c5
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k c5 -v --timeout 200 --timeout-method thread > gpurun_out/c5/pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|assert" gpurun_out/c5/pytest.log | head; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/c5/bench.json 2> gpurun_out/c5/bench.log
rc=$?; cat gpurun_out/c5/bench.json; [ $rc -ne 0 ] && { tail -5 gpurun_out/c5/bench.log; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5/prof -o run --output-format csv -- python3 bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; find gpurun_out/c5/prof -name "*stats*" | head
exit $rc
