set -e
mkdir -p gpurun_out/g2
timeout -k 10 300 python -u scratch/dbg_store2.py
timeout -k 10 900 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests -m gpu > gpurun_out/g2/pytest.log 2>&1 || { tail -40 gpurun_out/g2/pytest.log; exit 1; }
tail -2 gpurun_out/g2/pytest.log
tools/ab.sh gpurun_out/g2/f64 2 "--config c4 --dtype float64 --epochs 32 --steps 3 --warmup 1" old base
tools/ab.sh gpurun_out/g2/f32 2 "--config c4 --epochs 128 --steps 5 --warmup 2" old base
tools/ab.sh gpurun_out/g2/c3 2 "--config c3 --epochs 128 --steps 5 --warmup 2" old base
tools/ab.sh gpurun_out/g2/c5f64 1 "--config c5 --dtype float64 --steps 2 --warmup 1" old base rowsnt
