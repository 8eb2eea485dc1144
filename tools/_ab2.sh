set -e
tools/ab.sh gpurun_out/ab2/f64 2 "--config c4 --dtype float64 --epochs 32 --steps 3 --warmup 1" base sc1 bnt one_nt
tools/ab.sh gpurun_out/ab2/f32 2 "--config c4 --epochs 128 --steps 5 --warmup 2" base sc1 bnt
tools/ab.sh gpurun_out/ab2/c3 2 "--config c3 --epochs 128 --steps 5 --warmup 2" base sc1 bnt
