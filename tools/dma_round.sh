set -u
export PYTHONDONTWRITEBYTECODE=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "float32 or sampled or engines or epoch" > gpurun_out/pt_dma.log 2>&1; rc=$?; tail -2 gpurun_out/pt_dma.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for v in base nodp; do BARGS="--config c4 --steps 3" EPOCHS=512 bash tools/ablate.sh $v || exit 1; done; done
for v in base nodp; do BARGS="--config c2 --steps 20" EPOCHS=1 bash tools/ablate.sh $v || exit 1; done
