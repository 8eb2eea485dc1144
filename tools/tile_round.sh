set -u
export PYTHONDONTWRITEBYTECODE=1
for cfg in c3 c4; do
  for v in base tf16 tf32; do
    BARGS="--config $cfg --steps 3" EPOCHS=512 bash tools/ablate.sh $v 2>&1 | sed "s/^/$cfg /" || exit 1
  done
done
