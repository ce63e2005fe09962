set -u
T=r05t
mkdir -p gpurun_out/$T
for rep in 1 2; do
  bash tools/ab_run.sh $T "--config c5" tr1 tr3 || exit 1
done
