set -u
T=r05s
mkdir -p gpurun_out/$T
for rep in 1 2; do
  bash tools/ab_run.sh $T "--config c5" ph10 ph7 ph1 || exit 1
done
