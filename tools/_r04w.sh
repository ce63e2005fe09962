set -u
mkdir -p gpurun_out/r04w
for pr in -1 0 -1 0; do
  SAFELIFE_MT_AHEAD_PRIORITY=$pr timeout -k 10 300 python3 bench.py --config c5 --rng seeded --steps 100 --warmup 10 --no-cpu-baseline --pmc off > gpurun_out/r04w/c5g_p$pr.json 2> gpurun_out/r04w/c5g_p$pr.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,2), d['ms_per_step'], d['roofline']['kernel_ms'])" gpurun_out/r04w/c5g_p$pr.json prio$pr
done
