set -u
T=r05aj
mkdir -p gpurun_out/$T
SAFELIFE_HIP_LIB=$PWD/variants/g_ballot.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_mt.py -x -q --timeout 300 --timeout-method thread -k "fill" > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
run() { # tag lib env...
  local tag=$1 lib=$2; shift 2
  env "$@" SAFELIFE_HIP_LIB=$PWD/variants/$lib.so timeout -k 10 300 python3 bench.py --config c5 --rng seeded --no-cpu-baseline --pmc off > gpurun_out/$T/$tag.json 2> gpurun_out/$T/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/$T/$tag.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,2), 'M/s', d['ms_per_step'], d['roofline'].get('kernel_ms'))" gpurun_out/$T/$tag.json $tag
}
for rep in 1 2; do
  run atom g_atom || exit 1
  run atom_p3 g_atom SAFELIFE_MT_PRIO=3 || exit 1
  run ballot g_ballot || exit 1
  run ballot_p3 g_ballot SAFELIFE_MT_PRIO=3 || exit 1
done
run atom_r420 g_atom SAFELIFE_MT_ROUNDS=420 || exit 1
run atom_r560 g_atom SAFELIFE_MT_ROUNDS=560 || exit 1
run atom_r1260 g_atom SAFELIFE_MT_ROUNDS=1260 || exit 1
