# C3 in-launch resets with per-env flags (round 5): what the publish costs.
#   tf_norel  no agent-scope release before a finished env's flag (timing only: the
#             reset's stores may then land before the step's)
#   tf_nowait no release and no wait for the step's stores (timing only)
F = "sl_bits.hip"
NOREL = [(F, """        wait_vm();                  // every lane's stores of this step have completed
        if (lane == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            wait_vm();
            __hip_atomic_store(&fl[b], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }""", """        wait_vm();                  // every lane's stores of this step have completed
        if (lane == 0) {
            __hip_atomic_store(&fl[b], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }""")]
NOWAIT = [(F, """        wait_vm();                  // every lane's stores of this step have completed
        if (lane == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            wait_vm();
            __hip_atomic_store(&fl[b], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }""", """        if (lane == 0) {
            __hip_atomic_store(&fl[b], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }""")]
VARIANTS = {"tf_norel": NOREL, "tf_nowait": NOWAIT}
# more workers: fewer envs per worker, so a worker's resets (one wave, one after
# another) do not set the launch's end
for _n in (256, 512, 1024):
    VARIANTS["tw%d" % _n] = [(F, "constexpr int kTailWorkers = 64;",
                              "constexpr int kTailWorkers = %d;" % _n)]
VARIANTS["tw512_norel"] = VARIANTS["tw512"] + NOREL
