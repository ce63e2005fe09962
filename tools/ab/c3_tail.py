# (timing record; applies to commit 898e89f, whose tail workers the next commit removed)
# C3 tail resets: what the in-launch reset protocol costs (timing-only variants).
#   tl_head   as committed: every step wave adds to a sharded done counter (agent scope)
#   tl_nodone no done counters: workers give up after a short spin budget (timing only:
#             entries published later stay unreset)
#   tl_norel  tl_nodone without the producer's agent-scope release
#   tl_off    tail workers off (the reset-list kernel, as in round 3)
F = "sl_bits.hip"
NODONE = [
    (F, """    if (lane == 0)
        __hip_atomic_fetch_add(&tw.done[b % kDoneShards], (int64_t)1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);""", ""),
    (F, "constexpr int kTailSpins = 1 << 18;", "constexpr int kTailSpins = 64;"),
]
NOREL = NODONE + [(F, """            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            wait_vm();
            const int64_t slot""", """            const int64_t slot""")]
OFF = [(F, """    ka.fx.tail_workers = (fx.fuse_reset && fx.pool.K > 0 && !fx.capture && st.B < (1ll << 31))
                             ? kTailWorkers : 0;""", """    ka.fx.tail_workers = 0;""")]
VARIANTS = {"tl_head": [], "tl_nodone": NODONE, "tl_norel": NOREL, "tl_off": OFF}
