"""C5 seeded: the bit ring's decisions ORed in per draw (LDS atomics, as before round 5's
ballot) against the shipped ballot form.  Priority: SAFELIFE_MT_PRIO=3 at run time."""

_SRC = open("safelife-k2_amd/csrc/sl_mt.hip").read()   # (run from the repo root)
_i = _SRC.index("                    // the wave's 64 consecutive decisions by one ballot")
_j = _SRC.index("                } else {", _i)
VARIANTS = {
    "atom": [("sl_mt.hip", _SRC[_i:_j],
              "                    const int k = 312 * (r % kMaxBitRounds) + p;\n"
              "                    if (u < a.bits_thr)\n"
              "                        __hip_atomic_fetch_or(&B[k >> 5], 1u << (k & 31), __ATOMIC_RELAXED,\n"
              "                                              __HIP_MEMORY_SCOPE_WORKGROUP);\n")],
    "cur": [],
}
