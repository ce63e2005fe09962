"""C5 seeded, generator tuning (round 5, after the board planes): the bit ring's 64
decisions of a wave by one ballot instead of per-draw LDS atomics, and the generating /
jumping waves' issue priority (SAFELIFE_MT_PRIO=3 at run time)."""
_ATOM = """                if (a.bits) {
                    const int k = 312 * (r % kMaxBitRounds) + p;
                    if (u < a.bits_thr)
                        __hip_atomic_fetch_or(&B[k >> 5], 1u << (k & 31), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);
                } else {"""
_BALLOT = """                if (a.bits) {
                    const uint64_t m = __ballot(u < a.bits_thr);
                    if ((t & 63) == 0 && m) {
                        const int k0 = 312 * (r % kMaxBitRounds) + p;
                        const int wi = k0 >> 5, sh = k0 & 31;
                        const uint32_t lo = (uint32_t)m, hi = (uint32_t)(m >> 32);
                        const uint32_t v0 = lo << sh;
                        const uint32_t v1 = sh ? (lo >> (32 - sh)) | (hi << sh) : hi;
                        const uint32_t v2 = sh ? hi >> (32 - sh) : 0u;
                        if (v0) __hip_atomic_fetch_or(&B[wi], v0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        if (v1) __hip_atomic_fetch_or(&B[wi + 1], v1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        if (v2) __hip_atomic_fetch_or(&B[wi + 2], v2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                } else {"""
_PRIO = [("sl_mt.hip", "    int32_t ahead;           // k_mt_gen look-ahead mode: the range after the last fill's\n};",
          "    int32_t ahead;           // k_mt_gen look-ahead mode: the range after the last fill's\n    int32_t prio;\n};"),
         ("sl_mt.hip", "k_mt_gen(MtArgs a) {\n", "k_mt_gen(MtArgs a) {\n    if (a.prio) __builtin_amdgcn_s_setprio(3);\n"),
         ("sl_mt.hip", "k_mt_jump(MtArgs a) {\n", "k_mt_jump(MtArgs a) {\n    if (a.prio) __builtin_amdgcn_s_setprio(3);\n"),
         ("sl_mt.hip", "    a.init_off = 0;\n    // the blocks, then",
          "    a.init_off = 0;\n    a.prio = getenv(\"SAFELIFE_MT_PRIO\") ? atoi(getenv(\"SAFELIFE_MT_PRIO\")) : 0;\n    // the blocks, then"),
         ("sl_mt.hip", "#include <cstring>", "#include <cstdlib>\n#include <cstring>")]
VARIANTS = {
    "g_atom": _PRIO,
    "g_ballot": _PRIO + [("sl_mt.hip", _ATOM, _BALLOT)],
}
