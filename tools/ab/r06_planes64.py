# A/B variants of the 64x64 plane-mode step kernel (round 6), timing only unless noted:
#   fullrow  -- a dirty plane word row is stored whole (all 64 lanes, exact results) instead
#               of the dirty lanes' dwords only (partial 128-B lines)
#   storeall -- every kept plane word stored every step (exact; the bytes of a full write)
STORE_OLD = """                if (!pin || d)
                    __builtin_nontemporal_store(PL(PB, k, w), &bp[ps.pos(k + 16 * w) * 64]);"""
VARIANTS = {
    "p64_base": [],
    "p64_fullrow": [("sl_bits.hip", STORE_OLD, """                if (!pin || wave_or(d))
                    __builtin_nontemporal_store(PL(PB, k, w), &bp[ps.pos(k + 16 * w) * 64]);""")],
    "p64_storeall": [("sl_bits.hip", STORE_OLD, """                __builtin_nontemporal_store(PL(PB, k, w), &bp[ps.pos(k + 16 * w) * 64]);"""),
                     ("sl_bits.hip", "    if (!pin || wave_or(dw[0] | dw[1] | d9[0] | d9[1])) {", "    if (true) {")],
}
# round 6, later: the tree's kernel (compile-time keep mask for the C3 planes, one action
# path through the staged planes) built as its own variant for the interleaved A/B
VARIANTS["p64_v4"] = []
