# C3: per-half row stores.  A store instruction of the 64x64 kernel covers rows y and
# 32 + y (even lanes hold rows 0-31, odd lanes rows 32-63); today a changed row y
# writes both.  Here each half's changed rows are their own wave-wide OR and the lanes
# of an unchanged half are masked off the store: 128 instead of 256 bytes for a row
# whose partner did not change.
F = "sl_bits.hip"
R = [
    (F, """__device__ __forceinline__ u32 mux_edits(u32 P[32], int ne, const int eidx[4], const u32 eval[4],
                                         int lane) {
    u32 erow = 0;""", """__device__ __forceinline__ u32 mux_edits(u32 P[32], int ne, const int eidx[4], const u32 eval[4],
                                         int lane, u32 &erow1) {
    u32 erow = 0;
    erow1 = 0;"""),
    (F, """            erow |= bit;""", """            if (y >> 5) erow1 |= bit;
            else erow |= bit;"""),
    (F, """    const u32 erow = mux_edits(PB, ne, eidx, eval, lane);""",
        """    u32 erow1;
    const u32 erow = mux_edits(PB, ne, eidx, eval, lane, erow1);"""),
    (F, """    const u32 rb = wave_or(cb[0] | cb[1]) | erow;""",
        """    const u32 cbl = cb[0] | cb[1];
    const u32 rb0 = wave_or((lane & 1) ? 0u : cbl) | erow;      // rows 0-31 (even lanes)
    const u32 rb1 = wave_or((lane & 1) ? cbl : 0u) | erow1;     // rows 32-63 (odd lanes)
    const u32 rb = rb0 | rb1;"""),
    (F, """                for (int y = 0; y < 32; y++)
                    if ((rb >> y) & 1u) gb[y * 32] = PB[y] & 0x8FFF8FFFu;""",
        """                for (int y = 0; y < 32; y++)
                    if ((rb >> y) & 1u)
                        if (((((lane & 1) ? rb1 : rb0)) >> y) & 1u) gb[y * 32] = PB[y] & 0x8FFF8FFFu;"""),
    (F, """            for (int y = 0; y < 32; y++)
                if ((rb >> y) & 1u) __builtin_nontemporal_store(PB[y], &gb[y * 32]);""",
        """            for (int y = 0; y < 32; y++)
                if ((rb >> y) & 1u)
                    if (((((lane & 1) ? rb1 : rb0)) >> y) & 1u)
                        __builtin_nontemporal_store(PB[y], &gb[y * 32]);"""),
]
VARIANTS = {"h_base": [], "h_half": R}
