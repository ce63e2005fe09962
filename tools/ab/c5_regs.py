# C5 kernel register-pressure variants (tools/build_variant.py)
F = "sl_bits128.hip"
S_LATE = [(F, """        if (roll < 0) {
            load_pairs<RS>(gs + 32 * t * RS, S);      // in flight under the rule
        } else {""", """        if (roll >= 0) {"""),
          (F, """        if (roll < 0) {
            transpose32(S);
        } else {""", """        if (roll < 0) {
            load_pairs<RS>(gs + 32 * t * RS, S);
            transpose32(S);
        } else {""")]
W3 = [(F, "constexpr int kMinWaves = 2;", "constexpr int kMinWaves = 3;")]
VARIANTS = {
    "c5_base": [],
    "c5_slate": S_LATE,
    "c5_slate_w3": S_LATE + W3,
    "c5_w3": W3,
}
SECTOR = [(F, """        const u32 rb = wave_or(cb[0] | cb[1]) | erow;
        if (rb) {
            transpose32(P);
            store_pairs<RS>(gb + 32 * t * RS, P, rb);
        }""", """        const u32 rb = wave_or(cb[0] | cb[1]) | erow;
        if (rb) {
            u32 lm = cb[0] | cb[1];
            lm |= dpp<0x121>(lm);
            lm |= dpp<0x122>(lm);
            lm |= dpp<0x124>(lm);
            lm |= dpp<0x128>(lm);
            lm |= erow;
            transpose32(P);
#pragma unroll
            for (int y = 0; y < 32; y++)
                if ((rb >> y) & 1u)
                    if ((lm >> y) & 1u) gb[(32 * t + y) * RS] = P[y];
        }"""),
          (F, """            if (rg) {
                transpose32(G);
                store_pairs<RS>(gg + 32 * t * RS, G, rg);
            }""", """            if (rg) {
                u32 lm = cg[0] | cg[1];
                lm |= dpp<0x121>(lm);
                lm |= dpp<0x122>(lm);
                lm |= dpp<0x124>(lm);
                lm |= dpp<0x128>(lm);
                transpose32(G);
#pragma unroll
                for (int y = 0; y < 32; y++)
                    if ((rg >> y) & 1u)
                        if ((lm >> y) & 1u) gg[(32 * t + y) * RS] = G[y];
            }""")]
VARIANTS["c5_sector"] = S_LATE + SECTOR
VARIANTS["c5_sector_w3"] = S_LATE + SECTOR + W3

def sector128(dpps):
    ors = "".join("            lm |= dpp<%s>(lm);\n" % d for d in dpps)
    orsg = "".join("                lm |= dpp<%s>(lm);\n" % d for d in dpps)
    return [(F, """        const u32 rb = wave_or(cb[0] | cb[1]) | erow;
        if (rb) {
            transpose32(P);
            store_pairs<RS>(gb + 32 * t * RS, P, rb);
        }""", """        const u32 rb = wave_or(cb[0] | cb[1]) | erow;
        if (rb) {
            u32 lm = cb[0] | cb[1];
%s            lm |= erow;
            transpose32(P);
#pragma unroll
            for (int y = 0; y < 32; y++)
                if ((rb >> y) & 1u)
                    if ((lm >> y) & 1u) gb[(32 * t + y) * RS] = P[y];
        }""" % ors),
          (F, """            if (rg) {
                transpose32(G);
                store_pairs<RS>(gg + 32 * t * RS, G, rg);
            }""", """            if (rg) {
                u32 lm = cg[0] | cg[1];
%s                transpose32(G);
#pragma unroll
                for (int y = 0; y < 32; y++)
                    if ((rg >> y) & 1u)
                        if ((lm >> y) & 1u) gg[(32 * t + y) * RS] = G[y];
            }""" % orsg)]
VARIANTS["c5_s32"] = S_LATE + sector128(["0xB1", "0x4E", "0x141"])
VARIANTS["c5_s16"] = S_LATE + sector128(["0xB1", "0x4E"])
VARIANTS["c5_s4"] = S_LATE + sector128([])

F64 = "sl_bits.hip"
def sector64(dpps):
    ors = "".join("        lm |= dpp<%s>(lm);\n" % d for d in dpps)
    return [(F64, """    const u32 rb = wave_or(cb[0] | cb[1]) | erow;
    if (rb || OBS) {""", """    const u32 rb = wave_or(cb[0] | cb[1]) | erow;
    u32 lm = cb[0] | cb[1];
%s    lm |= erow;
    if (rb || OBS) {""" % ors),
            (F64, """            if (rb) store_pairs<32>(gb, PB, rb);""", """            if (rb) {
#pragma unroll
                for (int y = 0; y < 32; y++)
                    if ((rb >> y) & 1u)
                        if ((lm >> y) & 1u) gb[y * 32] = PB[y];
            }"""),
            (F64, """            store_pairs<32>(gg, PG, rg);""", """            u32 lg = cg[0] | cg[1];
%s#pragma unroll
            for (int y = 0; y < 32; y++)
                if ((rg >> y) & 1u)
                    if ((lg >> y) & 1u) gg[y * 32] = PG[y];""" % ors.replace("lm", "lg"))]
VARIANTS["c3_base"] = []
VARIANTS["c3_s32"] = sector64(["0x4E", "0x124", "0x128"])
VARIANTS["c3_s16"] = sector64(["0x4E"])
VARIANTS["c3_s4"] = sector64([])
