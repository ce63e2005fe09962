# C3 packed views: two cells per lane per store (global_store_dword, 4-B aligned in the
# whole obs array; an env starting mid-dword stores its first cell alone, and an odd
# remainder its last) -- 9 store instructions per lane instead of 17, the LDS gathers
# unchanged.  (16-B chunks measured slower in round 3, tools/ab/c3p_chunks.py.)
F = "sl_bits.hip"
OLD = """    uint16_t *o = lfx.obs_out + b * (int64_t)nv;
    const int dr = 64 / vw, dc = 64 - dr * vw;
    int r = lane / vw, c = lane - r * vw;
    if (small) {
        for (int i = lane; i < nv; i += 64) {
            o[i] = cells[lds_cell_idx((ty + r) & (N - 1), (tx + c) & (N - 1))];
            r += dr;
            c += dc;
            if (c >= vw) {
                c -= vw;
                r++;
            }
        }
    } else {"""
NEW = """    uint16_t *o = lfx.obs_out + b * (int64_t)nv;
    const int dr = 64 / vw, dc = 64 - dr * vw;
    int r = lane / vw, c = lane - r * vw;
    if (small) {
        const int s0 = (int)((b * (int64_t)nv) & 1);     // env starts mid-dword
        const int np = (nv - s0) >> 1;
        if (s0 && lane == 0) o[0] = cells[lds_cell_idx(ty & (N - 1), tx & (N - 1))];
        if (((nv - s0) & 1) && lane == 1)
            o[nv - 1] = cells[lds_cell_idx((ty + vh - 1) & (N - 1), (tx + vw - 1) & (N - 1))];
        uint32_t *o32 = reinterpret_cast<uint32_t *>(o + s0);
        const int c0 = s0 + 2 * lane;
        int rr = c0 / vw, cc = c0 - rr * vw;
        const int d2r = 128 / vw, d2c = 128 - d2r * vw;
        for (int p = lane; p < np; p += 64) {
            const int r1 = cc + 1 == vw ? rr + 1 : rr, c1 = cc + 1 == vw ? 0 : cc + 1;
            const uint32_t v0 = cells[lds_cell_idx((ty + rr) & (N - 1), (tx + cc) & (N - 1))];
            const uint32_t v1 = cells[lds_cell_idx((ty + r1) & (N - 1), (tx + c1) & (N - 1))];
            o32[p] = v0 | (v1 << 16);
            rr += d2r;
            cc += d2c;
            if (cc >= vw) {
                cc -= vw;
                rr++;
            }
        }
        (void)r;
        (void)c;
    } else {"""
VARIANTS = {"dw_base": [], "dw_pairs": [(F, OLD, NEW)]}
