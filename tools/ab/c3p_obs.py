# C3 with fused packed views: the view gather of write_obs (sl_bits.hip) four cells
# in flight per lane instead of one (LDS reads issued together, then the stores)
F = "sl_bits.hip"
OLD = """    if (small) {
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
NEW = """    if (small) {
        const auto next = [&](int &rr, int &cc) {
            rr += dr;
            cc += dc;
            if (cc >= vw) {
                cc -= vw;
                rr++;
            }
        };
        int i = lane;
        for (; i + 192 < nv; i += 256) {
            int k[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                k[u] = lds_cell_idx((ty + r) & (N - 1), (tx + c) & (N - 1));
                next(r, c);
            }
            uint16_t v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) v[u] = cells[k[u]];
#pragma unroll
            for (int u = 0; u < 4; u++) o[i + 64 * u] = v[u];
        }
        for (; i < nv; i += 64) {
            o[i] = cells[lds_cell_idx((ty + r) & (N - 1), (tx + c) & (N - 1))];
            next(r, c);
        }
    } else {"""
VARIANTS = {"gather4": [(F, OLD, NEW)]}
# the views written as dword pairs (half the store instructions; the env's first /
# last cell alone when its view starts / ends off a 4-byte boundary)
NEW_PAIRS = """    if (small) {
        const int off = (int)((b * nv) & 1);
        if (off && lane == 0) o[0] = cells[lds_cell_idx(ty & (N - 1), tx & (N - 1))];
        const int npair = (nv - off) >> 1;
        const int d2r = 128 / vw, d2c = 128 - d2r * vw;
        int i2 = off + 2 * lane;
        int rr = i2 / vw, cc = i2 - rr * vw;
        uint32_t *o32 = reinterpret_cast<uint32_t *>(o + off);
        for (int p = lane; p < npair; p += 64) {
            int r1 = rr, c1 = cc + 1;
            if (c1 >= vw) {
                c1 = 0;
                r1++;
            }
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
        if (((nv - off) & 1) && lane == 0) {
            const int rl = (nv - 1) / vw, cl = nv - 1 - rl * vw;
            o[nv - 1] = cells[lds_cell_idx((ty + rl) & (N - 1), (tx + cl) & (N - 1))];
        }
    } else {"""
VARIANTS["pairs"] = [(F, OLD, NEW_PAIRS)]
