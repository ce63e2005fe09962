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
