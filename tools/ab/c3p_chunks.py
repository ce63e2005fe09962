# C3 with fused packed views: write_obs (sl_bits.hip) stores the view as 16-byte chunks
# (8 cells each, aligned in the whole obs array; the env's first / last chunk, shared
# with the neighbouring envs, cell by cell) -- 3 store instructions per lane instead
# of 17, each chunk's 8 LDS gathers in flight together
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
        const int64_t a0 = b * (int64_t)nv;
        const int s0 = (int)(a0 & 7);               // the view's first cell in its chunk
        const int nq = (s0 + nv + 7) >> 3;          // 16-byte chunks the view touches
        uint16_t *o0 = lfx.obs_out + (a0 - s0);     // 16-byte aligned
        int v = 8 * lane - s0;                      // view cell of the chunk's first slot
        const int vq = v + 8 * vw;                  // >= 0
        int rr = vq / vw - 8, cc = vq - (vq / vw) * vw;
        const int d2r = 512 / vw, d2c = 512 - d2r * vw;
        for (int t = lane; t < nq; t += 64) {
            u32 h[8];
            int r1 = rr, c1 = cc;
#pragma unroll
            for (int u = 0; u < 8; u++) {
                h[u] = cells[lds_cell_idx((ty + r1) & (N - 1), (tx + c1) & (N - 1))];
                if (++c1 == vw) {
                    c1 = 0;
                    r1++;
                }
            }
            if (v >= 0 && v + 8 <= nv) {
                uint4 q;
                q.x = h[0] | (h[1] << 16);
                q.y = h[2] | (h[3] << 16);
                q.z = h[4] | (h[5] << 16);
                q.w = h[6] | (h[7] << 16);
                reinterpret_cast<uint4 *>(o0)[t] = q;
            } else {
#pragma unroll
                for (int u = 0; u < 8; u++)
                    if (v + u >= 0 && v + u < nv) o0[8 * t + u] = (uint16_t)h[u];
            }
            v += 512;
            rr += d2r;
            cc += d2c;
            if (cc >= vw) {
                cc -= vw;
                rr++;
            }
        }
    } else {"""
VARIANTS = {"p_base": [], "p_chunks": [(F, OLD, NEW)]}
