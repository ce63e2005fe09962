# C3 with fused packed views: write_obs's gather fully unrolled for views of up to 18
# rows of 64 cells (33x33 = 1 089): every LDS read issued before the first store
# (reads past the view stay inside the board: rows and columns wrap at 64), then the
# stores; larger views keep the loop.
F = "sl_bits.hip"
OLD = """    if (small) {
        for (int i = lane; i < nv; i += 64) {"""
NEW = """    if (small && nv <= 18 * 64) {
        u32 v[18];
#pragma unroll
        for (int k = 0; k < 18; k++) {
            v[k] = cells[lds_cell_idx((ty + r) & (N - 1), (tx + c) & (N - 1))];
            r += dr;
            c += dc;
            if (c >= vw) {
                c -= vw;
                r++;
            }
        }
#pragma unroll
        for (int k = 0; k < 18; k++)
            if (lane + 64 * k < nv) o[lane + 64 * k] = (uint16_t)v[k];
    } else if (small) {
        for (int i = lane; i < nv; i += 64) {"""
VARIANTS = {"g_unroll": [(F, OLD, NEW)]}
VARIANTS["g_base"] = []
