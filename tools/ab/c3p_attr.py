# Timing-only attribution of the packed view's cost (outputs WRONG in every variant but
# pa_base: never shipped, never parity-tested).  pa_ret: write_obs returns at once;
# pa_nostore: the gather runs, its values are consumed by an empty asm instead of stored;
# pa_nogather: the stores run with a lane-computed value instead of the LDS gather.
F = "sl_bits.hip"
HEAD = """    lds_u16 *cells = reinterpret_cast<lds_u16 *>(buf);
    (void)fx;
    const FastExtra &lfx = kernarg().fx;     // read late: no SGPRs held through the step
    const int vh = lfx.obs_vh, vw = lfx.obs_vw;"""
STORE = """            o[i] = cells[lds_cell_idx((ty + r) & (N - 1), (tx + c) & (N - 1))];
            r += dr;"""
VARIANTS = {
    "pa_base": [],
    "pa_ret": [(F, HEAD, HEAD.replace("(void)fx;", "(void)fx;\n    if (b >= 0) return;"))],
    "pa_nostore": [(F, STORE, STORE.replace(
        "o[i] = cells[lds_cell_idx((ty + r) & (N - 1), (tx + c) & (N - 1))];",
        "{ u32 x_ = cells[lds_cell_idx((ty + r) & (N - 1), (tx + c) & (N - 1))]; asm volatile(\"\" :: \"v\"(x_)); }"))],
    "pa_nogather": [(F, STORE, STORE.replace(
        "o[i] = cells[lds_cell_idx((ty + r) & (N - 1), (tx + c) & (N - 1))];",
        "o[i] = (uint16_t)(lds_cell_idx((ty + r) & (N - 1), (tx + c) & (N - 1)));"))],
}
# round 2 of the probe: pa_noexit skips the exit moves (ne = 0; wrong for levels with
# exits); pa_batch8 keeps the outputs exact and issues 8 LDS gathers before their 8
# stores (software-pipelined; the shipped loop waits on each read before its store).
LOOP = """    if (small) {
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
BATCH = """    if (small) {
        for (int i0 = lane; i0 < nv; i0 += 8 * 64) {
            u32 v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                v[u] = cells[lds_cell_idx((ty + r) & (N - 1), (tx + c) & (N - 1))];
                r += dr;
                c += dc;
                if (c >= vw) {
                    c -= vw;
                    r++;
                }
            }
#pragma unroll
            for (int u = 0; u < 8; u++)
                if (i0 + 64 * u < nv) o[i0 + 64 * u] = (uint16_t)v[u];
        }
    } else {"""
VARIANTS["pa_noexit"] = [(F, "const int ne = min(fl.exit_count(), SL_MAX_EXITS);", "const int ne = 0 * min(fl.exit_count(), SL_MAX_EXITS);")]
VARIANTS["pa_batch8"] = [(F, LOOP, BATCH)]
