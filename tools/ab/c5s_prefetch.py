# C5 replay draw pass (k_stream_draw128): the first batch of a tensor's uniforms is
# issued as soon as the tensor's total is known, before the owner lanes write their
# cells' slots (the uniforms' addresses do not depend on the slots), so their HBM
# latency runs under the slot writes instead of after them.
F = "sl_bits128.hip"
R = [
    (F, """#pragma unroll
        for (int k = 0; k < NB * 2; k++) spw[k * 64 + lane] = 0u;
#pragma unroll 1
        for (int c0 = 0; c0 < total; c0 += kOwnSlots) {""",
     """        // the first batch of uniforms, in flight under the slot writes below
        double u0[kDrawBatch];
#pragma unroll
        for (int k = 0; k < kDrawBatch; k++) {
            const int i = 64 * k + lane;
            const int64_t r = pos + i;
            u0[k] = (i < total && r < n_draws) ? draws[r & draw_mask] : 1.0;
        }
#pragma unroll
        for (int k = 0; k < NB * 2; k++) spw[k * 64 + lane] = 0u;
#pragma unroll 1
        for (int c0 = 0; c0 < total; c0 += kOwnSlots) {"""),
    (F, """                    id[k] = i < n ? (u32)slots[i] : 0u;
                    u[k] = (i < n && r < n_draws) ? draws[r & draw_mask] : 1.0;""",
     """                    id[k] = i < n ? (u32)slots[i] : 0u;
                    u[k] = (c0 == 0 && i0 == 0) ? u0[k]
                                                : ((i < n && r < n_draws) ? draws[r & draw_mask] : 1.0);"""),
]
VARIANTS = {"pf_base": [], "pf_first": R}
B4 = [(F, "constexpr int kDrawBatch = 8;", "constexpr int kDrawBatch = 4;")]
B16 = [(F, "constexpr int kDrawBatch = 8;", "constexpr int kDrawBatch = 16;")]
VARIANTS.update({"pf_b4": B4, "pf_first_b4": R + B4, "pf_first_b16": R + B16})
