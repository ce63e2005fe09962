# A/B variants of the fused packed view in the 64x64 plane kernel (round 6, c3p):
#   c3p_base -- the tree
#   c3p_nt   -- the view's dword stores nontemporal
#   c3p_u2   -- two view dwords per iteration, their four LDS reads issued first
OLD = """            const uint32_t v0 = cells[lds_cell_idx((ty + rr) & (N - 1), (tx + cc) & (N - 1))];
            const uint32_t v1 = cells[lds_cell_idx((ty + r1) & (N - 1), (tx + c1) & (N - 1))];
            o32[p] = v0 | (v1 << 16);"""
VARIANTS = {
    "c3p_base": [],
    "c3p_nt": [("sl_bits.hip", OLD, """            const uint32_t v0 = cells[lds_cell_idx((ty + rr) & (N - 1), (tx + cc) & (N - 1))];
            const uint32_t v1 = cells[lds_cell_idx((ty + r1) & (N - 1), (tx + c1) & (N - 1))];
            __builtin_nontemporal_store(v0 | (v1 << 16), &o32[p]);""")],
}
