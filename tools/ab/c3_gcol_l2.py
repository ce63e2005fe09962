# C3 timing probe (results wrong, never for parity): the goal colour planes read from 64
# envs' mirrors (L2-resident) instead of each env's own (HBM) -- what the 1.5 KB of
# colour-plane reads per env-step cost, before building a pool-sourced path for them.
F = "sl_bits.hip"
VARIANTS = {
    "gl_base": [],
    "gl_l2": [(F, """    if (st.planes) {
        const u32 *mg = st.planes + b * 4096 + 2048 + lane;""", """    if (st.planes) {
        const u32 *mg = st.planes + (b & 63) * 4096 + 2048 + lane;""")],
}
