# C5 replay: attribution of k_stream_draw128's time (timing only, results wrong):
# norank skips the rank loop's slot writes and ballots; noload skips the uniforms' loads
F = "sl_bits128.hip"
RANK = """                    const uint64_t m0 = __ballot(e0), m1 = __ballot(e1);"""
VARIANTS = {
    "norank": [(F, """                u32 m = rows[t];
                while (m) {""", """                u32 m = rows[t] & 0u;
                while (m) {""")],
    "noload": [(F, """                    u[k] = (i < n && r < n_draws) ? draws[r] : 1.0;""",
                """                    u[k] = (i < n && r < n_draws) ? (double)r * 1e-9 : 1.0;""")],
}
