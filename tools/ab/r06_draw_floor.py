# The bit-ring draw pass without its deposit loop (WRONG spawns; timing floor only):
# how much of k_stream_draw128_bits is the per-cell deposit (round 6)
OLD = """            u32 m = R0[t] | R1[t], s0 = 0u, s1 = 0u;
            while (m) {
                const int i = __builtin_ctz(m);
                m &= m - 1u;
                if ((R0[t] >> i) & 1u) {
                    s0 |= (u32)(sb & 1u) << i;
                    sb >>= 1;
                }
                if ((R1[t] >> i) & 1u) {
                    s1 |= (u32)(sb & 1u) << i;
                    sb >>= 1;
                }
            }"""
NEW = """            const u32 s0 = (u32)sb & R0[t], s1 = (u32)(sb >> 32) & R1[t];"""
VARIANTS = {"draw_floor": [("sl_bits128.hip", OLD, NEW)]}
