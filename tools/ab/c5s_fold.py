# C5 replay launches (round 5): the action folded into the count prologue
# (k_stream_prologue128_act) and the offsets scan in two launches
# (sl_scan_consume_i64); each undone alone, and both.
B = "sl_bits128.hip"
E = "sl_env.hip"
NOFOLD = [(B, "constexpr bool kFoldAction = true;", "constexpr bool kFoldAction = false;")]
SCAN3 = [(E, """                       : sl_scan_consume_i64(sc.counts, sc.offsets, 2 * st.B, base,
                                             fx.stream_pos, (void *)s);""",
          """                       : sl_exclusive_scan_i64(sc.counts, sc.offsets, 2 * st.B, base,
                                               fx.stream_pos, (void *)s);""")]
VARIANTS = {"cur": [], "nofold": NOFOLD, "scan3": SCAN3, "r4launch": NOFOLD + SCAN3}
