# C5 seeded (device MT19937 stream): waves per jump workgroup (k_mt_jump<NWJ>): more
# waves split the polynomial's coefficients finer (each wave correlates 1/NWJ of them).
F = "sl_mt.hip"
VARIANTS = {"mj%d" % n: [(F, "constexpr int kJumpWaves = 4;", "constexpr int kJumpWaves = %d;" % n)]
            for n in (4, 8, 16)}
