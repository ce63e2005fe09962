# nontemporal policy on the goal-mirror and per-env record traffic
NT = [("sl_bits.hip", """            p.g[k][0] = mg[(9 + k) * 64];
            p.g[k][1] = mg[(25 + k) * 64];""", """            p.g[k][0] = __builtin_nontemporal_load(mg + (9 + k) * 64);
            p.g[k][1] = __builtin_nontemporal_load(mg + (25 + k) * 64);"""),
      ("sl_bits.hip", "            for (int q = 0; q < 32; q++) PG[q] = mg[q * 64];    // goal planes",
       "            for (int q = 0; q < 32; q++) PG[q] = __builtin_nontemporal_load(mg + q * 64);"),
      ("sl_bits.hip", "                    for (int k = 0; k < 16; k++) mg[(k + 16 * w) * 64] = PL(PG, k, w);",
       "                    for (int k = 0; k < 16; k++) __builtin_nontemporal_store(PL(PG, k, w), mg + (k + 16 * w) * 64);"),
      ("sl_bits128.hip", """            gcol[k][0] = m[(9 + k) * 64];
            gcol[k][1] = m[(25 + k) * 64];""", """            gcol[k][0] = __builtin_nontemporal_load(m + (9 + k) * 64);
            gcol[k][1] = __builtin_nontemporal_load(m + (25 + k) * 64);"""),
      ("sl_bits.h", "    return *reinterpret_cast<const u32 *>(p + off);",
       "    return __builtin_nontemporal_load(reinterpret_cast<const u32 *>(p + off));")]
VARIANTS = {"m_base": [], "m_nt": NT}
