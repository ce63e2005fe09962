# nontemporal board/goal stores in the bit-sliced step kernels (tools/build_variant.py)
NT64 = [("sl_bits.hip", "            if (rb) store_pairs<32>(gb, PB, rb);",
         """            if (rb) {
#pragma unroll
                for (int y = 0; y < 32; y++)
                    if ((rb >> y) & 1u) __builtin_nontemporal_store(PB[y], &gb[y * 32]);
            }"""),
        ("sl_bits.hip", "            store_pairs<32>(gg, PG, rg);", """#pragma unroll
            for (int y = 0; y < 32; y++)
                if ((rg >> y) & 1u) __builtin_nontemporal_store(PG[y], &gg[y * 32]);""")]
NT128 = [("sl_bits128.hip", "if ((lm >> y) & 1u) gb[(32 * t + y) * RS] = P[y];",
          "if ((lm >> y) & 1u) __builtin_nontemporal_store(P[y], &gb[(32 * t + y) * RS]);"),
         ("sl_bits128.hip", "if ((lm >> y) & 1u) gg[(32 * t + y) * RS] = G[y];",
          "if ((lm >> y) & 1u) __builtin_nontemporal_store(G[y], &gg[(32 * t + y) * RS]);")]
# DMA reads with the nontemporal cache policy (aux = slc|nt-ish bits)
VARIANTS = {
    "nt_base": [],
    "nt_st": NT64 + NT128,
}
