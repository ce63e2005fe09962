F = "sl_bits128.hip"
VARIANTS = {
    "n128_base": [],
    "n128_nt": [(F, "        load_pairs<RS>(gb + 32 * t * RS, P);", "        load_pairs_nt<RS>(gb + 32 * t * RS, P);"),
                (F, "            load_pairs<RS>(gg + 32 * t * RS, G);", "            load_pairs_nt<RS>(gg + 32 * t * RS, G);")],
}
