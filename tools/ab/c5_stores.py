# C5 band stores: changed 64-byte sectors (per-lane exec mask per row) vs changed rows
# (wave-uniform branch per row, no exec-mask traffic).
F = "sl_bits128.hip"
VARIANTS = {
    "s_sector": [],
    "s_rows": [(F, "                    if ((lm >> y) & 1u) __builtin_nontemporal_store(P[y], &gb[(32 * t + y) * RS]);",
                "                    __builtin_nontemporal_store(P[y], &gb[(32 * t + y) * RS]);"),
               (F, "            const u32 lm = sector_rows(cb[0] | cb[1]);\n            transpose32(P);",
                "            transpose32(P);")],
}
