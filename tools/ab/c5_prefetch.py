# C5: band-ahead L2 prefetch (prefetch_band, LDS-DMA into a dump row) on / off.
F = "sl_bits128.hip"
VARIANTS = {
    "p_off": [(F, "            if (t < NB - 1) prefetch_band(gg + 32 * (t + 1) * RS, dump);\n", ""),
              (F, "        if (t < NB - 1) prefetch_band(gb + 32 * (t + 1) * RS, dump);\n", "")],
    "p_on": [],
}
VARIANTS["p_all"] = [(F, "        if (t < NB - 1) prefetch_band(gb + 32 * (t + 1) * RS, dump);\n",
                      "        if (t == 0)\n#pragma unroll\n            for (int u = 1; u < NB; u++) prefetch_band(gb + 32 * u * RS, dump);\n")]
