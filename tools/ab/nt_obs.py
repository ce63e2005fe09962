VARIANTS = {"o_base": [], "o_nt": [
    ("sl_bits.hip", "            o[i] = cells[lds_cell_idx((ty + r) & (N - 1), (tx + c) & (N - 1))];",
     "            __builtin_nontemporal_store((uint16_t)cells[lds_cell_idx((ty + r) & (N - 1), (tx + c) & (N - 1))], o + i);")]}
