"""Timing probe (exact outputs): the C5 board band's two transposes done three times each
(two extra transposes cancel), to price the transposes a plane-major board would save."""
_IN = "        const u32 last = P[31];\n        transpose32(P);\n"
_OUT = "            transpose32(P);\n#pragma unroll\n            for (int y = 0; y < 32; y++)\n                if ((rb >> y) & 1u) __builtin_nontemporal_store(P[y], &gb[(32 * t + y) * RS]);"
VARIANTS = {
    "tr1": [],
    "tr3": [("sl_bits128.hip", _IN, _IN + "        transpose32(P);\n        transpose32(P);\n"),
            ("sl_bits128.hip", _OUT, "            transpose32(P);\n            transpose32(P);\n" + _OUT)],
}
