# C5 replay: the draw pass's uniform loads in flight per lane (kDrawBatch).  A C5 env
# draws ~1 300 uniforms per step (~21 per lane): with 8 in flight the wave waits on
# three dependent load batches; 16 / 24 issue them in two / one.
F = "sl_bits128.hip"
OLD = "constexpr int kDrawBatch = 8;"
VARIANTS = {"db_8": [], "db_16": [(F, OLD, "constexpr int kDrawBatch = 16;")],
            "db_24": [(F, OLD, "constexpr int kDrawBatch = 24;")]}
