# C5 spawn draws: per-lane Philox loop (lane_draws) vs the wave-compacted queue
# (compact_draws), and the Philox rounds rolled vs two per iteration.
F = "sl_bits128.hip"
D = "sl_device.h"
LANE = (F, "philox_spawn_compact(*this, elig, sp, sc, tensor, slots);", "philox_spawn(*this, elig, sp, sc, tensor);")
ROLL1 = (D, "#pragma unroll 2\n    for (int r = 0; r < 10; r++) {", "#pragma unroll 1\n    for (int r = 0; r < 10; r++) {")
VARIANTS = {
    "d_lane_u1": [LANE, ROLL1],
    "d_lane_u2": [LANE],
    "d_comp_u1": [ROLL1],
    "d_comp_u2": [],
}
