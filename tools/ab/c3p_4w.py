# C3 with fused packed views: k_env_step_bits64<true, 0> at a 4-waves/SIMD launch bound
# (130 VGPRs at 3) -- register use and spills (tools/build_variant.py)
F = "sl_bits.hip"
VARIANTS = {
    "obs4w": [(F, "__global__ void __launch_bounds__(64, (OBS || MODE == SPAWN_STREAM) ? kMinWavesObs : kMinWaves)",
               "__global__ void __launch_bounds__(64, MODE == SPAWN_STREAM ? kMinWavesObs : kMinWaves)")],
}
# register use without the bits-12-14 view path (measurement only: wrong views there)
VARIANTS["nohi"] = [(F, "            if (OBS) {      // bits 12-14 in use: add the goal colours bit-sliced",
                     "            if (false) {      // bits 12-14 in use: add the goal colours bit-sliced")]
VARIANTS["nohi4w"] = VARIANTS["obs4w"] + VARIANTS["nohi"]
# where the 130 VGPRs come from (measurement only)
VARIANTS["nowrite"] = [(F, "        write_obs(buf, fx, fl, b, lane);", "")]
VARIANTS["nogoal"] = [(F, "                for (int k = 0; k < 3; k++) PL(PB, 12 + k, w) = gv[k][w] & ~white;",
                       "                for (int k = 0; k < 3; k++) PL(PB, 12 + k, w) = 0;")]
VARIANTS["nogoal4w"] = VARIANTS["obs4w"] + VARIANTS["nogoal"]
VARIANTS["nowrite4w"] = VARIANTS["obs4w"] + VARIANTS["nowrite"]
VARIANTS["nowrite_nogoal4w"] = VARIANTS["obs4w"] + VARIANTS["nowrite"] + VARIANTS["nogoal"]
