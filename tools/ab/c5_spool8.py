# C5: the round-2 "8-plane spool" variant of k_env_step_bits128, rebuilt from its
# description: the start-board spool without planes 12-14 (no cell type
# uses those bits, so they read as 0) -- 8 KiB instead of 11 KiB per wave -- at the
# default launch bound (spool8) and at a 4-waves/SIMD bound (spool8_4w, the build that
# spilled and faulted on the box in round 2).  For offline ISA reading
# (tools/isa_lds_dma_check.py); not to be run on the GPU.
F = "sl_bits128.hip"
SPOOL8 = [(F, "constexpr int kPoolPlanes = 11;      // planes 0, 2, 7-15\n"
              "__device__ __forceinline__ int pool_plane(int s) { return s == 0 ? 0 : (s == 1 ? 2 : s + 5); }",
           "constexpr int kPoolPlanes = 8;       // planes 0, 2, 7-11, 15\n"
           "__device__ __forceinline__ int pool_plane(int s) {\n"
           "    return s == 0 ? 0 : (s == 1 ? 2 : (s < 7 ? s + 5 : 15));\n}")]
VARIANTS = {
    "spool8": SPOOL8,
    "spool8_4w": SPOOL8 + [(F, "constexpr int kMinWaves = 2;  // waves per SIMD",
                           "constexpr int kMinWaves = 4;  // waves per SIMD")],
}
