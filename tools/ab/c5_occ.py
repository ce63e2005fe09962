# C5: sensitivity of k_env_step_bits128 to occupancy (LDS padding forces fewer waves/CU)
F = "sl_bits128.hip"
def pad(kib):
    return [(F, "__shared__ __attribute__((aligned(16))) u32 spool_[kPoolPlanes * 256];",
             "__shared__ __attribute__((aligned(16))) u32 spool_[kPoolPlanes * 256 + %d];\n"
             "    if (lane == 999) spool_[kPoolPlanes * 256 + %d - 1] = 0;" % (kib * 256, kib * 256))]
VARIANTS = {
    "occ_base": [],
    "occ_2w": pad(9),      # 20 KiB per wave: 8 waves/CU = 2/SIMD
}
