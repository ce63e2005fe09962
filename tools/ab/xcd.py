# XCD-aware env order: workgroups are dealt round-robin over the 8 XCDs, so with
# env = blockIdx the 32 envs sharing a 128-byte line of a per-env field array (and two
# neighbouring views' boundary lines) sit in 8 different L2s.  Here workgroup i runs env
# (i % 8) * (B / 8) + i / 8 (B a multiple of 8): runs of B / 8 consecutive envs per XCD.
F = "sl_bits.hip"
F128 = "sl_bits128.hip"
REMAP = """    const int64_t nb8 = ka.st.B >> 3;
    const int64_t b = (ka.st.B & 7) ? (int64_t)blockIdx.x
                                     : (int64_t)(blockIdx.x & 7) * nb8 + (blockIdx.x >> 3);"""
X64 = [(F, "    const int64_t b = blockIdx.x;          // one wave per env", REMAP)]
X128 = [(F128, """    const int64_t b = blockIdx.x;
    const int lane = threadIdx.x;
    const int64_t off = b * (int64_t)(N * N);
    u32 *gb""", REMAP + """
    const int lane = threadIdx.x;
    const int64_t off = b * (int64_t)(N * N);
    u32 *gb""")]
VARIANTS = {"x_base": [], "x_xcd": X64 + X128}
