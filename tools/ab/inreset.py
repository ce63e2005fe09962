# resets inside the 64x64 step kernel through a non-inlined call (no reset-list kernel)
F = "sl_bits.hip"
VARIANTS = {"ir_base": [], "ir_call": [
    (F, """// all kernel arguments of k_env_step_bits64 in one struct at kernarg offset 0, so a""",
        """__device__ __attribute__((noinline)) void wave_reset_call(const sl_env_state &st,
                                                         const sl_level_pool &pool,
                                                         const ResetArgs &ra, int64_t b, int lane) {
    wave_reset(st, pool, ra, b, lane);
}

// all kernel arguments of k_env_step_bits64 in one struct at kernarg offset 0, so a"""),
    (F, """    if (fx.fuse_reset && reset && lane == 0) {
        // queue the env for the reset kernel (k_env_reset_list)
        int64_t *cnt = fx.scratch + 8 * st.B + 2 + (a.step & 1);
        const int i = (int)atomicAdd((unsigned long long *)cnt, 1ull);
        reset_list(fx.scratch)[i] = (int32_t)b;
    }
}""", """    if (OBS && fx.fuse_reset && reset && lane == 0) {
        // queue the env for the reset kernel (k_env_reset_list)
        int64_t *cnt = fx.scratch + 8 * st.B + 2 + (a.step & 1);
        const int i = (int)atomicAdd((unsigned long long *)cnt, 1ull);
        reset_list(fx.scratch)[i] = (int32_t)b;
    }
    if (!OBS && fx.fuse_reset && reset) {
        wait_vm();
        const StepKArgs &k = kernarg();
        wave_reset_call(k.st, k.fx.pool, k.fx.ra, b, lane);
    }
}"""),
    (F, """    if (fx.fuse_reset && fx.pool.K > 0) {
        const unsigned grid = (unsigned)(st.B < 512 ? st.B : 512);""", """    if (fx.fuse_reset && fx.pool.K > 0 && fx.obs_out) {
        const unsigned grid = (unsigned)(st.B < 512 ? st.B : 512);"""),
]}
