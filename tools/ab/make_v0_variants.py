"""Generate A/B source variants of the 64x64 kernel from a base sl_bits.hip."""
import sys

base_path, out_dir = sys.argv[1], sys.argv[2]
V0 = open(base_path).read()


def rep(s, old, new):
    assert old in s, old[:80]
    return s.replace(old, new)


def p_resetlist(s):
    s = rep(s, """    if (fx.fuse_reset && __builtin_amdgcn_readfirstlane(reset)) {
        __builtin_amdgcn_s_waitcnt(0);     // the epilogue's exit stores land first
        wave_reset(st, fx.pool, fx.ra, b, lane);
    }""", """    if (fx.fuse_reset && reset && lane == 0) {
        // queue the env for the reset kernel (k_env_reset_list)
        int64_t *cnt = fx.scratch + 8 * st.B + 2 + (a.step & 1);
        const int i = (int)atomicAdd((unsigned long long *)cnt, 1ull);
        reinterpret_cast<int32_t *>(fx.scratch + 2 * st.B)[i] = (int32_t)b;
    }""")
    s = rep(s, """}  // namespace

namespace sl {""", """__global__ void __launch_bounds__(64)
k_env_reset_list(sl_env_state st, sl_level_pool pool, ResetArgs ra, int64_t *scratch,
                 uint32_t step) {
    int64_t *cnt = scratch + 8 * st.B + 2;
    if (blockIdx.x == 0 && threadIdx.x == 0) cnt[(step + 1) & 1] = 0;
    const int n = (int)__builtin_amdgcn_readfirstlane((int)cnt[step & 1]);
    const int32_t *list = reinterpret_cast<const int32_t *>(scratch + 2 * st.B);
    for (int i = blockIdx.x; i < n; i += gridDim.x)
        wave_reset(st, pool, ra, __builtin_amdgcn_readfirstlane(list[i]), threadIdx.x);
}

}  // namespace

namespace sl {""")
    s = rep(s, """                       actions, ctp, ctc, reward, done, flags, ep_len, ep_rew);
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;""", """                       actions, ctp, ctc, reward, done, flags, ep_len, ep_rew);
    if (hipGetLastError() != hipSuccess) return SL_EHIP;
    if (fx.fuse_reset && fx.pool.K > 0) {
        const unsigned grid = (unsigned)(st.B < 8192 ? st.B : 8192);
        hipLaunchKernelGGL(k_env_reset_list, dim3(grid), dim3(64), 0, s, st, fx.pool, fx.ra,
                           fx.scratch, a.step);
    }
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;""")
    return s


def p_dpp(s):
    s = rep(s, """__device__ __forceinline__ u32 wave_or(u32 v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v |= (u32)__shfl_xor((int)v, o, 64);
    return (u32)__builtin_amdgcn_readfirstlane((int)v);
}""", """template <int CTRL>
__device__ __forceinline__ u32 dpp(u32 v) {
    return (u32)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ int wave_total(int x) {
    u32 v = (u32)x;
    v += dpp<0xB1>(v);
    v += dpp<0x4E>(v);
    v += dpp<0x141>(v);
    v += dpp<0x140>(v);
    return (int)((u32)__builtin_amdgcn_readlane((int)v, 0) + (u32)__builtin_amdgcn_readlane((int)v, 16) +
                 (u32)__builtin_amdgcn_readlane((int)v, 32) + (u32)__builtin_amdgcn_readlane((int)v, 48));
}
__device__ __forceinline__ u32 wave_or(u32 v) {
    v |= dpp<0xB1>(v);
    v |= dpp<0x4E>(v);
    v |= dpp<0x141>(v);
    v |= dpp<0x140>(v);
    return (u32)__builtin_amdgcn_readlane((int)v, 0) | (u32)__builtin_amdgcn_readlane((int)v, 16) |
           (u32)__builtin_amdgcn_readlane((int)v, 32) | (u32)__builtin_amdgcn_readlane((int)v, 48);
}""")
    s = s.replace("wave_sum(", "wave_total(")
    return s


def p_ldsedit(s):
    s = rep(s, """    read_pairs(buf, lane, PB);
    if (roll < 0) {
        wait_lgkm();
        dma_board(st.start_board + off, buf, lane);
    }
    transpose32(PB);
    u32 erow = 0;                      // row pairs (y, y + 32) holding an edit
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (k < ne) {
            const int y = eidx[k] >> 6, x = eidx[k] & 63;
            const int tl = 2 * (x >> 1) + (y >> 5);            // lane holding the cell
            const u32 bit = 1u << (y & 31);
            const u32 m0 = (lane == tl && !(x & 1)) ? bit : 0u;
            const u32 m1 = (lane == tl && (x & 1)) ? bit : 0u;
            erow |= bit;
#pragma unroll
            for (int p = 0; p < 16; p++) {
                const u32 v = ((eval[k] >> p) & 1u) ? ~0u : 0u;
                PL(PB, p, 0) = mux(m0, v, PL(PB, p, 0));
                PL(PB, p, 1) = mux(m1, v, PL(PB, p, 1));
            }
        }
    }""", """    u32 erow = 0;                      // row pairs (y, y + 32) holding an edit
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (k < ne) {
            const int y = eidx[k] >> 6, x = eidx[k] & 63;
            erow |= 1u << (y & 31);
            if (lane == 0) {
                const int dw = y * 32 + (((x >> 1) + 16 * (y >> 5)) & 31);
                ((__attribute__((address_space(3))) uint16_t *)(buf + dw))[x & 1] = (uint16_t)eval[k];
            }
        }
    }
    read_pairs(buf, lane, PB);
    if (roll < 0) {
        wait_lgkm();
        dma_board(st.start_board + off, buf, lane);
    }
    transpose32(PB);""")
    return s


variants = {"ab_v0": V0, "ab_reslist": p_resetlist(V0), "ab_dpp": p_dpp(V0),
            "ab_ldsedit": p_ldsedit(V0), "ab_all3": p_ldsedit(p_dpp(p_resetlist(V0)))}
for k, v in variants.items():
    open("%s/%s.hip" % (out_dir, k), "w").write(v)
    print(k)


def p_startterms(s):
    # fold the start-board side-effect terms as the pool planes arrive
    a = s.index("__device__ __forceinline__ void score_planes(const u32 B[32], const u32 gc[3][2], const u32 S[32],")
    b = s.index("// ---------------------------------------------------------------- stores")
    s = s[:a] + open(sys.argv[3]).read() + s[b:]
    a = s.index("__device__ __forceinline__ void pool_planes(")
    b = s.index("__device__ __forceinline__ void wait_vm()")
    s = s[:a] + open(sys.argv[4]).read() + s[b:]
    s = rep(s, "    score_planes(P, gcol, P, &pts, &scr, &pos, &side);",
            "    score_planes(P, gcol, StartTerms{}, &pts, &scr, &pos, &side);")
    s = rep(s, """    u32 PS[32];
    if (roll >= 0) {
        pool_planes(fx.pool, __builtin_amdgcn_readfirstlane(st.level_index[b]), roll >> 16,
                    roll & 0xFFFF, lane, PS);
    } else {
        wait_vm();
        read_pairs(buf, lane, PS);
        transpose32(PS);
    }""", """    StartTerms stt;
    if (roll >= 0) {
        stt = pool_start_terms(fx.pool, __builtin_amdgcn_readfirstlane(st.level_index[b]),
                               roll >> 16, roll & 0xFFFF, lane, PB);
    } else {
        wait_vm();
        u32 PS[32];
        read_pairs(buf, lane, PS);
        transpose32(PS);
        stt = start_terms_from_planes(PB, PS);
    }""")
    s = rep(s, "    score_planes(PB, gcol, PS, &pts, &scr, &pos, &side);",
            "    score_planes(PB, gcol, stt, &pts, &scr, &pos, &side);")
    return s


if len(sys.argv) > 4:
    rd = p_dpp(p_resetlist(V0))
    more = {"ab_rd": rd, "ab_rd_st": p_startterms(rd)}
    for k, v in more.items():
        open("%s/%s.hip" % (out_dir, k), "w").write(v)
        print(k)
