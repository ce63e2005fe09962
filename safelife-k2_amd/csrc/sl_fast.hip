// sl_fast.hip -- the env-step kernel for 64-wide boards (the headline 64x64 config).
//
// Same semantics as k_env_step_generic (sl_env.hip), re-laid-out for CDNA4:
//
//  * one wave64 per env, four envs per 256-thread workgroup, no LDS, no barriers;
//  * lane = (strip, column group): 16 lanes span a 64-cell row (4 cells = 8 bytes
//    each, so a wave-wide load is four fully-used 128-byte row segments) and the 4
//    strips of 16 lanes each own H/4 consecutive rows;
//  * a row's 4 cells live packed two per 32-bit register (two uint16 halves), so
//    every bitwise op, v_alignbit, v_pk_lshrrev_b16 and v_mul_u32_u24 below
//    evaluates the rule for 2 cells at once;
//  * horizontal neighbours: the 16-lane DPP rotations row_ror:1 / row_ror:15 wrap
//    exactly at W = 64 (the torus), so the left / right neighbour words cost one
//    DPP move each and three v_alignbit funnel shifts;
//  * vertical neighbours: each lane walks its strip top to bottom with a rolling
//    window of row summaries (the two halo rows are re-read from L2);
//  * each row summary folds the 3 cells of a row into ones (OR), twos (>= 2,
//    majority) and a count; the column pass folds 3 row summaries the same way
//    (reference advance_board.c:12-32,51-86 does the same
//    separable fold cell by cell);
//  * scores are kept incrementally: points / perf score / possible / side-effect
//    totals change only where a cell changed, so the per-cell scoring work, the
//    start-board read and the store are all skipped (wave-uniformly) on rows
//    where nothing changed -- on still-life boards almost every row.
//    The totals equal the full sums the generic kernel computes (tested).
#include "sl_env_common.h"

using namespace sl;

namespace {

constexpr uint32_t ONE2 = 0x00010001u;

__device__ __forceinline__ uint32_t pk_shr(uint32_t val, uint32_t amt) {
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    us2 v = __builtin_bit_cast(us2, val), s = __builtin_bit_cast(us2, amt);
    return __builtin_bit_cast(uint32_t, (us2)(v >> s));   // v_pk_lshrrev_b16
}

__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t x, uint32_t y) {
    return (m & x) | (~m & y);                            // v_bfi_b32
}

// 0xFFFF in every 16-bit half whose bit 0 (bit 16) is set: x is 0/1 per half
__device__ __forceinline__ uint32_t expand(uint32_t x) { return __umul24(x, 0xFFFFu); }

// lane (l - 1) mod 16 / (l + 1) mod 16 inside each 16-lane DPP row
__device__ __forceinline__ uint32_t from_left(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x121, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t from_right(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x12F, 0xF, 0xF, false);
}

struct CW {          // contribution words of a row pair-register
    uint32_t c, a, am;
};

// c(n) per cell (see sl_device.h): P|I|S flags, alive destructible-or-exit +
// colours at bits 8-11, spawner colours at bits 13-15.
__device__ __forceinline__ CW cword(uint32_t v, bool spawn) {
    CW r;
    r.a = v & ONE2;
    r.am = expand(r.a);
    const uint32_t t = ((v << 5) & 0x01000100u) | v;       // exit bit |= destructible
    uint32_t c = ((t & 0x0F000F00u) & r.am) | (v & 0x00E000E0u) | r.a;
    if (spawn) {
        const uint32_t sm = expand((v >> 7) & ONE2);
        c |= ((v & 0x0E000E00u) << 4) & sm;
    }
    r.c = c;
    return r;
}

struct RowSum {
    uint32_t o0, t0, n0, o1, t1, n1;
};

__device__ __forceinline__ RowSum row_sum(uint32_t c0, uint32_t c1) {
    const uint32_t cl = from_left(c1);                       // cells 4cg-2, 4cg-1
    const uint32_t cr = from_right(c0);                      // cells 4cg+4, 4cg+5
    const uint32_t L = __builtin_amdgcn_alignbit(c0, cl, 16);   // 4cg-1, 4cg
    const uint32_t M = __builtin_amdgcn_alignbit(c1, c0, 16);   // 4cg+1, 4cg+2
    const uint32_t Rr = __builtin_amdgcn_alignbit(cr, c1, 16);  // 4cg+3, 4cg+4
    RowSum s;
    const uint32_t mA = M & ONE2;
    s.o0 = L | c0 | M;
    s.t0 = bfi(L ^ c0, M, L);
    s.n0 = (L & ONE2) + (c0 & ONE2) + mA;
    s.o1 = M | c1 | Rr;
    s.t1 = bfi(M ^ c1, Rr, M);
    s.n1 = mA + (c1 & ONE2) + (Rr & ONE2);
    return s;
}

// rule for one pair-register given the folded neighbourhood.
//   returns the new pair; *elig = per-half bit 0 set where the cell draws a uniform;
//   *spv = the value a spawn would write (per half).
__device__ __forceinline__ uint32_t decide(uint32_t v, const CW &w, uint32_t oU, uint32_t tU,
                                           uint32_t nU, uint32_t oC, uint32_t tC, uint32_t nC,
                                           uint32_t oD, uint32_t tD, uint32_t nD, bool spawn,
                                           uint32_t *elig, uint32_t *spv) {
    const uint32_t ones = oU | oC | oD;
    const uint32_t twos = tU | tC | tD | bfi(oU ^ oC, oD, oU);
    const uint32_t cnt = nU + nC + nD;
    const uint32_t pi = pk_shr(ones, 0x00060006u - w.a);           // P (alive) / I (dead)
    const uint32_t x = pk_shr((w.a << 4) | 0x00080008u, cnt) & ONE2; // survive / birth
    const uint32_t hold = (v >> 4) | pi;                             // frozen | P / I
    const uint32_t change = bfi(hold, 0u, x ^ w.a);                  // kill or birth
    const uint32_t cols = (twos | (ones >> 4)) & 0x0E000E00u;
    const uint32_t bv = cols | ((twos >> 5) & 0x00080008u) | ONE2;   // newborn
    const uint32_t out = bfi(expand(change), bfi(w.am, 0u, bv), v);
    if (spawn) {
        *elig = (ones >> 7) & ~(hold | x | w.a) & ONE2;
        *spv = cols | 0x00090009u;
    } else {
        *elig = 0;
    }
    return out;
}

__device__ __forceinline__ uint32_t apply_spawn(uint32_t out, uint32_t elig, uint32_t spv,
                                                int cell0, uint32_t gid, const StepArgs &a,
                                                uint32_t tensor, double thr) {
    if (elig & 1u) {
        if (philox_uniform((uint32_t)cell0, gid, a.step, tensor, a.seed) < thr)
            out = (out & 0xFFFF0000u) | (spv & 0xFFFFu);
    }
    if (elig & 0x10000u) {
        if (philox_uniform((uint32_t)cell0 + 1u, gid, a.step, tensor, a.seed) < thr)
            out = (out & 0x0000FFFFu) | (spv & 0xFFFF0000u);
    }
    return out;
}

__device__ __forceinline__ void delta_cell(uint32_t ob, uint32_t nb, uint32_t og, uint32_t ng,
                                           uint32_t s, int d[4]) {
    if (ob == nb && og == ng) return;
    int p0, q0, r0, p1, q1, r1;
    cell_scores(ob, og, &p0, &q0, &r0);
    cell_scores(nb, ng, &p1, &q1, &r1);
    d[0] += p1 - p0;
    d[1] += q1 - q0;
    d[2] += r1 - r0;
    d[3] += side_term(nb, s, ng) - side_term(ob, s, og);
}

template <int H>
__global__ void __launch_bounds__(256, 3)
k_env_step_w64(sl_env_state st, StepArgs a, const int64_t *__restrict__ act,
               double *__restrict__ reward_out, uint8_t *__restrict__ done_out,
               uint8_t *__restrict__ flags_out, int32_t *__restrict__ ep_len_out,
               int32_t *__restrict__ ep_rew_out) {
    constexpr int R = H / 4;           // rows per strip
    constexpr int RW = 16;             // uint2 words per row
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= st.B) return;             // whole wave leaves together
    const int cg = lane & 15;
    const int y0 = (lane >> 4) * R;
    const int64_t off = b * (int64_t)(H * 64);
    uint2 *gb = reinterpret_cast<uint2 *>(st.board + off);
    uint2 *gg = reinterpret_cast<uint2 *>(st.goals + off);
    const uint2 *gs = reinterpret_cast<const uint2 *>(st.start_board + off);

    uint2 vb[R + 2], vg[R + 2];
#pragma unroll
    for (int k = 0; k < R + 2; k++) {
        int y = y0 - 1 + k;
        y = y < 0 ? y + H : (y >= H ? y - H : y);
        vb[k] = gb[y * RW + cg];
        vg[k] = gg[y * RW + cg];
    }
    uint32_t sp_b = 0, sp_g = 0;
#pragma unroll
    for (int k = 1; k <= R; k++) {
        sp_b |= vb[k].x | vb[k].y;
        sp_g |= vg[k].x | vg[k].y;
    }
    const bool spawn_b = __ballot((sp_b & 0x00800080u) != 0) != 0;   // any spawner: board
    const bool spawn_g = __ballot((sp_g & 0x00800080u) != 0) != 0;   //              goals
    const double thr = (double)st.spawn_prob[b];
    const uint32_t gid = a.env0 + (uint32_t)b;

    CW wb0 = cword(vb[0].x, spawn_b), wb1 = cword(vb[0].y, spawn_b);
    CW wg0 = cword(vg[0].x, spawn_g), wg1 = cword(vg[0].y, spawn_g);
    RowSum pb = row_sum(wb0.c, wb1.c), pg = row_sum(wg0.c, wg1.c);
    wb0 = cword(vb[1].x, spawn_b); wb1 = cword(vb[1].y, spawn_b);
    wg0 = cword(vg[1].x, spawn_g); wg1 = cword(vg[1].y, spawn_g);
    RowSum cb = row_sum(wb0.c, wb1.c), cgs = row_sum(wg0.c, wg1.c);

    int d[4] = {0, 0, 0, 0};           // d points, d score, d possible, d side
#pragma clang loop unroll(full)
    for (int r = 0; r < R; r++) {
        const int k = r + 1;
        const int y = y0 + r;
        const CW nb0w = cword(vb[k + 1].x, spawn_b), nb1w = cword(vb[k + 1].y, spawn_b);
        const CW ng0w = cword(vg[k + 1].x, spawn_g), ng1w = cword(vg[k + 1].y, spawn_g);
        const RowSum nbs = row_sum(nb0w.c, nb1w.c), ngs = row_sum(ng0w.c, ng1w.c);

        uint32_t eb0, eb1, eg0, eg1, sb0, sb1, sg0, sg1;
        uint32_t b0 = decide(vb[k].x, wb0, pb.o0, pb.t0, pb.n0, cb.o0, cb.t0, cb.n0, nbs.o0,
                             nbs.t0, nbs.n0, spawn_b, &eb0, &sb0);
        uint32_t b1 = decide(vb[k].y, wb1, pb.o1, pb.t1, pb.n1, cb.o1, cb.t1, cb.n1, nbs.o1,
                             nbs.t1, nbs.n1, spawn_b, &eb1, &sb1);
        uint32_t g0 = decide(vg[k].x, wg0, pg.o0, pg.t0, pg.n0, cgs.o0, cgs.t0, cgs.n0, ngs.o0,
                             ngs.t0, ngs.n0, spawn_g, &eg0, &sg0);
        uint32_t g1 = decide(vg[k].y, wg1, pg.o1, pg.t1, pg.n1, cgs.o1, cgs.t1, cgs.n1, ngs.o1,
                             ngs.t1, ngs.n1, spawn_g, &eg1, &sg1);
        if (spawn_b || spawn_g) {
            if (__ballot((eb0 | eb1 | eg0 | eg1) != 0)) {
                const int cell = y * 64 + cg * 4;
                b0 = apply_spawn(b0, eb0, sb0, cell, gid, a, 0u, thr);
                b1 = apply_spawn(b1, eb1, sb1, cell + 2, gid, a, 0u, thr);
                g0 = apply_spawn(g0, eg0, sg0, cell, gid, a, 1u, thr);
                g1 = apply_spawn(g1, eg1, sg1, cell + 2, gid, a, 1u, thr);
            }
        }
        const bool chb = ((b0 ^ vb[k].x) | (b1 ^ vb[k].y)) != 0;
        const bool chg = ((g0 ^ vg[k].x) | (g1 ^ vg[k].y)) != 0;
        if (__ballot(chb || chg)) {
            if (chb) gb[y * RW + cg] = make_uint2(b0, b1);
            if (chg) gg[y * RW + cg] = make_uint2(g0, g1);
            if (chb || chg) {
                const uint2 s = gs[y * RW + cg];
                delta_cell(vb[k].x & 0xFFFF, b0 & 0xFFFF, vg[k].x & 0xFFFF, g0 & 0xFFFF,
                           s.x & 0xFFFF, d);
                delta_cell(vb[k].x >> 16, b0 >> 16, vg[k].x >> 16, g0 >> 16, s.x >> 16, d);
                delta_cell(vb[k].y & 0xFFFF, b1 & 0xFFFF, vg[k].y & 0xFFFF, g1 & 0xFFFF,
                           s.y & 0xFFFF, d);
                delta_cell(vb[k].y >> 16, b1 >> 16, vg[k].y >> 16, g1 >> 16, s.y >> 16, d);
            }
        }
        pb = cb; cb = nbs; pg = cgs; cgs = ngs;
        wb0 = nb0w; wb1 = nb1w; wg0 = ng0w; wg1 = ng1w;
    }
#pragma unroll
    for (int q = 0; q < 4; q++) d[q] = wave_sum(d[q]);
    if (lane != 0) return;
    const int64_t B = st.B;
    const int points = st.old_points[b] + (int)act[B + b] + d[0];
    const int score = st.score[b] + (int)act[2 * B + b] + d[1];
    const int possible = st.possible[b] + d[2];
    const int side = st.side_effect[b] + (int)act[3 * B + b] + d[3];
    env_epilogue(st, a, b, (int)act[b], points, score, possible, side, reward_out, done_out,
                 flags_out, ep_len_out, ep_rew_out);
}

}  // namespace

namespace sl {

bool launch_step_fast(const sl_env_state &st, const StepArgs &a, const int64_t *act,
                      double *reward, uint8_t *done, uint8_t *flags, int32_t *ep_len,
                      int32_t *ep_rew, hipStream_t s, int *rc) {
    *rc = SL_OK;
    if (st.W != 64) return false;
    const unsigned grid = (unsigned)((st.B + 3) / 4);
    switch (st.H) {
        case 64:
            hipLaunchKernelGGL(k_env_step_w64<64>, dim3(grid), dim3(256), 0, s, st, a, act, reward,
                               done, flags, ep_len, ep_rew);
            break;
        default:
            return false;
    }
    if (hipGetLastError() != hipSuccess) *rc = SL_EHIP;
    return true;
}

}  // namespace sl
