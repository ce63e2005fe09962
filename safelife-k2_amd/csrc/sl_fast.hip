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

#ifndef SL_FAST_UNR
#define SL_FAST_UNR 2      // rows per unrolled chunk of the 16-row strip
#endif
#ifndef SL_FAST_OCC
#define SL_FAST_OCC 4      // waves per SIMD the register budget is sized for
#endif

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

// -- cold paths, kept out of line so the unrolled hot loop stays small ----------

// spawn draws for one row (board pair 0/1, goal pair 0/1); rare: only rows where a
// cell next to a spawner is eligible
__device__ __forceinline__ uint4 spawn_row(uint4 o, uint4 e, uint4 sv, int cell, uint32_t gid,
                                        uint32_t step, uint64_t seed, double thr) {
    uint32_t ow[4] = {o.x, o.y, o.z, o.w};
    const uint32_t ew[4] = {e.x, e.y, e.z, e.w}, sw[4] = {sv.x, sv.y, sv.z, sv.w};
#pragma unroll
    for (int q = 0; q < 4; q++) {           // q: 0,1 board pairs; 2,3 goal pairs
        const uint32_t tensor = q >> 1;
        const int c0 = cell + 2 * (q & 1);
#pragma unroll
        for (int h = 0; h < 2; h++) {
            if ((ew[q] >> (16 * h)) & 1u) {
                if (philox_uniform((uint32_t)(c0 + h), gid, step, tensor, seed) < thr) {
                    const uint32_t m = 0xFFFFu << (16 * h);
                    ow[q] = (ow[q] & ~m) | (sw[q] & m);
                }
            }
        }
    }
    return make_uint4(ow[0], ow[1], ow[2], ow[3]);
}

// score deltas of the 4 cells of a row that changed (board and/or goals)
__device__ __forceinline__ int4 delta_row(uint2 ob, uint2 nb, uint2 og, uint2 ng, uint2 s) {
    const uint32_t obw[2] = {ob.x, ob.y}, nbw[2] = {nb.x, nb.y};
    const uint32_t ogw[2] = {og.x, og.y}, ngw[2] = {ng.x, ng.y}, sw[2] = {s.x, s.y};
    int d0 = 0, d1 = 0, d2 = 0, d3 = 0;
#pragma unroll
    for (int j = 0; j < 2; j++)
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int sh = 16 * h;
            const uint32_t o = (obw[j] >> sh) & 0xFFFF, n = (nbw[j] >> sh) & 0xFFFF;
            const uint32_t go = (ogw[j] >> sh) & 0xFFFF, gn = (ngw[j] >> sh) & 0xFFFF;
            const uint32_t sv = (sw[j] >> sh) & 0xFFFF;
            if (o == n && go == gn) continue;
            int p0, q0, r0, p1, q1, r1;
            cell_scores(o, go, &p0, &q0, &r0);
            cell_scores(n, gn, &p1, &q1, &r1);
            d0 += p1 - p0;
            d1 += q1 - q0;
            d2 += r1 - r0;
            d3 += side_term(n, sv, gn) - side_term(o, sv, go);
        }
    return make_int4(d0, d1, d2, d3);
}

__device__ __forceinline__ int wrap_row(int y, int H) { return y < 0 ? y + H : (y >= H ? y - H : y); }

// H: board height (W = 64); UNR: rows per unrolled chunk (divides H/4); the next
// chunk's rows are prefetched while the current chunk is computed.
template <int H, int UNR>
__global__ void __launch_bounds__(256, SL_FAST_OCC)
k_env_step_w64(sl_env_state st, StepArgs a, const int64_t *__restrict__ act,
               double *__restrict__ reward_out, uint8_t *__restrict__ done_out,
               uint8_t *__restrict__ flags_out, int32_t *__restrict__ ep_len_out,
               int32_t *__restrict__ ep_rew_out) {
    constexpr int R = H / 4;           // rows per strip
    constexpr int RW = 16;             // uint2 words per row
    constexpr int NCH = R / UNR;
    static_assert(R % UNR == 0, "UNR must divide the strip height");
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= st.B) return;             // whole wave leaves together
    const int cg = lane & 15;
    const int y0 = (lane >> 4) * R;
    const int64_t off = b * (int64_t)(H * 64);
    uint2 *gb = reinterpret_cast<uint2 *>(st.board + off);
    uint2 *gg = reinterpret_cast<uint2 *>(st.goals + off);
    const uint2 *gs = reinterpret_cast<const uint2 *>(st.start_board + off);

    // rows y0-1 and y0 (halo + first centre), then the first chunk of "next" rows
    const uint2 hb = gb[wrap_row(y0 - 1, H) * RW + cg], hg = gg[wrap_row(y0 - 1, H) * RW + cg];
    uint2 vb = gb[y0 * RW + cg], vg = gg[y0 * RW + cg];
    // the bottom halo row is the next strip's first row, which that strip (the same
    // wave) overwrites in its first chunk: read it before any store
    const int ybot = wrap_row(y0 + R, H);
    const uint2 tb = gb[ybot * RW + cg], tg = gg[ybot * RW + cg];
    uint2 nxb[UNR], nxg[UNR];
#pragma unroll
    for (int j = 0; j < UNR; j++) {
        if (1 + j < R) {
            nxb[j] = gb[(y0 + 1 + j) * RW + cg];
            nxg[j] = gg[(y0 + 1 + j) * RW + cg];
        } else {
            nxb[j] = tb;
            nxg[j] = tg;
        }
    }
    // any spawner on the board / goals: the whole strip group must agree, so test
    // every row once up front (cheap: one OR per row word, one ballot)
    uint32_t spb = hb.x | hb.y | vb.x | vb.y | tb.x | tb.y;
    uint32_t spg = hg.x | hg.y | vg.x | vg.y | tg.x | tg.y;
#pragma unroll
    for (int j = 0; j < UNR; j++) {
        spb |= nxb[j].x | nxb[j].y;
        spg |= nxg[j].x | nxg[j].y;
    }
    if (NCH > 1) {
        // rows beyond the first chunk: test them too (they are re-read later from L2)
#pragma unroll 4
        for (int k = UNR + 1; k < R; k++) {
            const uint2 xb = gb[(y0 + k) * RW + cg], xg = gg[(y0 + k) * RW + cg];
            spb |= xb.x | xb.y;
            spg |= xg.x | xg.y;
        }
    }
    const bool spawn_b = __ballot((spb & 0x00800080u) != 0) != 0;
    const bool spawn_g = __ballot((spg & 0x00800080u) != 0) != 0;
    const double thr = (double)st.spawn_prob[b];
    const uint32_t gid = a.env0 + (uint32_t)b;

    CW wb0 = cword(hb.x, spawn_b), wb1 = cword(hb.y, spawn_b);
    CW wg0 = cword(hg.x, spawn_g), wg1 = cword(hg.y, spawn_g);
    RowSum pb = row_sum(wb0.c, wb1.c), pg = row_sum(wg0.c, wg1.c);
    wb0 = cword(vb.x, spawn_b); wb1 = cword(vb.y, spawn_b);
    wg0 = cword(vg.x, spawn_g); wg1 = cword(vg.y, spawn_g);
    RowSum cb = row_sum(wb0.c, wb1.c), cgs = row_sum(wg0.c, wg1.c);

    int d[4] = {0, 0, 0, 0};           // d points, d score, d possible, d side
#pragma unroll 1
    for (int ch = 0; ch < NCH; ch++) {
        uint2 pfb[UNR], pfg[UNR];
        if (ch + 1 < NCH) {
#pragma unroll
            for (int j = 0; j < UNR; j++) {
                const int k = (ch + 1) * UNR + 1 + j;          // strip-relative row
                if (k < R) {
                    pfb[j] = gb[(y0 + k) * RW + cg];
                    pfg[j] = gg[(y0 + k) * RW + cg];
                } else {
                    pfb[j] = tb;
                    pfg[j] = tg;
                }
            }
        }
#pragma unroll
        for (int j = 0; j < UNR; j++) {
            const int y = y0 + ch * UNR + j;           // centre row
            const CW nb0w = cword(nxb[j].x, spawn_b), nb1w = cword(nxb[j].y, spawn_b);
            const CW ng0w = cword(nxg[j].x, spawn_g), ng1w = cword(nxg[j].y, spawn_g);
            const RowSum nbs = row_sum(nb0w.c, nb1w.c), ngs = row_sum(ng0w.c, ng1w.c);

            uint32_t o[4], e[4], sv[4];
            o[0] = decide(vb.x, wb0, pb.o0, pb.t0, pb.n0, cb.o0, cb.t0, cb.n0, nbs.o0, nbs.t0,
                          nbs.n0, spawn_b, &e[0], &sv[0]);
            o[1] = decide(vb.y, wb1, pb.o1, pb.t1, pb.n1, cb.o1, cb.t1, cb.n1, nbs.o1, nbs.t1,
                          nbs.n1, spawn_b, &e[1], &sv[1]);
            o[2] = decide(vg.x, wg0, pg.o0, pg.t0, pg.n0, cgs.o0, cgs.t0, cgs.n0, ngs.o0, ngs.t0,
                          ngs.n0, spawn_g, &e[2], &sv[2]);
            o[3] = decide(vg.y, wg1, pg.o1, pg.t1, pg.n1, cgs.o1, cgs.t1, cgs.n1, ngs.o1, ngs.t1,
                          ngs.n1, spawn_g, &e[3], &sv[3]);
            if (spawn_b || spawn_g) {
                const bool any_e = (e[0] | e[1] | e[2] | e[3]) != 0;
                if (__ballot(any_e)) {
                    if (any_e) {
                        const uint4 r4 = spawn_row(make_uint4(o[0], o[1], o[2], o[3]),
                                                   make_uint4(e[0], e[1], e[2], e[3]),
                                                   make_uint4(sv[0], sv[1], sv[2], sv[3]),
                                                   y * 64 + cg * 4, gid, a.step, a.seed, thr);
                        o[0] = r4.x; o[1] = r4.y; o[2] = r4.z; o[3] = r4.w;
                    }
                }
            }
            const bool chb = ((o[0] ^ vb.x) | (o[1] ^ vb.y)) != 0;
            const bool chg = ((o[2] ^ vg.x) | (o[3] ^ vg.y)) != 0;
            if (__ballot(chb || chg)) {
                if (chb) gb[y * RW + cg] = make_uint2(o[0], o[1]);
                if (chg) gg[y * RW + cg] = make_uint2(o[2], o[3]);
                if (chb || chg) {
                    const int4 dd = delta_row(vb, make_uint2(o[0], o[1]), vg,
                                              make_uint2(o[2], o[3]), gs[y * RW + cg]);
                    d[0] += dd.x; d[1] += dd.y; d[2] += dd.z; d[3] += dd.w;
                }
            }
            pb = cb; cb = nbs; pg = cgs; cgs = ngs;
            wb0 = nb0w; wb1 = nb1w; wg0 = ng0w; wg1 = ng1w;
            vb = nxb[j]; vg = nxg[j];
        }
        if (ch + 1 < NCH) {
#pragma unroll
            for (int j = 0; j < UNR; j++) {
                nxb[j] = pfb[j];
                nxg[j] = pfg[j];
            }
        }
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
            hipLaunchKernelGGL((k_env_step_w64<64, SL_FAST_UNR>), dim3(grid), dim3(256), 0, s, st,
                               a, act, reward, done, flags, ep_len, ep_rew);
            break;
        default:
            return false;
    }
    if (hipGetLastError() != hipSuccess) *rc = SL_EHIP;
    return true;
}

}  // namespace sl
