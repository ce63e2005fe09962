// sl_fast.hip -- the fused env-step kernel for 64-wide boards (the headline 64x64 config).
//
// Same semantics as k_env_action + k_env_step_generic (sl_env.hip), re-laid-out
// for CDNA4:
//
//  * one wave64 per env, four envs per 256-thread workgroup, no barriers after
//    the prologue;
//  * the action (execute_action / move_agent, safelife_game.py:308-393) is
//    evaluated by lane 0 against an overlay of at most 4 cells and broadcast as
//    uniform (row, column, value) edits that every lane applies to the rows it
//    loads -- the row loads are in flight while lane 0 works;
//  * lane = (strip, column group): 16 lanes span a 64-cell row (4 cells = 8 bytes
//    each, so a wave-wide load is four fully-used 128-byte row segments) and the 4
//    strips of 16 lanes each own H/4 consecutive rows;
//  * a row's 4 cells live packed two per 32-bit register (two uint16 halves), so
//    every bitwise op, v_bitop3, v_perm, v_pk_lshrrev_b16 and v_mul_u32_u24 below
//    evaluates the rule for 2 cells at once;
//  * horizontal neighbours: the 16-lane DPP rotations row_ror:1 / row_ror:15 wrap
//    exactly at W = 64 (the torus), so the left / right neighbour words cost one
//    DPP move each and three funnel shifts;
//  * vertical neighbours: each lane walks its strip top to bottom with a rolling
//    window of row summaries; rows are fetched UNR at a time, one chunk ahead;
//  * each row summary folds the 3 cells of a row into ones (OR), twos (>= 2,
//    majority) and a count; the column pass folds 3 row summaries the same way
//    (the reference's advance_board.c:12-32,51-86 does the
//    same separable fold cell by cell);
//  * spawner code lives in a second copy of the row loop and only runs for envs
//    whose level holds a spawning cell (sl_env_state.spawn_flags);
//  * scores are kept incrementally: points / perf score / possible / side-effect
//    totals change only where a cell changed, so the per-cell scoring work (an
//    LDS table lookup), the start-board read and the store are all skipped
//    (wave-uniformly) on rows where nothing changed.  The totals equal the full
//    sums the generic kernel computes (tests: test_fast_kernel_vs_generic).
#include "sl_action.h"

#pragma clang diagnostic ignored "-Wunneeded-internal-declaration"  // IMPL-specific helpers

using namespace sl;
using namespace sl::fast;

namespace {

constexpr uint32_t ONE2 = 0x00010001u;

#ifndef SL_FAST_UNR
#define SL_FAST_UNR 2      // rows per unrolled chunk of the 16-row strip
#endif
#ifndef SL_FAST_OCC
#define SL_FAST_OCC 4      // waves per SIMD the register budget is sized for
#endif
// timing-only ablations (results are wrong when set): 1 no score deltas,
// 2 no stores, 4 no rule (output = input)
#ifndef SL_FAST_ABL
#define SL_FAST_ABL 0
#endif
// 0: register-staged strips (4 envs per workgroup); 1: LDS-staged (1 env per workgroup);
// 2: bit-sliced columns (sl_bits.hip)
#ifndef SL_FAST_IMPL
#define SL_FAST_IMPL 2
#endif

__device__ __forceinline__ uint32_t pk_shr(uint32_t val, uint32_t amt) {
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    us2 v = __builtin_bit_cast(us2, val), s = __builtin_bit_cast(us2, amt);
    return __builtin_bit_cast(uint32_t, (us2)(v >> s));   // v_pk_lshrrev_b16
}

__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t x, uint32_t y) {
    return (m & x) | (~m & y);                            // v_bfi_b32 / v_bitop3
}

// 0xFFFF in every 16-bit half whose bit 0 (bit 16) is set: x is 0/1 per half
__device__ __forceinline__ uint32_t expand(uint32_t x) { return __umul24(x, 0xFFFFu); }

// lane (l - 1) mod 16 / (l + 1) mod 16 inside each 16-lane DPP row
__device__ __forceinline__ uint32_t from_left(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x121, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t from_right(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x12F, 0xF, 0xF, false);
}

struct CW {          // contribution words of a row pair-register
    uint32_t c, a, am;
};

// c(n) per cell (see sl_device.h): alive, P|I|S flags, alive destructible-or-exit +
// colours at bits 8-11, spawner colours at bits 13-15.
template <bool SPAWN>
__device__ __forceinline__ CW cword(uint32_t v) {
    CW r;
    r.a = v & ONE2;
    r.am = expand(r.a);
    const uint32_t t = ((v << 5) & 0x01000100u) | v;       // exit bit |= destructible
    uint32_t c = ((t & 0x0F000F00u) & r.am) | (v & 0x00E100E1u);
    if (SPAWN) {
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
template <bool SPAWN>
__device__ __forceinline__ uint32_t decide(uint32_t v, const CW &w, uint32_t oU, uint32_t tU,
                                           uint32_t nU, uint32_t oC, uint32_t tC, uint32_t nC,
                                           uint32_t oD, uint32_t tD, uint32_t nD,
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
    if (SPAWN) {
        *elig = (ones >> 7) & ~(hold | x | w.a) & ONE2;
        *spv = cols | 0x00090009u;
    } else {
        *elig = 0;
        *spv = 0;
    }
    return out;
}

__device__ __forceinline__ uint32_t spawn_pair(uint32_t o, uint32_t e, uint32_t sv, int cell,
                                               uint32_t gid, uint32_t step, uint32_t tensor,
                                               uint64_t seed, double thr) {
    if (e & 1u)
        if (philox_uniform((uint32_t)cell, gid, step, tensor, seed) < thr)
            o = (o & 0xFFFF0000u) | (sv & 0xFFFFu);
    if (e & 0x10000u)
        if (philox_uniform((uint32_t)cell + 1u, gid, step, tensor, seed) < thr)
            o = (o & 0x0000FFFFu) | (sv & 0xFFFF0000u);
    return o;
}

// score deltas of the 4 cells of a row that changed (board and/or goals)
__device__ __forceinline__ void delta_row(const ScoreTbl &tb, uint2 ob, uint2 nb, uint2 og,
                                          uint2 ng, uint2 s, int d[4]) {
    const uint32_t obw[2] = {ob.x, ob.y}, nbw[2] = {nb.x, nb.y};
    const uint32_t ogw[2] = {og.x, og.y}, ngw[2] = {ng.x, ng.y}, sw[2] = {s.x, s.y};
#pragma unroll
    for (int j = 0; j < 2; j++)
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int sh = 16 * h;
            const uint32_t o = (obw[j] >> sh) & 0xFFFF, n = (nbw[j] >> sh) & 0xFFFF;
            const uint32_t go = (ogw[j] >> sh) & 0xFFFF, gn = (ngw[j] >> sh) & 0xFFFF;
            const uint32_t sv = (sw[j] >> sh) & 0xFFFF;
            if (o != n || go != gn) {
                int p0, q0, r0, e0, p1, q1, r1, e1;
                cell_terms_lds(&tb, o, go, sv, &p0, &q0, &r0, &e0);
                cell_terms_lds(&tb, n, gn, sv, &p1, &q1, &r1, &e1);
                d[0] += p1 - p0;
                d[1] += q1 - q0;
                d[2] += r1 - r0;
                d[3] += e1 - e0;
            }
        }
}

__device__ __forceinline__ int wrap_row(int y, int H) { return y < 0 ? y + H : (y >= H ? y - H : y); }

// uniform cell edits broadcast from lane 0
struct Edits {
    int n;
    int y[4], cg[4], sh[4], j[4];
    uint32_t v[4];
    uint32_t rowmask;    // strip-relative row slots (0 .. R+1) that hold an edit
};

__device__ __forceinline__ uint2 patch(uint2 w, int y, int cg, const Edits &ed) {
    for (int k = 0; k < ed.n; k++) {
        if (y == ed.y[k] && cg == ed.cg[k]) {
            const uint32_t m = 0xFFFFu << ed.sh[k], nv = ed.v[k] << ed.sh[k];
            if (ed.j[k]) w.y = (w.y & ~m) | nv;
            else w.x = (w.x & ~m) | nv;
        }
    }
    return w;
}

__device__ __forceinline__ bool has_edit(int y, int cg, const Edits &ed) {
    bool h = false;
    for (int k = 0; k < ed.n; k++) h |= (y == ed.y[k] && cg == ed.cg[k]);
    return h;
}

// ---------------------------------------------------------------- row loop
struct Ctx {
    uint2 *gb, *gg;
    const uint2 *gs;
    int cg, y0;
    uint32_t gid, step;
    uint64_t seed;
    double thr;
};

template <int H, int UNR, bool SPAWN>
__device__ __forceinline__ void strip_loop(const Ctx &c, const Edits &ed, const ScoreTbl &tb,
                                           uint2 hb, uint2 hg, uint2 vb, uint2 vg, uint2 tb2,
                                           uint2 tg2, uint2 (&nxb)[UNR], uint2 (&nxg)[UNR],
                                           int d[4]) {
    constexpr int R = H / 4, RW = 16, NCH = R / UNR;
    const int cg = c.cg, y0 = c.y0;
    if (ed.rowmask & 1u) hb = patch(hb, wrap_row(y0 - 1, H), cg, ed);
    if (ed.rowmask & 2u) vb = patch(vb, y0, cg, ed);
    CW wb0 = cword<SPAWN>(hb.x), wb1 = cword<SPAWN>(hb.y);
    CW wg0 = cword<SPAWN>(hg.x), wg1 = cword<SPAWN>(hg.y);
    RowSum pb = row_sum(wb0.c, wb1.c), pg = row_sum(wg0.c, wg1.c);
    wb0 = cword<SPAWN>(vb.x); wb1 = cword<SPAWN>(vb.y);
    wg0 = cword<SPAWN>(vg.x); wg1 = cword<SPAWN>(vg.y);
    RowSum cb = row_sum(wb0.c, wb1.c), cgs = row_sum(wg0.c, wg1.c);

#pragma unroll 1
    for (int ch = 0; ch < NCH; ch++) {
        uint2 pfb[UNR], pfg[UNR];
        if (ch + 1 < NCH) {
#pragma unroll
            for (int j = 0; j < UNR; j++) {
                const int k = (ch + 1) * UNR + 1 + j;          // strip-relative row
                if (k < R) {
                    pfb[j] = c.gb[(y0 + k) * RW + cg];
                    pfg[j] = c.gg[(y0 + k) * RW + cg];
                } else {
                    pfb[j] = tb2;
                    pfg[j] = tg2;
                }
            }
        }
#pragma unroll
        for (int j = 0; j < UNR; j++) {
            const int r = ch * UNR + j;
            const int y = y0 + r;                              // centre row
            uint2 nb = nxb[j];
            if ((ed.rowmask >> (r + 2)) & 1u) nb = patch(nb, wrap_row(y + 1, H), cg, ed);
            const uint2 ng = nxg[j];
            const CW nb0w = cword<SPAWN>(nb.x), nb1w = cword<SPAWN>(nb.y);
            const CW ng0w = cword<SPAWN>(ng.x), ng1w = cword<SPAWN>(ng.y);
            const RowSum nbs = row_sum(nb0w.c, nb1w.c), ngs = row_sum(ng0w.c, ng1w.c);

            uint32_t e0, e1, e2, e3, s0, s1, s2, s3;
            uint32_t o0 = decide<SPAWN>(vb.x, wb0, pb.o0, pb.t0, pb.n0, cb.o0, cb.t0, cb.n0,
                                        nbs.o0, nbs.t0, nbs.n0, &e0, &s0);
            uint32_t o1 = decide<SPAWN>(vb.y, wb1, pb.o1, pb.t1, pb.n1, cb.o1, cb.t1, cb.n1,
                                        nbs.o1, nbs.t1, nbs.n1, &e1, &s1);
            uint32_t o2 = decide<SPAWN>(vg.x, wg0, pg.o0, pg.t0, pg.n0, cgs.o0, cgs.t0, cgs.n0,
                                        ngs.o0, ngs.t0, ngs.n0, &e2, &s2);
            uint32_t o3 = decide<SPAWN>(vg.y, wg1, pg.o1, pg.t1, pg.n1, cgs.o1, cgs.t1, cgs.n1,
                                        ngs.o1, ngs.t1, ngs.n1, &e3, &s3);
            if (SL_FAST_ABL & 4) {
                asm volatile("" :: "v"(o0), "v"(o1), "v"(o2), "v"(o3));
                o0 = vb.x; o1 = vb.y; o2 = vg.x; o3 = vg.y;
            }
            if (SPAWN) {
                const bool any_e = (e0 | e1 | e2 | e3) != 0;
                if (__ballot(any_e)) {
                    if (any_e) {
                        const int cell = y * 64 + cg * 4;
                        o0 = spawn_pair(o0, e0, s0, cell, c.gid, c.step, 0u, c.seed, c.thr);
                        o1 = spawn_pair(o1, e1, s1, cell + 2, c.gid, c.step, 0u, c.seed, c.thr);
                        o2 = spawn_pair(o2, e2, s2, cell, c.gid, c.step, 1u, c.seed, c.thr);
                        o3 = spawn_pair(o3, e3, s3, cell + 2, c.gid, c.step, 1u, c.seed, c.thr);
                    }
                }
            }
            // vb carries the action's edits; memory still holds the pre-action row, so
            // a row with an edit is written back even if the advance kept it
            const bool sc_b = ((o0 ^ vb.x) | (o1 ^ vb.y)) != 0;
            const bool sc_g = ((o2 ^ vg.x) | (o3 ^ vg.y)) != 0;
            const bool edited = ((ed.rowmask >> (r + 1)) & 1u) && has_edit(y, cg, ed);
            if (__ballot(sc_b || sc_g || edited)) {
                if (!(SL_FAST_ABL & 2)) {
                    if (sc_b || edited) c.gb[y * RW + cg] = make_uint2(o0, o1);
                    if (sc_g) c.gg[y * RW + cg] = make_uint2(o2, o3);
                }
                if (!(SL_FAST_ABL & 1) && (sc_b || sc_g))
                    delta_row(tb, vb, make_uint2(o0, o1), vg, make_uint2(o2, o3),
                              c.gs[y * RW + cg], d);
            }
            pb = cb; cb = nbs; pg = cgs; cgs = ngs;
            wb0 = nb0w; wb1 = nb1w; wg0 = ng0w; wg1 = ng1w;
            vb = nb; vg = ng;
        }
        if (ch + 1 < NCH) {
#pragma unroll
            for (int j = 0; j < UNR; j++) {
                nxb[j] = pfb[j];
                nxg[j] = pfg[j];
            }
        }
    }
}

// H: board height (W = 64); UNR: rows per unrolled chunk (divides H/4)
template <int H, int UNR>
__global__ void __launch_bounds__(256, SL_FAST_OCC)
k_env_step_w64(sl_env_state st, StepArgs a, const int32_t *__restrict__ actions, int ctp,
               int ctc, double *__restrict__ reward_out, uint8_t *__restrict__ done_out,
               uint8_t *__restrict__ flags_out, int32_t *__restrict__ ep_len_out,
               int32_t *__restrict__ ep_rew_out) {
    constexpr int R = H / 4;           // rows per strip
    constexpr int RW = 16;             // uint2 words per row
    static_assert(R % UNR == 0, "UNR must divide the strip height");
    __shared__ ScoreTbl tbl;
    if (threadIdx.x < 64) {
        const uint32_t g = threadIdx.x >> 3, cc = threadIdx.x & 7;
        const int t = point_value(g, cc);
        tbl.e[threadIdx.x] = (uint16_t)((t + 3) | ((sgn(t) + 1) << 4) | (possible_value(g) << 6));
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t b = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
    if (b >= st.B) return;             // whole wave leaves together
    const int cg = lane & 15;
    const int y0 = (lane >> 4) * R;
    const int64_t off = b * (int64_t)(H * 64);
    Ctx c;
    c.gb = reinterpret_cast<uint2 *>(st.board + off);
    c.gg = reinterpret_cast<uint2 *>(st.goals + off);
    c.gs = reinterpret_cast<const uint2 *>(st.start_board + off);
    c.cg = cg;
    c.y0 = y0;
    c.gid = a.env0 + (uint32_t)b;
    c.step = a.step;
    c.seed = a.seed;

    // -- rows needed before any store: halo above, first centre, halo below
    const int ybot = wrap_row(y0 + R, H);
    uint2 hb = c.gb[wrap_row(y0 - 1, H) * RW + cg], hg = c.gg[wrap_row(y0 - 1, H) * RW + cg];
    uint2 vb = c.gb[y0 * RW + cg], vg = c.gg[y0 * RW + cg];
    const uint2 tb2 = c.gb[ybot * RW + cg], tg2 = c.gg[ybot * RW + cg];
    uint2 nxb[UNR], nxg[UNR];
#pragma unroll
    for (int j = 0; j < UNR; j++) {
        if (1 + j < R) {
            nxb[j] = c.gb[(y0 + 1 + j) * RW + cg];
            nxg[j] = c.gg[(y0 + 1 + j) * RW + cg];
        } else {
            nxb[j] = tb2;
            nxg[j] = tg2;
        }
    }

    // -- the action, on lane 0 (its cell reads overlap the row loads above)
    ActResult ar{0, 0, 0, 0};
    Overlay ov;
    ov.src.bd = st.board + off;
    ov.n = 0;
    if (lane == 0) ar = lane_action(st, b, actions[b], ctp, ctc, &tbl, ov);
    Edits ed;
    ed.n = __builtin_amdgcn_readfirstlane(ov.n);
    ed.rowmask = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        ed.y[k] = ed.cg[k] = ed.j[k] = ed.sh[k] = 0;
        ed.v[k] = 0;
        if (k < ed.n) {
            const int i = __builtin_amdgcn_readfirstlane(ov.idx[k]);
            const int ey = i >> 6, ex = i & 63;
            ed.y[k] = ey;
            ed.cg[k] = ex >> 2;
            ed.j[k] = (ex >> 1) & 1;
            ed.sh[k] = 16 * (ex & 1);
            ed.v[k] = (uint32_t)__builtin_amdgcn_readfirstlane((int)ov.val[k]);
            const int r = ey % R;       // slot in its own strip, and the halo slots
            ed.rowmask |= 1u << (r + 1);
            if (r == R - 1) ed.rowmask |= 1u;          // halo above of the next strip
            if (r == 0) ed.rowmask |= 1u << (R + 1);  // halo below of the previous strip
        }
    }
    c.thr = (double)st.spawn_prob[b];

    int d[4] = {0, 0, 0, 0};           // d points, d score, d possible, d side
    if (st.spawn_flags[b])
        strip_loop<H, UNR, true>(c, ed, tbl, hb, hg, vb, vg, tb2, tg2, nxb, nxg, d);
    else
        strip_loop<H, UNR, false>(c, ed, tbl, hb, hg, vb, vg, tb2, tg2, nxb, nxg, d);
#pragma unroll
    for (int q = 0; q < 4; q++) d[q] = wave_sum(d[q]);
    // every row store of this wave lands before lane 0 recolours the exit cells
    __builtin_amdgcn_s_waitcnt(0);
    if (lane != 0) return;
    const int points = st.old_points[b] + ar.dp + d[0];
    const int score = st.score[b] + ar.dq + d[1];
    const int possible = st.possible[b] + d[2];
    const int side = st.side_effect[b] + ar.dse + d[3];
    env_epilogue(st, a, b, ar.reward, points, score, possible, side, reward_out, done_out,
                 flags_out, ep_len_out, ep_rew_out);
}

// ============================================================================
// LDS-staged variant: one env per 128-thread workgroup (2 waves x 4 strips of
// H/8 rows).  Each wave copies its half of the board and goals HBM -> LDS with
// global_load_lds_dwordx4 (16 KiB per env in flight at once, no VGPRs), the
// action is applied to the LDS copy and to memory by one lane, and the rows are
// then read from LDS (wrapped halo rows included) by a rolled loop -- small
// code, no register staging, every load of the env issued up front.
// ============================================================================
template <int H, int UNR, bool SPAWN>
__device__ __forceinline__ void strip_loop_lds(const Ctx &c, const uint2 *lb, const uint2 *lg,
                                               const ScoreTbl &tb, int R, int d[4]) {
    constexpr int RW = 16;
    const int cg = c.cg, y0 = c.y0;
    uint2 hb = lb[wrap_row(y0 - 1, H) * RW + cg], hg = lg[wrap_row(y0 - 1, H) * RW + cg];
    uint2 vb = lb[y0 * RW + cg], vg = lg[y0 * RW + cg];
    CW wb0 = cword<SPAWN>(hb.x), wb1 = cword<SPAWN>(hb.y);
    CW wg0 = cword<SPAWN>(hg.x), wg1 = cword<SPAWN>(hg.y);
    RowSum pb = row_sum(wb0.c, wb1.c), pg = row_sum(wg0.c, wg1.c);
    wb0 = cword<SPAWN>(vb.x); wb1 = cword<SPAWN>(vb.y);
    wg0 = cword<SPAWN>(vg.x); wg1 = cword<SPAWN>(vg.y);
    RowSum cb = row_sum(wb0.c, wb1.c), cgs = row_sum(wg0.c, wg1.c);
#pragma unroll UNR
    for (int r = 0; r < R; r++) {
        const int y = y0 + r;                              // centre row
        const int yn = wrap_row(y + 1, H);
        const uint2 nb = lb[yn * RW + cg], ng = lg[yn * RW + cg];
        const CW nb0w = cword<SPAWN>(nb.x), nb1w = cword<SPAWN>(nb.y);
        const CW ng0w = cword<SPAWN>(ng.x), ng1w = cword<SPAWN>(ng.y);
        const RowSum nbs = row_sum(nb0w.c, nb1w.c), ngs = row_sum(ng0w.c, ng1w.c);
        uint32_t e0, e1, e2, e3, s0, s1, s2, s3;
        uint32_t o0 = decide<SPAWN>(vb.x, wb0, pb.o0, pb.t0, pb.n0, cb.o0, cb.t0, cb.n0, nbs.o0,
                                    nbs.t0, nbs.n0, &e0, &s0);
        uint32_t o1 = decide<SPAWN>(vb.y, wb1, pb.o1, pb.t1, pb.n1, cb.o1, cb.t1, cb.n1, nbs.o1,
                                    nbs.t1, nbs.n1, &e1, &s1);
        uint32_t o2 = decide<SPAWN>(vg.x, wg0, pg.o0, pg.t0, pg.n0, cgs.o0, cgs.t0, cgs.n0,
                                    ngs.o0, ngs.t0, ngs.n0, &e2, &s2);
        uint32_t o3 = decide<SPAWN>(vg.y, wg1, pg.o1, pg.t1, pg.n1, cgs.o1, cgs.t1, cgs.n1,
                                    ngs.o1, ngs.t1, ngs.n1, &e3, &s3);
        if (SL_FAST_ABL & 4) {
            asm volatile("" :: "v"(o0), "v"(o1), "v"(o2), "v"(o3));
            o0 = vb.x; o1 = vb.y; o2 = vg.x; o3 = vg.y;
        }
        if (SPAWN) {
            const bool any_e = (e0 | e1 | e2 | e3) != 0;
            if (__ballot(any_e)) {
                if (any_e) {
                    const int cell = y * 64 + cg * 4;
                    o0 = spawn_pair(o0, e0, s0, cell, c.gid, c.step, 0u, c.seed, c.thr);
                    o1 = spawn_pair(o1, e1, s1, cell + 2, c.gid, c.step, 0u, c.seed, c.thr);
                    o2 = spawn_pair(o2, e2, s2, cell, c.gid, c.step, 1u, c.seed, c.thr);
                    o3 = spawn_pair(o3, e3, s3, cell + 2, c.gid, c.step, 1u, c.seed, c.thr);
                }
            }
        }
        const bool sc_b = ((o0 ^ vb.x) | (o1 ^ vb.y)) != 0;
        const bool sc_g = ((o2 ^ vg.x) | (o3 ^ vg.y)) != 0;
        if (__ballot(sc_b || sc_g)) {
            if (!(SL_FAST_ABL & 2)) {
                if (sc_b) c.gb[y * RW + cg] = make_uint2(o0, o1);
                if (sc_g) c.gg[y * RW + cg] = make_uint2(o2, o3);
            }
            if (!(SL_FAST_ABL & 1) && (sc_b || sc_g))
                delta_row(tb, vb, make_uint2(o0, o1), vg, make_uint2(o2, o3), c.gs[y * RW + cg],
                          d);
        }
        pb = cb; cb = nbs; pg = cgs; cgs = ngs;
        wb0 = nb0w; wb1 = nb1w; wg0 = ng0w; wg1 = ng1w;
        vb = nb; vg = ng;
    }
}

template <int H, int UNR>
__global__ void __launch_bounds__(128)
k_env_step_w64_lds(sl_env_state st, StepArgs a, const int32_t *__restrict__ actions, int ctp,
                   int ctc, double *__restrict__ reward_out, uint8_t *__restrict__ done_out,
                   uint8_t *__restrict__ flags_out, int32_t *__restrict__ ep_len_out,
                   int32_t *__restrict__ ep_rew_out) {
    constexpr int WPE = 2;                    // waves per env
    constexpr int R = H / (4 * WPE);          // rows per strip
    constexpr int HALF = H / WPE * 128;       // bytes of one wave's half board
    __shared__ __attribute__((aligned(16))) uint2 lbd[H * 16];
    __shared__ __attribute__((aligned(16))) uint2 lgd[H * 16];
    __shared__ ScoreTbl tbl;
    __shared__ int red[WPE][4];
    const int64_t b = blockIdx.x;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t off = b * (int64_t)(H * 64);
    {   // HBM -> LDS, this wave's half of board and goals, 1 KiB per instruction
        const char *sb = reinterpret_cast<const char *>(st.board + off) + wv * HALF;
        const char *sg = reinterpret_cast<const char *>(st.goals + off) + wv * HALF;
        char *db = reinterpret_cast<char *>(lbd) + wv * HALF;
        char *dg = reinterpret_cast<char *>(lgd) + wv * HALF;
#pragma unroll
        for (int k = 0; k < HALF / 1024; k++) {
            __builtin_amdgcn_global_load_lds((const void *)(sb + k * 1024 + lane * 16),
                                             (__attribute__((address_space(3))) void *)(db + k * 1024),
                                             16, 0, 0);
            __builtin_amdgcn_global_load_lds((const void *)(sg + k * 1024 + lane * 16),
                                             (__attribute__((address_space(3))) void *)(dg + k * 1024),
                                             16, 0, 0);
        }
    }
    if (threadIdx.x < 64) {
        const uint32_t g = threadIdx.x >> 3, cc = threadIdx.x & 7;
        const int t = point_value(g, cc);
        tbl.e[threadIdx.x] = (uint16_t)((t + 3) | ((sgn(t) + 1) << 4) | (possible_value(g) << 6));
    }
    // the action, on thread 0 (constant-memory score lookups: the LDS table is
    // not ready before the barrier), while the copies are in flight
    ActResult ar{0, 0, 0, 0};
    Overlay ov;
    ov.src.bd = st.board + off;
    ov.n = 0;
    if (threadIdx.x == 0) ar = lane_action(st, b, actions[b], ctp, ctc, nullptr, ov);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();                          // copies landed, table filled
    if (threadIdx.x == 0) {
        uint16_t *gbd = st.board + off;
        uint16_t *lb16 = reinterpret_cast<uint16_t *>(lbd);
        for (int k = 0; k < ov.n; k++) {
            lb16[ov.idx[k]] = (uint16_t)ov.val[k];
            gbd[ov.idx[k]] = (uint16_t)ov.val[k];
        }
    }
    __syncthreads();                          // edits visible in LDS, stored in memory
    Ctx c;
    c.gb = reinterpret_cast<uint2 *>(st.board + off);
    c.gg = reinterpret_cast<uint2 *>(st.goals + off);
    c.gs = reinterpret_cast<const uint2 *>(st.start_board + off);
    c.cg = lane & 15;
    c.y0 = (wv * 4 + (lane >> 4)) * R;
    c.gid = a.env0 + (uint32_t)b;
    c.step = a.step;
    c.seed = a.seed;
    c.thr = (double)st.spawn_prob[b];
    int d[4] = {0, 0, 0, 0};
    if (st.spawn_flags[b])
        strip_loop_lds<H, UNR, true>(c, lbd, lgd, tbl, R, d);
    else
        strip_loop_lds<H, UNR, false>(c, lbd, lgd, tbl, R, d);
#pragma unroll
    for (int q = 0; q < 4; q++) d[q] = wave_sum(d[q]);
    if (lane == 0)
        for (int q = 0; q < 4; q++) red[wv][q] = d[q];
    __syncthreads();                          // every row store of both waves is done
    if (threadIdx.x != 0) return;
    for (int q = 0; q < 4; q++) d[q] = red[0][q] + red[1][q];
    const int points = st.old_points[b] + ar.dp + d[0];
    const int score = st.score[b] + ar.dq + d[1];
    const int possible = st.possible[b] + d[2];
    const int side = st.side_effect[b] + ar.dse + d[3];
    env_epilogue(st, a, b, ar.reward, points, score, possible, side, reward_out, done_out,
                 flags_out, ep_len_out, ep_rew_out);
}

}  // namespace

namespace sl {

bool fast_shape(int H, int W) { return W == 64 && H == 64; }

bool launch_fast_fuses_reset(const sl_env_state &st, const FastExtra &fx) {
    (void)st;
    return SL_FAST_IMPL == 2 && fx.fuse_reset && fx.pool.K > 0;
}

// the 64x64 bit-sliced kernel writes packed observations itself (FastExtra.obs_out)
bool launch_fast_fuses_obs() { return SL_FAST_IMPL == 2; }

int launch_step_fast(const sl_env_state &st, const StepArgs &a, const FastExtra &fx,
                     const int32_t *actions, int ctp, int ctc, double *reward, uint8_t *done,
                     uint8_t *flags, int32_t *ep_len, int32_t *ep_rew, hipStream_t s) {
    if (!fast_shape(st.H, st.W)) return SL_ETOOBIG;
#if SL_FAST_IMPL == 2
    return launch_step_bits(st, a, fx, actions, ctp, ctc, reward, done, flags, ep_len, ep_rew, s);
#elif SL_FAST_IMPL == 1
    hipLaunchKernelGGL((k_env_step_w64_lds<64, SL_FAST_UNR>), dim3((unsigned)st.B), dim3(128), 0,
                       s, st, a, actions, ctp, ctc, reward, done, flags, ep_len, ep_rew);
#else
    const unsigned grid = (unsigned)((st.B + 3) / 4);
    hipLaunchKernelGGL((k_env_step_w64<64, SL_FAST_UNR>), dim3(grid), dim3(256), 0, s, st, a,
                       actions, ctp, ctc, reward, done, flags, ep_len, ep_rew);
#endif
    if (fx.ev_end) (void)hipEventRecord((hipEvent_t)fx.ev_end, s);
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}

}  // namespace sl
