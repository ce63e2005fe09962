// sl_bits.hip -- the bit-sliced fused env-step kernel for 64x64 boards.
//
// Same semantics as k_env_action + k_env_step_generic (sl_env.hip) and the
// packed fast kernel (sl_fast.hip); different data layout, chosen for CDNA4's
// VALU-issue limit:
//
//  * one wave64 per env; lane l owns the column pair (2j, 2j+1), j = l >> 1, for
//    the 32-row half h = l & 1 (rows 32h .. 32h+31);
//  * each lane loads its 32 dwords D[y] = cell(32h+y, 2j) | cell(32h+y, 2j+1) << 16
//    (every load instruction covers two full 128-byte rows) and transposes them in
//    registers (32x32 bit transpose: 2 v_perm stages + 3 bfi stages, 256 VALU
//    ops), giving 16 bit planes x 2 words: plane k, word w, bit y = bit k of
//    cell(32h + y, 2j + w);
//  * the rule (advance_board.c:34-120) is then evaluated as
//    bitwise logic on 32 cells per operation: vertical neighbours are funnel
//    shifts (v_alignbit) against the other half's word (DPP quad_perm lane swap),
//    horizontal neighbours are the lane's other word or a 2-lane whole-wave DPP
//    rotation (wave_ror:1 / wave_rol:1, wrapping at W = 64), the 3x3 alive count
//    is a bit-sliced adder and the >= 2 tests are majority functions -- about
//    120 VALU ops per 32 cells against ~1300 for the packed two-cells-per-register
//    form;
//  * points, performance score, possible score and side effects
//    (safelife_game.py:590-631, env_wrappers.py:319-342) are recomputed in full
//    every step from the new planes with bitwise masks and v_bcnt;
//  * the new planes are transposed back and only the rows that changed are
//    stored (a wave-wide OR of the per-column change masks picks them).
// The action (execute_action / move_agent, safelife_game.py:308-393) runs on lane
// 0 while the column loads are in flight; its cell edits are broadcast and
// written into the planes before the rule.  Envs that finish are queued; a second
// kernel (k_env_reset_list) resets exactly those, one wave each, so the step
// kernel carries no reset code (121 VGPRs, 4 waves/SIMD, no spills).
#include "sl_action.h"

using namespace sl;
using namespace sl::fast;

namespace {

typedef uint32_t u32;

#ifndef SL_BITS_WPB
#define SL_BITS_WPB 1        // envs (waves) per workgroup
#endif
#ifndef SL_BITS_UACT
#define SL_BITS_UACT 0       // 1: the action runs wave-uniform (scalar unit); 0: on lane 0
#endif
#ifndef SL_BITS_UEPI
#define SL_BITS_UEPI 0       // 1: the epilogue runs wave-uniform; 0: on lane 0
#endif
// timing-only ablations (results are wrong when set; never in the shipped build):
//   1 no goals rule, 2 no board rule, 4 no scoring, 8 no board row stores,
//   16 no action / epilogue
#ifndef SL_BITS_ABL
#define SL_BITS_ABL 0
#endif
#ifndef SL_BITS_MIRROR
#define SL_BITS_MIRROR 1     // keep / use the bit-plane mirror of the goals
#endif
#ifndef SL_BITS_MINW
#define SL_BITS_MINW 4       // waves per SIMD the register budget is sized for
#endif

constexpr int N = 64;        // rows = columns = lanes

// ---------------------------------------------------------------- primitives
__device__ __forceinline__ u32 maj(u32 a, u32 b, u32 c) { return (a & b) | (c & (a | b)); }
__device__ __forceinline__ u32 mux(u32 s, u32 a, u32 b) { return (s & a) | (~s & b); }

// whole-wave lane rotations (wrap at 64 lanes); every lane has a source, so no old value
__device__ __forceinline__ u32 lane_m1(u32 v) {      // value of lane l - 1
    return (u32)__builtin_amdgcn_mov_dpp((int)v, 0x13C, 0xF, 0xF, false);  // wave_ror:1
}
__device__ __forceinline__ u32 lane_p1(u32 v) {      // value of lane l + 1
    return (u32)__builtin_amdgcn_mov_dpp((int)v, 0x134, 0xF, 0xF, false);  // wave_rol:1
}
__device__ __forceinline__ u32 lane_x1(u32 v) {      // value of lane l ^ 1 (the other half)
    return (u32)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
}

// the three columns around each of the lane's two columns: word w of a plane is
// column 2j + w, so column 2j - 1 is word 1 of lane l - 2 and column 2j + 2 is
// word 0 of lane l + 2 (the same half; the 64-lane rotation wraps at W = 64)
struct H3 {
    u32 l0, r1;          // column 2j - 1, column 2j + 2
};
__device__ __forceinline__ H3 horiz(u32 w0, u32 w1) {
    return H3{lane_m1(lane_m1(w1)), lane_p1(lane_p1(w0))};
}

// rows y - 1 and y + 1 of a lane's 32-row word (the other half supplies the wrap)
struct V3 {
    u32 up, dn;
};
__device__ __forceinline__ V3 vert(u32 x) {
    const u32 o = lane_x1(x);
    return V3{__builtin_amdgcn_alignbit(x, o, 31u), __builtin_amdgcn_alignbit(o, x, 1u)};
}

template <int J, u32 M>
__device__ __forceinline__ void swap_stage(u32 A[32]) {
#pragma unroll
    for (int k = 0; k < 32; k++)
        if (!(k & J)) {
            const u32 a = A[k], b = A[k + J];
            A[k] = (M & a) | (~M & (b << J));
            A[k + J] = (M & (a >> J)) | (~M & b);
        }
}

// in-place 32x32 bit transpose: bit y of A'[c] = bit c of A[y] (an involution)
__device__ __forceinline__ void transpose32(u32 A[32]) {
#pragma unroll
    for (int k = 0; k < 16; k++) {      // 16-bit halves
        const u32 a = A[k], b = A[k + 16];
        A[k] = __builtin_amdgcn_perm(b, a, 0x05040100u);
        A[k + 16] = __builtin_amdgcn_perm(b, a, 0x07060302u);
    }
#pragma unroll
    for (int g = 0; g < 32; g += 16)    // bytes
#pragma unroll
        for (int k = g; k < g + 8; k++) {
            const u32 a = A[k], b = A[k + 8];
            A[k] = __builtin_amdgcn_perm(b, a, 0x06020400u);
            A[k + 8] = __builtin_amdgcn_perm(b, a, 0x07030501u);
        }
    swap_stage<4, 0x0F0F0F0Fu>(A);
    swap_stage<2, 0x33333333u>(A);
    swap_stage<1, 0x55555555u>(A);
}

// plane k, word w of a transposed column
#define PL(P, k, w) P[(k) + 16 * (w)]

// p points at the lane's first dword (row 32h, columns 2j, 2j+1); rows are 32 dwords
__device__ __forceinline__ void load_pairs(const u32 *__restrict__ p, u32 D[32]) {
#pragma unroll
    for (int y = 0; y < 32; y++) D[y] = p[y * 32];
}

template <int CTRL>
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
}

// ---------------------------------------------------------------- the rule
struct SpawnCtx {
    uint32_t gid, step;
    uint64_t seed;
    double thr;
};

// One CA step of the 64x64 column planes P (in place).  chg[w] = cells that changed.
// Appendix A: alive x survives iff frozen | P | cnt in {3,4}; dead x unless frozen | I
// is born iff cnt == 3 (colours: >= 2 alive of a colour, or any spawner of it;
// destructible: >= 2 alive destructible-or-exit), else spawns with probability p
// when a spawner is in the block.  Births and spawns clear every other bit.
// The spawner terms (spawner colours, the draws) are a second phase that only runs
// when the wave's planes hold a spawning cell, so the common path stays lean.
__device__ __forceinline__ void rule_planes(u32 P[32], u32 chg[2], int lane, const SpawnCtx &sc,
                                            u32 tensor) {
    // Each 3x3 quantity is folded vertically (rows y-1, y, y+1 of the lane's word)
    // and then horizontally (word 0 sees columns 2j-1, 2j, 2j+1; word 1 sees 2j,
    // 2j+1, 2j+2), one quantity at a time so only the reduced results stay live.
    u32 eq3[2], eq34[2];
    {   // 9-cell alive count: 3-row sums s = s0 + 2 s1, then t0 + 2h over 3 columns
        u32 s0[2], s1[2];
#pragma unroll
        for (int w = 0; w < 2; w++) {
            const u32 a = PL(P, 0, w);
            const V3 v = vert(a);
            s0[w] = v.up ^ a ^ v.dn;
            s1[w] = maj(v.up, a, v.dn);
        }
        const H3 h0 = horiz(s0[0], s0[1]), h1 = horiz(s1[0], s1[1]);
#pragma unroll
        for (int w = 0; w < 2; w++) {
            const u32 L0 = w ? s0[0] : h0.l0, R0 = w ? h0.r1 : s0[1];
            const u32 L1 = w ? s1[0] : h1.l0, R1 = w ? h1.r1 : s1[1];
            const u32 t0 = L0 ^ s0[w] ^ R0, c0 = maj(L0, s0[w], R0);
            const u32 a1 = L1 ^ s1[w] ^ R1, b1 = maj(L1, s1[w], R1);
            const u32 hh1 = ~b1 & (a1 ^ c0);                         // h == 1
            const u32 hh2 = (b1 & ~a1 & ~c0) | (~b1 & a1 & c0);      // h == 2
            eq3[w] = t0 & hh1;
            eq34[w] = mux(t0, hh1, hh2);
        }
    }
    // >= 2 of the 9 cells: alive & (destructible | exit), alive & colour k
    u32 two[4][2];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        u32 o[2], t[2];
#pragma unroll
        for (int w = 0; w < 2; w++) {
            const u32 a = PL(P, 0, w);
            const u32 x = q == 0 ? a & (PL(P, 3, w) | PL(P, 8, w)) : a & PL(P, 8 + q, w);
            const V3 v = vert(x);
            o[w] = v.up | x | v.dn;
            t[w] = maj(v.up, x, v.dn);
        }
        const H3 ho = horiz(o[0], o[1]), ht = horiz(t[0], t[1]);
        two[q][0] = ht.l0 | t[0] | t[1] | maj(ho.l0, o[0], o[1]);
        two[q][1] = t[0] | t[1] | ht.r1 | maj(o[0], o[1], ho.r1);
    }
    // any of the 9 cells: preserve, inhibit, spawn
    u32 any[3][2];
#pragma unroll
    for (int f = 0; f < 3; f++) {
        u32 o[2];
#pragma unroll
        for (int w = 0; w < 2; w++) {
            const u32 x = PL(P, 5 + f, w);
            const V3 v = vert(x);
            o[w] = v.up | x | v.dn;
        }
        const H3 h = horiz(o[0], o[1]);
        any[f][0] = h.l0 | o[0] | o[1];
        any[f][1] = o[0] | o[1] | h.r1;
    }
    u32 kill[2], birth[2], pairD[2], colk[3][2], elig[2];
#pragma unroll
    for (int w = 0; w < 2; w++) {
        const u32 A = PL(P, 0, w), F = PL(P, 4, w);
        kill[w] = A & ~(F | any[0][w] | eq34[w]);
        const u32 dead_ok = ~(A | F | any[1][w]);
        birth[w] = dead_ok & eq3[w];
        pairD[w] = two[0][w];
#pragma unroll
        for (int k = 0; k < 3; k++) colk[k][w] = two[1 + k][w];
        elig[w] = dead_ok & ~eq3[w] & any[2][w];
    }
    __builtin_amdgcn_sched_barrier(0);
    // ---- spawner phase: spawner colours reach every newborn; eligible cells draw
    u32 sp[2] = {0u, 0u};
    if (__ballot((PL(P, 7, 0) | PL(P, 7, 1)) != 0u) != 0ull) {     // 64-bit wave mask
        u32 vsc[3][2];
#pragma unroll
        for (int k = 0; k < 3; k++)
#pragma unroll
            for (int w = 0; w < 2; w++) {
                const u32 x = PL(P, 7, w) & PL(P, 9 + k, w);
                const V3 v = vert(x);
                vsc[k][w] = v.up | x | v.dn;
            }
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const H3 h = horiz(vsc[k][0], vsc[k][1]);
            colk[k][0] |= h.l0 | vsc[k][0] | vsc[k][1];
            colk[k][1] |= vsc[k][0] | vsc[k][1] | h.r1;
        }
        const int row0 = 32 * (lane & 1), col0 = 2 * (lane >> 1);
#pragma unroll
        for (int w = 0; w < 2; w++) {
            u32 e = elig[w], s = 0;
            while (e) {
                const int y = __builtin_ctz(e);
                e &= e - 1;
                const u32 cell = (u32)((row0 + y) * N + col0 + w);
                if (philox_uniform(cell, sc.gid, sc.step, tensor, sc.seed) < sc.thr) s |= 1u << y;
            }
            sp[w] = s;
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    // ---- new planes
#pragma unroll
    for (int w = 0; w < 2; w++) {
        const u32 c = kill[w] | birth[w] | sp[w];
        const u32 born = birth[w] | sp[w];
        chg[w] = c;
        PL(P, 0, w) ^= c;
        PL(P, 3, w) = mux(c, (birth[w] & pairD[w]) | sp[w], PL(P, 3, w));
#pragma unroll
        for (int k = 0; k < 3; k++) PL(P, 9 + k, w) = mux(c, born & colk[k][w], PL(P, 9 + k, w));
        PL(P, 1, w) &= ~c;
        PL(P, 2, w) &= ~c;
#pragma unroll
        for (int k = 4; k <= 8; k++) PL(P, k, w) &= ~c;
#pragma unroll
        for (int k = 12; k <= 15; k++) PL(P, k, w) &= ~c;
    }
}

// ---------------------------------------------------------------- scoring
// point_table (safelife_game.py:554-565) as compile-time column sets per value class
__host__ __device__ constexpr int pt_value(int g, int c) {
    constexpr int8_t t[64] = {0,  -1, 0,  0, 0,  0, 0,  0,  -3, 3,  -3, 0, -3, 0, -3, -3,
                              0,  -3, 5,  0, 0,  0, 3,  0,  -3, 0,  0,  3, 0,  0, 0,  0,
                              3,  -3, 3,  0, 5,  3, 3,  3,  -3, 3,  -3, 0, -3, 5, -3, -3,
                              3,  -3, 3,  0, 3,  0, 5,  3,  0,  -1, 0,  0, 0,  0, 0,  0};
    return t[g * 8 + c];
}
__host__ __device__ constexpr int pt_set(int g, int v) {
    int s = 0;
    for (int c = 0; c < 8; c++)
        if (pt_value(g, c) == v) s |= 1 << c;
    return s;
}

__device__ __forceinline__ u32 minterm(u32 c0, u32 c1, u32 c2, int i) {
    return ((i & 1) ? c0 : ~c0) & ((i & 2) ? c1 : ~c1) & ((i & 4) ? c2 : ~c2);
}
// cells whose colour index lies in the compile-time set s
__device__ __forceinline__ u32 colour_in(u32 c0, u32 c1, u32 c2, int s) {
    u32 r = 0;
#pragma unroll
    for (int i = 0; i < 8; i++)
        if ((s >> i) & 1) r |= minterm(c0, c1, c2, i);
    return r;
}

struct Totals {
    int points, score, possible, side;
};

// Full sums over the board (B: board planes, gc: goal colour planes, S: start-board planes):
//   points   = sum point_table[g, c] * alive                      (safelife_game.py:590-599)
//   score    = sum sign(point_table)[g, c] * m,  m = alive & !(frozen & !movable)  (:601-631)
//   possible = sum [g not in {black, white}]
//   side     = #cells that are a side effect                      (env_wrappers.py:326-342)
__device__ __forceinline__ void score_planes(const u32 B[32], const u32 gc[3][2], const u32 S[32],
                                             int *pts, int *scr, int *pos, int *side) {
    int p = 0, q = 0, r = 0, e = 0;
#pragma unroll
    for (int w = 0; w < 2; w++) {
        const u32 c0 = PL(B, 9, w), c1 = PL(B, 10, w), c2 = PL(B, 11, w);
        const u32 g0 = gc[0][w], g1 = gc[1][w], g2 = gc[2][w];
        u32 m5 = 0, m3 = 0, m1 = 0, mm3 = 0;
#pragma unroll
        for (int g = 0; g < 8; g++) {
            const u32 gm = minterm(g0, g1, g2, g);
            if (pt_set(g, 5)) m5 |= gm & colour_in(c0, c1, c2, pt_set(g, 5));
            if (pt_set(g, 3)) m3 |= gm & colour_in(c0, c1, c2, pt_set(g, 3));
            if (pt_set(g, -1)) m1 |= gm & colour_in(c0, c1, c2, pt_set(g, -1));
            if (pt_set(g, -3)) mm3 |= gm & colour_in(c0, c1, c2, pt_set(g, -3));
        }
        const u32 A = PL(B, 0, w);
        p += 5 * __builtin_popcount(A & m5) + 3 * __builtin_popcount(A & m3) -
             __builtin_popcount(A & m1) - 3 * __builtin_popcount(A & mm3);
        const u32 m = A & ~(PL(B, 4, w) & ~(PL(B, 2, w) | PL(B, 15, w)));
        q += __builtin_popcount(m & (m5 | m3)) - __builtin_popcount(m & (m1 | mm3));
        r += __builtin_popcount((g0 ^ g1) | (g0 ^ g2));
        // side effects: b, s without the player bits; exits compare equal
        u32 d = PL(B, 0, w) ^ PL(S, 0, w);
        d |= PL(B, 2, w) ^ PL(S, 2, w);
#pragma unroll
        for (int k = 7; k < 16; k++) d |= PL(B, k, w) ^ PL(S, k, w);
        const u32 start_red_gone = PL(S, 0, w) & PL(S, 9, w) & ~(PL(B, 0, w) & PL(B, 9, w));
        const u32 blue_goal_alive = g2 & ~g1 & ~g0 & PL(B, 0, w) & ~PL(B, 9, w);
        e += __builtin_popcount(d & ~PL(S, 8, w) & ~start_red_gone & ~blue_goal_alive);
    }
    *pts = p;
    *scr = q;
    *pos = r;
    *side = e;
}

// ---------------------------------------------------------------- stores
// the lane's rows y with bit y of rm set (both halves: rm is a wave-wide union) are
// written back, one dword (two cells) per lane
__device__ __forceinline__ void store_pairs(u32 *__restrict__ p, const u32 D[32], u32 rm) {
#pragma unroll
    for (int y = 0; y < 32; y++)
        if ((rm >> y) & 1u) p[y * 32] = D[y];
}

// ---------------------------------------------------------------- LDS staging
// A wave's 8 KiB LDS buffer holds one 64x64 board, row-major, with the 16-byte
// chunks of rows 32..63 rotated by 4 chunks so that the even (rows 0..31) and odd
// (rows 32..63) lanes of a column-pair read fall in different banks.
typedef __attribute__((address_space(3))) u32 lds_u32;

__device__ __forceinline__ void dma_board(const uint16_t *__restrict__ src, lds_u32 *buf,
                                          int lane) {
    const char *s = reinterpret_cast<const char *>(src);
#pragma unroll
    for (int k = 0; k < 8; k++) {          // 8 x (64 lanes x 16 B), LDS chunk q = 64k + lane
        const int q = k * 64 + lane, row = q >> 3, pos = q & 7;
        const int c = (pos - ((row >> 5) << 2)) & 7;
        __builtin_amdgcn_global_load_lds((const void *)(s + row * 128 + c * 16),
                                         (__attribute__((address_space(3))) void *)(buf + k * 256),
                                         16, 0, 0);
    }
}

// the lane's 32 dwords (rows 32h + y, column pair j) from the staged board
__device__ __forceinline__ void read_pairs(const lds_u32 *buf, int lane, u32 D[32]) {
    const int h = lane & 1, j = lane >> 1;
    const lds_u32 *p = buf + h * 1024 + ((j + 16 * h) & 31);
#pragma unroll
    for (int y = 0; y < 32; y++) D[y] = p[y * 32];
}

// The start-board planes the side-effect term needs (0, 2, 7-15), from the level
// pool's precomputed bit planes: the start board of an env reset from the pool is
// level li rolled by (dy, dx) (sl_env_state.start_roll).  Column c of the start
// board is level column c - dx; its 64-bit row column rotated by dy gives rows
// 32h .. 32h+31 as one funnel shift.  The pool stays in L2 / the Infinity Cache,
// so this costs no HBM traffic and no transpose.  The level's planes 0-3 and 6-15
// (7 KiB, seven 1 KiB DMA rows) are copied into the wave's board buffer as soon as
// the board has been read out of it, so their (queueing-dominated) latency runs
// under the action and the rule (issued at scoring time, it was ~40% of a wave's
// life; held in registers instead, it spills).
__device__ __forceinline__ void pool_dma(const sl_level_pool &pool, int li, lds_u32 *buf,
                                         int lane) {
    const char *pl = reinterpret_cast<const char *>(pool.board_planes + (int64_t)li * 16 * N);
#pragma unroll
    for (int k = 0; k < 7; k++) {       // LDS row k <- planes (0,1), (2,3), (6,7) .. (14,15)
        const int p0 = k < 2 ? 2 * k : 2 * k + 2;
        __builtin_amdgcn_global_load_lds((const void *)(pl + p0 * N * 8 + lane * 16),
                                         (__attribute__((address_space(3))) void *)(buf + k * 256),
                                         16, 0, 0);
    }
}
__device__ __forceinline__ void pool_planes_lds(const lds_u32 *buf, int dy, int dx, int lane,
                                                u32 S[32]) {
    const int c0 = (2 * (lane >> 1) - dx) & 63, c1 = (c0 + 1) & 63;
    const int r = (32 * (lane & 1) - dy) & 63;
    const bool lo_first = r < 32;
    const u32 sh = (u32)(r & 31);
#pragma unroll
    for (int p = 0; p < 16; p++) {
        if (p == 1 || (p >= 3 && p <= 6)) {
            PL(S, p, 0) = 0u;
            PL(S, p, 1) = 0u;
            continue;
        }
        const int slot = p < 4 ? p : p - 2;             // LDS plane slot
        const lds_u32 *q = buf + slot * 128;            // 64 columns x 2 dwords
        const u32 a0 = q[2 * c0], a1 = q[2 * c0 + 1], b0 = q[2 * c1], b1 = q[2 * c1 + 1];
        PL(S, p, 0) = lo_first ? __builtin_amdgcn_alignbit(a1, a0, sh)
                               : __builtin_amdgcn_alignbit(a0, a1, sh);
        PL(S, p, 1) = lo_first ? __builtin_amdgcn_alignbit(b1, b0, sh)
                               : __builtin_amdgcn_alignbit(b0, b1, sh);
    }
}

__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void wait_lgkm() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// ---------------------------------------------------------------- per-env record
// The per-env fields the action, the spawn/start terms and the epilogue read are
// fetched by ONE load instruction at kernel start: lane k of the record register
// holds dword k below, and every later read is a v_readlane.  The lane-0 action and
// epilogue then wait on no dependent HBM round trips (agent position -> cells,
// ring head -> ring entry -> bonus); before, those chains cost ~27% of the kernel.
enum : int {
    R_ACT = 0, R_GO, R_AX, R_AY, R_SCORE, R_BASE, R_POSS, R_SPAWN, R_ROLL, R_LI, R_OLDP,
    R_NSTEPS, R_EPLEN, R_EPREW, R_EXC, R_PLEN, R_PHEAD, R_SIDE, R_POK,
    R_MP = 19,           // min_performance, 2 dwords
    R_EY = 21,           // exit_y[8] (int16), 4 dwords
    R_EX = 25,           // exit_x[8], 4 dwords
    R_PX = 32,           // prior_x[16]
    R_PY = 48            // prior_y[16]
};

__device__ __forceinline__ u32 load_record(const sl_env_state &st, const int32_t *actions,
                                           int64_t b, int lane) {
    const char *p = reinterpret_cast<const char *>(st.game_over);      // spare lanes
    int64_t off = b * 4;
#define SL_SEL(k, ptr)                                                                    \
    if ((ptr) != nullptr) p = lane == (k) ? reinterpret_cast<const char *>(ptr) : p
    SL_SEL(R_ACT, actions);
    SL_SEL(R_AX, st.agent_x);
    SL_SEL(R_AY, st.agent_y);
    SL_SEL(R_SCORE, st.score);
    SL_SEL(R_BASE, st.baseline);
    SL_SEL(R_POSS, st.possible);
    SL_SEL(R_SPAWN, st.spawn_prob);
    SL_SEL(R_ROLL, st.start_roll);
    SL_SEL(R_LI, st.level_index);
    SL_SEL(R_OLDP, st.old_points);
    SL_SEL(R_NSTEPS, st.num_steps);
    SL_SEL(R_EPLEN, st.episode_length);
    SL_SEL(R_EPREW, st.episode_reward);
    SL_SEL(R_EXC, st.exit_count);
    SL_SEL(R_PLEN, st.prior_len);
    SL_SEL(R_PHEAD, st.prior_head);
    SL_SEL(R_SIDE, st.side_effect);
    SL_SEL(R_POK, st.planes_ok);
#undef SL_SEL
    if (lane >= R_MP && lane < R_MP + 2) {
        p = reinterpret_cast<const char *>(st.min_performance);
        off = b * 8 + 4 * (lane - R_MP);
    } else if (lane >= R_EY && lane < R_EY + 4) {
        p = reinterpret_cast<const char *>(st.exit_y);
        off = b * 16 + 4 * (lane - R_EY);
    } else if (lane >= R_EX && lane < R_EX + 4) {
        p = reinterpret_cast<const char *>(st.exit_x);
        off = b * 16 + 4 * (lane - R_EX);
    } else if (lane >= R_PX) {
        p = reinterpret_cast<const char *>(lane < R_PY ? st.prior_x : st.prior_y);
        off = b * 64 + 4 * ((lane - R_PX) & 15);
    }
    return *reinterpret_cast<const u32 *>(p + off);
}

__device__ __forceinline__ int rec(u32 V, int k) { return __builtin_amdgcn_readlane((int)V, k); }
__device__ __forceinline__ double rec_f64(u32 V, int k) {
    return __hiloint2double(rec(V, k + 1), rec(V, k));
}

// the action's view of the env: record fields in, state writes out
struct RecEnv {
    const sl_env_state &st;
    int64_t b;
    int go, ax, ay, score, base, poss;
    double mp;
    __device__ int game_over() const { return go; }
    __device__ int agent_x() const { return ax; }
    __device__ int agent_y() const { return ay; }
    __device__ bool can_exit() const { return can_exit_now(mp, score, base, poss); }
    __device__ void set_orientation(int o) { st.orientation[b] = o; }
    __device__ void set_game_over() {
        go = 1;
        st.game_over[b] = 1;
    }
    __device__ void set_agent(int x, int y) {
        ax = x;
        ay = y;
        st.agent_x[b] = x;
        st.agent_y[b] = y;
    }
};

// the epilogue's view (epilogue_core): record fields plus the post-action agent
struct RecFields {
    u32 V;
    int go, ax, ay;
    double bval;
    __device__ int old_points() const { return rec(V, R_OLDP); }
    __device__ int num_steps() const { return rec(V, R_NSTEPS); }
    __device__ int episode_length() const { return rec(V, R_EPLEN); }
    __device__ int episode_reward() const { return rec(V, R_EPREW); }
    __device__ double min_performance() const { return rec_f64(V, R_MP); }
    __device__ int baseline() const { return rec(V, R_BASE); }
    __device__ int exit_count() const { return rec(V, R_EXC); }
    __device__ int exit_y(int e) const {
        return (int)(int16_t)(rec(V, R_EY + (e >> 1)) >> (16 * (e & 1)));
    }
    __device__ int exit_x(int e) const {
        return (int)(int16_t)(rec(V, R_EX + (e >> 1)) >> (16 * (e & 1)));
    }
    __device__ int game_over() const { return go; }
    __device__ int agent_x() const { return ax; }
    __device__ int agent_y() const { return ay; }
    __device__ int prior_len() const { return rec(V, R_PLEN); }
    __device__ int prior_head() const { return rec(V, R_PHEAD); }
    __device__ int prior_x(int k) const { return rec(V, R_PX + k); }
    __device__ int prior_y(int k) const { return rec(V, R_PY + k); }
    __device__ int side_effect() const { return rec(V, R_SIDE); }
    __device__ double bonus(int) const { return bval; }
};

// unedited cells for the action, from the staged board (dma_board's layout)
typedef __attribute__((address_space(3))) const uint16_t lds_cu16;
struct LdsCells {
    const lds_u32 *buf;
    __device__ __forceinline__ uint32_t operator()(int i) const {
        const int row = i >> 6, col = i & 63;
        const int pos = ((col >> 3) + ((row >> 5) << 2)) & 7;
        return reinterpret_cast<lds_cu16 *>(buf)[row * 64 + pos * 8 + (col & 7)];
    }
};

// SafeLifeEnv.reset (safelife_env.py:188-198) of env b by one wave, right after the
// step that finished the episode (ContinuingEnv + run_agents' reset-on-done).
// Same result as reset_one (sl_env.hip): the rolled level is copied into board,
// goals and start board; points, perf baseline and possible are the bit-sliced sums
// over it; the exit list is collected row by row in np.nonzero order.
__device__ __forceinline__ void wave_reset(const sl_env_state &st, const sl_level_pool &pool,
                                        const ResetArgs &ra, int64_t b, int lane) {
    int li = 0, dy = 0, dx = 0;
    if (lane == 0) {
        const LevelChoice c = choose_level(pool, ra, ra.env0 + (uint32_t)b, st.episodes[b], N, N);
        li = c.idx;
        dy = c.dy;
        dx = c.dx;
    }
    li = __builtin_amdgcn_readfirstlane(li);
    dy = __builtin_amdgcn_readfirstlane(dy);
    dx = __builtin_amdgcn_readfirstlane(dx);
    const int h = lane & 1, j = lane >> 1;
    const uint16_t *lb = pool.board + (int64_t)li * (N * N), *lg = pool.goals + (int64_t)li * (N * N);
    const int c0 = (2 * j - dx) & 63, c1 = (2 * j + 1 - dx) & 63;
    const int64_t off = b * (int64_t)(N * N);
    const int lane_off = h * 1024 + j;
    u32 *gs = reinterpret_cast<u32 *>(st.start_board + off) + lane_off;
    u32 *gg = reinterpret_cast<u32 *>(st.goals + off) + lane_off;
    u32 *gb = reinterpret_cast<u32 *>(st.board + off) + lane_off;
    // the lane's 32 dwords of a rolled pool level (all gathers in flight at once:
    // this runs in its own kernel, registers are plentiful)
    auto rolled = [&](const uint16_t *lv, u32 D[32]) {
#pragma unroll
        for (int y = 0; y < 32; y++) {
            const int sr = ((32 * h + y - dy) & 63) * N;
            D[y] = (u32)lv[sr + c0] | ((u32)lv[sr + c1] << 16);
        }
    };
    // goals: copy, then keep their colour planes for the sums
    u32 P[32];
    rolled(lg, P);
#pragma unroll
    for (int y = 0; y < 32; y++) gg[y * 32] = P[y];
    transpose32(P);
    u32 *mg = (SL_BITS_MIRROR && st.planes) ? st.planes + b * 4096 + 2048 + lane : nullptr;
    if (mg) {      // the goals' bit-plane mirror
#pragma unroll
        for (int q = 0; q < 32; q++) mg[q * 64] = P[q];
    }
    u32 gcol[3][2];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        gcol[k][0] = PL(P, 9 + k, 0);
        gcol[k][1] = PL(P, 9 + k, 1);
    }
    const bool sg = __ballot((PL(P, 7, 0) | PL(P, 7, 1)) != 0u) != 0ull;
    // start board: copy, then the sums over the initial board and goals
    rolled(lb, P);
#pragma unroll
    for (int y = 0; y < 32; y++) gs[y * 32] = P[y];
    transpose32(P);
    int pts, scr, pos, side;
    score_planes(P, gcol, P, &pts, &scr, &pos, &side);
    const int s1 = wave_total((pts + 192) | ((scr + 64) << 16));
    const int s2 = wave_total(pos);
    const bool sb = __ballot((PL(P, 7, 0) | PL(P, 7, 1)) != 0u) != 0ull;
    int ev = 0;
    if (lane == 0)
        ev = reset_scalars(st, pool, ra, b, li, dy, dx, (s1 & 0xFFFF) - 192 * 64,
                           ((s1 >> 16) & 0xFFFF) - 64 * 64, s2, (sb ? 1 : 0) | (sg ? 2 : 0));
    ev = __builtin_amdgcn_readfirstlane(ev);
    const u32 ex0 = PL(P, 8, 0), ex1 = PL(P, 8, 1);       // exit planes
    // the board: the start board with its exits coloured (update_exit_colors)
    {
        u32 D[32];
        rolled(lb, D);
#pragma unroll
        for (int y = 0; y < 32; y++) {
            u32 d = D[y];
            if (d & (u32)EXIT) d = (d & 0xFFFF0000u) | (u32)ev;
            if (d & ((u32)EXIT << 16)) d = (d & 0x0000FFFFu) | ((u32)ev << 16);
            gb[y * 32] = d;
        }
    }
    // exits in np.nonzero (row-major) order: repeatedly take the wave-wide smallest
    // key row * 64 + column among the lanes' remaining exit bits (one round per exit)
    const int n_exit = wave_total(__builtin_popcount(ex0) + __builtin_popcount(ex1));
    {
        u32 e0 = ex0, e1 = ex1;
        const int kmax = n_exit < SL_MAX_EXITS ? n_exit : SL_MAX_EXITS;   // uniform
        for (int k = 0; k < kmax; k++) {
            const u32 k0 = e0 ? (u32)((32 * h + __builtin_ctz(e0)) * N + 2 * j) : 0xFFFFu;
            const u32 k1 = e1 ? (u32)((32 * h + __builtin_ctz(e1)) * N + 2 * j + 1) : 0xFFFFu;
            u32 m = k0 < k1 ? k0 : k1;
            m = min(m, dpp<0xB1>(m));
            m = min(m, dpp<0x4E>(m));
            m = min(m, dpp<0x141>(m));
            m = min(m, dpp<0x140>(m));
            const u32 key = min(min((u32)__builtin_amdgcn_readlane((int)m, 0),
                                    (u32)__builtin_amdgcn_readlane((int)m, 16)),
                                min((u32)__builtin_amdgcn_readlane((int)m, 32),
                                    (u32)__builtin_amdgcn_readlane((int)m, 48)));
            if (k0 == key) e0 &= e0 - 1;
            if (k1 == key) e1 &= e1 - 1;
            if (lane == 0) {
                st.exit_y[b * SL_MAX_EXITS + k] = (int16_t)(key >> 6);
                st.exit_x[b * SL_MAX_EXITS + k] = (int16_t)(key & 63);
            }
        }
    }
    if (lane == 0) {
        if (mg) st.planes_ok[b] = 2;   // after reset_scalars cleared it
        st.exit_count[b] = n_exit;
        for (int e = n_exit; e < SL_MAX_EXITS; e++) {
            st.exit_y[b * SL_MAX_EXITS + e] = 0;
            st.exit_x[b * SL_MAX_EXITS + e] = 0;
        }
    }
}

__device__ __forceinline__ void step_env(const sl_env_state &st, const StepArgs &a,
                                         const FastExtra &fx, int64_t b, int lane, lds_u32 *buf,
                                         const int32_t *__restrict__ actions, int ctp, int ctc,
                                         double *reward_out, uint8_t *done_out,
                                         uint8_t *flags_out, int32_t *ep_len_out,
                                         int32_t *ep_rew_out) {
    const int64_t off = b * (int64_t)(N * N);
    const int lane_off = (lane & 1) * 1024 + (lane >> 1);     // dwords: row 32h, column pair j
    u32 *gb = reinterpret_cast<u32 *>(st.board + off) + lane_off;
    u32 *gg = reinterpret_cast<u32 *>(st.goals + off) + lane_off;
    // bit-plane mirrors (sl_env_state.planes): read instead of u16 + transpose when valid
    // goals mirror, word-major: word q of lane l at planes[b*4096 + 2048 + q*64 + l]
    // (the goals rarely change, so it saves their transpose at almost no write cost;
    // a board mirror would be rewritten every step and does not pay)
    u32 *mg = (SL_BITS_MIRROR && st.planes) ? st.planes + b * 4096 + 2048 + lane : nullptr;
    const u32 V = load_record(st, actions, b, lane);           // issued first
    dma_board(st.board + off, buf, lane);                       // board cells -> LDS
    // goals: a goals board without spawners that came through a step unchanged is at
    // a fixed point of the (then deterministic) rule and never changes again
    // (planes_ok bit 2); such envs read only the three colour planes of the mirror,
    // which are speculatively in flight before the record says which case holds
    u32 gcol[3][2];                    // goal colour planes, kept for the scores
    if (mg) {
#pragma unroll
        for (int k = 0; k < 3; k++) {
            gcol[k][0] = mg[(9 + k) * 64];
            gcol[k][1] = mg[(25 + k) * 64];
        }
    }
    const int pok = (mg && st.planes_ok) ? rec(V, R_POK) & 6 : 0;

    SpawnCtx sc;
    sc.gid = a.env0 + (uint32_t)b;
    sc.step = a.step;
    sc.seed = a.seed;
    sc.thr = (double)__int_as_float(rec(V, R_SPAWN));

    // ---- goals
    if ((pok & 6) != 6) {
        u32 PG[32];
        if (pok & 2) {
#pragma unroll
            for (int q = 0; q < 32; q++) PG[q] = mg[q * 64];    // goal planes
        } else {
            load_pairs(gg, PG);                                 // goal cells
            transpose32(PG);
        }
        u32 cg[2];
        if (SL_BITS_ABL & 1) { cg[0] = cg[1] = 0; asm volatile("" : "+v"(PG[0])); }
        else rule_planes(PG, cg, lane, sc, 1u);
        const u32 rg = wave_or(cg[0] | cg[1]);
        if (mg) {      // mirror: the words whose 32 cells changed (all of them if rebuilt)
            const bool all = !(pok & 2);
#pragma unroll
            for (int w = 0; w < 2; w++)
                if (all || cg[w])
#pragma unroll
                    for (int k = 0; k < 16; k++) mg[(k + 16 * w) * 64] = PL(PG, k, w);
            const bool fixed = rg == 0 && __ballot((PL(PG, 7, 0) | PL(PG, 7, 1)) != 0u) == 0ull;
            const int ok = 2 | (fixed ? 4 : 0);
            if (ok != pok && lane == 0) st.planes_ok[b] = ok;
        }
#pragma unroll
        for (int k = 0; k < 3; k++) {
            gcol[k][0] = PL(PG, 9 + k, 0);
            gcol[k][1] = PL(PG, 9 + k, 1);
        }
        if (rg) {
            transpose32(PG);
            store_pairs(gg, PG, rg);
        }
    }
    __builtin_amdgcn_sched_barrier(0);

    // ---- board: from LDS; the start board comes from the level pool (cache) when
    // the env was reset from it, else from HBM through the same LDS buffer
    int roll = -1;
    if (fx.pool.K > 0 && fx.pool.board_planes && st.start_roll) roll = rec(V, R_ROLL);
    wait_vm();

    // the action (lane 0), on the staged board and the record
    OverlayT<LdsCells> ov;
    ov.src.buf = buf;
    ov.n = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        ov.idx[k] = 0;
        ov.val[k] = 0;
    }
    RecEnv env{st, b, rec(V, R_GO), rec(V, R_AX), rec(V, R_AY), rec(V, R_SCORE),
               rec(V, R_BASE), rec(V, R_POSS), rec_f64(V, R_MP)};
    int act_reward = 0;
    if (!(SL_BITS_ABL & 16) && (SL_BITS_UACT || lane == 0))
        act_reward = act_core(env, rec(V, R_ACT), N, N, ctp, ctc, ov);
    act_reward = __builtin_amdgcn_readfirstlane(act_reward);
    const int ne = __builtin_amdgcn_readfirstlane(ov.n);
    int eidx[4];
    u32 eval[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        eidx[k] = __builtin_amdgcn_readfirstlane(ov.idx[k]);
        eval[k] = (u32)__builtin_amdgcn_readfirstlane((int)ov.val[k]);
    }
    RecFields fl{V, __builtin_amdgcn_readfirstlane(env.go), __builtin_amdgcn_readfirstlane(env.ax),
                 __builtin_amdgcn_readfirstlane(env.ay), 0.0};
    if (a.bonus_period > 0)        // issued now, consumed by the epilogue
        fl.bval = a.bonus_table[bonus_dist(fl.ax, fl.ay, fl.prior_x(fl.prior_head()),
                                           fl.prior_y(fl.prior_head()), fl.prior_len(),
                                           a.bonus_period, a.bonus_len)];

    u32 PB[32];
    read_pairs(buf, lane, PB);
    wait_lgkm();
    if (roll < 0) dma_board(st.start_board + off, buf, lane);
    else pool_dma(fx.pool, rec(V, R_LI), buf, lane);
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
    }
    u32 cb[2];
    if (SL_BITS_ABL & 2) { cb[0] = PB[0] & 1; cb[1] = 0; }
    else rule_planes(PB, cb, lane, sc, 0u);
    __builtin_amdgcn_sched_barrier(0);

    // ---- scores over the new board and goals
    u32 PS[32];
    wait_vm();
    if (roll >= 0) {
        pool_planes_lds(buf, roll >> 16, roll & 0xFFFF, lane, PS);
    } else {
        read_pairs(buf, lane, PS);
        transpose32(PS);
    }
    int pts, scr, pos, side;
    if (SL_BITS_ABL & 4) { pts = PB[3] & 3; scr = PS[5] & 1; pos = gcol[0][1] & 1; side = 0; }
    else score_planes(PB, gcol, PS, &pts, &scr, &pos, &side);
    // totals (packed two per word: per-lane ranges [-192, 320] and [-64, 64]);
    // reduced before the board store so the scoring is not sunk past it
    const int s1 = wave_total((pts + 192) | ((scr + 64) << 16));
    const int s2 = wave_total(pos | (side << 16));
    __builtin_amdgcn_sched_barrier(0);

    // ---- write back the changed rows of the board, exits already in the colour the
    // epilogue gives them (update_exit_colors), so its exit writes and these row
    // stores carry the same values and need no ordering
    const int points = (s1 & 0xFFFF) - 192 * 64;
    const int score = ((s1 >> 16) & 0xFFFF) - 64 * 64;
    const int possible = s2 & 0xFFFF;
    const int side_total = (s2 >> 16) & 0xFFFF;
    const u32 rb = wave_or(cb[0] | cb[1]) | erow;
    if (rb && !(SL_BITS_ABL & 8)) {
        const bool can = can_exit_now(fl.min_performance(), score, fl.baseline(), possible);
#pragma unroll
        for (int w = 0; w < 2; w++)
            PL(PB, 9, w) = can ? (PL(PB, 9, w) | PL(PB, 8, w)) : (PL(PB, 9, w) & ~PL(PB, 8, w));
        transpose32(PB);
        store_pairs(gb, PB, rb);
    }
    int reset = 0;
    if (!(SL_BITS_ABL & 16) && (SL_BITS_UEPI || lane == 0))
        reset = epilogue_core(st, a, b, fl, act_reward, points, score, possible, side_total,
                              reward_out, done_out, flags_out, ep_len_out, ep_rew_out);
    reset = __builtin_amdgcn_readfirstlane(reset);
    if (fx.fuse_reset && reset && lane == 0) {
        // queue the env for the reset kernel (k_env_reset_list)
        int64_t *cnt = fx.scratch + 8 * st.B + 2 + (a.step & 1);
        const int i = (int)atomicAdd((unsigned long long *)cnt, 1ull);
        reinterpret_cast<int32_t *>(fx.scratch + 2 * st.B)[i] = (int32_t)b;
    }
}

__global__ void __launch_bounds__(64 * SL_BITS_WPB, SL_BITS_MINW)
k_env_step_bits64(sl_env_state st, StepArgs a, FastExtra fx, const int32_t *__restrict__ actions, int ctp,
                  int ctc, double *__restrict__ reward_out, uint8_t *__restrict__ done_out,
                  uint8_t *__restrict__ flags_out, int32_t *__restrict__ ep_len_out,
                  int32_t *__restrict__ ep_rew_out) {
    const int64_t b = (int64_t)blockIdx.x * SL_BITS_WPB +
                      __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    __shared__ __attribute__((aligned(16))) u32 stage[SL_BITS_WPB][N * N / 2];
    if (b >= st.B) return;                 // whole waves only
    lds_u32 *buf = (lds_u32 *)&stage[threadIdx.x >> 6][0];
    step_env(st, a, fx, b, lane, buf, actions, ctp, ctc, reward_out, done_out, flags_out,
             ep_len_out, ep_rew_out);
}

// Resets the envs the step kernel queued (one wave per env, grid-stride over the
// list).  Also zeroes the other step parity's list length for the next step.
__global__ void __launch_bounds__(64)
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

namespace sl {

int launch_step_bits(const sl_env_state &st, const StepArgs &a, const FastExtra &fx,
                     const int32_t *actions, int ctp, int ctc, double *reward, uint8_t *done,
                     uint8_t *flags, int32_t *ep_len, int32_t *ep_rew, hipStream_t s) {
    if (st.H != N || st.W != N) return SL_ETOOBIG;
    const unsigned grid = (unsigned)((st.B + SL_BITS_WPB - 1) / SL_BITS_WPB);
    hipLaunchKernelGGL(k_env_step_bits64, dim3(grid), dim3(64 * SL_BITS_WPB), 0, s, st, a, fx,
                       actions, ctp, ctc, reward, done, flags, ep_len, ep_rew);
    if (hipGetLastError() != hipSuccess) return SL_EHIP;
    if (fx.fuse_reset && fx.pool.K > 0) {
        const unsigned grid = (unsigned)(st.B < 512 ? st.B : 512);
        hipLaunchKernelGGL(k_env_reset_list, dim3(grid), dim3(64), 0, s, st, fx.pool, fx.ra,
                           fx.scratch, a.step);
    }
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}

}  // namespace sl
