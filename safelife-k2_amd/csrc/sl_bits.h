// sl_bits.h -- building blocks of the bit-sliced env-step kernels (sl_bits.hip for
// 64x64 boards, sl_bits128.hip for 128x128 boards).
//
// A lane holds two board columns over 32 rows as 16 bit planes x 2 words: plane k,
// word w, bit y = bit k of cell(row0 + y, col0 + w) (PL(P, k, w) below).  The rule
// (advance_board.c:34-120) and the scores are then bitwise
// logic on 32 cells per VALU op.  How the 3x3 neighbourhood of a word is formed
// depends on how the board is spread over the wave, so the rule takes a geometry
// policy:
//   g.vert(P, w, f)  rows y-1 / y+1 of the quantity f(P, w) (a bitwise function of
//                    the planes), including the rows just outside the word;
//   g.horiz(w0, w1)  columns col0-1 / col0+2 of a per-word quantity;
//   g.halo_spawn()   a spawner sits in a row just outside the wave's words;
//   g.block(y)       the 2x2 spawn block holding rows y, y + 1 of the lane's two
//                    columns (the Philox counter of their draws, spawn_uniform);
//   g.spawn(...)     the spawns among the eligible cells (SPAWN_PHILOX / _STREAM /
//                    _COUNT below).
#pragma once
#include "sl_action.h"


namespace sl {
namespace bits {

typedef uint32_t u32;

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
__device__ __forceinline__ u32 lane_x1(u32 v) {      // value of lane l ^ 1
    return (u32)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
}

struct H3 {
    u32 l0, r1;          // column col0 - 1, column col0 + 2
};
struct V3 {
    u32 up, dn;          // rows y - 1, y + 1
};
// o: bit 31 = the row above the word's row 0, bit 0 = the row below its row 31
__device__ __forceinline__ V3 vert_with(u32 x, u32 o) {
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

// plane k, word w of a transposed column pair
#define PL(P, k, w) P[(k) + 16 * (w)]

// a lane's 32 dwords, row stride S dwords (p points at its first one)
template <int S>
__device__ __forceinline__ void load_pairs(const u32 *__restrict__ p, u32 D[32]) {
#pragma unroll
    for (int y = 0; y < 32; y++) D[y] = p[y * S];
}
// the same with the nontemporal cache policy (state read once per step)
template <int S>
__device__ __forceinline__ void load_pairs_nt(const u32 *__restrict__ p, u32 D[32]) {
#pragma unroll
    for (int y = 0; y < 32; y++) D[y] = __builtin_nontemporal_load(p + y * S);
}

template <int CTRL>
__device__ __forceinline__ u32 dpp(u32 v) {
    return (u32)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}

// Row masks (bit y) of the 64-byte sectors to write when lanes 16k .. 16k+15 hold
// consecutive dwords of a row (the 128x128 layout): a lane's changed rows ORed over
// its 16-lane DPP row.  Whole sectors are written, so HBM sees no partial bursts.
__device__ __forceinline__ u32 sector_rows(u32 m) {
    m |= dpp<0xB1>(m);     // quad_perm [1,0,3,2]
    m |= dpp<0x4E>(m);     // quad_perm [2,3,0,1]
    m |= dpp<0x141>(m);    // row_half_mirror
    m |= dpp<0x140>(m);    // row_mirror
    return m;
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

// this lane's index, recomputed where it is used (v_mbcnt): the asm keeps the compiler
// from hoisting it, and every address derived from it, out of a loop and holding them
// (or spilling them) through it; two VALU per use against a register held throughout
__device__ __forceinline__ int lane_now() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void wait_lgkm() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// ---------------------------------------------------------------- the rule
struct SpawnCtx {
    uint32_t gid, step;
    uint64_t seed;
    double thr;
    uint32_t lim;      // Philox compare limit, ceil(thr * 2^32) - 1 (set_spawn_prob)
};
// thr = (double)(float)p, the reference's compare (advance_board.c:109-113), and its
// integer form for 32-bit Philox words: word * 2^-32 < thr  <=>  word <= lim (0 < thr <
// 1; both exact).  Computed once per env, wave-uniform, so the draws hold no double.
__device__ __forceinline__ void set_spawn_prob(SpawnCtx &sc, float p) {
    sc.thr = (double)p;
    sc.lim = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(ceil(sc.thr * 4294967296.0) - 1.0));
}

// How a geometry draws the spawns of its eligible cells (Geo::spawn):
//   SPAWN_PHILOX  Philox keyed by (cell, env, step, tensor): no ordering needed;
//   SPAWN_STREAM  the reference's order (SL_RNG_STREAM): a tensor's eligible cells take
//                 consecutive uniforms of a supplied stream, row-major (stream_draws);
//   SPAWN_COUNT   no draws: only count the eligible cells (the replay prologue kernels
//                 that size each tensor's slice of the stream);
//   SPAWN_DECIDED the reference's order, drawn before the step by a kernel of its own
//                 (128x128: k_stream_draw128): the geometry holds the spawning cells.
enum : int { SPAWN_PHILOX = 0, SPAWN_STREAM = 1, SPAWN_COUNT = 2, SPAWN_DECIDED = 3 };

// the supplied stream (StepArgs draws / n_draws) and the error word (scratch[8B])
struct StreamSrc {
    const double *draws;
    int64_t n;
    int64_t *err;
    int64_t mask = -1;      // StepArgs::draw_mask
    const uint32_t *bits = nullptr;   // StepArgs::draw_bits
};

// Philox spawn draws of the eligible cells elig[w] (bit y of word w), per lane: the
// lane's two columns over rows y, y + 1 (y even) are one 2x2 block, one Philox
// evaluation (spawn_uniform, sl_device.h).  sp[w] gets the eligible cells whose
// uniform is below the threshold.  A wave takes as many evaluations as its busiest
// lane has blocks holding an eligible cell (the words' rows start at an even row).
template <class Geo>
__device__ __forceinline__ void lane_draws(const Geo &g, const u32 elig[2], u32 sp[2],
                                           const SpawnCtx &sc, u32 tensor) {
    const u32 lim = sc.lim;
    const u32 any = elig[0] | elig[1];
    u32 blocks = (any | (any >> 1)) & 0x55555555u, s0 = 0u, s1 = 0u;
    while (blocks) {
        const int y = __builtin_ctz(blocks);
        blocks &= blocks - 1;
        uint32_t r[4];
        philox4x32(g.block(y), sc.gid, sc.step, tensor, sc.seed, r);
        s0 |= ((r[0] <= lim ? 1u : 0u) | (r[2] <= lim ? 2u : 0u)) << y;
        s1 |= ((r[1] <= lim ? 1u : 0u) | (r[3] <= lim ? 2u : 0u)) << y;
    }
    sp[0] = s0 & elig[0];
    sp[1] = s1 & elig[1];
}
template <class Geo>
__device__ __forceinline__ void philox_spawn(const Geo &g, const u32 elig[2], u32 sp[2],
                                             const SpawnCtx &sc, u32 tensor) {
    if (sc.thr <= 0.0) {                         // u < p never holds
    } else if (sc.thr >= 1.0) {                  // u < p always holds
        sp[0] = elig[0];
        sp[1] = elig[1];
    } else {
        lane_draws(g, elig, sp, sc, tensor);
    }
}

// number of set bits of m in the lanes below this one
__device__ __forceinline__ int lanes_below(uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0u));
}

typedef __attribute__((address_space(3))) uint16_t lds_u16;
// LDS slots compact_draws needs: one per 2x2 block a wave can hold (64 lanes x 16)
constexpr int kDrawSlots = 1024;

// The same draws as lane_draws, with the wave's eligible blocks spread over all its
// lanes.  Spawning cells cluster round the spawners, so a few lanes hold most blocks
// and lane_draws runs as many Philox evaluations as the busiest lane has blocks
// (C5 steady state: 28 per env-step) while the other lanes idle; here the wave runs
// ceil(blocks / 64) (C5: 10).  Each lane queues its blocks as (lane, y / 2) in the
// LDS slots from its exclusive prefix (the counts' bits by ballot + v_mbcnt), lane i
// of round r evaluates slot 64 r + i (the block number from Geo::block_of) and writes
// its four compare bits into the slot's top nibble, and the owner reads them back.
// The wave is the whole workgroup; LDS operations of one wave execute in order.
template <class Geo>
__device__ __forceinline__ void compact_draws(const Geo &g, const u32 elig[2], u32 sp[2],
                                              const SpawnCtx &sc, u32 tensor, lds_u16 *slots) {
    const u32 lim = sc.lim;
    const u32 any = elig[0] | elig[1];
    const u32 blocks = (any | (any >> 1)) & 0x55555555u;
    const int cnt = __builtin_popcount(blocks);
    int pre = 0, total = 0;
#pragma unroll
    for (int bit = 0; bit < 5; bit++) {         // cnt <= 16
        const uint64_t m = __ballot((cnt >> bit) & 1);
        pre += lanes_below(m) << bit;
        total += __builtin_popcountll(m) << bit;
    }
    const int lane = (int)__lane_id();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");     // the last call's reads
    __builtin_amdgcn_wave_barrier();
    {
        u32 m = blocks;
        int k = pre;
        while (m) {
            const int y = __builtin_ctz(m);
            m &= m - 1;
            slots[k++] = (uint16_t)((lane << 4) | (y >> 1));
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll 1
    for (int base = 0; base < total; base += 64) {
        const int i = base + lane;
        if (i < total) {
            const u32 it = slots[i];
            uint32_t r[4];
            philox4x32(g.block_of((int)(it >> 4), (int)(it & 15u) << 1), sc.gid, sc.step, tensor,
                       sc.seed, r);
            const u32 res = (r[0] <= lim ? 1u : 0u) | (r[1] <= lim ? 2u : 0u) |
                            (r[2] <= lim ? 4u : 0u) | (r[3] <= lim ? 8u : 0u);
            slots[i] = (uint16_t)(it | (res << 12));
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    u32 s0 = 0u, s1 = 0u;
    {
        u32 m = blocks;
        int k = pre;
        while (m) {
            const int y = __builtin_ctz(m);
            m &= m - 1;
            const u32 res = (u32)slots[k++] >> 12;
            s0 |= ((res & 1u) | ((res >> 1) & 2u)) << y;      // r[0]: row y, r[2]: row y + 1
            s1 |= (((res >> 1) & 1u) | ((res >> 2) & 2u)) << y;
        }
    }
    sp[0] = s0 & elig[0];
    sp[1] = s1 & elig[1];
}
template <class Geo>
__device__ __forceinline__ void philox_spawn_compact(const Geo &g, const u32 elig[2], u32 sp[2],
                                                     const SpawnCtx &sc, u32 tensor,
                                                     lds_u16 *slots) {
    if (sc.thr <= 0.0) {
    } else if (sc.thr >= 1.0) {
        sp[0] = elig[0];
        sp[1] = elig[1];
    } else {
        compact_draws(g, elig, sp, sc, tensor, slots);
    }
}

// Reference-order draws (SL_RNG_STREAM; random.c:47-52 consumed by advance_board.c:
// 109-113): the eligible cells of a tensor take the uniforms draws[pos], draws[pos+1],
// ... in row-major order -- one per eligible cell whatever p is -- and spawn iff
// u < (double)(float)p.  Row bit y of word w of a lane is cell (row, 2j + w); the
// cells before it are those of the earlier rows, those of lower lanes holding the
// same row, and for w = 1 the lane's own word 0.  Rows are visited four at a time:
// per row one ballot per word gives the row's eligible lanes (v_mbcnt counts the lower
// ones), then the four rows' loads are issued together.  SPLIT: even lanes hold rows
// y and odd lanes rows 32 + y (the 64x64 layout); else every lane holds row y.
// Returns the number of uniforms the words consumed (wave-uniform).
template <bool SPLIT>
__device__ __forceinline__ int stream_draws(const u32 elig[2], u32 sp[2], double thr,
                                            const StreamSrc &src, int64_t pos, int lane) {
    constexpr uint64_t even = 0x5555555555555555ull;
    const bool odd = SPLIT && (lane & 1);
    const uint64_t grp = SPLIT ? (odd ? ~even : even) : ~0ull;
    const int own = __builtin_popcount(elig[0]) + __builtin_popcount(elig[1]);
    sp[0] = 0u;
    sp[1] = 0u;
    if (thr <= 0.0 || thr >= 1.0) {              // the draws are consumed, never compared
        if (thr >= 1.0) {
            sp[0] = elig[0];
            sp[1] = elig[1];
        }
        return wave_total(own);
    }
    const int first = SPLIT ? wave_total(odd ? 0 : own) : 0;     // cells in rows 0..31
    const u32 rows = wave_or(elig[0] | elig[1]);
    int pre_a = 0, pre_b = 0;       // eligible cells of the visited rows (even / odd lanes)
#pragma unroll
    for (int c = 0; c < 32; c += 4) {
        if (((rows >> c) & 0xFu) == 0u) continue;
        int64_t r[4][2];
        bool e[4][2];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int y = c + k;
            e[k][0] = (elig[0] >> y) & 1u;
            e[k][1] = (elig[1] >> y) & 1u;
            const uint64_t m0 = __ballot(e[k][0]), m1 = __ballot(e[k][1]);
            const int64_t at = pos + (odd ? first + pre_b : pre_a) + lanes_below(m0 & grp) +
                               lanes_below(m1 & grp);
            r[k][0] = at;
            r[k][1] = at + (e[k][0] ? 1 : 0);
            if (SPLIT) {
                pre_a += __builtin_popcountll(m0 & even) + __builtin_popcountll(m1 & even);
                pre_b += __builtin_popcountll(m0 & ~even) + __builtin_popcountll(m1 & ~even);
            } else {
                pre_a += __builtin_popcountll(m0) + __builtin_popcountll(m1);
            }
        }
        double u[4][2];
#pragma unroll
        for (int k = 0; k < 4; k++)
#pragma unroll
            for (int w = 0; w < 2; w++)
                u[k][w] = (e[k][w] && r[k][w] < src.n)
                              ? stream_u(src.draws, src.bits, r[k][w], src.mask) : 1.0;
#pragma unroll
        for (int k = 0; k < 4; k++)
#pragma unroll
            for (int w = 0; w < 2; w++) {
                if (e[k][w] && r[k][w] >= src.n) atomicOr((unsigned long long *)src.err, 1ull);
                if (e[k][w] && u[k][w] < thr) sp[w] |= 1u << (c + k);
            }
    }
    return pre_a + pre_b;
}

// One CA step of the planes P (in place).  chg[w] = cells that changed.
// Appendix A: alive x survives iff frozen | P | cnt in {3,4}; dead x unless frozen | I
// is born iff cnt == 3 (colours: >= 2 alive of a colour, or any spawner of it;
// destructible: >= 2 alive destructible-or-exit), else spawns with probability p
// when a spawner is in the block.  Births and spawns clear every other bit.
// The spawner terms (spawner colours, the draws) are a second phase that only runs
// when the wave's planes (or halo rows) hold a spawning cell, so the common path
// stays lean.  Each 3x3 quantity is folded vertically (rows y-1, y, y+1) and then
// horizontally (word 0 sees columns col0-1 .. col0+1; word 1 sees col0 .. col0+2),
// one quantity at a time so only the reduced results stay live.
// held (optional): the changed cells that held a bit of a plane other than 0, 3, 9-11
// before the step (the planes a change clears but never sets), for plane-mode stores
template <class Geo>
__device__ __forceinline__ void rule_planes(u32 P[32], u32 chg[2], Geo &&g, const SpawnCtx &sc,
                                            u32 tensor, u32 *held = nullptr) {
    u32 eq3[2], eq34[2];
    {   // 9-cell alive count: 3-row sums s = s0 + 2 s1, then t0 + 2h over 3 columns
        u32 s0[2], s1[2];
#pragma unroll
        for (int w = 0; w < 2; w++) {
            const u32 a = PL(P, 0, w);
            const V3 v = g.vert(P, w, [](const auto &Q, int ww) { return PL(Q, 0, ww); });
            s0[w] = v.up ^ a ^ v.dn;
            s1[w] = maj(v.up, a, v.dn);
        }
        const H3 h0 = g.horiz(s0[0], s0[1]), h1 = g.horiz(s1[0], s1[1]);
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
        const auto f = [q](const auto &Q, int ww) {
            const u32 a = PL(Q, 0, ww);
            return q == 0 ? a & (PL(Q, 3, ww) | PL(Q, 8, ww)) : a & PL(Q, 8 + q, ww);
        };
        u32 o[2], t[2];
#pragma unroll
        for (int w = 0; w < 2; w++) {
            const u32 x = f(P, w);
            const V3 v = g.vert(P, w, f);
            o[w] = v.up | x | v.dn;
            t[w] = maj(v.up, x, v.dn);
        }
        const H3 ho = g.horiz(o[0], o[1]), ht = g.horiz(t[0], t[1]);
        two[q][0] = ht.l0 | t[0] | t[1] | maj(ho.l0, o[0], o[1]);
        two[q][1] = t[0] | t[1] | ht.r1 | maj(o[0], o[1], ho.r1);
    }
    // any of the 9 cells: preserve, inhibit, spawn
    u32 any[3][2];
#pragma unroll
    for (int fl = 0; fl < 3; fl++) {
        u32 o[2];
#pragma unroll
        for (int w = 0; w < 2; w++) {
            const u32 x = PL(P, 5 + fl, w);
            const V3 v = g.vert(P, w, [fl](const auto &Q, int ww) { return PL(Q, 5 + fl, ww); });
            o[w] = v.up | x | v.dn;
        }
        const H3 h = g.horiz(o[0], o[1]);
        any[fl][0] = h.l0 | o[0] | o[1];
        any[fl][1] = o[0] | o[1] | h.r1;
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
    if (__ballot((PL(P, 7, 0) | PL(P, 7, 1)) != 0u || g.halo_spawn()) != 0ull) {
        u32 vsc[3][2];
#pragma unroll
        for (int k = 0; k < 3; k++)
#pragma unroll
            for (int w = 0; w < 2; w++) {
                const auto f = [k](const auto &Q, int ww) { return PL(Q, 7, ww) & PL(Q, 9 + k, ww); };
                const u32 x = f(P, w);
                const V3 v = g.vert(P, w, f);
                vsc[k][w] = v.up | x | v.dn;
            }
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const H3 h = g.horiz(vsc[k][0], vsc[k][1]);
            colk[k][0] |= h.l0 | vsc[k][0] | vsc[k][1];
            colk[k][1] |= vsc[k][0] | vsc[k][1] | h.r1;
        }
        g.spawn(elig, sp, sc, tensor);
    }
    __builtin_amdgcn_sched_barrier(0);
    // ---- new planes
#pragma unroll
    for (int w = 0; w < 2; w++) {
        const u32 c = kill[w] | birth[w] | sp[w];
        const u32 born = birth[w] | sp[w];
        chg[w] = c;
        if (held) {
            u32 o = PL(P, 1, w) | PL(P, 2, w);
#pragma unroll
            for (int k = 4; k <= 8; k++) o |= PL(P, k, w);
#pragma unroll
            for (int k = 12; k <= 15; k++) o |= PL(P, k, w);
            held[w] = o & c;
        }
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

// Full sums over the words (B: board planes, gc: goal colour planes, S: start-board planes):
//   points   = sum point_table[g, c] * alive                      (safelife_game.py:590-599)
//   score    = sum sign(point_table)[g, c] * m,  m = alive & !(frozen & !movable)  (:601-631)
//   possible = sum [g not in {black, white}]
//   side     = #cells that are a side effect                      (env_wrappers.py:326-342)
// GC_IN_B: the goal colour planes are B's planes 12-14 (the fused-view kernel puts
// them there when the board's own bits 12-14 are all clear, so those bits count as 0
// in the side-effect compare; white goals may be cleared: rows black and white of the
// point table are equal, and neither counts as possible); gc is then not read.
template <bool GC_IN_B = false>
__device__ __forceinline__ void score_planes(const u32 B[32], const u32 gc[3][2], const u32 S[32],
                                             int *pts, int *scr, int *pos, int *side) {
    int p = 0, q = 0, r = 0, e = 0;
#pragma unroll
    for (int w = 0; w < 2; w++) {
        const u32 c0 = PL(B, 9, w), c1 = PL(B, 10, w), c2 = PL(B, 11, w);
        const u32 g0 = GC_IN_B ? PL(B, 12, w) : gc[0][w];
        const u32 g1 = GC_IN_B ? PL(B, 13, w) : gc[1][w];
        const u32 g2 = GC_IN_B ? PL(B, 14, w) : gc[2][w];
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
        for (int k = 7; k < 16; k++)
            d |= ((GC_IN_B && k >= 12 && k <= 14) ? 0u : PL(B, k, w)) ^ PL(S, k, w);
        const u32 start_red_gone = PL(S, 0, w) & PL(S, 9, w) & ~(PL(B, 0, w) & PL(B, 9, w));
        const u32 blue_goal_alive = g2 & ~g1 & ~g0 & PL(B, 0, w) & ~PL(B, 9, w);
        e += __builtin_popcount(d & ~PL(S, 8, w) & ~start_red_gone & ~blue_goal_alive);
    }
    *pts = p;
    *scr = q;
    *pos = r;
    *side = e;
}

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
    R_SPF = 29,          // spawn_flags: bit0 the board, bit1 the goals may hold a spawner
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
    SL_SEL(R_SPF, st.spawn_flags);
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

}  // namespace bits
}  // namespace sl
