// sl_device.h -- device-side building blocks shared by the gfx950 kernels.
//
// Cell bit layout: safelife_game.py:74-120 (constants.h:4-25 on the C side).
// The per-cell rule is SURVEY.md Appendix A, a restatement of
// speedups_src/advance_board.c:34-120: the neighbourhood is the wrapped 3x3
// block INCLUDING the cell, counted with multiplicity (H or W == 2 wrap onto
// the same cells twice, exactly as the reference's two 1-d passes do).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sl {

constexpr uint32_t ALIVE = 0x0001, AGENT = 0x0002, PUSHABLE = 0x0004, DESTR = 0x0008;
constexpr uint32_t FROZEN = 0x0010, PRESERVE = 0x0020, INHIBIT = 0x0040, SPAWN = 0x0080;
constexpr uint32_t EXIT = 0x0100, COLOR_R = 0x0200, COLOR_G = 0x0400, COLOR_B = 0x0800;
constexpr uint32_t COLORS = 0x0E00, PULLABLE = 0x8000;
constexpr uint32_t PLAYER = AGENT | INHIBIT | PRESERVE | FROZEN | DESTR;      // 122
constexpr uint32_t LEVEL_EXIT = FROZEN | EXIT;                               // 272
constexpr uint32_t LIFE = ALIVE | DESTR;                                     // 9
constexpr uint32_t MOVABLE = PUSHABLE | PULLABLE;
constexpr uint32_t POWERS = ALIVE | INHIBIT | PRESERVE | SPAWN;
// cell bits no cell type uses (safelife_game.py CellTypes); the 128x128 kernel keeps
// no start-board planes for them (spawn_flags bit 2 flags a start board that has them)
constexpr uint32_t kCellHiBits = 0x7000;
// the cell bits the 128x128 kernel's goal plane mirror holds (alive, destructible,
// frozen, colours); goals using any other bit set spawn_flags bit 3
constexpr uint32_t kGoalPlaneBits = ALIVE | DESTR | FROZEN | COLORS;

// ----------------------------------------------------------------------------
// Philox4x32-10, counter (c0..c3), key = seed.  Identical to oracle/sl_oracle.c.
// ----------------------------------------------------------------------------
__device__ __forceinline__ void philox4x32(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                           uint64_t seed, uint32_t out[4]) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    // two rounds per iteration (no register rotation moves); fully unrolled inside the
    // bit-sliced kernels' draw loops it cost the 64x64 kernel 64 spilled VGPRs.  Each
    // product is one v_mad_u64_u32 (hi and lo together; a v_mul_hi_u32 + v_mul_lo_u32
    // pair before: C5 1.169 -> 1.165 ms, tools/ab/c5_philox_mad.py)
#pragma unroll 2
    for (int r = 0; r < 10; r++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0;
    out[1] = c1;
    out[2] = c2;
    out[3] = c3;
}

// a uniform double in [0,1) with 53 random bits (numpy's construction) from one
// evaluation: level choices, rolls and action samples
__device__ __forceinline__ double philox_uniform(uint32_t c0, uint32_t c1, uint32_t c2,
                                                 uint32_t c3, uint64_t seed) {
    uint32_t x[4];
    philox4x32(c0, c1, c2, c3, seed, x);
    uint32_t a = x[0] >> 5, b = x[1] >> 6;
    return ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
}

// Philox-mode spawn draws (the build's own throughput RNG; the reference has only its
// global stream, replayed by SL_RNG_STREAM).  The four cells of the 2x2 block
// (y >> 1, x >> 1) share one evaluation, counter (block, env, step, tensor) with
// block = (y >> 1) * ceil(W / 2) + (x >> 1); cell (y, x) takes output word
// (y & 1) * 2 + (x & 1) as the uniform word * 2^-32 (exact in a double), so a
// clustered group of eligible cells costs a quarter of the Philox work.
__device__ __forceinline__ uint32_t spawn_block(int y, int x, int W) {
    return (uint32_t)((y >> 1) * ((W + 1) >> 1) + (x >> 1));
}
__device__ __forceinline__ double spawn_word_uniform(uint32_t w) {
    return (double)w * (1.0 / 4294967296.0);
}
__device__ __forceinline__ double spawn_uniform(int y, int x, int W, uint32_t env, uint32_t step,
                                                uint32_t tensor, uint64_t seed) {
    uint32_t r[4];
    philox4x32(spawn_block(y, x, W), env, step, tensor, seed, r);
    return spawn_word_uniform(r[(y & 1) * 2 + (x & 1)]);
}

// ----------------------------------------------------------------------------
// Per-cell rule over a board held in LDS (row-major, H x W, uint16).
//
// Each neighbour n contributes one word
//     c(n) = P|I|S flags (bits 5-7)
//          | (alive ? (destructible-or-exit)<<8 | colours : 0)   (bits 8-11)
//          | (spawner ? colours << 4 : 0)                         (bits 13-15)
// and the 3x3 block is folded into
//     ones = OR of c(n)          twos = bits set in >= 2 of the c(n)
// so  newborn colours = (twos | ones >> 4) & COLORS,
//     newborn destructible = twos bit 8.
// ----------------------------------------------------------------------------
struct CellNb {
    uint32_t ones, twos, cnt;
};

__device__ __forceinline__ uint32_t contrib(uint32_t v) {
    uint32_t alive = v & ALIVE;
    uint32_t f2 = (v | ((v & DESTR) << 5)) & (EXIT | COLORS);
    uint32_t c = v & (PRESERVE | INHIBIT | SPAWN);
    c |= alive ? f2 : 0u;
    c |= (v & SPAWN) ? ((v & COLORS) << 4) : 0u;
    return c;
}

__device__ __forceinline__ CellNb gather_lds(const uint16_t *b, int H, int W, int y, int x) {
    const int ym = (y == 0 ? H - 1 : y - 1) * W, y0 = y * W, yp = (y == H - 1 ? 0 : y + 1) * W;
    const int xm = x == 0 ? W - 1 : x - 1, xp = x == W - 1 ? 0 : x + 1;
    const int idx[9] = {ym + xm, ym + x, ym + xp, y0 + xm, y0 + x, y0 + xp,
                        yp + xm, yp + x, yp + xp};
    CellNb n{0u, 0u, 0u};
#pragma unroll
    for (int k = 0; k < 9; k++) {
        uint32_t v = b[idx[k]];
        uint32_t c = contrib(v);
        n.twos |= n.ones & c;
        n.ones |= c;
        n.cnt += v & ALIVE;
    }
    return n;
}

// Rule outcome for cell value v with neighbourhood n.
//   returns the new value assuming no spawn; *elig = the cell draws a uniform,
//   *spawn_val = the value if that draw spawns.
__device__ __forceinline__ uint32_t rule_cell(uint32_t v, const CellNb &n, bool *elig,
                                              uint32_t *spawn_val) {
    *elig = false;
    const uint32_t colors = (n.twos | (n.ones >> 4)) & COLORS;
    if (v & ALIVE) {
        bool keep = (v & FROZEN) || (n.ones & PRESERVE) || n.cnt == 3 || n.cnt == 4;
        return keep ? v : 0u;
    }
    if ((v & FROZEN) || (n.ones & INHIBIT)) return v;
    if (n.cnt == 3) return ALIVE | colors | ((n.twos & EXIT) >> 5);
    if (n.ones & SPAWN) {
        *elig = true;
        *spawn_val = ALIVE | DESTR | colors;
    }
    return v;
}

// ----------------------------------------------------------------------------
// Goal / score tables (safelife_game.py:554-565, 601-631) packed for lookup.
//   point_table[g][c] in {-3,-1,0,3,5}; sign table; max-of-sign row.
// ----------------------------------------------------------------------------
// rows: goal colour g (KRGYBMCW), columns: cell colour c.  Kept in constant memory
// (a per-lane indexed local array would live in scratch).
__constant__ int8_t kPointTable[64] = {
    0, -1, 0, 0, 0, 0, 0, 0,
    -3, 3, -3, 0, -3, 0, -3, -3,
    0, -3, 5, 0, 0, 0, 3, 0,
    -3, 0, 0, 3, 0, 0, 0, 0,
    3, -3, 3, 0, 5, 3, 3, 3,
    -3, 3, -3, 0, -3, 5, -3, -3,
    3, -3, 3, 0, 3, 0, 5, 3,
    0, -1, 0, 0, 0, 0, 0, 0};

__device__ __forceinline__ int point_value(uint32_t g, uint32_t c) {
    return kPointTable[(g << 3) | c];
}

__device__ __forceinline__ int sgn(int x) { return (x > 0) - (x < 0); }

// row maxima of sign(point_table): black and white goals 0, others +1
__device__ __forceinline__ int possible_value(uint32_t g) { return (g != 0 && g != 7) ? 1 : 0; }

// Per-cell contributions of (board cell b, goal cell g) to
//   points  = point_table[gc, bc] * alive
//   score   = sign(point_table)[gc, bc] * m,  m = alive & !(frozen & !movable)
//   possible= max(sign row)[gc]
__device__ __forceinline__ void cell_scores(uint32_t b, uint32_t g, int *pts, int *scr, int *pos) {
    uint32_t gc = (g & COLORS) >> 9, bc = (b & COLORS) >> 9;
    int t = point_value(gc, bc);
    bool alive = b & ALIVE;
    bool m = alive && ((b & (FROZEN | MOVABLE)) != FROZEN);
    *pts = alive ? t : 0;
    *scr = m ? sgn(t) : 0;
    *pos = possible_value(gc);
}

// SimpleSideEffectPenalty per-cell term (env_wrappers.py:326-342): 1 = side effect.
__device__ __forceinline__ int side_term(uint32_t b, uint32_t s, uint32_t g) {
    const uint32_t keep = 0xFFFFu & ~PLAYER;
    s &= keep;
    b = (s & EXIT) ? s : (b & keep);        // exits compare as their start value
    const uint32_t red_life = ALIVE | COLOR_R;
    bool start_red = (s & red_life) == red_life;
    bool end_red = (b & red_life) == red_life;
    bool goal_blue = (g & COLORS) == COLOR_B;
    bool end_alive = (b & red_life) == ALIVE;
    bool non_effect = (b == s) || (start_red && !end_red) || (goal_blue && end_alive);
    return non_effect ? 0 : 1;
}

// ----------------------------------------------------------------------------
// block helpers (256 threads = 4 waves of 64)
// ----------------------------------------------------------------------------
__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    return v;
}

}  // namespace sl
