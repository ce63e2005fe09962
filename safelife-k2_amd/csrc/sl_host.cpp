// sl_host.cpp -- the host (CPU) advance of one board, for numpy callers of
// speedups.advance_board ("numpy in -> host path").  The
// reference's numpy callers -- side_effects.py:136-139 (2 000+ advances per episode),
// proc_gen.py:382,625 -- hand it single small boards on the CPU, where one device
// round trip (~70 us) costs far more than the work.
//
// The decision of every cell is bit-sliced, as in the device kernels (sl_bits.h
// rule_planes), laid out for a 64-bit CPU: a board row of W cells is NW = ceil(W / 64)
// uint64 words per bit plane, bit x of word x / 64 = cell x.  The 3x3 neighbourhood
// (with multiplicity when H or W is 2) is a horizontal pass per row -- words rotated
// by one cell with the wrap at W -- then a vertical pass over rows y - 1, y, y + 1
// (mod H), as advance_board.c:34-120 combines rows, then columns.  Only five planes
// decide (alive, frozen, preserving, inhibiting, spawning): a live cell dies unless it
// is frozen, next to a preserver or has 3 or 4 live cells among its 9 (itself
// included); a dead cell that is not frozen or next to an inhibitor is born with
// exactly 3, else, next to a spawner, draws a uniform and spawns if u < (double)(float)p
// (advance_board.c:88-119).  Only changed cells are rewritten; the others are
// copied, as the reference copies them.  The new cell's destructible and colour bits
// come from pairs of live neighbours (and spawners' colours), which only a born cell
// needs: those are read from its 3x3 cells directly (born_value), not bit-sliced for
// the whole board.  Draws are taken in row-major order from the caller's uniforms,
// one per eligible cell.
//
// Plane extraction uses AVX-512BW (one vptestmw per 32 cells and plane) where the CPU
// has it, else a scalar loop.
#include <stdint.h>
#include <string.h>
#include <vector>
#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace {

typedef uint64_t u64;

// cell bits (constants.h)
enum { ALIVE = 1, DESTRUCTIBLE = 8, FROZEN = 16, PRESERVING = 32, INHIBITING = 64,
       SPAWNING = 128, EXIT = 256, COLORS = 7 << 9 };
// the deciding planes, in this order
enum { PA, PF, PP, PI, PS, NPL };
static const int PLANE_BIT[NPL] = {0, 4, 5, 6, 7};

inline u64 maj(u64 a, u64 b, u64 c) { return (a & b) | (c & (a | b)); }
inline u64 mux(u64 s, u64 a, u64 b) { return (s & a) | (~s & b); }

// One row of W cells as NW words.  lft: the value of cell x - 1 at x; rgt: of x + 1
// (both wrap at W).  Bits >= W of the last word stay 0.
template <int NW>
struct RowOps {
    u64 last_mask;      // valid bits of the last word
    int top;            // bit index of cell W - 1 within the last word
    inline void lft(const u64 *r, u64 *o) const {
        const u64 wrap = (r[NW - 1] >> top) & 1u;
        for (int i = NW - 1; i > 0; i--) o[i] = (r[i] << 1) | (r[i - 1] >> 63);
        o[0] = (r[0] << 1) | wrap;
        o[NW - 1] &= last_mask;
    }
    inline void rgt(const u64 *r, u64 *o) const {
        const u64 wrap = r[0] & 1u;
        for (int i = 0; i < NW - 1; i++) o[i] = (r[i] >> 1) | (r[i + 1] << 63);
        o[NW - 1] = (r[NW - 1] >> 1) | (wrap << top);
    }
};

template <int NW>
inline void extract_row_scalar(const uint16_t *row, int W, u64 (*pl)[NW]) {
    for (int k = 0; k < NPL; k++)
        for (int i = 0; i < NW; i++) pl[k][i] = 0;
    for (int x = 0; x < W; x++) {
        const unsigned c = row[x];
        if (!(c & 0xF1u)) continue;
        const int i = x >> 6;
        const u64 b = (u64)1 << (x & 63);
        for (int k = 0; k < NPL; k++)
            if (c & (1u << PLANE_BIT[k])) pl[k][i] |= b;
    }
}

#if defined(__x86_64__)
template <int NW>
__attribute__((target("avx512bw,avx512f,avx512vl")))
void extract_board_avx512(const uint16_t *b, int H, int W, u64 (*pl)[NPL][NW]) {
    const int nchunk = (W + 31) >> 5;
    const int tail = W - 32 * (nchunk - 1);
    const __mmask32 tail_mask = tail >= 32 ? 0xFFFFFFFFu : ((1u << tail) - 1u);
    __m512i bit[NPL];
    for (int k = 0; k < NPL; k++) bit[k] = _mm512_set1_epi16((short)(1 << PLANE_BIT[k]));
    for (int y = 0; y < H; y++) {
        const uint16_t *row = b + (size_t)y * W;
        u64 (*p)[NW] = pl[y];
        for (int k = 0; k < NPL; k++)
            for (int i = 0; i < NW; i++) p[k][i] = 0;
        for (int c = 0; c < nchunk; c++) {
            const __mmask32 m = c == nchunk - 1 ? tail_mask : 0xFFFFFFFFu;
            const __m512i v = _mm512_maskz_loadu_epi16(m, row + 32 * c);
            const int sh = 32 * (c & 1);
            for (int k = 0; k < NPL; k++)
                p[k][c >> 1] |= (u64)_mm512_test_epi16_mask(v, bit[k]) << sh;
        }
    }
}
static const bool HAVE_AVX512BW = __builtin_cpu_supports("avx512bw") &&
                                  __builtin_cpu_supports("avx512vl");
#else
static const bool HAVE_AVX512BW = false;
#endif

static thread_local std::vector<u64> g_scratch;

// The horizontal quantities of one row (NH of them, NW words each).
enum { HS0, HS1,            // alive: 3-cell sum bit 0, bit 1
       HP, HI, HSP,         // preserving, inhibiting, spawning: any of 3
       NH };

// The new value of a cell born (spawned: `spawned`) at (y, x), from its 9 cells of
// the old board, each counted as often as it occurs (H or W == 2): destructible iff
// spawned or >= 2 live cells are destructible or exits (bit 8, which the reference
// merges with destructible: advance_board.c:44-46); colour k iff >= 2 live cells have
// it or a spawner among the 9 has it (advance_board.c:11-21,108-117).
inline uint16_t born_value(const uint16_t *b, int H, int W, int y, int x, bool spawned) {
    int nd = 0, nc[3] = {0, 0, 0};
    unsigned spc = 0;
    for (int dy = -1; dy <= 1; dy++) {
        const int yy = y + dy < 0 ? H - 1 : (y + dy >= H ? 0 : y + dy);
        const uint16_t *row = b + (size_t)yy * W;
        for (int dx = -1; dx <= 1; dx++) {
            const int xx = x + dx < 0 ? W - 1 : (x + dx >= W ? 0 : x + dx);
            const unsigned c = row[xx];
            if (c & SPAWNING) spc |= c & COLORS;
            if (c & ALIVE) {
                nd += (c & (DESTRUCTIBLE | EXIT)) != 0;
                nc[0] += (c >> 9) & 1;
                nc[1] += (c >> 10) & 1;
                nc[2] += (c >> 11) & 1;
            }
        }
    }
    unsigned v = ALIVE | spc;
    if (spawned || nd >= 2) v |= DESTRUCTIBLE;
    for (int k = 0; k < 3; k++)
        if (nc[k] >= 2) v |= 1u << (9 + k);
    return (uint16_t)v;
}

template <int NW>
int64_t advance_nw(const uint16_t *in, uint16_t *out, int H, int W, float spawn_prob,
                   const double *draws, int64_t n_draws) {
    RowOps<NW> ro;
    ro.top = (W - 1) & 63;
    ro.last_mask = ro.top == 63 ? ~(u64)0 : (((u64)1 << (ro.top + 1)) - 1);
    // planes [H][NPL][NW], horizontal quantities [H][NH][NW]
    const size_t need = (size_t)H * (NPL + NH) * NW;
    if (g_scratch.size() < need) g_scratch.resize(need);
    u64 *mem = g_scratch.data();
    u64 (*pl)[NPL][NW] = reinterpret_cast<u64 (*)[NPL][NW]>(mem);
    u64 (*hz)[NH][NW] = reinterpret_cast<u64 (*)[NH][NW]>(mem + (size_t)H * NPL * NW);
#if defined(__x86_64__)
    if (HAVE_AVX512BW)
        extract_board_avx512<NW>(in, H, W, pl);
    else
#endif
        for (int y = 0; y < H; y++) extract_row_scalar<NW>(in + (size_t)y * W, W, pl[y]);

    // ---- horizontal pass
    u64 spawners = 0;
    for (int y = 0; y < H; y++) {
        const u64 (*p)[NW] = pl[y];
        u64 (*h)[NW] = hz[y];
        u64 l[NW], r[NW];
        ro.lft(p[PA], l);
        ro.rgt(p[PA], r);
        for (int i = 0; i < NW; i++) {
            h[HS0][i] = l[i] ^ p[PA][i] ^ r[i];
            h[HS1][i] = maj(l[i], p[PA][i], r[i]);
        }
        for (int f = 0; f < 3; f++) {
            const u64 *s = p[PP + f];
            ro.lft(s, l);
            ro.rgt(s, r);
            for (int i = 0; i < NW; i++) h[HP + f][i] = l[i] | s[i] | r[i];
        }
        for (int i = 0; i < NW; i++) spawners |= p[PS][i];
    }

    // ---- vertical pass, rule, draws, changed cells.  `counting`: no output (out ==
    // NULL, or the caller's draws ran out) -- only the eligible cells are counted
    bool counting = out == nullptr;
    if (!counting) memcpy(out, in, (size_t)H * W * sizeof(uint16_t));
    const double thr = (double)spawn_prob;
    int64_t used = 0;
    for (int y = 0; y < H; y++) {
        const int yu = y == 0 ? H - 1 : y - 1, yd = y == H - 1 ? 0 : y + 1;
        const u64 (*U)[NW] = hz[yu];
        const u64 (*C)[NW] = hz[y];
        const u64 (*D)[NW] = hz[yd];
        const u64 (*p)[NW] = pl[y];
        for (int i = 0; i < NW; i++) {
            // 9-cell alive count n = a0 + 2 (c0 + a1) + 4 b1
            const u64 a0 = U[HS0][i] ^ C[HS0][i] ^ D[HS0][i];
            const u64 c0 = maj(U[HS0][i], C[HS0][i], D[HS0][i]);
            const u64 a1 = U[HS1][i] ^ C[HS1][i] ^ D[HS1][i];
            const u64 b1 = maj(U[HS1][i], C[HS1][i], D[HS1][i]);
            const u64 h1 = ~b1 & (a1 ^ c0);
            const u64 h2 = (b1 & ~a1 & ~c0) | (~b1 & a1 & c0);
            const u64 eq3 = a0 & h1;
            const u64 eq34 = mux(a0, h1, h2);
            const u64 anyP = U[HP][i] | C[HP][i] | D[HP][i];
            const u64 anyI = U[HI][i] | C[HI][i] | D[HI][i];
            const u64 A = p[PA][i], F = p[PF][i];
            const u64 valid = i == NW - 1 ? ro.last_mask : ~(u64)0;
            const u64 kill = A & ~(F | anyP | eq34);
            const u64 dead_ok = ~(A | F | anyI) & valid;
            const u64 birth = dead_ok & eq3;
            u64 sp = 0;
            if (spawners) {
                u64 elig = dead_ok & ~eq3 & (U[HSP][i] | C[HSP][i] | D[HSP][i]);
                if (!counting && used + __builtin_popcountll(elig) > n_draws)
                    counting = true;      // not enough uniforms: count the rest only
                if (counting) {
                    used += __builtin_popcountll(elig);
                    continue;
                }
                while (elig) {
                    const int bx = __builtin_ctzll(elig);
                    elig &= elig - 1;
                    if (draws[used++] < thr) sp |= (u64)1 << bx;
                }
            }
            if (counting) continue;
            uint16_t *orow = out + (size_t)y * W + 64 * i;
            for (u64 m = kill; m; m &= m - 1) orow[__builtin_ctzll(m)] = 0;
            for (u64 m = birth | sp; m; m &= m - 1) {
                const int bx = __builtin_ctzll(m);
                orow[bx] = born_value(in, H, W, y, 64 * i + bx, (sp >> bx) & 1);
            }
        }
    }
    return counting && out != nullptr ? -(used + 1) : used;
}

}  // namespace

extern "C" {

// Host advance of one uint16 [H, W] board (row-major, H, W >= 2, W <= 512).  draws:
// the caller's next n_draws spawn uniforms in reference order.  Returns the number of
// draws consumed (>= 0); -(needed + 1) if the board needs more than n_draws (then
// `out` is unspecified: call again with `needed` draws); with out == NULL, the number
// of eligible cells (the draws an advance consumes; draws unused).  INT64_MIN for a
// bad shape.
int64_t sl_host_advance(const uint16_t *in, uint16_t *out, int64_t H, int64_t W,
                        float spawn_prob, const double *draws, int64_t n_draws) {
    if (H < 2 || W < 2 || W > 512 || H > (1 << 20)) return INT64_MIN;
    const int h = (int)H, w = (int)W;
    switch ((w + 63) >> 6) {
        case 1: return advance_nw<1>(in, out, h, w, spawn_prob, draws, n_draws);
        case 2: return advance_nw<2>(in, out, h, w, spawn_prob, draws, n_draws);
        case 3: return advance_nw<3>(in, out, h, w, spawn_prob, draws, n_draws);
        case 4: return advance_nw<4>(in, out, h, w, spawn_prob, draws, n_draws);
        case 5: return advance_nw<5>(in, out, h, w, spawn_prob, draws, n_draws);
        case 6: return advance_nw<6>(in, out, h, w, spawn_prob, draws, n_draws);
        case 7: return advance_nw<7>(in, out, h, w, spawn_prob, draws, n_draws);
        default: return advance_nw<8>(in, out, h, w, spawn_prob, draws, n_draws);
    }
}

}  // extern "C"
