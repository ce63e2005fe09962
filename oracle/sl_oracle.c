/*
 * sl_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * Plain-C CPU restatement of the SafeLife rule engine, written from the per-cell
 * specification, not from the reference's two-pass
 * implementation.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library.
 *
 * Reference algorithm restated:
 *   /root/reference/safelife/speedups_src/advance_board.c:34-120  (advance_board)
 *   /root/reference/safelife/speedups_src/advance_board.c:6-9     (masks)
 *   /root/reference/safelife/speedups_src/constants.h:4-25        (bit enum)
 *   /root/reference/safelife/speedups_src/random.c:47-52          (one uniform per
 *        eligible cell, compared as  u < (double)(float)spawn_prob)
 *
 * Pinned by tests/golden/advance_known_answers.npz and the stochastic-stream
 * fixtures produced from the reference extension itself (tests/golden/make_golden.py).
 *
 * RNG modes (the "draws" of a board step are consumed in row-major order over
 * ELIGIBLE cells only -- dead, not frozen, no inhibitor in the 3x3 neighbourhood,
 * neighbour count != 3, and a spawner in the 3x3 neighbourhood):
 *   ORC_RNG_STREAM : draws[pos++] from a caller-supplied uniform stream (the
 *                    reference's numpy MT19937 buffer, replayed);
 *   ORC_RNG_PHILOX : Philox4x32-10 keyed by (seed), counter (cell, env, step, tensor)
 *                    -- the build's own production RNG (no reference analogue).
 */
#include <stdint.h>
#include <string.h>
#include <math.h>

enum {
    ORC_RNG_STREAM = 0,
    ORC_RNG_PHILOX = 1,
};

#define B_ALIVE 0x0001u
#define B_DESTR 0x0008u
#define B_FROZEN 0x0010u
#define B_PRESERVE 0x0020u
#define B_INHIBIT 0x0040u
#define B_SPAWN 0x0080u
#define B_EXIT 0x0100u
#define B_COLORS 0x0E00u

/* ---------------- Philox4x32-10 (Salmon et al., SC'11) ---------------- */
static inline void philox_round(uint32_t c[4], const uint32_t k[2]) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c[1] ^ k[0];
    uint32_t n2 = hi0 ^ c[3] ^ k[1];
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
}

void orc_philox4x32(uint32_t out[4], uint32_t c0, uint32_t c1, uint32_t c2,
                    uint32_t c3, uint64_t seed) {
    uint32_t c[4] = {c0, c1, c2, c3};
    uint32_t k[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (int r = 0; r < 10; r++) {
        philox_round(c, k);
        k[0] += 0x9E3779B9u;
        k[1] += 0xBB67AE85u;
    }
    memcpy(out, c, sizeof(c));
}

/* uniform double in [0,1) with 53 random bits, same construction numpy uses */
double orc_philox_uniform(uint32_t cell, uint32_t env, uint32_t step,
                          uint32_t tensor, uint64_t seed) {
    uint32_t x[4];
    orc_philox4x32(x, cell, env, step, tensor, seed);
    uint32_t a = x[0] >> 5, b = x[1] >> 6;
    return ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
}

/* Philox-mode spawn draw of cell (y, x) of a W-column tensor (the build's own RNG; the
   reference has only its global stream): the four cells of the 2x2 block
   (y >> 1, x >> 1) share one Philox4x32-10 evaluation, counter (block, env, step,
   tensor) with block = (y >> 1) * ceil(W / 2) + (x >> 1); cell (y, x) takes output
   word (y & 1) * 2 + (x & 1), as word * 2^-32.  Same as spawn_uniform (sl_device.h). */
double orc_spawn_uniform(int y, int x, int W, uint32_t env, uint32_t step, uint32_t tensor,
                         uint64_t seed) {
    uint32_t r[4];
    orc_philox4x32(r, (uint32_t)((y >> 1) * ((W + 1) >> 1) + (x >> 1)), env, step, tensor, seed);
    return (double)r[(y & 1) * 2 + (x & 1)] * (1.0 / 4294967296.0);
}

/* ---------------- per-cell rule (Appendix A) ---------------- */
typedef struct {
    int cnt;          /* alive cells in 3x3 incl. self, with multiplicity */
    int any_p, any_i, any_s;
    int pair_d;       /* >= 2 alive cells that are destructible-or-exit */
    int col;          /* colour bits 9..11 for a newborn */
} nbhd_t;

static void gather(const uint16_t *b, int H, int W, int y, int x, nbhd_t *n) {
    int nd = 0, nc[3] = {0, 0, 0}, sc = 0;
    memset(n, 0, sizeof(*n));
    for (int dy = -1; dy <= 1; dy++) {
        int yy = (y + dy + H) % H;
        for (int dx = -1; dx <= 1; dx++) {
            int xx = (x + dx + W) % W;
            uint16_t v = b[yy * W + xx];
            int alive = v & B_ALIVE;
            n->cnt += alive;
            n->any_p |= (v & B_PRESERVE) != 0;
            n->any_i |= (v & B_INHIBIT) != 0;
            n->any_s |= (v & B_SPAWN) != 0;
            if (alive && (v & (B_DESTR | B_EXIT))) nd++;
            for (int k = 0; k < 3; k++)
                if (alive && (v & (0x200u << k))) nc[k]++;
            if (v & B_SPAWN) sc |= v & B_COLORS;
        }
    }
    n->pair_d = nd >= 2;
    int col = sc;
    for (int k = 0; k < 3; k++)
        if (nc[k] >= 2) col |= 0x200 << k;
    n->col = col;
}

/* eligible == this cell consumes exactly one uniform draw */
static int eligible(uint16_t v, const nbhd_t *n) {
    if (v & B_ALIVE) return 0;
    if ((v & B_FROZEN) || n->any_i) return 0;
    if (n->cnt == 3) return 0;
    return n->any_s;
}

int64_t orc_count_eligible(const uint16_t *in, int H, int W) {
    int64_t c = 0;
    nbhd_t n;
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            gather(in, H, W, y, x, &n);
            c += eligible(in[y * W + x], &n);
        }
    return c;
}

/*
 * Advance one H x W board.  Returns 0, or -1 on bad shape / exhausted stream.
 *   rng_mode ORC_RNG_STREAM: draws[*pos], *pos advanced per eligible cell;
 *            draws may be NULL when p <= 0 (never spawns) or p >= 1 (always).
 *   rng_mode ORC_RNG_PHILOX: uniform from (cell, env_id, step, tensor, seed).
 */
int orc_advance(const uint16_t *in, uint16_t *out, int H, int W, float p,
                int rng_mode, const double *draws, int64_t ndraws, int64_t *pos,
                uint64_t seed, uint32_t env_id, uint32_t step, uint32_t tensor) {
    if (H < 2 || W < 2) return -1;
    const double thr = (double)p;
    nbhd_t n;
    for (int y = 0; y < H; y++) {
        for (int x = 0; x < W; x++) {
            uint16_t v = in[y * W + x];
            uint16_t r = v;
            gather(in, H, W, y, x, &n);
            if (v & B_ALIVE) {
                if (!((v & B_FROZEN) || n.any_p || n.cnt == 3 || n.cnt == 4)) r = 0;
            } else if ((v & B_FROZEN) || n.any_i) {
                r = v;
            } else if (n.cnt == 3) {
                r = (uint16_t)(B_ALIVE | n.col | (n.pair_d ? B_DESTR : 0));
            } else if (n.any_s) {
                double u;
                if (rng_mode == ORC_RNG_PHILOX) {
                    u = orc_spawn_uniform(y, x, W, env_id, step, tensor, seed);
                } else if (draws == NULL) {
                    if (!(thr <= 0.0 || thr >= 1.0)) return -1;
                    u = thr <= 0.0 ? 1.0 : 0.0;
                } else {
                    if (*pos >= ndraws) return -1;
                    u = draws[(*pos)++];
                }
                if (u < thr) r = (uint16_t)(B_ALIVE | B_DESTR | n.col);
            }
            out[y * W + x] = r;
        }
    }
    return 0;
}

/* batched convenience: boards [B,H,W], contiguous; stream shared in env order */
int orc_advance_batch(const uint16_t *in, uint16_t *out, int64_t B, int H, int W,
                      float p, int rng_mode, const double *draws, int64_t ndraws,
                      int64_t *pos, uint64_t seed, uint32_t env0, uint32_t step,
                      uint32_t tensor) {
    const int64_t hw = (int64_t)H * W;
    for (int64_t b = 0; b < B; b++) {
        int rc = orc_advance(in + b * hw, out + b * hw, H, W, p, rng_mode, draws,
                             ndraws, pos, seed, (uint32_t)(env0 + b), step, tensor);
        if (rc) return rc;
    }
    return 0;
}
