/*
 * san_check.c -- TEST INFRASTRUCTURE ONLY.  Drives the oracle's C (sl_oracle.c,
 * sl_cpu_step.c) under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5:
 * sanitizers on the host code).  Built by `make -C oracle san`, run by
 * tests/test_sanitizers_cpu.py.  Synthetic levels: random life of random colours,
 * walls, crates, spawners, an agent and exits, on boards from 2x2 to 64x64, so the
 * wrap-around, tiny-board and spawn paths are all visited.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int orc_advance(const uint16_t *in, uint16_t *out, int H, int W, float p, int rng_mode,
                const double *draws, int64_t ndraws, int64_t *pos, uint64_t seed,
                uint32_t env_id, uint32_t step, uint32_t tensor);
int64_t orc_count_eligible(const uint16_t *in, int H, int W);

typedef struct {
    int32_t K, H, W;
    const uint16_t *board, *goals;
    const int32_t *agent_x, *agent_y, *orientation;
    const double *spawn_prob, *min_performance;
} orc_pool;
typedef struct {
    int32_t time_limit, view_h, view_w, remove_white, obs;
    int32_t bonus_period, level_random, augment, n_total;
    double penalty_coef, wrapper_min_perf, bonus, bonus_power;
    uint64_t seed;
} orc_cfg;
void *orc_batch_create(int64_t n, int H, int W, int64_t env0);
void orc_batch_free(void *h);
int orc_batch_reset(void *h, const orc_pool *pool, const orc_cfg *cfg);
int orc_batch_step(void *h, const int32_t *actions, const orc_pool *pool, const orc_cfg *cfg,
                   double *reward, uint8_t *done, uint16_t *obs, int threads);

static uint32_t rng_state = 12345u;
static uint32_t rnd(void) {
    rng_state = rng_state * 1664525u + 1013904223u;
    return rng_state >> 8;
}
static double unif(void) { return (double)rnd() / 16777216.0; }

static void random_level(uint16_t *b, uint16_t *g, int H, int W, int32_t *ax, int32_t *ay) {
    for (int i = 0; i < H * W; i++) {
        const double u = unif();
        uint16_t v = 0;
        if (u < 0.3) v = (uint16_t)(9 | ((rnd() & 7) << 9));
        else if (u < 0.33) v = (uint16_t)(152 | ((rnd() & 7) << 9));   /* spawner */
        else if (u < 0.35) v = 16;                                     /* wall */
        else if (u < 0.36) v = 0x8000 | 4 | 16;                        /* crate */
        else if (u < 0.37) v = 64;                                     /* inhibitor */
        b[i] = v;
        g[i] = unif() < 0.3 ? (uint16_t)((rnd() & 7) << 9) : 0;
    }
    *ax = (int32_t)(rnd() % (uint32_t)W);
    *ay = (int32_t)(rnd() % (uint32_t)H);
    b[*ay * W + *ax] = 122;
    const int ex = (*ax + W / 2) % W, ey = (*ay + H / 2) % H;
    if (ex != *ax || ey != *ay) b[ey * W + ex] = 272;
}

static int run_shape(int H, int W, int B, int T) {
    enum { K = 4 };
    uint16_t *board = malloc(sizeof(uint16_t) * K * H * W), *goals = malloc(sizeof(uint16_t) * K * H * W);
    int32_t ax[K], ay[K], orient[K];
    double sp[K], mp[K];
    for (int k = 0; k < K; k++) {
        random_level(board + k * H * W, goals + k * H * W, H, W, &ax[k], &ay[k]);
        orient[k] = (int32_t)(rnd() & 3);
        sp[k] = 0.3;
        mp[k] = k & 1 ? -1.0 : 0.01;
    }
    /* the rule engine in both RNG modes */
    uint16_t *out = malloc(sizeof(uint16_t) * H * W);
    const int64_t ne = orc_count_eligible(board, H, W);
    double *draws = malloc(sizeof(double) * (size_t)(ne + 1));
    for (int64_t i = 0; i <= ne; i++) draws[i] = unif();
    int64_t pos = 0;
    if (orc_advance(board, out, H, W, 0.3f, 0, draws, ne, &pos, 0, 0, 0, 0) || pos != ne) return 1;
    if (orc_advance(board, out, H, W, 0.3f, 1, NULL, 0, NULL, 9, 1, 2, 3)) return 1;
    /* the env chain, with resets (short time limit) and packed views wider than the board */
    orc_pool pool = {K, H, W, board, goals, ax, ay, orient, sp, mp};
    orc_cfg cfg = {7, 33, 33, 1, 1, 4, 1, 1, B, 1.0, 0.01, 0.1, 0.01, 77};
    void *h = orc_batch_create(B, H, W, 3);
    if (!h || orc_batch_reset(h, &pool, &cfg)) return 1;
    int32_t *act = malloc(sizeof(int32_t) * B);
    double *rew = malloc(sizeof(double) * B);
    uint8_t *done = malloc((size_t)B);
    uint16_t *obs = malloc(sizeof(uint16_t) * B * 33 * 33);
    for (int t = 0; t < T; t++) {
        for (int i = 0; i < B; i++) act[i] = (int32_t)(rnd() % 9);
        if (orc_batch_step(h, act, &pool, &cfg, rew, done, obs, 1)) return 1;
    }
    orc_batch_free(h);
    free(board); free(goals); free(out); free(draws); free(act); free(rew); free(done); free(obs);
    return 0;
}

int main(void) {
    static const int shapes[][2] = {{2, 2}, {3, 5}, {2, 7}, {25, 25}, {26, 26}, {64, 64}, {17, 40}};
    for (size_t s = 0; s < sizeof(shapes) / sizeof(shapes[0]); s++) {
        if (run_shape(shapes[s][0], shapes[s][1], 8, 40)) {
            printf("FAIL %dx%d\n", shapes[s][0], shapes[s][1]);
            return 1;
        }
    }
    printf("san_check ok\n");
    return 0;
}
