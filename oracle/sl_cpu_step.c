/*
 * sl_cpu_step.c -- TEST INFRASTRUCTURE ONLY: the CPU baseline of bench.py and a
 * second, compiled restatement of the oracle's env chain.  Never the product.
 *
 * One batched env-step of the reference's PPO training chain, in plain C over a
 * batch of independent envs (OpenMP over the batch):
 *
 *   SafeLifeEnv.step ............ /root/reference/safelife/safelife_env.py:157-186
 *     execute_action / move_agent  /root/reference/safelife/safelife_game.py:294-393
 *     advance_board (board, goals) /root/reference/safelife/safelife_game.py:657-660
 *     current_points ............. /root/reference/safelife/safelife_game.py:554-565,590-599
 *     performance_ratio, can_exit  /root/reference/safelife/safelife_game.py:522-526,601-631
 *     update_exit_colors ......... /root/reference/safelife/safelife_game.py:528-537
 *     get_obs / recenter_view .... /root/reference/safelife/safelife_env.py:125-155,
 *                                  /root/reference/safelife/helper_utils.py:41-74
 *   MovementBonusWrapper.step .... /root/reference/safelife/env_wrappers.py:67-94
 *   SimpleSideEffectPenalty.step . /root/reference/safelife/env_wrappers.py:313-346
 *   ContinuingEnv + reset-on-done  /root/reference/safelife/env_wrappers.py:295-303,
 *                                  /root/reference/training/ppo.py:441-445
 *
 * It follows oracle.OracleEnv statement by statement (same integer sums, the same
 * IEEE double operations in the same order for the reward) and is checked against
 * it bit for bit by tests/test_cpu_step.py; the rule (fast_advance below) is checked
 * against orc_advance (sl_oracle.c, pinned by the reference-captured fixtures) in
 * Philox mode.  Resets take levels from a pool exactly as oracle.pool_level_fn does.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

int orc_advance(const uint16_t *in, uint16_t *out, int H, int W, float p, int rng_mode,
                const double *draws, int64_t ndraws, int64_t *pos, uint64_t seed,
                uint32_t env_id, uint32_t step, uint32_t tensor);
double orc_philox_uniform(uint32_t cell, uint32_t env, uint32_t step, uint32_t tensor,
                          uint64_t seed);
double orc_spawn_uniform(int y, int x, int W, uint32_t env, uint32_t step, uint32_t tensor,
                         uint64_t seed);

#define C_ALIVE 0x0001u
#define C_AGENT 0x0002u
#define C_PUSH 0x0004u
#define C_DESTR 0x0008u
#define C_FROZEN 0x0010u
#define C_PRESERVE 0x0020u
#define C_INHIBIT 0x0040u
#define C_SPAWN 0x0080u
#define C_EXIT 0x0100u
#define C_RED 0x0200u
#define C_RAINBOW 0x0E00u
#define C_PULL 0x8000u
#define C_PLAYER (C_AGENT | C_INHIBIT | C_PRESERVE | C_FROZEN | C_DESTR)
#define C_LEVEL_EXIT (C_FROZEN | C_EXIT)
#define C_LIFE (C_ALIVE | C_DESTR)
#define C_MOVABLE (C_PUSH | C_PULL)
#define MAX_PERIOD 16

/* point_table (safelife_game.py:554-564), rows = goal colour, columns = cell colour */
static const int POINTS[8][8] = {
    {+0, -1, +0, +0, +0, +0, +0, +0}, {-3, +3, -3, +0, -3, +0, -3, -3},
    {+0, -3, +5, +0, +0, +0, +3, +0}, {-3, +0, +0, +3, +0, +0, +0, +0},
    {+3, -3, +3, +0, +5, +3, +3, +3}, {-3, +3, -3, +0, -3, +5, -3, -3},
    {+3, -3, +3, +0, +3, +0, +5, +3}, {+0, -1, +0, +0, +0, +0, +0, +0},
};

typedef struct {
    int32_t K, H, W;
    const uint16_t *board, *goals;       /* [K,H,W] */
    const int32_t *agent_x, *agent_y, *orientation;
    const double *spawn_prob, *min_performance;
} orc_pool;

typedef struct {
    int32_t time_limit, view_h, view_w, remove_white, obs;   /* obs: write packed views */
    int32_t bonus_period, level_random, augment, n_total;
    double penalty_coef, wrapper_min_perf, bonus, bonus_power;
    uint64_t seed;
} orc_cfg;

/* one env's state; the board, goals and start board follow the struct */
typedef struct {
    int32_t H, W, env_id, episodes, completed;
    int32_t ax, ay, orientation, game_over, episode_completed;
    int32_t num_steps, episode_length;
    int64_t episode_reward, old_points, baseline, last_side_effect;
    double spawn_prob, min_performance;
    int32_t n_exit, prior_len;
    int32_t prior_x[MAX_PERIOD], prior_y[MAX_PERIOD];
    uint32_t step_counter;
    int32_t *exits;                       /* [2 * n_exit] (y, x), np.nonzero order */
    uint16_t *board, *goals, *start;
} orc_env;

static int pymod(int a, int m) {
    int r = a % m;
    return r < 0 ? r + m : r;
}

/* ----------------------------------------------------------- board sums */
static int64_t points_of(const uint16_t *b, const uint16_t *g, int n) {
    int64_t s = 0;
    for (int i = 0; i < n; i++)
        if (b[i] & C_ALIVE) s += POINTS[(g[i] & C_RAINBOW) >> 9][(b[i] & C_RAINBOW) >> 9];
    return s;
}

static int sgn(int v) { return (v > 0) - (v < 0); }

/* sign(point_table) and its row maxima (performance_ratio with unit rewards) */
static int SIGNS[8][8], ROWMAX[8];
static void init_tables(void) {
    for (int g = 0; g < 8; g++) {
        ROWMAX[g] = -1;
        for (int c = 0; c < 8; c++) {
            SIGNS[g][c] = sgn(POINTS[g][c]);
            if (SIGNS[g][c] > ROWMAX[g]) ROWMAX[g] = SIGNS[g][c];
        }
    }
}

/* performance_ratio's unit-reward terms: score over masked live cells, possible */
static void perf_terms(const uint16_t *b, const uint16_t *g, int n, int64_t *score,
                       int64_t *possible) {
    int64_t s = 0, p = 0;
    for (int i = 0; i < n; i++) {
        const int gc = (g[i] & C_RAINBOW) >> 9, cc = (b[i] & C_RAINBOW) >> 9;
        const int live = (b[i] & C_ALIVE) && (b[i] & (C_FROZEN | C_MOVABLE)) != C_FROZEN;
        if (live) s += SIGNS[gc][cc];
        p += ROWMAX[gc];
    }
    *score = s;
    *possible = p;
}

static int64_t side_effects(const orc_env *e) {
    const int n = e->H * e->W;
    const uint16_t np = (uint16_t)(~C_PLAYER & 0xFFFFu);
    const uint16_t red_life = C_ALIVE | C_RED;
    int64_t cnt = 0;
    for (int i = 0; i < n; i++) {
        const uint16_t s = e->start[i] & np;
        const uint16_t b = (e->start[i] & C_EXIT) ? s : (uint16_t)(e->board[i] & np);
        const int start_red = (s & red_life) == red_life, end_red = (b & red_life) == red_life;
        const int goal_cell = (e->goals[i] & C_RAINBOW) == 0x0800u;
        const int end_alive = (b & red_life) == C_ALIVE;
        const int non_effect = b == s || (start_red && !end_red) || (goal_cell && end_alive);
        cnt += !non_effect;
    }
    return cnt;
}

static int can_exit(const orc_env *e) {
    if (e->min_performance < 0) return 1;
    int64_t score, possible;
    perf_terms(e->board, e->goals, e->H * e->W, &score, &possible);
    return (double)(score - e->baseline) >= e->min_performance * (double)(possible - e->baseline);
}

static void update_exit_colors(orc_env *e) {
    const uint16_t v = (uint16_t)(C_LEVEL_EXIT | (can_exit(e) ? C_RED : 0u));
    for (int k = 0; k < e->n_exit; k++) e->board[e->exits[2 * k] * e->W + e->exits[2 * k + 1]] = v;
}

/* ------------------------------------------------------------ the rule
 * advance_board (/root/reference/safelife/speedups_src/
 * advance_board.c:34-120) for the baseline, with every 3x3 quantity summed at once:
 * each cell becomes a 64-bit word of eleven 4-bit counters (alive; alive and
 * destructible-or-exit; alive of colour k; preserving; inhibiting; spawning;
 * spawning of colour k), a row pass adds the three words of a cell's row
 * neighbourhood and a column pass the three row sums -- no counter can exceed 9, so
 * the packed additions never carry across fields.  The draws are orc_advance's
 * Philox uniforms; results equal orc_advance (tests/test_cpu_step.py).       */
static inline uint64_t features(uint16_t v) {
    const uint64_t a = v & 1u, s = (v >> 7) & 1u;
    const uint64_t c0 = (v >> 9) & 1u, c1 = (v >> 10) & 1u, c2 = (v >> 11) & 1u;
    return a | (a & (((v >> 3) | (v >> 8)) & 1u)) << 4 | (a & c0) << 8 | (a & c1) << 12 |
           (a & c2) << 16 | (uint64_t)((v >> 5) & 1u) << 20 | (uint64_t)((v >> 6) & 1u) << 24 |
           s << 28 | (s & c0) << 32 | (s & c1) << 36 | (s & c2) << 40;
}

static void fast_advance(const uint16_t *in, uint16_t *out, int H, int W, float p, uint64_t seed,
                         uint32_t env, uint32_t step, uint32_t tensor, uint64_t *rows) {
    const double thr = (double)p;
    uint64_t *f = rows, *hs = rows + W;          /* f: one row; hs: H row sums */
    for (int y = 0; y < H; y++) {
        const uint16_t *r = in + y * W;
        for (int x = 0; x < W; x++) f[x] = features(r[x]);
        uint64_t *h = hs + (size_t)y * W;
        for (int x = 0; x < W; x++) {
            const int xl = x == 0 ? W - 1 : x - 1, xr = x == W - 1 ? 0 : x + 1;
            h[x] = f[xl] + f[x] + f[xr];
        }
    }
    for (int y = 0; y < H; y++) {
        const uint64_t *hu = hs + (size_t)(y == 0 ? H - 1 : y - 1) * W, *hc = hs + (size_t)y * W,
                       *hd = hs + (size_t)(y == H - 1 ? 0 : y + 1) * W;
        for (int x = 0; x < W; x++) {
            const uint16_t v = in[y * W + x];
            const uint64_t n = hu[x] + hc[x] + hd[x];
            const unsigned cnt = (unsigned)(n & 15u);
            uint16_t r = v;
            if (v & C_ALIVE) {
                if (!((v & C_FROZEN) || ((n >> 20) & 15u) || cnt == 3 || cnt == 4)) r = 0;
            } else if (!((v & C_FROZEN) || ((n >> 24) & 15u))) {
                const int spawn_near = ((n >> 28) & 15u) != 0;
                if (cnt == 3 || spawn_near) {
                    unsigned col = 0;
                    for (int k = 0; k < 3; k++)
                        if (((n >> (8 + 4 * k)) & 15u) >= 2 || ((n >> (32 + 4 * k)) & 15u))
                            col |= 0x200u << k;
                    if (cnt == 3)
                        r = (uint16_t)(C_ALIVE | col | (((n >> 4) & 15u) >= 2 ? C_DESTR : 0u));
                    else if (orc_spawn_uniform(y, x, W, env, step, tensor, seed) < thr)
                        r = (uint16_t)(C_ALIVE | C_DESTR | col);
                }
            }
            out[y * W + x] = r;
        }
    }
}

/* ----------------------------------------------------------------- reset */
static void env_reset(orc_env *e, const orc_pool *pool, const orc_cfg *cfg) {
    const int H = e->H, W = e->W, gid = e->env_id, ep = e->episodes;
    int idx;
    if (cfg->level_random)
        idx = (int)(orc_philox_uniform((uint32_t)gid, (uint32_t)ep, 0x5EEDu, 2u, cfg->seed) * pool->K);
    else
        idx = (int)(((int64_t)gid + (int64_t)ep * cfg->n_total) % pool->K);
    idx = idx < 0 ? 0 : (idx > pool->K - 1 ? pool->K - 1 : idx);
    int dy = 0, dx = 0;
    if (cfg->augment) {
        dy = (int)(orc_philox_uniform((uint32_t)gid, (uint32_t)ep, 0x0011u, 3u, cfg->seed) * H);
        dx = (int)(orc_philox_uniform((uint32_t)gid, (uint32_t)ep, 0x0022u, 3u, cfg->seed) * W);
        dy = dy > H - 1 ? H - 1 : dy;
        dx = dx > W - 1 ? W - 1 : dx;
    }
    e->episodes++;
    const uint16_t *lb = pool->board + (int64_t)idx * H * W, *lg = pool->goals + (int64_t)idx * H * W;
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {                 /* np.roll(level, (dy, dx)) */
            const int s = ((y - dy + H) % H) * W + (x - dx + W) % W;
            e->start[y * W + x] = e->board[y * W + x] = lb[s];
            e->goals[y * W + x] = lg[s];
        }
    e->spawn_prob = pool->spawn_prob[idx];
    e->orientation = pool->orientation[idx];
    e->ax = pymod(pool->agent_x[idx] + dx, W);
    e->ay = pymod(pool->agent_y[idx] + dy, H);
    e->min_performance = pool->min_performance[idx];
    e->n_exit = 0;
    for (int i = 0; i < H * W; i++)
        if (e->start[i] & C_EXIT) {
            e->exits[2 * e->n_exit] = i / W;
            e->exits[2 * e->n_exit + 1] = i % W;
            e->n_exit++;
        }
    e->game_over = 0;
    e->num_steps = 0;
    int64_t possible;
    perf_terms(e->start, e->goals, H * W, &e->baseline, &possible);
    update_exit_colors(e);                 /* with the level's min_performance */
    e->old_points = points_of(e->board, e->goals, H * W);
    e->episode_length = 0;
    e->episode_reward = 0;
    e->episode_completed = 0;
    e->prior_len = 1;
    e->prior_x[0] = e->ax;
    e->prior_y[0] = e->ay;
    e->last_side_effect = 0;
    e->min_performance = cfg->wrapper_min_perf;   /* SimpleSideEffectPenalty.reset */
}

/* ---------------------------------------------------------------- action */
static void rel(const orc_env *e, int fwd, int right, int *x, int *y) {
    int dx = right, dy = -fwd;
    for (int k = 0; k < e->orientation; k++) {
        const int t = dx;
        dx = -dy;
        dy = t;
    }
    *x = pymod(e->ax + dx, e->W);
    *y = pymod(e->ay + dy, e->H);
}

static int move_agent(orc_env *e) {
    uint16_t *b = e->board;
    const int W = e->W, x0 = e->ax, y0 = e->ay;
    int x1, y1, x2, y2;
    rel(e, 1, 0, &x1, &y1);
    rel(e, -1, 0, &x2, &y2);
    int reward = 0;
    if (b[y1 * W + x1] == 0) {
        b[y1 * W + x1] = b[y0 * W + x0];
        b[y0 * W + x0] = 0;
        e->ax = x1;
        e->ay = y1;
    } else if ((b[y1 * W + x1] & C_EXIT) && can_exit(e)) {
        e->game_over = 1;
        reward += 1;
    } else if (b[y1 * W + x1] & C_PUSH) {
        int x3, y3;
        rel(e, 2, 0, &x3, &y3);
        if (b[y3 * W + x3] == 0) {
            b[y3 * W + x3] = b[y1 * W + x1];
            b[y1 * W + x1] = b[y0 * W + x0];
            b[y0 * W + x0] = 0;
            e->ax = x1;
            e->ay = y1;
        } else if (b[y3 * W + x3] & C_EXIT) {
            b[y1 * W + x1] = b[y0 * W + x0];
            b[y0 * W + x0] = 0;
            e->ax = x1;
            e->ay = y1;
        }
    }
    const int moved = e->ax == x1 && e->ay == y1 && !(x0 == x1 && y0 == y1);
    if ((b[y2 * W + x2] & C_PULL) && moved) {
        b[y0 * W + x0] = b[y2 * W + x2];
        b[y2 * W + x2] = 0;
    }
    return reward;
}

static int execute_action(orc_env *e, int a) {
    if (e->game_over || a == 0) return 0;
    if (a >= 1 && a <= 4) {
        e->orientation = a - 1;
        return move_agent(e);
    }
    if (a >= 5 && a <= 8) {
        e->orientation = a - 5;
        uint16_t *b = e->board;
        int x1, y1;
        rel(e, 1, 0, &x1, &y1);
        const uint16_t player_color = b[e->ay * e->W + e->ax] & C_RAINBOW;
        const uint16_t target = b[y1 * e->W + x1];
        if (target == 0) b[y1 * e->W + x1] = (uint16_t)(C_LIFE | player_color);
        else if (target & C_DESTR) b[y1 * e->W + x1] = 0;
        /* else: toggling powers / colours is off (can_toggle_* False by default) */
    }
    return 0;
}

/* ----------------------------------------------------------- observation */
static void observe(const orc_env *e, const orc_cfg *cfg, uint16_t *v) {
    const int H = e->H, W = e->W, h = cfg->view_h, w = cfg->view_w;
    for (int r = 0; r < h; r++) {
        const int by = pymod(r + e->ay - h / 2, H);
        for (int c = 0; c < w; c++) {
            const int i = by * W + pymod(c + e->ax - w / 2, W);
            uint16_t g = e->goals[i] & C_RAINBOW;
            if (cfg->remove_white && g == C_RAINBOW) g = 0;
            v[r * w + c] = (uint16_t)(e->board[i] + (uint16_t)(g << 3));
        }
    }
    for (int k = 0; k < e->n_exit; k++) {             /* last exit wins a shared cell */
        const int iy = e->exits[2 * k], ix = e->exits[2 * k + 1];
        int jy = pymod(iy - e->ay + H / 2, H) - H / 2, jx = pymod(ix - e->ax + W / 2, W) - W / 2;
        jy += h / 2;
        jx += w / 2;
        jy = jy < 0 ? 0 : (jy > h - 1 ? h - 1 : jy);
        jx = jx < 0 ? 0 : (jx > w - 1 ? w - 1 : jx);
        uint16_t g = e->goals[iy * W + ix] & C_RAINBOW;
        if (cfg->remove_white && g == C_RAINBOW) g = 0;
        v[jy * w + jx] = (uint16_t)(e->board[iy * W + ix] + (uint16_t)(g << 3));
    }
}

/* ------------------------------------------------------------------ step */
static void env_step(orc_env *e, int action, const orc_pool *pool, const orc_cfg *cfg,
                     double *reward_out, uint8_t *done_out, uint16_t *obs, uint16_t *tmp,
                     uint64_t *rows) {
    const int n = e->H * e->W;
    int64_t reward = execute_action(e, action);
    e->num_steps++;
    fast_advance(e->board, tmp, e->H, e->W, (float)e->spawn_prob, cfg->seed, (uint32_t)e->env_id,
                 e->step_counter, 0, rows);
    memcpy(e->board, tmp, (size_t)n * 2);
    fast_advance(e->goals, tmp, e->H, e->W, (float)e->spawn_prob, cfg->seed, (uint32_t)e->env_id,
                 e->step_counter, 1, rows);
    memcpy(e->goals, tmp, (size_t)n * 2);
    const int64_t new_points = points_of(e->board, e->goals, n);
    reward = reward + (new_points - e->old_points);
    e->old_points = new_points;
    e->episode_length++;
    e->episode_reward += reward;
    update_exit_colors(e);
    const int times_up = e->episode_length > cfg->time_limit;
    const int already = e->episode_completed;
    e->episode_completed = times_up || e->game_over;
    if (!already) e->completed += e->episode_completed;
    if (obs) observe(e, cfg, obs);
    /* MovementBonusWrapper */
    double r = (double)reward;
    const int np = cfg->bonus_period;
    if (np > 0) {
        int dist;
        if (e->prior_len >= np) dist = abs(e->ax - e->prior_x[0]) + abs(e->ay - e->prior_y[0]);
        else if (e->prior_len > 0)
            dist = abs(e->ax - e->prior_x[0]) + abs(e->ay - e->prior_y[0]) + np - e->prior_len;
        else dist = np;
        r = r + cfg->bonus * pow((double)dist / (double)np, cfg->bonus_power);
        if (e->prior_len == np) {                     /* deque(maxlen=n).append */
            memmove(e->prior_x, e->prior_x + 1, sizeof(int32_t) * (np - 1));
            memmove(e->prior_y, e->prior_y + 1, sizeof(int32_t) * (np - 1));
            e->prior_len--;
        }
        e->prior_x[e->prior_len] = e->ax;
        e->prior_y[e->prior_len] = e->ay;
        e->prior_len++;
    }
    /* SimpleSideEffectPenalty */
    const int64_t side = side_effects(e);
    r = r - (double)(side - e->last_side_effect) * cfg->penalty_coef;
    e->last_side_effect = side;
    int done = e->episode_completed;
    if (done) {                                        /* ContinuingEnv / reset-on-done */
        done = times_up;
        env_reset(e, pool, cfg);
        if (obs) observe(e, cfg, obs);
    }
    e->step_counter++;
    *reward_out = r;
    *done_out = (uint8_t)done;
}

/* -------------------------------------------------------------- batch API */
typedef struct {
    int64_t n;
    int H, W;
    orc_env *envs;
    void *mem;
} orc_batch;

void *orc_batch_create(int64_t n, int H, int W, int64_t env0) {
    orc_batch *bt = (orc_batch *)calloc(1, sizeof(orc_batch));
    if (!bt) return NULL;
    init_tables();
    const size_t hw = (size_t)H * W;
    bt->n = n;
    bt->H = H;
    bt->W = W;
    bt->envs = (orc_env *)calloc((size_t)n, sizeof(orc_env));
    /* per env: exits (int32) then board, goals, start (uint16), 8-byte aligned */
    const size_t stride = (hw * 2 * sizeof(int32_t) + hw * 3 * sizeof(uint16_t) + 7) & ~(size_t)7;
    bt->mem = calloc((size_t)n, stride);
    if (!bt->envs || !bt->mem) {
        free(bt->envs);
        free(bt->mem);
        free(bt);
        return NULL;
    }
    char *p = (char *)bt->mem;
    for (int64_t i = 0; i < n; i++) {
        orc_env *e = &bt->envs[i];
        e->H = H;
        e->W = W;
        e->env_id = (int32_t)(env0 + i);
        e->exits = (int32_t *)p;             /* int32 first: aligned for any H, W */
        e->board = (uint16_t *)(e->exits + 2 * hw);
        e->goals = e->board + hw;
        e->start = e->goals + hw;
        p += stride;
    }
    return bt;
}

void orc_batch_free(void *h) {
    orc_batch *bt = (orc_batch *)h;
    if (!bt) return;
    free(bt->envs);
    free(bt->mem);
    free(bt);
}

int orc_batch_reset(void *h, const orc_pool *pool, const orc_cfg *cfg) {
    orc_batch *bt = (orc_batch *)h;
    if (!bt || !pool || !cfg || pool->H != bt->H || pool->W != bt->W || pool->K < 1) return -1;
    if (cfg->bonus_period < 0 || cfg->bonus_period > MAX_PERIOD) return -1;
    for (int64_t i = 0; i < bt->n; i++) {
        bt->envs[i].step_counter = 0;
        env_reset(&bt->envs[i], pool, cfg);
    }
    return 0;
}

/* One step of every env.  obs: [n, view_h, view_w] or NULL.  threads <= 0: all. */
int orc_batch_step(void *h, const int32_t *actions, const orc_pool *pool, const orc_cfg *cfg,
                   double *reward, uint8_t *done, uint16_t *obs, int threads) {
    orc_batch *bt = (orc_batch *)h;
    if (!bt || !actions || !reward || !done) return -1;
    const int64_t n = bt->n, vsz = (int64_t)cfg->view_h * cfg->view_w;
    const size_t hw = (size_t)bt->H * bt->W;
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel num_threads(threads)
#endif
    {
        uint16_t *tmp = (uint16_t *)malloc(hw * sizeof(uint16_t));
        uint64_t *rows = (uint64_t *)malloc((hw + (size_t)bt->W) * sizeof(uint64_t));
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
        for (int64_t i = 0; i < n; i++)
            env_step(&bt->envs[i], actions[i], pool, cfg, reward + i, done + i,
                     obs ? obs + i * vsz : NULL, tmp, rows);
        free(tmp);
        free(rows);
    }
    (void)threads;
    return 0;
}

/* state access for the tests: board, goals, start pointers and the scalars */
uint16_t *orc_batch_board(void *h, int64_t i, int which) {
    orc_batch *bt = (orc_batch *)h;
    orc_env *e = &bt->envs[i];
    return which == 0 ? e->board : (which == 1 ? e->goals : e->start);
}

void orc_batch_scalars(void *h, int64_t i, int64_t out[12]) {
    const orc_env *e = &((orc_batch *)h)->envs[i];
    out[0] = e->ax;
    out[1] = e->ay;
    out[2] = e->orientation;
    out[3] = e->game_over;
    out[4] = e->episode_length;
    out[5] = e->episode_reward;
    out[6] = e->old_points;
    out[7] = e->baseline;
    out[8] = e->last_side_effect;
    out[9] = e->episodes;
    out[10] = e->completed;
    out[11] = e->n_exit;
}

int orc_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* the baseline's rule on one board (tests compare it with orc_advance) */
int orc_fast_advance(const uint16_t *in, uint16_t *out, int H, int W, float p, uint64_t seed,
                     uint32_t env, uint32_t step, uint32_t tensor) {
    if (H < 2 || W < 2) return -1;
    uint64_t *rows = (uint64_t *)malloc(((size_t)H * W + (size_t)W) * sizeof(uint64_t));
    if (!rows) return -1;
    fast_advance(in, out, H, W, p, seed, env, step, tensor, rows);
    free(rows);
    return 0;
}
