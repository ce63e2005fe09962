/*
 * safelife_hip.h -- C ABI of the MI355X (gfx950) SafeLife stepper.
 *
 * Plain pointers and sizes only; every pointer argument marked "dev" is device
 * memory on the current HIP device, every call is stream-ordered on `stream`
 * (a hipStream_t passed as void*, NULL = default stream) and returns 0 or a
 * negative SL_E* code.  No global state: two streams may run independent
 * batches concurrently.  Layouts are row-major uint16 [B, H, W] boards
 * (bit layout of safelife_game.py:74-120 / speedups_src/constants.h:4-25).
 *
 * Reference interfaces each entry point replaces:
 *   sl_advance          speedups.advance_board(board, spawn_prob=0.3)
 *                       /root/reference/safelife/speedups_src/module.c:19-44
 *                       (batched over B boards; the reference does one per call)
 *   sl_count_eligible   the draw count of one advance_board call
 *                       (random_float() calls, advance_board.c:110) -- used to
 *                       place each board's draws in the reference stream
 *                       (speedups.seed / random.c:28-52)
 *   sl_env_step         SafeLifeEnv.step (safelife_env.py:157-186) under the
 *                       PPO chain MovementBonusWrapper -> SimpleSideEffectPenalty
 *                       -> ContinuingEnv (training/safelife_ppo.py:128-139,
 *                       env_wrappers.py:67-88,319-346,298-303) for B envs at once,
 *                       as driven by PPO.run_agents (training/ppo.py:436-452)
 *   sl_env_reset        SafeLifeEnv.reset (safelife_env.py:188-198) + the
 *                       wrappers' resets (env_wrappers.py:90-94,313-317) for the
 *                       envs selected by a mask, from a device level pool
 *                       (the level_iterator / safelife_loader contract,
 *                       file_finder.py:143-201)
 *   sl_env_obs          SafeLifeEnv.get_obs (safelife_env.py:125-155) +
 *                       recenter_view (helper_utils.py:41-74)
 *   sl_side_effect_densities  side_effect_score's rollout + density maps
 *                       (side_effects.py:59-92,131-139), batched over episodes
 *   sl_level_pool_prepare  derived pool data for the device level pool
 *                       (levels as loaded by safelife_game.py:184-212)
 *   sl_sample_actions   np.random.choice(len(policy), p=policy) per env in
 *                       PPO.run_agents (training/ppo.py:440)
 *   sl_gae              returns + advantages of PPO.gen_training_batch
 *                       (training/ppo.py:487-503)
 */
#ifndef SAFELIFE_HIP_H
#define SAFELIFE_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SL_OK 0
#define SL_EINVAL (-1)      /* bad shape or argument */
#define SL_EHIP (-2)        /* HIP runtime / launch error */
#define SL_ETOOBIG (-3)     /* board too large for the selected kernel */

#define SL_RNG_STREAM 0     /* replay a supplied uniform stream (reference order) */
#define SL_RNG_PHILOX 1     /* counter-based Philox4x32-10 (production): the four
                               cells of a 2x2 block share one evaluation,
                               counter (block, env, step, tensor), 32-bit words */

#define SL_KERNEL_AUTO 0     /* bit-sliced kernels for 64x64, 128x128 and boards
                                up to 32x64 (both RNG modes; replay adds an
                                action kernel, a count kernel and a scan per
                                step), the generic
                                kernel for other shapes                      */
#define SL_KERNEL_GENERIC 1  /* LDS-staged per-cell kernel, any shape        */
#define SL_KERNEL_FAST 2     /* require the fast kernel (error if none)      */

/* bits of the replay stream's error flag (scratch word 8B, sl_env_cfg.scratch) */
#define SL_STREAM_ERR_RANGE 1      /* the supplied stream ran out, or the device
                                      generator could not serve a step's draw range
                                      (ring too small, or rewound): re-seed / enlarge */
#define SL_STREAM_ERR_THRESHOLD 2  /* a bit ring (sl_mt19937.bit_ring) served an env
                                      whose spawn threshold is not the ring's */

/* sl_env_cfg.board_mode: a 128x128 step without capture -- with no views, or with
 * packed views of at most 96 rows -- keeps the board in sl_env_state.board_planes
 * (SL_BOARD_AUTO) and writes only a few uint16 rows; a caller that reads the uint16
 * board after (nearly) every step asks for it whole instead (SL_BOARD_UINT16: the step
 * kernel writes every changed row, and no sync is needed before a read) */
#define SL_BOARD_AUTO 0
#define SL_BOARD_UINT16 1

#define SL_MAX_EXITS 8      /* exits tracked per env (benchmark levels have 1) */
#define SL_BONUS_PERIOD_MAX 16

#define SL_OBS_NONE 0
#define SL_OBS_PACKED 1     /* uint16 [B, vh, vw]           (output_channels=None) */
#define SL_OBS_CHANNELS 2   /* uint16 [B, vh, vw, nch]      (output_channels=(...)) */
#define SL_OBS_CHANNELS_U8 3 /* uint8 [B, vh, vw, nch]      (same values, 1 byte)  */
#define SL_OBS_CHANNELS_F32 4 /* float [B, vh, vw, nch]     0.0 / 1.0: the policy's
                                 layer0 (training/safelife_ppo.py:147-152)        */
#define SL_OBS_CHANNELS_BF16 5 /* bfloat16 [B, vh, vw, nch] 0.0 / 1.0             */

/* Library / device info. */
const char *sl_version(void);
const char *sl_build_id(void);   /* hash of the sources this library was built from */
int sl_device_arch(char *buf, int len);   /* e.g. "gfx950" */

/* Timing events (hipEvent_t as void*) for in-process kernel timing. */
int sl_event_create(void **ev);
int sl_event_destroy(void *ev);
int sl_event_elapsed_ms(void *begin, void *end, float *ms);   /* after completion */
/* Bandwidth reference for roofline reporting (not on the env path): copies n16
 * 16-byte words src -> dst (dev, 16-B aligned) with a grid-stride vector kernel
 * (1024 workgroups, one load per lane per iteration) -- what a plain streaming
 * read+write of the same bytes draws on this GPU. */
int sl_copy16(const void *src, void *dst, int64_t n16, void *stream);

/* ---------------------------------------------------------------- boards -- */

/*
 * Advance B independent boards one step: out[b] = rule(in[b]).
 *   in, out      dev uint16 [B,H,W]; must not alias.  H, W >= 2.
 *   spawn_prob   dev float [B] or NULL (then spawn_prob_scalar for all boards);
 *                each draw u spawns iff u < (double)spawn_prob (a C float, as
 *                the reference parses it with format "f", module.c:22-24).
 *   rng_mode     SL_RNG_STREAM: board b consumes draws[draw_offsets[b] + k] for
 *                its k-th eligible cell in row-major order (draws/draw_offsets
 *                may be NULL when no board can draw: p <= 0 or p >= 1 decide
 *                without a draw).  SL_RNG_PHILOX: u = philox(seed; cell, env0+b,
 *                step, tensor).
 */
int sl_advance(const uint16_t *in, uint16_t *out, int64_t B, int H, int W,
               const float *spawn_prob, float spawn_prob_scalar, int rng_mode,
               uint64_t seed, uint32_t env0, uint32_t step, uint32_t tensor,
               const double *draws, const int64_t *draw_offsets, void *stream);

/* counts[b] = number of uniform draws board b consumes in one advance. */
int sl_count_eligible(const uint16_t *in, int64_t *counts, int64_t B, int H, int W,
                      void *stream);

/*
 * HOST advance of one board (no GPU; csrc/sl_host.cpp): speedups.advance_board's
 * numpy path (module.c:19-44 for a numpy board).
 *   in, out      host uint16 [H,W], row-major, must not alias; 2 <= H, 2 <= W <= 512.
 *   draws        the caller's next n_draws spawn uniforms in reference order (one
 *                per eligible cell, row-major, random.c:47-52).
 * Returns the uniforms consumed (>= 0); -(needed + 1) when the board needs more
 * than n_draws (out unspecified: call again with `needed`); with out == NULL, the
 * number of eligible cells; INT64_MIN for a bad shape.  Thread-safe.
 */
int64_t sl_host_advance(const uint16_t *in, uint16_t *out, int64_t H, int64_t W,
                        float spawn_prob, const double *draws, int64_t n_draws);

/* out[i] = base + sum_{j<i} in[j]; *total_out (dev, may be NULL) = base + sum. */
int sl_exclusive_scan_i64(const int64_t *in, int64_t *out, int64_t n,
                          const int64_t *base, int64_t *total_out, void *stream);

/* -------------------------------------------- seeded reference stream -- */

/*
 * The reference's spawn stream on the device: numpy's legacy RandomState(seed)
 * .random_sample() -- MT19937 seeded by init_genrand, doubles (a >> 5, b >> 6) / 2^53
 * from consecutive outputs -- which speedups.seed(seed) makes the reference draw
 * from in 10 000-double chunks (speedups_src/random.c:14-26,28-44,47-52,
 * module.c:246-253).  Draw d lands in ring[d & (ring_draws - 1)].
 *
 * The stream is cut into blocks of 624 * rounds raw outputs (312 * rounds draws);
 * block q is generated by chain q mod n_chains, whose state then jumps n_chains
 * blocks ahead (x^(n_chains * block) mod the characteristic polynomial, applied
 * to the block's own first raw words).  All buffers are caller-allocated device
 * memory:
 *   chains   uint32 [n_chains, 624]          the MT state of each chain's next block
 *   prefix   uint32 [n_chains, SL_MT_PREFIX] scratch
 *   polys    uint32 [log2(n_chains) + 1, SL_MT_POLY_WORDS] jump polynomials
 *   ctl      int64 [SL_MT_CTL_WORDS] (8): [0] next block to generate, [1] a done
 *            counter, [2] error flags (bit0: a fill asked for a range the ring or
 *            the chains cannot serve), [3] the first block, [4] the next block whose
 *            chain has to jump, [5] a done counter, [6] and [7] the last fill's draw
 *            range [lo, hi) (written by every fill, read by the look-ahead)
 * n_chains is a power of two (one fill generates at most n_chains blocks), rounds
 * >= 33, ring_draws a power of two >= 2 blocks.
 */
#define SL_MT_PREFIX 21216       /* 34 x 624 raw words */
#define SL_MT_CTL_WORDS 8
#define SL_MT_POLY_WORDS 640
typedef struct sl_mt19937 {
    int32_t n_chains;
    int32_t rounds;
    int64_t ring_draws;
    double *ring;
    uint32_t *chains;
    uint32_t *prefix;
    uint32_t *polys;
    int64_t *ctl;                   /* dev int64 [SL_MT_CTL_WORDS] */
    /* look-ahead (sl_mt19937_lookahead): after each fill, the blocks of the next
     * fill's likely range are generated on this second stream, beside the step that
     * consumes the current range; the next fill waits for them.  NULL = off.  The
     * event handles and the flag are the library's. */
    void *ahead_stream;
    void *ev_fill, *ev_ahead;
    int32_t ahead_pending;
    /* bit ring (round 5): bit_ring != 0 makes `ring` a ring of decisions -- draw d is
     * bit (d & 31) of uint32 word (d & (ring_draws - 1)) >> 5 of ring (read as
     * uint32_t, ring_draws / 8 bytes), set iff the draw's double is < bits_thr -- for
     * batches whose envs all spawn with that one threshold (double)(float)p: the
     * replay kernels need only u < p, and the ring then holds 1/64 of the bytes.
     * rounds must be a multiple of 4 (a block's draws fill whole words).  A step in
     * which an env that draws has another threshold sets bit 1 of the stream error
     * flag (SL_STREAM_ERR_THRESHOLD; bit 0 stays the ring's range error).
     * bit_ring == 0 (a zeroed struct): a ring of doubles, bits_thr unused. */
    int32_t bit_ring;
    double bits_thr;
} sl_mt19937;

/* Seed: the stream of RandomState(seed), positioned so that draws from first_draw
 * on can be generated (host polynomial work, then device init; synchronises
 * `stream`).  Re-seed to move the position backwards. */
int sl_mt19937_seed(sl_mt19937 *mt, uint32_t seed, int64_t first_draw, void *stream);
/* Generate every not yet generated block holding a draw below *hi (dev int64);
 * *lo (dev) is the first draw the caller will read.  err (dev int64, may be NULL)
 * is OR-ed with 1 when the range cannot be served (re-seed).  With the look-ahead
 * on, `stream` first waits for the last fill's look-ahead, and after the fill the
 * blocks of [*hi, *hi + 1.25 (*hi - *lo)) (capped by the ring) are generated on the
 * look-ahead stream; mt's flag is updated (mt is const for the device state only). */
int sl_mt19937_fill(const sl_mt19937 *mt, const int64_t *lo, const int64_t *hi, int64_t *err,
                    void *stream);
/* Turn the look-ahead on (ahead_stream = a hipStream_t) or off (NULL); creates /
 * keeps the two events.  sl_mt19937_release destroys them (the device buffers are
 * the caller's). */
int sl_mt19937_lookahead(sl_mt19937 *mt, void *ahead_stream);
int sl_mt19937_release(sl_mt19937 *mt);
/* Host reference pieces (no GPU): the seeded window, x^n mod phi, a jump of a
 * window by a polynomial, and n draws from a window (tests; seeding). */
int sl_mt19937_host_window(uint32_t seed, uint32_t *window624);
int sl_mt19937_host_jump_poly(uint64_t n, uint32_t *poly);
int sl_mt19937_host_jump(const uint32_t *window_in, const uint32_t *poly, uint32_t *window_out);
int sl_mt19937_host_draws(const uint32_t *window, int64_t n, double *out);

/* ------------------------------------------------------- side effects -- */

/*
 * The rollout + density half of side_effect_score (side_effects.py:59-92,
 * 131-139) for E finished episodes at once.  Per episode e: b0 = init_board[e]
 * is advanced num_steps[e] times, then num_samples times alternately with
 * b1 = final_board[e] (b0 then b1, the reference's order); after each of those
 * advances both boards are added to their cell-type density maps
 * (_add_cell_distribution), which are finally divided by num_samples.
 *   num_steps_dev / num_steps_host  the same [E] values, device and host copy
 *   spawn_prob     dev float [E]
 *   rng_mode       SL_RNG_STREAM: E must be 1; draws are consumed from
 *                  draws[*stream_pos] on in the reference's order (advanced);
 *                  SL_RNG_PHILOX: u = philox(seed; cell, env0 + e, advance
 *                  index of that board, 4 + (0: b0, 1: b1)).
 *   keys           dev uint16 [E, max_keys]: the union of both maps' cell-type
 *                  keys, ascending; n_keys dev [E] its size (> max_keys means
 *                  the maps are incomplete: raise max_keys); present dev
 *                  [E, max_keys]: bit0 key occurs in the inaction map (b0),
 *                  bit1 in the action map (b1)
 *   inaction, action  dev double [E, max_keys, H, W] densities per key
 *   workspace      dev scratch of sl_side_effect_workspace() bytes
 * max_keys <= 1024.  The earth mover's distance over the maps
 * (side_effects.py:12-56, third-party pyemd) is host code above this call.
 */
/*
 * Earth mover's distance of side_effect_score (host code; no GPU needed).
 * Replaces pyemd.emd(a[changed], b[changed], dist, extra_mass_penalty) at
 * /root/reference/safelife/side_effects.py:56 (its caller's cell selection and
 * ground distance: side_effects.py:36-55).
 *   p, q         host double [n]: the two densities at the n selected cells
 *   ys, xs       host int32 [n]: the cells' row / column on an H x W board
 *   cost_table   host double [2H-1][2W-1]: ground distance between two cells by their
 *                signed offset (y_i - y_j + H - 1, x_i - x_j + W - 1)
 *   extra_mass_penalty  per unit of |sum p - sum q|; -1: the largest distance used
 *   out          the distance (FastEMD emd_hat semantics, see sl_emd.cpp)
 */
int sl_emd_cells(const double *p, const double *q, const int32_t *ys, const int32_t *xs,
                 int64_t n, const double *cost_table, int H, int W,
                 double extra_mass_penalty, double *out);

int sl_side_effect_workspace(int64_t E, int H, int W, int64_t *bytes);
int sl_side_effect_densities(const uint16_t *init_board, const uint16_t *final_board,
                             const int32_t *num_steps_dev, const int32_t *num_steps_host,
                             const float *spawn_prob, int64_t E, int H, int W,
                             int num_samples, int rng_mode, uint64_t seed, uint32_t env0,
                             const double *draws, int64_t *stream_pos, int max_keys,
                             uint16_t *keys, int32_t *n_keys, int32_t *present,
                             double *inaction, double *action, void *workspace,
                             int64_t workspace_bytes, void *stream);

/* ------------------------------------------------------------------ envs -- */

/* Per-env state, structure of arrays, all dev pointers, length B unless noted. */
typedef struct sl_env_state {
    int64_t B;
    int32_t H, W;
    uint16_t *board;          /* [B,H,W]  game.board                          */
    uint16_t *goals;          /* [B,H,W]  game.goals                          */
    uint16_t *start_board;    /* [B,H,W]  game._init_data['board']            */
    int32_t *agent_x, *agent_y, *orientation;
    int32_t *game_over;
    int32_t *episode_length;
    int32_t *episode_reward;  /* SafeLifeEnv's own (integer) reward sum       */
    int32_t *old_points;      /* SafeLifeEnv._old_game_value                  */
    int32_t *baseline;        /* perf baseline over _init_data (per episode)  */
    int32_t *score;           /* current perf score (unit rewards)            */
    int32_t *possible;        /* perf possible score                          */
    int32_t *side_effect;     /* SimpleSideEffectPenalty.last_side_effect     */
    float *spawn_prob;
    double *min_performance;  /* game.min_performance                         */
    int32_t *prior_x;         /* [B, SL_BONUS_PERIOD_MAX] position ring        */
    int32_t *prior_y;
    int32_t *prior_len;       /* entries in the ring (deque length)           */
    int32_t *prior_head;      /* index of the oldest entry                    */
    int32_t *exit_count;
    int16_t *exit_y, *exit_x; /* [B, SL_MAX_EXITS], np.nonzero order          */
    int32_t *level_index;     /* level of the current episode                 */
    int32_t *episodes;        /* episodes started by this env                 */
    int32_t *num_steps;       /* game.num_steps                               */
    int32_t *spawn_flags;     /* bit0: board, bit1: goals may hold a spawning
                                 cell (set at reset; spawning bits are never
                                 created by the rule or the actions -- except a
                                 power toggle, which the kernels allow for -- only
                                 moved).  The replay prologues skip the eligible
                                 count of a tensor whose bit is clear: a caller
                                 writing state sets both bits.
                                 128x128 boards only (0 on other shapes):
                                 bit2: the start board may use cell bits 12-14
                                 (no cell type does; set at reset from the level):
                                 the 128x128 kernel keeps no start planes for them
                                 and takes such an env's exact side-effect term in
                                 a second pass.  A caller writing start boards
                                 sets it where they carry those bits.
                                 bit3: a goal cell uses bits other than alive,
                                 destructible, frozen and colours (set at reset):
                                 with bits 1 and 3 clear the 128x128 kernel keeps
                                 the goals' six planes in the mirror and reads
                                 them from there.                              */
    int32_t *start_roll;      /* (dy << 16) | dx: start_board[b] equals pool
                                 level level_index[b] rolled by (dy, dx) (set by
                                 every reset); -1: start_board was written by
                                 the caller.  Lets the 64x64 kernel read the
                                 start board from the cache-resident pool.     */
    uint32_t *planes;         /* bit-plane mirror of the goals kept by the
                                 bit-sliced kernels, or NULL (then 128x128
                                 boards take the generic kernel).
                                 64x64: [B,2,32,64], half 1 (half 0 reserved):
                                 [b][1][q][lane], word q = plane q & 15 of
                                 column 2(lane>>1) + (q>>4), rows
                                 32(lane&1)..+31 (sl_bits.hip).
                                 128x128: [B,4,32,64], [b][t][q][lane], word q
                                 = plane q & 15 of column 2 lane + (q>>4),
                                 rows 32t..32t+31 (sl_bits128.hip).
                                 Derived data, never read unless planes_ok
                                 bit 1 is set.                                 */
    int32_t *planes_ok;       /* [B] bit1: goals mirror valid; bit2: goals at
                                 a fixed point (no spawner, unchanged by the
                                 last step: the rule is skipped); bit3: the
                                 board's draw planes (elig_planes) hold its
                                 eligible cells as the last step left them;
                                 bit4 (128x128): the mirror holds all six goal
                                 planes (spawn_flags bit3), not only colours;
                                 bit5 (128x128): the goals are the pool level's,
                                 as reset (set by the reset, cleared by the first
                                 change): their colours come from the pool's
                                 goal_planes; bit6 (128x128): board_planes hold
                                 the board; bit7: with bit6, the uint16 board
                                 is complete too (else only its band-edge rows);
                                 bit8: with bit6, the board's planes 12-14 are
                                 zero and not kept.
                                 Anything
                                 that writes the goals other than the 64x64
                                 kernel and its reset clears it.               */
    uint32_t *elig_planes;    /* replay mode, 128x128, [B][1024] words: the
                                 draw planes [tensor][band t][word w][lane] (bit
                                 y of word w of lane j = cell (32t + y, 2j + w)).
                                 The step kernel leaves the advanced board's
                                 eligible cells in tensor 0's (planes_ok bit 3);
                                 the next step's count patches the rows its
                                 action edited and counts them; the draw pass
                                 replaces each drawing tensor's eligible cells
                                 with those whose uniforms spawn, before the
                                 step kernel runs.  Or NULL (the step kernel
                                 then ranks and draws itself)                  */
    uint32_t *board_planes;   /* 128x128, or NULL: [B,4,32,64] u32 in the goals
                                 mirror's layout ([b][t][q][lane], word q =
                                 plane q & 15 of column 2 lane + (q >> 4), rows
                                 32t..32t+31).  When set, a step of the fast
                                 kernel without capture -- Philox or replay with
                                 draw planes; no obs_out, or packed views of at
                                 most 96 rows, which it writes from the planes;
                                 sl_env_cfg.board_mode SL_BOARD_AUTO -- keeps
                                 the board here (planes_ok bit6) and writes of
                                 the uint16 board only its band-edge rows (32t,
                                 32t + 31) and the cells the action and exits
                                 edit: bit7 then says the uint16 board is
                                 complete.  sl_env_board_sync completes it (a
                                 per-env no-op for envs not in planes or
                                 already complete); the library's other entry
                                 points that read or write st->board do so
                                 themselves.  A caller that writes the uint16
                                 board clears planes_ok (as for the goals
                                 mirror).  64x64: board_planes == planes puts
                                 the board's planes in half 0 of the goals
                                 mirror (Philox steps without views; bit 7
                                 only after a sync or a reset).                */
    uint32_t board_zero;      /* plane mode (64x64, 128x128): cell bits (planes) that are
                                 0 in every board of the batch and that no rule,
                                 action or reset can set (the caller's promise:
                                 none in its levels or written boards, not
                                 LIFE / COLOR_R, not toggled powers / colours);
                                 their planes are neither loaded nor stored.
                                 To widen it, complete the board first
                                 (sl_env_board_sync) and clear planes_ok bits
                                 6-7.  0 = every plane.                        */
    int32_t planes_live;      /* host flag, kept by the library: a plane-mode
                                 step set it (some board may be in planes);
                                 a demotion clears it.  While 0 the syncs the
                                 entry points run are skipped.  Zero-init; a
                                 caller stepping a slice (a copy of this
                                 struct) ORs the slice's flag back in.         */
} sl_env_state;

/* A device-resident level pool (the level_iterator's levels). */
typedef struct sl_level_pool {
    int32_t K, H, W;
    const uint16_t *board;    /* [K,H,W] as stored (exits uncoloured)         */
    const uint16_t *goals;    /* [K,H,W]                                      */
    const int32_t *agent_x, *agent_y, *orientation;
    const float *spawn_prob;
    const double *min_performance;  /* the level's own value (used for the
                                       reset-time exit colour only)           */
    uint64_t *board_planes;   /* bit planes of the pool boards, or NULL
                                 (sl_level_pool_prepare; the bit-sliced kernels'
                                 start-board source):
                                 64x64 pools: uint64 [K,16,W], element [k][p][x]
                                 bit y = bit p of board[k][y][x];
                                 128x128 pools: uint32 [K,16,4,W] (8*K*16*W
                                 bytes), element [k][p][q][x] bit r = bit p of
                                 board[k][32q + r][x]                          */
    uint32_t *goal_planes;    /* 128x128 pools: the goals' colour planes, uint32
                                 [K,3,4,W], element [k][c][q][x] bit r = bit 9+c
                                 of goals[k][32q + r][x]; or NULL.  The 128x128
                                 kernel scores goals still as the level had them
                                 from here (cache-resident) instead of the
                                 env's mirror (sl_level_pool_prepare fills it) */
} sl_level_pool;

/* Fill pool->board_planes (caller-allocated, dev, layout above; H must be 64 or
 * 128) from pool->board.  Derived data only; the reference keeps levels as npz
 * (safelife_game.py:184-194). */
int sl_level_pool_prepare(sl_level_pool *pool, void *stream);

/*
 * Trajectory capture (SafeLifeRecorder, /root/reference/safelife/env_wrappers.py:97-136):
 * sl_env_step copies the state of n chosen envs twice per step -- right after the
 * board advance, before any reset (the frame the reference captures after
 * env.step), and after the step's resets (the first frame of the next episode,
 * meaningful where flags & 4).  Copies only; the stepping itself is unchanged.
 */
typedef struct sl_capture {
    int32_t n;                    /* envs recorded (0: none)                       */
    const int32_t *env;           /* dev [n] env indices                           */
    uint16_t *board, *goals;      /* dev [n, H, W]  after the advance              */
    int32_t *orientation;         /* dev [n]                                        */
    uint8_t *flags;               /* dev [n]  the step's info flags                */
    uint16_t *reset_board, *reset_goals;   /* dev [n, H, W]  after the resets     */
    int32_t *reset_orientation;   /* dev [n]                                        */
} sl_capture;

typedef struct sl_env_cfg {
    int32_t time_limit;             /* SafeLifeEnv.time_limit (1000)          */
    int32_t auto_reset;             /* 1: ContinuingEnv + caller reset-on-done */
    int32_t can_toggle_powers, can_toggle_colors;
    double penalty_coef;            /* SimpleSideEffectPenalty (scheduled)    */
    double wrapper_min_performance; /* SimpleSideEffectPenalty.min_performance;
                                       applied at reset (NaN = keep level's)  */
    const double *bonus_table;      /* dev [bonus_len]: movement_bonus *
                                       (d/period)**power for integer d        */
    int32_t bonus_len;
    int32_t bonus_period;           /* movement_bonus_period (<= 16; 0 = off) */
    int32_t rng_mode;               /* SL_RNG_*                               */
    uint64_t seed;
    uint32_t step;                  /* batched-step index (Philox counter)     */
    uint32_t env0;                  /* global id of env 0 (multi-GPU shards)   */
    const double *draws;            /* SL_RNG_STREAM: dev uniform stream       */
    int64_t n_draws;
    int64_t *stream_pos;            /* dev [1]: next unread draw (advanced)    */
    int64_t *scratch;               /* dev [8*B + 16] workspace, zeroed once
                                     * before the first step (layout:
                                     * sl_env_common.h Scratch).  With auto_reset the
                                     * 64x64 / 128x128 kernels queue finished envs
                                     * in per-parity lists (words 8B+2, 8B+3) that
                                     * stay valid only over consecutive steps
                                     * (step, step+1, ...) with auto_reset set: zero
                                     * words 8B+2..8B+3 again after any other
                                     * sequence (rewound step index, auto_reset
                                     * toggled, state written by the caller)     */
    int32_t level_mode;             /* 0: level = (env0+b + episodes*n_total)%K,
                                       1: Philox-random level                  */
    int32_t n_total_envs;           /* envs across all shards                  */
    int32_t augment_roll;           /* 1: random toroidal roll per episode     */
    void *ev_begin, *ev_end;        /* optional hipEvent_t pair recorded right
                                       before and after the board-advance (step)
                                       kernel's launch (profiling; an event record
                                       holds the next dispatch until written)  */
    int32_t kernel;                 /* SL_KERNEL_*: which advance kernel       */
    void *obs_out;                  /* dev: sl_env_step also writes every env's
                                       observation after the step (auto-resets
                                       included), exactly as sl_env_obs with the
                                       fields below would; NULL = no observation.
                                       The 64x64 kernel writes packed views from
                                       the board it holds on chip (no re-read) */
    int32_t obs_mode, obs_vh, obs_vw, obs_remove_white, obs_nch;
    int32_t obs_channels[16];
    const sl_capture *capture;      /* host pointer or NULL: trajectory capture
                                       (needs auto_reset and info_flags)      */
    int32_t stream_phase;           /* SL_RNG_STREAM with the batch split over
                                       shards (SURVEY §8(e) collective 3: the
                                       reference's one stream runs env after env
                                       over ALL shards, training/ppo.py:436-452):
                                       0 = the whole step, this batch alone;
                                       1 = count phase: the actions, then each
                                       env's eligible cells; *stream_pos = this
                                       batch's draw total (no draw, no advance);
                                       2 = draw phase (after a phase-1 call on the
                                       same state): this batch's draws start at
                                       *stream_base -- the global position plus
                                       the totals of the shards before it --, the
                                       step completes, *stream_pos = *stream_base
                                       + the batch's total                     */
    const int64_t *stream_base;     /* dev [1]: phase 2's first uniform        */
    const sl_mt19937 *mt;           /* SL_RNG_STREAM: host pointer or NULL.  When
                                       set, the draws come from this device
                                       generator's ring (draws / n_draws are not
                                       read): after the offsets scan each step
                                       fills it for the step's range, so the
                                       stream is RandomState(seed) from
                                       *stream_pos on with no host buffer      */
    int32_t board_mode;             /* SL_BOARD_*: where a 128x128 step leaves the
                                       board (sl_env_state.board_planes)       */
} sl_env_cfg;

/*
 * One env-step for all B envs (in place on `st`).
 *   actions     dev int32 [B], 0..8 (safelife_env.py:61-71)
 *   reward      dev double [B]      chain reward (float64, as Python computes it)
 *   done        dev uint8 [B]       done as returned to the caller (times_up)
 *   info_flags  dev uint8 [B] or NULL: bit0 times_up, bit1 game_over,
 *               bit2 env was reset this step
 *   ep_len, ep_reward  dev int32 [B] or NULL: finished-episode length / reward
 * With cfg->auto_reset the done/game-over envs are reset from `pool` before
 * returning (so the next sl_env_obs sees the new episode); the 64x64 kernel
 * does this inside the step kernel, the other paths with a second kernel.
 */
int sl_env_step(sl_env_state *st, const sl_level_pool *pool, const int32_t *actions,
                const sl_env_cfg *cfg, double *reward, uint8_t *done,
                uint8_t *info_flags, int32_t *ep_len, int32_t *ep_reward,
                void *stream);

/* Complete the uint16 board of every env whose board lives in st->board_planes
 * (planes_ok bit6 without bit7): needed before reading st->board directly after
 * steps that kept the board in planes.  No-op without board_planes. */
int sl_env_board_sync(sl_env_state *st, void *stream);

/* Reset the envs with mask[b] != 0 (mask NULL = all) from `pool`. */
int sl_env_reset(sl_env_state *st, const sl_level_pool *pool, const uint8_t *mask,
                 const sl_env_cfg *cfg, void *stream);

/*
 * Observations centred on each agent.
 *   obs_mode SL_OBS_PACKED: out uint16 [B,vh,vw]; SL_OBS_CHANNELS: uint16
 *   [B,vh,vw,nch] with channel k = bit channels[k]; SL_OBS_CHANNELS_U8: uint8;
 *   SL_OBS_CHANNELS_F32 / _BF16: the same bits as 0.0 / 1.0 floats.
 *   channels: host int array [nch] (<= 16) -- copied into kernel arguments.
 */
int sl_env_obs(const sl_env_state *st, int vh, int vw, int remove_white_goals,
               int obs_mode, const int32_t *channels, int nch, void *out,
               void *stream);

/* ------------------------------------------------- game-level pieces -- */
/*
 * The SafeLifeGame methods sl_env_step fuses, one at a time, for callers that drive
 * the game directly (/root/reference/safelife/safelife_game.py).  A state struct
 * whose pointers are offset by i0 envs (B = n) addresses envs [i0, i0 + n).
 *
 * sl_env_action       execute_action / move_agent / relative_loc
 *                     (safelife_game.py:294-393) for actions 0..8 of
 *                     safelife_env.py:61-71: the board cells, agent, orientation
 *                     and game_over in place.  act: dev int64 [4*B]: act[b] = the
 *                     action's reward (points_on_level_exit), act[B+b], [2B+b],
 *                     [3B+b] = its change to points / perf score / side effects.
 *                     The exit check reads score / possible (sl_env_rescore).
 * sl_env_advance      SafeLifeGame.advance_board (safelife_game.py:657-660): per env
 *                     num_steps += 1, board then goals advanced.  RNG from cfg
 *                     (rng_mode, seed, step, env0, draws / n_draws / stream_pos:
 *                     replay consumes env after env, board then goals, exactly as
 *                     two speedups.advance_board calls per env do), cfg->scratch
 *                     as for sl_env_step; the other cfg fields are not read.
 * sl_env_rescore      current_points (safelife_game.py:590-599) -> points (dev
 *                     int32 [B] or NULL) and performance_ratio's score terms
 *                     (:601-631) -> st->score, st->possible, for the current board.
 * sl_env_exit_colors  mode 0: update_exit_colors (safelife_game.py:528-537) from
 *                     st->score / possible / baseline / min_performance;
 *                     mode 1: exit cells set back to their start-board values.
 */
int sl_env_action(sl_env_state *st, const int32_t *actions, int can_toggle_powers,
                  int can_toggle_colors, int64_t *act, void *stream);
int sl_env_advance(sl_env_state *st, const sl_env_cfg *cfg, void *stream);
int sl_env_rescore(sl_env_state *st, int32_t *points, void *stream);
int sl_env_exit_colors(sl_env_state *st, int mode, void *stream);

/* ------------------------------------------------------- PPO caller -- */

/*
 * actions[b] = np.random.choice(A, p=probs[b]) (numpy's legacy RandomState.choice:
 * p taken as float64, cdf = cumsum(p) / cdf[-1], index = #{k : cdf[k] <= u}).
 *   probs       dev float32 (probs_f64 = 0) or float64 [B, ld], first A used
 *   rng_mode    SL_RNG_STREAM: u = uniforms[b] (dev double [B], e.g. the global
 *               numpy stream); SL_RNG_PHILOX: u = philox(seed; 0, env0 + b, step, 2)
 *   atol        numpy's tolerance on |sum(p) - 1| (sqrt(eps) of float64, or of
 *               the probabilities' dtype when larger)
 *   err         dev uint8 [B] or NULL: bit0 some p < 0, bit1 |kahan_sum(p) - 1|
 *               > atol -- the ValueErrors numpy raises; the caller raises them
 */
int sl_sample_actions(const void *probs, int probs_f64, int64_t B, int A, int64_t ld,
                      int rng_mode, const double *uniforms, uint64_t seed, uint32_t env0,
                      uint32_t step, double atol, int32_t *actions, uint8_t *err,
                      void *stream);

/*
 * Discounted returns and GAE advantages over a rollout of T steps x N envs with G
 * discount factors, in the reference's dtypes and evaluation order:
 *   rewards      dev double [T, N]   (clipped to +-reward_clip when > 0)
 *   end_episode  dev uint8 [T, N]
 *   values       dev float [T+1, N, G]
 *   gamma, lmda  dev float [G]       (lmda = the reference's lmda * gamma, float32)
 *   returns, advantages  dev double [T, N, G]
 */
int sl_gae(const double *rewards, const uint8_t *end_episode, const float *values,
           const float *gamma, const float *lmda, int G, int T, int64_t N,
           double reward_clip, double *returns, double *advantages, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* SAFELIFE_HIP_H */
