// sl_env_common.h -- pieces shared by the env-step kernels (generic and fast paths).
#pragma once
#include "sl_device.h"
#include "../../include/safelife_hip.h"

namespace sl {

// scratch layout (int64 words), see sl_env_cfg.scratch (8*B + 16 words):
//   [0, 2B)   per-(env, tensor) draw counts (replay mode; consumed by the scan before
//             the step kernel runs); its first B int32 slots then hold the list of
//             envs to reset after the step (64x64 and 128x128 kernels)
//   [2B, 4B)  per-(env, tensor) stream offsets   (replay mode)
//   [4B, 8B)  per env: action reward, d_points, d_score, d_side of the action's
//             cell edits (the generic path; the bit-sliced replay prologues write
//             the reward only; 128x128 replay with elig_planes: [B, 2B) holds the
//             rows the action edited, then the tensors that draw, bit0 board, bit1 goals;
//             [2B, 3B) the count of the board eligibility the step left)
//   [8B]      error flags (bit0: draw stream exhausted)
//   [8B+2], [8B+3]  reset-list lengths for even / odd steps (each step's reset
//             kernel zeroes the other one)
struct Scratch {
    int64_t *counts, *offsets, *act, *err;
};
__host__ __device__ inline Scratch scratch_of(int64_t *s, int64_t B) {
    return Scratch{s, s + 2 * B, s + 4 * B, s + 8 * B};
}
__host__ __device__ inline int32_t *reset_list(int64_t *s) { return reinterpret_cast<int32_t *>(s); }

// the board planes a cell's spawn eligibility reads (alive, frozen, inhibiting,
// spawning): what the 128x128 replay paths evaluate eligibility from
__host__ __device__ constexpr int elig_plane(int s) { return s == 0 ? 0 : (s == 1 ? 4 : s + 4); }
// sl_env_state.elig_planes per env (u32 words): the draw planes
// [tensor][band][word][lane] of the 128x128 replay.  The step kernel leaves the
// eligible cells of its advanced board in tensor 0's planes (the next step's
// eligibility before the action); k_stream_prologue128 patches the rows the action
// edited, counts, and leaves each drawing tensor's eligible cells there;
// k_stream_draw128 replaces them with the cells that spawn; the step kernel reads those
constexpr int kEligStride = 1024, kDrawPlanes = 0;

struct StepArgs {
    int32_t time_limit, auto_reset, bonus_len, bonus_period;
    double penalty_coef;
    const double *bonus_table;
    uint64_t seed;
    uint32_t step, env0;
    const double *draws;
    int64_t n_draws;
    int64_t draw_mask = -1;      // draw r is draws[r & draw_mask]: -1 for a linear buffer,
                                 // ring_draws - 1 for the device generator's ring (sl_mt.hip)
    const uint32_t *draw_bits = nullptr;   // the generator's bit ring (sl_mt19937.bit_ring):
                                           // draw r below the ring's threshold iff bit r
    double bits_thr = -1.0;                // that threshold
};

// Stream draw r as the replay kernels compare it (u < the env's threshold): the
// supplied / generated double, or from a bit ring -1.0 (below) / 2.0 (not below) --
// exact for an env whose threshold is the ring's (stream_offsets checks every drawing
// env's, bits_thr_check)
__device__ __forceinline__ double stream_u(const double *draws, const uint32_t *bits, int64_t r,
                                           int64_t mask) {
    const int64_t i = r & mask;
    if (bits) return ((bits[i >> 5] >> (i & 31)) & 1u) ? -1.0 : 2.0;
    return draws[i];
}

__device__ __forceinline__ int pymod(int a, int m) {
    int r = a % m;
    return r < 0 ? r + m : r;
}

__device__ __forceinline__ bool can_exit_now(double mp, int score, int baseline, int possible) {
    if (mp < 0.0) return true;
    // no contraction: Python evaluates the product, then compares
    return (double)(score - baseline) >= __dmul_rn(mp, (double)(possible - baseline));
}

// movement-bonus distance (MovementBonusWrapper.step, env_wrappers.py:72-80): from
// the oldest ring position, padded by the missing entries while the ring fills;
// clamped to the table (bonus_table[d] = bonus * (d / n) ** power, host-computed)
__device__ __forceinline__ int bonus_dist(int ax, int ay, int px, int py, int len, int n,
                                          int bonus_len) {
    const int d = (len > 0) ? abs(ax - px) + abs(ay - py) + (len < n ? n - len : 0) : n;
    return min(d, bonus_len - 1);
}

// Reads of the per-env fields the epilogue needs, straight from sl_env_state.
// The 64x64 kernel substitutes a prefetched copy (sl_bits.hip).
struct GlobalFields {
    const sl_env_state &st;
    int64_t b;
    const double *bonus_table;
    __device__ int old_points() const { return st.old_points[b]; }
    __device__ int num_steps() const { return st.num_steps[b]; }
    __device__ int episode_length() const { return st.episode_length[b]; }
    __device__ int episode_reward() const { return st.episode_reward[b]; }
    __device__ double min_performance() const { return st.min_performance[b]; }
    __device__ int baseline() const { return st.baseline[b]; }
    __device__ int exit_count() const { return st.exit_count[b]; }
    __device__ int exit_y(int e) const { return st.exit_y[b * SL_MAX_EXITS + e]; }
    __device__ int exit_x(int e) const { return st.exit_x[b * SL_MAX_EXITS + e]; }
    __device__ int game_over() const { return st.game_over[b]; }
    __device__ int agent_x() const { return st.agent_x[b]; }
    __device__ int agent_y() const { return st.agent_y[b]; }
    __device__ int prior_len() const { return st.prior_len[b]; }
    __device__ int prior_head() const { return st.prior_head[b]; }
    __device__ int prior_x(int k) const { return st.prior_x[b * SL_BONUS_PERIOD_MAX + k]; }
    __device__ int prior_y(int k) const { return st.prior_y[b * SL_BONUS_PERIOD_MAX + k]; }
    __device__ int side_effect() const { return st.side_effect[b]; }
    __device__ double bonus(int d) const { return bonus_table[d]; }
};

// Per-env bookkeeping after the board advance.  Executed by one lane, or by a whole
// wave with wave-uniform arguments (every lane then stores the same values, and the
// integer work runs on the scalar unit).
//   f: the env's fields before the bookkeeping (after the action);
//   points / score / possible / side: the new totals over the advanced board.
// Mirrors SafeLifeEnv.step (safelife_env.py:160-175), update_exit_colors
// (safelife_game.py:531-537), MovementBonusWrapper.step (env_wrappers.py:67-88),
// SimpleSideEffectPenalty.step (env_wrappers.py:319-346) and ContinuingEnv.step
// (env_wrappers.py:298-303) in that order.
template <class F>
__device__ __forceinline__ bool epilogue_core(const sl_env_state &st, const StepArgs &a,
                                              int64_t b, const F &f, int act_reward, int points,
                                              int score, int possible, int side,
                                              double *reward_out, uint8_t *done_out,
                                              uint8_t *flags_out, int32_t *ep_len_out,
                                              int32_t *ep_rew_out, int *can_out = nullptr) {
    const int W = st.W;
    uint16_t *gb = st.board + b * (int64_t)st.H * W;
    const int r_int = act_reward + (points - f.old_points());
    st.old_points[b] = points;
    st.num_steps[b] = f.num_steps() + 1;
    const int ep_len = f.episode_length() + 1;
    const int ep_rew = f.episode_reward() + r_int;
    st.episode_length[b] = ep_len;
    st.episode_reward[b] = ep_rew;
    st.score[b] = score;
    st.possible[b] = possible;
    const bool can = can_exit_now(f.min_performance(), score, f.baseline(), possible);
    const uint16_t ev = (uint16_t)(LEVEL_EXIT | (can ? COLOR_R : 0u));
    if (can_out) *can_out = can ? 1 : 0;
    const int ne = min(f.exit_count(), SL_MAX_EXITS);
    for (int e = 0; e < ne; e++)      // exits are frozen and never change otherwise
        gb[f.exit_y(e) * W + f.exit_x(e)] = ev;
    const bool times_up = ep_len > a.time_limit;
    const bool over = f.game_over() != 0;
    const bool completed = times_up || over;

    double r = (double)r_int;
    if (a.bonus_period > 0) {
        const int n = a.bonus_period;
        const int len = f.prior_len(), head = f.prior_head();
        const int ax = f.agent_x(), ay = f.agent_y();
        int32_t *px = st.prior_x + b * SL_BONUS_PERIOD_MAX;
        int32_t *py = st.prior_y + b * SL_BONUS_PERIOD_MAX;
        const int dist = bonus_dist(ax, ay, f.prior_x(head), f.prior_y(head), len, n,
                                    a.bonus_len);
        r = __dadd_rn(r, f.bonus(dist));
        if (len < n) {
            const int slot = head + len >= n ? head + len - n : head + len;   // head, len < n
            px[slot] = ax;
            py[slot] = ay;
            st.prior_len[b] = len + 1;
        } else {
            px[head] = ax;
            py[head] = ay;
            st.prior_head[b] = head + 1 == n ? 0 : head + 1;
        }
    }
    // reward -= delta_effect * coef: a rounded product, then a rounded difference
    // (an fma here would differ from Python in the last bit)
    r = __dsub_rn(r, __dmul_rn((double)(side - f.side_effect()), a.penalty_coef));
    st.side_effect[b] = side;

    reward_out[b] = r;
    done_out[b] = (uint8_t)(a.auto_reset ? times_up : completed);
    if (flags_out)
        flags_out[b] = (uint8_t)((times_up ? 1 : 0) | (over ? 2 : 0) |
                                 ((a.auto_reset && completed) ? 4 : 0));
    if (ep_len_out) ep_len_out[b] = completed ? ep_len : 0;
    if (ep_rew_out) ep_rew_out[b] = completed ? ep_rew : 0;
    return a.auto_reset && completed;      // the env is reset after this step
}

__device__ __forceinline__ bool env_epilogue(const sl_env_state &st, const StepArgs &a,
                                             int64_t b, int act_reward, int points, int score,
                                             int possible, int side, double *reward_out,
                                             uint8_t *done_out, uint8_t *flags_out,
                                             int32_t *ep_len_out, int32_t *ep_rew_out) {
    return epilogue_core(st, a, b, GlobalFields{st, b, a.bonus_table}, act_reward, points,
                         score, possible, side, reward_out, done_out, flags_out, ep_len_out,
                         ep_rew_out);
}

// ---------------------------------------------------------------------------
// resets (SafeLifeEnv.reset, safelife_env.py:188-198, from a level pool)
// ---------------------------------------------------------------------------
struct ResetArgs {
    int32_t toggle_powers;
    double wrapper_min_perf;
    uint64_t seed;
    uint32_t env0;
    int32_t level_mode, n_total, augment;
    int32_t bonus_period;
};

struct LevelChoice {
    int idx, dy, dx;
};

// the level and toroidal roll of env gid's episode `ep` (the level iterator's
// choice, file_finder.py:143-201, made deterministic per global env id)
__device__ __forceinline__ LevelChoice choose_level(const sl_level_pool &pool, const ResetArgs &a,
                                                   uint32_t gid, int ep, int H, int W) {
    int idx;
    if (a.level_mode == 1)
        idx = (int)(philox_uniform(gid, (uint32_t)ep, 0x5EEDu, 2u, a.seed) * pool.K);
    else
        idx = (int)(((int64_t)gid + (int64_t)ep * a.n_total) % pool.K);
    idx = min(max(idx, 0), pool.K - 1);
    int dy = 0, dx = 0;
    if (a.augment) {
        dy = min((int)(philox_uniform(gid, (uint32_t)ep, 0x0011u, 3u, a.seed) * H), H - 1);
        dx = min((int)(philox_uniform(gid, (uint32_t)ep, 0x0022u, 3u, a.seed) * W), W - 1);
    }
    return LevelChoice{idx, dy, dx};
}

// choose_level by a whole wave: lane 0 picks the level, lanes 1 and 2 the roll, so
// the three Philox draws run side by side instead of one after another on one lane.
// Every lane returns the same choice, bit-identical to choose_level's.
__device__ __forceinline__ LevelChoice choose_level_wave(const sl_level_pool &pool,
                                                        const ResetArgs &a, uint32_t gid,
                                                        int ep, int H, int W, int lane) {
    const uint32_t key = lane == 0 ? 0x5EEDu : (lane == 1 ? 0x0011u : 0x0022u);
    const double u = philox_uniform(gid, (uint32_t)ep, key, lane == 0 ? 2u : 3u, a.seed);
    int v;
    if (lane == 0) {
        v = a.level_mode == 1 ? (int)(u * pool.K)
                              : (int)(((int64_t)gid + (int64_t)ep * a.n_total) % pool.K);
        v = min(max(v, 0), pool.K - 1);
    } else {
        const int n = lane == 1 ? H : W;
        v = a.augment ? min((int)(u * n), n - 1) : 0;
    }
    return LevelChoice{__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 1),
                       __builtin_amdgcn_readlane(v, 2)};
}

// the pool fields of level idx a reset copies into the env's scalars; loaded as soon
// as the level is known, so they arrive while the board gathers are in flight
struct LevelScalars {
    double mp;
    int ax, ay, orientation;
    float spawn_prob;
};

__device__ __forceinline__ LevelScalars level_scalars(const sl_level_pool &pool, int idx) {
    return LevelScalars{pool.min_performance[idx], pool.agent_x[idx], pool.agent_y[idx],
                        pool.orientation[idx], pool.spawn_prob[idx]};
}

__device__ __forceinline__ uint16_t reset_scalars_from(const sl_env_state &st, const ResetArgs &a,
                                                       int64_t b, int idx, int dy, int dx,
                                                       const LevelScalars &ls, int ep,
                                                       int points, int base, int possible,
                                                       int spawn_bits);

// Per-env scalar state of a fresh episode (SafeLifeEnv.reset + revert,
// safelife_env.py:188-198, safelife_game.py:196-212; MovementBonusWrapper.reset and
// SimpleSideEffectPenalty.reset, env_wrappers.py:90-94,313-317).  One thread.
//   points / base / possible: sums over the (rolled) initial board and goals;
//   spawn_bits: bit0 board, bit1 goals hold a spawning cell; bit2 a start-board cell
//   uses bits 12-14 (no cell type does; the 128x128 kernel's spool leaves them out);
//   bit3 a goal cell uses bits outside kGoalPlaneBits (no goal plane mirror).
//   Returns the exit
//   cell value the reset board carries (update_exit_colors after revert).
__device__ __forceinline__ uint16_t reset_scalars(const sl_env_state &st,
                                                  const sl_level_pool &pool, const ResetArgs &a,
                                                  int64_t b, int idx, int dy, int dx, int points,
                                                  int base, int possible, int spawn_bits) {
    return reset_scalars_from(st, a, b, idx, dy, dx, level_scalars(pool, idx), st.episodes[b],
                              points, base, possible, spawn_bits);
}

// the same from the level's fields already loaded (level_scalars) and the env's
// episode count `ep` as read before the reset
__device__ __forceinline__ uint16_t reset_scalars_from(const sl_env_state &st, const ResetArgs &a,
                                                       int64_t b, int idx, int dy, int dx,
                                                       const LevelScalars &ls, int ep,
                                                       int points, int base, int possible,
                                                       int spawn_bits) {
    const int H = st.H, W = st.W;
    const double lvl_mp = ls.mp;
    const bool can = can_exit_now(lvl_mp, base, base, possible);
    const int ax = pymod(ls.ax + dx, W), ay = pymod(ls.ay + dy, H);
    st.agent_x[b] = ax;
    st.agent_y[b] = ay;
    st.orientation[b] = ls.orientation;
    st.game_over[b] = 0;
    st.num_steps[b] = 0;
    st.spawn_flags[b] = ((spawn_bits & 1) || a.toggle_powers ? 1 : 0) | (spawn_bits & 14);
    st.episode_length[b] = 0;
    st.episode_reward[b] = 0;
    st.old_points[b] = points;
    st.baseline[b] = base;
    st.score[b] = base;
    st.possible[b] = possible;
    st.side_effect[b] = 0;
    st.spawn_prob[b] = ls.spawn_prob;
    st.min_performance[b] = isnan(a.wrapper_min_perf) ? lvl_mp : a.wrapper_min_perf;
    st.prior_x[b * SL_BONUS_PERIOD_MAX] = ax;
    st.prior_y[b * SL_BONUS_PERIOD_MAX] = ay;
    st.prior_len[b] = 1;
    st.prior_head[b] = 0;
    st.level_index[b] = idx;
    if (st.start_roll) st.start_roll[b] = (dy << 16) | dx;
    // the 64x64 reset re-validates; a 128x128 env's goals are the level's (bit 5)
    if (st.planes_ok) st.planes_ok[b] = (H == 128 && W == 128) ? 32 : 0;
    st.episodes[b] = ep + 1;
    return (uint16_t)(LEVEL_EXIT | (can ? COLOR_R : 0u));
}

// fused bit-sliced paths (sl_bits*.hip): action + advance + scores (+ reset)
struct FastExtra {
    sl_level_pool pool;     // K == 0: no pool given
    ResetArgs ra;
    int32_t fuse_reset;     // auto-reset: the step kernel lists finished envs and a
                            // follow-up kernel resets exactly those
    int64_t *scratch;       // sl_env_cfg.scratch (reset list + counters)
    void *ev_end;           // hipEvent_t recorded right after the step kernel's launch
                            // (before any follow-up kernel), or NULL
    uint16_t *obs_out;      // 64x64 kernel: views written from the on-chip board (NULL:
    int32_t obs_vh, obs_vw, obs_rw;   // none); view shape, remove_white
    int32_t obs_mode;       // SL_OBS_PACKED or a channel mode (then obs_out is the
    int32_t obs_nch;        // [B, vh, vw, nch] array of SL_OBS_CHANNELS*)
    uint64_t obs_chpack;    // channel k in bits 4k .. 4k + 3
    uint32_t obs_one;       // a channel element's 1 (1, 0x3F80 bf16, 0x3F800000 f32)
    const sl_capture *capture;        // trajectory capture (NULL: none): phase 0 is
                                      // launched between the step and reset kernels
    int32_t stream;         // SL_RNG_STREAM: replay prologue (action + eligible counts),
                            // offsets scan, then the step kernel's SPAWN_STREAM form
    int64_t *stream_pos;    // replay mode: the stream position (in / out, device)
    void *ev_begin;         // hipEvent_t recorded right before the step kernel, or NULL
    int32_t stream_phase;   // replay split over shards (sl_env_cfg.stream_phase): 0
                            // whole step, 1 action + counts + total, 2 offsets from
    const int64_t *stream_base;   // *stream_base + the step
    const sl_mt19937 *mt;   // replay from the device generator (sl_env_cfg.mt) or NULL:
                            // stream_offsets fills its ring for the step's range
    double bits_thr = -1.0; // the device generator's bit ring: its threshold (else < 0);
    int32_t thr_checked = 0;// the 128x128 count prologue checks it (stream_offsets then
                            // launches no k_bits_thr_check)
    int32_t plane_mode = 0; // 128x128 step without capture (no views, or packed views of
                            // <= kViewMaxRows128 rows written from the planes; replay
                            // with draw planes), board_planes set: the board is kept in
                            // sl_env_state.board_planes
};
// replay-mode phases of a bit-sliced launcher: whether it runs the action + count
// prologue, and whether it continues past the offsets scan to the step kernel
__host__ inline bool stream_counts(const FastExtra &fx) { return fx.stream_phase != 2; }
__host__ inline bool stream_steps(const FastExtra &fx) { return fx.stream_phase != 1; }
// replay mode: exclusive scan of the prologue's per-(env, tensor) eligible counts into
// each tensor's first uniform, advancing *fx.stream_pos (sl_env.hip)
int stream_offsets(const sl_env_state &st, const FastExtra &fx, hipStream_t s);
// the device generator's bit ring: flag (err |= 1) any env with draws this step whose
// threshold is not the ring's (sl_env.hip)
int bits_thr_check(const sl_env_state &st, const sl_mt19937 *mt, const int64_t *counts,
                   int64_t *err, hipStream_t s);
// copies of the captured envs' state (sl_capture): phase 0 after the advance (and
// the step's flags), phase 1 after the resets
int launch_capture(const sl_env_state &st, const sl_capture &c, const uint8_t *flags, int phase,
                   hipStream_t s);
// bit-sliced 128x128 kernel (sl_bits128.hip); needs the goals mirror (st.planes).
// With fx.fuse_reset it queues the envs that finished and launches
// k_env_reset_list_wide for them.
bool bits128_shape(const sl_env_state &st);
// the bit-sliced kernel for boards up to 32 x 64 (sl_bits_small.hip)
bool small_shape(const sl_env_state &st);
// (auto-reset: envs whose episode ended are reset by their own wave from fx.pool)
int launch_step_small(const sl_env_state &st, const StepArgs &a, const FastExtra &fx,
                      const int32_t *actions, int ctp, int ctc, double *reward, uint8_t *done,
                      uint8_t *flags, int32_t *ep_len, int32_t *ep_rew, hipStream_t s);
int launch_step_bits128(const sl_env_state &st, const StepArgs &a, const FastExtra &fx,
                        const int32_t *actions, int ctp, int ctc, double *reward, uint8_t *done,
                        uint8_t *flags, int32_t *ep_len, int32_t *ep_rew, hipStream_t s);
// the action of every env (k_env_action, one lane per env): state and cell edits in
// HBM, reward into act[b]; the 128x128 kernel's pre-pass (sl_env.hip)
// 128x128 board planes (sl_env_state.board_planes): complete the uint16 board of envs
// kept in planes; demote: then mark the planes stale (before a step or edit that
// works on the uint16 board).  No-op unless the state has board planes.
int sync_board_planes(const sl_env_state &st, int demote, hipStream_t s);
// 64x64 (sl_bits.hip): plane mode when st.board_planes == st.planes (the board in half
// 0 of the goals mirror); the sync of such a state
bool planes64_shape(const sl_env_state &st);
int sync_board_planes64(const sl_env_state &st, int demote, hipStream_t s);
int launch_env_action(const sl_env_state &st, const int32_t *actions, int ctp, int ctc,
                      int64_t *act, hipStream_t s);
// resets of the envs queued in the scratch list for step `step`, one 1024-thread
// block each (sl_env.hip)
int launch_reset_list_wide(const sl_env_state &st, const sl_level_pool &pool, const ResetArgs &ra,
                           int64_t *scratch, uint32_t step, hipStream_t s);
// the 128x128 step kernel writes packed views of at most this many rows from the board
// planes (sl_bits128.hip view_band: one run of view rows per 32-row band)
constexpr int kViewMaxRows128 = 96;
// bit-sliced 64x64 kernel (sl_bits.hip)
int launch_step_bits(const sl_env_state &st, const StepArgs &a, const FastExtra &fx,
                     const int32_t *actions, int ctp, int ctc, double *reward, uint8_t *done,
                     uint8_t *flags, int32_t *ep_len, int32_t *ep_rew, hipStream_t s);

}  // namespace sl
