// sl_env.hip -- batched SafeLife env step / reset / observation for gfx950.
//
// One env-step of the PPO chain, for B envs held as uint16 [B,H,W] device boards:
//   k_env_action      execute_action / move_agent / relative_loc
//                     (safelife_game.py:294-393), one lane per env
//   k_env_count       replay mode only: draws each board will consume
//   k_env_step_generic  advance board+goals (safelife_game.py:657-660), points
//                     (:590-599), performance ratio (:601-631), exit colours
//                     (:528-537), SafeLifeEnv.step bookkeeping (safelife_env.py:
//                     157-186), MovementBonusWrapper (env_wrappers.py:67-88) and
//                     SimpleSideEffectPenalty (env_wrappers.py:319-346); one
//                     workgroup per env, board+goals staged in LDS
//   k_env_reset       SafeLifeEnv.reset + wrapper resets from a level pool
//   k_env_obs         get_obs + recenter_view (safelife_env.py:125-155,
//                     helper_utils.py:41-74)
#include "sl_env_common.h"
#include "sl_env_action.h"
#include "sl_obs.h"

#include <math.h>

using namespace sl;
using namespace sl::obs;

namespace {

constexpr int NT = 256;
constexpr int kMaxCells = 16384;          // board+goals in LDS: 64 KiB

// the action of every env, one lane each (sl_env_action.h)
template <bool DELTAS>
__global__ void __launch_bounds__(256)
k_env_action(sl_env_state st, const int32_t *__restrict__ actions, int ctp, int ctc,
             int64_t *__restrict__ act) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= st.B) return;
    env_action_one<DELTAS>(st, actions, ctp, ctc, act, b);
}

// ---------------------------------------------------------------------------
// shared block pieces
// ---------------------------------------------------------------------------
__device__ __forceinline__ void stage(uint16_t *dst, const uint16_t *src, int hw) {
    if ((((uintptr_t)src) & 15) == 0 && (hw & 7) == 0) {
        const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
        uint4 *d4 = reinterpret_cast<uint4 *>(dst);
        for (int i = threadIdx.x; i < (hw >> 3); i += NT) d4[i] = s4[i];
    } else {
        for (int i = threadIdx.x; i < hw; i += NT) dst[i] = src[i];
    }
}

__device__ __forceinline__ int block_rank(bool flag, int *wave_tot, int *total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    unsigned long long m = __ballot(flag);
    int below = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wave_tot[wid] = __popcll(m);
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) {
        int t = wave_tot[w];
        off += (w < wid) ? t : 0;
        tot += t;
    }
    __syncthreads();
    *total = tot;
    return off + below;
}

// reduce 4 ints over the block; result valid in thread 0
__device__ __forceinline__ void block_sum4(int v[4], int (*red)[4]) {
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = wave_sum(v[k]);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0)
        for (int k = 0; k < 4; k++) red[wid][k] = v[k];
    __syncthreads();
    if (threadIdx.x == 0)
        for (int k = 0; k < 4; k++) {
            int t = 0;
            for (int w = 0; w < NT / 64; w++) t += red[w][k];
            v[k] = t;
        }
}

__global__ void __launch_bounds__(NT)
k_env_count(sl_env_state st, int64_t *__restrict__ counts) {
    extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
    __shared__ int red[NT / 64][4];
    const int H = st.H, W = st.W, hw = H * W;
    const int64_t b = blockIdx.x;
    uint16_t *lb = lds, *lg = lds + hw;
    stage(lb, st.board + b * hw, hw);
    stage(lg, st.goals + b * hw, hw);
    __syncthreads();
    int v[4] = {0, 0, 0, 0};
    for (int i = threadIdx.x; i < hw; i += NT) {
        const int y = i / W, x = i - y * W;
        bool e;
        uint32_t sv;
        rule_cell(lb[i], gather_lds(lb, H, W, y, x), &e, &sv);
        v[0] += e;
        rule_cell(lg[i], gather_lds(lg, H, W, y, x), &e, &sv);
        v[1] += e;
    }
    block_sum4(v, red);
    if (threadIdx.x == 0) {
        counts[2 * b] = v[0];
        counts[2 * b + 1] = v[1];
    }
}


template <int RNG>
__global__ void __launch_bounds__(NT)
k_env_step_generic(sl_env_state st, StepArgs a, const int64_t *__restrict__ act,
                   const int64_t *__restrict__ offsets, int64_t *__restrict__ err,
                   double *__restrict__ reward_out, uint8_t *__restrict__ done_out,
                   uint8_t *__restrict__ flags_out, int32_t *__restrict__ ep_len_out,
                   int32_t *__restrict__ ep_rew_out) {
    extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
    __shared__ int red[NT / 64][4];
    __shared__ int wave_tot[NT / 64];
    const int H = st.H, W = st.W, hw = H * W;
    const int64_t b = blockIdx.x;
    uint16_t *lb = lds, *lg = lds + hw;
    uint16_t *gb = st.board + b * hw, *gg = st.goals + b * hw;
    const uint16_t *gs = st.start_board + b * hw;
    stage(lb, gb, hw);
    stage(lg, gg, hw);
    __syncthreads();

    const double thr = (double)st.spawn_prob[b];
    int64_t pos_b = 0, pos_g = 0;
    if (RNG == SL_RNG_STREAM) {
        pos_b = offsets[2 * b];
        pos_g = offsets[2 * b + 1];
    }
    int acc[4] = {0, 0, 0, 0};   // points, score, possible, side effects
    const int nchunk = (hw + NT - 1) / NT;
    for (int c = 0; c < nchunk; c++) {
        const int i = c * NT + threadIdx.x;
        uint32_t vb = 0, vg = 0, nb = 0, ng = 0, sb = 0, sg = 0;
        bool eb = false, eg = false;
        if (i < hw) {
            const int y = i / W, x = i - y * W;
            vb = lb[i];
            vg = lg[i];
            nb = rule_cell(vb, gather_lds(lb, H, W, y, x), &eb, &sb);
            ng = rule_cell(vg, gather_lds(lg, H, W, y, x), &eg, &sg);
        }
        double ub = 1.0, ug = 1.0;
        if (RNG == SL_RNG_STREAM) {
            int tb, tg;
            const int rb = block_rank(eb, wave_tot, &tb);
            const int rg = block_rank(eg, wave_tot, &tg);
            if (eb) {
                if (thr <= 0.0) ub = 1.0;
                else if (thr >= 1.0) ub = 0.0;
                else if (pos_b + rb < a.n_draws) ub = stream_u(a.draws, a.draw_bits, pos_b + rb, a.draw_mask);
                else atomicOr((unsigned long long *)err, 1ull);
            }
            if (eg) {
                if (thr <= 0.0) ug = 1.0;
                else if (thr >= 1.0) ug = 0.0;
                else if (pos_g + rg < a.n_draws) ug = stream_u(a.draws, a.draw_bits, pos_g + rg, a.draw_mask);
                else atomicOr((unsigned long long *)err, 1ull);
            }
            pos_b += tb;
            pos_g += tg;
        } else {
            const int y = i / W, x = i - y * W;
            if (eb) ub = spawn_uniform(y, x, W, a.env0 + (uint32_t)b, a.step, 0u, a.seed);
            if (eg) ug = spawn_uniform(y, x, W, a.env0 + (uint32_t)b, a.step, 1u, a.seed);
        }
        if (eb && ub < thr) nb = sb;
        if (eg && ug < thr) ng = sg;
        if (i < hw) {
            const uint32_t s = gs[i];
            int p, q, r;
            cell_scores(nb, ng, &p, &q, &r);
            acc[0] += p;
            acc[1] += q;
            acc[2] += r;
            acc[3] += side_term(nb, s, ng);
            gg[i] = (uint16_t)ng;
            if (!(s & EXIT)) gb[i] = (uint16_t)nb;   // exits: recoloured below
        }
    }
    block_sum4(acc, red);
    if (threadIdx.x != 0) return;

    env_epilogue(st, a, b, (int)act[b], acc[0], acc[1], acc[2], acc[3], reward_out, done_out,
                 flags_out, ep_len_out, ep_rew_out);
}

// ---------------------------------------------------------------------------
// game-level pieces (sl_env_advance / sl_env_rescore / sl_env_exit_colors):
// SafeLifeGame.advance_board, current_points / performance_ratio and
// update_exit_colors for callers that drive the game without the env step
// ---------------------------------------------------------------------------
// SafeLifeGame.advance_board (safelife_game.py:657-660): num_steps += 1, then board
// and goals advanced (board draws first).  One block per env, both tensors staged in
// LDS; no scoring, no exit recolour (exits are frozen: the rule leaves them as they
// are).  Invalidates the goals mirror.
template <int RNG>
__global__ void __launch_bounds__(NT)
k_env_advance(sl_env_state st, StepArgs a, const int64_t *__restrict__ offsets,
              int64_t *__restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
    __shared__ int wave_tot[NT / 64];
    const int H = st.H, W = st.W, hw = H * W;
    const int64_t b = blockIdx.x;
    uint16_t *lb = lds, *lg = lds + hw;
    uint16_t *gb = st.board + b * hw, *gg = st.goals + b * hw;
    stage(lb, gb, hw);
    stage(lg, gg, hw);
    __syncthreads();
    const double thr = (double)st.spawn_prob[b];
    int64_t pos_b = 0, pos_g = 0;
    if (RNG == SL_RNG_STREAM) {
        pos_b = offsets[2 * b];
        pos_g = offsets[2 * b + 1];
    }
    const int nchunk = (hw + NT - 1) / NT;
    for (int c = 0; c < nchunk; c++) {
        const int i = c * NT + threadIdx.x;
        uint32_t nb = 0, ng = 0, sb = 0, sg = 0;
        bool eb = false, eg = false;
        if (i < hw) {
            const int y = i / W, x = i - y * W;
            nb = rule_cell(lb[i], gather_lds(lb, H, W, y, x), &eb, &sb);
            ng = rule_cell(lg[i], gather_lds(lg, H, W, y, x), &eg, &sg);
        }
        double ub = 1.0, ug = 1.0;
        if (RNG == SL_RNG_STREAM) {
            int tb, tg;
            const int rb = block_rank(eb, wave_tot, &tb);
            const int rg = block_rank(eg, wave_tot, &tg);
            if (eb) {
                if (thr <= 0.0) ub = 1.0;
                else if (thr >= 1.0) ub = 0.0;
                else if (pos_b + rb < a.n_draws) ub = stream_u(a.draws, a.draw_bits, pos_b + rb, a.draw_mask);
                else atomicOr((unsigned long long *)err, 1ull);
            }
            if (eg) {
                if (thr <= 0.0) ug = 1.0;
                else if (thr >= 1.0) ug = 0.0;
                else if (pos_g + rg < a.n_draws) ug = stream_u(a.draws, a.draw_bits, pos_g + rg, a.draw_mask);
                else atomicOr((unsigned long long *)err, 1ull);
            }
            pos_b += tb;
            pos_g += tg;
        } else {
            const int y = i / W, x = i - y * W;
            if (eb) ub = spawn_uniform(y, x, W, a.env0 + (uint32_t)b, a.step, 0u, a.seed);
            if (eg) ug = spawn_uniform(y, x, W, a.env0 + (uint32_t)b, a.step, 1u, a.seed);
        }
        if (eb && ub < thr) nb = sb;
        if (eg && ug < thr) ng = sg;
        if (i < hw) {
            gb[i] = (uint16_t)nb;
            gg[i] = (uint16_t)ng;
        }
    }
    if (threadIdx.x == 0) {
        st.num_steps[b] += 1;
        if (st.planes_ok) st.planes_ok[b] = 0;
    }
}

// current_points (safelife_game.py:590-599) and the unit-reward performance terms
// (:601-631) of the current board and goals: score[b], possible[b] refreshed (what
// can_exit reads), points[b] written when points != NULL.  One block per env.
__global__ void __launch_bounds__(NT)
k_env_rescore(sl_env_state st, int32_t *__restrict__ points) {
    __shared__ int red[NT / 64][4];
    const int hw = st.H * st.W;
    const int64_t b = blockIdx.x;
    const uint16_t *gb = st.board + b * hw, *gg = st.goals + b * hw;
    int acc[4] = {0, 0, 0, 0};
    for (int i = threadIdx.x; i < hw; i += NT) {
        int p, q, r;
        cell_scores(gb[i], gg[i], &p, &q, &r);
        acc[0] += p;
        acc[1] += q;
        acc[2] += r;
    }
    block_sum4(acc, red);
    if (threadIdx.x == 0) {
        st.score[b] = acc[1];
        st.possible[b] = acc[2];
        if (points) points[b] = acc[0];
    }
}

// update_exit_colors (safelife_game.py:531-537) from the stored score terms
// (mode 0), or the exit cells restored to their start-board values (mode 1: the raw
// level cells deserialize / revert put back, safelife_game.py:196-212).  One lane per
// env.
__global__ void __launch_bounds__(256)
k_env_exit_colors(sl_env_state st, int mode) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= st.B) return;
    const int64_t hw = (int64_t)st.H * st.W;
    uint16_t *gb = st.board + b * hw;
    const uint16_t *gs = st.start_board + b * hw;
    const bool can = can_exit_now(st.min_performance[b], st.score[b], st.baseline[b],
                                  st.possible[b]);
    const uint16_t ev = (uint16_t)(LEVEL_EXIT | (can ? COLOR_R : 0u));
    const int ne = min(st.exit_count[b], SL_MAX_EXITS);
    for (int e = 0; e < ne; e++) {
        const int k = st.exit_y[b * SL_MAX_EXITS + e] * st.W + st.exit_x[b * SL_MAX_EXITS + e];
        gb[k] = mode ? gs[k] : ev;
    }
}

// ---------------------------------------------------------------------------
// reset from the level pool
// ---------------------------------------------------------------------------
// spawn_flags bits 2 and 3 describe 128x128 boards only (the one kernel that reads
// them); the other shapes' resets, whichever kernel runs them, leave them clear
__device__ __forceinline__ bool is128(int H, int W) { return H == 128 && W == 128; }

struct ResetShared {
    int red[NT / 64][4];
    int wave_tot[NT / 64];
    int exit_y[SL_MAX_EXITS], exit_x[SL_MAX_EXITS];
    int ev, idx, dy, dx;
    int hi;         // a start-board cell uses bits 12-14 (spawn_flags bit 2)
    int gx;         // a goal cell uses bits outside kGoalPlaneBits (spawn_flags bit 3)
};

__device__ void reset_one(const sl_env_state &st, const sl_level_pool &pool, const ResetArgs &a,
                          int64_t b, ResetShared &sh) {
    int (*red)[4] = sh.red;
    int *wave_tot = sh.wave_tot;
    int *sh_exit_y = sh.exit_y, *sh_exit_x = sh.exit_x;
    int &sh_ev = sh.ev, &sh_idx = sh.idx, &sh_dy = sh.dy, &sh_dx = sh.dx;
    const int H = st.H, W = st.W, hw = H * W;
    const uint32_t gid = a.env0 + (uint32_t)b;
    if (threadIdx.x == 0) {
        const LevelChoice c = choose_level(pool, a, gid, st.episodes[b], H, W);
        sh_idx = c.idx; sh_dy = c.dy; sh_dx = c.dx;
        sh.hi = 0;
        sh.gx = 0;
    }
    __syncthreads();
    const int idx = sh_idx, dy = sh_dy, dx = sh_dx;
    const uint16_t *pb = pool.board + (int64_t)idx * hw, *pg = pool.goals + (int64_t)idx * hw;

    // pass 1: reductions + ordered exit list of the (rolled) initial board
    int acc[4] = {0, 0, 0, 0};   // points, score(=baseline), possible, spawn flags
    int n_exit = 0;
    const int nchunk = (hw + NT - 1) / NT;
    for (int c = 0; c < nchunk; c++) {
        const int i = c * NT + threadIdx.x;
        bool ex = false;
        if (i < hw) {
            const int y = i / W, x = i - y * W;
            const int src = pymod(y - dy, H) * W + pymod(x - dx, W);
            const uint32_t vb = pb[src], vg = pg[src];
            int p, q, r;
            cell_scores(vb, vg, &p, &q, &r);
            acc[0] += p;
            acc[1] += q;
            acc[2] += r;
            acc[3] += ((vb & SPAWN) ? 1 : 0) + ((vg & SPAWN) ? 65536 : 0);  // counts < 2^16
            if (vb & kCellHiBits) sh.hi = 1;
            if (vg & ~kGoalPlaneBits) sh.gx = 1;
            ex = (vb & EXIT) != 0;
        }
        int tot;
        const int rank = block_rank(ex, wave_tot, &tot);
        if (ex && n_exit + rank < SL_MAX_EXITS) {
            sh_exit_y[n_exit + rank] = i / W;
            sh_exit_x[n_exit + rank] = i % W;
        }
        n_exit += tot;
    }
    block_sum4(acc, red);
    if (threadIdx.x == 0) {
        const int spawn_bits = ((acc[3] & 0xFFFF) ? 1 : 0) | ((acc[3] >> 16) ? 2 : 0) |
                               (is128(H, W) ? (sh.hi ? 4 : 0) | (sh.gx ? 8 : 0) : 0);
        sh_ev = reset_scalars(st, pool, a, b, idx, dy, dx, acc[0], acc[1], acc[2], spawn_bits);
        st.exit_count[b] = n_exit;
        for (int e = 0; e < SL_MAX_EXITS; e++) {
            st.exit_y[b * SL_MAX_EXITS + e] = (int16_t)(e < n_exit ? sh_exit_y[e] : 0);
            st.exit_x[b * SL_MAX_EXITS + e] = (int16_t)(e < n_exit ? sh_exit_x[e] : 0);
        }
    }
    __syncthreads();
    const uint16_t ev = (uint16_t)sh_ev;
    uint16_t *gb = st.board + b * hw, *gg = st.goals + b * hw, *gs = st.start_board + b * hw;
    for (int i = threadIdx.x; i < hw; i += NT) {
        const int y = i / W, x = i - y * W;
        const int src = pymod(y - dy, H) * W + pymod(x - dx, W);
        const uint16_t vb = pb[src];
        gs[i] = vb;
        gb[i] = (vb & EXIT) ? ev : vb;
        gg[i] = pg[src];
    }
}

// The same reset by a 1024-thread block, for the envs a step kernel queued (the
// 128x128 kernel).  The exit cells are appended to an LDS list by atomics and put
// into np.nonzero order afterwards, so the load pass has no barrier and all of a
// thread's gathers are in flight together.  A level with more exit cells than the
// list holds (never seen) is scanned in order by one thread.
constexpr int NTR = 1024;
constexpr int kExitCap = 64;
struct WideResetShared {
    int red[NTR / 64][4];
    int exl[kExitCap];
    int nex, ev, idx, dy, dx;
    int hi;         // a start-board cell uses bits 12-14 (spawn_flags bit 2)
    int gx;         // a goal cell uses bits outside kGoalPlaneBits (spawn_flags bit 3)
};

__device__ void reset_wide(const sl_env_state &st, const sl_level_pool &pool, const ResetArgs &a,
                           int64_t b, WideResetShared &sh) {
    const int H = st.H, W = st.W, hw = H * W;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    int ep = 0;
    LevelScalars ls{};
    if (wid == 0) {        // the three Philox draws side by side on lanes 0-2
        ep = __builtin_amdgcn_readfirstlane(st.episodes[b]);
        const LevelChoice c = choose_level_wave(pool, a, a.env0 + (uint32_t)b, ep, H, W, lane);
        ls = level_scalars(pool, c.idx);      // thread 0's, in flight with the gathers
        if (lane == 0) {
            sh.idx = c.idx;
            sh.dy = c.dy;
            sh.dx = c.dx;
            sh.nex = 0;
            sh.hi = 0;
            sh.gx = 0;
        }
    }
    __syncthreads();
    const int idx = sh.idx, dy = sh.dy, dx = sh.dx;
    const uint16_t *pb = pool.board + (int64_t)idx * hw, *pg = pool.goals + (int64_t)idx * hw;

    int acc[4] = {0, 0, 0, 0};   // points, score (= baseline), possible, spawn flags
#pragma unroll 4
    for (int i = tid; i < hw; i += NTR) {
        const int y = i / W, x = i - y * W;
        const int src = pymod(y - dy, H) * W + pymod(x - dx, W);
        const uint32_t vb = pb[src], vg = pg[src];
        int p, q, r;
        cell_scores(vb, vg, &p, &q, &r);
        acc[0] += p;
        acc[1] += q;
        acc[2] += r;
        acc[3] += ((vb & SPAWN) ? 1 : 0) + ((vg & SPAWN) ? 65536 : 0);
        if (vb & kCellHiBits) sh.hi = 1;
        if (vg & ~kGoalPlaneBits) sh.gx = 1;
        if (vb & EXIT) {
            const int k = atomicAdd(&sh.nex, 1);
            if (k < kExitCap) sh.exl[k] = i;
        }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) acc[k] = wave_sum(acc[k]);
    if (lane == 0)
        for (int k = 0; k < 4; k++) sh.red[wid][k] = acc[k];
    __syncthreads();
    if (tid == 0) {
        int t[4] = {0, 0, 0, 0};
        for (int w = 0; w < NTR / 64; w++)
            for (int k = 0; k < 4; k++) t[k] += sh.red[w][k];
        const int spawn_bits = ((t[3] & 0xFFFF) ? 1 : 0) | ((t[3] >> 16) ? 2 : 0) |
                               (is128(H, W) ? (sh.hi ? 4 : 0) | (sh.gx ? 8 : 0) : 0);
        sh.ev = reset_scalars_from(st, a, b, idx, dy, dx, ls, ep, t[0], t[1], t[2], spawn_bits);
        const int nex = sh.nex;
        int16_t *ey = st.exit_y + b * SL_MAX_EXITS, *ex = st.exit_x + b * SL_MAX_EXITS;
        int n = 0;
        if (nex <= kExitCap) {           // row-major order = ascending flat index
            for (int k = 1; k < nex; k++) {
                const int v = sh.exl[k];
                int j = k - 1;
                while (j >= 0 && sh.exl[j] > v) {
                    sh.exl[j + 1] = sh.exl[j];
                    j--;
                }
                sh.exl[j + 1] = v;
            }
            for (; n < nex && n < SL_MAX_EXITS; n++) {
                ey[n] = (int16_t)(sh.exl[n] / W);
                ex[n] = (int16_t)(sh.exl[n] % W);
            }
        } else {
            for (int i = 0; i < hw && n < SL_MAX_EXITS; i++) {
                const int y = i / W, x = i - y * W;
                if (pb[pymod(y - dy, H) * W + pymod(x - dx, W)] & EXIT) {
                    ey[n] = (int16_t)y;
                    ex[n] = (int16_t)x;
                    n++;
                }
            }
        }
        for (int e = n; e < SL_MAX_EXITS; e++) {
            ey[e] = 0;
            ex[e] = 0;
        }
        st.exit_count[b] = nex;
    }
    __syncthreads();
    const uint16_t ev = (uint16_t)sh.ev;
    uint16_t *gb = st.board + b * hw, *gg = st.goals + b * hw, *gs = st.start_board + b * hw;
    if ((W & 1) == 0) {                  // cell pairs: one dword store per tensor
        uint32_t *gb2 = reinterpret_cast<uint32_t *>(gb), *gg2 = reinterpret_cast<uint32_t *>(gg);
        uint32_t *gs2 = reinterpret_cast<uint32_t *>(gs);
#pragma unroll 4
        for (int i = tid; i < (hw >> 1); i += NTR) {
            const int y = (2 * i) / W, x = 2 * i - y * W;
            const int sr = pymod(y - dy, H) * W;
            const int c0 = pymod(x - dx, W), c1 = c0 + 1 == W ? 0 : c0 + 1;
            const uint32_t b0 = pb[sr + c0], b1 = pb[sr + c1];
            gs2[i] = b0 | (b1 << 16);
            gb2[i] = ((b0 & EXIT) ? ev : b0) | ((uint32_t)((b1 & EXIT) ? ev : b1) << 16);
            gg2[i] = (uint32_t)pg[sr + c0] | ((uint32_t)pg[sr + c1] << 16);
        }
    } else {
        for (int i = tid; i < hw; i += NTR) {
            const int y = i / W, x = i - y * W;
            const int src = pymod(y - dy, H) * W + pymod(x - dx, W);
            const uint16_t vb = pb[src];
            gs[i] = vb;
            gb[i] = (vb & EXIT) ? ev : vb;
            gg[i] = pg[src];
        }
    }
}

// Resets the envs a step kernel queued in the scratch list (sl_env_common.h), one
// block each; zeroes the other step parity's list length for the next step.
__global__ void __launch_bounds__(NTR)
k_env_reset_list_wide(sl_env_state st, sl_level_pool pool, ResetArgs ra, int64_t *scratch,
                      uint32_t step) {
    __shared__ WideResetShared sh;
    int64_t *cnt = scratch + 8 * st.B + 2;
    if (blockIdx.x == 0 && threadIdx.x == 0) cnt[(step + 1) & 1] = 0;
    const int n = (int)cnt[step & 1];
    const int32_t *list = reset_list(scratch);
    for (int i = blockIdx.x; i < n; i += gridDim.x) {
        reset_wide(st, pool, ra, list[i], sh);
        __syncthreads();
    }
}

// The packed views of the envs k_env_reset_list_wide reset this step (a 128x128 step
// whose kernel wrote the other views from the board planes): one wave per listed env,
// four per workgroup, from the new episode's uint16 board (written by the previous
// launch).
__global__ void __launch_bounds__(256)
k_env_obs_reset_list(sl_env_state st, ObsArgs a, const int64_t *scratch, uint32_t step,
                     uint16_t *out) {
    const int n = (int)scratch[8 * st.B + 2 + (step & 1)];
    const int32_t *list = reset_list(const_cast<int64_t *>(scratch));
    const int lane = threadIdx.x & 63;
    for (int i = blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += gridDim.x * 4)
        obs_packed_wave(st, a, list[i], lane, out);
}

// pool->board_planes (H == 64): [k][p][x] bit y = bit p of pool->board[k][y][x];
// (H == 128): 32-bit words [k][p][q][x] bit r = bit p of pool->board[k][32q + r][x]
__global__ void __launch_bounds__(NT) k_pool_planes(sl_level_pool pool) {
    const int nq = pool.H / 32;            // 32-row words per column (2 or 4)
    const int64_t n = (int64_t)pool.K * 16 * nq * pool.W;
    for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
        const int64_t k = i / (16 * nq * pool.W);
        int r = (int)(i - k * 16 * nq * pool.W);
        const int p = r / (nq * pool.W);
        r -= p * nq * pool.W;
        const int q = r / pool.W, x = r - q * pool.W;
        const uint16_t *bd = pool.board + (k * pool.H + 32 * q) * pool.W + x;
        uint32_t v = 0;
        for (int y = 0; y < 32; y++) v |= (uint32_t)((bd[y * pool.W] >> p) & 1u) << y;
        if (pool.H == 64) {
            uint32_t *w = reinterpret_cast<uint32_t *>(pool.board_planes) +
                          2 * ((k * 16 + p) * pool.W + x) + q;
            *w = v;
        } else {
            reinterpret_cast<uint32_t *>(pool.board_planes)[i] = v;
        }
    }
}

// pool->goal_planes (H == 128): 32-bit words [k][c][q][x] bit r = bit 9 + c of
// pool->goals[k][32q + r][x]
__global__ void __launch_bounds__(NT) k_pool_goal_planes(sl_level_pool pool) {
    const int nq = pool.H / 32;
    const int64_t n = (int64_t)pool.K * 3 * nq * pool.W;
    for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
        const int64_t k = i / (3 * nq * pool.W);
        int r = (int)(i - k * 3 * nq * pool.W);
        const int c = r / (nq * pool.W);
        r -= c * nq * pool.W;
        const int q = r / pool.W, x = r - q * pool.W;
        const uint16_t *gd = pool.goals + (k * pool.H + 32 * q) * pool.W + x;
        uint32_t v = 0;
        for (int y = 0; y < 32; y++) v |= (uint32_t)((gd[y * pool.W] >> (9 + c)) & 1u) << y;
        pool.goal_planes[i] = v;
    }
}

// explicit resets (mask or all envs): grid-stride over envs, one block per env
__global__ void __launch_bounds__(NT)
k_env_reset(sl_env_state st, sl_level_pool pool, const uint8_t *__restrict__ mask,
            const uint8_t *__restrict__ flags, ResetArgs a) {
    __shared__ ResetShared sh;
    for (int64_t b = blockIdx.x; b < st.B; b += gridDim.x) {
        if (mask && !mask[b]) continue;
        if (flags && !(flags[b] & 4)) continue;
        reset_one(st, pool, a, b, sh);
        __syncthreads();
    }
}

// auto-reset after a step: each block checks NT envs' flags with one coalesced load,
// gathers the finished ones (typically 0-2 of 256) and resets only those
__global__ void __launch_bounds__(NT)
k_env_reset_scan(sl_env_state st, sl_level_pool pool, const uint8_t *__restrict__ flags,
                 ResetArgs a) {
    __shared__ ResetShared sh;
    __shared__ int list[NT];
    __shared__ int cnt;
    const int64_t b0 = (int64_t)blockIdx.x * NT;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    const int64_t mine = b0 + threadIdx.x;
    if (mine < st.B && (flags[mine] & 4)) list[atomicAdd(&cnt, 1)] = threadIdx.x;
    __syncthreads();
    const int n = cnt;
    for (int k = 0; k < n; k++) {          // envs are independent: order is irrelevant
        reset_one(st, pool, a, b0 + list[k], sh);
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// observations
// ---------------------------------------------------------------------------
// channel k of cell i = bit a.ch[k] of view[i], stored as the pattern 0 / `one` of an
// element type of T's width (0/1 integers, or 0.0/1.0 as float32 / bfloat16 -- the
// policy's layer0, training/safelife_ppo.py:147-152, without a separate cast pass)
template <typename T>
__device__ __forceinline__ void store_channels(void *out, int64_t b, const uint16_t *view, int nv,
                                               const ObsArgs &a, uint32_t one) {
    T *o = (T *)out + b * (int64_t)nv * a.nch;
    for (int j = threadIdx.x; j < nv * a.nch; j += NT) {
        const int i = j / a.nch, k = j - i * a.nch;
        o[j] = (T)(((view[i] >> a.ch[k]) & 1u) ? one : 0u);
    }
}

__global__ void __launch_bounds__(NT)
k_env_obs(sl_env_state st, ObsArgs a, void *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) uint16_t view[];
    const int64_t b = blockIdx.x;
    const int H = st.H, W = st.W, hw = H * W, nv = a.vh * a.vw;
    const uint16_t *gb = st.board + b * hw, *gg = st.goals + b * hw;
    const int y0 = st.agent_y[b], x0 = st.agent_x[b];
    const int ty = y0 - a.vh / 2, tx = x0 - a.vw / 2;
    for (int i = threadIdx.x; i < nv; i += NT) {
        const int r = i / a.vw, c = i - r * a.vw;
        const int src = pymod(ty + r, H) * W + pymod(tx + c, W);
        view[i] = obs_value(gb[src], gg[src], a.remove_white);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const int ne = min(st.exit_count[b], SL_MAX_EXITS);
        for (int e = 0; e < ne; e++) {
            const int iy = st.exit_y[b * SL_MAX_EXITS + e], ix = st.exit_x[b * SL_MAX_EXITS + e];
            int jy = pymod(iy - y0 + H / 2, H) - H / 2;
            int jx = pymod(ix - x0 + W / 2, W) - W / 2;
            jy = min(max(jy + a.vh / 2, 0), a.vh - 1);
            jx = min(max(jx + a.vw / 2, 0), a.vw - 1);
            view[jy * a.vw + jx] = obs_value(gb[iy * W + ix], gg[iy * W + ix], a.remove_white);
        }
    }
    __syncthreads();
    if (a.mode == SL_OBS_PACKED) {
        uint16_t *o = (uint16_t *)out + b * nv;
        for (int i = threadIdx.x; i < nv; i += NT) o[i] = view[i];
    } else if (a.mode == SL_OBS_CHANNELS) {
        store_channels<uint16_t>(out, b, view, nv, a, 1u);
    } else if (a.mode == SL_OBS_CHANNELS_U8) {
        store_channels<uint8_t>(out, b, view, nv, a, 1u);
    } else if (a.mode == SL_OBS_CHANNELS_F32) {
        store_channels<uint32_t>(out, b, view, nv, a, 0x3F800000u);    // 1.0f
    } else {
        store_channels<uint16_t>(out, b, view, nv, a, 0x3F80u);        // 1.0 bf16
    }
}

__global__ void __launch_bounds__(256)
k_env_obs_packed(sl_env_state st, ObsArgs a, uint16_t *__restrict__ out) {
    const int64_t b = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (b >= st.B) return;
    obs_packed_wave(st, a, b, threadIdx.x & 63, out);
}

// channel obs.  Per view cell the wave first stores in LDS the cell's CHANNEL MASK
// m = sum_k bit(v, ch[k]) << k (one AND for the usual channels 0..nch-1); output
// element e = (cell, k) is then bit k of m[cell].  The env's output bytes
// [b R, (b+1) R) are written as 16-byte vectors where they cover a whole aligned
// chunk (R = 32 670 B at 33x33x15 u16 is only 2-byte aligned, so the partial chunks
// at both ends are written element by element).  A chunk's 16 / ESZ element bits are
// gathered from one to three masks and expanded to bytes / halfwords / words by a
// multiply-and-mask spread (no per-element shifts or selects).  ESZ = element bytes;
// `one` = the element's 1 (1, 0x3F80 bf16, 0x3F800000 f32).  LDS: 4 views per
// workgroup, sized by the launch (vpad cells each).
template <int ESZ>
__global__ void __launch_bounds__(256)
k_env_obs_channels(sl_env_state st, ObsArgs a, uint64_t chpack, uint32_t one, int vpad,
                   uint8_t *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) uint16_t obs_lds[];
    const int wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int64_t b = (int64_t)blockIdx.x * 4 + wid;
    if (b >= st.B) return;
    obs_channels_wave<ESZ>(st, a, ChanMap{chpack, a.nch}, one, b, threadIdx.x & 63,
                           obs_lds + wid * vpad, out);
}

bool set_lds(const void *fn, size_t bytes) {
    if (bytes <= 65536) return true;
    return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) ==
           hipSuccess;
}

unsigned reset_grid(int64_t B) { return (unsigned)(B < 2048 ? B : 2048); }

bool state_ok(const sl_env_state *st) {
    return st && st->B >= 0 && st->H >= 2 && st->W >= 2 && st->board && st->goals &&
           st->start_board && (int64_t)st->H * st->W <= kMaxCells;
}

ResetArgs reset_args(const sl_env_cfg *cfg) {
    ResetArgs r;
    r.wrapper_min_perf = cfg->wrapper_min_performance;
    r.seed = cfg->seed;
    r.env0 = cfg->env0;
    r.level_mode = cfg->level_mode;
    r.n_total = cfg->n_total_envs > 0 ? cfg->n_total_envs : 1;
    r.augment = cfg->augment_roll;
    r.bonus_period = cfg->bonus_period;
    r.toggle_powers = cfg->can_toggle_powers;
    return r;
}

int obs_args(int vh, int vw, int remove_white, int mode, const int32_t *channels, int nch,
             ObsArgs *a) {
    if (vh < 1 || vw < 1 || (int64_t)vh * vw > kMaxCells) return SL_EINVAL;
    if (mode < SL_OBS_PACKED || mode > SL_OBS_CHANNELS_BF16) return SL_EINVAL;
    a->vh = vh;
    a->vw = vw;
    a->remove_white = remove_white;
    a->mode = mode;
    a->nch = 0;
    if (mode != SL_OBS_PACKED) {
        if (!channels || nch < 1 || nch > 16) return SL_EINVAL;
        a->nch = nch;
        for (int k = 0; k < nch; k++) {
            if (channels[k] < 0 || channels[k] > 15) return SL_EINVAL;
            a->ch[k] = channels[k];
        }
    }
    return SL_OK;
}

int launch_obs(const sl_env_state &st, const ObsArgs &a, void *out, hipStream_t s) {
    if (st.B == 0) return SL_OK;
    const int nv = a.vh * a.vw;
    if (a.mode == SL_OBS_PACKED && nv <= kObsMaxCells) {
        hipLaunchKernelGGL(k_env_obs_packed, dim3((unsigned)((st.B + 3) / 4)), dim3(256), 0, s, st,
                           a, (uint16_t *)out);
        return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
    }
    if ((((uintptr_t)out) & 15) == 0 && nv <= kObsMaxCells) {
        uint64_t chpack = 0;
        for (int k = 0; k < a.nch; k++) chpack |= (uint64_t)a.ch[k] << (4 * k);
        const uint32_t one = a.mode == SL_OBS_CHANNELS_F32 ? 0x3F800000u
                             : a.mode == SL_OBS_CHANNELS_BF16 ? 0x3F80u : 1u;
        const dim3 grid((unsigned)((st.B + 3) / 4));
        uint8_t *o = (uint8_t *)out;
        // + 2 cells: a chunk's bit gather may read up to two masks past the last cell
        const int vpad = (nv + 2 + 7) & ~7;
        const size_t lds = (size_t)4 * vpad * sizeof(uint16_t);
        if (a.mode == SL_OBS_CHANNELS_U8)
            hipLaunchKernelGGL(k_env_obs_channels<1>, grid, dim3(256), lds, s, st, a, chpack, one,
                               vpad, o);
        else if (a.mode == SL_OBS_CHANNELS_F32)
            hipLaunchKernelGGL(k_env_obs_channels<4>, grid, dim3(256), lds, s, st, a, chpack, one,
                               vpad, o);
        else
            hipLaunchKernelGGL(k_env_obs_channels<2>, grid, dim3(256), lds, s, st, a, chpack, one,
                               vpad, o);
        return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
    }
    // unaligned output or a large view: the LDS-staged kernel, one workgroup per env
    const size_t lds = (size_t)nv * sizeof(uint16_t);
    if (!set_lds((const void *)k_env_obs, lds)) return SL_ETOOBIG;
    hipLaunchKernelGGL(k_env_obs, dim3((unsigned)st.B), dim3(NT), lds, s, st, a, out);
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}

}  // namespace

namespace sl {
int launch_env_action(const sl_env_state &st, const int32_t *actions, int ctp, int ctc,
                      int64_t *act, hipStream_t s) {
    hipLaunchKernelGGL(k_env_action<false>, dim3((unsigned)((st.B + 255) / 256)), dim3(256), 0,
                       s, st, actions, ctp, ctc, act);
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}

int launch_obs_reset_list(const sl_env_state &st, const ObsArgs &a, uint16_t *out,
                          const int64_t *scratch, uint32_t step, hipStream_t s) {
    const unsigned grid = (unsigned)(st.B < 1024 ? (st.B + 3) / 4 : 256);
    hipLaunchKernelGGL(k_env_obs_reset_list, dim3(grid), dim3(256), 0, s, st, a, scratch, step, out);
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}

int launch_reset_list_wide(const sl_env_state &st, const sl_level_pool &pool, const ResetArgs &ra,
                           int64_t *scratch, uint32_t step, hipStream_t s) {
    const unsigned grid = (unsigned)(st.B < 256 ? st.B : 256);
    hipLaunchKernelGGL(k_env_reset_list_wide, dim3(grid), dim3(NTR), 0, s, st, pool, ra, scratch,
                       step);
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}
}  // namespace sl

extern "C" const char *sl_version(void) { return "safelife-hip 0.2 (gfx950)"; }

// sl_build_id(): sl_buildid.cpp, compiled with every link (the hash of all sources)

extern "C" int sl_device_arch(char *buf, int len) {
    int dev;
    hipDeviceProp_t p;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess)
        return SL_EHIP;
    int n = 0;
    while (p.gcnArchName[n] && n < len - 1) {
        buf[n] = p.gcnArchName[n];
        n++;
    }
    if (len > 0) buf[n] = 0;
    return SL_OK;
}

extern "C" int sl_event_create(void **ev) {
    if (!ev) return SL_EINVAL;
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return SL_EHIP;
    *ev = (void *)e;
    return SL_OK;
}

extern "C" int sl_event_destroy(void *ev) {
    return hipEventDestroy((hipEvent_t)ev) == hipSuccess ? SL_OK : SL_EHIP;
}

extern "C" int sl_event_elapsed_ms(void *begin, void *end, float *ms) {
    if (!begin || !end || !ms) return SL_EINVAL;
    return hipEventElapsedTime(ms, (hipEvent_t)begin, (hipEvent_t)end) == hipSuccess ? SL_OK
                                                                                    : SL_EHIP;
}

namespace {
// one 16-byte load per lane per iteration over 1024 workgroups: the fastest of the
// copy shapes measured on MI355X (tools/bwtest.hip: 5.9 TB/s read + write; more
// loads in flight or more workgroups 4.5-5.2)
__global__ void __launch_bounds__(256) k_copy16(const uint4 *__restrict__ src,
                                                uint4 *__restrict__ dst, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) dst[i] = src[i];
}
}  // namespace

extern "C" int sl_copy16(const void *src, void *dst, int64_t n16, void *stream) {
    if (n16 < 0 || (n16 > 0 && (!src || !dst)) || ((uintptr_t)src & 15) || ((uintptr_t)dst & 15))
        return SL_EINVAL;
    if (n16 == 0) return SL_OK;
    hipLaunchKernelGGL(k_copy16, dim3(1024), dim3(256), 0, (hipStream_t)stream,
                       (const uint4 *)src, (uint4 *)dst, n16);
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}

extern "C" int sl_level_pool_prepare(sl_level_pool *pool, void *stream) {
    if (!pool || pool->K <= 0 || (pool->H != 64 && pool->H != 128) || pool->W < 2 ||
        !pool->board || !pool->board_planes)
        return SL_EINVAL;
    const int64_t n = (int64_t)pool->K * 16 * (pool->H / 32) * pool->W;
    const unsigned grid = (unsigned)std::min<int64_t>((n + NT - 1) / NT, 4096);
    hipLaunchKernelGGL(k_pool_planes, dim3(grid), dim3(NT), 0, (hipStream_t)stream, *pool);
    if (pool->goal_planes && pool->H == 128) {
        if (!pool->goals) return SL_EINVAL;
        const int64_t ng = (int64_t)pool->K * 3 * (pool->H / 32) * pool->W;
        const unsigned gg = (unsigned)std::min<int64_t>((ng + NT - 1) / NT, 4096);
        hipLaunchKernelGGL(k_pool_goal_planes, dim3(gg), dim3(NT), 0, (hipStream_t)stream, *pool);
    }
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}

namespace {
// A bit ring serves only envs whose threshold is the ring's: any env that draws this
// step with another one flags the stream error -- bit 1 (SL_STREAM_ERR_THRESHOLD), not
// the ring's range bit 0: the fix is a ring of doubles, not a re-seed
__global__ void __launch_bounds__(256)
k_bits_thr_check(const float *__restrict__ spawn_prob, const int64_t *__restrict__ counts,
                 int64_t B, double thr, int64_t *__restrict__ err) {
    const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (b < B && (counts[2 * b] | counts[2 * b + 1]) && (double)spawn_prob[b] != thr)
        atomicOr((unsigned long long *)err, (unsigned long long)SL_STREAM_ERR_THRESHOLD);
}
}  // namespace

int sl::bits_thr_check(const sl_env_state &st, const sl_mt19937 *mt, const int64_t *counts,
                       int64_t *err, hipStream_t s) {
    if (!mt || !mt->bit_ring || st.B == 0) return SL_OK;
    hipLaunchKernelGGL(k_bits_thr_check, dim3((unsigned)((st.B + 255) / 256)), dim3(256), 0, s,
                       st.spawn_prob, counts, st.B, mt->bits_thr, err);
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}

int sl::stream_offsets(const sl_env_state &st, const FastExtra &fx, hipStream_t s) {
    const Scratch sc = scratch_of(fx.scratch, st.B);
    if (fx.mt && fx.stream_phase != 2 && !fx.thr_checked) {
        const int rcb = bits_thr_check(st, fx.mt, sc.counts, sc.err, s);
        if (rcb) return rcb;
    }
    // phase 0: from the stream position; 1: from 0 (only the total matters, it lands
    // in *stream_pos); 2: from the shard's base the caller placed in *stream_base
    const int64_t *base = fx.stream_phase == 1 ? nullptr
                          : fx.stream_phase == 2 ? fx.stream_base : fx.stream_pos;
    const int rc = sl_exclusive_scan_i64(sc.counts, sc.offsets, 2 * st.B, base, fx.stream_pos,
                                         (void *)s);
    // the device generator: every block holding a draw of [offsets[0], *stream_pos)
    if (rc || !fx.mt || fx.stream_phase == 1) return rc;
    return sl_mt19937_fill(fx.mt, sc.offsets, fx.stream_pos, sc.err, (void *)s);
}

extern "C" int sl_env_reset(sl_env_state *st, const sl_level_pool *pool, const uint8_t *mask,
                            const sl_env_cfg *cfg, void *stream) {
    if (!state_ok(st) || !pool || !cfg || pool->K <= 0 || pool->H != st->H || pool->W != st->W)
        return SL_EINVAL;
    if (st->B == 0) return SL_OK;
    hipLaunchKernelGGL(k_env_reset, dim3(reset_grid(st->B)), dim3(NT), 0, (hipStream_t)stream,
                       *st, *pool, mask, (const uint8_t *)nullptr, reset_args(cfg));
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}

// The board planes' sync (sync_board_planes), skipped while no step of this state has
// left a board in planes since the last demotion (sl_env_state.planes_live: a step that
// is not in plane mode, e.g. with channel views, launched no-op syncs otherwise)
static int sync_planes(const sl_env_state *st, hipStream_t s) {
    return st->planes_live ? sync_board_planes(*st, 0, s) : SL_OK;
}
static int demote_planes(sl_env_state *st, hipStream_t s) {
    if (!st->planes_live) return SL_OK;
    const int rc = sync_board_planes(*st, 1, s);
    if (!rc) st->planes_live = 0;
    return rc;
}

extern "C" int sl_env_step(sl_env_state *st, const sl_level_pool *pool, const int32_t *actions,
                           const sl_env_cfg *cfg, double *reward, uint8_t *done,
                           uint8_t *info_flags, int32_t *ep_len, int32_t *ep_reward,
                           void *stream) {
    if (!state_ok(st) || !cfg || !actions || !reward || !done || !cfg->scratch) return SL_EINVAL;
    if (cfg->bonus_period < 0 || cfg->bonus_period > SL_BONUS_PERIOD_MAX) return SL_EINVAL;
    if (cfg->bonus_period > 0 && (!cfg->bonus_table || cfg->bonus_len < 1)) return SL_EINVAL;
    if (cfg->auto_reset && (!pool || !info_flags || pool->K <= 0 || pool->H != st->H ||
                            pool->W != st->W))
        return SL_EINVAL;
    const int64_t B = st->B;
    if (B == 0) return SL_OK;
    hipStream_t s = (hipStream_t)stream;
    Scratch sc = scratch_of(cfg->scratch, B);
    const size_t lds = (size_t)2 * st->H * st->W * sizeof(uint16_t);

    StepArgs a;
    a.time_limit = cfg->time_limit;
    a.auto_reset = cfg->auto_reset;
    a.bonus_len = cfg->bonus_len;
    a.bonus_period = cfg->bonus_period;
    a.penalty_coef = cfg->penalty_coef;
    a.bonus_table = cfg->bonus_table;
    a.seed = cfg->seed;
    a.step = cfg->step;
    a.env0 = cfg->env0;
    a.draws = cfg->draws;
    a.n_draws = cfg->n_draws;

    if (cfg->rng_mode != SL_RNG_STREAM && cfg->rng_mode != SL_RNG_PHILOX) return SL_EINVAL;
    const bool replay = cfg->rng_mode == SL_RNG_STREAM;
    if (replay && cfg->mt) {       // draws from the device generator's ring
        a.draws = cfg->mt->ring;
        a.n_draws = INT64_MAX;
        a.draw_mask = cfg->mt->ring_draws - 1;
        if (cfg->mt->bit_ring) {
            a.draw_bits = reinterpret_cast<const uint32_t *>(cfg->mt->ring);
            a.bits_thr = cfg->mt->bits_thr;
        }
    }
    if (replay && (!cfg->stream_pos || (!a.draws && a.n_draws > 0))) return SL_EINVAL;
    if (cfg->stream_phase < 0 || cfg->stream_phase > 2 || (cfg->stream_phase && !replay) ||
        (cfg->stream_phase == 2 && !cfg->stream_base))
        return SL_EINVAL;
    const bool bits_ok = cfg->kernel != SL_KERNEL_GENERIC;
    const bool fast = bits_ok && st->H == 64 && st->W == 64;
    const bool fast128 = bits_ok && bits128_shape(*st);
    const bool small = bits_ok && !fast && small_shape(*st);
    if (cfg->kernel == SL_KERNEL_FAST && !fast && !fast128 && !small) return SL_ETOOBIG;
    bool reset_done = false;
    FastExtra fx;
    fx.fuse_reset = cfg->auto_reset ? 1 : 0;
    if (pool) fx.pool = *pool;
    else fx.pool = sl_level_pool{};
    fx.ra = reset_args(cfg);
    fx.scratch = cfg->scratch;
    fx.ev_end = cfg->ev_end;
    const sl_capture *cap = (cfg->capture && cfg->capture->n > 0) ? cfg->capture : nullptr;
    if (cap && (!cap->env || !cap->board || !cap->goals || !cap->orientation || !cap->flags ||
                !cap->reset_board || !cap->reset_goals || !cap->reset_orientation ||
                !info_flags || !cfg->auto_reset))
        return SL_EINVAL;
    fx.capture = cap;
    fx.stream = replay ? 1 : 0;
    fx.stream_pos = cfg->stream_pos;
    fx.stream_phase = cfg->stream_phase;
    fx.stream_base = cfg->stream_base;
    fx.mt = replay ? cfg->mt : nullptr;
    if (fx.mt && fx.mt->bit_ring) fx.bits_thr = fx.mt->bits_thr;
    fx.ev_begin = cfg->ev_begin;
    // the small-board kernel resets finished envs inside the step; with a capture the
    // resets run in the follow-up scan so the pre-reset frame can be copied first.
    // The 64x64 / 128x128 launchers copy that frame between their step kernel and
    // their reset-list kernel, so they keep the list (and its per-parity lengths,
    // which only the reset-list kernel clears) going through captured steps.
    if (cap && small) fx.fuse_reset = 0;
    ObsArgs oa;
    if (cfg->obs_out) {
        const int rc = obs_args(cfg->obs_vh, cfg->obs_vw, cfg->obs_remove_white, cfg->obs_mode,
                                cfg->obs_channels, cfg->obs_nch, &oa);
        if (rc) return rc;
    }
    // 128x128 board planes: a step of the fast kernel without capture keeps the board
    // in them -- with no views, or with packed views of at most kViewMaxRows rows,
    // which the step kernel writes from the planes (fuse_obs128); any other step first
    // completes (and demotes) it.  (Replay: with draw planes, the decided form.)
    const bool planes128 = st->board_planes && st->planes_ok && st->H == 128 && st->W == 128;
    if (cfg->board_mode != SL_BOARD_AUTO && cfg->board_mode != SL_BOARD_UINT16) return SL_EINVAL;
    const bool fuse_obs128 = fast128 && planes128 && cfg->obs_out && !cap &&
                             cfg->board_mode != SL_BOARD_UINT16 &&
                             (!replay || st->elig_planes) && oa.mode == SL_OBS_PACKED &&
                             oa.vh <= kViewMaxRows128 && oa.vw <= 128;
    fx.plane_mode = (fast128 && planes128 && (!cfg->obs_out || fuse_obs128) && !cap &&
                     (!replay || st->elig_planes) && cfg->board_mode != SL_BOARD_UINT16) ? 1 : 0;
    // 64x64: a Philox step without views or capture (sl_bits.hip, plane mode)
    const bool planes64 = planes64_shape(*st);
    if (planes64)       // (packed views: written from the planes, fused_obs64 below)
        fx.plane_mode = (fast && !cap && !replay && cfg->board_mode != SL_BOARD_UINT16 &&
                         (!cfg->obs_out || (oa.mode == SL_OBS_PACKED &&
                                            oa.vh * oa.vw <= kObsMaxCells))) ? 1 : 0;
    if ((planes128 || planes64) && !fx.plane_mode) {
        const int rc = demote_planes(st, s);
        if (rc) return rc;
    }
    // (a plane-mode step below leaves boards in planes)
    if (fx.plane_mode && cfg->stream_phase != 1) st->planes_live = 1;
    // observations: packed views of 64x64 boards come out of the step kernel itself
    // ... and channel views too (one wave writes its env's 16-byte chunks from the
    // view masks it builds in LDS: views up to kFusedChanCells cells, 16-B aligned out)
    const bool fuse_obs =
        cfg->obs_out && fast &&
        ((oa.mode == SL_OBS_PACKED && oa.vh * oa.vw <= kObsMaxCells) ||
         (oa.mode != SL_OBS_PACKED && oa.vh <= 64 && oa.vw <= 64 &&
          oa.vh * oa.vw + 2 <= kFusedChanCells && (((uintptr_t)cfg->obs_out) & 15) == 0));
    fx.obs_out = (fuse_obs || fuse_obs128) ? (uint16_t *)cfg->obs_out : nullptr;
    fx.obs_vh = cfg->obs_vh;
    fx.obs_vw = cfg->obs_vw;
    fx.obs_rw = cfg->obs_remove_white;
    fx.obs_mode = SL_OBS_PACKED;
    fx.obs_nch = 0;
    fx.obs_chpack = 0;
    fx.obs_one = 1u;
    if (cfg->obs_out) {
        fx.obs_mode = oa.mode;
        fx.obs_nch = oa.nch;
        for (int k = 0; k < oa.nch; k++) fx.obs_chpack |= (uint64_t)oa.ch[k] << (4 * k);
        fx.obs_one = oa.mode == SL_OBS_CHANNELS_F32 ? 0x3F800000u
                     : oa.mode == SL_OBS_CHANNELS_BF16 ? 0x3F80u : 1u;
    }
    if (fast128) {
        int rc = launch_step_bits128(*st, a, fx, actions, cfg->can_toggle_powers,
                                     cfg->can_toggle_colors, reward, done, info_flags, ep_len,
                                     ep_reward, s);
        if (rc || cfg->stream_phase == 1) return rc;
        reset_done = fx.fuse_reset && fx.pool.K > 0;
    } else if (small) {
        int rc = launch_step_small(*st, a, fx, actions, cfg->can_toggle_powers,
                                   cfg->can_toggle_colors, reward, done, info_flags, ep_len,
                                   ep_reward, s);
        if (rc || cfg->stream_phase == 1) return rc;
        reset_done = fx.fuse_reset && fx.pool.K > 0 && fx.pool.H == st->H && fx.pool.W == st->W;
    } else if (fast) {
        int rc = launch_step_bits(*st, a, fx, actions, cfg->can_toggle_powers,
                                  cfg->can_toggle_colors, reward, done, info_flags, ep_len,
                                  ep_reward, s);
        if (rc || cfg->stream_phase == 1) return rc;
        reset_done = fx.fuse_reset && fx.pool.K > 0;
    } else {
        if (!replay || stream_counts(fx)) {
            hipLaunchKernelGGL(k_env_action<true>, dim3((unsigned)((B + 255) / 256)), dim3(256), 0,
                               s, *st, actions, cfg->can_toggle_powers, cfg->can_toggle_colors,
                               sc.act);
            if (hipGetLastError() != hipSuccess) return SL_EHIP;
        }
        if (replay) {
            if (stream_counts(fx)) {
                if (!set_lds((const void *)k_env_count, lds)) return SL_ETOOBIG;
                hipLaunchKernelGGL(k_env_count, dim3((unsigned)B), dim3(NT), lds, s, *st, sc.counts);
                if (hipGetLastError() != hipSuccess) return SL_EHIP;
            }
            int rc = stream_offsets(*st, fx, s);
            if (rc || cfg->stream_phase == 1) return rc;
            if (!set_lds((const void *)k_env_step_generic<SL_RNG_STREAM>, lds)) return SL_ETOOBIG;
            hipLaunchKernelGGL(k_env_step_generic<SL_RNG_STREAM>, dim3((unsigned)B), dim3(NT), lds,
                               s, *st, a, sc.act, sc.offsets, sc.err, reward, done, info_flags,
                               ep_len, ep_reward);
        } else {
            if (!set_lds((const void *)k_env_step_generic<SL_RNG_PHILOX>, lds)) return SL_ETOOBIG;
            if (cfg->ev_begin) (void)hipEventRecord((hipEvent_t)cfg->ev_begin, s);
            hipLaunchKernelGGL(k_env_step_generic<SL_RNG_PHILOX>, dim3((unsigned)B), dim3(NT), lds,
                               s, *st, a, sc.act, sc.offsets, sc.err, reward, done, info_flags,
                               ep_len, ep_reward);
        }
    }
    if (hipGetLastError() != hipSuccess) return SL_EHIP;
    // the bit-sliced 64x64 / 128x128 launchers record ev_end themselves, between the
    // step kernel and their reset-list kernel
    if (cfg->ev_end && !fast && !fast128) (void)hipEventRecord((hipEvent_t)cfg->ev_end, s);

    if (cap && !fast && !fast128) {
        const int rc = launch_capture(*st, *cap, info_flags, 0, s);
        if (rc) return rc;
    }
    if (cfg->auto_reset && !reset_done) {
        hipLaunchKernelGGL(k_env_reset_scan, dim3((unsigned)((B + NT - 1) / NT)), dim3(NT), 0, s,
                           *st, *pool, (const uint8_t *)info_flags, reset_args(cfg));
        if (hipGetLastError() != hipSuccess) return SL_EHIP;
    }
    if (cfg->obs_out) {
        if (fuse_obs128) {
            // the step kernel wrote every view from the planes; the envs the reset-list
            // kernel reset get theirs from the new episode's uint16 board
            if (reset_done) {
                const int rc = launch_obs_reset_list(*st, oa, (uint16_t *)cfg->obs_out,
                                                     cfg->scratch, cfg->step, s);
                if (rc) return rc;
            }
        } else if (!fuse_obs || (cfg->auto_reset && !reset_done)) {
            const int rc = launch_obs(*st, oa, cfg->obs_out, s);
            if (rc) return rc;
        }
        // else: the reset-list kernel wrote the views of the envs it reset
    }
    if (cap) return launch_capture(*st, *cap, info_flags, 1, s);
    return SL_OK;
}

// ---------------------------------------------------------------------------
// trajectory capture (sl_capture): one block per captured env, one uint16 cell per
// thread per iteration (a few envs per step: not worth vector copies)
// ---------------------------------------------------------------------------
namespace {
__global__ void __launch_bounds__(NT)
k_capture(sl_env_state st, sl_capture c, const uint8_t *__restrict__ flags, int phase) {
    const int i = blockIdx.x;
    const int64_t b = c.env[i];
    if (b < 0 || b >= st.B) return;
    const int64_t hw = (int64_t)st.H * st.W;
    uint16_t *ob = (phase ? c.reset_board : c.board) + i * hw;
    uint16_t *og = (phase ? c.reset_goals : c.goals) + i * hw;
    const uint16_t *sb = st.board + b * hw, *sg = st.goals + b * hw;
    for (int64_t k = threadIdx.x; k < hw; k += NT) {
        ob[k] = sb[k];
        og[k] = sg[k];
    }
    if (threadIdx.x == 0) {
        (phase ? c.reset_orientation : c.orientation)[i] = st.orientation[b];
        if (!phase) c.flags[i] = flags[b];
    }
}

}  // namespace

int sl::launch_capture(const sl_env_state &st, const sl_capture &c, const uint8_t *flags,
                       int phase, hipStream_t s) {
    hipLaunchKernelGGL(k_capture, dim3((unsigned)c.n), dim3(NT), 0, s, st, c, flags, phase);
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}

extern "C" int sl_env_obs(const sl_env_state *st, int vh, int vw, int remove_white_goals,
                          int obs_mode, const int32_t *channels, int nch, void *out,
                          void *stream) {
    if (!state_ok(st) || !out) return SL_EINVAL;
    ObsArgs a;
    int rc = obs_args(vh, vw, remove_white_goals, obs_mode, channels, nch, &a);
    if (rc) return rc;
    rc = sync_planes(st, (hipStream_t)stream);
    if (rc) return rc;
    return launch_obs(*st, a, out, (hipStream_t)stream);
}

extern "C" int sl_env_board_sync(sl_env_state *st, void *stream) {
    if (!state_ok(st)) return SL_EINVAL;
    return sync_planes(st, (hipStream_t)stream);
}

// ---------------------------------------------------------------------------
// game-level entry points (include/safelife_hip.h)
// ---------------------------------------------------------------------------
extern "C" int sl_env_action(sl_env_state *st, const int32_t *actions, int can_toggle_powers,
                             int can_toggle_colors, int64_t *act, void *stream) {
    if (!state_ok(st) || !actions || !act) return SL_EINVAL;
    if (st->B == 0) return SL_OK;
    const int rc = demote_planes(st, (hipStream_t)stream);
    if (rc) return rc;
    hipLaunchKernelGGL(k_env_action<true>, dim3((unsigned)((st->B + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, *st, actions, can_toggle_powers, can_toggle_colors,
                       act);
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}

extern "C" int sl_env_advance(sl_env_state *st, const sl_env_cfg *cfg, void *stream) {
    if (!state_ok(st) || !cfg || !cfg->scratch) return SL_EINVAL;
    if (cfg->rng_mode != SL_RNG_STREAM && cfg->rng_mode != SL_RNG_PHILOX) return SL_EINVAL;
    const bool replay = cfg->rng_mode == SL_RNG_STREAM;
    if (replay && !cfg->mt && (!cfg->stream_pos || (!cfg->draws && cfg->n_draws > 0)))
        return SL_EINVAL;
    if (replay && !cfg->stream_pos) return SL_EINVAL;
    const int64_t B = st->B;
    if (B == 0) return SL_OK;
    hipStream_t s = (hipStream_t)stream;
    const int rcs = demote_planes(st, s);
    if (rcs) return rcs;
    const Scratch sc = scratch_of(cfg->scratch, B);
    const size_t lds = (size_t)2 * st->H * st->W * sizeof(uint16_t);
    StepArgs a{};
    a.seed = cfg->seed;
    a.step = cfg->step;
    a.env0 = cfg->env0;
    a.draws = cfg->draws;
    a.n_draws = cfg->n_draws;
    if (replay && cfg->mt) {
        a.draws = cfg->mt->ring;
        a.n_draws = INT64_MAX;
        a.draw_mask = cfg->mt->ring_draws - 1;
        if (cfg->mt->bit_ring) {
            a.draw_bits = reinterpret_cast<const uint32_t *>(cfg->mt->ring);
            a.bits_thr = cfg->mt->bits_thr;
        }
    }
    if (replay) {
        if (!set_lds((const void *)k_env_count, lds)) return SL_ETOOBIG;
        hipLaunchKernelGGL(k_env_count, dim3((unsigned)B), dim3(NT), lds, s, *st, sc.counts);
        if (hipGetLastError() != hipSuccess) return SL_EHIP;
        int rc = bits_thr_check(*st, cfg->mt, sc.counts, sc.err, s);
        if (!rc)
            rc = sl_exclusive_scan_i64(sc.counts, sc.offsets, 2 * B, cfg->stream_pos,
                                       cfg->stream_pos, stream);
        if (!rc && cfg->mt) rc = sl_mt19937_fill(cfg->mt, sc.offsets, cfg->stream_pos, sc.err, stream);
        if (rc) return rc;
        if (!set_lds((const void *)k_env_advance<SL_RNG_STREAM>, lds)) return SL_ETOOBIG;
        hipLaunchKernelGGL(k_env_advance<SL_RNG_STREAM>, dim3((unsigned)B), dim3(NT), lds, s,
                           *st, a, sc.offsets, sc.err);
    } else {
        if (!set_lds((const void *)k_env_advance<SL_RNG_PHILOX>, lds)) return SL_ETOOBIG;
        hipLaunchKernelGGL(k_env_advance<SL_RNG_PHILOX>, dim3((unsigned)B), dim3(NT), lds, s,
                           *st, a, sc.offsets, sc.err);
    }
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}

extern "C" int sl_env_rescore(sl_env_state *st, int32_t *points, void *stream) {
    if (!state_ok(st)) return SL_EINVAL;
    if (st->B == 0) return SL_OK;
    const int rc = sync_planes(st, (hipStream_t)stream);
    if (rc) return rc;
    hipLaunchKernelGGL(k_env_rescore, dim3((unsigned)st->B), dim3(NT), 0, (hipStream_t)stream,
                       *st, points);
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}

extern "C" int sl_env_exit_colors(sl_env_state *st, int mode, void *stream) {
    if (!state_ok(st) || (mode != 0 && mode != 1)) return SL_EINVAL;
    if (st->B == 0) return SL_OK;
    const int rc = demote_planes(st, (hipStream_t)stream);
    if (rc) return rc;
    hipLaunchKernelGGL(k_env_exit_colors, dim3((unsigned)((st->B + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, *st, mode);
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}
