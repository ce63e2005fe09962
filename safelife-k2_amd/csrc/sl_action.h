// sl_action.h -- pieces shared by the fused bit-sliced step kernels (sl_bits.hip,
// sl_bits128.hip, sl_bits_small.hip): the score lookup table and the single-lane action evaluator.
#pragma once
#include "sl_env_common.h"

namespace sl {
namespace fast {

// ---------------------------------------------------------------- scoring
// LDS lookup table, index (goal colour << 3) | cell colour:
//   bits 0-3: point_table + 3, bits 4-5: sign(point_table) + 1, bit 6: max(sign row)
struct ScoreTbl {
    uint16_t e[64];
};

__device__ __forceinline__ uint32_t score_entry(uint32_t g, uint32_t c) {
    const int t = point_value(g, c);
    return (uint32_t)((t + 3) | ((sgn(t) + 1) << 4) | (possible_value(g) << 6));
}

__device__ __forceinline__ void cell_terms_lds(const ScoreTbl *tb, uint32_t b, uint32_t g,
                                               uint32_t s, int *p, int *q, int *r, int *se) {
    const uint32_t i = ((g >> 6) & 0x38u) | ((b >> 9) & 7u);
    const uint32_t e = tb ? tb->e[i] : score_entry(i >> 3, i & 7);
    const bool alive = b & ALIVE;
    const bool m = alive && ((b & (FROZEN | MOVABLE)) != FROZEN);
    *p = alive ? (int)(e & 15u) - 3 : 0;
    *q = m ? (int)((e >> 4) & 3u) - 1 : 0;
    *r = (int)((e >> 6) & 1u);
    *se = side_term(b, s, g);
}

// ---------------------------------------------------------------- action
// execute_action / move_agent (safelife_game.py:308-393) on a 4-cell overlay of
// the board.  Run by one lane (or wave-uniformly); produces the cell edits, the
// action reward and (lane_action) the score deltas of the edited cells.
//   Src: where the unedited cells come from (the board in HBM, or a copy in LDS)
struct GlobalCells {
    const uint16_t *bd;
    __device__ __forceinline__ uint32_t operator()(int i) const { return bd[i]; }
};

template <class Src>
struct OverlayT {
    int n;
    int idx[4];
    uint32_t val[4];
    Src src;
    // fully unrolled, statically indexed: the slots stay in registers
    __device__ uint32_t get(int i) const {
        uint32_t r = 0;
        bool hit = false;
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (k < n && idx[k] == i) {
                r = val[k];
                hit = true;
            }
        return hit ? r : src(i);
    }
    __device__ void set(int i, uint32_t v) {
        bool hit = false;
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (k < n && idx[k] == i) {
                val[k] = v;
                hit = true;
            }
        if (!hit) {
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (k == n) {
                    idx[k] = i;
                    val[k] = v;
                }
            n++;
        }
    }
};
using Overlay = OverlayT<GlobalCells>;

struct ActResult {
    int reward, dp, dq, dse;
};

__device__ __forceinline__ int pm(int a, int m) {
    int r = a % m;
    return r < 0 ? r + m : r;
}
// the torus wrap of a coordinate at most one period outside [0, m) (m >= 2: every
// neighbour offset of the action is within +-2), without a division
__device__ __forceinline__ int wrap1(int a, int m) {
    return a < 0 ? a + m : (a >= m ? a - m : a);
}

// the per-env fields the action reads and writes, straight from sl_env_state
struct GlobalEnv {
    const sl_env_state &st;
    int64_t b;
    __device__ int game_over() const { return st.game_over[b]; }
    __device__ int agent_x() const { return st.agent_x[b]; }
    __device__ int agent_y() const { return st.agent_y[b]; }
    __device__ bool can_exit() const {
        return can_exit_now(st.min_performance[b], st.score[b], st.baseline[b], st.possible[b]);
    }
    __device__ void set_orientation(int o) { st.orientation[b] = o; }
    __device__ void set_game_over() { st.game_over[b] = 1; }
    __device__ void set_agent(int x, int y) {
        st.agent_x[b] = x;
        st.agent_y[b] = y;
    }
};

// action a (0..8, safelife_env.py:61-71) on env e; the reward is 1 when the agent
// walks into an open exit (move_agent, safelife_game.py:356-364), else 0
// cell (y, x) is overlay index y * S + x, S = STRIDE (0: W); a kernel whose cell
// source is a padded row image passes the padding stride and decodes indices by shifts
template <int STRIDE = 0, class Env, class Src>
__device__ __forceinline__ int act_core(Env &e, int a, int H, int W, int ctp, int ctc,
                                        OverlayT<Src> &ov) {
    const int S = STRIDE ? STRIDE : W;
    ov.n = 0;
    if (e.game_over() || a < 1 || a > 8) return 0;
    int reward = 0;
    const int orient = (a - 1) & 3;
    e.set_orientation(orient);
    const int fx = orient == 1 ? 1 : (orient == 3 ? -1 : 0);
    const int fy = orient == 0 ? -1 : (orient == 2 ? 1 : 0);
    const int x0 = e.agent_x(), y0 = e.agent_y();
    const int x1 = wrap1(x0 + fx, W), y1 = wrap1(y0 + fy, H);
    const int i0 = y0 * S + x0, i1 = y1 * S + x1;
    if (a <= 4) {
        const int i2 = wrap1(y0 - fy, H) * S + wrap1(x0 - fx, W);
        int nx = x0, ny = y0;
        const uint32_t c1 = ov.get(i1);
        if (c1 == 0) {
            ov.set(i1, ov.get(i0));
            ov.set(i0, 0);
            nx = x1; ny = y1;
        } else if ((c1 & EXIT) && e.can_exit()) {
            e.set_game_over();
            reward = 1;
        } else if (c1 & PUSHABLE) {
            const int i3 = wrap1(y0 + 2 * fy, H) * S + wrap1(x0 + 2 * fx, W);
            const uint32_t c3 = ov.get(i3);
            if (c3 == 0) {
                ov.set(i3, ov.get(i1));
                ov.set(i1, ov.get(i0));
                ov.set(i0, 0);
                nx = x1; ny = y1;
            } else if (c3 & EXIT) {
                ov.set(i1, ov.get(i0));
                ov.set(i0, 0);
                nx = x1; ny = y1;
            }
        }
        const bool moved = (nx == x1 && ny == y1) && !(x0 == x1 && y0 == y1);
        if (moved && (ov.get(i2) & PULLABLE)) {
            ov.set(i0, ov.get(i2));
            ov.set(i2, 0);
        }
        e.set_agent(nx, ny);
    } else {
        const uint32_t pc = ov.get(i0) & COLORS;
        const uint32_t t = ov.get(i1);
        if (t == 0) {
            ov.set(i1, LIFE | pc);
        } else if (t & DESTR) {
            ov.set(i1, 0);
        } else {
            const uint32_t tbits = (ctp ? POWERS : 0u) | (ctc ? COLORS : 0u);
            ov.set(i0, ov.get(i0) ^ (t & tbits));
        }
    }
    return reward;
}

template <bool DELTA = true>
__device__ ActResult lane_action(const sl_env_state &st, int64_t b, int a, int ctp, int ctc,
                                 const ScoreTbl *tb, Overlay &ov) {
    const int H = st.H, W = st.W;
    const int64_t hw = (int64_t)H * W;
    const uint16_t *gd = st.goals + b * hw, *sd = st.start_board + b * hw;
    GlobalEnv e{st, b};
    ActResult res{act_core(e, a, H, W, ctp, ctc, ov), 0, 0, 0};
    if (DELTA) for (int k = 0; k < ov.n; k++) {
        const int i = ov.idx[k];
        int p0, q0, r0, e0, p1, q1, r1, e1;
        cell_terms_lds(tb, ov.src(i), gd[i], sd[i], &p0, &q0, &r0, &e0);
        cell_terms_lds(tb, ov.val[k], gd[i], sd[i], &p1, &q1, &r1, &e1);
        res.dp += p1 - p0;
        res.dq += q1 - q0;
        res.dse += e1 - e0;
    }
    return res;
}

}  // namespace fast
}  // namespace sl
