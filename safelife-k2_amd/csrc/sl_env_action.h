// sl_env_action.h -- SafeLifeGame.execute_action / move_agent for one env by one
// lane (safelife_game.py:294-393): the body of k_env_action (sl_env.hip).  (Round 5
// also ran it on lane 0 of the 128x128 replay count prologue's waves, folding the
// action launch into that kernel: 48.9 vs 50.2 M env-steps/s, not kept;
// tools/ab/c5s_fold.py.)
#pragma once
#include "sl_env_common.h"

namespace sl {

__device__ __forceinline__ void forward_vec(int orientation, int *fx, int *fy) {
    // relative_loc(n_forward=1): dx=0, dy=-1 rotated clockwise `orientation` times
    int dx = 0, dy = -1;
    for (int k = 0; k < (orientation & 3); k++) {
        int t = dx;
        dx = -dy;
        dy = t;
    }
    *fx = dx;
    *fy = dy;
}

// ---------------------------------------------------------------------------
// actions: one lane per env (cells touched: agent, front, behind, 2 ahead)
// ---------------------------------------------------------------------------
// (points, score, side-effect) terms of one cell; see cell_scores / side_term
__device__ __forceinline__ void cell_terms(uint32_t bv, uint32_t gv, uint32_t sv, int *p, int *q,
                                           int *se) {
    int r;
    cell_scores(bv, gv, p, q, &r);
    *se = side_term(bv, sv, gv);
}

// The action edits at most the 4 cells agent / front / behind / two ahead.  DELTAS:
// their contribution to the running scores is re-evaluated too (pre vs post edit, act
// words 1-3), and the goals mirror is marked stale (the per-cell path does not keep
// it); without DELTAS only the reward is written (the 128x128 kernel's pre-pass).
template <bool DELTAS>
__device__ __forceinline__ void env_action_one(const sl_env_state &st,
                                               const int32_t *__restrict__ actions, int ctp,
                                               int ctc, int64_t *__restrict__ act, int64_t b) {
    if (DELTAS && st.planes_ok) st.planes_ok[b] = 0;
    const int H = st.H, W = st.W;
    const int64_t hw = (int64_t)H * W;
    uint16_t *bd = st.board + b * hw;
    const uint16_t *gd = st.goals + b * hw, *sd = st.start_board + b * hw;
    int reward = 0, d_pts = 0, d_scr = 0, d_side = 0;
    uint32_t edit_rows = 0xFFFFFFFFu;      // rows the action may have edited (0xFF: none)
    const int a = actions[b];
    if (!st.game_over[b] && a >= 1 && a <= 8) {
        const int orient = (a - 1) & 3;
        st.orientation[b] = orient;
        int fx, fy;
        forward_vec(orient, &fx, &fy);
        const int x0 = st.agent_x[b], y0 = st.agent_y[b];
        const int x1 = pymod(x0 + fx, W), y1 = pymod(y0 + fy, H);
        // distinct cells the action may touch
        int cells[4] = {y0 * W + x0, y1 * W + x1, pymod(y0 - fy, H) * W + pymod(x0 - fx, W),
                        pymod(y0 + 2 * fy, H) * W + pymod(x0 + 2 * fx, W)};
        bool uniq[4];
        for (int k = 0; k < 4; k++) {
            uniq[k] = true;
            for (int j = 0; j < k; j++) uniq[k] = uniq[k] && cells[j] != cells[k];
        }
        if (DELTAS)
            for (int k = 0; k < 4; k++)
                if (uniq[k]) {
                    int p, q, se;
                    cell_terms(bd[cells[k]], gd[cells[k]], sd[cells[k]], &p, &q, &se);
                    d_pts -= p; d_scr -= q; d_side -= se;
                }
        if (a <= 4) {
            // move_agent(1)
            const int x2 = pymod(x0 - fx, W), y2 = pymod(y0 - fy, H);
            int nx = x0, ny = y0;
            uint32_t c1 = bd[y1 * W + x1];
            if (c1 == 0) {
                bd[y1 * W + x1] = bd[y0 * W + x0];
                bd[y0 * W + x0] = 0;
                nx = x1; ny = y1;
            } else if ((c1 & EXIT) &&
                       can_exit_now(st.min_performance[b], st.score[b], st.baseline[b],
                                    st.possible[b])) {
                st.game_over[b] = 1;
                reward += 1;
            } else if (c1 & PUSHABLE) {
                const int x3 = pymod(x0 + 2 * fx, W), y3 = pymod(y0 + 2 * fy, H);
                uint32_t c3 = bd[y3 * W + x3];
                if (c3 == 0) {
                    bd[y3 * W + x3] = bd[y1 * W + x1];
                    bd[y1 * W + x1] = bd[y0 * W + x0];
                    bd[y0 * W + x0] = 0;
                    nx = x1; ny = y1;
                } else if (c3 & EXIT) {
                    bd[y1 * W + x1] = bd[y0 * W + x0];
                    bd[y0 * W + x0] = 0;
                    nx = x1; ny = y1;
                }
            }
            const bool moved = (nx == x1 && ny == y1) && !(x0 == x1 && y0 == y1);
            if (moved && (bd[y2 * W + x2] & PULLABLE)) {
                bd[y0 * W + x0] = bd[y2 * W + x2];
                bd[y2 * W + x2] = 0;
            }
            st.agent_x[b] = nx;
            st.agent_y[b] = ny;
        } else {
            // TOGGLE
            const uint32_t pc = bd[y0 * W + x0] & COLORS;
            const uint32_t t = bd[y1 * W + x1];
            if (t == 0) {
                bd[y1 * W + x1] = (uint16_t)(LIFE | pc);
            } else if (t & DESTR) {
                bd[y1 * W + x1] = 0;
            } else {
                uint32_t tb = (ctp ? POWERS : 0u) | (ctc ? COLORS : 0u);
                bd[y0 * W + x0] = (uint16_t)(bd[y0 * W + x0] ^ (t & tb));
            }
        }
        if (DELTAS)
            for (int k = 0; k < 4; k++)
                if (uniq[k]) {
                    int p, q, se;
                    cell_terms(bd[cells[k]], gd[cells[k]], sd[cells[k]], &p, &q, &se);
                    d_pts += p; d_scr += q; d_side += se;
                }
        // the 128x128 replay count mirror (sl_env_state.elig_planes) is behind by the
        // rows of these cells: the count prologue re-reads them from the board
        if (!DELTAS && st.elig_planes && H == 128 && W == 128) {
            uint32_t rows = 0xFFFFFFFFu;
            for (int k = 0; k < 4; k++) {
                const uint32_t y = (uint32_t)(cells[k] >> 7);
                bool seen = false;
                for (int j = 0; j < 4; j++) seen = seen || ((rows >> (8 * j)) & 0xFFu) == y;
                if (!seen) rows = (rows << 8) | y;
            }
            edit_rows = rows;
        }
    }
    act[b] = reward;
    if (!DELTAS && st.elig_planes) act[st.B + b] = (int64_t)edit_rows;
    if (DELTAS) {
        act[st.B + b] = d_pts;
        act[2 * st.B + b] = d_scr;
        act[3 * st.B + b] = d_side;
    }
}
}  // namespace sl
