// sl_bits128.hip -- the bit-sliced fused env-step kernel for 128x128 boards
// (BASELINE config C5: navigation levels with spawners and oscillators).
//
// Same semantics as k_env_action + k_env_step_generic (sl_env.hip); the layout is
// the 64x64 kernel's (sl_bits.hip) stretched to 128 columns:
//
//  * one wave64 per env; lane j owns the column pair (2j, 2j+1), so the wave spans
//    the 128 columns and the whole-wave DPP rotations wrap exactly at W = 128;
//  * the 128 rows are four bands of 32, processed one after another: a band's 32
//    dwords D[y] = cell(32t+y, 2j) | cell(32t+y, 2j+1) << 16 are loaded (every load
//    instruction covers one full 256-byte row) and transposed in registers into 16
//    bit planes x 2 words;
//  * the rows just outside a band (32t-1 and 32t+32, wrapping at H = 128) enter the
//    rule as halo words (bit 31 = the row above, bit 0 = the row below): every 3x3
//    quantity the rule folds is evaluated on the band's planes and on the halo
//    planes, and a funnel shift (v_alignbit) joins them.  The eight halo rows are
//    read before any band is written back, so every band sees the pre-step board;
//  * points, performance score, possible score and side effects
//    (safelife_game.py:590-631, env_wrappers.py:319-342) are summed band by band;
//    only the rows that changed are stored;
//  * goals: a bit-plane mirror (sl_env_state.planes, [B][band][32 words][64 lanes])
//    holds their planes.  Goals without spawners that came through a step unchanged
//    are at a fixed point of the rule (planes_ok bit 2): the rule is skipped and only
//    their three colour planes are read, per band, for the scores;
//  * the action (execute_action / move_agent, safelife_game.py:308-393) runs on lane
//    0 against the board in HBM before any band is stored; its cell edits are
//    broadcast and written into the band planes and halo rows before the rule;
//  * exits are rewritten by the epilogue after the band stores have completed.
// Finished envs are reset by the generic follow-up kernel (k_env_reset_scan).
#include "sl_bits.h"

using namespace sl;
using namespace sl::fast;
using namespace sl::bits;

namespace {

#ifndef SL_B128_MINW
#define SL_B128_MINW 2       // waves per SIMD the register budget is sized for
#endif

constexpr int N = 128;       // rows = columns
constexpr int RS = N / 2;    // dwords per row
constexpr int NB = N / 32;   // bands of 32 rows
constexpr int MW = 32 * 64;  // mirror dwords per band (32 words x 64 lanes)

// The rows just outside a band as "planes": element p is a word with bit 31 = bit p
// of the row above's cell pair and bit 0 = bit p of the row below's, computed where
// the rule uses it (two registers live instead of the full 32-word array).
struct HaloView {
    u32 up, dn;
    __device__ __forceinline__ u32 operator[](int p) const {
        return ((up >> p) << 31) | ((dn >> p) & 1u);
    }
};

// Neighbourhood of a band word: columns from the neighbouring lanes (2j - 1 is word
// 1 of lane j - 1, 2j + 2 word 0 of lane j + 1), rows outside the band from the halo
// (plane k, word w: bit 31 = row 32t - 1, bit 0 = row 32t + 32).
struct GeoBand {
    int lane, row0;
    HaloView hv;
    template <class F>
    __device__ __forceinline__ V3 vert(const u32 *P, int w, F f) const {
        return vert_with(f(P, w), f(hv, w));
    }
    __device__ __forceinline__ H3 horiz(u32 w0, u32 w1) const {
        return H3{lane_m1(w1), lane_p1(w0)};
    }
    __device__ __forceinline__ bool halo_spawn() const {
        return (PL(hv, 7, 0) | PL(hv, 7, 1)) != 0u;
    }
    __device__ __forceinline__ u32 cell(int y, int w) const {
        return (u32)((row0 + y) * N + 2 * lane + w);
    }
};

// the halo rows of band t from the eight preloaded ones (t is wave-uniform)
__device__ __forceinline__ u32 pick4(const u32 h[4], int t) {
    return t == 0 ? h[0] : t == 1 ? h[1] : t == 2 ? h[2] : h[3];
}

// Applies the action's cell edits (wave-uniform (flat index, value) pairs) to band
// t's planes on the lane owning the cell; returns the band rows (bit y) edited.
__device__ __forceinline__ u32 apply_edits(u32 P[32], int ne, const int eidx[4],
                                           const u32 eval[4], int row0, int lane) {
    u32 erow = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (k < ne) {
            const int y = (eidx[k] >> 7) - row0, x = eidx[k] & (N - 1);
            if (y >= 0 && y < 32) {
                const u32 bit = 1u << y;
                const bool mine = lane == (x >> 1);
                const u32 m0 = (mine && !(x & 1)) ? bit : 0u;
                const u32 m1 = (mine && (x & 1)) ? bit : 0u;
                erow |= bit;
#pragma unroll
                for (int p = 0; p < 16; p++) {
                    const u32 v = ((eval[k] >> p) & 1u) ? ~0u : 0u;
                    PL(P, p, 0) = mux(m0, v, PL(P, p, 0));
                    PL(P, p, 1) = mux(m1, v, PL(P, p, 1));
                }
            }
        }
    }
    return erow;
}

// the same edits on a halo row's raw cell pair (row index r)
__device__ __forceinline__ u32 edit_row(u32 d, int r, int ne, const int eidx[4],
                                        const u32 eval[4], int lane) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (k < ne && (eidx[k] >> 7) == r) {
            const int x = eidx[k] & (N - 1);
            if (lane == (x >> 1))
                d = (x & 1) ? (d & 0x0000FFFFu) | (eval[k] << 16) : (d & 0xFFFF0000u) | eval[k];
        }
    }
    return d;
}

__global__ void __launch_bounds__(64, SL_B128_MINW)
k_env_step_bits128(sl_env_state st, StepArgs a, const int32_t *__restrict__ actions, int ctp,
                   int ctc, double *__restrict__ reward_out, uint8_t *__restrict__ done_out,
                   uint8_t *__restrict__ flags_out, int32_t *__restrict__ ep_len_out,
                   int32_t *__restrict__ ep_rew_out) {
    const int64_t b = blockIdx.x;
    const int lane = threadIdx.x;
    const int64_t off = b * (int64_t)(N * N);
    u32 *gb = reinterpret_cast<u32 *>(st.board + off) + lane;      // row r: gb[r * RS]
    u32 *gg = reinterpret_cast<u32 *>(st.goals + off) + lane;
    const u32 *gs = reinterpret_cast<const u32 *>(st.start_board + off) + lane;
    u32 *mg = st.planes + b * (int64_t)(NB * MW) + lane;            // mirror [t][q][lane]

    const u32 V = load_record(st, actions, b, lane);
    // pre-step halo rows of every band: above (32t - 1) and below (32t + 32)
    u32 bu[NB], bd[NB];
#pragma unroll
    for (int t = 0; t < NB; t++) {
        bu[t] = gb[((32 * t - 1) & (N - 1)) * RS];
        bd[t] = gb[((32 * t + 32) & (N - 1)) * RS];
    }
    const int pok = rec(V, R_POK) & 6;

    SpawnCtx sc;
    sc.gid = a.env0 + (uint32_t)b;
    sc.step = a.step;
    sc.seed = a.seed;
    sc.thr = (double)__int_as_float(rec(V, R_SPAWN));

    // ---- goals: advanced band by band unless at a fixed point; the mirror keeps
    // their planes (all words rewritten when it was stale, else the changed ones)
    if ((pok & 6) != 6) {
        u32 gu[NB], gd[NB];
#pragma unroll
        for (int t = 0; t < NB; t++) {
            gu[t] = gg[((32 * t - 1) & (N - 1)) * RS];
            gd[t] = gg[((32 * t + 32) & (N - 1)) * RS];
        }
        const bool all = !(pok & 2);
        u32 changed = 0, spawners = 0;
#pragma unroll 1
        for (int t = 0; t < NB; t++) {
            u32 G[32];
            load_pairs<RS>(gg + 32 * t * RS, G);
            transpose32(G);
            u32 cg[2];
            rule_planes(G, cg, GeoBand{lane, 32 * t, HaloView{pick4(gu, t), pick4(gd, t)}}, sc,
                        1u);
            const u32 rg = wave_or(cg[0] | cg[1]);
            u32 *m = mg + t * MW;
#pragma unroll
            for (int w = 0; w < 2; w++)
                if (all || cg[w])
#pragma unroll
                    for (int k = 0; k < 16; k++) m[(k + 16 * w) * 64] = PL(G, k, w);
            changed |= rg;
            spawners |= PL(G, 7, 0) | PL(G, 7, 1);
            if (rg) {
                transpose32(G);
                store_pairs<RS>(gg + 32 * t * RS, G, rg);
            }
        }
        const bool fixed = changed == 0 && __ballot(spawners != 0u) == 0ull;
        const int ok = 2 | (fixed ? 4 : 0);
        if (ok != pok && lane == 0) st.planes_ok[b] = ok;
        wait_vm();          // the mirror words are read back below
    }
    __builtin_amdgcn_sched_barrier(0);

    // ---- the action (lane 0) on the pre-step board
    OverlayT<GlobalCells> ov;
    ov.src.bd = st.board + off;
    ov.n = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        ov.idx[k] = 0;
        ov.val[k] = 0;
    }
    RecEnv env{st, b, rec(V, R_GO), rec(V, R_AX), rec(V, R_AY), rec(V, R_SCORE),
               rec(V, R_BASE), rec(V, R_POSS), rec_f64(V, R_MP)};
    int act_reward = 0;
    if (lane == 0) act_reward = act_core(env, rec(V, R_ACT), N, N, ctp, ctc, ov);
    act_reward = __builtin_amdgcn_readfirstlane(act_reward);
    const int ne = __builtin_amdgcn_readfirstlane(ov.n);
    int eidx[4];
    u32 eval[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        eidx[k] = __builtin_amdgcn_readfirstlane(ov.idx[k]);
        eval[k] = (u32)__builtin_amdgcn_readfirstlane((int)ov.val[k]);
    }
    RecFields fl{V, __builtin_amdgcn_readfirstlane(env.go), __builtin_amdgcn_readfirstlane(env.ax),
                 __builtin_amdgcn_readfirstlane(env.ay), 0.0};
    if (a.bonus_period > 0)        // issued now, consumed by the epilogue
        fl.bval = a.bonus_table[bonus_dist(fl.ax, fl.ay, fl.prior_x(fl.prior_head()),
                                           fl.prior_y(fl.prior_head()), fl.prior_len(),
                                           a.bonus_period, a.bonus_len)];
    if (ne > 0) {
#pragma unroll
        for (int t = 0; t < NB; t++) {
            bu[t] = edit_row(bu[t], (32 * t - 1) & (N - 1), ne, eidx, eval, lane);
            bd[t] = edit_row(bd[t], (32 * t + 32) & (N - 1), ne, eidx, eval, lane);
        }
    }

    // ---- board, band by band: rule, scores, changed rows back
    int pts = 0, scr = 0, pos = 0, side = 0;
#pragma unroll 1
    for (int t = 0; t < NB; t++) {
        u32 P[32], S[32];
        load_pairs<RS>(gb + 32 * t * RS, P);
        transpose32(P);
        const u32 erow = apply_edits(P, ne, eidx, eval, 32 * t, lane);
        u32 cb[2];
        rule_planes(P, cb, GeoBand{lane, 32 * t, HaloView{pick4(bu, t), pick4(bd, t)}}, sc, 0u);
        __builtin_amdgcn_sched_barrier(0);
        load_pairs<RS>(gs + 32 * t * RS, S);
        u32 gcol[3][2];
        const u32 *m = mg + t * MW;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            gcol[k][0] = m[(9 + k) * 64];
            gcol[k][1] = m[(25 + k) * 64];
        }
        transpose32(S);
        int p, q, r, e;
        score_planes(P, gcol, S, &p, &q, &r, &e);
        pts += p;
        scr += q;
        pos += r;
        side += e;
        const u32 rb = wave_or(cb[0] | cb[1]) | erow;
        if (rb) {
            transpose32(P);
            store_pairs<RS>(gb + 32 * t * RS, P, rb);
        }
    }
    const int points = wave_total(pts), score = wave_total(scr);
    const int possible = wave_total(pos), side_total = wave_total(side);
    wait_vm();              // row stores land before the epilogue rewrites the exits
    if (lane == 0)
        epilogue_core(st, a, b, fl, act_reward, points, score, possible, side_total, reward_out,
                      done_out, flags_out, ep_len_out, ep_rew_out);
}

}  // namespace

namespace sl {

bool bits128_shape(const sl_env_state &st) {
    return st.H == N && st.W == N && st.planes && st.planes_ok;
}

int launch_step_bits128(const sl_env_state &st, const StepArgs &a, const int32_t *actions,
                        int ctp, int ctc, double *reward, uint8_t *done, uint8_t *flags,
                        int32_t *ep_len, int32_t *ep_rew, hipStream_t s) {
    if (!bits128_shape(st)) return SL_ETOOBIG;
    hipLaunchKernelGGL(k_env_step_bits128, dim3((unsigned)st.B), dim3(64), 0, s, st, a, actions,
                       ctp, ctc, reward, done, flags, ep_len, ep_rew);
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}

}  // namespace sl
