// sl_bits_small.hip -- the bit-sliced fused env-step kernel for small boards
// (H <= 32, W <= 64: BASELINE config C2's 25x25 proc-gen levels, the 26x26 v1.0
// benchmark levels).
//
// Same semantics as k_env_action + k_env_step_generic (sl_env.hip); the layout is the
// 64x64 kernel's (sl_bits.hip) folded to one row band:
//
//  * one wave64 per env; lane j < nl = ceil(W / 2) owns the column pair (2j, 2j+1)
//    over ALL rows: bit y of plane k, word w = bit k of cell(y, 2j + w), so a whole
//    board is 16 planes x 2 words per lane and the rule (sl_bits.h rule_planes,
//    SURVEY.md Appendix A / advance_board.c:34-120) runs on 2 x H cells per op;
//  * vertical neighbours are rotations within the low H bits (the torus wrap at H);
//  * horizontal neighbours come from the neighbouring column pairs through
//    ds_bpermute, which wraps at W for any W (the whole-wave DPP rotations of the
//    64x64 kernel wrap at 64 lanes only).  For odd W the last lane's second word is
//    a copy of column 0 -- exactly the right neighbour its first word needs -- and
//    everything it computes for that word is discarded;
//  * the action (execute_action / move_agent, safelife_game.py:308-393) runs on lane
//    0 against the board staged in LDS; its edits are muxed into the planes;
//  * points, performance score, possible score and side effects
//    (safelife_game.py:590-631, env_wrappers.py:319-342) are recomputed in full from
//    the planes; only changed rows are stored; the epilogue is the shared one.
// Finished envs are reset by their own wave at the end of the step (small_reset).
// Philox draws, or the reference's stream order after a replay prologue
// (k_stream_prologue_small).
#include "sl_bits.h"

using namespace sl;
using namespace sl::fast;
using namespace sl::bits;

namespace {

constexpr int kMaxH = 32, kMaxW = 64;

template <int MODE>
struct GeoSmall {
    int lane, H, W, nl;
    u32 mh;                  // the low H bits
    int src_l, src_r;        // lanes holding columns 2j - 1 and 2j + 2
    bool odd_last;           // this lane's word 1 is the column-0 copy (odd W)
    StreamSrc src;           // SPAWN_STREAM: the supplied uniforms from this tensor's first
    int64_t pos;
    int count;               // SPAWN_COUNT: this lane's eligible cells
    template <class F>
    __device__ __forceinline__ V3 vert(const u32 *P, int w, F f) const {
        const u32 x = f(P, w);
        return V3{((x << 1) | (x >> (H - 1))) & mh, ((x >> 1) | ((x & 1u) << (H - 1))) & mh};
    }
    __device__ __forceinline__ H3 horiz(u32 w0, u32 w1) const {
        const u32 right_col = odd_last ? w0 : w1;          // this lane's last real column
        return H3{(u32)__builtin_amdgcn_ds_bpermute(4 * src_l, (int)right_col),
                  (u32)__builtin_amdgcn_ds_bpermute(4 * src_r, (int)w0)};
    }
    __device__ __forceinline__ bool halo_spawn() const { return false; }
    // the 2x2 spawn block of rows y, y + 1 (y even) of the lane's column pair
    __device__ __forceinline__ u32 block(int y) const { return (u32)((y >> 1) * nl + lane); }
    // (the column-0 copy's draws are discarded with the rest of that word; in replay
    // mode it draws nothing, so it cannot shift the real cells' ranks)
    __device__ __forceinline__ void spawn(const u32 elig[2], u32 sp[2], const SpawnCtx &sc,
                                          u32 tensor) {
        const u32 e[2] = {elig[0], odd_last ? 0u : elig[1]};
        if (MODE == SPAWN_PHILOX) {
            philox_spawn(*this, elig, sp, sc, tensor);
        } else if (MODE == SPAWN_STREAM) {
            (void)stream_draws<false>(e, sp, sc.thr, src, pos, lane);
        } else {
            count += __builtin_popcount(e[0]) + __builtin_popcount(e[1]);
        }
    }
};

// the geometry of lane `lane` on an H x W board (lanes >= ceil(W / 2) hold nothing)
template <int MODE>
__device__ __forceinline__ GeoSmall<MODE> small_geo(int lane, int H, int W) {
    GeoSmall<MODE> g;
    const int nl = (W + 1) >> 1;
    const bool active = lane < nl;
    g.lane = lane;
    g.H = H;
    g.W = W;
    g.nl = nl;
    g.mh = H == 32 ? ~0u : ((1u << H) - 1u);
    g.src_l = active ? (lane == 0 ? nl - 1 : lane - 1) : lane;
    g.src_r = active ? (lane + 1 == nl ? 0 : lane + 1) : lane;
    g.odd_last = (W & 1) && lane == nl - 1;
    g.src = StreamSrc{nullptr, 0, nullptr};
    g.pos = 0;
    g.count = 0;
    return g;
}

typedef __attribute__((address_space(3))) u32 lds_u32;
typedef __attribute__((address_space(3))) const uint16_t lds_cu16;

// unedited cells for the action, from the staged board: row y is 32 dwords, and the
// action indexes cell (y, x) as y * 64 + x (act_core<64>)
struct SmallCells {
    const lds_u32 *buf;
    __device__ __forceinline__ uint32_t operator()(int i) const {
        return reinterpret_cast<lds_cu16 *>(buf)[i];
    }
};

// Board, goals and start board are staged in LDS as rows of 64 u16 (cell (y, x) at
// y * 64 + x), each tensor read by the whole wave with coalesced u16 loads (cells
// lane + 64 k), eight per lane and tensor in flight at once.  For odd W column 0 is
// also written at x = W, so the last lane's second word reads as its copy.
typedef __attribute__((address_space(3))) uint16_t lds_u16;
constexpr int kGroup = 8;

template <int NTEN = 3>
__device__ __forceinline__ void stage_tensors(const uint16_t *const src[NTEN],
                                              lds_u16 *const dst[NTEN], int HW, int W, int lane) {
    const int dy = 64 / W, dx = 64 - dy * W;
    int y = lane / W, x = lane - (lane / W) * W;
    for (int i0 = lane; i0 < HW; i0 += 64 * kGroup) {
        uint32_t v[NTEN][kGroup];
        int pos[kGroup];
#pragma unroll
        for (int g = 0; g < kGroup; g++) {
            const int i = i0 + 64 * g;
            pos[g] = -1;
            if (i < HW) {
#pragma unroll
                for (int t = 0; t < NTEN; t++) v[t][g] = src[t][i];
                pos[g] = y * 64 + x + ((x == 0 && (W & 1)) ? 0x10000 : 0);
            }
            y += dy;
            x += dx;
            if (x >= W) {
                x -= W;
                y++;
            }
        }
#pragma unroll
        for (int g = 0; g < kGroup; g++)
            if (pos[g] >= 0) {
                const int p = pos[g] & 0xFFFF;
#pragma unroll
                for (int t = 0; t < NTEN; t++) {
                    dst[t][p] = (uint16_t)v[t][g];
                    if (pos[g] >> 16) dst[t][p + W] = (uint16_t)v[t][g];    // column-0 copy
                }
            }
    }
}

// the lane's dwords D[y] = cell(y, 2j) | cell(y, 2j + 1) << 16 (0 outside the board)
__device__ __forceinline__ void lds_rows(const lds_u16 *t, int H, bool active, int lane,
                                         u32 D[32]) {
    const lds_u32 *p = reinterpret_cast<const lds_u32 *>(t) + lane;
#pragma unroll
    for (int y = 0; y < kMaxH; y++) D[y] = (active && y < H) ? p[y * 32] : 0u;
}

#ifndef SL_SMALL_MINW
#define SL_SMALL_MINW 3      // waves per SIMD the register budget is sized for (4 spills
                             // a few registers and measured no faster)
#endif

// all kernel arguments in one struct at kernarg offset 0: the epilogue re-reads its
// ~20 pointers where it runs (kargs()), so they are not held in SGPRs through the step
struct SmallKArgs {
    sl_env_state st;
    StepArgs a;
    const int32_t *actions;
    int ctp, ctc;
    double *reward_out;
    uint8_t *done_out, *flags_out;
    int32_t *ep_len_out, *ep_rew_out;
    sl_level_pool pool;       // auto-reset source (K == 0: no reset here)
    ResetArgs ra;
    int64_t *scratch;         // sl_env_cfg.scratch (replay mode: act, offsets, err)
};

__device__ __forceinline__ const SmallKArgs &kargs() {
    auto kp = __builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(kp));
    return *(const SmallKArgs *)kp;
}

// SafeLifeEnv.reset (safelife_env.py:188-198) of env b by its own wave, right after
// the step that ended the episode (ContinuingEnv + run_agents' reset-on-done): the
// same result as reset_one (sl_env.hip).  Pass 1 sums points / baseline / possible
// over the level (a roll permutes cells, so the level's own order is used) and lists
// the exits of the ROLLED board in np.nonzero order (row-major chunks of 64 cells, a
// ballot prefix count within a chunk); pass 2 copies the rolled level into board
// (exits coloured), goals and start board.
__device__ __forceinline__ void small_reset(const sl_env_state &st, const sl_level_pool &pool,
                                            const ResetArgs &ra, int64_t b, int lane) {
    const int H = st.H, W = st.W, hw = H * W;
    int li = 0, dy = 0, dx = 0;
    if (lane == 0) {
        const LevelChoice c = choose_level(pool, ra, ra.env0 + (uint32_t)b, st.episodes[b], H, W);
        li = c.idx;
        dy = c.dy;
        dx = c.dx;
    }
    li = __builtin_amdgcn_readfirstlane(li);
    dy = __builtin_amdgcn_readfirstlane(dy);
    dx = __builtin_amdgcn_readfirstlane(dx);
    const uint16_t *lb = pool.board + (int64_t)li * hw, *lg = pool.goals + (int64_t)li * hw;
    const int dy64 = 64 / W, dx64 = 64 - dy64 * W;
    const uint64_t below = (1ull << lane) - 1ull;
    int p = 0, q = 0, r = 0, spb = 0, n_exit = 0;
    {
        int y = lane / W, x = lane - (lane / W) * W;
        for (int i0 = 0; i0 < hw; i0 += 64) {
            const int i = i0 + lane;
            bool ex = false;
            if (i < hw) {
                const int src = wrap1(y - dy, H) * W + wrap1(x - dx, W);
                const uint32_t vb = lb[src], vg = lg[src];
                int pp, qq, rr;
                cell_scores(vb, vg, &pp, &qq, &rr);
                p += pp;
                q += qq;
                r += rr;
                spb |= ((vb & SPAWN) ? 1 : 0) | ((vg & SPAWN) ? 2 : 0);
                ex = (vb & EXIT) != 0;
            }
            const uint64_t m = __ballot(ex);
            const int rank = __builtin_popcountll(m & below);
            if (ex && n_exit + rank < SL_MAX_EXITS) {
                st.exit_y[b * SL_MAX_EXITS + n_exit + rank] = (int16_t)y;
                st.exit_x[b * SL_MAX_EXITS + n_exit + rank] = (int16_t)x;
            }
            n_exit += __builtin_popcountll(m);
            y += dy64;
            x += dx64;
            if (x >= W) {
                x -= W;
                y++;
            }
        }
    }
    p = wave_total(p);
    q = wave_total(q);
    r = wave_total(r);
    spb = (int)wave_or((u32)spb);
    int ev = 0;
    if (lane == 0) {
        ev = reset_scalars(st, pool, ra, b, li, dy, dx, p, q, r, spb);
        st.exit_count[b] = n_exit;
        for (int e = n_exit; e < SL_MAX_EXITS; e++) {
            st.exit_y[b * SL_MAX_EXITS + e] = 0;
            st.exit_x[b * SL_MAX_EXITS + e] = 0;
        }
    }
    ev = __builtin_amdgcn_readfirstlane(ev);
    const int64_t off = b * (int64_t)hw;
    uint16_t *gb = st.board + off, *gg = st.goals + off, *gs = st.start_board + off;
    int y = lane / W, x = lane - (lane / W) * W;
    for (int i = lane; i < hw; i += 64) {
        const int src = wrap1(y - dy, H) * W + wrap1(x - dx, W);
        const uint16_t vb = lb[src];
        gs[i] = vb;
        gb[i] = (vb & EXIT) ? (uint16_t)ev : vb;
        gg[i] = lg[src];
        y += dy64;
        x += dx64;
        if (x >= W) {
            x -= W;
            y++;
        }
    }
}

// MODE: SPAWN_PHILOX, or SPAWN_STREAM (replay: k_env_action has run the action and
// k_stream_prologue_small sized the draws; the step reads act[b] and each tensor's first uniform
// from the scratch words)
template <int MODE>
__global__ void __launch_bounds__(64, SL_SMALL_MINW)
k_env_step_small(SmallKArgs ka) {
    const sl_env_state &st = ka.st;
    const StepArgs &a = ka.a;
    const int32_t *__restrict__ actions = ka.actions;
    const int ctp = ka.ctp, ctc = ka.ctc;
    const int64_t b = blockIdx.x;
    const int lane = threadIdx.x;
    const int H = st.H, W = st.W, nl = (W + 1) >> 1;
    // board, goals, start board: H rows of 32 dwords each (dynamic: 9.4 KiB at 25 rows,
    // so four waves per SIMD fit the CU's LDS)
    extern __shared__ __attribute__((aligned(16))) u32 dyn_stage[];
    u32 *stage[3] = {dyn_stage, dyn_stage + H * 32, dyn_stage + 2 * H * 32};
    lds_u32 *buf = (lds_u32 *)stage[0];
    const bool active = lane < nl;
    const int c0 = 2 * lane, c1 = 2 * lane + 1;             // stores: c1 < W unless odd_last
    GeoSmall<MODE> geo = small_geo<MODE>(lane, H, W);
    int64_t pos_b = 0, pos_g = 0;
    if (MODE == SPAWN_STREAM) {
        const Scratch w = scratch_of(ka.scratch, st.B);
        geo.src = StreamSrc{a.draws, a.n_draws, w.err, a.draw_mask, a.draw_bits};
        pos_b = w.offsets[2 * b];
        pos_g = w.offsets[2 * b + 1];
    }
    // valid cells per word: rows < H of real columns
    const u32 wm0 = active ? geo.mh : 0u, wm1 = (active && !geo.odd_last) ? geo.mh : 0u;

    const int64_t off = b * (int64_t)H * W;
    const u32 V = load_record(st, actions, b, lane);
    {
        const uint16_t *src[3] = {st.board + off, st.goals + off, st.start_board + off};
        lds_u16 *dst[3] = {(lds_u16 *)stage[0], (lds_u16 *)stage[1], (lds_u16 *)stage[2]};
        // rows of odd boards end in the column-0 copy; the rest of a row stays unread
        stage_tensors(src, dst, H * W, W, lane);
    }
    wait_lgkm();
    u32 PB[32], PG[32];
    lds_rows((const lds_u16 *)stage[1], H, active, lane, PG);

    SpawnCtx sc;
    sc.gid = a.env0 + (uint32_t)b;
    sc.step = a.step;
    sc.seed = a.seed;
    set_spawn_prob(sc, __int_as_float(rec(V, R_SPAWN)));

    // ---- goals: rule, then store the changed rows
    transpose32(PG);
    u32 cg[2];
    geo.pos = pos_g;
    rule_planes(PG, cg, geo, sc, 1u);
    cg[0] &= wm0;
    cg[1] &= wm1;
    const u32 rg = wave_or(cg[0] | cg[1]);
    u32 gcol[3][2];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        gcol[k][0] = PL(PG, 9 + k, 0) & wm0;
        gcol[k][1] = PL(PG, 9 + k, 1) & wm1;
    }
    if (rg) {
        transpose32(PG);
        uint16_t *gg = st.goals + off;
#pragma unroll
        for (int y = 0; y < kMaxH; y++)
            if (((rg >> y) & 1u) && active) {
                gg[y * W + c0] = (uint16_t)PG[y];
                if (!geo.odd_last) gg[y * W + c1] = (uint16_t)(PG[y] >> 16);
            }
    }
    __builtin_amdgcn_sched_barrier(0);

    // ---- board: the action reads the staged cells, then the rows become planes
    OverlayT<SmallCells> ov;
    ov.src.buf = buf;
    ov.n = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        ov.idx[k] = 0;
        ov.val[k] = 0;
    }
    RecEnv env{st, b, rec(V, R_GO), rec(V, R_AX), rec(V, R_AY), rec(V, R_SCORE),
               rec(V, R_BASE), rec(V, R_POSS), rec_f64(V, R_MP)};
    int act_reward = 0;
    if (MODE == SPAWN_STREAM) {        // k_env_action ran the action (no edits left)
        act_reward = (int)scratch_of(ka.scratch, st.B).act[b];
    } else {
        if (lane == 0) act_reward = act_core<64>(env, rec(V, R_ACT), H, W, ctp, ctc, ov);
        act_reward = __builtin_amdgcn_readfirstlane(act_reward);
    }
    // the action's cell edits go straight into the staged board (lane 0; the wave's LDS
    // operations run in order, so the row reads below see them), the column-0 copy of
    // an odd board too; erow = the rows holding an edit
    u32 erow = 0;
    if (lane == 0) {
        lds_u16 *cells = (lds_u16 *)stage[0];
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (k < ov.n) {
                const int i = ov.idx[k];
                cells[i] = (uint16_t)ov.val[k];
                if ((W & 1) && (i & 63) == 0) cells[i + W] = (uint16_t)ov.val[k];
                erow |= 1u << (i >> 6);
            }
    }
    erow = (u32)__builtin_amdgcn_readfirstlane((int)erow);
    RecFields fl{V, __builtin_amdgcn_readfirstlane(env.go), __builtin_amdgcn_readfirstlane(env.ax),
                 __builtin_amdgcn_readfirstlane(env.ay), 0.0};
    if (a.bonus_period > 0)
        fl.bval = a.bonus_table[bonus_dist(fl.ax, fl.ay, fl.prior_x(fl.prior_head()),
                                           fl.prior_y(fl.prior_head()), fl.prior_len(),
                                           a.bonus_period, a.bonus_len)];
    lds_rows((const lds_u16 *)stage[0], H, active, lane, PB);
    transpose32(PB);
    u32 cb[2];
    geo.pos = pos_b;
    rule_planes(PB, cb, geo, sc, 0u);
    __builtin_amdgcn_sched_barrier(0);

    // ---- scores over the real cells of the new board and goals
    u32 PS[32];
    lds_rows((const lds_u16 *)stage[2], H, active, lane, PS);
    transpose32(PS);
#pragma unroll
    for (int p = 0; p < 16; p++) {
        PL(PB, p, 0) &= wm0;
        PL(PB, p, 1) &= wm1;
        PL(PS, p, 0) &= wm0;
        PL(PS, p, 1) &= wm1;
    }
    int pts, scr, pos, side;
    score_planes(PB, gcol, PS, &pts, &scr, &pos, &side);
    const int s1 = wave_total((pts + 192) | ((scr + 64) << 16));
    const int s2 = wave_total(pos | (side << 16));
    const int points = (s1 & 0xFFFF) - 192 * 64;
    const int score = ((s1 >> 16) & 0xFFFF) - 64 * 64;
    const int possible = s2 & 0xFFFF;
    const int side_total = (s2 >> 16) & 0xFFFF;
    __builtin_amdgcn_sched_barrier(0);

    // ---- changed rows, exits in the colour the epilogue gives them
    const u32 rb = wave_or((cb[0] & wm0) | (cb[1] & wm1)) | erow;
    if (rb) {
        const bool can = can_exit_now(fl.min_performance(), score, fl.baseline(), possible);
#pragma unroll
        for (int w = 0; w < 2; w++)
            PL(PB, 9, w) = can ? (PL(PB, 9, w) | PL(PB, 8, w)) : (PL(PB, 9, w) & ~PL(PB, 8, w));
        transpose32(PB);
        uint16_t *gb = st.board + off;
#pragma unroll
        for (int y = 0; y < kMaxH; y++)
            if (((rb >> y) & 1u) && active) {
                gb[y * W + c0] = (uint16_t)PB[y];
                if (!geo.odd_last) gb[y * W + c1] = (uint16_t)(PB[y] >> 16);
            }
    }
    int rs = 0;
    if (lane == 0) {
        const SmallKArgs &k = kargs();
        rs = epilogue_core(k.st, k.a, b, fl, act_reward, points, score, possible, side_total,
                           k.reward_out, k.done_out, k.flags_out, k.ep_len_out, k.ep_rew_out)
                 ? 1 : 0;
    }
    rs = __builtin_amdgcn_readfirstlane(rs);
    if (rs) {
        const SmallKArgs &k = kargs();
        if (k.pool.K > 0) {
            wait_vm();         // this step's stores to the env have completed
            small_reset(k.st, k.pool, k.ra, b, lane);
        }
    }
}

// ============================================================================
// Four envs per wave (boards up to 32 x 32: C2's 25x25 proc-gen levels, the 26x26
// v1.0 benchmark levels).  The layout above uses nl = ceil(W/2) <= 16 lanes of 64 on
// such boards; here env e of the wave (global env 4 * blockIdx + e) owns lanes
// 16e .. 16e+15 -- one DPP row -- so each wave64 instruction advances four boards.
// Per-env sums and masks are DPP row reductions (seg_total / seg_or), horizontal
// neighbours stay ds_bpermute within the segment, the per-env record is four
// registers (lane 16e + k of register q = field 16q + k of env e, fetched with
// ds_bpermute), and the action and epilogue run on each segment's first lane.  Exits
// are coloured in the planes (their rows stored when the colour changes), so the
// epilogue writes no cells.  Envs whose episode ended are reset one at a time by the
// whole wave (small_reset).
// ============================================================================
constexpr int kSegW = 32;            // widest board

__device__ __forceinline__ u32 seg_or(u32 v) {          // OR over the lane's DPP row
    v |= dpp<0x121>(v);    // row_ror:1
    v |= dpp<0x122>(v);    // row_ror:2
    v |= dpp<0x124>(v);    // row_ror:4
    v |= dpp<0x128>(v);    // row_ror:8
    return v;
}
__device__ __forceinline__ int seg_total(int x) {        // sum over the lane's DPP row
    u32 v = (u32)x;
    v += dpp<0x121>(v);
    v += dpp<0x122>(v);
    v += dpp<0x124>(v);
    v += dpp<0x128>(v);
    return (int)v;
}

// Spawn draws with per-lane env parameters (each segment is another env): Philox
// blocks as lane_draws, with the lane's own threshold.
template <class Geo>
__device__ __forceinline__ void seg_philox(const Geo &g, const u32 elig[2], u32 sp[2],
                                           const SpawnCtx &sc, u32 tensor) {
    sp[0] = 0u;
    sp[1] = 0u;
    if (sc.thr >= 1.0) {
        sp[0] = elig[0];
        sp[1] = elig[1];
    } else if (sc.thr > 0.0) {
        const u32 lim = sc.lim;
        const u32 any = elig[0] | elig[1];
        u32 blocks = (any | (any >> 1)) & 0x55555555u, s0 = 0u, s1 = 0u;
        while (blocks) {
            const int y = __builtin_ctz(blocks);
            blocks &= blocks - 1;
            uint32_t r[4];
            philox4x32(g.block(y), sc.gid, sc.step, tensor, sc.seed, r);
            s0 |= ((r[0] <= lim ? 1u : 0u) | (r[2] <= lim ? 2u : 0u)) << y;
            s1 |= ((r[1] <= lim ? 1u : 0u) | (r[3] <= lim ? 2u : 0u)) << y;
        }
        sp[0] = s0 & elig[0];
        sp[1] = s1 & elig[1];
    }
}

// Reference-order draws (stream_draws, sl_bits.h) per segment: ranks count the lower
// lanes of the lane's own segment, the row prefix and the stream position are the
// lane's env's own.
__device__ __forceinline__ void seg_stream(const u32 elig[2], u32 sp[2], double thr,
                                           const StreamSrc &src, int64_t pos, int lane) {
    const uint64_t seg = 0xFFFFull << (16 * (lane >> 4));
    const bool draw = thr > 0.0 && thr < 1.0;
    const u32 rows = wave_or(elig[0] | elig[1]);
    int pre = 0;
    u32 s0 = 0u, s1 = 0u;
#pragma unroll
    for (int c = 0; c < 32; c += 4) {
        if (((rows >> c) & 0xFu) == 0u) continue;
        int64_t r[4][2];
        bool e[4][2];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int y = c + k;
            e[k][0] = (elig[0] >> y) & 1u;
            e[k][1] = (elig[1] >> y) & 1u;
            const uint64_t m0 = __ballot(e[k][0]) & seg, m1 = __ballot(e[k][1]) & seg;
            const int64_t at = pos + pre + lanes_below(m0) + lanes_below(m1);
            r[k][0] = at;
            r[k][1] = at + (e[k][0] ? 1 : 0);
            pre += __builtin_popcountll(m0) + __builtin_popcountll(m1);
        }
        double u[4][2];
#pragma unroll
        for (int k = 0; k < 4; k++)
#pragma unroll
            for (int w = 0; w < 2; w++)
                u[k][w] = (draw && e[k][w] && r[k][w] < src.n)
                              ? stream_u(src.draws, src.bits, r[k][w], src.mask) : 1.0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (draw && ((e[k][0] && r[k][0] >= src.n) || (e[k][1] && r[k][1] >= src.n)))
                atomicOr((unsigned long long *)src.err, 1ull);
            s0 |= ((e[k][0] && (thr >= 1.0 || u[k][0] < thr)) ? 1u : 0u) << (c + k);
            s1 |= ((e[k][1] && (thr >= 1.0 || u[k][1] < thr)) ? 1u : 0u) << (c + k);
        }
    }
    sp[0] = s0;
    sp[1] = s1;
}

// DPPN: the neighbouring column pairs come from DPP row rotations (row_ror:1 / :15,
// no LDS round trip): a segment's spare lanes hold copies so that the rotations wrap
// at nl -- lane nl a copy of lane 0 (the right neighbour of lane nl - 1) and lane 15
// a copy of lane nl - 1 (the left neighbour of lane 0); nl = 16 wraps by itself.  For
// nl = 15 one spare lane cannot be both, and ds_bpermute is used instead.
template <int MODE, bool DPPN>
struct GeoSeg {
    int lane, j, H, W, nl;      // lane of the wave; j = lane within the env's segment
    u32 mh;                     // the low H bits
    int src_l, src_r;           // lanes holding columns 2j - 1 and 2j + 2 (ds_bpermute)
    bool odd_last;              // word 1 is the column-0 copy (odd W)
    bool real;                  // the lane holds its own column pair (not a copy)
    StreamSrc src;
    int64_t pos;
    int count;
    template <class F>
    __device__ __forceinline__ V3 vert(const u32 *P, int w, F f) const {
        const u32 x = f(P, w);
        return V3{((x << 1) | (x >> (H - 1))) & mh, ((x >> 1) | ((x & 1u) << (H - 1))) & mh};
    }
    __device__ __forceinline__ H3 horiz(u32 w0, u32 w1) const {
        const u32 right_col = odd_last ? w0 : w1;
        if (DPPN) return H3{dpp<0x121>(right_col), dpp<0x12F>(w0)};    // row_ror:1, :15
        return H3{(u32)__builtin_amdgcn_ds_bpermute(4 * src_l, (int)right_col),
                  (u32)__builtin_amdgcn_ds_bpermute(4 * src_r, (int)w0)};
    }
    __device__ __forceinline__ bool halo_spawn() const { return false; }
    __device__ __forceinline__ u32 block(int y) const { return (u32)((y >> 1) * nl + j); }
    // copies and the column-0 copy draw nothing (their results are discarded, and in
    // replay mode they must not shift the real cells' ranks)
    __device__ __forceinline__ void spawn(const u32 elig[2], u32 sp[2], const SpawnCtx &sc,
                                          u32 tensor) {
        const u32 e[2] = {real ? elig[0] : 0u, (real && !odd_last) ? elig[1] : 0u};
        if (MODE == SPAWN_PHILOX) {
            seg_philox(*this, e, sp, sc, tensor);
        } else if (MODE == SPAWN_STREAM) {
            seg_stream(e, sp, sc.thr, src, pos, lane);
        } else {
            count += __builtin_popcount(e[0]) + __builtin_popcount(e[1]);
        }
    }
};

// per-env record: field f of the lane's env (all lanes of the wave active)
struct SegRecord {
    u32 R[4];
    int base;                    // byte address of the segment's lane 0 for ds_bpermute
    __device__ __forceinline__ int get(int f) const {
        return __builtin_amdgcn_ds_bpermute(base + 4 * (f & 15), (int)R[f >> 4]);
    }
};
__device__ __forceinline__ SegRecord load_seg_record(const sl_env_state &st, const int32_t *actions,
                                                     int64_t b, bool live, int lane) {
    SegRecord r;
    r.base = 4 * (lane & ~15);
#pragma unroll
    for (int q = 0; q < 4; q++)
        r.R[q] = live ? load_record(st, actions, b, 16 * q + (lane & 15)) : 0u;
    return r;
}

// what epilogue_core reads, gathered while every lane is active (the epilogue then
// runs on the segments' first lanes only); exits are already in the planes
struct SegFields {
    int op, ns, el, er, base, go, ax, ay, plen, phead, px, py, side;
    double mp, bval;
    __device__ int old_points() const { return op; }
    __device__ int num_steps() const { return ns; }
    __device__ int episode_length() const { return el; }
    __device__ int episode_reward() const { return er; }
    __device__ double min_performance() const { return mp; }
    __device__ int baseline() const { return base; }
    __device__ int exit_count() const { return 0; }
    __device__ int exit_y(int) const { return 0; }
    __device__ int exit_x(int) const { return 0; }
    __device__ int game_over() const { return go; }
    __device__ int agent_x() const { return ax; }
    __device__ int agent_y() const { return ay; }
    __device__ int prior_len() const { return plen; }
    __device__ int prior_head() const { return phead; }
    __device__ int prior_x(int) const { return px; }
    __device__ int prior_y(int) const { return py; }
    __device__ int side_effect() const { return side; }
    __device__ double bonus(int) const { return bval; }
};

// Board, goals and start board of the wave's four envs into LDS by DMA: the four
// envs are consecutive, so each tensor's part is one contiguous block of 4 * H * W
// u16 in HBM (it starts 8-byte aligned: b0 is a multiple of 4), copied dword by dword
// with global_load_lds (no registers held, every copy in flight at once).  Tensor t
// sits at u16 offset t * seg_stride(H, W) of the stage, env e's cell (y, x) at e * H * W +
// y * W + x within it.
// u16 per staged tensor: the four envs' 4 * H * W cells rounded up to whole 64-dword
// DMA granules (the clamped lanes of the last granule write up to its end)
__host__ __device__ __forceinline__ int seg_stride(int H, int W) {
    return 128 * ((2 * H * W + 63) / 64);
}
__device__ __forceinline__ void dma_seg(const sl_env_state &st, int64_t b0, int nenv,
                                        lds_u32 *stage, int lane) {
    const int64_t HW = (int64_t)st.H * st.W;
    const int nbytes = (int)(nenv * HW * 2), nd = nbytes >> 2;
    const uint16_t *src[3] = {st.board + b0 * HW, st.goals + b0 * HW, st.start_board + b0 * HW};
#pragma unroll
    for (int t = 0; t < 3; t++) {
        const char *g = reinterpret_cast<const char *>(src[t]);
        lds_u32 *dst = stage + t * (seg_stride(st.H, st.W) / 2);
        for (int k = 0; k * 64 < nd; k++) {
            const int d = k * 64 + lane;
            __builtin_amdgcn_global_load_lds((const void *)(g + 4 * (d < nd ? d : 0)),
                                             (__attribute__((address_space(3))) void *)(dst + k * 64),
                                             4, 0, 0);
        }
    }
}
// an odd cell count leaves each tensor's last u16 outside the dwords: copied after the
// DMA has landed (its clamped lanes write the dwords past the block)
__device__ __forceinline__ void dma_seg_tail(const sl_env_state &st, int64_t b0, int nenv,
                                             lds_u32 *stage, int lane) {
    const int64_t HW = (int64_t)st.H * st.W;
    const int n = (int)(nenv * HW);
    if ((n & 1) && lane < 3) {
        const uint16_t *src = (lane == 0 ? st.board : lane == 1 ? st.goals : st.start_board) +
                              b0 * HW;
        reinterpret_cast<lds_u16 *>(stage + lane * (seg_stride(st.H, st.W) / 2))[n - 1] =
            src[n - 1];
    }
}

// the lane's dwords D[y] = cell(y, 2j) | cell(y, 2j + 1) << 16 of a staged tensor
// (t: the env's cells; for odd W the last lane's second column is column 0)
__device__ __forceinline__ void seg_rows(const lds_u16 *t, int H, int W, bool active, int j,
                                         bool odd_last, u32 D[32]) {
    const int x0 = 2 * j, x1 = odd_last ? 0 : 2 * j + 1;
#pragma unroll
    for (int y = 0; y < kMaxH; y++)
        D[y] = (active && y < H) ? (u32)t[y * W + x0] | ((u32)t[y * W + x1] << 16) : 0u;
}

struct SegCells {       // unedited cells for the action (cell (y, x) at y * W + x)
    const lds_u16 *cells;
    __device__ __forceinline__ uint32_t operator()(int i) const { return cells[i]; }
};

// 2 waves/SIMD is the register budget: a 4096-env batch is 1024 waves, one per SIMD
template <int MODE, bool DPPN>
__global__ void __launch_bounds__(64, 2)
k_env_step_seg4(SmallKArgs ka) {
    const sl_env_state &st = ka.st;
    const StepArgs &a = ka.a;
    const int lane = threadIdx.x, e = lane >> 4, j = lane & 15;
    const int64_t b0 = 4 * (int64_t)blockIdx.x;
    const int nenv = (int)min((int64_t)4, st.B - b0);
    const int64_t b = b0 + e;
    const bool live = e < nenv;                       // this segment holds an env
    const int H = st.H, W = st.W, nl = (W + 1) >> 1;
    const bool active = live && j < nl;
    extern __shared__ __attribute__((aligned(16))) u32 dyn_stage[];
    lds_u16 *stage = (lds_u16 *)dyn_stage;
    const int env_off = e * H * W;
    const int sstride = seg_stride(H, W);
    lds_u16 *sb = stage + env_off, *sg = sb + sstride, *ss = sg + sstride;

    // the column pair this lane holds: its own, or (DPPN) the copy a rotation needs
    const int js = j < nl ? j : (DPPN ? (j == 15 ? nl - 1 : (j == nl ? 0 : -1)) : -1);
    const bool holds = live && js >= 0;
    GeoSeg<MODE, DPPN> geo;
    geo.lane = lane;
    geo.j = j;
    geo.H = H;
    geo.W = W;
    geo.nl = nl;
    geo.mh = H == 32 ? ~0u : ((1u << H) - 1u);
    geo.src_l = (lane & ~15) + (active ? (j == 0 ? nl - 1 : j - 1) : j);
    geo.src_r = (lane & ~15) + (active ? (j + 1 == nl ? 0 : j + 1) : j);
    geo.odd_last = (W & 1) && js == nl - 1;
    geo.real = active;
    geo.src = StreamSrc{a.draws, a.n_draws, nullptr, a.draw_mask, a.draw_bits};
    geo.count = 0;
    const u32 wm0 = active ? geo.mh : 0u, wm1 = (active && !geo.odd_last) ? geo.mh : 0u;
    int64_t pos_b = 0, pos_g = 0;
    if (MODE == SPAWN_STREAM && live) {
        const Scratch w = scratch_of(ka.scratch, st.B);
        geo.src.err = w.err;
        pos_b = w.offsets[2 * b];
        pos_g = w.offsets[2 * b + 1];
    }

    dma_seg(st, b0, nenv, (lds_u32 *)dyn_stage, lane);
    const SegRecord rc = load_seg_record(st, ka.actions, live ? b : b0, live, lane);
    wait_vm();
    dma_seg_tail(st, b0, nenv, (lds_u32 *)dyn_stage, lane);
    wait_lgkm();
    u32 PB[32], PG[32];
    seg_rows(sg, H, W, holds, js, geo.odd_last, PG);

    SpawnCtx sc;
    sc.gid = a.env0 + (uint32_t)b;
    sc.step = a.step;
    sc.seed = a.seed;
    set_spawn_prob(sc, __int_as_float(rc.get(R_SPAWN)));

    // ---- goals: rule, then store the changed rows
    transpose32(PG);
    u32 cg[2];
    geo.pos = pos_g;
    rule_planes(PG, cg, geo, sc, 1u);
    cg[0] &= wm0;
    cg[1] &= wm1;
    const u32 rg = seg_or(cg[0] | cg[1]);
    u32 gcol[3][2];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        gcol[k][0] = PL(PG, 9 + k, 0) & wm0;
        gcol[k][1] = PL(PG, 9 + k, 1) & wm1;
    }
    const int64_t off = b * (int64_t)H * W;
    const int c0 = 2 * j, c1 = 2 * j + 1;
    if (__ballot(rg != 0u)) {
        transpose32(PG);
        uint16_t *gg = st.goals + off;
#pragma unroll
        for (int y = 0; y < kMaxH; y++)
            if (((rg >> y) & 1u) && active) {
                gg[y * W + c0] = (uint16_t)PG[y];
                if (!geo.odd_last) gg[y * W + c1] = (uint16_t)(PG[y] >> 16);
            }
    }
    __builtin_amdgcn_sched_barrier(0);

    // ---- the action: each segment's first lane, on its staged board (edits go
    // straight into the stage, the column-0 copy of an odd board too)
    const int go0 = rc.get(R_GO), ax0 = rc.get(R_AX), ay0 = rc.get(R_AY);
    RecEnv env{st, b, go0, ax0, ay0, rc.get(R_SCORE), rc.get(R_BASE), rc.get(R_POSS),
               __hiloint2double(rc.get(R_MP + 1), rc.get(R_MP))};
    SegFields fl;
    fl.op = rc.get(R_OLDP);
    fl.ns = rc.get(R_NSTEPS);
    fl.el = rc.get(R_EPLEN);
    fl.er = rc.get(R_EPREW);
    fl.base = env.base;
    fl.mp = env.mp;
    fl.plen = rc.get(R_PLEN);
    fl.phead = rc.get(R_PHEAD);
    fl.side = rc.get(R_SIDE);
    const int act = rc.get(R_ACT);
    const int phead = min(max(fl.phead, 0), 15);
    // the prior ring entry at the head, by a second bpermute with a per-lane field
    const int pxh = __builtin_amdgcn_ds_bpermute(rc.base + 4 * phead, (int)rc.R[R_PX >> 4]);
    const int pyh = __builtin_amdgcn_ds_bpermute(rc.base + 4 * phead, (int)rc.R[R_PY >> 4]);
    int act_reward = 0;
    u32 erow = 0;
    if (MODE == SPAWN_STREAM) {
        act_reward = live ? (int)scratch_of(ka.scratch, st.B).act[b] : 0;
    } else if (j == 0 && live) {
        OverlayT<SegCells> ov;
        ov.src.cells = sb;
        ov.n = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            ov.idx[k] = 0;
            ov.val[k] = 0;
        }
        act_reward = act_core(env, act, H, W, ka.ctp, ka.ctc, ov);
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (k < ov.n) {
                const int i = ov.idx[k];
                sb[i] = (uint16_t)ov.val[k];
                erow |= 1u << (i / W);
            }
    }
    // the post-action agent and game-over flag, and the edited rows, to the segment
    const int sl0 = (lane & ~15) * 4;
    fl.go = __builtin_amdgcn_ds_bpermute(sl0, env.go);
    fl.ax = __builtin_amdgcn_ds_bpermute(sl0, env.ax);
    fl.ay = __builtin_amdgcn_ds_bpermute(sl0, env.ay);
    act_reward = __builtin_amdgcn_ds_bpermute(sl0, act_reward);
    erow = (u32)__builtin_amdgcn_ds_bpermute(sl0, (int)erow);
    fl.px = pxh;
    fl.py = pyh;
    fl.bval = 0.0;
    if (a.bonus_period > 0 && live)
        fl.bval = a.bonus_table[bonus_dist(fl.ax, fl.ay, fl.px, fl.py, fl.plen, a.bonus_period,
                                           a.bonus_len)];
    seg_rows(sb, H, W, holds, js, geo.odd_last, PB);
    transpose32(PB);
    const u32 old9[2] = {PL(PB, 9, 0), PL(PB, 9, 1)};
    u32 cb[2];
    geo.pos = pos_b;
    rule_planes(PB, cb, geo, sc, 0u);
    __builtin_amdgcn_sched_barrier(0);

    // ---- scores over the real cells of the new board and goals
    u32 PS[32];
    seg_rows(ss, H, W, holds, js, geo.odd_last, PS);
    transpose32(PS);
#pragma unroll
    for (int p = 0; p < 16; p++) {
        PL(PB, p, 0) &= wm0;
        PL(PB, p, 1) &= wm1;
        PL(PS, p, 0) &= wm0;
        PL(PS, p, 1) &= wm1;
    }
    int pts, scr, pos, side;
    score_planes(PB, gcol, PS, &pts, &scr, &pos, &side);
    const int s1 = seg_total((pts + 192) | ((scr + 64) << 16));
    const int s2 = seg_total(pos | (side << 16));
    const int points = (s1 & 0xFFFF) - 192 * 16;
    const int score = ((s1 >> 16) & 0xFFFF) - 64 * 16;
    const int possible = s2 & 0xFFFF;
    const int side_total = (s2 >> 16) & 0xFFFF;
    __builtin_amdgcn_sched_barrier(0);

    // ---- exits coloured in the planes (update_exit_colors); the rows whose cells
    // changed -- by the rule, the action or an exit's colour -- are stored
    const bool can = can_exit_now(fl.mp, score, fl.base, possible);
    u32 ch = (cb[0] & wm0) | (cb[1] & wm1);
#pragma unroll
    for (int w = 0; w < 2; w++) {
        const u32 n9 = can ? (PL(PB, 9, w) | PL(PB, 8, w)) : (PL(PB, 9, w) & ~PL(PB, 8, w));
        ch |= (n9 ^ (PL(PB, 8, w) & (w ? old9[1] : old9[0]))) & PL(PB, 8, w) & (w ? wm1 : wm0);
        PL(PB, 9, w) = n9;
    }
    const u32 rb = seg_or(ch) | erow;
    if (__ballot(rb != 0u)) {
        transpose32(PB);
        uint16_t *gb = st.board + off;
#pragma unroll
        for (int y = 0; y < kMaxH; y++)
            if (((rb >> y) & 1u) && active) {
                gb[y * W + c0] = (uint16_t)PB[y];
                if (!geo.odd_last) gb[y * W + c1] = (uint16_t)(PB[y] >> 16);
            }
    }
    int rs = 0;
    if (j == 0 && live) {
        const SmallKArgs &k = kargs();
        rs = epilogue_core(k.st, k.a, b, fl, act_reward, points, score, possible, side_total,
                           k.reward_out, k.done_out, k.flags_out, k.ep_len_out, k.ep_rew_out)
                 ? 1 : 0;
    }
    uint64_t resets = __ballot(rs != 0);
    if (resets) {
        const SmallKArgs &k = kargs();
        if (k.pool.K > 0) {
            wait_vm();         // this step's stores to the envs have completed
            while (resets) {
                const int l = __builtin_ctzll(resets);
                resets &= resets - 1;
                small_reset(k.st, k.pool, k.ra, b0 + (l >> 4), lane);
            }
        }
    }
}

// Replay-mode count of env b (SL_RNG_STREAM), one wave, after k_env_action (one lane
// per env) has applied the actions -- state and cell edits in HBM, rewards in scratch
// act[] -- so the board staged here is the acted-on one: the eligible cells of the
// board and of the goals (scratch counts[2b], [2b+1]; sl_exclusive_scan_i64 turns them
// into each tensor's first uniform).  The work of k_env_count (sl_env.hip) on the
// bit-sliced rule; a tensor without spawners is not read.
__global__ void __launch_bounds__(64)
k_stream_prologue_small(SmallKArgs ka) {
    const sl_env_state &st = ka.st;
    const int64_t b = blockIdx.x;
    const int lane = threadIdx.x;
    const int H = st.H, W = st.W, nl = (W + 1) >> 1;
    extern __shared__ __attribute__((aligned(16))) u32 dyn_stage[];
    u32 *stage[2] = {dyn_stage, dyn_stage + H * 32};
    const bool active = lane < nl;
    const int64_t off = b * (int64_t)H * W;
    const u32 V = load_record(st, ka.actions, b, lane);
    const Scratch w = scratch_of(ka.scratch, st.B);
    // no spawner in the tensor (spawn_flags, set at reset; toggling powers can make
    // one on the board): no draws
    const int spf = rec(V, R_SPF) | (ka.ctp ? 1 : 0);
    int n[2] = {0, 0};
    if (spf & 3) {
        const uint16_t *src[2] = {st.board + off, st.goals + off};
        lds_u16 *dst[2] = {(lds_u16 *)stage[0], (lds_u16 *)stage[1]};
        stage_tensors<2>(src, dst, H * W, W, lane);
        wait_lgkm();
        SpawnCtx sc{0u, 0u, 0ull, 0.0};
#pragma unroll 1
        for (int t = 0; t < 2; t++) {
            if (!((spf >> t) & 1)) continue;
            u32 P[32];
            lds_rows((const lds_u16 *)stage[t], H, active, lane, P);
            transpose32(P);
            GeoSmall<SPAWN_COUNT> geo = small_geo<SPAWN_COUNT>(lane, H, W);
            u32 ch[2];
            rule_planes(P, ch, geo, sc, (u32)t);
            n[t] = wave_total(geo.count);
        }
    }
    if (lane == 0) {
        w.counts[2 * b] = n[0];
        w.counts[2 * b + 1] = n[1];
    }
}

}  // namespace

namespace sl {

bool small_shape(const sl_env_state &st) {
    return st.H >= 2 && st.H <= kMaxH && st.W >= 2 && st.W <= kMaxW;
}

int launch_step_small(const sl_env_state &st, const StepArgs &a, const FastExtra &fx,
                      const int32_t *actions, int ctp, int ctc, double *reward, uint8_t *done,
                      uint8_t *flags, int32_t *ep_len, int32_t *ep_rew, hipStream_t s) {
    if (!small_shape(st)) return SL_ETOOBIG;
    if (st.B > 0x7FFFFFFF) return SL_EINVAL;
    sl_level_pool pool = fx.pool;
    if (!fx.fuse_reset || pool.H != st.H || pool.W != st.W) pool.K = 0;
    const SmallKArgs ka{st, a, actions, ctp, ctc, reward, done, flags, ep_len, ep_rew, pool,
                        fx.ra, fx.scratch};
    const size_t lds = (size_t)3 * st.H * 32 * sizeof(uint32_t);
    const dim3 grid((unsigned)st.B);
    // boards up to 32 wide: four envs per wave
    const bool seg = st.W <= kSegW;
    const bool dppn = (st.W + 1) / 2 != 15;      // GeoSeg: DPP neighbours unless nl = 15
    const dim3 grid4((unsigned)((st.B + 3) / 4));
    const size_t lds4 = (size_t)3 * seg_stride(st.H, st.W) * sizeof(uint16_t);
    if (fx.stream) {
        if (stream_counts(fx)) {
            const int rca = launch_env_action(st, actions, ctp, ctc, scratch_of(fx.scratch, st.B).act, s);
            if (rca) return rca;
            hipLaunchKernelGGL(k_stream_prologue_small, grid, dim3(64),
                               (size_t)2 * st.H * 32 * sizeof(uint32_t), s, ka);
            if (hipGetLastError() != hipSuccess) return SL_EHIP;
        }
        const int rc = stream_offsets(st, fx, s);
        if (rc || !stream_steps(fx)) return rc;
        if (fx.ev_begin) (void)hipEventRecord((hipEvent_t)fx.ev_begin, s);
        if (seg && dppn)
            hipLaunchKernelGGL((k_env_step_seg4<SPAWN_STREAM, true>), grid4, dim3(64), lds4, s, ka);
        else if (seg)
            hipLaunchKernelGGL((k_env_step_seg4<SPAWN_STREAM, false>), grid4, dim3(64), lds4, s, ka);
        else
            hipLaunchKernelGGL(k_env_step_small<SPAWN_STREAM>, grid, dim3(64), lds, s, ka);
    } else {
        if (fx.ev_begin) (void)hipEventRecord((hipEvent_t)fx.ev_begin, s);
        if (seg && dppn)
            hipLaunchKernelGGL((k_env_step_seg4<SPAWN_PHILOX, true>), grid4, dim3(64), lds4, s, ka);
        else if (seg)
            hipLaunchKernelGGL((k_env_step_seg4<SPAWN_PHILOX, false>), grid4, dim3(64), lds4, s, ka);
        else
            hipLaunchKernelGGL(k_env_step_small<SPAWN_PHILOX>, grid, dim3(64), lds, s, ka);
    }
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}

}  // namespace sl
