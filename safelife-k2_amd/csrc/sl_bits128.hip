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
//    planes, and a funnel shift (v_alignbit) joins them.  Bands run in order, so a
//    band's upper halo is the previous band's last row (kept from its load) and its
//    lower halo the next band's first row (not yet written); every band sees the
//    pre-step board;
//  * points, performance score, possible score and side effects
//    (safelife_game.py:590-631, env_wrappers.py:319-342) are summed band by band;
//    the board's changed rows and the goals' changed 64-byte row sectors are stored;
//  * goals: a bit-plane mirror (sl_env_state.planes, [B][band][32 words][64 lanes])
//    holds their planes.  Goals without spawners that came through a step unchanged
//    are at a fixed point of the rule (planes_ok bit 2): the rule is skipped and only
//    their three colour planes are read, per band, for the scores;
//  * the action (execute_action / move_agent, safelife_game.py:308-393) has run
//    before this kernel: k_env_action (one lane per env, both RNG modes) leaves the
//    state and cell edits in HBM and the reward in the scratch (in replay mode
//    k_stream_prologue128 then counts the draws);
//  * exits are rewritten by the epilogue after the band stores have completed.
// Finished envs are queued and reset by a follow-up kernel (k_env_reset_list_wide,
// one 1024-thread block per env).
#include "sl_bits.h"

using namespace sl;
using namespace sl::fast;
using namespace sl::bits;

namespace {

// Measured on C5 (MI355X, round 1): the start board from the pool's bit planes,
// DMA'd into LDS at the band's start and read after the rule, beat HBM loads +
// transpose (43.9 vs 38.6 M env-steps/s) and beat gathering the planes from L2 into
// registers held across the rule (32.9 vs 37.1); prefetching the next band a band
// ahead gave nothing (the start-board loads queue behind it, vmcnt is in order).
constexpr int kMinWaves = 2;  // waves per SIMD the register budget is sized for

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
template <int MODE>
struct GeoBand {
    int lane, row0;
    HaloView hv;
    StreamSrc src;     // SPAWN_STREAM: the supplied uniforms; pos = the band's first,
    int64_t pos;       // used = how many the band consumed
    int used;
    int count;         // SPAWN_COUNT: this lane's eligible cells
    lds_u16 *slots;    // SPAWN_PHILOX: compact_draws' queue (kDrawSlots)
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
    // the 2x2 spawn block of band rows y, y + 1 (y even) of the lane's column pair
    __device__ __forceinline__ u32 block(int y) const {
        return block_of(lane, y);
    }
    __device__ __forceinline__ u32 block_of(int l, int y) const {
        return (u32)(((row0 + y) >> 1) * (N / 2) + l);
    }
    __device__ __forceinline__ void spawn(const u32 elig[2], u32 sp[2], const SpawnCtx &sc,
                                          u32 tensor) {
        if (MODE == SPAWN_PHILOX) {
            philox_spawn_compact(*this, elig, sp, sc, tensor, slots);
        } else if (MODE == SPAWN_STREAM) {
            used = stream_draws<false>(elig, sp, sc.thr, src, pos, lane);
        } else {
            count += __builtin_popcount(elig[0]) + __builtin_popcount(elig[1]);
        }
    }
};

// The start-board planes the side-effect term reads (0, 2, 7-15), from the level
// pool's bit planes when the env was reset from the pool: row y of
// band t is level row 32t + y - dy, one funnel shift of two adjacent 32-row words;
// column c is level column c - dx.  At a band's
// start one global_load_lds per plane copies the two level bands it spans (lanes
// 0-31: band q0, lanes 32-63: band q1, 128 columns each) into the wave's 11 KiB
// buffer, so the copy runs under the band's rule and holds no registers; after the
// rule each word is two LDS reads and a funnel shift.
constexpr int kPoolPlanes = 11;      // planes 0, 2, 7-15
__device__ __forceinline__ int pool_plane(int s) { return s == 0 ? 0 : (s == 1 ? 2 : s + 5); }

__device__ __forceinline__ void pool_dma128(const u32 *__restrict__ pp, int t, int dy, int lane,
                                            __attribute__((address_space(3))) u32 *buf) {
    const int r0 = (32 * t - dy) & (N - 1), q0 = r0 >> 5, q1 = (q0 + 1) & (NB - 1);
    const int qq = lane < 32 ? q0 : q1;
#pragma unroll
    for (int s = 0; s < kPoolPlanes; s++) {
        const u32 *src = pp + (pool_plane(s) * NB + qq) * N + 4 * (lane & 31);
        __builtin_amdgcn_global_load_lds((const void *)src,
                                         (__attribute__((address_space(3))) void *)(buf + s * 256),
                                         16, 0, 0);
    }
}

__device__ __forceinline__ void pool_start_lds(const __attribute__((address_space(3))) u32 *buf,
                                               int t, int dy, int c0, int c1, u32 S[32]) {
    const u32 sh = (u32)((32 * t - dy) & 31);
#pragma unroll
    for (int p = 0; p < 16; p++) {
        PL(S, p, 0) = 0u;
        PL(S, p, 1) = 0u;
    }
#pragma unroll
    for (int s = 0; s < kPoolPlanes; s++) {
        const int p = pool_plane(s);
        const __attribute__((address_space(3))) u32 *q = buf + s * 256;
        PL(S, p, 0) = __builtin_amdgcn_alignbit(q[128 + c0], q[c0], sh);
        PL(S, p, 1) = __builtin_amdgcn_alignbit(q[128 + c1], q[c1], sh);
    }
}

// all kernel arguments in one struct at kernarg offset 0: the epilogue re-reads its
// pointers where it runs (kargs128()), so they are not held in SGPRs through the bands
struct Step128KArgs {
    sl_env_state st;
    StepArgs a;
    FastExtra fx;
    const int32_t *actions;
    int ctp, ctc;
    double *reward_out;
    uint8_t *done_out, *flags_out;
    int32_t *ep_len_out, *ep_rew_out;
};

__device__ __forceinline__ const Step128KArgs &kargs128() {
    auto kp = __builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(kp));
    return *(const Step128KArgs *)kp;
}

// One env-step of env b, after the action: k_env_action has applied it -- state and cell edits in HBM, reward
// in scratch act[b] -- so this kernel holds no action code, no edit lists and no
// overlay.  MODE: SPAWN_PHILOX, or SPAWN_STREAM (each tensor's first uniform from the
// scratch offsets).
template <int MODE>
__global__ void __launch_bounds__(64, kMinWaves)
k_env_step_bits128(Step128KArgs ka) {
    const sl_env_state &st = ka.st;
    const StepArgs &a = ka.a;
    const FastExtra &fx = ka.fx;
    const int64_t b = blockIdx.x;
    const int lane = threadIdx.x;
    const int64_t off = b * (int64_t)(N * N);
    u32 *gb = reinterpret_cast<u32 *>(st.board + off) + lane;      // row r: gb[r * RS]
    u32 *gg = reinterpret_cast<u32 *>(st.goals + off) + lane;
    const u32 *gs = reinterpret_cast<const u32 *>(st.start_board + off) + lane;
    u32 *mg = st.planes + b * (int64_t)(NB * MW) + lane;            // mirror [t][q][lane]

    const u32 V = load_record(st, ka.actions, b, lane);
    __shared__ __attribute__((aligned(16))) u32 spool_[kPoolPlanes * 256];
    __attribute__((address_space(3))) u32 *spool = (__attribute__((address_space(3))) u32 *)spool_;
    __shared__ uint16_t slots_[kDrawSlots];
    lds_u16 *slots = (lds_u16 *)slots_;
    const int pok_all = rec(V, R_POK), pok = pok_all & 6;
    int gok = pok;              // the goals' planes_ok bits after this step
    const Scratch w = scratch_of(fx.scratch, st.B);
    // replay: the board's count mirror (planes 0, 4, 6, 7) is rewritten band by band
    u32 *me = (MODE == SPAWN_STREAM && st.elig_planes) ? st.elig_planes + b * 2048 + lane
                                                       : nullptr;

    SpawnCtx sc;
    sc.gid = a.env0 + (uint32_t)b;
    sc.step = a.step;
    sc.seed = a.seed;
    sc.thr = (double)__int_as_float(rec(V, R_SPAWN));
    StreamSrc ssrc{a.draws, a.n_draws, nullptr};
    int64_t pos_b = 0, pos_g = 0;
    if (MODE == SPAWN_STREAM) {
        ssrc.err = w.err;
        pos_b = w.offsets[2 * b];
        pos_g = w.offsets[2 * b + 1];
    }
    // Bands are processed in order 0..3, so the pre-step halo rows of band t are band
    // t - 1's last row (kept from its load: it is written back before band t runs),
    // and band t + 1's first row (not yet written); band 3's lower halo is row 0,
    // kept from band 0's load, and band 0's upper halo is row 127, read up front.

    // ---- goals: advanced band by band unless at a fixed point; the mirror keeps
    // their planes (all words rewritten when it was stale, else the changed ones)
    if ((pok & 6) != 6) {
        const bool all = !(pok & 2);
        u32 changed = 0, spawners = 0;
        u32 up = gg[(N - 1) * RS], row0 = 0;
#pragma unroll 1
        for (int t = 0; t < NB; t++) {
            u32 G[32];
            load_pairs_nt<RS>(gg + 32 * t * RS, G);
            const u32 dn = t < NB - 1 ? gg[(32 * t + 32) * RS] : row0;
            if (t == 0) row0 = G[0];
            const u32 last = G[31];
            transpose32(G);
            u32 cg[2];
            GeoBand<MODE> geo{lane, 32 * t, HaloView{up, t < NB - 1 ? dn : row0}, ssrc, pos_g, 0, 0, slots};
            rule_planes(G, cg, geo, sc, 1u);
            pos_g += geo.used;
            up = last;
            const u32 rg = wave_or(cg[0] | cg[1]);
            u32 *m = mg + t * MW;       // only the colour planes are ever read back
#pragma unroll
            for (int q = 0; q < 2; q++)
                if (all || cg[q])
#pragma unroll
                    for (int k = 9; k < 12; k++) m[(k + 16 * q) * 64] = PL(G, k, q);
            changed |= rg;
            spawners |= PL(G, 7, 0) | PL(G, 7, 1);
            if (rg) {
                const u32 lm = sector_rows(cg[0] | cg[1]);
                transpose32(G);
#pragma unroll
                for (int y = 0; y < 32; y++)
                    if ((rg >> y) & 1u)
                        if ((lm >> y) & 1u) __builtin_nontemporal_store(G[y], &gg[(32 * t + y) * RS]);
            }
        }
        const bool fixed = changed == 0 && __ballot(spawners != 0u) == 0ull;
        gok = 2 | (fixed ? 4 : 0);
        wait_vm();          // the mirror words are read back below
    }
    __builtin_amdgcn_sched_barrier(0);

    const int act_reward = (int)w.act[b];
    RecFields fl{V, rec(V, R_GO), rec(V, R_AX), rec(V, R_AY), 0.0};
    if (a.bonus_period > 0)        // issued now, consumed by the epilogue
        fl.bval = a.bonus_table[bonus_dist(fl.ax, fl.ay, fl.prior_x(fl.prior_head()),
                                           fl.prior_y(fl.prior_head()), fl.prior_len(),
                                           a.bonus_period, a.bonus_len)];

    // ---- board, band by band: rule, scores, changed rows back.  The start board
    // comes from the level pool's planes when the env was reset from it
    // (start_roll = (dy << 16) | dx), else from HBM (written by the caller).
    const sl_level_pool &pool = fx.pool;
    const int roll = (pool.board_planes && pool.K > 0 && pool.H == N &&
                      pool.W == N &&
                      st.start_roll) ? rec(V, R_ROLL) : -1;
    const u32 *pp = reinterpret_cast<const u32 *>(pool.board_planes) +
                    (int64_t)(roll >= 0 ? rec(V, R_LI) : 0) * (16 * NB * N);
    const int sdy = roll >> 16, sdx = roll & 0xFFFF;
    const int sc0 = (2 * lane - sdx) & (N - 1), sc1 = (sc0 + 1) & (N - 1);
    int pts = 0, scr = 0, pos = 0, side = 0;
    u32 up = gb[(N - 1) * RS], row0 = 0;
#pragma unroll 1
    for (int t = 0; t < NB; t++) {
        u32 P[32];
        load_pairs_nt<RS>(gb + 32 * t * RS, P);
        const u32 dn = t < NB - 1 ? gb[(32 * t + 32) * RS] : row0;
        if (roll >= 0) {
            wait_lgkm();        // the previous band's reads of the buffer are done
            pool_dma128(pp, t, sdy, lane, spool);
        }
        if (t == 0) row0 = P[0];
        const u32 last = P[31];
        transpose32(P);
        u32 cb[2];
        GeoBand<MODE> geo{lane, 32 * t, HaloView{up, t < NB - 1 ? dn : row0}, ssrc, pos_b, 0, 0, slots};
        rule_planes(P, cb, geo, sc, 0u);
        pos_b += geo.used;
        up = last;
        if (MODE == SPAWN_STREAM && me) {
#pragma unroll
            for (int s = 0; s < 4; s++)
#pragma unroll
                for (int q = 0; q < 2; q++)
                    __builtin_nontemporal_store(PL(P, elig_plane(s), q),
                                                &me[t * 512 + (2 * s + q) * 64]);
        }
        __builtin_amdgcn_sched_barrier(0);
        u32 gcol[3][2];
        const u32 *m = mg + t * MW;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            gcol[k][0] = m[(9 + k) * 64];
            gcol[k][1] = m[(25 + k) * 64];
        }
        int p, q, r, e;
        u32 S[32];
        if (roll < 0) {
            load_pairs<RS>(gs + 32 * t * RS, S);
            transpose32(S);
        } else {
            wait_vm();          // the band's pool planes have landed in LDS
            pool_start_lds(spool, t, sdy, sc0, sc1, S);
        }
        score_planes(P, gcol, S, &p, &q, &r, &e);
        pts += p;
        scr += q;
        pos += r;
        side += e;
        const u32 rb = wave_or(cb[0] | cb[1]);
        if (rb) {
            // only the changed rows, whole (a wave-uniform branch per row; the 64-byte
            // sector masks of the goals' stores measured 1.3% slower here, where
            // nearly every sector of a changed row changes)
            transpose32(P);
#pragma unroll
            for (int y = 0; y < 32; y++)
                if ((rb >> y) & 1u) __builtin_nontemporal_store(P[y], &gb[(32 * t + y) * RS]);
        }
    }
    const int points = wave_total(pts), score = wave_total(scr);
    const int possible = wave_total(pos), side_total = wave_total(side);
    // goals mirror bits, and bit 3 = the board count mirror is current (replay only:
    // a Philox step clears it)
    const int ok = gok | (me ? 8 : 0);
    if (ok != pok_all && lane == 0) st.planes_ok[b] = ok;
    wait_vm();              // row stores land before the epilogue rewrites the exits
    if (lane == 0) {
        const Step128KArgs &k = kargs128();
        const bool reset = epilogue_core(k.st, k.a, b, fl, act_reward, points, score, possible,
                                         side_total, k.reward_out, k.done_out, k.flags_out,
                                         k.ep_len_out, k.ep_rew_out);
        if (k.fx.fuse_reset && reset) {   // queued for k_env_reset_list_wide
            int64_t *cnt = k.fx.scratch + 8 * k.st.B + 2 + (k.a.step & 1);
            const int i = (int)atomicAdd((unsigned long long *)cnt, 1ull);
            reset_list(k.fx.scratch)[i] = (int32_t)b;
        }
    }
}

// Replay-mode count of env b (SL_RNG_STREAM), one wave, after k_env_action (one lane
// per env) has applied the actions -- state and cell edits in HBM, rewards in scratch
// act[] -- so the board read here is the acted-on one: the eligible cells of the board
// and of the goals, band by band (scratch counts[2b], [2b+1]; sl_exclusive_scan_i64
// turns them into each tensor's first uniform).  The work of k_env_count (sl_env.hip)
// on the bit-sliced rule.  The board is counted from its count mirror when that is
// current (planes_ok bit 3: the last step was a replay step and the action pre-pass
// patched its edits in): 8 KiB of planes per env instead of the 32 KiB board, and no
// transpose.
__global__ void __launch_bounds__(64)
k_stream_prologue128(Step128KArgs ka) {
    const sl_env_state &st = ka.st;
    const int64_t b = blockIdx.x;
    const int lane = threadIdx.x;
    const int64_t off = b * (int64_t)(N * N);
    const u32 *gb = reinterpret_cast<const u32 *>(st.board + off) + lane;
    const u32 *gg = reinterpret_cast<const u32 *>(st.goals + off) + lane;
    const u32 V = load_record(st, ka.actions, b, lane);
    const Scratch w = scratch_of(ka.fx.scratch, st.B);
    SpawnCtx sc{0u, 0u, 0ull, 0.0};
    const StreamSrc none{nullptr, 0, nullptr};
    // the eligible cells of one tensor, band by band
    auto count = [&](const u32 *g) {
        int n = 0;
#pragma unroll 1
        for (int t = 0; t < NB; t++) {
            const int ru = (32 * t - 1) & (N - 1), rd = (32 * t + 32) & (N - 1);
            const u32 up = g[ru * RS], dn = g[rd * RS];
            u32 P[32];
            load_pairs_nt<RS>(g + 32 * t * RS, P);
            transpose32(P);
            GeoBand<SPAWN_COUNT> geo{lane, 32 * t, HaloView{up, dn}, none, 0, 0, 0, nullptr};
            u32 ch[2];
            rule_planes(P, ch, geo, sc, 0u);
            n += geo.count;
        }
        return wave_total(n);
    };
    // the same count from the mirror's planes 0, 4, 6, 7 (the rest read as 0: they do
    // not enter eligibility); a band's outside rows are bit 31 / bit 0 of the
    // neighbouring bands' words
    auto count_mirror = [&](const u32 *me) {
        u32 M[NB][4][2];
#pragma unroll
        for (int t = 0; t < NB; t++)
#pragma unroll
            for (int s = 0; s < 4; s++)
#pragma unroll
                for (int q = 0; q < 2; q++) M[t][s][q] = me[t * 512 + (2 * s + q) * 64];
        // the rows the action pre-pass may have edited since the mirror was written
        // (scratch act[B + b], bytes 0xFF = none): re-read from the board
        const u32 rows = (u32)w.act[st.B + b];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const u32 y = (rows >> (8 * j)) & 0xFFu;
            if (y >= (u32)N) continue;                  // wave-uniform
            const u32 d = gb[y * RS], bit = 1u << (y & 31);
#pragma unroll
            for (int t = 0; t < NB; t++)
                if ((int)(y >> 5) == t)
#pragma unroll
                    for (int s = 0; s < 4; s++)
#pragma unroll
                        for (int q = 0; q < 2; q++)
                            M[t][s][q] = ((d >> (elig_plane(s) + 16 * q)) & 1u)
                                             ? (M[t][s][q] | bit) : (M[t][s][q] & ~bit);
        }
        int n = 0;
#pragma unroll
        for (int t = 0; t < NB; t++) {
            const int tu = (t + NB - 1) & (NB - 1), td = (t + 1) & (NB - 1);
            u32 P[32], up = 0u, dn = 0u;
#pragma unroll
            for (int k = 0; k < 32; k++) P[k] = 0u;
#pragma unroll
            for (int s = 0; s < 4; s++)
#pragma unroll
                for (int q = 0; q < 2; q++) {
                    const int p = elig_plane(s);
                    PL(P, p, q) = M[t][s][q];
                    up |= (M[tu][s][q] >> 31) << (p + 16 * q);
                    dn |= (M[td][s][q] & 1u) << (p + 16 * q);
                }
            GeoBand<SPAWN_COUNT> geo{lane, 32 * t, HaloView{up, dn}, none, 0, 0, 0, nullptr};
            u32 ch[2];
            rule_planes(P, ch, geo, sc, 0u);
            n += geo.count;
        }
        return wave_total(n);
    };
    // a board or goals without spawners (spawn_flags, set at reset: no rule or action
    // creates one) draws nothing; nor do goals at their fixed point (planes_ok bit 2)
    const int spf = rec(V, R_SPF) | (ka.ctp ? 1 : 0);     // toggling powers can make one
    const bool mirror = st.elig_planes && (rec(V, R_POK) & 8);
    const int nb = !(spf & 1) ? 0 : mirror ? count_mirror(st.elig_planes + b * 2048 + lane)
                                           : count(gb);
    const int ng = ((rec(V, R_POK) & 6) == 6 || !(spf & 2)) ? 0 : count(gg);
    if (lane == 0) {
        w.counts[2 * b] = nb;
        w.counts[2 * b + 1] = ng;
    }
}

}  // namespace

namespace sl {

bool bits128_shape(const sl_env_state &st) {
    return st.H == N && st.W == N && st.planes && st.planes_ok;
}

int launch_step_bits128(const sl_env_state &st, const StepArgs &a, const FastExtra &fx,
                        const int32_t *actions, int ctp, int ctc, double *reward, uint8_t *done,
                        uint8_t *flags, int32_t *ep_len, int32_t *ep_rew, hipStream_t s) {
    if (!bits128_shape(st)) return SL_ETOOBIG;
    const Step128KArgs ka{st, a, fx, actions, ctp, ctc, reward, done, flags, ep_len, ep_rew};
    const dim3 grid((unsigned)st.B);
    if (fx.stream) {
        if (stream_counts(fx)) {
            const int rca = launch_env_action(st, actions, ctp, ctc, scratch_of(fx.scratch, st.B).act, s);
            if (rca) return rca;
            hipLaunchKernelGGL(k_stream_prologue128, grid, dim3(64), 0, s, ka);
            if (hipGetLastError() != hipSuccess) return SL_EHIP;
        }
        const int rc = stream_offsets(st, fx, s);
        if (rc || !stream_steps(fx)) return rc;
        if (fx.ev_begin) (void)hipEventRecord((hipEvent_t)fx.ev_begin, s);
        hipLaunchKernelGGL(k_env_step_bits128<SPAWN_STREAM>, grid, dim3(64), 0, s, ka);
    } else {
        const int rc = launch_env_action(st, actions, ctp, ctc, scratch_of(fx.scratch, st.B).act, s);
        if (rc) return rc;
        if (fx.ev_begin) (void)hipEventRecord((hipEvent_t)fx.ev_begin, s);
        hipLaunchKernelGGL(k_env_step_bits128<SPAWN_PHILOX>, grid, dim3(64), 0, s, ka);
    }
    if (hipGetLastError() != hipSuccess) return SL_EHIP;
    if (fx.ev_end) (void)hipEventRecord((hipEvent_t)fx.ev_end, s);
    if (fx.capture) {          // the frame before this step's resets
        const int rc = launch_capture(st, *fx.capture, flags, 0, s);
        if (rc) return rc;
    }
    if (fx.fuse_reset && fx.pool.K > 0)
        return launch_reset_list_wide(st, fx.pool, fx.ra, fx.scratch, a.step, s);
    return SL_OK;
}

}  // namespace sl
