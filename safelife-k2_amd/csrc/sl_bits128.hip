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
//    state and cell edits in HBM and the reward in the scratch;
//  * replay mode (SL_RNG_STREAM, the reference's stream order) with draw planes
//    (sl_env_state.elig_planes): k_stream_prologue128 counts each tensor's eligible
//    cells -- for the board from the eligibility the last step left, patched around
//    the action's rows -- sl_exclusive_scan_i64 places them in the stream,
//    k_stream_draw128 decides every spawn, and this kernel (SPAWN_DECIDED) ANDs the
//    decisions into its spawns and leaves the advanced board's eligibility for the
//    next step's count;
//  * exits are rewritten by the epilogue after the band stores have completed.
// Finished envs are queued and reset by a follow-up kernel (k_env_reset_list_wide,
// one 1024-thread block per env).
#include "sl_bits.h"
#include "sl_env_action.h"
#include "sl_obs.h"

using namespace sl;
using namespace sl::fast;
using namespace sl::bits;

namespace {

// Measured on C5 (MI355X, round 1): the start board from the pool's bit planes,
// DMA'd into LDS at the band's start and read after the rule, beat HBM loads +
// transpose (43.9 vs 38.6 M env-steps/s) and beat gathering the planes from L2 into
// registers held across the rule (32.9 vs 37.1); prefetching the next band a band
// ahead gave nothing (the start-board loads queue behind it, vmcnt is in order).
// waves per SIMD the register budget is sized for: 4 (<= 128 VGPRs, with 10 KiB of LDS
// per wave) for the Philox and decided-replay forms; the stream form (replay without
// draw planes, a fallback) keeps its in-kernel ranks and stream loads at 3
constexpr int kMinWaves = 4;
constexpr int kMinWavesStream = 3;

constexpr int N = 128;       // rows = columns
constexpr int RS = N / 2;    // dwords per row
constexpr int NB = N / 32;   // bands of 32 rows
constexpr int MW = 32 * 64;  // mirror dwords per band (32 words x 64 lanes)

// A per-lane view of a per-env array (element i of lane l at base[i + l]): the base
// stays wave-uniform (SGPRs) and each access adds a 32-bit lane offset (lane_now), so
// the kernel holds no per-lane pointers through its bands.
template <class T>
struct LanePtr {
    T *base;
    __device__ __forceinline__ T &operator[](int i) const { return base[(uint32_t)(i + lane_now())]; }
    __device__ __forceinline__ T *operator+(int i) const { return base + (uint32_t)(i + lane_now()); }
};

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
    u32 e[2];          // SPAWN_COUNT: the band's eligible cells; SPAWN_DECIDED: the
                       // cells k_stream_draw128 decided spawn
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
        } else if (MODE == SPAWN_DECIDED) {
            sp[0] = elig[0] & e[0];
            sp[1] = elig[1] & e[1];
        } else {
            count += __builtin_popcount(elig[0]) + __builtin_popcount(elig[1]);
            e[0] = elig[0];
            e[1] = elig[1];
        }
    }
};

// The start-board planes the side-effect term reads (0, 2, 7-11, 15; 12-14 below),
// from the level pool's bit planes when the env was reset from the pool: row y of
// band t is level row 32t + y - dy, one funnel shift of two adjacent 32-row words;
// column c is level column c - dx.  At a band's
// start one global_load_lds per plane copies the two level bands it spans (lanes
// 0-31: band q0, lanes 32-63: band q1, 128 columns each) into the wave's 8 KiB
// buffer, so the copy runs under the band's rule and holds no registers; after the
// rule each word is two LDS reads and a funnel shift.  A start board written by the
// caller (start_roll = -1) is loaded from HBM at the band's start and its planes are
// put into the same buffer (as an unrolled level: dy = dx = 0).
// Cell bits 12-14 are used by no cell type, so the spool leaves their planes out
// (8 KiB + 2 KiB of draw slots: 4 waves/SIMD).  The side-effect term then compares the
// board's planes 12-14 against 0; an env whose start board may carry those bits
// (spawn_flags bit 2, set where a start board is written: the resets, from the level;
// the host, for boards it loads) gets the exact term from a second pass over the band
// (side_hi_fix).
constexpr int kPoolPlanes = 8;       // planes 0, 2, 7-11, 15
__device__ __forceinline__ int pool_plane(int s) {
    return s == 0 ? 0 : (s == 1 ? 2 : (s < 7 ? s + 5 : 15));
}

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

// a start band loaded by the caller's rows (start_roll = -1) into the spool, in
// pool_start_lds' layout with dy = dx = 0 (word w of lane j at column 2j + w)
__device__ __forceinline__ void start_band_lds(const u32 *__restrict__ src, int lane,
                                               __attribute__((address_space(3))) u32 *buf) {
    u32 S[32];
    load_pairs<RS>(src, S);
    transpose32(S);
#pragma unroll
    for (int s = 0; s < kPoolPlanes; s++) {
        buf[s * 256 + 2 * lane] = PL(S, pool_plane(s), 0);
        buf[s * 256 + 2 * lane + 1] = PL(S, pool_plane(s), 1);
    }
}

// The band's side-effect count with the start board's planes 12-14 taken into account
// (score_planes counted them as 0): B the band's advanced planes, S its start planes
// as read from the spool (12-14 zero), src the start band's rows in HBM.  Returns the
// correction to add.  Only for envs whose start board may use cell bits 12-14.
__device__ __forceinline__ int side_hi_fix(const u32 B[32], const u32 gc[3][2], u32 S[32],
                                           const u32 *__restrict__ src) {
    int e0, e1, x;
    score_planes(B, gc, S, &x, &x, &x, &e0);
    u32 h[3][2] = {{0u, 0u}, {0u, 0u}, {0u, 0u}};
#pragma unroll 1
    for (int y = 0; y < 32; y++) {
        const u32 d = src[y * RS];
#pragma unroll
        for (int k = 0; k < 3; k++) {
            h[k][0] |= ((d >> (12 + k)) & 1u) << y;
            h[k][1] |= ((d >> (28 + k)) & 1u) << y;
        }
    }
#pragma unroll
    for (int k = 0; k < 3; k++) {
        PL(S, 12 + k, 0) = h[k][0];
        PL(S, 12 + k, 1) = h[k][1];
    }
    score_planes(B, gc, S, &x, &x, &x, &e1);
    return e1 - e0;
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

// The goal planes the mirror holds in full for goals of the usual cell types (alive,
// destructible, frozen, colours: cell bits 0x0E19, no spawner); the colour planes 9-11
// are kept for every env.
constexpr int kGoalPlanes = 6;
__device__ __forceinline__ int goal_plane(int i) { return i < 3 ? (i == 0 ? 0 : i + 2) : i + 6; }

// the decided spawns of band t of a tensor (0 board, 1 goals) for the step kernel's
// rule: loaded at the band's start, under its row loads; none when the tensor draws
// nothing this step (`draws` false)
template <class G, class M>
__device__ __forceinline__ void draw_planes(G &geo, const M &me, int tensor, int t, bool draws) {
    geo.e[0] = geo.e[1] = 0u;
    if (draws) {
        const u32 *d = me + (kDrawPlanes + (tensor * NB + t) * 128);
        geo.e[0] = d[0];
        geo.e[1] = d[64];
    }
}

// Row y of eligibility planes pl (planes 0, 4, 6, 7 x 2 words, elig_plane) as a row
// dword (bit p + 16 w = plane p of column 2 lane + w), the form HaloView takes.
__device__ __forceinline__ u32 pack_row(const u32 pl[8], int y) {
    u32 d = 0u;
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
        for (int q = 0; q < 2; q++) d |= ((pl[2 * s + q] >> y) & 1u) << (elig_plane(s) + 16 * q);
    return d;
}

// The eligible cells of band t of the advanced board -- the next step's spawn
// eligibility before its action -- from the band's planes 0, 4, 6, 7 and the
// neighbouring rows up / dn (row dwords); the rest of the rule folds away.  Stored as
// the board's draw planes, which k_stream_prologue128 patches and counts.
template <class M>
__device__ __forceinline__ void next_elig(const u32 pl[8], u32 up, u32 dn, int t, int lane,
                                          const M &me, uint16_t *cnt) {
    u32 P[32];
#pragma unroll
    for (int k = 0; k < 32; k++) P[k] = 0u;
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
        for (int q = 0; q < 2; q++) PL(P, elig_plane(s), q) = pl[2 * s + q];
    const StreamSrc none{nullptr, 0, nullptr};
    const SpawnCtx sc{0u, 0u, 0ull, 0.0};
    GeoBand<SPAWN_COUNT> geo{lane, 32 * t, HaloView{up, dn}, none, 0, 0, 0, nullptr};
    u32 ch[2];
    rule_planes(P, ch, geo, sc, 0u);
    __builtin_nontemporal_store(geo.e[0], &me[kDrawPlanes + t * 128]);
    __builtin_nontemporal_store(geo.e[1], &me[kDrawPlanes + t * 128 + 64]);
    const int n = wave_total(__builtin_popcount(geo.e[0]) + __builtin_popcount(geo.e[1]));
    if (lane == 0) cnt[t] = (uint16_t)n;       // the band's count (<= 4096)
}

// The goals' colour planes (9-11) of band t: from the rolled pool level's goal planes
// while the goals are still the level's (gp: two level words and a funnel shift), else
// from the env's mirror (mg)
template <class M>
__device__ __forceinline__ void band_gcol(const u32 *gp, const M &mg, int t, int sdy, int sdx,
                                          u32 gcol[3][2]) {
    if (gp) {
        const int r0 = (32 * t - sdy) & (N - 1), q0 = r0 >> 5, q1 = (q0 + 1) & (NB - 1);
        const u32 sh = (u32)(r0 & 31);
        const int c0 = (2 * lane_now() - sdx) & (N - 1), c1 = (c0 + 1) & (N - 1);
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const u32 *g0 = gp + (k * NB + q0) * N, *g1 = gp + (k * NB + q1) * N;
            gcol[k][0] = __builtin_amdgcn_alignbit(g1[c0], g0[c0], sh);
            gcol[k][1] = __builtin_amdgcn_alignbit(g1[c1], g0[c1], sh);
        }
    } else {
        const u32 *m = mg + t * MW;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            gcol[k][0] = m[(9 + k) * 64];
            gcol[k][1] = m[(25 + k) * 64];
        }
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

// ---- packed views from the planes (plane mode with obs_out; SafeLifeEnv.get_obs,
// safelife_env.py:125-155, recenter_view, helper_utils.py:41-74).  A view cell is
// board + ((goals & COLORS) << 3), white goals removed; the view is centred on the
// agent with torus wrap.  The board never leaves the planes for it: after band t has
// advanced and been stored, the band's view-form planes (the goal colour planes added
// into board planes 12-15 by a bit-sliced 3-bit adder: exact for any board bits) are
// transposed once and staged as rows in the start-plane spool (free until the next
// band's DMA), and the view rows that fall in the band are stored from there, lane i
// taking the flat view cells i, i + 64, ... (coalesced).  A view of at most 96 rows
// (kViewMaxRows128) meets each band in one run of view rows.  Exits are rewritten after the epilogue
// (view_exits), where their colour is decided.

__device__ __forceinline__ void view_band(u32 P[32], const u32 gcol[3][2], int t, int agy,
                                          int agx, __attribute__((address_space(3))) u32 *spool,
                                          int64_t b) {
    const Step128KArgs &k = kargs128();
    const int vh = k.fx.obs_vh, vw = k.fx.obs_vw;
    const int ty = agy - vh / 2, tx = agx - vw / 2;
    const int s = (32 * t - ty) & (N - 1);           // view row of the band's row 0
    int va = 0, vb = 0;
    if (s < vh) {
        va = s;
        vb = min(s + 32, vh);
    } else if (s + 32 > N) {
        vb = min(s + 32 - N, vh);
    }
    if (va >= vb) return;                            // (wave-uniform)
    const bool rw = k.fx.obs_rw != 0;
#pragma unroll
    for (int w = 0; w < 2; w++) {
        u32 g0 = gcol[0][w], g1 = gcol[1][w], g2 = gcol[2][w];
        if (rw) {                                    // white goals are background
            const u32 wh = g0 & g1 & g2;
            g0 &= ~wh;
            g1 &= ~wh;
            g2 &= ~wh;
        }
        const u32 b12 = PL(P, 12, w), b13 = PL(P, 13, w), b14 = PL(P, 14, w);
        u32 c = b12 & g0;
        PL(P, 12, w) = b12 ^ g0;
        const u32 x13 = b13 ^ g1;
        PL(P, 13, w) = x13 ^ c;
        c = (b13 & g1) | (c & x13);
        const u32 x14 = b14 ^ g2;
        PL(P, 14, w) = x14 ^ c;
        c = (b14 & g2) | (c & x14);
        PL(P, 15, w) ^= c;                           // (the carry out of bit 15 drops)
    }
    transpose32(P);
    const int lane = lane_now();
#pragma unroll
    for (int y = 0; y < 32; y++) spool[y * 64 + lane] = P[y];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const lds_u16 *cells = (const lds_u16 *)spool;
    uint16_t *o = k.fx.obs_out + b * (int64_t)(vh * vw);
    const int i_end = vb * vw, dr = 64 / vw, dc = 64 - dr * vw;
    int i = va * vw + lane;
    int r = i / vw, c = i - r * vw;
#pragma unroll 4
    for (; i < i_end; i += 64) {
        const int row = (ty + r - 32 * t) & (N - 1), col = (tx + c) & (N - 1);
        __builtin_nontemporal_store((uint16_t)cells[row * N + col], &o[i]);
        r += dr;
        c += dc;
        if (c >= vw) {
            c -= vw;
            r++;
        }
    }
}

// The exits of the view (recenter_view's move_to_perimeter): every exit cell goes to
// its clipped position, the last exit in np.nonzero order winning a shared one.  An
// exit's value is the epilogue's (LEVEL_EXIT, red when the level can be exited: exits
// are frozen and never change otherwise) plus its goal colour.  The targets and the goal
// cells are loaded before the epilogue (in flight with its loads); the goal cell past
// the vector L1 (this wave stored the goals' changed rows, and waited for them).
struct ViewExit {
    int tgt;            // this lane's exit's view cell (-1: no exit, or a later one wins)
    u32 goal;           // its goal cell
};
__device__ __forceinline__ ViewExit view_exits_load(const sl_env_state &st, int64_t b, int agy,
                                                    int agx) {
    const Step128KArgs &k = kargs128();
    const int vh = k.fx.obs_vh, vw = k.fx.obs_vw;
    const int ne = min(__builtin_amdgcn_readfirstlane(st.exit_count[b]), SL_MAX_EXITS);
    const int lane = lane_now();
    ViewExit ve{-1, 0u};
    if (lane < ne) {
        const int iy = st.exit_y[b * SL_MAX_EXITS + lane], ix = st.exit_x[b * SL_MAX_EXITS + lane];
        int jy = pymod(iy - agy + N / 2, N) - N / 2;
        int jx = pymod(ix - agx + N / 2, N) - N / 2;
        jy = min(max(jy + vh / 2, 0), vh - 1);
        jx = min(max(jx + vw / 2, 0), vw - 1);
        ve.tgt = jy * vw + jx;
        const int ci = iy * N + ix;
        const u32 *gw = reinterpret_cast<const u32 *>(st.goals + b * (int64_t)(N * N)) + (ci >> 1);
        ve.goal = __hip_atomic_load(gw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> (16 * (ci & 1));
    }
    for (int j = 1; j < ne; j++) {        // a later exit on the same cell wins
        const int tj = __builtin_amdgcn_readlane(ve.tgt, j);
        if (j > lane && tj == ve.tgt) ve.tgt = -1;
    }
    return ve;
}
__device__ __forceinline__ void view_exits_store(const ViewExit &ve, int64_t b, int can) {
    const Step128KArgs &k = kargs128();
    if (ve.tgt < 0) return;
    const u32 ev = LEVEL_EXIT | (can ? COLOR_R : 0u);
    k.fx.obs_out[b * (int64_t)(k.fx.obs_vh * k.fx.obs_vw) + ve.tgt] =
        obs::obs_value(ev, ve.goal & 0xFFFFu, k.fx.obs_rw);
}

// One env-step of env b, after the action: k_env_action has applied it -- state and cell edits in HBM, reward
// in scratch act[b] -- so this kernel holds no action code, no edit lists and no
// overlay.  MODE: SPAWN_PHILOX; SPAWN_STREAM (each tensor's first uniform from the
// scratch offsets); or SPAWN_DECIDED (the spawns from the draw planes k_stream_draw128
// left, replay with sl_env_state.elig_planes).
// KEEP: the board planes any board of the batch can hold (sl_env_state.board_zero's
// complement, or a superset of it): the others are neither loaded nor stored in plane
// mode.  Instantiated for every plane and for the C5 levels' (cell bits 0, 1, 3-10:
// 10 of 16 planes, 37 % fewer plane bytes)
constexpr u32 kKeep128All = 0xFFFFu, kKeep128C5 = 0x07FBu;

template <int MODE, bool VIEW, u32 KEEP>
__device__ __forceinline__ void step128_body(const Step128KArgs &ka) {
    const sl_env_state &st = ka.st;
    const StepArgs &a = ka.a;
    const FastExtra &fx = ka.fx;
    const int64_t b = blockIdx.x;
    const int lane = threadIdx.x;
    const int64_t off = b * (int64_t)(N * N);
    const LanePtr<u32> gb{reinterpret_cast<u32 *>(st.board + off)};   // row r: gb[r * RS]
    const LanePtr<u32> gg{reinterpret_cast<u32 *>(st.goals + off)};
    const LanePtr<const u32> gs{reinterpret_cast<const u32 *>(st.start_board + off)};
    const LanePtr<u32> mg{st.planes + b * (int64_t)(NB * MW)};       // mirror [t][q][lane]

    const u32 V = load_record(st, ka.actions, b, lane);
    __shared__ __attribute__((aligned(16))) u32 spool_[kPoolPlanes * 256];
    __attribute__((address_space(3))) u32 *spool = (__attribute__((address_space(3))) u32 *)spool_;
    __shared__ uint16_t slots_[kDrawSlots];
    lds_u16 *slots = (lds_u16 *)slots_;
    const int pok_all = rec(V, R_POK), pok = pok_all & 6;
    int gok = pok_all & (6 | 16 | 32);   // the goals' planes_ok bits after this step
    const Scratch w = scratch_of(fx.scratch, st.B);
    // replay with draw planes: the spawns come decided from them (k_stream_draw128), for
    // the tensors that draw (scratch act[B + b] bit 0 board, bit 1 goals), and the
    // advanced board's eligible cells go back into the board's planes
    const LanePtr<u32> me{MODE == SPAWN_DECIDED ? st.elig_planes + b * kEligStride : nullptr};
    const int dfl = MODE == SPAWN_DECIDED ? (int)w.act[st.B + b] : 0;

    SpawnCtx sc;
    sc.gid = a.env0 + (uint32_t)b;
    sc.step = a.step;
    sc.seed = a.seed;
    set_spawn_prob(sc, __int_as_float(rec(V, R_SPAWN)));
    StreamSrc ssrc{a.draws, a.n_draws, nullptr, a.draw_mask, a.draw_bits};
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
    // their colour planes (all words rewritten when it was stale, else the changed
    // ones).  Goals whose cells use only planes 0, 3, 4 and 9-11 and hold no spawner
    // (spawn_flags bits 1 and 3 clear: the rule then creates no other bit) keep those
    // six planes there (planes_ok bit 4) and are read back from them -- 12 of the
    // 32 KiB of their cells, no transposes -- with the halo rows from the cells
    const int spf = rec(V, R_SPF);
    if ((pok & 6) != 6) {
        const bool all = !(pok & 2);
        const bool gplanes = (spf & (2 | 8)) == 0;
        const bool from_mirror = gplanes && (pok_all & 16) && (pok & 2);
        u32 changed = 0, spawners = 0;
        u32 up = gg[(N - 1) * RS], row0 = from_mirror ? gg[0] : 0u;
#pragma unroll 1
        for (int t = 0; t < NB; t++) {
            u32 G[32];
            u32 dn, last;
            if (from_mirror) {
                const u32 *m = mg + t * MW;
#pragma unroll
                for (int k = 0; k < 32; k++) G[k] = 0u;
#pragma unroll
                for (int q = 0; q < 2; q++)
#pragma unroll
                    for (int i = 0; i < kGoalPlanes; i++)
                        PL(G, goal_plane(i), q) = m[(goal_plane(i) + 16 * q) * 64];
                dn = t < NB - 1 ? gg[(32 * t + 32) * RS] : row0;
                last = gg[(32 * t + 31) * RS];
            } else {
                load_pairs_nt<RS>(gg + 32 * t * RS, G);
                dn = t < NB - 1 ? gg[(32 * t + 32) * RS] : row0;
                if (t == 0) row0 = G[0];
                last = G[31];
                transpose32(G);
            }
            u32 cg[2];
            GeoBand<MODE> geo{lane_now(), 32 * t, HaloView{up, t < NB - 1 ? dn : row0}, ssrc, pos_g, 0, 0, slots};
            if (MODE == SPAWN_DECIDED) draw_planes(geo, me, 1, t, dfl & 2);
            rule_planes(G, cg, geo, sc, 1u);
            pos_g += geo.used;
            up = last;
            const u32 rg = wave_or(cg[0] | cg[1]);
            u32 *m = mg + t * MW;
#pragma unroll
            for (int q = 0; q < 2; q++)
                if (all || (!from_mirror && gplanes) || cg[q]) {
                    if (gplanes) {
#pragma unroll
                        for (int i = 0; i < kGoalPlanes; i++)
                            m[(goal_plane(i) + 16 * q) * 64] = PL(G, goal_plane(i), q);
                    } else {
#pragma unroll
                        for (int k = 9; k < 12; k++) m[(k + 16 * q) * 64] = PL(G, k, q);
                    }
                }
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
        gok = 2 | (fixed ? 4 : 0) | (gplanes ? 16 : 0) | (changed == 0 ? pok_all & 32 : 0);
        wait_vm();          // the mirror words are read back below
    }
    __builtin_amdgcn_sched_barrier(0);


    // ---- board, band by band: rule, scores, changed rows back.  The start board
    // comes from the level pool's planes when the env was reset from it
    // (start_roll = (dy << 16) | dx), else from HBM (written by the caller).
    const sl_level_pool &pool = fx.pool;
    const int roll = (pool.board_planes && pool.K > 0 && pool.H == N &&
                      pool.W == N &&
                      st.start_roll) ? rec(V, R_ROLL) : -1;
    const u32 *pp = reinterpret_cast<const u32 *>(pool.board_planes) +
                    (int64_t)(roll >= 0 ? rec(V, R_LI) : 0) * (16 * NB * N);
    const int sdy = roll < 0 ? 0 : roll >> 16, sdx = roll < 0 ? 0 : roll & 0xFFFF;
    const bool start_hi = (rec(V, R_SPF) & 4) != 0;     // start board may use bits 12-14
    // goals still the level's (planes_ok bit 5, after this step's goals): their colour
    // planes from the pool (cache-resident) instead of the mirror (HBM)
    const u32 *gp = (roll >= 0 && (gok & 32) && pool.goal_planes)
                        ? pool.goal_planes + (int64_t)rec(V, R_LI) * (3 * NB * N) : nullptr;
    int pts = 0, scr = 0, pos = 0, side = 0;
    // plane mode (fx.plane_mode, Philox only): the board lives in st.board_planes, in
    // the mirror's layout; pin = this env's planes hold it (planes_ok bit 6; else this
    // step reads the uint16 board and writes every plane word).  Of the uint16 board
    // only the band-edge rows 32t and 32t + 31 are kept, for the halos
    const bool pmode = (MODE == SPAWN_PHILOX || MODE == SPAWN_DECIDED) && fx.plane_mode;
    const bool pin = pmode && (pok_all & 64);
    // planes_ok bit 8: the board's planes 12-14 are zero (no cell type uses those bits;
    // the rule and the actions never set them), so they are neither loaded nor stored.
    // Decided replay only: in the Philox form the selects cost more than the 6 KiB they
    // save (70.2 vs 72.9 M env-steps/s, +4 % for replay; profiles/r05am_ab_zero_planes.txt)
    const bool lo12 = MODE == SPAWN_DECIDED && pin && (pok_all & 256);
    u32 hi12 = 0u;              // a step into plane mode: any of them set
    const LanePtr<u32> bpl{pmode ? st.board_planes + b * (int64_t)(NB * MW) : nullptr};
    // ... and the cells round the agent the next step's action reads
    // (k_env_action_planes128: row agent_y, column agent_x in rows agent_y +- 1, 2)
    const int agy = __builtin_amdgcn_readfirstlane(rec(V, R_AY));
    const int agx = __builtin_amdgcn_readfirstlane(rec(V, R_AX));
    // the cells this step's action edited in the uint16 board (k_env_action_planes128)
    // (replay: the count prologue has put them into the planes already)
    const uint64_t ecells = (MODE == SPAWN_PHILOX && pin) ? (uint64_t)w.act[st.B + b] : ~0ull;
    const uint64_t evals = (MODE == SPAWN_PHILOX && pin) ? (uint64_t)w.act[2 * st.B + b] : 0ull;
    u32 up = gb[(N - 1) * RS], row0 = pin ? gb[0] : 0u;
    // SPAWN_DECIDED: the eligibility planes of the previous band (of band 0 in LDS, in
    // the draw slots this mode does not use), the advanced row 31 of the band before
    // that and row 0 of band 1: band t - 1's next eligibility is evaluated once band t
    // has advanced, bands 3 and 0 after the loop
    __attribute__((address_space(3))) u32 *e0 = (__attribute__((address_space(3))) u32 *)slots_;
    u32 EP[8], r31 = 0u, d1 = 0u;
    // and their count per band, for the next step's count (scratch act[2B + b], four
    // 16-bit band counts)
    uint16_t *ne_cnt = MODE == SPAWN_DECIDED ? reinterpret_cast<uint16_t *>(w.act + 2 * st.B + b)
                                             : nullptr;
#pragma unroll 1
    for (int t = 0; t < NB; t++) {
        u32 P[32];
        u32 last;
        bool patched = false;   // the action edited a cell of this band
        u32 pk = 0u;            // plane words the action's edits changed (this lane)
        if (pin) {
#pragma unroll
            for (int k = 0; k < 32; k++) {
                const int pl = k & 15;
                P[k] = ((lo12 && pl >= 12 && pl <= 14) || !((KEEP >> pl) & 1u))
                           ? 0u : __builtin_nontemporal_load(&bpl[t * MW + k * 64]);
            }
            last = gb[(32 * t + 31) * RS];     // (this band's edge store comes after)
        } else {
            load_pairs_nt<RS>(gb + 32 * t * RS, P);
        }
        const u32 dn = t < NB - 1 ? gb[(32 * t + 32) * RS] : row0;
        wait_lgkm();            // the previous band's reads of the buffer are done
        if (roll >= 0) pool_dma128(pp, t, sdy, lane_now(), spool);
        else start_band_lds(gs + 32 * t * RS, lane_now(), spool);
        if (!pin) {
            if (t == 0) row0 = P[0];
            last = P[31];
            transpose32(P);
        } else {
            // the action's edits: those cells' values from the uint16 board, into the
            // plane words of the lane holding each
#pragma unroll 1
            for (int m = 0; m < 4; m++) {
                const int i = (int)((ecells >> (16 * m)) & 0xFFFFu);
                if (i >= N * N || (i >> 12) != t) continue;
                const int x = i & (N - 1);
                const u32 d = (u32)(evals >> (16 * m)) & 0xFFFFu;      // the changed bits
                const u32 yr = (u32)((i >> 7) & 31);
                const bool mine = lane_now() == (x >> 1);
                patched = true;
                const u32 m2 = mine ? 1u << yr : 0u;
                // branch-free (uniform per-plane branches here cost 50 us per launch)
                const u32 m0 = (x & 1) ? 0u : m2, m1 = (x & 1) ? m2 : 0u;
                pk |= mine ? d << (16 * (x & 1)) : 0u;
#pragma unroll
                for (int p = 0; p < 16; p++) {
                    const u32 f = 0u - ((d >> p) & 1u);
                    PL(P, p, 0) ^= m0 & f;
                    PL(P, p, 1) ^= m1 & f;
                }
            }
        }
        // planes a birth or death clears but never sets: whether any changed cell
        // held one (their words are then stored too)
        u32 oth[2] = {0u, 0u};
        if (pin) {
#pragma unroll
            for (int w = 0; w < 2; w++) {
                u32 o = PL(P, 1, w) | PL(P, 2, w);
#pragma unroll
                for (int k = 4; k <= 8; k++) o |= PL(P, k, w);
#pragma unroll
                for (int k = 12; k <= 15; k++) o |= PL(P, k, w);
                oth[w] = o;
            }
        }
        u32 cb[2];
        GeoBand<MODE> geo{lane_now(), 32 * t, HaloView{up, t < NB - 1 ? dn : row0}, ssrc, pos_b, 0, 0, slots};
        if (MODE == SPAWN_DECIDED) draw_planes(geo, me, 0, t, dfl & 1);
        rule_planes(P, cb, geo, sc, 0u);
        pos_b += geo.used;
        up = last;
        if (MODE == SPAWN_DECIDED) {
            u32 EC[8];
#pragma unroll
            for (int s = 0; s < 4; s++)
#pragma unroll
                for (int q = 0; q < 2; q++) EC[2 * s + q] = PL(P, elig_plane(s), q);
            if (t >= 2) next_elig(EP, r31, pack_row(EC, 0), t - 1, lane_now(), me, ne_cnt);
            if (t == 1) d1 = pack_row(EC, 0);
            if (t >= 1) r31 = pack_row(EP, 31);
#pragma unroll
            for (int k = 0; k < 8; k++) {
                if (t == 0) e0[k * 64 + lane_now()] = EC[k];
                EP[k] = EC[k];
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        u32 gcol[3][2];
        band_gcol(gp, mg, t, sdy, sdx, gcol);
        int p, q, r, e;
        u32 S[32];
        wait_vm();              // the band's start planes have landed in LDS
        {
            const int sc0 = (2 * lane_now() - sdx) & (N - 1), sc1 = (sc0 + 1) & (N - 1);
            pool_start_lds(spool, t, sdy, sc0, sc1, S);
        }
        score_planes(P, gcol, S, &p, &q, &r, &e);
        if (start_hi) e += side_hi_fix(P, gcol, S, gs + 32 * t * RS);
        if (VIEW) {     // wave-uniform sums (SGPRs): four VGPRs fewer through the bands
            pts += wave_total(p);
            scr += wave_total(q);
            pos += wave_total(r);
            side += wave_total(e);
        } else {
            pts += p;
            scr += q;
            pos += r;
            side += e;
        }
        const u32 rb = wave_or(cb[0] | cb[1]);
        if (pin) {
            // the plane words a change can alter: alive, destructible and colours
            // (births set them, deaths clear them); the others only when a changed
            // cell held one of them.  Then the band's edge rows, packed from the planes
            if (rb) {
#pragma unroll
                for (int w = 0; w < 2; w++) {
                    __builtin_nontemporal_store(PL(P, 0, w), &bpl[t * MW + (0 + 16 * w) * 64]);
                    if ((KEEP >> 3) & 1u)
                        __builtin_nontemporal_store(PL(P, 3, w), &bpl[t * MW + (3 + 16 * w) * 64]);
#pragma unroll
                    for (int k = 9; k <= 11; k++)
                        if ((KEEP >> k) & 1u)
                            __builtin_nontemporal_store(PL(P, k, w), &bpl[t * MW + (k + 16 * w) * 64]);
                }
                if (wave_or((oth[0] & cb[0]) | (oth[1] & cb[1]))) {
#pragma unroll
                    for (int k = 0; k < 32; k++) {
                        const int pl = k & 15;
                        if (pl != 0 && pl != 3 && (pl < 9 || pl > 11) && ((KEEP >> pl) & 1u))
                            __builtin_nontemporal_store(P[k], &bpl[t * MW + k * 64]);
                    }
                }
                if (rb & 1u) {          // row 32t: bit 0 of every plane word
                    u32 r = 0u;
#pragma unroll
                    for (int k = 0; k < 32; k++) r = __builtin_amdgcn_alignbit(P[k], r, 1);
                    __builtin_nontemporal_store(r, &gb[(32 * t) * RS]);
                }
                if (rb >> 31) {         // row 32t + 31: bit 31 of every plane word
                    u32 r = 0u;
#pragma unroll
                    for (int k = 31; k >= 0; k--) r = __builtin_amdgcn_alignbit(r, P[k], 31);
                    __builtin_nontemporal_store(r, &gb[(32 * t + 31) * RS]);
                }
            }
            // the plane words the action's edits changed, in the lanes holding them
            if (patched) {
                const u32 pkw = wave_or(pk);
#pragma unroll
                for (int k = 0; k < 32; k++)
                    if (((KEEP >> (k & 15)) & 1u) && ((pkw >> k) & 1u))
                        if ((pk >> k) & 1u) bpl[t * MW + k * 64] = P[k];
            }
            // the cells the next action can read (changed or not: they may be stale
            // from steps with the agent elsewhere): row agy whole (moves left / right,
            // toggles) and column agx in rows agy +- 1, 2 (moves up / down)
            if ((agy >> 5) == t) {
                const u32 yr = (u32)(agy & 31);
                u32 r = 0u;
#pragma unroll
                for (int k = 0; k < 32; k++) r |= ((P[k] >> yr) & 1u) << k;
                __builtin_nontemporal_store(r, &gb[agy * RS]);
            }
#pragma unroll 1
            for (int d = -2; d <= 2; d++) {
                const int y = (agy + d) & (N - 1);
                if (d == 0 || (y >> 5) != t) continue;
                const u32 yr = (u32)(y & 31);
                u32 v = 0u;
                if (agx & 1) {
#pragma unroll
                    for (int p = 0; p < 16; p++) v |= ((PL(P, p, 1) >> yr) & 1u) << p;
                } else {
#pragma unroll
                    for (int p = 0; p < 16; p++) v |= ((PL(P, p, 0) >> yr) & 1u) << p;
                }
                if (lane_now() == (agx >> 1)) st.board[b * (int64_t)(N * N) + y * N + agx] = (uint16_t)v;
            }
        } else {
            if (pmode) {        // into plane mode: every plane word, and the rows below
#pragma unroll
                for (int k = 0; k < 32; k++)
                    if ((KEEP >> (k & 15)) & 1u)
                        __builtin_nontemporal_store(P[k], &bpl[t * MW + k * 64]);
                if (MODE == SPAWN_DECIDED) {
#pragma unroll
                    for (int w = 0; w < 2; w++) hi12 |= PL(P, 12, w) | PL(P, 13, w) | PL(P, 14, w);
                }
            }
            if (rb) {
                // only the changed rows, whole (a wave-uniform branch per row; the 64-byte
                // sector masks of the goals' stores measured 1.3% slower here, where
                // nearly every sector of a changed row changes)
                transpose32(P);
#pragma unroll
                for (int y = 0; y < 32; y++)
                    if ((rb >> y) & 1u) __builtin_nontemporal_store(P[y], &gb[(32 * t + y) * RS]);
                if (VIEW) transpose32(P);        // (a step into plane mode: planes again)
            }
        }
        if (VIEW) view_band(P, gcol, t, agy, agx, spool, b);
    }
    if (MODE == SPAWN_DECIDED) {
        u32 E0[8];
#pragma unroll
        for (int k = 0; k < 8; k++) E0[k] = e0[k * 64 + lane_now()];
        next_elig(EP, r31, pack_row(E0, 0), NB - 1, lane_now(), me, ne_cnt);
        next_elig(E0, pack_row(EP, 31), d1, 0, lane_now(), me, ne_cnt);
    }
    const int points = VIEW ? pts : wave_total(pts), score = VIEW ? scr : wave_total(scr);
    const int possible = VIEW ? pos : wave_total(pos);
    const int side_total = VIEW ? side : wave_total(side);
    // goals mirror bits, and bit 3 = the board's draw planes hold the advanced board's
    // eligible cells (decided replay only: any other step clears it)
    // bit 6: the planes hold the board; bit 7: so does the whole uint16 board (a step
    // into plane mode stored its changed rows as well)
    const bool z12 = MODE == SPAWN_DECIDED && (pin ? lo12 : __ballot(hi12 != 0u) == 0ull);
    const int ok = gok | (me.base ? 8 : 0) |
                   (pmode ? (pin ? 64 : 64 | 128) | (z12 ? 256 : 0) : 0);
    if (ok != pok_all && lane_now() == 0) st.planes_ok[b] = ok;
    // the epilogue's inputs, loaded now (in flight with the row stores) rather than held
    // through the bands: the reward, the bonus term and the record again (L2)
    const Step128KArgs &k = kargs128();
    const ViewExit vex = VIEW ? view_exits_load(k.st, b, agy, agx) : ViewExit{-1, 0u};
    const u32 VE = load_record(k.st, k.actions, b, lane_now());
    const int act_reward = (int)scratch_of(k.fx.scratch, k.st.B).act[b];
    RecFields fl{VE, rec(VE, R_GO), rec(VE, R_AX), rec(VE, R_AY), 0.0};
    if (k.a.bonus_period > 0)
        fl.bval = k.a.bonus_table[bonus_dist(fl.ax, fl.ay, fl.prior_x(fl.prior_head()),
                                             fl.prior_y(fl.prior_head()), fl.prior_len(),
                                             k.a.bonus_period, k.a.bonus_len)];
    wait_vm();              // row stores land before the epilogue rewrites the exits
    int can = 0;
    if (lane_now() == 0) {
        // (plane mode: the exits' colour is kept in the uint16 cells only -- no rule,
        // score or action term reads an exit's colour, and k_board_sync128 keeps them)
        const bool reset = epilogue_core(k.st, k.a, b, fl, act_reward, points, score, possible,
                                         side_total, k.reward_out, k.done_out, k.flags_out,
                                         k.ep_len_out, k.ep_rew_out, &can);
        if (k.fx.fuse_reset && reset) {   // queued for k_env_reset_list_wide
            int64_t *cnt = k.fx.scratch + 8 * k.st.B + 2 + (k.a.step & 1);
            const int i = (int)atomicAdd((unsigned long long *)cnt, 1ull);
            reset_list(k.fx.scratch)[i] = (int32_t)b;
        }
    }
    // (the view's band stores have completed: wait_vm above)
    if (VIEW) view_exits_store(vex, b, __builtin_amdgcn_readfirstlane(can));
}

// the step kernel: Philox, the stream fallback or decided replay; no views
template <int MODE, u32 KEEP>
__global__ void __launch_bounds__(64, MODE == SPAWN_STREAM ? kMinWavesStream : kMinWaves)
k_env_step_bits128(Step128KArgs ka) {
    step128_body<MODE, false, KEEP>(ka);
}

// ... with packed views written from the planes (plane mode, fx.obs_out)
template <int MODE, u32 KEEP>
__global__ void __launch_bounds__(64, kMinWaves)
k_env_step_bits128_view(Step128KArgs ka) {
    step128_body<MODE, true, KEEP>(ka);
}

// the instance for a plane-mode launch: the C5 planes when no board can hold another
template <int MODE>
void launch_step128(const Step128KArgs &ka, bool view, hipStream_t s) {
    const dim3 grid((unsigned)ka.st.B);
    const u32 keep = ~ka.st.board_zero & 0xFFFFu;
    const bool c5 = ka.fx.plane_mode && !(keep & ~kKeep128C5);
    if (view && c5)
        hipLaunchKernelGGL((k_env_step_bits128_view<MODE, kKeep128C5>), grid, dim3(64), 0, s, ka);
    else if (view)
        hipLaunchKernelGGL((k_env_step_bits128_view<MODE, kKeep128All>), grid, dim3(64), 0, s, ka);
    else if (c5)
        hipLaunchKernelGGL((k_env_step_bits128<MODE, kKeep128C5>), grid, dim3(64), 0, s, ka);
    else
        hipLaunchKernelGGL((k_env_step_bits128<MODE, kKeep128All>), grid, dim3(64), 0, s, ka);
}

// Replay-mode count of env b (SL_RNG_STREAM), one wave, after k_env_action (one lane
// per env) has applied the actions -- state and cell edits in HBM, rewards in scratch
// act[] -- so the board read here is the acted-on one: the eligible cells of the board
// and of the goals, band by band (scratch counts[2b], [2b+1]; sl_exclusive_scan_i64
// turns them into each tensor's first uniform).  The work of k_env_count (sl_env.hip)
// on the bit-sliced rule.  When the last step was a decided replay step (planes_ok
// bit 3) the board's eligible cells are already in its draw planes, bar the rows the
// action edited: 2 KiB per env and a few board rows instead of the 32 KiB board.
__device__ __forceinline__ void count_env128(const Step128KArgs &ka, int64_t b, int lane,
                                            int &nb_out, int &ng_out, int &dfl_out) {
    const sl_env_state &st = ka.st;
    const int64_t off = b * (int64_t)(N * N);
    const u32 *gb = reinterpret_cast<const u32 *>(st.board + off) + lane;
    const u32 *gg = reinterpret_cast<const u32 *>(st.goals + off) + lane;
    const u32 V = load_record(st, ka.actions, b, lane);
    const Scratch w = scratch_of(ka.fx.scratch, st.B);
    // the last step's band counts and the action's edited rows, loaded with the record
    // rather than after it (count_next's first round trip), and waited for while the
    // record is still in flight
    uint64_t nc_pre = 0;
    u32 rows_pre = 0xFFFFFFFFu;
    if (st.elig_planes) {
        nc_pre = (uint64_t)w.act[2 * st.B + b];
        rows_pre = (u32)w.act[st.B + b];
        asm volatile("" ::"s"(nc_pre), "s"(rows_pre));
    }
    SpawnCtx sc{0u, 0u, 0ull, 0.0};
    const StreamSrc none{nullptr, 0, nullptr};
    // the draw planes: each counted tensor's eligible cells, for k_stream_draw128
    u32 *dp = st.elig_planes ? st.elig_planes + b * kEligStride + kDrawPlanes + lane : nullptr;
    // plane mode (sl_env_state.board_planes, planes_ok bit 6): the board is read from
    // its planes -- only the four eligibility planes -- after the action's edits
    // (k_env_action_planes128 wrote the uint16 cells, listed in act[3B + b]) have been
    // put into them here, for this count and for the step kernel
    const bool pm = ka.fx.plane_mode && st.board_planes && (rec(V, R_POK) & 64);
    u32 *const bpw = pm ? st.board_planes + b * (int64_t)(NB * MW) : nullptr;
    const u32 zero = st.board_zero;          // planes no board holds (never stored)
    auto pload = [&](int t, int k) -> u32 {  // (past the vector L1: the edits just stored)
        if ((zero >> (k & 15)) & 1u) return 0u;
        return __hip_atomic_load(bpw + t * MW + k * 64 + lane, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
    };
    // the action's edited cells (act[3B + b], up to four 16-bit indices): lane 16 m + p
    // holds edit m's new cell value and puts its plane p into the planes (put_edits, an
    // OR or an AND of the cell's bit, nothing waited for); count_next patches its
    // window's words in registers, so the edits cost one load in flight with the others
    const uint64_t ec = pm ? (uint64_t)w.act[3 * st.B + b] : ~0ull;
    const int ei = (int)((ec >> (16 * (lane >> 4))) & 0xFFFFu);
    const u32 ev = (pm && ei < N * N) ? (u32)st.board[off + ei] : 0u;
    auto put_edits = [&]() {
        const int pl = lane & 15;
        if (!pm || ei >= N * N || ((zero >> pl) & 1u)) return;
        const int x = ei & (N - 1);
        const u32 bit = 1u << ((ei >> 7) & 31);
        u32 *wd = bpw + (ei >> 12) * MW + (pl + 16 * (x & 1)) * 64 + (x >> 1);
        if ((ev >> pl) & 1u)
            __hip_atomic_fetch_or(wd, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
            __hip_atomic_fetch_and(wd, ~bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    auto keep = [&](const GeoBand<SPAWN_COUNT> &geo, int tensor, int t) {
        if (dp) {
            dp[(tensor * NB + t) * 128] = geo.e[0];
            dp[(tensor * NB + t) * 128 + 64] = geo.e[1];
        }
    };
    // the eligible cells of one tensor, band by band
    auto count = [&](const u32 *g, int tensor) {
        int n = 0;
#pragma unroll 1
        for (int t = 0; t < NB; t++) {
            const int ru = (32 * t - 1) & (N - 1), rd = (32 * t + 32) & (N - 1);
            const u32 up = g[ru * RS], dn = g[rd * RS];      // (band-edge rows: whole)
            u32 P[32];
            if (pm && tensor == 0) {
#pragma unroll
                for (int k = 0; k < 32; k++) {
                    const int pl = k & 15;
                    P[k] = (pl == 0 || pl == 4 || pl == 6 || pl == 7) ? pload(t, k) : 0u;
                }
            } else {
                load_pairs_nt<RS>(g + 32 * t * RS, P);
                transpose32(P);
            }
            GeoBand<SPAWN_COUNT> geo{lane, 32 * t, HaloView{up, dn}, none, 0, 0, 0, nullptr};
            u32 ch[2];
            rule_planes(P, ch, geo, sc, 0u);
            n += geo.count;
            keep(geo, tensor, t);
        }
        return wave_total(n);
    };
    // the same count from the eligible cells the last (replay) step left in the board's
    // draw planes, with the rows the action pre-pass may have edited (scratch
    // act[B + b], bytes 0xFF = none; all within rows agent - 1 .. agent + 2) and their
    // neighbours re-evaluated: the board rows around them are loaded into one 32-row
    // window, the edited rows at 2..29 of it, and the window's eligibility replaces
    // rows y - 1 .. y + 1 of each edited row y.  Returns -1 when the edited rows do not
    // fit one window (the full count then runs).
    auto count_next = [&]() -> int {
        // their count, as the step left it (scratch act[2B + b]: four 16-bit band counts)
        const uint64_t nc = nc_pre;
        const int n0 = (int)((nc & 0xFFFFu) + ((nc >> 16) & 0xFFFFu) + ((nc >> 32) & 0xFFFFu) +
                             (nc >> 48));
        const u32 rows = rows_pre;
        int y0 = -1, dmin = 0, dmax = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int y = (int)((rows >> (8 * j)) & 0xFFu);
            if (y >= N) continue;                       // wave-uniform
            if (y0 < 0) y0 = y;
            const int d = ((y - y0 + N / 2) & (N - 1)) - N / 2;
            dmin = min(dmin, d);
            dmax = max(dmax, d);
        }
        if (y0 < 0) return n0;                          // nothing edited: as the step left it
        if (dmax - dmin > 27) return -1;
        const int base = (y0 + dmin - 2) & (N - 1), nrows = dmax - dmin + 5;
        // the window spans band tb from bit sh on and, when sh > 0, the start of the
        // next band: only those draw-plane words are read (in flight with the window's
        // rows), patched and written back
        const int sh = base & 31, tb = base >> 5, tn = (tb + 1) & (NB - 1);
        u32 oa[2], oc[2];
#pragma unroll
        for (int q = 0; q < 2; q++) {
            oa[q] = dp[tb * 128 + 64 * q];
            oc[q] = sh ? dp[tn * 128 + 64 * q] : 0u;
        }
        u32 P[32];
        if (pm) {           // the window's rows straight from the planes of bands tb, tn
            const u32 nm = nrows >= 32 ? 0xFFFFFFFFu : (1u << nrows) - 1u;
#pragma unroll
            for (int k = 0; k < 32; k++) {
                const int pl = k & 15;
                P[k] = 0u;
                if (pl == 0 || pl == 4 || pl == 6 || pl == 7) {
                    const u32 lo = pload(tb, k), hi = sh ? pload(tn, k) : 0u;
                    P[k] = (sh ? __builtin_amdgcn_alignbit(hi, lo, sh) : lo) & nm;
                }
            }
            // the edits, into the window's words (the planes in HBM get them after)
#pragma unroll
            for (int m = 0; m < 4; m++) {
                const int i = (int)((ec >> (16 * m)) & 0xFFFFu);
                if (i >= N * N) continue;                           // wave-uniform
                const int r = ((i >> 7) - base) & (N - 1), x = i & (N - 1);
                if (r >= nrows) continue;
                const u32 v = (u32)__builtin_amdgcn_readlane((int)ev, 16 * m);
                const u32 bit = 1u << r;
                const bool mine = lane == (x >> 1);
                if (x & 1) {
                    PL(P, 0, 1) = mine ? ((v & 1u) ? PL(P, 0, 1) | bit : PL(P, 0, 1) & ~bit) : PL(P, 0, 1);
                    PL(P, 4, 1) = mine ? ((v & 16u) ? PL(P, 4, 1) | bit : PL(P, 4, 1) & ~bit) : PL(P, 4, 1);
                    PL(P, 6, 1) = mine ? ((v & 64u) ? PL(P, 6, 1) | bit : PL(P, 6, 1) & ~bit) : PL(P, 6, 1);
                    PL(P, 7, 1) = mine ? ((v & 128u) ? PL(P, 7, 1) | bit : PL(P, 7, 1) & ~bit) : PL(P, 7, 1);
                } else {
                    PL(P, 0, 0) = mine ? ((v & 1u) ? PL(P, 0, 0) | bit : PL(P, 0, 0) & ~bit) : PL(P, 0, 0);
                    PL(P, 4, 0) = mine ? ((v & 16u) ? PL(P, 4, 0) | bit : PL(P, 4, 0) & ~bit) : PL(P, 4, 0);
                    PL(P, 6, 0) = mine ? ((v & 64u) ? PL(P, 6, 0) | bit : PL(P, 6, 0) & ~bit) : PL(P, 6, 0);
                    PL(P, 7, 0) = mine ? ((v & 128u) ? PL(P, 7, 0) | bit : PL(P, 7, 0) & ~bit) : PL(P, 7, 0);
                }
            }
        } else {
#pragma unroll
            for (int i = 0; i < 32; i++) P[i] = i < nrows ? gb[((base + i) & (N - 1)) * RS] : 0u;
            transpose32(P);
#pragma unroll
            for (int k = 0; k < 16; k++)
                if (k != 0 && k != 4 && k != 6 && k != 7) PL(P, k, 0) = PL(P, k, 1) = 0u;
        }
        GeoBand<SPAWN_COUNT> geo{lane, 0, HaloView{0u, 0u}, none, 0, 0, 0, nullptr};
        u32 ch[2];
        rule_planes(P, ch, geo, sc, 0u);
        u32 rm = 0u;                                    // window rows re-evaluated
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int y = (int)((rows >> (8 * j)) & 0xFFu);
            if (y < N) rm |= 7u << (((y - base) & (N - 1)) - 1);
        }
        int dn = 0;                                     // eligible cells gained - lost
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const u32 ma = rm << sh, na = (geo.e[q] & rm) << sh;
            const u32 a = oa[q];
            dn += __builtin_popcount(na) - __builtin_popcount(a & ma);
            dp[tb * 128 + 64 * q] = (a & ~ma) | na;
            if (sh) {
                const u32 mc = rm >> (32 - sh), nc = (geo.e[q] & rm) >> (32 - sh);
                const u32 c = oc[q];
                dn += __builtin_popcount(nc) - __builtin_popcount(c & mc);
                dp[tn * 128 + 64 * q] = (c & ~mc) | nc;
            }
        }
        return n0 + wave_total(dn);
    };
    // a board or goals without spawners (spawn_flags, set at reset: no rule or action
    // creates one) draws nothing; nor do goals at their fixed point (planes_ok bit 2)
    const int spf = rec(V, R_SPF) | (ka.ctp ? 1 : 0);     // toggling powers can make one
    const bool next = st.elig_planes && (rec(V, R_POK) & 8);
    int nb = 0;
    bool put = false;
    if (spf & 1) {
        nb = next ? count_next() : -1;
        if (nb < 0) {                   // the whole count reads the planes: edits first
            put_edits();
            put = true;
            wait_vm();
            nb = count(gb, 0);
        }
    }
    if (!put) put_edits();
    const int ng = ((rec(V, R_POK) & 6) == 6 || !(spf & 2)) ? 0 : count(gg, 1);
    const int dfl = (nb ? 1 : 0) | (ng ? 2 : 0);
    if (lane == 0) {
        w.counts[2 * b] = nb;
        w.counts[2 * b + 1] = ng;
        // the bit ring serves only envs with its threshold (k_bits_thr_check's test)
        if (ka.fx.bits_thr >= 0.0 && (nb | ng) && (double)st.spawn_prob[b] != ka.fx.bits_thr)
            atomicOr((unsigned long long *)w.err, (unsigned long long)SL_STREAM_ERR_THRESHOLD);
        // the tensors that draw, for the draws and the step (the action's edited rows
        // in this slot have been read)
        if (dp) w.act[st.B + b] = dfl;
    }
    nb_out = nb;
    ng_out = ng;
    dfl_out = dfl;
}

__global__ void __launch_bounds__(64)
k_stream_prologue128(Step128KArgs ka) {
    int nb, ng, dfl;
    count_env128(ka, blockIdx.x, threadIdx.x, nb, ng, dfl);
}

// The two 32x32 bit matrices held by lanes 0-31 and 32-63, transposed within each
// half (bit y of lane i's word -> bit i of lane y's word): five block-swap stages,
// the partner word (lane ^ s) from ds_swizzle, the swapped block by a rotation and a
// bitfield insert.
template <int S, u32 M>
__device__ __forceinline__ u32 swap_stage(u32 x, int lane) {
    const bool hi = (lane & S) != 0;
    const u32 p = (u32)__builtin_amdgcn_ds_swizzle((int)x, 0x1F | (S << 10));
    const u32 sh = __builtin_amdgcn_alignbit(p, p, hi ? S : 32 - S);     // rotate
    const u32 mm = hi ? ~M : M;
    return (x & mm) | (sh & ~mm);
}
__device__ __forceinline__ u32 transpose_halves(u32 x, int lane) {
    x = swap_stage<16, 0x0000FFFFu>(x, lane);
    x = swap_stage<8, 0x00FF00FFu>(x, lane);
    x = swap_stage<4, 0x0F0F0F0Fu>(x, lane);
    x = swap_stage<2, 0x33333333u>(x, lane);
    return swap_stage<1, 0x55555555u>(x, lane);
}

// inclusive sum over the lanes of each 32-lane half
__device__ __forceinline__ int scan_halves(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true);     // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true);     // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true);     // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true);     // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);    // row_bcast:15
    return v;
}

// Replay-mode draws of env b, after the offsets scan: each drawing tensor's eligible
// cells (the draw planes, from k_stream_prologue128) take the uniforms from its
// offset on in row-major order, one per eligible cell (random.c:47-52 consumed by
// advance_board.c:109-113), and the cells that spawn replace them in the draw planes.
// The step kernel then only ANDs them into its spawns.  Ranks without a pass per row:
//  * each band's two words are transposed across the lanes (transpose_halves): lane
//    32k + r then holds row r's cells of lanes 32k..32k+31 -- a "segment" of 64
//    cells, in the stream's order; segments run (band, row, half);
//  * segment sizes by popcount, their bases by a scan over the rows (DPP) and the
//    band totals;
//  * each lane walks its segments' cells and writes their ids (band, row, column
//    pair, word) into LDS slots at their ranks (ranks past kOwnSlots go in a later
//    chunk);
//  * lane i takes the ranks i, i + 64, ...: its slot and the uniform draws[pos + i]
//    (contiguous over the lanes: each load instruction one coalesced 512-byte run,
//    kDrawBatch in flight per lane); a spawn is ORed into the owner's word in LDS.
// Measured against a binary search per rank over the segment bases (C5, same box):
// 47.3 vs 46.8 M env-steps/s (tools/ab/c5s_owner.py); against a ballot per eligible
// row: 271 -> ~170 us per step.
constexpr int kDrawBatch = 8;
constexpr int kOwnSlots = 2048;
__device__ __forceinline__ void draw_env128(const Step128KArgs &ka, int64_t b, int lane, int dfl,
                                           int64_t pos_b, int64_t pos_g) {
    const sl_env_state &st = ka.st;
    const Scratch w = scratch_of(ka.fx.scratch, st.B);
    if (!(dfl & 3)) return;
    __shared__ uint16_t slots_[kOwnSlots];
    lds_u16 *slots = (lds_u16 *)slots_;
    __shared__ u32 spw_[NB * 2 * 64];
    typedef __attribute__((address_space(3))) u32 lds_u32;
    lds_u32 *spw = (lds_u32 *)spw_;
    const double thr = (double)st.spawn_prob[b];
    const double *draws = ka.a.draws;
    const int64_t n_draws = ka.a.n_draws, draw_mask = ka.a.draw_mask;
    u32 *dp = st.elig_planes + b * kEligStride + kDrawPlanes + lane;
#pragma unroll 1
    for (int tensor = 0; tensor < 2; tensor++) {
        if (!((dfl >> tensor) & 1)) continue;
        u32 E[NB][2];
#pragma unroll
        for (int t = 0; t < NB; t++)
#pragma unroll
            for (int q = 0; q < 2; q++) E[t][q] = dp[(tensor * NB + t) * 128 + 64 * q];
        if (thr <= 0.0 || thr >= 1.0) {        // consumed, never compared (stream_draws)
#pragma unroll
            for (int t = 0; t < NB; t++)
#pragma unroll
                for (int q = 0; q < 2; q++)
                    dp[(tensor * NB + t) * 128 + 64 * q] = thr >= 1.0 ? E[t][q] : 0u;
            continue;
        }
        const int64_t pos = tensor ? pos_g : pos_b;
        // the segments: bases, then each owner lane writes its cells' ids at their ranks
        int total = 0;
        const int half = lane >> 5;
        u32 R0[NB], R1[NB];
        int base[NB];
#pragma unroll
        for (int t = 0; t < NB; t++) {
            R0[t] = transpose_halves(E[t][0], lane);
            R1[t] = transpose_halves(E[t][1], lane);
            const int c = __builtin_popcount(R0[t]) + __builtin_popcount(R1[t]);
            const int cp = __builtin_amdgcn_ds_bpermute((lane ^ 32) << 2, c);
            const int rc = c + cp;                      // the row's cells (both halves)
            const int incl = scan_halves(rc);
            base[t] = total + incl - rc + (half ? cp : 0);
            total += __builtin_amdgcn_readlane(incl, 31);
        }
#pragma unroll
        for (int k = 0; k < NB * 2; k++) spw[k * 64 + lane] = 0u;
#pragma unroll 1
        for (int c0 = 0; c0 < total; c0 += kOwnSlots) {
#pragma unroll
            for (int t = 0; t < NB; t++) {
                u32 m = R0[t] | R1[t];
                int rk = base[t] - c0;
                while (m) {
                    const int i = __builtin_ctz(m);
                    m &= m - 1u;
                    const u32 e0 = (R0[t] >> i) & 1u, e1 = (R1[t] >> i) & 1u;
                    const u32 id = (u32)((t << 12) | ((lane & 31) << 7) | (32 * half + i));
                    if (e0 && (u32)rk < (u32)kOwnSlots) slots[rk] = (uint16_t)id;
                    rk += (int)e0;
                    if (e1 && (u32)rk < (u32)kOwnSlots) slots[rk] = (uint16_t)(id | 64u);
                    rk += (int)e1;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            const int n = min(total - c0, kOwnSlots);
#pragma unroll 1
            for (int i0 = 0; i0 < n; i0 += 64 * kDrawBatch) {
                double u[kDrawBatch];
                u32 id[kDrawBatch];
#pragma unroll
                for (int k = 0; k < kDrawBatch; k++) {
                    const int i = i0 + 64 * k + lane;
                    const int64_t r = pos + c0 + i;
                    id[k] = i < n ? (u32)slots[i] : 0u;
                    u[k] = (i < n && r < n_draws) ? draws[r & draw_mask] : 1.0;
                    if (i < n && r >= n_draws) atomicOr((unsigned long long *)w.err, 1ull);
                }
#pragma unroll
                for (int k = 0; k < kDrawBatch; k++)
                    if (u[k] < thr) {
                        const u32 t = id[k] >> 12, y = (id[k] >> 7) & 31u, q = (id[k] >> 6) & 1u;
                        __hip_atomic_fetch_or(&spw[(t * 2 + q) * 64 + (id[k] & 63u)], 1u << y,
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int t = 0; t < NB; t++)
#pragma unroll
            for (int q = 0; q < 2; q++)
                dp[(tensor * NB + t) * 128 + 64 * q] = spw[(t * 2 + q) * 64 + lane] & E[t][q];
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");   // before the next tensor's
        __builtin_amdgcn_wave_barrier();                        // segment writes
    }
}

__global__ void __launch_bounds__(64)
k_stream_draw128(Step128KArgs ka) {
    const int64_t b = blockIdx.x;
    const Scratch w = scratch_of(ka.fx.scratch, ka.st.B);
    draw_env128(ka, b, threadIdx.x, (int)w.act[ka.st.B + b], w.offsets[2 * b], w.offsets[2 * b + 1]);
}

// The draws from the device generator's bit ring (sl_mt.hip, sl_mt19937.bit_ring): the
// ring holds the decisions (u < p) themselves, so a segment's spawns are its next
// stream bits deposited into its eligible cells in order -- no slots, no uniforms,
// no LDS (so more waves in flight), a 64-bit window of the ring per segment.  The
// board's planes are loaded with the tensors-that-draw word and the offsets (one
// round trip), the ring words after the ranks (a second).
__global__ void __launch_bounds__(64)
k_stream_draw128_bits(Step128KArgs ka) {
    const int64_t b = blockIdx.x;
    const int lane = threadIdx.x;
    const sl_env_state &st = ka.st;
    const Scratch w = scratch_of(ka.fx.scratch, st.B);
    u32 *dp = st.elig_planes + b * kEligStride + kDrawPlanes + lane;
    const int dfl = (int)w.act[st.B + b];
    const int64_t pos_t[2] = {w.offsets[2 * b], w.offsets[2 * b + 1]};
    u32 E[NB][2];
#pragma unroll
    for (int t = 0; t < NB; t++)
#pragma unroll
        for (int q = 0; q < 2; q++) E[t][q] = dp[t * 128 + 64 * q];     // the board's
    const double thr = (double)st.spawn_prob[b];
    const uint32_t *bits = ka.a.draw_bits;
    const int64_t draw_mask = ka.a.draw_mask, wmask = draw_mask >> 5;
    const int half = lane >> 5;
#pragma unroll 1
    for (int tensor = 0; tensor < 2; tensor++) {
        if (!((dfl >> tensor) & 1)) continue;
        if (tensor == 1) {
#pragma unroll
            for (int t = 0; t < NB; t++)
#pragma unroll
                for (int q = 0; q < 2; q++) E[t][q] = dp[(NB + t) * 128 + 64 * q];
        }
        if (thr <= 0.0 || thr >= 1.0) {        // consumed, never compared (stream_draws)
#pragma unroll
            for (int t = 0; t < NB; t++)
#pragma unroll
                for (int q = 0; q < 2; q++)
                    dp[(tensor * NB + t) * 128 + 64 * q] = thr >= 1.0 ? E[t][q] : 0u;
            continue;
        }
        // segments (band, row, half) in stream order, as draw_env128 ranks them
        int total = 0;
        u32 R0[NB], R1[NB];
        int64_t at[NB];
#pragma unroll
        for (int t = 0; t < NB; t++) {
            R0[t] = transpose_halves(E[t][0], lane);
            R1[t] = transpose_halves(E[t][1], lane);
            const int c = __builtin_popcount(R0[t]) + __builtin_popcount(R1[t]);
            const int cp = __builtin_amdgcn_ds_bpermute((lane ^ 32) << 2, c);
            const int rc = c + cp;
            const int incl = scan_halves(rc);
            at[t] = (pos_t[tensor] + total + incl - rc + (half ? cp : 0)) & draw_mask;
            total += __builtin_amdgcn_readlane(incl, 31);
        }
        u32 w0[NB], w1[NB], w2[NB];
#pragma unroll
        for (int t = 0; t < NB; t++) {          // every band's ring words in flight
            const int64_t wi = at[t] >> 5;
            w0[t] = bits[wi];
            w1[t] = bits[(wi + 1) & wmask];
            w2[t] = bits[(wi + 2) & wmask];
        }
#pragma unroll
        for (int t = 0; t < NB; t++) {
            const int sh = (int)(at[t] & 31);
            uint64_t sb = ((((uint64_t)w1[t]) << 32) | w0[t]) >> sh;
            if (sh) sb |= ((uint64_t)w2[t]) << (64 - sh);
            // column pair i in order: the even column's cell (e) takes the next bit,
            // the odd one's (f) the bit after it when e is set -- branch-free, 12 VALU
            // a pair instead of 21 (the loop runs to the wave's fullest segment)
            const u32 r0 = R0[t], r1 = R1[t];
            u32 m = r0 | r1, s0 = 0u, s1 = 0u;
            while (m) {
                const int i = __builtin_ctz(m);
                m &= m - 1u;
                const u32 e = (r0 >> i) & 1u, f = (r1 >> i) & 1u, lo = (u32)sb;
                s0 |= (lo & e) << i;
                s1 |= ((lo >> e) & f) << i;
                sb >>= e + f;
            }
            // back to the planes' layout (transpose_halves is an involution)
            dp[(tensor * NB + t) * 128] = transpose_halves(s0, lane) & E[t][0];
            dp[(tensor * NB + t) * 128 + 64] = transpose_halves(s1, lane) & E[t][1];
        }
    }
}

// ---- board planes (sl_env_state.board_planes, plane mode)
// k_env_action for a plane-mode step (one lane per env): an env whose board is in
// planes (planes_ok bit 6) reads the cells its action can touch from the uint16 board
// -- the step kernel keeps them current (the agent's row, and its column two rows up
// and down) -- and writes its edits there.  Other envs take the uint16 action
// (env_action_one); an env with no scratch row list entry is then not in plane mode.
__global__ void __launch_bounds__(256)
k_env_action_planes128(sl_env_state st, const int32_t *__restrict__ actions, int ctp, int ctc,
                       int64_t *__restrict__ act) {
    const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= st.B) return;
    if (!(st.planes_ok[b] & 64)) {
        env_action_one<false>(st, actions, ctp, ctc, act, b);
        return;
    }
    uint16_t *bd = st.board + b * (int64_t)(N * N);
    const int a = actions[b];
    fast::GlobalEnv e{st, b};
    fast::OverlayT<fast::GlobalCells> ov;
    ov.src.bd = bd;
    ov.n = 0;
    const int reward = fast::act_core(e, a, N, N, ctp, ctc, ov);
    // the edits go to the uint16 cells only; the cells (up to four 16-bit indices,
    // 0xFFFF none) go to scratch act[B + b] and their changed bits to act[2B + b],
    // which the step kernel flips in its planes.  (Writing the edits into the planes here --
    // one XOR atomic per changed bit, or a read-modify-write of each edited cell's 16
    // words -- cost 31 / 44 us per launch against 9 us for the uint16 action.)
    uint64_t cells = ~0ull, vals = 0ull;
#pragma unroll
    for (int k = 0; k < 4; k++) {       // (static indices: the overlay stays in registers)
        if (k >= ov.n) continue;
        const int i = ov.idx[k];
        const u32 v = ov.val[k], d = v ^ ov.src(i);    // (read before the cell is written)
        if (!d) continue;
        bd[i] = (uint16_t)v;
        cells = (cells << 16) | (uint64_t)i;
        vals = (vals << 16) | (uint64_t)d;
    }
    if (st.elig_planes) {
        // replay: the count prologue (count_env128) puts the edits into the planes and
        // re-counts the rows round them (act[B + b], as env_action_one leaves them)
        uint32_t rows = 0xFFFFFFFFu;
#pragma unroll
        for (int m = 0; m < 4; m++) {
            const uint32_t i = (uint32_t)((cells >> (16 * m)) & 0xFFFFu);
            if (i >= (uint32_t)(N * N)) continue;
            const uint32_t y = i >> 7;
            bool seen = false;
            for (int j = 0; j < 4; j++) seen = seen || ((rows >> (8 * j)) & 0xFFu) == y;
            if (!seen) rows = (rows << 8) | y;
        }
        act[st.B + b] = (int64_t)rows;
        act[3 * st.B + b] = (int64_t)cells;
    } else {
        act[st.B + b] = (int64_t)cells;
        act[2 * st.B + b] = (int64_t)vals;
    }
    act[b] = reward;
}

// sl_env_board_sync / sync_board_planes: one wave per env
__global__ void __launch_bounds__(64) k_board_sync128(sl_env_state st, int demote) {
    const int64_t b = blockIdx.x;
    const int lane = threadIdx.x;
    const int pok = __builtin_amdgcn_readfirstlane(st.planes_ok[b]);
    if (!(pok & 64)) return;
    if (!(pok & 128)) {
        // the exit cells hold their colour in the uint16 board only (the epilogue
        // writes them): read before the rows are rewritten, put back after
        uint16_t *cells = st.board + b * (int64_t)(N * N);
        const int ne = min(__builtin_amdgcn_readfirstlane(st.exit_count[b]), SL_MAX_EXITS);
        int ei = -1;
        uint16_t ev = 0;
        if (lane < ne) {
            ei = st.exit_y[b * SL_MAX_EXITS + lane] * N + st.exit_x[b * SL_MAX_EXITS + lane];
            ev = cells[ei];
        }
        wait_vm();
        const u32 *bp = st.board_planes + b * (int64_t)(NB * MW) + lane;
        u32 *gb = reinterpret_cast<u32 *>(st.board + b * (int64_t)(N * N)) + lane;
        const u32 zero = st.board_zero;     // (planes no board holds: never stored)
#pragma unroll 1
        for (int t = 0; t < NB; t++) {
            u32 P[32];
#pragma unroll
            for (int k = 0; k < 32; k++) P[k] = ((zero >> (k & 15)) & 1u) ? 0u : bp[t * MW + k * 64];
            transpose32(P);
#pragma unroll
            for (int y = 0; y < 32; y++) gb[(32 * t + y) * RS] = P[y];
        }
        wait_vm();
        if (ei >= 0) cells[ei] = ev;
    }
    if (lane == 0) st.planes_ok[b] = demote ? pok & ~(64 | 128 | 256) : pok | 128;
}

}  // namespace

namespace sl {

bool bits128_shape(const sl_env_state &st) {
    return st.H == N && st.W == N && st.planes && st.planes_ok;
}

int sync_board_planes(const sl_env_state &st, int demote, hipStream_t s) {
    if (st.H == 64) return sync_board_planes64(st, demote, s);
    if (!st.board_planes || !st.planes_ok || st.H != N || st.W != N || st.B <= 0) return SL_OK;
    hipLaunchKernelGGL(k_board_sync128, dim3((unsigned)st.B), dim3(64), 0, s, st, demote);
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}

int launch_step_bits128(const sl_env_state &st, const StepArgs &a, const FastExtra &fx,
                        const int32_t *actions, int ctp, int ctc, double *reward, uint8_t *done,
                        uint8_t *flags, int32_t *ep_len, int32_t *ep_rew, hipStream_t s) {
    if (!bits128_shape(st)) return SL_ETOOBIG;
    const Step128KArgs ka{st, a, fx, actions, ctp, ctc, reward, done, flags, ep_len, ep_rew};
    const dim3 grid((unsigned)st.B);
    if (fx.stream) {
        if (stream_counts(fx)) {
            if (fx.plane_mode) {
                hipLaunchKernelGGL(k_env_action_planes128, dim3((unsigned)((st.B + 255) / 256)),
                                   dim3(256), 0, s, st, actions, ctp, ctc,
                                   scratch_of(fx.scratch, st.B).act);
                if (hipGetLastError() != hipSuccess) return SL_EHIP;
            } else {
                const int rca = launch_env_action(st, actions, ctp, ctc, scratch_of(fx.scratch, st.B).act, s);
                if (rca) return rca;
            }
            hipLaunchKernelGGL(k_stream_prologue128, grid, dim3(64), 0, s, ka);
            if (hipGetLastError() != hipSuccess) return SL_EHIP;
        }
        FastExtra fo = fx;
        fo.thr_checked = stream_counts(fx);     // (in the count prologue)
        const int rc = stream_offsets(st, fo, s);
        if (rc || !stream_steps(fx)) return rc;
        if (st.elig_planes) {       // draws decided up front
            if (a.draw_bits)
                hipLaunchKernelGGL(k_stream_draw128_bits, grid, dim3(64), 0, s, ka);
            else
                hipLaunchKernelGGL(k_stream_draw128, grid, dim3(64), 0, s, ka);
            if (hipGetLastError() != hipSuccess) return SL_EHIP;
            if (fx.ev_begin) (void)hipEventRecord((hipEvent_t)fx.ev_begin, s);
            launch_step128<SPAWN_DECIDED>(ka, fx.plane_mode && fx.obs_out, s);
        } else {
            if (fx.ev_begin) (void)hipEventRecord((hipEvent_t)fx.ev_begin, s);
            hipLaunchKernelGGL((k_env_step_bits128<SPAWN_STREAM, kKeep128All>), grid, dim3(64), 0, s, ka);
        }
    } else {
        if (fx.plane_mode) {
            hipLaunchKernelGGL(k_env_action_planes128, dim3((unsigned)((st.B + 255) / 256)),
                               dim3(256), 0, s, st, actions, ctp, ctc,
                               scratch_of(fx.scratch, st.B).act);
            if (hipGetLastError() != hipSuccess) return SL_EHIP;
        } else {
            const int rc = launch_env_action(st, actions, ctp, ctc, scratch_of(fx.scratch, st.B).act, s);
            if (rc) return rc;
        }
        if (fx.ev_begin) (void)hipEventRecord((hipEvent_t)fx.ev_begin, s);
        launch_step128<SPAWN_PHILOX>(ka, fx.plane_mode && fx.obs_out, s);
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
