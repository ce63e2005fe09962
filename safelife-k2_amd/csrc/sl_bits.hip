// sl_bits.hip -- the bit-sliced fused env-step kernel for 64x64 boards.
//
// Same semantics as k_env_action + k_env_step_generic (sl_env.hip); different data
// layout, chosen for CDNA4's VALU-issue limit:
//
//  * one wave64 per env; lane l owns the column pair (2j, 2j+1), j = l >> 1, for
//    the 32-row half h = l & 1 (rows 32h .. 32h+31);
//  * each lane loads its 32 dwords D[y] = cell(32h+y, 2j) | cell(32h+y, 2j+1) << 16
//    (every load instruction covers two full 128-byte rows) and transposes them in
//    registers (32x32 bit transpose: 2 v_perm stages + 3 bfi stages, 256 VALU
//    ops), giving 16 bit planes x 2 words: plane k, word w, bit y = bit k of
//    cell(32h + y, 2j + w);
//  * the rule (advance_board.c:34-120) is then evaluated as
//    bitwise logic on 32 cells per operation: vertical neighbours are funnel
//    shifts (v_alignbit) against the other half's word (DPP quad_perm lane swap),
//    horizontal neighbours are the lane's other word or a 2-lane whole-wave DPP
//    rotation (wave_ror:1 / wave_rol:1, wrapping at W = 64), the 3x3 alive count
//    is a bit-sliced adder and the >= 2 tests are majority functions -- about
//    120 VALU ops per 32 cells against ~1300 for the packed two-cells-per-register
//    form;
//  * points, performance score, possible score and side effects
//    (safelife_game.py:590-631, env_wrappers.py:319-342) are recomputed in full
//    every step from the new planes with bitwise masks and v_bcnt;
//  * the new planes are transposed back and only the rows that changed are
//    stored (a wave-wide OR of the per-column change masks picks them).
// The action (execute_action / move_agent, safelife_game.py:308-393) runs on lane
// 0 while the column loads are in flight; its cell edits are broadcast and
// written into the planes before the rule.  Envs that finish are queued; a second
// kernel (k_env_reset_list) resets exactly those, one wave each, so the step
// kernel carries no reset code (128 VGPRs, 4 waves/SIMD, no spills).  The <true>
// instantiation also writes the packed observation (write_obs, 130 VGPRs, 3 waves).
#include "sl_bits.h"
#include "sl_obs.h"

using namespace sl;
using namespace sl::fast;
using namespace sl::bits;

namespace {

constexpr int kMinWaves = 4;      // waves per SIMD the register budget is sized for
constexpr int kMinWavesObs = 3;   // the same for the instantiations that write views or
                                  // replay the reference stream

constexpr int N = 64;        // rows = columns = lanes

// Neighbourhood of the 64x64 layout: lane l holds columns 2j, 2j+1 (j = l >> 1) over
// rows 32h .. 32h+31 (h = l & 1).  Column 2j - 1 is word 1 of lane l - 2 and column
// 2j + 2 word 0 of lane l + 2 (the 64-lane rotation wraps at W = 64); the rows
// around a word come from the other half's word (lane l ^ 1), which also supplies
// the wrap at H = 64.
template <int MODE>
struct Geo64 {
    int lane;
    StreamSrc src;     // SPAWN_STREAM: the supplied uniforms; pos = this tensor's first
    int64_t pos;
    int count;         // SPAWN_COUNT: this lane's eligible cells
    template <class F>
    __device__ __forceinline__ V3 vert(const u32 *P, int w, F f) const {
        const u32 x = f(P, w);
        return vert_with(x, lane_x1(x));
    }
    __device__ __forceinline__ H3 horiz(u32 w0, u32 w1) const {
        return H3{lane_m1(lane_m1(w1)), lane_p1(lane_p1(w0))};
    }
    __device__ __forceinline__ bool halo_spawn() const { return false; }
    // the 2x2 spawn block of rows 32h + y, y + 1 (y even) of the lane's column pair
    __device__ __forceinline__ u32 block(int y) const {
        return (u32)(((32 * (lane & 1) + y) >> 1) * (N / 2) + (lane >> 1));
    }
    // spawners are rare on these boards: per-lane Philox draws, no LDS list
    __device__ __forceinline__ void spawn(const u32 elig[2], u32 sp[2], const SpawnCtx &sc,
                                          u32 tensor) {
        if (MODE == SPAWN_PHILOX) {
            philox_spawn(*this, elig, sp, sc, tensor);
        } else if (MODE == SPAWN_STREAM) {
            (void)stream_draws<true>(elig, sp, sc.thr, src, pos, lane);
        } else {
            count += __builtin_popcount(elig[0]) + __builtin_popcount(elig[1]);
        }
    }
};

// ---------------------------------------------------------------- LDS staging
// A wave's 8 KiB LDS buffer holds one 64x64 board, row-major, with the 16-byte
// chunks of rows 32..63 rotated by 4 chunks so that the even (rows 0..31) and odd
// (rows 32..63) lanes of a column-pair read fall in different banks.
typedef __attribute__((address_space(3))) u32 lds_u32;

__device__ __forceinline__ void dma_board(const uint16_t *__restrict__ src, lds_u32 *buf,
                                          int lane) {
    const char *s = reinterpret_cast<const char *>(src);
#pragma unroll
    for (int k = 0; k < 8; k++) {          // 8 x (64 lanes x 16 B), LDS chunk q = 64k + lane
        const int q = k * 64 + lane, row = q >> 3, pos = q & 7;
        const int c = (pos - ((row >> 5) << 2)) & 7;
        __builtin_amdgcn_global_load_lds((const void *)(s + row * 128 + c * 16),
                                         (__attribute__((address_space(3))) void *)(buf + k * 256),
                                         16, 0, 2);
    }
}

// the lane's 32 dwords (rows 32h + y, column pair j) from the staged board
__device__ __forceinline__ void read_pairs(const lds_u32 *buf, int lane, u32 D[32]) {
    const int h = lane & 1, j = lane >> 1;
    const lds_u32 *p = buf + h * 1024 + ((j + 16 * h) & 31);
#pragma unroll
    for (int y = 0; y < 32; y++) D[y] = p[y * 32];
}

// The start-board planes the side-effect term needs (0, 2, 7-15), from the level
// pool's precomputed bit planes: the start board of an env reset from the pool is
// level li rolled by (dy, dx) (sl_env_state.start_roll).  Column c of the start
// board is level column c - dx; its 64-bit row column rotated by dy gives rows
// 32h .. 32h+31 as one funnel shift.  The pool stays in L2 / the Infinity Cache,
// so this costs no HBM traffic and no transpose.  The level's planes 0-3 and 6-15
// (7 KiB, seven 1 KiB DMA rows) are copied into the wave's board buffer as soon as
// the board has been read out of it, so their (queueing-dominated) latency runs
// under the action and the rule (issued at scoring time, it was ~40% of a wave's
// life; held in registers instead, it spills).
// KEEP: the planes any board (and so any start board) can hold; a row whose two planes
// the scores do not need (1, 3, 6 are never read) or no board holds is not copied
template <u32 KEEP = 0xFFFFu>
__device__ __forceinline__ void pool_dma(const sl_level_pool &pool, int li, lds_u32 *buf,
                                         int lane) {
    const char *pl = reinterpret_cast<const char *>(pool.board_planes + (int64_t)li * 16 * N);
    constexpr u32 need = KEEP & 0xFF85u;         // planes 0, 2, 7-15
#pragma unroll
    for (int k = 0; k < 7; k++) {       // LDS row k <- planes (0,1), (2,3), (6,7) .. (14,15)
        const int p0 = k < 2 ? 2 * k : 2 * k + 2;
        if (!((need >> p0) & 3u)) continue;
        __builtin_amdgcn_global_load_lds((const void *)(pl + p0 * N * 8 + lane * 16),
                                         (__attribute__((address_space(3))) void *)(buf + k * 256),
                                         16, 0, 0);
    }
}
template <u32 KEEP = 0xFFFFu>
__device__ __forceinline__ void pool_planes_lds(const lds_u32 *buf, int dy, int dx, int lane,
                                                u32 S[32]) {
    const int c0 = (2 * (lane >> 1) - dx) & 63, c1 = (c0 + 1) & 63;
    const int r = (32 * (lane & 1) - dy) & 63;
    const bool lo_first = r < 32;
    const u32 sh = (u32)(r & 31);
#pragma unroll
    for (int p = 0; p < 16; p++) {
        if (p == 1 || (p >= 3 && p <= 6) || !((KEEP >> p) & 1u)) {
            PL(S, p, 0) = 0u;
            PL(S, p, 1) = 0u;
            continue;
        }
        const int slot = p < 4 ? p : p - 2;             // LDS plane slot
        const lds_u32 *q = buf + slot * 128;            // 64 columns x 2 dwords
        const u32 a0 = q[2 * c0], a1 = q[2 * c0 + 1], b0 = q[2 * c1], b1 = q[2 * c1 + 1];
        PL(S, p, 0) = lo_first ? __builtin_amdgcn_alignbit(a1, a0, sh)
                               : __builtin_amdgcn_alignbit(a0, a1, sh);
        PL(S, p, 1) = lo_first ? __builtin_amdgcn_alignbit(b1, b0, sh)
                               : __builtin_amdgcn_alignbit(b0, b1, sh);
    }
}


// unedited cells for the action, from the staged board (dma_board's layout)
typedef __attribute__((address_space(3))) const uint16_t lds_cu16;
struct LdsCells {
    const lds_u32 *buf;
    __device__ __forceinline__ uint32_t operator()(int i) const {
        const int row = i >> 6, col = i & 63;
        const int pos = ((col >> 3) + ((row >> 5) << 2)) & 7;
        return reinterpret_cast<lds_cu16 *>(buf)[row * 64 + pos * 8 + (col & 7)];
    }
};

// The action's cell edits (wave-uniform (flat index, value) pairs) written into the
// planes on the lane holding each cell; returns the row pairs (bit y: rows y, y + 32)
// holding an edit, whose stores are then forced.
__device__ __forceinline__ u32 mux_edits(u32 P[32], int ne, const int eidx[4], const u32 eval[4],
                                         int lane) {
    u32 erow = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (k < ne) {
            const int y = eidx[k] >> 6, x = eidx[k] & 63;
            const int tl = 2 * (x >> 1) + (y >> 5);            // lane holding the cell
            const u32 bit = 1u << (y & 31);
            const u32 m0 = (lane == tl && !(x & 1)) ? bit : 0u;
            const u32 m1 = (lane == tl && (x & 1)) ? bit : 0u;
            erow |= bit;
#pragma unroll
            for (int p = 0; p < 16; p++) {
                const u32 v = ((eval[k] >> p) & 1u) ? ~0u : 0u;
                PL(P, p, 0) = mux(m0, v, PL(P, p, 0));
                PL(P, p, 1) = mux(m1, v, PL(P, p, 1));
            }
        }
    }
    return erow;
}

// SafeLifeEnv.reset (safelife_env.py:188-198) of env b by one wave, right after the
// step that finished the episode (ContinuingEnv + run_agents' reset-on-done).
// Same result as reset_one (sl_env.hip): the rolled level is copied into board,
// goals and start board; points, perf baseline and possible are the bit-sliced sums
// over it; the exit list is collected row by row in np.nonzero order.
__device__ __forceinline__ void wave_reset(const sl_env_state &st, const sl_level_pool &pool,
                                        const ResetArgs &ra, int64_t b, int lane) {
    const int ep = __builtin_amdgcn_readfirstlane(st.episodes[b]);
    const LevelChoice lc = choose_level_wave(pool, ra, ra.env0 + (uint32_t)b, ep, N, N, lane);
    const int li = lc.idx, dy = lc.dy, dx = lc.dx;
    const LevelScalars ls = level_scalars(pool, li);     // in flight with the gathers
    const int h = lane & 1, j = lane >> 1;
    const uint16_t *lb = pool.board + (int64_t)li * (N * N), *lg = pool.goals + (int64_t)li * (N * N);
    const int c0 = (2 * j - dx) & 63, c1 = (2 * j + 1 - dx) & 63;
    const int64_t off = b * (int64_t)(N * N);
    const int lane_off = h * 1024 + j;
    u32 *gs = reinterpret_cast<u32 *>(st.start_board + off) + lane_off;
    u32 *gg = reinterpret_cast<u32 *>(st.goals + off) + lane_off;
    u32 *gb = reinterpret_cast<u32 *>(st.board + off) + lane_off;
    // the lane's 32 dwords of a rolled pool level (all gathers in flight at once:
    // this runs in its own kernel, registers are plentiful)
    auto rolled = [&](const uint16_t *lv, u32 D[32]) {
#pragma unroll
        for (int y = 0; y < 32; y++) {
            const int sr = ((32 * h + y - dy) & 63) * N;
            D[y] = (u32)lv[sr + c0] | ((u32)lv[sr + c1] << 16);
        }
    };
    // both gathers in flight together; the board's rows serve the start board (as
    // loaded), the sums (transposed copy) and the board itself (exits coloured)
    u32 P[32], D[32];
    rolled(lg, P);
    rolled(lb, D);
    // goals: copy, then keep their colour planes for the sums
#pragma unroll
    for (int y = 0; y < 32; y++) gg[y * 32] = P[y];
    transpose32(P);
    u32 *mg = st.planes ? st.planes + b * 4096 + 2048 + lane : nullptr;
    if (mg) {      // the goals' bit-plane mirror
#pragma unroll
        for (int q = 0; q < 32; q++) mg[q * 64] = P[q];
    }
    u32 gcol[3][2];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        gcol[k][0] = PL(P, 9 + k, 0);
        gcol[k][1] = PL(P, 9 + k, 1);
    }
    const bool sg = __ballot((PL(P, 7, 0) | PL(P, 7, 1)) != 0u) != 0ull;
    // start board: copy, then the sums over the initial board and goals
#pragma unroll
    for (int y = 0; y < 32; y++) {
        gs[y * 32] = D[y];
        P[y] = D[y];
    }
    transpose32(P);
    int pts, scr, pos, side;
    score_planes(P, gcol, P, &pts, &scr, &pos, &side);
    const int s1 = wave_total((pts + 192) | ((scr + 64) << 16));
    const int s2 = wave_total(pos);
    const bool sb = __ballot((PL(P, 7, 0) | PL(P, 7, 1)) != 0u) != 0ull;
    int ev = 0;
    if (lane == 0)
        ev = reset_scalars_from(st, ra, b, li, dy, dx, ls, ep, (s1 & 0xFFFF) - 192 * 64,
                                ((s1 >> 16) & 0xFFFF) - 64 * 64, s2, (sb ? 1 : 0) | (sg ? 2 : 0));
    ev = __builtin_amdgcn_readfirstlane(ev);
    const u32 ex0 = PL(P, 8, 0), ex1 = PL(P, 8, 1);       // exit planes
    // the board: the start board with its exits coloured (update_exit_colors)
    {
#pragma unroll
        for (int y = 0; y < 32; y++) {
            u32 d = D[y];
            if (d & (u32)EXIT) d = (d & 0xFFFF0000u) | (u32)ev;
            if (d & ((u32)EXIT << 16)) d = (d & 0x0000FFFFu) | ((u32)ev << 16);
            gb[y * 32] = d;
        }
    }
    // exits in np.nonzero (row-major) order: repeatedly take the wave-wide smallest
    // key row * 64 + column among the lanes' remaining exit bits (one round per exit)
    const int n_exit = wave_total(__builtin_popcount(ex0) + __builtin_popcount(ex1));
    {
        u32 e0 = ex0, e1 = ex1;
        const int kmax = n_exit < SL_MAX_EXITS ? n_exit : SL_MAX_EXITS;   // uniform
        for (int k = 0; k < kmax; k++) {
            const u32 k0 = e0 ? (u32)((32 * h + __builtin_ctz(e0)) * N + 2 * j) : 0xFFFFu;
            const u32 k1 = e1 ? (u32)((32 * h + __builtin_ctz(e1)) * N + 2 * j + 1) : 0xFFFFu;
            u32 m = k0 < k1 ? k0 : k1;
            m = min(m, dpp<0xB1>(m));
            m = min(m, dpp<0x4E>(m));
            m = min(m, dpp<0x141>(m));
            m = min(m, dpp<0x140>(m));
            const u32 key = min(min((u32)__builtin_amdgcn_readlane((int)m, 0),
                                    (u32)__builtin_amdgcn_readlane((int)m, 16)),
                                min((u32)__builtin_amdgcn_readlane((int)m, 32),
                                    (u32)__builtin_amdgcn_readlane((int)m, 48)));
            if (k0 == key) e0 &= e0 - 1;
            if (k1 == key) e1 &= e1 - 1;
            if (lane == 0) {
                st.exit_y[b * SL_MAX_EXITS + k] = (int16_t)(key >> 6);
                st.exit_x[b * SL_MAX_EXITS + k] = (int16_t)(key & 63);
            }
        }
    }
    if (lane == 0) {
        if (mg) st.planes_ok[b] = 2;   // after reset_scalars cleared it
        st.exit_count[b] = n_exit;
        for (int e = n_exit; e < SL_MAX_EXITS; e++) {
            st.exit_y[b * SL_MAX_EXITS + e] = 0;
            st.exit_x[b * SL_MAX_EXITS + e] = 0;
        }
    }
}

// all kernel arguments of k_env_step_bits64 in one struct at kernarg offset 0, so a
// phase can re-read one late through kernarg() (write_obs)
struct StepKArgs {
    sl_env_state st;
    StepArgs a;
    FastExtra fx;
    const int32_t *actions;
    int ctp, ctc;
    double *reward_out;
    uint8_t *done_out, *flags_out;
    int32_t *ep_len_out, *ep_rew_out;
};

// the kernel's arguments through a pointer the compiler cannot see as invariant: a
// field read through it is loaded where it is used, not hoisted into the SGPRs that
// the whole kernel then has to keep
__device__ __forceinline__ const StepKArgs &kernarg() {
    auto kp = __builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(kp));
    return *(const StepKArgs *)kp;
}

// ---------------------------------------------------------------- fused observation
// SafeLifeEnv.get_obs + recenter_view (safelife_env.py:125-155, helper_utils.py:41-74)
// of the board the kernel holds on chip, packed (output_channels=None): the same
// values k_env_obs_packed (sl_env.hip) computes from HBM after the step.  A view
// cell is board + ((goals & COLORS) << 3) (white goals optionally removed), i.e. the
// goal colour planes added into planes 12-14.  Board bits 12-14 are unused by every
// cell type, so (wave-uniform check) the planes are overwritten with the goal colours
// and ONE transpose yields both the board rows (masked with ~0x7000 per cell for the
// HBM store) and the view-form rows, which go to the wave's LDS buffer in dma_board's
// layout; a board with any of those bits set takes a bit-sliced add and two more
// transposes instead.  Each view cell is then one u16 LDS read.  Envs reset after the
// step get their view written by the reset-list kernel after their reset.
__device__ __forceinline__ void lds_put_board(lds_u32 *buf, int lane, const u32 D[32]) {
    const int h = lane & 1, j = lane >> 1;
    lds_u32 *p = buf + h * 1024 + ((j + 16 * h) & 31);
#pragma unroll
    for (int y = 0; y < 32; y++) p[y * 32] = D[y];
}

__device__ __forceinline__ int lds_cell_idx(int row, int col) {
    return row * 64 + ((col + 32 * (row >> 5)) & 63);
}

typedef __attribute__((address_space(3))) uint16_t lds_u16;

// Per-half OR: bit y of the result is set when any lane of this lane's parity (rows
// 32 (lane & 1) + y) has it -- quad xor 2, then two row rotations keep the parity
__device__ __forceinline__ uint64_t changed_rows64(u32 cl) {
    u32 x = cl | dpp<0x4E>(cl);           // quad_perm [2,3,0,1]
    x |= dpp<0x124>(x);                   // row_ror:4
    x |= dpp<0x128>(x);                   // row_ror:8
    const u32 lo = (u32)__builtin_amdgcn_readlane((int)x, 0) | (u32)__builtin_amdgcn_readlane((int)x, 16) |
                   (u32)__builtin_amdgcn_readlane((int)x, 32) | (u32)__builtin_amdgcn_readlane((int)x, 48);
    const u32 hi = (u32)__builtin_amdgcn_readlane((int)x, 1) | (u32)__builtin_amdgcn_readlane((int)x, 17) |
                   (u32)__builtin_amdgcn_readlane((int)x, 33) | (u32)__builtin_amdgcn_readlane((int)x, 49);
    return ((uint64_t)hi << 32) | lo;
}

// The rows of M (bit r = row r) stored from the LDS board (lds_put_board's layout:
// chunk c of row r at chunk (c + 4 (r >> 5)) & 7), ANDed with `keep`: slot s = lane >> 3
// of each store instruction takes the s-th listed row, lane & 7 its 16-byte chunk.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store_rows(lds_u32 *buf, uint8_t *rowlist, u32 *gb0, uint64_t M,
                                           u32 keep, int lane) {
    typedef __attribute__((address_space(3))) uint8_t lds_u8;
    typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
    lds_u8 *rl = (lds_u8 *)rowlist;
    if ((M >> lane) & 1ull) rl[lanes_below(M)] = (uint8_t)lane;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const int n = __builtin_popcountll(M);
    const int c = lane & 7;
    for (int s = lane >> 3; s < n; s += 8) {
        const int row = rl[s];
        u32x4 v = *(const lds_u32x4 *)(buf + row * 32 + (((c + 4 * (row >> 5)) & 7) << 2));
        v &= keep;
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(gb0) + row * 8 + c);
    }
}

// exit y (R_EY) or x (R_EX) number e of the record, e = this lane's own index
__device__ __forceinline__ int lane_exit(const RecFields &fl, int e, int field) {
    const u32 w = (u32)__builtin_amdgcn_ds_bpermute(4 * (field + (e >> 1)), (int)fl.V);
    return (int)(int16_t)(w >> (16 * (e & 1)));
}

__device__ __forceinline__ void write_obs(lds_u32 *buf, const FastExtra &fx, const RecFields &fl,
                                          int64_t b, int lane) {
    lds_u16 *cells = reinterpret_cast<lds_u16 *>(buf);
    (void)fx;
    const FastExtra &lfx = kernarg().fx;     // read late: no SGPRs held through the step
    const int vh = lfx.obs_vh, vw = lfx.obs_vw;
    const int nv = vh * vw;
    const int ty = fl.ay - vh / 2, tx = fl.ax - vw / 2;
    // exits onto their clipped view positions: lane k < ne handles exit k (values read
    // before any is moved); the last in np.nonzero order wins a shared target
    const int ne = min(fl.exit_count(), SL_MAX_EXITS);
    int tgt = -1;
    u32 val = 0u;
    const int iy = lane_exit(fl, lane & 7, R_EY), ix = lane_exit(fl, lane & 7, R_EX);  // all lanes
    if (lane < ne) {
        int jy = ((iy - fl.ay + N / 2) & (N - 1)) - N / 2;
        int jx = ((ix - fl.ax + N / 2) & (N - 1)) - N / 2;
        jy = min(max(jy + vh / 2, 0), vh - 1);
        jx = min(max(jx + vw / 2, 0), vw - 1);
        tgt = jy * vw + jx;
        val = cells[lds_cell_idx(iy, ix)];
        // a view no larger than the board shows each board cell at most once: the
        // exits are moved in the LDS board itself and the gather needs no per-cell test
        tgt = lds_cell_idx((ty + jy) & (N - 1), (tx + jx) & (N - 1)) | (tgt << 12);
    }
    const bool small = vh <= N && vw <= N;
    if (small)
        for (int k = 0; k < ne; k++)            // one store instruction per exit, in order
            if (lane == k) cells[tgt & 4095] = (uint16_t)val;
    uint16_t *o = lfx.obs_out + b * (int64_t)nv;
    const int dr = 64 / vw, dc = 64 - dr * vw;
    if (small) {
        // two cells per store (global_store_dword, 4-B aligned in the whole obs array;
        // an env starting mid-dword stores its first cell alone, an odd remainder its
        // last): 9 store instructions per lane instead of 17 (+1 %, tools/ab/c3p_dword.py)
        const int s0 = (int)((b * (int64_t)nv) & 1);     // env starts mid-dword
        const int np = (nv - s0) >> 1;
        if (s0 && lane == 0) o[0] = cells[lds_cell_idx(ty & (N - 1), tx & (N - 1))];
        if (((nv - s0) & 1) && lane == 1)
            o[nv - 1] = cells[lds_cell_idx((ty + vh - 1) & (N - 1), (tx + vw - 1) & (N - 1))];
        uint32_t *o32 = reinterpret_cast<uint32_t *>(o + s0);
        const int c0 = s0 + 2 * lane;
        int rr = c0 / vw, cc = c0 - rr * vw;
        const int d2r = 128 / vw, d2c = 128 - d2r * vw;
        for (int p = lane; p < np; p += 64) {
            const int r1 = cc + 1 == vw ? rr + 1 : rr, c1 = cc + 1 == vw ? 0 : cc + 1;
            const uint32_t v0 = cells[lds_cell_idx((ty + rr) & (N - 1), (tx + cc) & (N - 1))];
            const uint32_t v1 = cells[lds_cell_idx((ty + r1) & (N - 1), (tx + c1) & (N - 1))];
            o32[p] = v0 | (v1 << 16);
            rr += d2r;
            cc += d2c;
            if (cc >= vw) {
                cc -= vw;
                rr++;
            }
        }
    } else {
        int r = lane / vw, c = lane - r * vw;
        for (int i = lane; i < nv; i += 64) {
            u32 v = cells[lds_cell_idx((ty + r) & (N - 1), (tx + c) & (N - 1))];
            for (int k = 0; k < ne; k++)
                if (i == (__builtin_amdgcn_readlane(tgt, k) >> 12))
                    v = (u32)__builtin_amdgcn_readlane((int)val, k);
            o[i] = (uint16_t)v;
            r += dr;
            c += dc;
            if (c >= vw) {
                c -= vw;
                r++;
            }
        }
    }
}

// Fused channel views (output_channels = a channel list: the reference's default
// 15 channels, safelife_env.py:79,150-154) of the view-form board in LDS (the same
// board write_obs reads, exits moved in place; views no larger than the board): each
// view cell's channel mask goes to the wave's mask array, then the env's output
// bytes leave as 16-byte chunks (obs_store_channels, sl_obs.h) -- no re-read of the
// state from HBM as the separate k_env_obs_channels needs.
template <int ESZ>
__device__ __forceinline__ void write_obs_channels(lds_u32 *buf, uint16_t *vm, const RecFields &fl,
                                                   int64_t b, int lane) {
    lds_u16 *cells = reinterpret_cast<lds_u16 *>(buf);
    const FastExtra &lfx = kernarg().fx;     // read late: no SGPRs held through the step
    const int vh = lfx.obs_vh, vw = lfx.obs_vw;
    const int nv = vh * vw;
    const int ty = fl.ay - vh / 2, tx = fl.ax - vw / 2;
    const int ne = min(fl.exit_count(), SL_MAX_EXITS);
    int tgt = -1;
    u32 val = 0u;
    const int iy = lane_exit(fl, lane & 7, R_EY), ix = lane_exit(fl, lane & 7, R_EX);
    if (lane < ne) {
        int jy = ((iy - fl.ay + N / 2) & (N - 1)) - N / 2;
        int jx = ((ix - fl.ax + N / 2) & (N - 1)) - N / 2;
        jy = min(max(jy + vh / 2, 0), vh - 1);
        jx = min(max(jx + vw / 2, 0), vw - 1);
        val = cells[lds_cell_idx(iy, ix)];
        tgt = lds_cell_idx((ty + jy) & (N - 1), (tx + jx) & (N - 1));
    }
    for (int k = 0; k < ne; k++)              // in np.nonzero order: the last one wins
        if (lane == k) cells[tgt] = (uint16_t)val;
    const sl::obs::ChanMap cm{lfx.obs_chpack, lfx.obs_nch};
    const bool id = cm.ident();
    const int dr = 64 / vw, dc = 64 - dr * vw;
    int r = lane / vw, c = lane - r * vw;
    for (int i = lane; i < nv; i += 64) {
        vm[i] = (uint16_t)cm.mask(cells[lds_cell_idx((ty + r) & (N - 1), (tx + c) & (N - 1))], id);
        r += dr;
        c += dc;
        if (c >= vw) {
            c -= vw;
            r++;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    sl::obs::obs_store_channels<ESZ>(vm, nv, cm.nch, lfx.obs_one, b, lane,
                                     reinterpret_cast<uint8_t *>(lfx.obs_out));
}

// the instantiations' view modes: 0 none, 1 packed, 2 channels of 2-byte elements (u16,
// bf16), 3 of 1-byte (u8), 4 of 4-byte (f32)
constexpr int obs_esz(int OBS) { return OBS == 3 ? 1 : (OBS == 4 ? 4 : 2); }

// What an env's step needs first, issued ahead: the per-env record (lane k = field k)
// and the goals' three colour planes from the mirror (speculative: used when the
// mirror is valid).  The board itself is DMA'd into the wave's LDS buffer.
struct Pre {
    u32 V;
    u32 g[3][2];
};

__device__ __forceinline__ void issue_pre(const sl_env_state &st, const int32_t *actions,
                                          int64_t b, int lane, Pre &p) {
    p.V = load_record(st, actions, b, lane);
    if (st.planes) {
        const u32 *mg = st.planes + b * 4096 + 2048 + lane;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            p.g[k][0] = mg[(9 + k) * 64];
            p.g[k][1] = mg[(25 + k) * 64];
        }
    }
}

// One env-step of env b.  `pre` holds b's record and goal colour planes and b's board
// is in flight into `buf` (issued by the caller).  MODE: SPAWN_PHILOX, or SPAWN_STREAM
// (replay: k_env_action has run the action and k_stream_prologue64 sized the draws; the step reads
// act[b] and each tensor's first uniform from the scratch words).
template <int OBS, int MODE>
__device__ __forceinline__ void step_env(const sl_env_state &st, const StepArgs &a,
                                         const FastExtra &fx, int64_t b, int lane, lds_u32 *buf,
                                         uint16_t *vm, uint8_t *rowlist,
                                         const int32_t *__restrict__ actions,
                                         int ctp, int ctc, double *reward_out, uint8_t *done_out,
                                         uint8_t *flags_out, int32_t *ep_len_out,
                                         int32_t *ep_rew_out, const Pre &pre) {
    constexpr bool VIEW = OBS != 0, CH = OBS >= 2;
    const int64_t off = b * (int64_t)(N * N);
    const int lane_off = (lane & 1) * 1024 + (lane >> 1);     // dwords: row 32h, column pair j
    u32 *gb = reinterpret_cast<u32 *>(st.board + off) + lane_off;
    u32 *gg = reinterpret_cast<u32 *>(st.goals + off) + lane_off;
    // bit-plane mirrors (sl_env_state.planes): read instead of u16 + transpose when valid
    // goals mirror, word-major: word q of lane l at planes[b*4096 + 2048 + q*64 + l]
    // (the goals rarely change, so it saves their transpose at almost no write cost;
    // a board mirror would be rewritten every step and does not pay)
    u32 *mg = st.planes ? st.planes + b * 4096 + 2048 + lane : nullptr;
    const u32 V = pre.V;
    // goals: a goals board without spawners that came through a step unchanged is at
    // a fixed point of the (then deterministic) rule and never changes again
    // (planes_ok bit 2); such envs read only the three colour planes of the mirror,
    // which are speculatively in flight before the record says which case holds
    u32 gcol[3][2];                    // goal colour planes, kept for the scores
#pragma unroll
    for (int k = 0; k < 3; k++) {
        gcol[k][0] = pre.g[k][0];
        gcol[k][1] = pre.g[k][1];
    }
    const int pok = (mg && st.planes_ok) ? rec(V, R_POK) & 6 : 0;

    SpawnCtx sc;
    sc.gid = a.env0 + (uint32_t)b;
    sc.step = a.step;
    sc.seed = a.seed;
    set_spawn_prob(sc, __int_as_float(rec(V, R_SPAWN)));
    StreamSrc ssrc{a.draws, a.n_draws, nullptr, a.draw_mask, a.draw_bits};
    int64_t pos_b = 0, pos_g = 0;
    if (MODE == SPAWN_STREAM) {
        const Scratch w = scratch_of(fx.scratch, st.B);
        ssrc.err = w.err;
        pos_b = w.offsets[2 * b];
        pos_g = w.offsets[2 * b + 1];
    }

    // ---- goals
    if ((pok & 6) != 6) {
        u32 PG[32];
        if (pok & 2) {
#pragma unroll
            for (int q = 0; q < 32; q++) PG[q] = mg[q * 64];    // goal planes
        } else {
            load_pairs_nt<32>(gg, PG);                              // goal cells
            transpose32(PG);
        }
        u32 cg[2];
        rule_planes(PG, cg, Geo64<MODE>{lane, ssrc, pos_g, 0}, sc, 1u);
        const u32 rg = wave_or(cg[0] | cg[1]);
        if (mg) {      // mirror: the words whose 32 cells changed (all of them if rebuilt)
            const bool all = !(pok & 2);
#pragma unroll
            for (int w = 0; w < 2; w++)
                if (all || cg[w])
#pragma unroll
                    for (int k = 0; k < 16; k++) mg[(k + 16 * w) * 64] = PL(PG, k, w);
            const bool fixed = rg == 0 && __ballot((PL(PG, 7, 0) | PL(PG, 7, 1)) != 0u) == 0ull;
            const int ok = 2 | (fixed ? 4 : 0);
            if (ok != pok && lane == 0) st.planes_ok[b] = ok;
        }
#pragma unroll
        for (int k = 0; k < 3; k++) {
            gcol[k][0] = PL(PG, 9 + k, 0);
            gcol[k][1] = PL(PG, 9 + k, 1);
        }
        if (rg) {
            transpose32(PG);
#pragma unroll
            for (int y = 0; y < 32; y++)
                if ((rg >> y) & 1u) __builtin_nontemporal_store(PG[y], &gg[y * 32]);
        }
    }
    __builtin_amdgcn_sched_barrier(0);

    // ---- board: from LDS; the start board comes from the level pool (cache) when
    // the env was reset from it, else from HBM through the same LDS buffer
    int roll = -1;
    if (fx.pool.K > 0 && fx.pool.board_planes && st.start_roll) roll = rec(V, R_ROLL);
    wait_vm();

    // the action (lane 0), on the staged board and the record
    OverlayT<LdsCells> ov;
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
        act_reward = (int)scratch_of(fx.scratch, st.B).act[b];
    } else {
        if (lane == 0) act_reward = act_core(env, rec(V, R_ACT), N, N, ctp, ctc, ov);
        act_reward = __builtin_amdgcn_readfirstlane(act_reward);
    }
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

    u32 PB[32];
    read_pairs(buf, lane, PB);
    wait_lgkm();
    if (roll < 0) dma_board(st.start_board + off, buf, lane);
    else pool_dma(fx.pool, rec(V, R_LI), buf, lane);
    transpose32(PB);
    const u32 erow = mux_edits(PB, ne, eidx, eval, lane);
    u32 cb[2];
    rule_planes(PB, cb, Geo64<MODE>{lane, ssrc, pos_b, 0}, sc, 0u);
    __builtin_amdgcn_sched_barrier(0);
    // fused views: board bits 12-14 are unused by every cell type, so (wave-uniform
    // check) the goal colours go into planes 12-14 now -- the scores read them there
    // and the goal planes die before the scoring -- and ONE transpose later yields
    // both the board rows and the view rows
    const bool hi = VIEW && __ballot((PL(PB, 12, 0) | PL(PB, 13, 0) | PL(PB, 14, 0) |
                                      PL(PB, 12, 1) | PL(PB, 13, 1) | PL(PB, 14, 1)) != 0u) != 0ull;
    if (VIEW && !hi) {
        const int obs_rw = kernarg().fx.obs_rw;
#pragma unroll
        for (int w = 0; w < 2; w++) {
            const u32 white = obs_rw ? (gcol[0][w] & gcol[1][w] & gcol[2][w]) : 0u;
#pragma unroll
            for (int k = 0; k < 3; k++) PL(PB, 12 + k, w) = gcol[k][w] & ~white;
        }
    }

    // ---- scores over the new board and goals
    u32 PS[32];
    wait_vm();
    if (roll >= 0) {
        pool_planes_lds(buf, roll >> 16, roll & 0xFFFF, lane, PS);
    } else {
        read_pairs(buf, lane, PS);
        transpose32(PS);
    }
    int pts, scr, pos, side;
    if (VIEW && !hi) score_planes<true>(PB, gcol, PS, &pts, &scr, &pos, &side);
    else score_planes(PB, gcol, PS, &pts, &scr, &pos, &side);
    // totals (packed two per word: per-lane ranges [-192, 320] and [-64, 64]);
    // reduced before the board store so the scoring is not sunk past it
    const int s1 = wave_total((pts + 192) | ((scr + 64) << 16));
    const int s2 = wave_total(pos | (side << 16));
    __builtin_amdgcn_sched_barrier(0);

    // ---- write back the changed rows of the board, exits already in the colour the
    // epilogue gives them (update_exit_colors), so its exit writes and these row
    // stores carry the same values and need no ordering
    const int points = (s1 & 0xFFFF) - 192 * 64;
    const int score = ((s1 >> 16) & 0xFFFF) - 64 * 64;
    const int possible = s2 & 0xFFFF;
    const int side_total = (s2 >> 16) & 0xFFFF;
    const u32 rb = wave_or(cb[0] | cb[1]) | erow;
    if (rb || VIEW) {
        const bool can = can_exit_now(fl.min_performance(), score, fl.baseline(), possible);
#pragma unroll
        for (int w = 0; w < 2; w++)
            PL(PB, 9, w) = can ? (PL(PB, 9, w) | PL(PB, 8, w)) : (PL(PB, 9, w) & ~PL(PB, 8, w));
        transpose32(PB);
        if (VIEW && !hi) {
            lds_put_board(buf, lane, PB);      // the start board in buf has been read out
            // the changed rows from the LDS board (which the views read anyway), 8 whole
            // rows per store; planes 12-14 hold the goal colours: the store masks them
            // out again.  (From registers a store writes rows y and 32 + y together:
            // same box, packed views 264.5 vs 258.9 M env-steps/s, tools/ab/c3_rowlist.py;
            // without views the LDS round trip costs more than the bytes it saves,
            // 344.6 vs 356.7 M, so that path keeps the register stores below.)
            if (rb) {
                uint64_t M = changed_rows64(cb[0] | cb[1]);
#pragma unroll
                for (int k = 0; k < 4; k++)
                    if (k < ne) M |= 1ull << (eidx[k] >> 6);
                store_rows(buf, rowlist, reinterpret_cast<u32 *>(st.board + off), M, 0x8FFF8FFFu,
                           lane);
            }
        } else if (rb) {
#pragma unroll
            for (int y = 0; y < 32; y++)
                if ((rb >> y) & 1u) __builtin_nontemporal_store(PB[y], &gb[y * 32]);
        }
    }
    if (VIEW && !hi) {
        __builtin_amdgcn_sched_barrier(0);
        if (CH) write_obs_channels<obs_esz(OBS)>(buf, vm, fl, b, lane);
        else write_obs(buf, fx, fl, b, lane);
        __builtin_amdgcn_sched_barrier(0);
    }
    int reset = 0;
    if (lane == 0)
        reset = epilogue_core(st, a, b, fl, act_reward, points, score, possible, side_total,
                              reward_out, done_out, flags_out, ep_len_out, ep_rew_out);
    reset = __builtin_amdgcn_readfirstlane(reset);
    if (VIEW && hi && !(fx.fuse_reset && reset)) {
        // a board using bits 12-14 (no cell type does): the view from the stored state
        // once everything has landed -- the action's writes, this step's goal and row
        // stores and the epilogue's exit cells (this wave's own stores) -- as
        // k_env_obs_packed computes it; an env reset after the step gets its view from
        // the reset-list kernel instead
        wait_vm();
        const FastExtra &lfx = kernarg().fx;
        sl::obs::ObsArgs oa{};
        oa.vh = lfx.obs_vh;
        oa.vw = lfx.obs_vw;
        oa.remove_white = lfx.obs_rw;
        oa.mode = lfx.obs_mode;
        oa.nch = lfx.obs_nch;
        if (CH)
            sl::obs::obs_channels_wave<obs_esz(OBS)>(
                st, oa, sl::obs::ChanMap{lfx.obs_chpack, lfx.obs_nch}, lfx.obs_one, b, lane, vm,
                reinterpret_cast<uint8_t *>(lfx.obs_out));
        else
            sl::obs::obs_packed_wave(st, oa, b, lane, lfx.obs_out);
    }
    if (fx.fuse_reset && reset && lane == 0) {
        // queue the env for the reset kernel (k_env_reset_list)
        int64_t *cnt = fx.scratch + 8 * st.B + 2 + (a.step & 1);
        const int i = (int)atomicAdd((unsigned long long *)cnt, 1ull);
        reset_list(fx.scratch)[i] = (int32_t)b;
    }
}

// OBS: also write the observation (fx.obs_out): 1 packed, 2-4 channel views
// (obs_esz); MODE: see step_env
template <int OBS, int MODE>
__global__ void __launch_bounds__(64, (OBS || MODE == SPAWN_STREAM) ? kMinWavesObs : kMinWaves)
k_env_step_bits64(StepKArgs ka) {
    const int64_t b = blockIdx.x;          // one wave per env
    const int lane = threadIdx.x;
    __shared__ __attribute__((aligned(16))) u32 stage[N * N / 2];
    // channel views: the view's channel masks (write_obs_channels)
    __shared__ __attribute__((aligned(16))) uint16_t vmask[OBS >= 2 ? sl::obs::kFusedChanCells : 2];
    __shared__ uint8_t rowlist[OBS ? 64 : 1];   // changed rows by rank (store_rows)
    lds_u32 *buf = (lds_u32 *)&stage[0];
    Pre pre;
    issue_pre(ka.st, ka.actions, b, lane, pre);
    dma_board(ka.st.board + b * (int64_t)(N * N), buf, lane);
    step_env<OBS, MODE>(ka.st, ka.a, ka.fx, b, lane, buf, vmask, rowlist, ka.actions, ka.ctp, ka.ctc,
                        ka.reward_out, ka.done_out, ka.flags_out, ka.ep_len_out, ka.ep_rew_out,
                        pre);
}

// ---------------------------------------------------------------- plane mode
// The 64x64 board kept in bit planes across steps (round 6; the 128x128 kernel's
// round-5 design, sl_bits128.hip): half 0 of the goals mirror (sl_env_state.planes:
// word q of lane l at planes[b*4096 + q*64 + l] = plane q & 15 of column 2 (l >> 1) +
// (q >> 4), rows 32 (l & 1) .. +31; half 1 keeps the goals).  A Philox step without
// views or capture (sl_env_state.board_planes == planes) DMA's the plane words into
// the wave's buffer at once -- as the uint16 board was -- runs the action on them, and
// stores only the words that changed; no transposes.  Planes in
// sl_env_state.board_zero (all zero in every board of the batch, for good: the C3 / C4
// pools never use cell bits 7 and 11-14) are neither loaded nor stored, and the kept
// ones are packed (PlaneSlots): 6 of the 8 KiB are read.  planes_ok bit 6: the planes hold the board; bit 7: so does the uint16
// board (a sync, or a reset, wrote it), which a plane step otherwise leaves stale
// (exits aside: the epilogue writes them in both).
constexpr int kPok64Board = 64, kPok64Full = 128;

// The planes outside `zero` packed word after word: word q (plane q & 15 of column
// word q >> 4) at position pos(q), the number of kept words below it, so the kept words
// come first and one DMA instruction of 16 B per lane moves four of them (C3: 22 of 32
// words in 6 instructions, where 4-B DMAs word by word took 22 and ran 12 % slower).
// The layout follows sl_env_state.board_zero, which changes only after every board has
// left the planes.
template <u32 K16>       // the kept planes, fixed at compile time; 0: from board_zero
struct PlaneSlots {
    u32 keep;           // bit q: word q is kept (K16 == 0)
    __device__ __forceinline__ u32 keep32() const { return K16 ? K16 * 0x10001u : keep; }
    __device__ __forceinline__ bool kept(int q) const { return (keep32() >> q) & 1u; }
    // (at run time recomputed where used: two SALU, not 32 positions held in SGPRs all
    // kernel long; with K16 a constant)
    __device__ __forceinline__ int pos(int q) const {
        if (K16) return __builtin_popcount((K16 * 0x10001u) & ((1u << q) - 1u));
        u32 k = keep;
        asm volatile("" : "+s"(k));
        return __builtin_popcount(k & ((1u << q) - 1u));
    }
    __device__ __forceinline__ int kept16() const { return __builtin_popcount(keep32() & 0xFFFFu); }
    static __device__ __forceinline__ PlaneSlots of(u32 zero) {
        return PlaneSlots{(~zero & 0xFFFFu) * 0x10001u};
    }
};
// the instantiations: every plane, the C3 / C4 pools' planes (cell bits 0-6, 8-10, 15),
// and any other mask at run time
constexpr u32 kKeepAll = 0xFFFFu, kKeepC3 = 0x877Fu;

// the kept plane words of an env, DMA'd into the wave's buffer in their packed order
// (position p of lane l at buf[p * 64 + l]); no registers held while they are in flight
template <u32 K16>
__device__ __forceinline__ void dma_planes(const u32 *__restrict__ bp, PlaneSlots<K16> ps,
                                           lds_u32 *buf, int lane) {
    const int groups = (2 * ps.kept16() + 3) >> 2;
    const char *s = reinterpret_cast<const char *>(bp);
#pragma unroll
    for (int g = 0; g < 8; g++)
        if (g < groups)
            __builtin_amdgcn_global_load_lds((const void *)(s + g * 1024 + lane * 16),
                                             (__attribute__((address_space(3))) void *)(buf + g * 256),
                                             16, 0, 2);
}

// The cells act_core can read around (y0, x0) -- the row within +-2 columns, the
// column within +-2 rows: near_cell_index(k) -- gathered from the staged planes by
// lanes 0..8 at once (16 LDS reads for the wave, not 16 per cell on the action's lane),
// then read by the lane-0 action with v_readlane (whatever the exec mask)
__device__ __forceinline__ int near_cell_index(int k, int y0, int x0) {
    const int dy = k < 5 ? 0 : (k == 5 ? -1 : k == 6 ? 1 : k == 7 ? -2 : 2);
    const int dx = k >= 5 || k == 0 ? 0 : (k == 1 ? -1 : k == 2 ? 1 : k == 3 ? -2 : 2);
    return ((y0 + dy) & 63) * 64 + ((x0 + dx) & 63);
}
struct NearCells {
    int y0, x0;
    u32 v;              // lane k: cell near_cell_index(k)
    __device__ __forceinline__ uint32_t operator()(int i) const {
        const int dy = (((i >> 6) - y0 + 32) & 63) - 32, dx = (((i & 63) - x0 + 32) & 63) - 32;
        const int k = dy == 0 ? (dx == 0 ? 0 : dx == -1 ? 1 : dx == 1 ? 2 : dx == -2 ? 3 : 4)
                              : (dy == -1 ? 5 : dy == 1 ? 6 : dy == -2 ? 7 : 8);
        return (u32)__builtin_amdgcn_readlane((int)v, __builtin_amdgcn_readfirstlane(k));
    }
};
// cell i from the staged planes (this lane's; planes not kept are 0)
template <u32 K16>
__device__ __forceinline__ u32 lds_plane_cell(const lds_u32 *buf, PlaneSlots<K16> ps, int i) {
    const int y = i >> 6, x = i & 63;
    const lds_u32 *q = buf + 2 * (x >> 1) + (y >> 5);
    const u32 r = (u32)(y & 31);
    const int w = 16 * (x & 1);
    u32 v = 0;
#pragma unroll
    for (int p = 0; p < 16; p++) {
        const int pw = ps.pos(p) + (w ? ps.kept16() : 0);
        if (ps.kept(p)) v |= ((q[pw * 64] >> r) & 1u) << p;
    }
    return v;
}

// OBS: 1 also writes the packed views (write_obs) from the step's planes: the goal
// colours added into planes 12-14 (a bit-sliced adder, exact whatever the board's bits),
// ONE transpose, the view-form rows into the buffer
template <u32 K16, int OBS>
__global__ void __launch_bounds__(64, kMinWaves)
k_env_step_bits64_planes(StepKArgs ka) {
    const sl_env_state &st = ka.st;
    const StepArgs &a = ka.a;
    const FastExtra &fx = ka.fx;
    const int64_t b = blockIdx.x;          // one wave per env
    const int lane = threadIdx.x;
    __shared__ __attribute__((aligned(16))) u32 stage[N * N / 2];
    lds_u32 *buf = (lds_u32 *)&stage[0];
    const PlaneSlots<K16> ps = PlaneSlots<K16>::of(st.board_zero);
    Pre pre;
    issue_pre(st, ka.actions, b, lane, pre);
    // the board's planes, speculatively: an env whose planes do not hold its board (the
    // first step after a host write or a step in another mode) reloads its rows below
    dma_planes(st.planes + b * 4096, ps, buf, lane);
    const int64_t off = b * (int64_t)(N * N);
    const int lane_off = (lane & 1) * 1024 + (lane >> 1);     // dwords: row 32h, column pair j
    u32 *gg = reinterpret_cast<u32 *>(st.goals + off) + lane_off;
    u32 *mg = st.planes + b * 4096 + 2048 + lane;
    u32 *bp = st.planes + b * 4096 + lane;
    const u32 V = pre.V;
    const int pok_all = rec(V, R_POK);
    const bool pin = (pok_all & kPok64Board) != 0;
    u32 gcol[3][2];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        gcol[k][0] = pre.g[k][0];
        gcol[k][1] = pre.g[k][1];
    }
    const int pok = pok_all & 6;
    int gok = pok;                 // the goals' planes_ok bits after this step

    SpawnCtx sc;
    sc.gid = a.env0 + (uint32_t)b;
    sc.step = a.step;
    sc.seed = a.seed;
    set_spawn_prob(sc, __int_as_float(rec(V, R_SPAWN)));
    const StreamSrc ssrc{a.draws, a.n_draws, nullptr, a.draw_mask, a.draw_bits};

    // ---- goals (as in step_env: the mirror in half 1, the fixed-point skip)
    if ((pok & 6) != 6) {
        u32 PG[32];
        if (pok & 2) {
#pragma unroll
            for (int q = 0; q < 32; q++) PG[q] = mg[q * 64];
        } else {
            load_pairs_nt<32>(gg, PG);
            transpose32(PG);
        }
        u32 cg[2];
        rule_planes(PG, cg, Geo64<SPAWN_PHILOX>{lane, ssrc, 0, 0}, sc, 1u);
        const u32 rg = wave_or(cg[0] | cg[1]);
        const bool all = !(pok & 2);
#pragma unroll
        for (int w = 0; w < 2; w++)
            if (all || cg[w])
#pragma unroll
                for (int k = 0; k < 16; k++) mg[(k + 16 * w) * 64] = PL(PG, k, w);
        const bool fixed = rg == 0 && __ballot((PL(PG, 7, 0) | PL(PG, 7, 1)) != 0u) == 0ull;
        gok = 2 | (fixed ? 4 : 0);
#pragma unroll
        for (int k = 0; k < 3; k++) {
            gcol[k][0] = PL(PG, 9 + k, 0);
            gcol[k][1] = PL(PG, 9 + k, 1);
        }
        if (rg) {
            transpose32(PG);
#pragma unroll
            for (int y = 0; y < 32; y++)
                if ((rg >> y) & 1u) __builtin_nontemporal_store(PG[y], &gg[y * 32]);
        }
    }
    __builtin_amdgcn_sched_barrier(0);

    int roll = -1;
    if (fx.pool.K > 0 && fx.pool.board_planes && st.start_roll) roll = rec(V, R_ROLL);
    wait_vm();
    if (!pin) {
        // a step into plane mode: the uint16 board instead, transposed and put into the
        // buffer in the planes' layout, so everything below reads planes
        dma_board(st.board + off, buf, lane);
        wait_vm();
        u32 R[32];
        read_pairs(buf, lane, R);
        transpose32(R);
#pragma unroll
        for (int q = 0; q < 32; q++)
            if (ps.kept(q)) buf[ps.pos(q) * 64 + lane] = R[q];
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    // the action (lane 0) on the cells round the agent, gathered from the staged planes
    RecEnv env{st, b, rec(V, R_GO), rec(V, R_AX), rec(V, R_AY), rec(V, R_SCORE),
               rec(V, R_BASE), rec(V, R_POSS), rec_f64(V, R_MP)};
    int act_reward = 0;
    int eidx[4];
    u32 eval[4];
    const int ay0 = rec(V, R_AY), ax0 = rec(V, R_AX);
    const u32 near = lane < 9 ? lds_plane_cell(buf, ps, near_cell_index(lane, ay0, ax0)) : 0u;
    OverlayT<NearCells> ov;
    ov.src = NearCells{ay0, ax0, near};
    ov.n = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        ov.idx[k] = 0;
        ov.val[k] = 0;
    }
    if (lane == 0) act_reward = act_core(env, rec(V, R_ACT), N, N, ka.ctp, ka.ctc, ov);
    int ne = ov.n;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        eidx[k] = ov.idx[k];
        eval[k] = ov.val[k];
    }
    act_reward = __builtin_amdgcn_readfirstlane(act_reward);
    ne = __builtin_amdgcn_readfirstlane(ne);
#pragma unroll
    for (int k = 0; k < 4; k++) {
        eidx[k] = __builtin_amdgcn_readfirstlane(eidx[k]);
        eval[k] = (u32)__builtin_amdgcn_readfirstlane((int)eval[k]);
    }
    RecFields fl{V, __builtin_amdgcn_readfirstlane(env.go), __builtin_amdgcn_readfirstlane(env.ax),
                 __builtin_amdgcn_readfirstlane(env.ay), 0.0};
    if (a.bonus_period > 0)        // issued now, consumed by the epilogue
        fl.bval = a.bonus_table[bonus_dist(fl.ax, fl.ay, fl.prior_x(fl.prior_head()),
                                           fl.prior_y(fl.prior_head()), fl.prior_len(),
                                           a.bonus_period, a.bonus_len)];

    u32 PB[32];
#pragma unroll
    for (int q = 0; q < 32; q++) PB[q] = ps.kept(q) ? buf[ps.pos(q) * 64 + lane] : 0u;
    wait_lgkm();
    constexpr u32 KEEP = K16 ? K16 : 0xFFFFu;
    if (roll < 0) dma_board(st.start_board + off, buf, lane);
    else pool_dma<KEEP>(fx.pool, rec(V, R_LI), buf, lane);
    (void)mux_edits(PB, ne, eidx, eval, lane);
    // held: changed cells that held a plane a change clears but never sets
    u32 cb[2], held[2];
    rule_planes(PB, cb, Geo64<SPAWN_PHILOX>{lane, ssrc, 0, 0}, sc, 0u, held);
    // (a lane mask, not two words held through the scores: such a lane stores those
    // planes for every changed word)
    const uint64_t held_lanes = __ballot((held[0] | held[1]) != 0u);
    __builtin_amdgcn_sched_barrier(0);

    // ---- scores over the new board and goals
    u32 PS[32];
    wait_vm();
    if (roll >= 0) {
        pool_planes_lds<KEEP>(buf, roll >> 16, roll & 0xFFFF, lane, PS);
    } else {
        read_pairs(buf, lane, PS);
        transpose32(PS);
    }
    int pts, scr, pos, side;
    score_planes(PB, gcol, PS, &pts, &scr, &pos, &side);
    const int s1 = wave_total((pts + 192) | ((scr + 64) << 16));
    const int s2 = wave_total(pos | (side << 16));
    __builtin_amdgcn_sched_barrier(0);
    const int points = (s1 & 0xFFFF) - 192 * 64;
    const int score = ((s1 >> 16) & 0xFFFF) - 64 * 64;
    const int possible = s2 & 0xFFFF;
    const int side_total = (s2 >> 16) & 0xFFFF;

    // ---- exits in the colour the epilogue gives them (update_exit_colors), then the
    // plane words that changed (all of them on a step into plane mode)
    const bool can = can_exit_now(fl.min_performance(), score, fl.baseline(), possible);
    u32 d9[2];
#pragma unroll
    for (int w = 0; w < 2; w++) {
        const u32 o9 = PL(PB, 9, w);
        PL(PB, 9, w) = can ? (o9 | PL(PB, 8, w)) : (o9 & ~PL(PB, 8, w));
        d9[w] = o9 ^ PL(PB, 9, w);
    }
    u32 em[2] = {0u, 0u};           // the words the action's edits touched (this lane's)
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (k < ne) {
            const int y = eidx[k] >> 6, x = eidx[k] & 63;
            const u32 bit = lane == 2 * (x >> 1) + (y >> 5) ? 1u << (y & 31) : 0u;
            em[x & 1] |= bit;
        }
    }
    u32 dw[2], dall[2];
#pragma unroll
    for (int w = 0; w < 2; w++) {
        dw[w] = cb[w] | em[w];                       // words whose cells changed
        dall[w] = em[w] | (((held_lanes >> lane) & 1ull) ? cb[w] : 0u);   // ... other planes
    }
    if (!pin || wave_or(dw[0] | dw[1] | d9[0] | d9[1])) {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            if (!ps.kept(k)) continue;
#pragma unroll
            for (int w = 0; w < 2; w++) {
                const u32 d = (k == 0 || k == 3 || k == 10 || k == 11) ? dw[w]
                              : k == 9 ? (dw[w] | d9[w]) : dall[w];
                if (!pin || d)
                    __builtin_nontemporal_store(PL(PB, k, w), &bp[ps.pos(k + 16 * w) * 64]);
            }
        }
    }
    const int ok = gok | kPok64Board;
    if (ok != pok_all && lane == 0) st.planes_ok[b] = ok;
    if (OBS) {
        const bool rw = kernarg().fx.obs_rw != 0;
#pragma unroll
        for (int w = 0; w < 2; w++) {
            u32 g0 = gcol[0][w], g1 = gcol[1][w], g2 = gcol[2][w];
            if (rw) {                                // white goals are background
                const u32 wh = g0 & g1 & g2;
                g0 &= ~wh;
                g1 &= ~wh;
                g2 &= ~wh;
            }
            const u32 b12 = PL(PB, 12, w), b13 = PL(PB, 13, w), b14 = PL(PB, 14, w);
            u32 c = b12 & g0;
            PL(PB, 12, w) = b12 ^ g0;
            const u32 x13 = b13 ^ g1;
            PL(PB, 13, w) = x13 ^ c;
            c = (b13 & g1) | (c & x13);
            const u32 x14 = b14 ^ g2;
            PL(PB, 14, w) = x14 ^ c;
            c = (b14 & g2) | (c & x14);
            PL(PB, 15, w) ^= c;                      // (the carry out of bit 15 drops)
        }
        transpose32(PB);
        lds_put_board(buf, lane, PB);               // (the start planes have been read)
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_sched_barrier(0);
        write_obs(buf, fx, fl, b, lane);
        __builtin_amdgcn_sched_barrier(0);
    }
    int reset = 0;
    if (lane == 0)
        reset = epilogue_core(st, a, b, fl, act_reward, points, score, possible, side_total,
                              ka.reward_out, ka.done_out, ka.flags_out, ka.ep_len_out,
                              ka.ep_rew_out);
    reset = __builtin_amdgcn_readfirstlane(reset);
    if (fx.fuse_reset && reset && lane == 0) {
        int64_t *cnt = fx.scratch + 8 * st.B + 2 + (a.step & 1);
        const int i = (int)atomicAdd((unsigned long long *)cnt, 1ull);
        reset_list(fx.scratch)[i] = (int32_t)b;
    }
}

// sl_env_board_sync for 64x64 boards in planes: one wave per env
__global__ void __launch_bounds__(64) k_board_sync64(sl_env_state st, int demote) {
    const int64_t b = blockIdx.x;
    const int lane = threadIdx.x;
    const int pok = __builtin_amdgcn_readfirstlane(st.planes_ok[b]);
    if (!(pok & kPok64Board)) return;
    if (!(pok & kPok64Full)) {
        const PlaneSlots<0> ps = PlaneSlots<0>::of(st.board_zero);
        const u32 *bp = st.planes + b * 4096 + lane;
        u32 P[32];
#pragma unroll
        for (int q = 0; q < 32; q++) P[q] = ps.kept(q) ? bp[ps.pos(q) * 64] : 0u;
        transpose32(P);
        u32 *gb = reinterpret_cast<u32 *>(st.board + b * (int64_t)(N * N)) + (lane & 1) * 1024 +
                  (lane >> 1);
#pragma unroll
        for (int y = 0; y < 32; y++) gb[y * 32] = P[y];
    }
    if (lane == 0)
        st.planes_ok[b] = demote ? pok & ~(kPok64Board | kPok64Full) : pok | kPok64Full;
}

// Replay-mode count of env b (SL_RNG_STREAM), one wave, after k_env_action (one lane
// per env) has applied the actions -- state and cell edits in HBM, rewards in scratch
// act[] -- so the board read here is the acted-on one: the eligible cells, i.e. the
// uniforms the step will draw, of the board and of the goals (scratch counts[2b],
// [2b+1]; sl_exclusive_scan_i64 turns them into each tensor's first uniform).  The work
// of k_env_count (sl_env.hip) on the bit-sliced rule.  (The action ran on lane 0 of
// this wave before: one wave per env for a one-lane latency chain made this launch
// cost as much as a quarter of the step on boards without spawners.)
__global__ void __launch_bounds__(64)
k_stream_prologue64(StepKArgs ka) {
    const sl_env_state &st = ka.st;
    const int64_t b = blockIdx.x;
    const int lane = threadIdx.x;
    const int64_t off = b * (int64_t)(N * N);
    const int lane_off = (lane & 1) * 1024 + (lane >> 1);
    const u32 V = load_record(st, ka.actions, b, lane);
    const Scratch w = scratch_of(ka.fx.scratch, st.B);
    // a board or goals without spawners (spawn_flags, set at reset: no rule or action
    // creates one) draws nothing: its count is 0 without a read
    const int spf = rec(V, R_SPF) | (ka.ctp ? 1 : 0);     // toggling powers can make one
    SpawnCtx sc{0u, 0u, 0ull, 0.0};
    u32 P[32], ch[2];
    int nb = 0;
    if (spf & 1) {
        load_pairs_nt<32>(reinterpret_cast<const u32 *>(st.board + off) + lane_off, P);
        transpose32(P);
        Geo64<SPAWN_COUNT> gbd{lane, StreamSrc{nullptr, 0, nullptr}, 0, 0};
        rule_planes(P, ch, gbd, sc, 0u);
        nb = wave_total(gbd.count);
    }
    // goals at their fixed point (planes_ok bit 2) hold no spawner: no draws
    const int pok = (st.planes && st.planes_ok) ? rec(V, R_POK) & 6 : 0;
    int ng = 0;
    if ((pok & 6) != 6 && (spf & 2)) {
        if (pok & 2) {
            const u32 *mg = st.planes + b * 4096 + 2048 + lane;
#pragma unroll
            for (int q = 0; q < 32; q++) P[q] = mg[q * 64];
        } else {
            load_pairs_nt<32>(reinterpret_cast<const u32 *>(st.goals + off) + lane_off, P);
            transpose32(P);
        }
        Geo64<SPAWN_COUNT> ggl{lane, StreamSrc{nullptr, 0, nullptr}, 0, 0};
        rule_planes(P, ch, ggl, sc, 1u);
        ng = wave_total(ggl.count);
    }
    if (lane == 0) {
        w.counts[2 * b] = nb;
        w.counts[2 * b + 1] = ng;
    }
}

// Resets the envs the step kernel queued (one wave per env, grid-stride over the
// list).  Also zeroes the other step parity's list length for the next step.
// With obs_out, each reset env's packed view is then written from the new episode
// (the step kernel wrote the views of all other envs).
__global__ void __launch_bounds__(64)
k_env_reset_list(sl_env_state st, sl_level_pool pool, ResetArgs ra, int64_t *scratch,
                 uint32_t step, sl::obs::ObsArgs oa, uint64_t chpack, uint32_t one,
                 uint16_t *obs_out) {
    // channel views of the reset envs: their masks
    __shared__ __attribute__((aligned(16))) uint16_t vmask[sl::obs::kFusedChanCells];
    int64_t *cnt = scratch + 8 * st.B + 2;
    if (blockIdx.x == 0 && threadIdx.x == 0) cnt[(step + 1) & 1] = 0;
    const int32_t *list = reset_list(scratch);
    // the first entry is loaded together with the length (grid <= B <= list size; the
    // value is used only when the entry is in the list)
    const int first = list[blockIdx.x];
    const int n = (int)__builtin_amdgcn_readfirstlane((int)cnt[step & 1]);
    for (int i = blockIdx.x; i < n; i += gridDim.x) {
        const int64_t b = __builtin_amdgcn_readfirstlane(i == (int)blockIdx.x ? first : list[i]);
        wave_reset(st, pool, ra, b, threadIdx.x);
        if (obs_out) {
            wait_vm();      // the reset's stores have landed (no stale lines: this wave
                            // alone touches env b, and L1 starts clean each launch)
            const sl::obs::ChanMap cm{chpack, oa.nch};
            uint8_t *o8 = reinterpret_cast<uint8_t *>(obs_out);
            if (oa.mode == SL_OBS_PACKED)
                sl::obs::obs_packed_wave(st, oa, b, threadIdx.x, obs_out);
            else if (oa.mode == SL_OBS_CHANNELS_U8)
                sl::obs::obs_channels_wave<1>(st, oa, cm, one, b, threadIdx.x, vmask, o8);
            else if (oa.mode == SL_OBS_CHANNELS_F32)
                sl::obs::obs_channels_wave<4>(st, oa, cm, one, b, threadIdx.x, vmask, o8);
            else
                sl::obs::obs_channels_wave<2>(st, oa, cm, one, b, threadIdx.x, vmask, o8);
        }
    }
}

// the step kernel's view mode for fx (k_env_step_bits64's OBS)
int obs_kind(const FastExtra &fx) {
    if (!fx.obs_out) return 0;
    switch (fx.obs_mode) {
    case SL_OBS_PACKED: return 1;
    case SL_OBS_CHANNELS_U8: return 3;
    case SL_OBS_CHANNELS_F32: return 4;
    default: return 2;               // u16 and bf16 channels
    }
}

template <int MODE>
void launch_bits64(int kind, unsigned grid, const StepKArgs &ka, hipStream_t s) {
    switch (kind) {
    case 0: hipLaunchKernelGGL((k_env_step_bits64<0, MODE>), dim3(grid), dim3(64), 0, s, ka); break;
    case 1: hipLaunchKernelGGL((k_env_step_bits64<1, MODE>), dim3(grid), dim3(64), 0, s, ka); break;
    case 2: hipLaunchKernelGGL((k_env_step_bits64<2, MODE>), dim3(grid), dim3(64), 0, s, ka); break;
    case 3: hipLaunchKernelGGL((k_env_step_bits64<3, MODE>), dim3(grid), dim3(64), 0, s, ka); break;
    default: hipLaunchKernelGGL((k_env_step_bits64<4, MODE>), dim3(grid), dim3(64), 0, s, ka); break;
    }
}

}  // namespace

namespace sl {

bool planes64_shape(const sl_env_state &st) {
    return st.H == N && st.W == N && st.planes && st.planes_ok && st.board_planes == st.planes;
}

int sync_board_planes64(const sl_env_state &st, int demote, hipStream_t s) {
    if (!planes64_shape(st) || st.B <= 0) return SL_OK;
    hipLaunchKernelGGL(k_board_sync64, dim3((unsigned)st.B), dim3(64), 0, s, st, demote);
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}

int launch_step_bits(const sl_env_state &st, const StepArgs &a, const FastExtra &fx,
                     const int32_t *actions, int ctp, int ctc, double *reward, uint8_t *done,
                     uint8_t *flags, int32_t *ep_len, int32_t *ep_rew, hipStream_t s) {
    if (st.H != N || st.W != N) return SL_ETOOBIG;
    const unsigned grid = (unsigned)st.B;
    const StepKArgs ka{st, a, fx, actions, ctp, ctc, reward, done, flags, ep_len, ep_rew};
    if (fx.obs_out && (fx.obs_vh < 1 || fx.obs_vw < 1 || fx.obs_vh * fx.obs_vw > 4096))
        return SL_EINVAL;
    if (fx.stream) {
        if (stream_counts(fx)) {
            const int rca = launch_env_action(st, actions, ctp, ctc, scratch_of(fx.scratch, st.B).act, s);
            if (rca) return rca;
            hipLaunchKernelGGL(k_stream_prologue64, dim3(grid), dim3(64), 0, s, ka);
            if (hipGetLastError() != hipSuccess) return SL_EHIP;
        }
        const int rc = stream_offsets(st, fx, s);
        if (rc || !stream_steps(fx)) return rc;
        if (fx.ev_begin) (void)hipEventRecord((hipEvent_t)fx.ev_begin, s);
        launch_bits64<SPAWN_STREAM>(obs_kind(fx), grid, ka, s);
    } else {
        if (fx.ev_begin) (void)hipEventRecord((hipEvent_t)fx.ev_begin, s);
        if (fx.plane_mode) {
            const u32 keep = ~st.board_zero & 0xFFFFu;
            if (fx.obs_out) {
                if (keep == kKeepC3)
                    hipLaunchKernelGGL((k_env_step_bits64_planes<kKeepC3, 1>), dim3(grid), dim3(64), 0, s, ka);
                else if (keep == kKeepAll)
                    hipLaunchKernelGGL((k_env_step_bits64_planes<kKeepAll, 1>), dim3(grid), dim3(64), 0, s, ka);
                else
                    hipLaunchKernelGGL((k_env_step_bits64_planes<0, 1>), dim3(grid), dim3(64), 0, s, ka);
            } else if (keep == kKeepC3) {
                hipLaunchKernelGGL((k_env_step_bits64_planes<kKeepC3, 0>), dim3(grid), dim3(64), 0, s, ka);
            } else if (keep == kKeepAll) {
                hipLaunchKernelGGL((k_env_step_bits64_planes<kKeepAll, 0>), dim3(grid), dim3(64), 0, s, ka);
            } else {
                hipLaunchKernelGGL((k_env_step_bits64_planes<0, 0>), dim3(grid), dim3(64), 0, s, ka);
            }
        }
        else
            launch_bits64<SPAWN_PHILOX>(obs_kind(fx), grid, ka, s);
    }
    if (hipGetLastError() != hipSuccess) return SL_EHIP;
    if (fx.ev_end) (void)hipEventRecord((hipEvent_t)fx.ev_end, s);
    if (fx.capture) {          // the frame before this step's resets
        const int rc = launch_capture(st, *fx.capture, flags, 0, s);
        if (rc) return rc;
    }
    if (fx.fuse_reset && fx.pool.K > 0) {
        const unsigned grid = (unsigned)(st.B < 512 ? st.B : 512);
        sl::obs::ObsArgs oa{};
        oa.vh = fx.obs_vh;
        oa.vw = fx.obs_vw;
        oa.remove_white = fx.obs_rw;
        oa.mode = fx.obs_mode;
        oa.nch = fx.obs_nch;
        hipLaunchKernelGGL(k_env_reset_list, dim3(grid), dim3(64), 0, s, st, fx.pool, fx.ra,
                           fx.scratch, a.step, oa, fx.obs_chpack, fx.obs_one, fx.obs_out);
    }
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}

}  // namespace sl
