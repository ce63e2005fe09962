// sl_obs.h -- observation building blocks shared by the observation kernels
// (sl_env.hip) and the 64x64 reset-list kernel (sl_bits.hip): SafeLifeEnv.get_obs
// (safelife_env.py:125-155) + recenter_view (helper_utils.py:41-74) of one env by one
// wave.
#pragma once
#include "sl_env_common.h"

namespace sl {
namespace obs {

struct ObsArgs {
    int vh, vw, remove_white, mode, nch;
    int ch[16];
};

__device__ __forceinline__ uint16_t obs_value(uint32_t bv, uint32_t gv, int remove_white) {
    uint32_t g = gv & COLORS;
    if (remove_white && g == COLORS) g = 0;
    return (uint16_t)((bv + (g << 3)) & 0xFFFFu);
}

// ---- wave-per-env observation kernels ---------------------------------------
// One wave per env, four per workgroup, no block barrier.  Lane l handles the view
// cells i = l + 64k (flat row-major order).  The cells' board and goals loads are
// issued eight at a time, all independent, so a wave keeps 16 gathers in flight.
// Exits are moved onto their clipped position on the view (recenter_view,
// helper_utils.py:55-72); the targets and values are wave-uniform and computed up
// front; the last exit in np.nonzero order wins a shared target.
constexpr int kObsGroup = 8;
constexpr int kObsMaxCells = 4096;        // view cells handled by the wave kernels
constexpr int kFusedChanCells = 1096;     // view cells + 2 the 64x64 step kernel's channel
                                          // views take (33 x 33 = 1 089)

struct ObsWave {
    const uint16_t *gb, *gg;
    int ty, tx, ne;
    int tgt[SL_MAX_EXITS];
    uint32_t val[SL_MAX_EXITS];
};

__device__ __forceinline__ void obs_wave_init(const sl_env_state &st, const ObsArgs &a, int64_t b,
                                              ObsWave &w) {
    const int H = st.H, W = st.W;
    const int64_t hw = (int64_t)H * W;
    w.gb = st.board + b * hw;
    w.gg = st.goals + b * hw;
    const int y0 = st.agent_y[b], x0 = st.agent_x[b];
    w.ty = y0 - a.vh / 2;
    w.tx = x0 - a.vw / 2;
    w.ne = min(st.exit_count[b], SL_MAX_EXITS);
#pragma unroll
    for (int k = 0; k < SL_MAX_EXITS; k++) {
        w.tgt[k] = -1;
        w.val[k] = 0;
        if (k < w.ne) {
            const int iy = st.exit_y[b * SL_MAX_EXITS + k], ix = st.exit_x[b * SL_MAX_EXITS + k];
            int jy = pymod(iy - y0 + H / 2, H) - H / 2;
            int jx = pymod(ix - x0 + W / 2, W) - W / 2;
            jy = min(max(jy + a.vh / 2, 0), a.vh - 1);
            jx = min(max(jx + a.vw / 2, 0), a.vw - 1);
            w.tgt[k] = jy * a.vw + jx;
            w.val[k] = obs_value(w.gb[iy * W + ix], w.gg[iy * W + ix], a.remove_white);
        }
    }
}

// values of the cells i = i0 + 64g (g < kObsGroup); (r, c) = position of i0, advanced
template <class F>
__device__ __forceinline__ void obs_wave_cells(const sl_env_state &st, const ObsArgs &a,
                                               const ObsWave &w, int nv, int &i0, int &r, int &c,
                                               F &&emit) {
    const int dr = 64 / a.vw, dc = 64 - dr * a.vw;
    uint32_t bv[kObsGroup], gv[kObsGroup];
#pragma unroll
    for (int g = 0; g < kObsGroup; g++) {
        bv[g] = 0;
        gv[g] = 0;
        if (i0 + 64 * g < nv) {
            const int src = pymod(w.ty + r, st.H) * st.W + pymod(w.tx + c, st.W);
            bv[g] = w.gb[src];
            gv[g] = w.gg[src];
        }
        r += dr;
        c += dc;
        if (c >= a.vw) {
            c -= a.vw;
            r++;
        }
    }
#pragma unroll
    for (int g = 0; g < kObsGroup; g++) {
        const int i = i0 + 64 * g;
        if (i < nv) {
            uint32_t v = obs_value(bv[g], gv[g], a.remove_white);
#pragma unroll
            for (int k = 0; k < SL_MAX_EXITS; k++)
                if (k < w.ne && i == w.tgt[k]) v = w.val[k];
            emit(i, v);
        }
    }
    i0 += 64 * kObsGroup;
}

__device__ __forceinline__ void obs_packed_wave(const sl_env_state &st, const ObsArgs &a,
                                                int64_t b, int lane, uint16_t *__restrict__ out) {
    ObsWave w;
    obs_wave_init(st, a, b, w);
    const int nv = a.vh * a.vw;
    uint16_t *o = out + b * nv;
    int i0 = lane, r = lane / a.vw, c = lane - (lane / a.vw) * a.vw;
    while (i0 < nv)
        obs_wave_cells(st, a, w, nv, i0, r, c, [&](int i, uint32_t v) { o[i] = (uint16_t)v; });
}

// ---- channel observations (output_channels = (c_0 .. c_{nch-1})) --------------------
// Element (cell i, channel k) of an env's view is bit c_k of the view value, stored as
// 0 / `one` (1, 0x3F80 bf16, 0x3F800000 f32) in ESZ bytes: safelife_env.py:150-154.
// A view cell is first reduced to its CHANNEL MASK m = sum_k bit(v, c_k) << k (one AND
// for the usual channels 0..nch-1, the reference's default range(15)); the mask array
// of the env's view sits in LDS and the env's output bytes are written as 16-byte
// vectors where they cover a whole aligned chunk (33x33x15 u16 = 32 670 B per env is
// only 2-byte aligned, so the partial chunks at both ends go element by element).
struct ChanMap {
    uint64_t chpack;         // channel k in bits 4k .. 4k+3
    int nch;
    __device__ __forceinline__ bool ident() const {
        bool id = true;
        for (int k = 0; k < nch; k++) id = id && ((chpack >> (4 * k)) & 15u) == (uint64_t)k;
        return id;
    }
    __device__ __forceinline__ uint32_t mask(uint32_t v, bool id) const {
        if (id) return v & ((1u << nch) - 1u);
        uint32_t m = 0u;
        for (int k = 0; k < nch; k++) m |= ((v >> ((chpack >> (4 * k)) & 15u)) & 1u) << k;
        return m;
    }
};

// vm: the env's nv channel masks in LDS (+ 2 readable cells past the end); one wave
template <int ESZ>
__device__ __forceinline__ void obs_store_channels(const uint16_t *vm, int nv, int nch, uint32_t one,
                                                   int64_t b, int lane, uint8_t *__restrict__ out) {
    const int64_t n_el = (int64_t)nv * nch;                  // elements per env
    const int64_t base = b * n_el * ESZ;                      // first byte
    const int64_t end = base + n_el * ESZ;
    const int64_t c0 = (base + 15) & ~(int64_t)15, c1 = end & ~(int64_t)15;
    // partial chunks at both ends (< 16 bytes each): one element per lane
    const int head = (int)(((c0 < end ? c0 : end) - base) / ESZ);
    const int tail = c1 >= c0 ? (int)((end - c1) / ESZ) : 0;
    int e = -1;                                               // elements per env < 2^16
    if (lane < head) e = lane;
    else if (lane >= 32 && lane - 32 < tail) e = (int)((c1 - base) / ESZ) + (lane - 32);
    if (e >= 0) {
        const int cell = e / nch, k = e - cell * nch;
        const uint32_t v = ((vm[cell] >> k) & 1u) ? one : 0u;
        for (int t = 0; t < ESZ; t++) out[base + e * ESZ + t] = (uint8_t)(v >> (8 * t));
    }
    // whole chunks; a lane's next chunk starts 1024 / ESZ elements on, i.e. dcell
    // cells and dk channels (no division in the loop)
    constexpr int NE = 16 / ESZ, STEP = 1024 / ESZ;
    const int dcell = STEP / nch, dk = STEP - dcell * nch;
    int cell0, k0;
    {
        const int e0 = (int)((c0 - base) / ESZ) + lane * NE;
        cell0 = e0 / nch;
        k0 = e0 - cell0 * nch;
    }
    for (int64_t q = c0 + 16 * (int64_t)lane; q < c1; q += 16 * 64) {
        // the chunk's NE element bits, low bit first
        uint32_t bits = (uint32_t)vm[cell0] >> k0;
        int have = nch - k0, cn = cell0 + 1;
        while (have < NE) {
            bits |= (uint32_t)vm[cn++] << have;
            have += nch;
        }
        cell0 += dcell;
        k0 += dk;
        if (k0 >= nch) {
            k0 -= nch;
            cell0++;
        }
        uint32_t wv[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (ESZ == 1)        // 4 bits -> 4 bytes
                wv[j] = ((((bits >> (4 * j)) & 15u) * 0x00204081u) & 0x01010101u) * one;
            else if (ESZ == 2)   // 2 bits -> 2 halfwords
                wv[j] = ((((bits >> (2 * j)) & 3u) * 0x8001u) & 0x00010001u) * one;
            else                 // 1 bit -> 1 word
                wv[j] = ((bits >> j) & 1u) * one;
        }
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 v4 = {wv[0], wv[1], wv[2], wv[3]};
        __builtin_nontemporal_store(v4, reinterpret_cast<u32x4 *>(out + q));
    }
}

// One env's channel view from the stored state in HBM (get_obs after the step), by one
// wave; vm: nv + 2 u16 of LDS for the masks
template <int ESZ>
__device__ __forceinline__ void obs_channels_wave(const sl_env_state &st, const ObsArgs &a,
                                                  const ChanMap &cm, uint32_t one, int64_t b,
                                                  int lane, uint16_t *vm, uint8_t *__restrict__ out) {
    ObsWave w;
    obs_wave_init(st, a, b, w);
    const int nv = a.vh * a.vw;
    const bool id = cm.ident();
    int i0 = lane, r = lane / a.vw, c = lane - (lane / a.vw) * a.vw;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");   // earlier readers of vm
    __builtin_amdgcn_wave_barrier();
    while (i0 < nv)
        obs_wave_cells(st, a, w, nv, i0, r, c,
                       [&](int i, uint32_t v) { vm[i] = (uint16_t)cm.mask(v, id); });
    // LDS operations of one wave complete in order: the reads below see the writes
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    obs_store_channels<ESZ>(vm, nv, cm.nch, one, b, lane, out);
}

}  // namespace obs
}  // namespace sl
