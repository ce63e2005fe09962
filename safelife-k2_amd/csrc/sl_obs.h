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

}  // namespace obs
}  // namespace sl
