// sl_board.hip -- batched board-level entry points for gfx950.
//
//   sl_advance          speedups.advance_board over B boards (module.c:19-44)
//   sl_count_eligible   draws one advance consumes (advance_board.c:110)
//   sl_exclusive_scan_i64
//
// Layout: one workgroup (256 threads, 4 wave64) per board; the board is staged in
// LDS with coalesced loads and every output cell reads its wrapped 3x3 block
// from LDS.  Stream replay needs each eligible cell's row-major rank inside its
// board: cells are visited in 256-cell chunks in row-major order and ranked by a
// ballot/popcount prefix within each wave plus a 4-entry cross-wave prefix.
#include "sl_device.h"
#include "../../include/safelife_hip.h"

using namespace sl;

namespace {

constexpr int NT = 256;

__device__ __forceinline__ void stage_board(uint16_t *dst, const uint16_t *src, int hw) {
    // 16-byte loads when the board base is 16-B aligned and hw % 8 == 0
    if ((((uintptr_t)src) & 15) == 0 && (hw & 7) == 0) {
        const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
        uint4 *d4 = reinterpret_cast<uint4 *>(dst);
        for (int i = threadIdx.x; i < (hw >> 3); i += NT) d4[i] = s4[i];
    } else {
        for (int i = threadIdx.x; i < hw; i += NT) dst[i] = src[i];
    }
}

// exclusive rank of `flag` among the block's threads (thread order) + block total
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

template <int RNG>
__global__ void __launch_bounds__(NT)
k_advance(const uint16_t *__restrict__ in, uint16_t *__restrict__ out, int H, int W,
          const float *__restrict__ spawn_prob, float p_scalar, uint64_t seed, uint32_t env0,
          uint32_t step, uint32_t tensor, const double *__restrict__ draws,
          const int64_t *__restrict__ offsets) {
    extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
    __shared__ int wave_tot[NT / 64];
    const int hw = H * W;
    const int64_t b = blockIdx.x;
    const uint16_t *src = in + b * hw;
    uint16_t *dst = out + b * hw;
    stage_board(lds, src, hw);
    __syncthreads();
    const double thr = (double)(spawn_prob ? spawn_prob[b] : p_scalar);
    int64_t pos = (RNG == SL_RNG_STREAM && offsets) ? offsets[b] : 0;
    const int nchunk = (hw + NT - 1) / NT;
    for (int c = 0; c < nchunk; c++) {
        const int i = c * NT + threadIdx.x;
        uint32_t v = 0, r = 0, sv = 0;
        bool elig = false;
        if (i < hw) {
            const int y = i / W, x = i - y * W;
            v = lds[i];
            CellNb n = gather_lds(lds, H, W, y, x);
            r = rule_cell(v, n, &elig, &sv);
        }
        double u = 1.0;
        if (RNG == SL_RNG_STREAM) {
            int tot;
            int rank = block_rank(elig, wave_tot, &tot);
            if (elig) {
                if (thr <= 0.0) u = 1.0;
                else if (thr >= 1.0) u = 0.0;
                else u = draws[pos + rank];
            }
            pos += tot;
        } else if (elig) {
            u = philox_uniform((uint32_t)i, env0 + (uint32_t)b, step, tensor, seed);
        }
        if (elig && u < thr) r = sv;
        if (i < hw) dst[i] = (uint16_t)r;
    }
}

__global__ void __launch_bounds__(NT)
k_count_eligible(const uint16_t *__restrict__ in, int64_t *__restrict__ counts, int H, int W) {
    extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
    __shared__ int wave_tot[NT / 64];
    const int hw = H * W;
    const int64_t b = blockIdx.x;
    stage_board(lds, in + b * hw, hw);
    __syncthreads();
    int mine = 0;
    for (int i = threadIdx.x; i < hw; i += NT) {
        const int y = i / W, x = i - y * W;
        bool elig;
        uint32_t sv;
        CellNb n = gather_lds(lds, H, W, y, x);
        rule_cell(lds[i], n, &elig, &sv);
        mine += elig;
    }
    mine = wave_sum(mine);
    if ((threadIdx.x & 63) == 0) wave_tot[threadIdx.x >> 6] = mine;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t t = 0;
        for (int w = 0; w < NT / 64; w++) t += wave_tot[w];
        counts[b] = t;
    }
}

// single-workgroup exclusive scan (parity / replay path only: n <= a few 1e5)
__global__ void __launch_bounds__(1024)
k_scan_i64(const int64_t *__restrict__ in, int64_t *__restrict__ out, int64_t n,
           const int64_t *__restrict__ base, int64_t *__restrict__ total_out) {
    __shared__ int64_t part[1024];
    __shared__ int64_t carry;
    if (threadIdx.x == 0) carry = base ? base[0] : 0;
    __syncthreads();
    for (int64_t s = 0; s < n; s += 1024) {
        int64_t i = s + threadIdx.x;
        int64_t v = i < n ? in[i] : 0;
        part[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            int64_t t = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
            __syncthreads();
            part[threadIdx.x] += t;
            __syncthreads();
        }
        if (i < n) out[i] = carry + part[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == 0) carry += part[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0 && total_out) total_out[0] = carry;
}

constexpr int kMaxBoardCells = 32768;   // 64 KiB of LDS per board

bool lds_ok(const void *fn, size_t bytes) {
    if (bytes <= 65536) return true;
    return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)bytes) == hipSuccess;
}

}  // namespace

extern "C" int sl_advance(const uint16_t *in, uint16_t *out, int64_t B, int H, int W,
                          const float *spawn_prob, float spawn_prob_scalar, int rng_mode,
                          uint64_t seed, uint32_t env0, uint32_t step, uint32_t tensor,
                          const double *draws, const int64_t *draw_offsets, void *stream) {
    if (H < 2 || W < 2 || B < 0 || !in || !out || in == out) return SL_EINVAL;
    if ((int64_t)H * W > kMaxBoardCells) return SL_ETOOBIG;
    if (rng_mode != SL_RNG_STREAM && rng_mode != SL_RNG_PHILOX) return SL_EINVAL;
    if (B == 0) return SL_OK;
    hipStream_t s = (hipStream_t)stream;
    size_t lds = (size_t)H * W * sizeof(uint16_t);
    if (rng_mode == SL_RNG_STREAM) {
        bool may_draw = spawn_prob != nullptr ||
                        (spawn_prob_scalar > 0.0f && spawn_prob_scalar < 1.0f);
        if (may_draw && (!draws || !draw_offsets)) return SL_EINVAL;
        if (!lds_ok((const void *)k_advance<SL_RNG_STREAM>, lds)) return SL_ETOOBIG;
        hipLaunchKernelGGL(k_advance<SL_RNG_STREAM>, dim3((unsigned)B), dim3(NT), lds, s, in,
                           out, H, W, spawn_prob, spawn_prob_scalar, seed, env0, step, tensor,
                           draws, draw_offsets);
    } else {
        if (!lds_ok((const void *)k_advance<SL_RNG_PHILOX>, lds)) return SL_ETOOBIG;
        hipLaunchKernelGGL(k_advance<SL_RNG_PHILOX>, dim3((unsigned)B), dim3(NT), lds, s, in,
                           out, H, W, spawn_prob, spawn_prob_scalar, seed, env0, step, tensor,
                           draws, draw_offsets);
    }
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}

extern "C" int sl_count_eligible(const uint16_t *in, int64_t *counts, int64_t B, int H, int W,
                                 void *stream) {
    if (H < 2 || W < 2 || B < 0 || !in || !counts) return SL_EINVAL;
    if ((int64_t)H * W > kMaxBoardCells) return SL_ETOOBIG;
    if (B == 0) return SL_OK;
    size_t lds = (size_t)H * W * sizeof(uint16_t);
    if (!lds_ok((const void *)k_count_eligible, lds)) return SL_ETOOBIG;
    hipLaunchKernelGGL(k_count_eligible, dim3((unsigned)B), dim3(NT), lds, (hipStream_t)stream,
                       in, counts, H, W);
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}

extern "C" int sl_exclusive_scan_i64(const int64_t *in, int64_t *out, int64_t n,
                                     const int64_t *base, int64_t *total_out, void *stream) {
    if (n < 0 || (n > 0 && (!in || !out))) return SL_EINVAL;
    hipLaunchKernelGGL(k_scan_i64, dim3(1), dim3(1024), 0, (hipStream_t)stream, in, out, n,
                       base, total_out);
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}
