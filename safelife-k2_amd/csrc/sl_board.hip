// sl_board.hip -- batched board-level entry points for gfx950.
//
//   sl_advance          speedups.advance_board over B boards (module.c:19-44)
//   sl_count_eligible   draws one advance consumes (advance_board.c:110)
//   sl_exclusive_scan_i64      three-launch chunked scan (k_scan_reduce / _chunks / _apply)
//   sl_side_effect_densities   the rollout + density half of side_effect_score
//                              (side_effects.py:59-92,131-139), batched over episodes
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
            const int y = i / W;
            u = spawn_uniform(y, i - y * W, W, env0 + (uint32_t)b, step, tensor, seed);
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
// Exclusive scan of int64 counts in three launches (no host sync, no inter-block
// waiting): k_scan_reduce writes each 1024-element chunk's total into the first
// output slot of the chunk, k_scan_chunks scans those totals in place (plus *base)
// and writes the grand total, k_scan_apply scans each chunk and adds its offset.
constexpr int kScanT = 1024;

// inclusive scan over the block's 1024 threads (wave64 shuffles + 16 wave totals)
__device__ __forceinline__ int64_t block_scan_incl(int64_t v, int64_t *wtot, int64_t *total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    if (lane == 63) wtot[wid] = v;
    __syncthreads();
    int64_t pre = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kScanT / 64; w++) {
        const int64_t t = wtot[w];
        pre += w < wid ? t : 0;
        all += t;
    }
    __syncthreads();
    *total = all;
    return pre + v;
}

__global__ void __launch_bounds__(kScanT)
k_scan_reduce(const int64_t *__restrict__ in, int64_t *__restrict__ out, int64_t n) {
    __shared__ int64_t wtot[kScanT / 64];
    const int64_t i = (int64_t)blockIdx.x * kScanT + threadIdx.x;
    int64_t total;
    (void)block_scan_incl(i < n ? in[i] : 0, wtot, &total);
    if (threadIdx.x == 0) out[(int64_t)blockIdx.x * kScanT] = total;
}

__global__ void __launch_bounds__(kScanT)
k_scan_chunks(int64_t *__restrict__ out, int64_t nchunks, const int64_t *base,
              int64_t *total_out) {
    __shared__ int64_t wtot[kScanT / 64];
    int64_t carry = base ? base[0] : 0;      // read before total_out (may alias) is written
    for (int64_t s = 0; s < nchunks; s += kScanT) {
        const int64_t j = s + threadIdx.x;
        const int64_t v = j < nchunks ? out[j * kScanT] : 0;
        int64_t total;
        const int64_t incl = block_scan_incl(v, wtot, &total);
        if (j < nchunks) out[j * kScanT] = carry + incl - v;
        carry += total;
    }
    __syncthreads();
    if (threadIdx.x == 0 && total_out) total_out[0] = carry;
}

// n <= 1024 in one launch (the side-effect rollouts' per-iteration pair of counts)
__global__ void __launch_bounds__(kScanT)
k_scan_small(const int64_t *__restrict__ in, int64_t *__restrict__ out, int64_t n,
             const int64_t *base, int64_t *total_out) {
    __shared__ int64_t wtot[kScanT / 64];
    const int64_t carry = base ? base[0] : 0;
    const int64_t i = threadIdx.x, v = i < n ? in[i] : 0;
    int64_t total;
    const int64_t incl = block_scan_incl(v, wtot, &total);
    if (i < n) out[i] = carry + incl - v;
    if (threadIdx.x == 0 && total_out) total_out[0] = carry + total;
}

__global__ void __launch_bounds__(kScanT)
k_scan_apply(const int64_t *__restrict__ in, int64_t *__restrict__ out, int64_t n) {
    __shared__ int64_t wtot[kScanT / 64];
    __shared__ int64_t off;
    const int64_t c0 = (int64_t)blockIdx.x * kScanT, i = c0 + threadIdx.x;
    if (threadIdx.x == 0) off = out[c0];     // the chunk's offset (k_scan_chunks)
    __syncthreads();
    const int64_t v = i < n ? in[i] : 0;
    int64_t total;
    const int64_t incl = block_scan_incl(v, wtot, &total);
    if (i < n) out[i] = off + incl - v;
}

// ---------------------------------------------------------------------------
// Side-effect rollouts (side_effects.py:131-139).  Board 2e is episode e's b0 (the
// inaction run from the initial board), board 2e+1 its b1 (the actual final board).
// At rollout iteration `it` (S = num_samples, st = num_steps[e]):
//   b0 advances while it < st + S (its advance index is it),
//   b1 advances while st <= it < st + S (advance index it - st),
//   and both are sampled after the advance when st <= it < st + S,
// which is the reference's order: st pre-steps of b0, then per sample b0, b1.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool ro_active(int which, int it, int st, int S) {
    return which == 0 ? it < st + S : (it >= st && it < st + S);
}

template <int RNG>
__global__ void __launch_bounds__(NT)
k_rollout_advance(const uint16_t *__restrict__ in, uint16_t *__restrict__ out, int H, int W,
                  const int32_t *__restrict__ steps, int S, int it,
                  const float *__restrict__ spawn_prob, uint64_t seed, uint32_t env0,
                  const double *__restrict__ draws, const int64_t *__restrict__ offsets) {
    extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
    __shared__ int wave_tot[NT / 64];
    const int hw = H * W;
    const int64_t bi = blockIdx.x, e = bi >> 1;
    const int which = (int)(bi & 1), st = steps[e];
    const uint16_t *src = in + bi * hw;
    uint16_t *dst = out + bi * hw;
    if (!ro_active(which, it, st, S)) {
        for (int i = threadIdx.x; i < hw; i += NT) dst[i] = src[i];
        return;
    }
    const uint32_t t = (uint32_t)(which == 0 ? it : it - st);
    stage_board(lds, src, hw);
    __syncthreads();
    const double thr = (double)spawn_prob[e];
    int64_t pos = (RNG == SL_RNG_STREAM) ? offsets[which] : 0;
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
            if (elig) u = draws[pos + rank];
            pos += tot;
        } else if (elig) {
            const int y = i / W;
            u = spawn_uniform(y, i - y * W, W, env0 + (uint32_t)e, t, 4u + (uint32_t)which, seed);
        }
        if (elig && u < thr) r = sv;
        if (i < hw) dst[i] = (uint16_t)r;
    }
}

// The density key of a cell (_add_cell_distribution, side_effects.py:60-79): 0 for
// cells not counted (empty, agent, frozen & immovable & indestructible); else the
// cell without its destructible bit, which alive and hard-spawner bases get back.
__device__ __forceinline__ uint32_t density_key(uint32_t c) {
    if ((c & (FROZEN | DESTR | MOVABLE)) == FROZEN) return 0;
    uint32_t m = c & ~DESTR & 0xFFFFu;
    if (m == 0 || (m & AGENT)) return 0;
    const uint32_t base = m & ~COLORS;
    if (base == ALIVE || base == (FROZEN | SPAWN)) m |= DESTR;
    return m;
}

// pass 1: mark every key a sampled board holds (bitmap [2E][2048] words)
__global__ void __launch_bounds__(NT)
k_density_mark(const uint16_t *__restrict__ boards, int hw, const int32_t *__restrict__ steps,
               int S, int it, uint32_t *__restrict__ bitmap) {
    const int64_t bi = blockIdx.y, e = bi >> 1;
    const int st = steps[e];
    if (!(it >= st && it < st + S)) return;
    for (int i = blockIdx.x * NT + threadIdx.x; i < hw; i += gridDim.x * NT) {
        const uint32_t k = density_key(boards[bi * hw + i]);
        if (k) atomicOr(&bitmap[bi * 2048 + (k >> 5)], 1u << (k & 31));
    }
}

// the union of an episode's two key sets, ascending, with presence bits
__global__ void __launch_bounds__(NT)
k_density_compact(const uint32_t *__restrict__ bitmap, int max_keys, uint16_t *__restrict__ keys,
                  int32_t *__restrict__ n_keys, int32_t *__restrict__ present) {
    __shared__ int wave_tot[NT / 64];
    const int64_t e = blockIdx.x;
    const uint32_t *b0 = bitmap + (2 * e) * 2048, *b1 = bitmap + (2 * e + 1) * 2048;
    int base = 0;
    for (int c = 0; c < 2048; c += NT) {        // 8 chunks of 256 words, in order
        const int wd = c + threadIdx.x;
        const uint32_t u = b0[wd] | b1[wd];
        // exclusive prefix of the popcounts over the block (thread order = word order)
        int tot;
        int rank = 0;
        {
            const int cnt = __popc(u);
            // simple block scan via per-wave inclusive scans
            const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
            int v = cnt;
            for (int o = 1; o < 64; o <<= 1) {
                const int t = __shfl_up(v, o, 64);
                if (lane >= o) v += t;
            }
            if (lane == 63) wave_tot[wid] = v;
            __syncthreads();
            int off = 0;
            tot = 0;
            for (int w = 0; w < NT / 64; w++) {
                off += (w < wid) ? wave_tot[w] : 0;
                tot += wave_tot[w];
            }
            __syncthreads();
            rank = off + v - cnt;
        }
        uint32_t m = u;
        int k = base + rank;
        while (m) {
            const int bit = __ffs(m) - 1;
            m &= m - 1;
            if (k < max_keys) {
                keys[e * max_keys + k] = (uint16_t)(wd * 32 + bit);
                present[e * max_keys + k] = (int)((b0[wd] >> bit) & 1u) |
                                            (int)(((b1[wd] >> bit) & 1u) << 1);
            }
            k++;
        }
        base += tot;
    }
    if (threadIdx.x == 0) n_keys[e] = base;
}

// pass 2: count each sampled cell into its key's map (dens [E][max_keys][hw] per run)
__global__ void __launch_bounds__(NT)
k_density_count(const uint16_t *__restrict__ boards, int hw, const int32_t *__restrict__ steps,
                int S, int it, const uint16_t *__restrict__ keys,
                const int32_t *__restrict__ n_keys, int max_keys, double *__restrict__ inaction,
                double *__restrict__ action) {
    __shared__ uint16_t kl[1024];
    const int64_t bi = blockIdx.y, e = bi >> 1;
    const int which = (int)(bi & 1), st = steps[e];
    if (!(it >= st && it < st + S)) return;
    const int nk = min(n_keys[e], max_keys);
    for (int k = threadIdx.x; k < nk; k += NT) kl[k] = keys[e * max_keys + k];
    __syncthreads();
    double *dens = (which == 0 ? inaction : action) + e * (int64_t)max_keys * hw;
    for (int i = blockIdx.x * NT + threadIdx.x; i < hw; i += gridDim.x * NT) {
        const uint32_t key = density_key(boards[bi * hw + i]);
        if (!key) continue;
        int lo = 0, hi = nk - 1;                 // keys ascending
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (kl[mid] < key) lo = mid + 1;
            else hi = mid;
        }
        if (nk > 0 && kl[lo] == key) dens[(int64_t)lo * hw + i] += 1.0;   // else: overflow
    }
}

// x /= n, as _norm_cell_distribution does (a true division, not a reciprocal product)
__global__ void __launch_bounds__(NT)
k_density_norm(double *__restrict__ a, double *__restrict__ b, int64_t n, double den) {
    for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
        a[i] = a[i] / den;
        b[i] = b[i] / den;
    }
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
    hipStream_t s = (hipStream_t)stream;
    if (n <= kScanT) {
        hipLaunchKernelGGL(k_scan_small, dim3(1), dim3(kScanT), 0, s, in, out, n, base, total_out);
        return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
    }
    const int64_t nchunks = (n + kScanT - 1) / kScanT;
    if (nchunks > 0x7FFFFFFF) return SL_EINVAL;
    if (nchunks > 0) {
        hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)nchunks), dim3(kScanT), 0, s, in, out, n);
        if (hipGetLastError() != hipSuccess) return SL_EHIP;
    }
    hipLaunchKernelGGL(k_scan_chunks, dim3(1), dim3(kScanT), 0, s, out, nchunks, base, total_out);
    if (hipGetLastError() != hipSuccess) return SL_EHIP;
    if (nchunks > 0)
        hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)nchunks), dim3(kScanT), 0, s, in, out, n);
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}

// ---------------------------------------------------------------------------
// side-effect rollouts + densities
// ---------------------------------------------------------------------------
extern "C" int sl_side_effect_workspace(int64_t E, int H, int W, int64_t *bytes) {
    if (E < 0 || H < 2 || W < 2 || !bytes) return SL_EINVAL;
    const int64_t hw = (int64_t)H * W;
    // two board buffers [2E][hw] u16, bitmaps [2E][2048] u32, 4 int64 for replay
    *bytes = 2 * (2 * E * hw * 2) + 2 * E * 2048 * 4 + 64;
    return SL_OK;
}

extern "C" int sl_side_effect_densities(const uint16_t *init_board, const uint16_t *final_board,
                                        const int32_t *num_steps_dev,
                                        const int32_t *num_steps_host,
                                        const float *spawn_prob, int64_t E, int H, int W,
                                        int num_samples, int rng_mode, uint64_t seed,
                                        uint32_t env0, const double *draws,
                                        int64_t *stream_pos, int max_keys, uint16_t *keys,
                                        int32_t *n_keys, int32_t *present, double *inaction,
                                        double *action, void *workspace,
                                        int64_t workspace_bytes, void *stream) {
    if (E < 0 || H < 2 || W < 2 || num_samples < 1 || max_keys < 1 || max_keys > 1024)
        return SL_EINVAL;
    if ((int64_t)H * W > kMaxBoardCells) return SL_ETOOBIG;
    if (rng_mode != SL_RNG_STREAM && rng_mode != SL_RNG_PHILOX) return SL_EINVAL;
    if (rng_mode == SL_RNG_STREAM && (E > 1 || !draws || !stream_pos)) return SL_EINVAL;
    if (E == 0) return SL_OK;
    if (!init_board || !final_board || !num_steps_dev || !num_steps_host || !spawn_prob ||
        !keys || !n_keys || !present || !inaction || !action || !workspace)
        return SL_EINVAL;
    int64_t need;
    sl_side_effect_workspace(E, H, W, &need);
    if (workspace_bytes < need) return SL_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const int hw = H * W;
    const int64_t nb = 2 * E;
    uint16_t *buf0 = (uint16_t *)workspace;
    uint16_t *buf1 = buf0 + nb * hw;
    uint32_t *bitmap = (uint32_t *)(buf1 + nb * hw);
    int64_t *ri = (int64_t *)(bitmap + nb * 2048);     // counts[2], offsets[2], pos0
    ri = (int64_t *)(((uintptr_t)ri + 7) & ~(uintptr_t)7);
    int max_steps = 0;
    for (int64_t e = 0; e < E; e++) {
        if (num_steps_host[e] < 0) return SL_EINVAL;
        max_steps = num_steps_host[e] > max_steps ? num_steps_host[e] : max_steps;
    }
    const int iters = max_steps + num_samples;
    const size_t lds = (size_t)hw * sizeof(uint16_t);
    if (!lds_ok((const void *)k_rollout_advance<SL_RNG_STREAM>, lds) ||
        !lds_ok((const void *)k_rollout_advance<SL_RNG_PHILOX>, lds))
        return SL_ETOOBIG;
    const dim3 cell_grid((unsigned)((hw + NT - 1) / NT), (unsigned)nb);
    const int64_t map_elems = E * (int64_t)max_keys * hw;
    if (hipMemsetAsync(bitmap, 0, nb * 2048 * 4, s) != hipSuccess ||
        hipMemsetAsync(inaction, 0, map_elems * 8, s) != hipSuccess ||
        hipMemsetAsync(action, 0, map_elems * 8, s) != hipSuccess)
        return SL_EHIP;
    if (rng_mode == SL_RNG_STREAM &&
        hipMemcpyAsync(ri + 4, stream_pos, 8, hipMemcpyDeviceToDevice, s) != hipSuccess)
        return SL_EHIP;
    for (int pass = 0; pass < 2; pass++) {
        // boards: b0 = initial, b1 = final (interleaved per episode)
        if (hipMemcpy2DAsync(buf0, 2 * hw * 2, init_board, hw * 2, hw * 2, E,
                             hipMemcpyDeviceToDevice, s) != hipSuccess ||
            hipMemcpy2DAsync(buf0 + hw, 2 * hw * 2, final_board, hw * 2, hw * 2, E,
                             hipMemcpyDeviceToDevice, s) != hipSuccess)
            return SL_EHIP;
        if (rng_mode == SL_RNG_STREAM && pass == 1 &&
            hipMemcpyAsync(stream_pos, ri + 4, 8, hipMemcpyDeviceToDevice, s) != hipSuccess)
            return SL_EHIP;
        uint16_t *cur = buf0, *nxt = buf1;
        for (int it = 0; it < iters; it++) {
            if (rng_mode == SL_RNG_STREAM) {
                // reference order: b0's draws, then b1's (when it advances)
                const int st0 = num_steps_host[0];
                const int n_adv = (it >= st0 && it < st0 + num_samples) ? 2
                                  : (it < st0 + num_samples ? 1 : 0);
                if (n_adv) {
                    hipLaunchKernelGGL(k_count_eligible, dim3((unsigned)n_adv), dim3(NT), lds, s,
                                       cur, ri, H, W);
                    hipLaunchKernelGGL(k_scan_small, dim3(1), dim3(kScanT), 0, s, ri, ri + 2,
                                       (int64_t)n_adv, stream_pos, stream_pos);
                }
                hipLaunchKernelGGL(k_rollout_advance<SL_RNG_STREAM>, dim3((unsigned)nb),
                                   dim3(NT), lds, s, cur, nxt, H, W, num_steps_dev, num_samples,
                                   it, spawn_prob, seed, env0, draws, ri + 2);
            } else {
                hipLaunchKernelGGL(k_rollout_advance<SL_RNG_PHILOX>, dim3((unsigned)nb),
                                   dim3(NT), lds, s, cur, nxt, H, W, num_steps_dev, num_samples,
                                   it, spawn_prob, seed, env0, draws, (const int64_t *)nullptr);
            }
            uint16_t *t = cur;
            cur = nxt;
            nxt = t;
            if (pass == 0)
                hipLaunchKernelGGL(k_density_mark, cell_grid, dim3(NT), 0, s, cur, hw,
                                   num_steps_dev, num_samples, it, bitmap);
            else
                hipLaunchKernelGGL(k_density_count, cell_grid, dim3(NT), 0, s, cur, hw,
                                   num_steps_dev, num_samples, it, keys, n_keys, max_keys,
                                   inaction, action);
        }
        if (pass == 0)
            hipLaunchKernelGGL(k_density_compact, dim3((unsigned)E), dim3(NT), 0, s, bitmap,
                               max_keys, keys, n_keys, present);
        if (hipGetLastError() != hipSuccess) return SL_EHIP;
    }
    hipLaunchKernelGGL(k_density_norm, dim3(1024), dim3(NT), 0, s, inaction, action, map_elems,
                       (double)num_samples);
    return hipGetLastError() == hipSuccess ? SL_OK : SL_EHIP;
}
