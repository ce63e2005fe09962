# C5 replay: k_stream_draw128 without rank searches -- each segment's owner lane (after
# the transposes) writes the ids of its cells into LDS slots at their ranks, and lane i
# then reads slot i beside its uniform draws[pos + i]
F = "sl_bits128.hip"
START = "        // the segments: bases and cells\n"
END = """                    __hip_atomic_fetch_or(&spw[cell[k] >> 5], 1u << (cell[k] & 31u),
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
"""
NEW = """        // the segments: bases, then each owner lane writes its cells' ids at their ranks
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
                    u[k] = (i < n && r < n_draws) ? draws[r] : 1.0;
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
"""
import os
_src = open(os.path.join("safelife-k2_amd", "csrc", F)).read()    # run from the repo root
_old = _src[_src.index(START):_src.index(END) + len(END)]
DECL_OLD = """    __shared__ u32 segb_[kSegs];
    __shared__ u32 segr_[2 * kSegs];   // [segment][word]"""
DECL_NEW = """    __shared__ uint16_t slots_[kOwnSlots];
    lds_u16 *slots = (lds_u16 *)slots_;"""
USE_OLD = """    lds_u32 *segb = (lds_u32 *)segb_;
    lds_u32 *segr = (lds_u32 *)segr_;
"""
K_OLD = "constexpr int kSegs = NB * 64;\n"
K_NEW = "constexpr int kSegs = NB * 64;\nconstexpr int kOwnSlots = 2048;\n"
VARIANTS = {"owner": [(F, _old, NEW), (F, DECL_OLD, DECL_NEW), (F, USE_OLD, ""), (F, K_OLD, K_NEW)]}
