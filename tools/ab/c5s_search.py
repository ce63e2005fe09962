# C5 replay: k_stream_draw128's rank searches for a batch of ranks run step-major
# (every rank's LDS read of a step issued before any is waited on) instead of one rank
# after another (each search a chain of eight dependent LDS round trips)
F = "sl_bits128.hip"
START = "        for (int i0 = 0; i0 < total; i0 += 64 * kDrawBatch) {"
END = """                    __hip_atomic_fetch_or(&spw[cell[k] >> 5], 1u << (cell[k] & 31u),
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
"""


def new(KB):
    return """        for (int i0 = 0; i0 < total; i0 += 64 * KB) {
            int ii[KB], sg[KB];
#pragma unroll
            for (int k = 0; k < KB; k++) {
                ii[k] = min(i0 + 64 * k + lane, total - 1);
                sg[k] = 0;                              // the last segment based at <= i
            }
#pragma unroll
            for (int step = kSegs / 2; step >= 1; step >>= 1)
#pragma unroll
                for (int k = 0; k < KB; k++)
                    if ((int)segb[sg[k] + step] <= ii[k]) sg[k] += step;
            u32 Rx[KB], Ry[KB];
            int kk[KB], at[KB];
#pragma unroll
            for (int k = 0; k < KB; k++) {
                Rx[k] = segr[2 * sg[k]];
                Ry[k] = segr[2 * sg[k] + 1];
                kk[k] = ii[k] - (int)segb[sg[k]];
                at[k] = 0;
            }
#pragma unroll
            for (int step = 16; step >= 1; step >>= 1)
#pragma unroll
                for (int k = 0; k < KB; k++) {
                    const u32 msk = (1u << step) - 1u;
                    const int cl = __builtin_popcount((Rx[k] >> at[k]) & msk) +
                                   __builtin_popcount((Ry[k] >> at[k]) & msk);
                    if (kk[k] >= cl) {
                        kk[k] -= cl;
                        at[k] += step;
                    }
                }
            double u[KB];
            u32 cell[KB];
#pragma unroll
            for (int k = 0; k < KB; k++) {
                const int i = i0 + 64 * k + lane;
                const u32 q = (kk[k] == 0 && ((Rx[k] >> at[k]) & 1u)) ? 0u : 1u;
                const u32 t = (u32)sg[k] >> 6, row = ((u32)sg[k] >> 1) & 31u;
                const u32 j = 32u * ((u32)sg[k] & 1u) + (u32)at[k];
                cell[k] = (((t * 2 + q) * 64 + j) << 5) | row;
                const int64_t r = pos + i;
                u[k] = (i < total && r < n_draws) ? draws[r] : 1.0;
                if (i < total && r >= n_draws) atomicOr((unsigned long long *)w.err, 1ull);
            }
#pragma unroll
            for (int k = 0; k < KB; k++)
                if (u[k] < thr)
                    __hip_atomic_fetch_or(&spw[cell[k] >> 5], 1u << (cell[k] & 31u),
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
""".replace("KB", str(KB))


import os
_src = open(os.path.join("safelife-k2_amd", "csrc", F)).read()    # run from the repo root
_old = _src[_src.index(START):_src.index(END) + len(END)]
VARIANTS = {"sm4": [(F, _old, new(4))], "sm8": [(F, _old, new(8))], "sm2": [(F, _old, new(2))]}
