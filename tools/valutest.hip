// VALU issue-rate probes on one GPU (not part of the product): how many wave64
// integer bit instructions a SIMD retires per cycle, with 1..8 waves per SIMD, for the
// op kinds the bit-sliced step kernels are made of (v_xor_b32, v_bitop3_b32,
// v_alignbit_b32, DPP moves, v_bfi_b32).  Each lane runs 8 independent accumulator
// chains so no dependency stalls.  hipcc -O3 --offload-arch=gfx950 tools/valutest.hip
//   -o tools/_bin/valutest
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int ITERS = 4096;

template <int OP>
__global__ void __launch_bounds__(64) k_ops(unsigned *out, unsigned seed) {
    unsigned a[8];
#pragma unroll
    for (int k = 0; k < 8; k++) a[k] = seed * (threadIdx.x + 1) + k * 0x9E3779B9u;
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const unsigned n1 = a[(k + 1) & 7], n2 = a[(k + 3) & 7];
            if (OP == 0) a[k] ^= n2;                                          // v_xor_b32
            else if (OP == 1) a[k] = __builtin_amdgcn_alignbit(a[k], n1, (unsigned)k + 1);
            else if (OP == 2) a[k] = (a[k] & n1) ^ (n2 & ~a[k]);             // v_bitop3_b32
            else if (OP == 3) a[k] ^= (unsigned)__builtin_amdgcn_mov_dpp((int)n1, 0x4E, 0xF, 0xF, false);
            else a[k] = (a[k] & n1) | (~a[k] & n2);                           // v_bfi_b32
        }
    }
    unsigned r = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) r ^= a[k];
    if (r == 0x12345678u) out[0] = r;
}

int main() {
    unsigned *out;
    hipMalloc(&out, 64);
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const char *names[5] = {"xor", "alignbit", "logic3", "dpp+xor", "bfi"};
    for (int op = 0; op < 5; op++)
        for (int wps = 1; wps <= 8; wps *= 2) {
            const int grid = cus * 4 * wps;           // waves per SIMD = wps
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            auto launch = [&]() {
                switch (op) {
                case 0: hipLaunchKernelGGL(k_ops<0>, dim3(grid), dim3(64), 0, 0, out, 7u); break;
                case 1: hipLaunchKernelGGL(k_ops<1>, dim3(grid), dim3(64), 0, 0, out, 7u); break;
                case 2: hipLaunchKernelGGL(k_ops<2>, dim3(grid), dim3(64), 0, 0, out, 7u); break;
                case 3: hipLaunchKernelGGL(k_ops<3>, dim3(grid), dim3(64), 0, 0, out, 7u); break;
                default: hipLaunchKernelGGL(k_ops<4>, dim3(grid), dim3(64), 0, 0, out, 7u); break;
                }
            };
            launch();
            hipDeviceSynchronize();
            hipEventRecord(e0);
            for (int r = 0; r < 5; r++) launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            ms /= 5;
            // instructions per wave are counted by rocprofv3 (SQ_INSTS_VALU); here the
            // loop body's source ops: 8 per iteration (OP 2, 3: 2-3 VALU each)
            const double wave_ops = 8.0 * ITERS;
            printf("%-9s waves/SIMD %d  %.3f ms  %.3f source-ops/cycle/SIMD at 2.4 GHz\n", names[op],
                   wps, ms, wave_ops * grid / (cus * 4.0) / (ms * 1e-3 * 2.4e9));
            hipEventDestroy(e0);
            hipEventDestroy(e1);
        }
    return 0;
}
