// Streaming bandwidth probes on one GPU (not part of the product): copy / read / write
// variants over 1 GiB, 16 B per lane, plain and nontemporal.  hipcc -O3
// --offload-arch=gfx950 tools/bwtest.hip -o tools/_bin/bwtest
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef unsigned v4u __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ void __launch_bounds__(256) k_copy(const v4u *__restrict__ s, v4u *__restrict__ d,
                                              long n) {
    const long stride = (long)gridDim.x * 256;
    long i = (long)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = NT ? __builtin_nontemporal_load(s + i + u * stride) : s[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (NT) __builtin_nontemporal_store(v[u], d + i + u * stride);
            else d[i + u * stride] = v[u];
        }
    }
    for (; i < n; i += stride) d[i] = s[i];
}

template <int U>
__global__ void __launch_bounds__(256) k_read(const v4u *__restrict__ s, unsigned *out, long n) {
    const long stride = (long)gridDim.x * 256;
    unsigned acc = 0;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const v4u v = s[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void __launch_bounds__(256) k_write(v4u *__restrict__ d, long n) {
    const long stride = (long)gridDim.x * 256;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
        d[i] = v4u{(unsigned)i, 1u, 2u, 3u};
}

template <class F>
static double timeit(F f) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int r = 0; r < 3; r++) f();
    hipEventRecord(a);
    for (int r = 0; r < 20; r++) f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / 20;
}

int main() {
    const long nbytes = 1L << 30, n = nbytes / 16;
    v4u *s, *d;
    unsigned *o;
    if (hipMalloc(&s, nbytes) || hipMalloc(&d, nbytes) || hipMalloc(&o, 64)) return 1;
    hipMemset(s, 1, nbytes);
    int grids[] = {1024, 2048, 4096, 8192, 16384};
    for (int g : grids) {
        double t1 = timeit([&] { hipLaunchKernelGGL((k_copy<1, false>), dim3(g), dim3(256), 0, 0, s, d, n); });
        double t4 = timeit([&] { hipLaunchKernelGGL((k_copy<4, false>), dim3(g), dim3(256), 0, 0, s, d, n); });
        double t4n = timeit([&] { hipLaunchKernelGGL((k_copy<4, true>), dim3(g), dim3(256), 0, 0, s, d, n); });
        double t8 = timeit([&] { hipLaunchKernelGGL((k_copy<8, false>), dim3(g), dim3(256), 0, 0, s, d, n); });
        double tr = timeit([&] { hipLaunchKernelGGL((k_read<1>), dim3(g), dim3(256), 0, 0, s, o, n); });
        double tw = timeit([&] { hipLaunchKernelGGL(k_write, dim3(g), dim3(256), 0, 0, d, n); });
        printf("grid %5d  copy(rd+wr TB/s) u1 %.2f u4 %.2f u4nt %.2f u8 %.2f | read %.2f | write %.2f\n",
               g, 2 * nbytes / t1 / 1e9, 2 * nbytes / t4 / 1e9, 2 * nbytes / t4n / 1e9,
               2 * nbytes / t8 / 1e9, nbytes / tr / 1e9, nbytes / tw / 1e9);
    }
    return 0;
}
