// copy_probe.hip — r06: which hand-written device copy reaches the guide's ~6.3 TB/s (MI355X_MICROARCH.md: float4 copy)
// on this pool's boxes, for gca_bench_copy (the bench's HBM ceiling yardstick). Variants over one buffer pair of
// NBYTES (default 2 GiB, 8x the Infinity Cache); rate = 2 x bytes / time (read + write), HIP events, mean of 10 after 3.
//   gs<B,U,NT>   grid-stride, B workgroups of 256, U x 16 B per thread in flight (loads, then stores), NT non-temporal
//   once<U,NT>   one pass: every thread copies U x 16 B once (n / (256 U) workgroups)
//   chunk<C,U>   each workgroup copies a contiguous C-KiB chunk, U x 16 B per thread per round
// Build: hipcc -O3 --offload-arch=gfx950 scripts/copy_probe.hip -o scripts/copy_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef float vf4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__device__ __forceinline__ void copy_u(const vf4* __restrict__ s, vf4* __restrict__ d, int64_t base, int64_t step,
                                       int64_t n) {
    vf4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const int64_t i = base + step * k;
        if (i < n) v[k] = NT ? __builtin_nontemporal_load(s + i) : s[i];
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const int64_t i = base + step * k;
        if (i < n) {
            if (NT) __builtin_nontemporal_store(v[k], d + i);
            else d[i] = v[k];
        }
    }
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void gs_k(const vf4* __restrict__ s, vf4* __restrict__ d, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * 256 * U;
    for (int64_t b = (int64_t)blockIdx.x * 256 * U + threadIdx.x; b < n; b += stride) copy_u<U, NT>(s, d, b, 256, n);
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void once_k(const vf4* __restrict__ s, vf4* __restrict__ d, int64_t n) {
    copy_u<U, NT>(s, d, (int64_t)blockIdx.x * 256 * U + threadIdx.x, 256, n);
}

template <int CK, int U>
__global__ __launch_bounds__(256) void chunk_k(const vf4* __restrict__ s, vf4* __restrict__ d, int64_t n) {
    constexpr int64_t C = (int64_t)CK * 1024 / 16;  // float4 per chunk
    const int64_t c0 = (int64_t)blockIdx.x * C;
    for (int64_t b = c0 + threadIdx.x; b < c0 + C && b < n; b += 256 * U) copy_u<U, false>(s, d, b, 256, min(n, c0 + C));
}

template <class F>
static float time_ms(F launch) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) launch();
    (void)hipEventRecord(a);
    for (int i = 0; i < 10; ++i) launch();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / 10.0f;
}

int main(int argc, char** argv) {
    const int64_t nbytes = (argc > 1 ? atoll(argv[1]) : 2048) << 20;
    const int64_t n = nbytes / 16;
    vf4 *s, *d;
    if (hipMalloc(&s, nbytes) != hipSuccess || hipMalloc(&d, nbytes) != hipSuccess) {
        printf("{\"error\": \"hipMalloc\"}\n");
        return 1;
    }
    (void)hipMemset(s, 1, nbytes);
    (void)hipMemset(d, 0, nbytes);
    printf("{\"bytes\": %lld", (long long)nbytes);
    auto rate = [&](float ms) { return 2.0 * nbytes / (ms * 1e-3) / 1e9; };
#define GS(B, U, NT) printf(", \"gs_b%d_u%d_nt%d_gbs\": %.0f", B, U, NT, \
        rate(time_ms([&] { hipLaunchKernelGGL((gs_k<U, NT>), dim3(B), dim3(256), 0, 0, s, d, n); })))
#define ONCE(U, NT) printf(", \"once_u%d_nt%d_gbs\": %.0f", U, NT, \
        rate(time_ms([&] { hipLaunchKernelGGL((once_k<U, NT>), dim3((unsigned)((n + 256 * U - 1) / (256 * U))), dim3(256), 0, 0, s, d, n); })))
#define CHUNK(C, U) printf(", \"chunk%dk_u%d_gbs\": %.0f", C, U, \
        rate(time_ms([&] { hipLaunchKernelGGL((chunk_k<C, U>), dim3((unsigned)((n * 16 + C * 1024 - 1) / (C * 1024))), dim3(256), 0, 0, s, d, n); })))
    GS(4096, 4, false); GS(4096, 4, true); GS(2048, 4, false); GS(8192, 4, false); GS(16384, 4, false);
    GS(4096, 8, false); GS(2048, 8, false); GS(1024, 8, false); GS(4096, 2, false); GS(8192, 2, false);
    GS(16384, 1, false); GS(32768, 1, false);
    ONCE(1, false); ONCE(2, false); ONCE(4, false); ONCE(8, false); ONCE(4, true);
    CHUNK(64, 4); CHUNK(256, 4); CHUNK(1024, 4); CHUNK(256, 8);
    printf("}\n");
    return 0;
}
