// bw_probe.hip — HBM ceilings for the Alexandridis step's access pattern on one MI355X.
//   (1) float4 copy (read + write) of a large buffer: the practical HBM roofline
//   (2) read-only float4 stream
//   (3) the alex_step byte pattern (41 B/cell: grid u8 r+w, age i16 r+w, veg, den, dousing u8,
//       p_slope 8 x f32 planes, E x 256 x 256) with trivial compute, 16 cells per lane like the kernel
// Build: hipcc -O3 --offload-arch=gfx950 scripts/bw_probe.hip -o scripts/bw_probe
// Prints one JSON line.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("{\"error\": \"%s\"}\n", hipGetErrorString(e_)); return 1; } } while (0)

__global__ void copy_k(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}
__global__ void read_k(const float4* __restrict__ a, float* __restrict__ out, size_t n) {
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[0] = s;
}
// one lane = 16 consecutive cells of one row; one block = 256 lanes = 16 rows x 256 cols (one tile)
__global__ __launch_bounds__(256) void alex_pattern_k(const uint8_t* __restrict__ g, uint8_t* __restrict__ go,
                                                      const int16_t* __restrict__ a, int16_t* __restrict__ ao,
                                                      const uint8_t* __restrict__ v, const uint8_t* __restrict__ d,
                                                      const uint8_t* __restrict__ du, const float* __restrict__ ps,
                                                      int HW) {
    const int tiles = HW / 4096;
    const int e = blockIdx.x / tiles, t = blockIdx.x % tiles;
    const size_t off = (size_t)e * HW + (size_t)t * 4096 + threadIdx.x * 16;
    const uint4 g4 = *(const uint4*)(g + off);
    const uint4 v4 = *(const uint4*)(v + off);
    const uint4 d4 = *(const uint4*)(d + off);
    const uint4 u4 = *(const uint4*)(du + off);
    const uint4 a0 = *(const uint4*)(a + off);
    const uint4 a1 = *(const uint4*)(a + off + 8);
    float acc = 0.f;
    const float* pE = ps + (size_t)e * 8 * HW + (size_t)t * 4096 + threadIdx.x * 16;
#pragma unroll
    for (int dd = 0; dd < 8; ++dd) {
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const float4 p4 = *(const float4*)(pE + (size_t)dd * HW + 4 * m);
            acc += p4.x + p4.y + p4.z + p4.w;
        }
    }
    const uint32_t mix = (acc > 1e30f) ? 1u : 0u;
    *(uint4*)(go + off) = make_uint4(g4.x ^ v4.x ^ mix, g4.y ^ d4.y, g4.z ^ u4.z, g4.w);
    *(uint4*)(ao + off) = make_uint4(a0.x, a0.y ^ mix, a0.z, a0.w);
    *(uint4*)(ao + off + 8) = a1;
}

int main() {
    const size_t nbytes = (size_t)8 << 30;  // 8 GiB copy source
    float4 *A, *B;
    float* out;
    CK(hipMalloc(&A, nbytes));
    CK(hipMalloc(&B, nbytes));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(A, 0, nbytes));
    const size_t n4 = nbytes / 16;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms;
    const int blocks = 256 * 8 * 4;
    copy_k<<<blocks, 256>>>(A, B, n4);
    CK(hipEventRecord(e0));
    for (int i = 0; i < 10; ++i) copy_k<<<blocks, 256>>>(A, B, n4);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double copy_gbs = 2.0 * nbytes * 10 / (ms * 1e-3) / 1e9;
    read_k<<<blocks, 256>>>(A, out, n4);
    CK(hipEventRecord(e0));
    for (int i = 0; i < 10; ++i) read_k<<<blocks, 256>>>(A, out, n4);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double read_gbs = 1.0 * nbytes * 10 / (ms * 1e-3) / 1e9;
    CK(hipFree(A));
    CK(hipFree(B));
    // alex pattern: E = 4096, 256 x 256
    const int E = 4096, HW = 65536;
    const size_t cells = (size_t)E * HW;
    uint8_t *g, *go, *v, *d, *du;
    int16_t *a, *ao;
    float* ps;
    CK(hipMalloc(&g, cells)); CK(hipMalloc(&go, cells)); CK(hipMalloc(&v, cells)); CK(hipMalloc(&d, cells));
    CK(hipMalloc(&du, cells)); CK(hipMalloc(&a, 2 * cells)); CK(hipMalloc(&ao, 2 * cells));
    CK(hipMalloc(&ps, 32 * cells));
    CK(hipMemset(ps, 0, 32 * cells));
    const int nblk = E * (HW / 4096);
    alex_pattern_k<<<nblk, 256>>>(g, go, a, ao, v, d, du, ps, HW);
    CK(hipEventRecord(e0));
    for (int i = 0; i < 10; ++i) alex_pattern_k<<<nblk, 256>>>(g, go, a, ao, v, d, du, ps, HW);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double alex_ms = ms / 10;
    const double alex_gbs = 41.0 * cells / (alex_ms * 1e-3) / 1e9;
    printf("{\"copy_gbs\": %.1f, \"read_gbs\": %.1f, \"alex_pattern_ms\": %.4f, \"alex_pattern_gbs\": %.1f}\n", copy_gbs,
           read_gbs, alex_ms, alex_gbs);
    return 0;
}
