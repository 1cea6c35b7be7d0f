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

typedef float f4v __attribute__((ext_vector_type(4)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ntl(const float4* p) {
    const f4v v = __builtin_nontemporal_load((const f4v*)p);
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void nts(float4 v, float4* p) { __builtin_nontemporal_store((f4v){v.x, v.y, v.z, v.w}, (f4v*)p); }
__device__ __forceinline__ void nts(uint4 v, uint4* p) { __builtin_nontemporal_store((u4v){v.x, v.y, v.z, v.w}, (u4v*)p); }

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
__global__ __launch_bounds__(256) void copy4_k(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
    // 4 independent float4 per lane per iteration (4 KiB per wave in flight)
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i + 3 * stride < n; i += 4 * stride) {
        const float4 v0 = a[i], v1 = a[i + stride], v2 = a[i + 2 * stride], v3 = a[i + 3 * stride];
        b[i] = v0; b[i + stride] = v1; b[i + 2 * stride] = v2; b[i + 3 * stride] = v3;
    }
}
__global__ __launch_bounds__(256) void copy4nt_k(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i + 3 * stride < n; i += 4 * stride) {
        const float4 v0 = ntl(a + i), v1 = ntl(a + i + stride), v2 = ntl(a + i + 2 * stride), v3 = ntl(a + i + 3 * stride);
        nts(v0, b + i); nts(v1, b + i + stride); nts(v2, b + i + 2 * stride); nts(v3, b + i + 3 * stride);
    }
}
// one tile per block, contiguous (one-shot, like alex_step): 16 KiB per block
__global__ __launch_bounds__(256) void copy_tile_k(const float4* __restrict__ a, float4* __restrict__ b) {
    const size_t base = (size_t)blockIdx.x * 1024 + threadIdx.x * 4;
    const float4 v0 = a[base], v1 = a[base + 1], v2 = a[base + 2], v3 = a[base + 3];
    b[base] = v0; b[base + 1] = v1; b[base + 2] = v2; b[base + 3] = v3;
}
// one lane = 16 consecutive cells of one row; one block = 256 lanes = 16 rows x 256 cols (one tile)
template <bool NTL, bool NTS>
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
            const float4* src = (const float4*)(pE + (size_t)dd * HW + 4 * m);
            const float4 p4 = NTL ? ntl(src) : *src;
            acc += p4.x + p4.y + p4.z + p4.w;
        }
    }
    const uint32_t mix = (acc > 1e30f) ? 1u : 0u;
    const uint4 o0 = make_uint4(g4.x ^ v4.x ^ mix, g4.y ^ d4.y, g4.z ^ u4.z, g4.w);
    const uint4 o1 = make_uint4(a0.x, a0.y ^ mix, a0.z, a0.w);
    if (NTS) {
        nts(o0, (uint4*)(go + off));
        nts(o1, (uint4*)(ao + off));
        nts(a1, (uint4*)(ao + off + 8));
    } else {
        *(uint4*)(go + off) = o0;
        *(uint4*)(ao + off) = o1;
        *(uint4*)(ao + off + 8) = a1;
    }
}


// edge-slope pattern (25 B/cell: the 8-plane pattern with 4 slope planes, + planes 0..2 of row r+1, which
// the next row's lanes read as their own). COAL = 0: lane = 16 consecutive cells, 64 B contiguous per
// lane per plane (4 x dwordx4 at stride 64 B across lanes); COAL = 1: the plane's 1 KiB row segment is
// read as 4 instructions of 16 consecutive lanes x 16 B (lane-interleaved storage order).
template <int COAL>
__global__ __launch_bounds__(256) void alex_es_pattern_k(const uint8_t* __restrict__ g, uint8_t* __restrict__ go,
                                                         const int16_t* __restrict__ a, int16_t* __restrict__ ao,
                                                         const uint8_t* __restrict__ v, const uint8_t* __restrict__ d,
                                                         const uint8_t* __restrict__ du, const float* __restrict__ es,
                                                         int HW, int W) {
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
    const int row = (t * 16 + (threadIdx.x >> 4));
    const int q = threadIdx.x & 15;
    const float* pE = es + (size_t)e * 4 * HW + (size_t)row * W;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        const int plane = k < 4 ? k : 6 - k;
        const int rr = (k >= 4 && row + 1 < HW / W) ? 1 : 0;
        const float* base = pE + (size_t)plane * HW + (size_t)rr * W;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const float4* src = (const float4*)(base + (COAL ? (64 * m + 4 * q) : (16 * q + 4 * m)));
            const float4 p4 = *src;
            acc += p4.x + p4.y + p4.z + p4.w;
        }
    }
    const uint32_t mix = (acc > 1e30f) ? 1u : 0u;
    *(uint4*)(go + off) = make_uint4(g4.x ^ v4.x ^ mix, g4.y ^ d4.y, g4.z ^ u4.z, g4.w);
    *(uint4*)(ao + off) = make_uint4(a0.x, a0.y ^ mix, a0.z, a0.w);
    *(uint4*)(ao + off + 8) = a1;
}

// wave-sequential static layout: each wave's 1024 cells keep their static bytes (4 slope planes x 4 B + vd 1 B
// = 17 B/cell) in one contiguous 17 KiB block read front to back, 1 KiB per load instruction; the row r+1 slope
// planes (12 B/cell) come from the next wave's block (cache hits); dynamic grid u8 + age i16 read and written.
__global__ __launch_bounds__(256) void alex_wave_pattern_k(const uint8_t* __restrict__ g, uint8_t* __restrict__ go,
                                                           const int16_t* __restrict__ a, int16_t* __restrict__ ao,
                                                           const float4* __restrict__ st, int nwaves) {
    const int lane = threadIdx.x & 63;
    const int wv = blockIdx.x * 4 + (threadIdx.x >> 6);
    const size_t off = (size_t)wv * 1024 + lane * 16;
    const uint4 g4 = *(const uint4*)(g + off);
    const uint4 a0 = *(const uint4*)(a + off);
    const uint4 a1 = *(const uint4*)(a + off + 8);
    const float4* blk = st + (size_t)wv * 1088;  // 17 KiB = 1088 float4
    const float4* nxt = st + (size_t)min(wv + 1, nwaves - 1) * 1088;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 17; ++i) {
        const float4 v = blk[i * 64 + lane];
        acc += v.x + v.y + v.z + v.w;
    }
#pragma unroll
    for (int i = 0; i < 12; ++i) {
        const float4 v = nxt[i * 64 + lane];
        acc += v.x + v.y + v.z + v.w;
    }
    const uint32_t mix = (acc > 1e30f) ? 1u : 0u;
    *(uint4*)(go + off) = make_uint4(g4.x ^ mix, g4.y, g4.z, g4.w);
    *(uint4*)(ao + off) = make_uint4(a0.x, a0.y ^ mix, a0.z, a0.w);
    *(uint4*)(ao + off + 8) = a1;
}

#define TIME10(launch, out_ms) do { launch; CK(hipEventRecord(e0)); for (int i_ = 0; i_ < 10; ++i_) { launch; } \
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&out_ms, e0, e1)); out_ms /= 10; } while (0)

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
    printf("{");
    const int bl[3] = {2048, 8192, 32768};
    for (int k = 0; k < 3; ++k) {
        TIME10((copy_k<<<bl[k], 256>>>(A, B, n4)), ms);
        printf("\"copy_b%d_gbs\": %.1f, ", bl[k], 2.0 * nbytes / (ms * 1e-3) / 1e9);
        TIME10((copy4_k<<<bl[k], 256>>>(A, B, n4)), ms);
        printf("\"copy4_b%d_gbs\": %.1f, ", bl[k], 2.0 * nbytes / (ms * 1e-3) / 1e9);
        TIME10((copy4nt_k<<<bl[k], 256>>>(A, B, n4)), ms);
        printf("\"copy4nt_b%d_gbs\": %.1f, ", bl[k], 2.0 * nbytes / (ms * 1e-3) / 1e9);
    }
    TIME10((copy_tile_k<<<(unsigned)(n4 / 1024), 256>>>(A, B)), ms);
    printf("\"copy_tile_gbs\": %.1f, ", 2.0 * nbytes / (ms * 1e-3) / 1e9);
    TIME10((read_k<<<8192, 256>>>(A, out, n4)), ms);
    printf("\"read_gbs\": %.1f, ", 1.0 * nbytes / (ms * 1e-3) / 1e9);
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
    TIME10((alex_pattern_k<false, false><<<nblk, 256>>>(g, go, a, ao, v, d, du, ps, HW)), ms);
    printf("\"alex_pattern_ms\": %.4f, \"alex_pattern_gbs\": %.1f, ", ms, 41.0 * cells / (ms * 1e-3) / 1e9);
    TIME10((alex_pattern_k<true, false><<<nblk, 256>>>(g, go, a, ao, v, d, du, ps, HW)), ms);
    printf("\"alex_pattern_ntl_ms\": %.4f, ", ms);
    TIME10((alex_pattern_k<false, true><<<nblk, 256>>>(g, go, a, ao, v, d, du, ps, HW)), ms);
    printf("\"alex_pattern_nts_ms\": %.4f, ", ms);
    TIME10((alex_pattern_k<true, true><<<nblk, 256>>>(g, go, a, ao, v, d, du, ps, HW)), ms);
    printf("\"alex_pattern_ntls_ms\": %.4f, ", ms);
    TIME10((alex_es_pattern_k<0><<<nblk, 256>>>(g, go, a, ao, v, d, du, ps, HW, 256)), ms);
    printf("\"es_pattern_lane64_ms\": %.4f, \"es_pattern_lane64_gbs\": %.1f, ", ms, 25.0 * cells / (ms * 1e-3) / 1e9);
    TIME10((alex_es_pattern_k<1><<<nblk, 256>>>(g, go, a, ao, v, d, du, ps, HW, 256)), ms);
    printf("\"es_pattern_coal_ms\": %.4f, \"es_pattern_coal_gbs\": %.1f, ", ms, 25.0 * cells / (ms * 1e-3) / 1e9);
    // the same access pattern at the step kernel's occupancy: 36 KB of (unused) LDS per block -> 4 blocks / CU
    TIME10((alex_es_pattern_k<1><<<nblk, 256, 36864>>>(g, go, a, ao, v, d, du, ps, HW, 256)), ms);
    printf("\"es_pattern_coal_occ4_ms\": %.4f, ", ms);
    TIME10((alex_es_pattern_k<1><<<nblk, 256, 27648>>>(g, go, a, ao, v, d, du, ps, HW, 256)), ms);
    printf("\"es_pattern_coal_occ5_ms\": %.4f, ", ms);
    TIME10((alex_es_pattern_k<1><<<nblk, 256, 18432>>>(g, go, a, ao, v, d, du, ps, HW, 256)), ms);
    printf("\"es_pattern_coal_occ8_ms\": %.4f, ", ms);
    TIME10((alex_wave_pattern_k<<<nblk, 256>>>(g, go, a, ao, reinterpret_cast<const float4*>(ps), nblk * 4)), ms);
    printf("\"wave_seq_pattern_ms\": %.4f, \"wave_seq_pattern_gbs\": %.1f}\n", ms, 23.0 * cells / (ms * 1e-3) / 1e9);
    return 0;
}
