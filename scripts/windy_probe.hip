// windy_probe.hip — what separates the Windy CA step (BASELINE config 2: 1024 x 256^2, 64 MiB in + 64 MiB out,
// 29.5-30.5 us) from a same-size device copy (21.5 us)? Access-pattern probes with trivial compute, HIP events,
// mean of 50 launches each after 10 warm-ups. Build: hipcc -O3 --offload-arch=gfx950 scripts/windy_probe.hip -o
// scripts/windy_probe. Prints one JSON line (microseconds per launch).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("{\"error\": \"%s\"}\n", hipGetErrorString(e_)); return 1; } } while (0)

constexpr int E = 1024, H = 256, W = 256;
constexpr size_t N = (size_t)E * H * W;

__global__ void empty_k(int* p) { if (p && threadIdx.x == 1023) p[0] = 1; }

// grid-stride 16-B copy (what torch's copy_ does, roughly)
__global__ __launch_bounds__(256) void copy16_k(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

// the rows kernel's map: block = 4 waves, wave = a strip of SH rows of one env, lane = 4 columns (one dword);
// HALO: rows s0-1 .. s0+SH loaded (SH + 2 loads), SH stores; all loads issued first
template <int SH, bool HALO>
__global__ __launch_bounds__(256) void rows4_k(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int bpe) {
    const int env = blockIdx.x / bpe, sblk = blockIdx.x - env * bpe;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int s0 = (sblk * 4 + wave) * SH;
    if (s0 >= H) return;
    const uint8_t* S = src + (size_t)env * H * W + 4 * lane;
    uint8_t* D = dst + (size_t)env * H * W + 4 * lane;
    uint32_t v[SH + 2];
#pragma unroll
    for (int k = 0; k < SH + 2; ++k) {
        const int r = s0 - 1 + k;
        v[k] = (HALO || (k >= 1 && k <= SH)) && r >= 0 && r < H ? *reinterpret_cast<const uint32_t*>(S + r * W) : 0u;
    }
#pragma unroll
    for (int k = 0; k < SH; ++k) *reinterpret_cast<uint32_t*>(D + (s0 + k) * W) = v[k + 1] ^ v[k] ^ v[k + 2];
}

// the same map with 16 columns per lane: a wave covers 4 image rows x 256 columns per instruction
template <int SH>
__global__ __launch_bounds__(256) void rows16_k(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int bpe) {
    const int env = blockIdx.x / bpe, sblk = blockIdx.x - env * bpe;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int s0 = (sblk * 4 + wave) * SH;  // SH rows per wave, 4 rows per instruction
    const int rl = lane >> 4, c = 16 * (lane & 15);
    const uint8_t* S = src + (size_t)env * H * W + c;
    uint8_t* D = dst + (size_t)env * H * W + c;
    uint4 v[SH / 4 + 2];
#pragma unroll
    for (int k = 0; k < SH / 4 + 2; ++k) {
        const int r = s0 - 4 + 4 * k + rl;
        v[k] = r >= 0 && r < H ? *reinterpret_cast<const uint4*>(S + r * W) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < SH / 4; ++k) {
        const uint4 a = v[k + 1], b = v[k], d = v[k + 2];
        *reinterpret_cast<uint4*>(D + (s0 + 4 * k + rl) * W) = make_uint4(a.x ^ b.x ^ d.x, a.y ^ b.y ^ d.y,
                                                                          a.z ^ b.z ^ d.z, a.w ^ b.w ^ d.w);
    }
}

// persistent: G blocks walk the strips of rows4_k<16, true> grid-stride
__global__ __launch_bounds__(256) void rows4_persist_k(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                       int nblocks) {
    constexpr int SH = 16;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int b = blockIdx.x; b < nblocks; b += gridDim.x) {
        const int env = b >> 2, sblk = b & 3;
        const int s0 = (sblk * 4 + wave) * SH;
        const uint8_t* S = src + (size_t)env * H * W + 4 * lane;
        uint8_t* D = dst + (size_t)env * H * W + 4 * lane;
        uint32_t v[SH + 2];
#pragma unroll
        for (int k = 0; k < SH + 2; ++k) {
            const int r = s0 - 1 + k;
            v[k] = r >= 0 && r < H ? *reinterpret_cast<const uint32_t*>(S + r * W) : 0u;
        }
#pragma unroll
        for (int k = 0; k < SH; ++k) *reinterpret_cast<uint32_t*>(D + (s0 + k) * W) = v[k + 1] ^ v[k] ^ v[k + 2];
    }
}

template <class F>
static float time_us(F launch) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 10; ++i) launch();
    (void)hipEventRecord(a);
    for (int i = 0; i < 50; ++i) launch();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms * 1000.0f / 50.0f;
}

int main() {
    uint8_t *src, *dst;
    CK(hipMalloc(&src, N));
    CK(hipMalloc(&dst, N));
    CK(hipMemset(src, 3, N));
    const int bpe16 = 4;  // 16-row strips, 4 waves per block: 64 rows per block
    const float t_empty = time_us([&] { hipLaunchKernelGGL(empty_k, dim3(E * bpe16), dim3(256), 0, 0, nullptr); });
    const float t_copy16 = time_us([&] {
        hipLaunchKernelGGL(copy16_k, dim3(4096), dim3(256), 0, 0, (const uint4*)src, (uint4*)dst, N / 16);
    });
    const float t_memcpy = time_us([&] { (void)hipMemcpyAsync(dst, src, N, hipMemcpyDeviceToDevice, 0); });
    const float t_rows4 = time_us([&] {
        hipLaunchKernelGGL((rows4_k<16, true>), dim3(E * bpe16), dim3(256), 0, 0, src, dst, bpe16);
    });
    const float t_rows4_nohalo = time_us([&] {
        hipLaunchKernelGGL((rows4_k<16, false>), dim3(E * bpe16), dim3(256), 0, 0, src, dst, bpe16);
    });
    const float t_rows4_sh64 = time_us([&] {
        hipLaunchKernelGGL((rows4_k<64, true>), dim3(E), dim3(256), 0, 0, src, dst, 1);
    });
    const float t_rows16 = time_us([&] {
        hipLaunchKernelGGL((rows16_k<16>), dim3(E * 4), dim3(256), 0, 0, src, dst, 4);
    });
    const float t_rows16_sh64 = time_us([&] {
        hipLaunchKernelGGL((rows16_k<64>), dim3(E), dim3(256), 0, 0, src, dst, 1);
    });
    float t_persist[3];
    const int grids[3] = {1024, 2048, 3072};
    for (int g = 0; g < 3; ++g)
        t_persist[g] = time_us([&] {
            hipLaunchKernelGGL(rows4_persist_k, dim3(grids[g]), dim3(256), 0, 0, src, dst, E * bpe16);
        });
    printf("{\"empty_4096_blocks_us\": %.2f, \"copy16_us\": %.2f, \"memcpy_us\": %.2f, \"rows4_halo_us\": %.2f, "
           "\"rows4_nohalo_us\": %.2f, \"rows4_sh64_us\": %.2f, \"rows16_us\": %.2f, \"rows16_sh64_us\": %.2f, "
           "\"rows4_persist_1024_us\": %.2f, \"rows4_persist_2048_us\": %.2f, \"rows4_persist_3072_us\": %.2f}\n",
           t_empty, t_copy16, t_memcpy, t_rows4, t_rows4_nohalo, t_rows4_sh64, t_rows16, t_rows16_sh64, t_persist[0],
           t_persist[1], t_persist[2]);
    return 0;
}
