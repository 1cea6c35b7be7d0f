// march_probe.hip — would a marching Alexandridis step (one wave walks a 256-column strip of SH rows of one env,
// lane = 4 columns, no LDS, no barriers; row r+1's slope planes are held from the previous iteration instead of
// being re-read) stream faster than the tiled kernel (1.393 ms on the headline 4096 x 256^2)? Access pattern of
// that design with synthetic VALU work per row (VW dependent-chain instructions per lane, folded into the stores so
// nothing is dead), HIP events, mean of 10 launches. Per cell: slopes 16 B, grid 1 + 1, ages 2 + 2, vd 1, dousing
// bits 1/8 = 23.125 B. Build: hipcc -O3 --offload-arch=gfx950 scripts/march_probe.hip -o scripts/march_probe.
// Prints one JSON line (ms per launch).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("{\"error\": \"%s\"}\n", hipGetErrorString(e_)); return 1; } } while (0)

constexpr int E = 4096, H = 256, W = 256, R = 6;
constexpr size_t HW = (size_t)H * W, N = (size_t)E * HW;

// SH rows per wave, DEPTH rows of loads in flight ahead of the row being computed, VW VALU ops per row
template <int SH, int DEPTH, int VW>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) void march_k(const uint8_t* __restrict__ g, uint8_t* __restrict__ go,
                                               const int16_t* __restrict__ a, int16_t* __restrict__ ao,
                                               const uint8_t* __restrict__ vd, const uint16_t* __restrict__ db,
                                               const float4* __restrict__ es) {
    constexpr int SPE = H / SH;  // strips per env
    const int wv = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int e = wv / SPE, s0 = (wv - e * SPE) * SH;
    const uint8_t* gE = g + e * HW;
    const float4* sE = es + e * 4 * HW / 4;  // plane k row r: sE[(k * HW + r * W) / 4 + lane]
    // fire ring: rows s0 - R - 1 .. s0 + R in the prologue
    uint32_t ring[2 * R + 2];
#pragma unroll
    for (int k = 0; k < 2 * R + 2; ++k) {
        const int r = s0 - R - 1 + k;
        ring[k] = (r >= 0 && r < H) ? *reinterpret_cast<const uint32_t*>(gE + r * W + 4 * lane) : 0u;
    }
    float4 sl[DEPTH + 2][4];
    uint32_t gn[DEPTH + 1], vv[DEPTH + 1];
    uint2 ag[DEPTH + 1];
    uint32_t dd[DEPTH + 1];
    const uint8_t* vE = vd + e * HW;
    const int16_t* aE = a + e * HW;
    const uint16_t* dE = db + e * (HW / 16);
    auto issue = [&](int i, int slot) {  // loads of strip row i (slopes of row i + 1); 32-bit lane offsets
        const int r = s0 + i;
        const int rs = min(r + 1, H - 1);
        const uint32_t lo = (uint32_t)(r * W + 4 * lane);
#pragma unroll
        for (int k = 0; k < 4; ++k) sl[(slot + 1) % (DEPTH + 2)][k] = sE[(uint32_t)(k * HW + rs * W) / 4 + lane];
        const int rg = r + R + 1;
        gn[slot % (DEPTH + 1)] = rg < H ? *reinterpret_cast<const uint32_t*>(gE + lo + (R + 1) * W) : 0u;
        vv[slot % (DEPTH + 1)] = *reinterpret_cast<const uint32_t*>(vE + lo);
        ag[slot % (DEPTH + 1)] = *reinterpret_cast<const uint2*>(aE + lo);
        dd[slot % (DEPTH + 1)] = dE[lo >> 4];
    };
    // row s0's own planes
#pragma unroll
    for (int k = 0; k < 4; ++k) sl[0][k] = sE[(k * HW + s0 * W) / 4 + lane];
#pragma unroll
    for (int i = 0; i < DEPTH; ++i) issue(i, i);
    uint32_t vsum = 0;
#pragma unroll
    for (int k = 0; k < 2 * R + 2; ++k) vsum += ring[k];
#pragma unroll
    for (int i = 0; i < SH; ++i) {
        if (i + DEPTH < SH) issue(i + DEPTH, i + DEPTH);
        const int r = s0 + i;
        const float4* cur = sl[i % (DEPTH + 2)];
        const float4* nxt = sl[(i + 1) % (DEPTH + 2)];
        float acc = cur[0].x + cur[1].y + cur[2].z + cur[3].w + nxt[0].y + nxt[1].z + nxt[2].w;
        acc += cur[0].w + cur[1].x + cur[2].y + cur[3].z + nxt[0].x + nxt[1].y + nxt[2].z;
        const uint32_t gnew = gn[i % (DEPTH + 1)];
        vsum += gnew - ring[i % (2 * R + 2)];
        ring[i % (2 * R + 2)] = gnew;
        uint32_t x = vsum ^ vv[i % (DEPTH + 1)] ^ dd[i % (DEPTH + 1)];
        float f = acc;
#pragma unroll
        for (int t = 0; t < VW / 2; ++t) {  // opaque to the scheduler: two independent chains
            asm volatile("v_mad_u32_u24 %0, %0, %1, 7" : "+v"(x) : "v"(vv[0]));
            asm volatile("v_fma_f32 %0, %0, %1, 1.0" : "+v"(f) : "v"(acc));
        }
        const uint32_t mix = (f > 1e30f || x == 0x12345u) ? 1u : 0u;
        const uint32_t own = ring[(i + R + 1) % (2 * R + 2)];
        const uint32_t lo = (uint32_t)(r * W + 4 * lane);
        *reinterpret_cast<uint32_t*>(go + e * HW + lo) = own ^ mix;
        uint2 aa = ag[i % (DEPTH + 1)];
        aa.x ^= mix;
        *reinterpret_cast<uint2*>(ao + e * HW + lo) = aa;
        __builtin_amdgcn_sched_barrier(0);  // one row per iteration: no loads hoisted across rows
    }
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

// LDS bytes per block pin the occupancy: 0 = the kernel's own (4 waves / SIMD), 54 KiB = 3 blocks (12 waves) / CU
template <int SH, int DEPTH, int VW>
static float run(const uint8_t* g, uint8_t* go, const int16_t* a, int16_t* ao, const uint8_t* vd, const uint16_t* db,
                 const float4* es, int lds = 0) {
    const int blocks = E * (H / SH) / 4;
    return time_ms([&] { hipLaunchKernelGGL((march_k<SH, DEPTH, VW>), dim3(blocks), dim3(256), lds, 0, g, go, a, ao, vd, db, es); });
}

int main() {
    uint8_t *g, *go, *vd;
    int16_t *a, *ao;
    uint16_t* db;
    float4* es;
    CK(hipMalloc(&g, N));
    CK(hipMalloc(&go, N));
    CK(hipMalloc(&vd, N));
    CK(hipMalloc(&a, 2 * N));
    CK(hipMalloc(&ao, 2 * N));
    CK(hipMalloc(&db, N / 8));
    CK(hipMalloc(&es, 16 * N));
    CK(hipMemset(g, 1, N));
    CK(hipMemset(vd, 2, N));
    CK(hipMemset(a, 0, 2 * N));
    CK(hipMemset(db, 0, N / 8));
    CK(hipMemset(es, 0, 16 * N));
    printf("{\"cells\": %zu, \"bytes_per_cell\": 23.125", N);
#define P(SH, D, VW) printf(", \"sh%d_d%d_vw%d_ms\": %.4f", SH, D, VW, run<SH, D, VW>(g, go, a, ao, vd, db, es))
#define P3(SH, D, VW) printf(", \"sh%d_d%d_vw%d_occ3_ms\": %.4f", SH, D, VW, run<SH, D, VW>(g, go, a, ao, vd, db, es, 54 * 1024))
    P(16, 1, 0); P(16, 2, 0); P(16, 2, 600); P(16, 2, 800); P(16, 2, 1000);
    P3(16, 1, 0); P3(16, 2, 0); P3(16, 2, 600); P3(16, 2, 800); P3(16, 2, 1000);
    printf("}\n");
    return 0;
}
