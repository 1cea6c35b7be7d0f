// layout_probe.hip — r05: does the marching step's HBM layout bound it? The access pattern of alex_march_kernel
// (march_probe.hip's loop: one wave per SH-row strip of one env, lane = 4 columns, slope planes of row r+1 held from
// the previous iteration, the fire ring's rows R+1 ahead) with no rule arithmetic, in two layouts of the same
// 23.125 B/cell:
//   L = 0  the env's layout: 4 edge-slope planes (HW x f32 each), vd (HW u8), dousing bits, grid, ages as separate
//          arrays — 7 load streams per wave at 256 KiB-or-more strides;
//   L = 1  the read-only fields of a row interleaved in one block: [plane 0..3 of row r (4 KiB) | vd of row r
//          (256 B) | dousing bits of row r (32 B)], rows consecutive — one read-only stream per wave.
// FRAME: the fused frame's extra stream, each row's f32 RGB (12 B/cell) as three contiguous 1-KiB dwordx4 stores per
// wave (the pattern the frame's LDS transposition produces), at 2 / 3 / 4 waves per SIMD; POL = the frame stores'
// cache policy: 0 nt (the kernel's), 1 default, 2 sc1, 3 sc0 sc1, 4 sc1 nt.
// HIP events, mean of 10 launches after 3. Build: hipcc -O3 --offload-arch=gfx950 scripts/layout_probe.hip -o
// scripts/layout_probe. Prints one JSON line (ms per launch).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("{\"error\": \"%s\"}\n", hipGetErrorString(e_)); return 1; } } while (0)

typedef float vf4 __attribute__((ext_vector_type(4)));
typedef uint32_t vu2 __attribute__((ext_vector_type(2)));

constexpr int E = 4096, H = 256, W = 256, R = 6;
constexpr size_t HW = (size_t)H * W, N = (size_t)E * HW;
constexpr size_t ROWB = 4 * 4 * W + W + W / 8;  // L = 1: bytes of one row's read-only block (4384)

template <int SH, int L, int OCC, bool FRAME, int POL = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void probe_k(
    const uint8_t* __restrict__ g, uint8_t* __restrict__ go, const int16_t* __restrict__ a, int16_t* __restrict__ ao,
    const uint8_t* __restrict__ vd, const uint16_t* __restrict__ db, const vf4* __restrict__ es,
    const uint8_t* __restrict__ st, vf4* __restrict__ rgb) {
    constexpr int SPE = H / SH;
    const int wv = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int e = wv / SPE, s0 = (wv - e * SPE) * SH;
    const uint8_t* gE = g + e * HW;
    const vf4* sE = es + e * 4 * HW / 4;
    const uint8_t* stE = st + (size_t)e * H * ROWB;
    uint32_t ring[2 * R + 2];
#pragma unroll
    for (int k = 0; k < 2 * R + 2; ++k) {
        const int r = s0 - R - 1 + k;
        ring[k] = (r >= 0 && r < H) ? *reinterpret_cast<const uint32_t*>(gE + r * W + 4 * lane) : 0u;
    }
    vf4 sl[3][4];
    uint32_t gn[2], vv[2], dd[2];
    vu2 ag[2];
    const uint8_t* vE = vd + e * HW;
    const int16_t* aE = a + e * HW;
    const uint16_t* dE = db + e * (HW / 16);
    auto slopes = [&](int rs, vf4 (&o)[4]) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if constexpr (L == 0)
                o[k] = __builtin_nontemporal_load(&sE[(uint32_t)(k * HW + rs * W) / 4 + lane]);
            else
                o[k] = __builtin_nontemporal_load(reinterpret_cast<const vf4*>(stE + (size_t)rs * ROWB + k * 4 * W) + lane);
        }
    };
    auto issue = [&](int i, int slot) {
        const int r = s0 + i;
        const int rs = min(r + 1, H - 1);
        const uint32_t lo = (uint32_t)(r * W + 4 * lane);
        slopes(rs, sl[(slot + 1) % 3]);
        const int rg = r + R + 1;
        gn[slot & 1] = rg < H ? *reinterpret_cast<const uint32_t*>(gE + lo + (R + 1) * W) : 0u;
        if constexpr (L == 0) {
            vv[slot & 1] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(vE + lo));
            dd[slot & 1] = dE[lo >> 4];
        } else {
            const uint8_t* rb = stE + (size_t)r * ROWB + 16 * W;
            vv[slot & 1] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(rb) + lane);
            dd[slot & 1] = reinterpret_cast<const uint16_t*>(rb + W)[lane >> 2];
        }
        ag[slot & 1] = __builtin_nontemporal_load(reinterpret_cast<const vu2*>(aE + lo));
    };
    slopes(s0, sl[0]);
    issue(0, 0);
    uint32_t vsum = 0;
#pragma unroll
    for (int k = 0; k < 2 * R + 2; ++k) vsum += ring[k];
#pragma unroll
    for (int i = 0; i < SH; ++i) {
        if (i + 1 < SH) issue(i + 1, i + 1);
        const int r = s0 + i;
        const vf4* cur = sl[i % 3];
        const vf4* nxt = sl[(i + 1) % 3];
        float acc = cur[0].x + cur[1].y + cur[2].z + cur[3].w + nxt[0].y + nxt[1].z + nxt[2].w;
        acc += cur[0].w + cur[1].x + cur[2].y + cur[3].z + nxt[0].x + nxt[1].y + nxt[2].z;
        const uint32_t gnew = gn[i & 1];
        vsum += gnew - ring[i % (2 * R + 2)];
        ring[i % (2 * R + 2)] = gnew;
        const uint32_t x = vsum ^ vv[i & 1] ^ dd[i & 1];
        const uint32_t mix = (acc > 1e30f || x == 0x12345u) ? 1u : 0u;
        const uint32_t own = ring[(i + R + 1) % (2 * R + 2)];
        const uint32_t lo = (uint32_t)(r * W + 4 * lane);
        __builtin_nontemporal_store(own ^ mix, reinterpret_cast<uint32_t*>(go + e * HW + lo));
        vu2 aa = ag[i & 1];
        aa.x ^= mix;
        __builtin_nontemporal_store(aa, reinterpret_cast<vu2*>(ao + e * HW + lo));
        if constexpr (FRAME) {  // the row's f32 RGB, 3 KiB contiguous: three 1-KiB dwordx4 stores per wave
            vf4* fr = rgb + ((size_t)e * HW + (size_t)r * W) * 3 / 4;
            const float m = (float)(own ^ mix);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const vf4 v = (vf4){m, acc, m, (float)k};
                vf4* dst = fr + 64 * k + lane;
                if constexpr (POL == 0) __builtin_nontemporal_store(v, dst);
                else if constexpr (POL == 1) *dst = v;
                else if constexpr (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(dst), "v"(v) : "memory");
                else if constexpr (POL == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" :: "v"(dst), "v"(v) : "memory");
                else asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" :: "v"(dst), "v"(v) : "memory");
            }
        }
        __builtin_amdgcn_sched_barrier(0);
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

int main() {
    uint8_t *g, *go, *vd, *st;
    vf4* rgb;
    int16_t *a, *ao;
    uint16_t* db;
    vf4* es;
    CK(hipMalloc(&g, N));
    CK(hipMalloc(&go, N));
    CK(hipMalloc(&vd, N));
    CK(hipMalloc(&a, 2 * N));
    CK(hipMalloc(&ao, 2 * N));
    CK(hipMalloc(&db, N / 8));
    CK(hipMalloc(&es, 16 * N));
    CK(hipMalloc(&st, (size_t)E * H * ROWB));
    CK(hipMalloc(&rgb, 12 * N));
    CK(hipMemset(g, 1, N));
    CK(hipMemset(vd, 2, N));
    CK(hipMemset(a, 0, 2 * N));
    CK(hipMemset(db, 0, N / 8));
    CK(hipMemset(es, 0, 16 * N));
    CK(hipMemset(st, 0, (size_t)E * H * ROWB));
    printf("{\"cells\": %zu, \"bytes_per_cell\": 23.125", N);
#define P(SH, L, OCC, FR, POL) printf(", \"sh%d_L%d_occ%d%s_pol%d_ms\": %.4f", SH, L, OCC, FR ? "_frame" : "", POL, \
        time_ms([&] { hipLaunchKernelGGL((probe_k<SH, L, OCC, FR, POL>), dim3(E * (H / SH) / 4), dim3(256), 0, 0, g, go, \
                                         a, ao, vd, db, es, st, rgb); }))
    for (int rep = 0; rep < 2; ++rep) {
        P(16, 0, 3, false, 0);
        P(16, 0, 2, true, 0); P(16, 0, 2, true, 1); P(16, 0, 2, true, 2); P(16, 0, 2, true, 3); P(16, 0, 2, true, 4);
    }
    printf("}\n");
    return 0;
}
