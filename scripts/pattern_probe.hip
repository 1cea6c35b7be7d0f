// pattern_probe.hip — r06: can the headline kernel's access-pattern floor itself move? gca_bench_march_pattern's loads
// and stores (alex_march_kernel<6, false, false, 1> at W = 256, 4096 x 256^2, 23.125 B / cell) in variants:
//   base      as the library probe: XCD-ordered blocks, 3 waves / SIMD, row r+1 in flight, non-temporal streams
//   ahead2    rows r+1 and r+2 in flight (twice the bytes in flight per wave)
//   occ4      4 waves / SIMD
//   plain     every load / store plain (no nt)
//   linear    blocks in launch order (no XCD remap)
//   sh32      32-row strips (half the waves, each twice as long)
// HIP events, mean of 10 launches after 3, three interleaved passes. Prints one JSON line (ms per launch).
// Build: hipcc -O3 --offload-arch=gfx950 scripts/pattern_probe.hip -o scripts/pattern_probe
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef float vf4 __attribute__((ext_vector_type(4)));
typedef uint32_t vu2 __attribute__((ext_vector_type(2)));

constexpr int E = 4096, H = 256, W = 256, R = 6, NF = 2 * R + 2;
constexpr size_t HW = (size_t)H * W, N = (size_t)E * HW;

template <class T>
__device__ __forceinline__ T ld(const T* p, bool nt) {
    return nt ? __builtin_nontemporal_load(p) : *p;
}
template <class T>
__device__ __forceinline__ void st(T v, T* p, bool nt) {
    if (nt) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <int SH, int AHEAD, int OCC, bool NT, bool XCD>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void probe_k(
    const uint8_t* __restrict__ g, uint8_t* __restrict__ go, const int16_t* __restrict__ a, int16_t* __restrict__ ao,
    const uint8_t* __restrict__ vd, const uint16_t* __restrict__ db, const vf4* __restrict__ es, int nwaves) {
    const int lane = threadIdx.x & 63, wl = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int lb = (int)blockIdx.x;
    if (XCD) {
        const int nb = (int)gridDim.x, xcd = (int)blockIdx.x & 7, slot = (int)blockIdx.x >> 3;
        const int qn8 = nb >> 3, rn8 = nb & 7;
        lb = (xcd < rn8 ? xcd * (qn8 + 1) : rn8 * (qn8 + 1) + (xcd - rn8) * qn8) + slot;
    }
    const int wv = lb * 4 + wl;
    if (wv >= nwaves) return;
    constexpr int SPE = H / SH;
    const int e = wv / SPE, s0 = (wv - e * SPE) * SH;
    const uint8_t* gE = g + (size_t)e * HW;
    const vf4* sE = es + (size_t)e * HW;  // 4 planes of HW f32 = HW vf4
    const uint8_t* vE = vd + (size_t)e * HW;
    const int16_t* aE = a + (size_t)e * HW;
    const uint16_t* dE = db + (size_t)e * (HW / 16);
    uint32_t ring[NF];
#pragma unroll
    for (int k = 0; k < NF; ++k) {
        const int r = s0 - R - 1 + k;
        ring[k] = (r >= 0 && r < H) ? *reinterpret_cast<const uint32_t*>(gE + r * W + 4 * lane) : 0u;
    }
    constexpr int NS = AHEAD + 2;
    vf4 sl[NS][4];
    uint32_t gn[AHEAD + 1], vv[AHEAD + 1], dd[AHEAD + 1];
    vu2 ag[AHEAD + 1];
    auto slopes = [&](int rs, vf4(&o)[4]) {
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = ld(&sE[(k * HW + (size_t)rs * W) / 4 + lane], NT);
    };
    auto issue = [&](int i) {
        const int r = s0 + i;
        const int rs = min(r + 1, H - 1);
        const uint32_t lo = (uint32_t)(r * W + 4 * lane);
        slopes(rs, sl[(i + 1) % NS]);
        const int rg = r + R + 1;
        gn[i % (AHEAD + 1)] = rg < H ? *reinterpret_cast<const uint32_t*>(gE + lo + (R + 1) * W) : 0u;
        vv[i % (AHEAD + 1)] = ld(reinterpret_cast<const uint32_t*>(vE + lo), NT);
        dd[i % (AHEAD + 1)] = dE[lo >> 4];
        ag[i % (AHEAD + 1)] = ld(reinterpret_cast<const vu2*>(aE + lo), NT);
    };
    slopes(s0, sl[0]);
#pragma unroll
    for (int i = 0; i < AHEAD; ++i) issue(i);
    uint32_t vsum = 0;
#pragma unroll
    for (int k = 0; k < NF; ++k) vsum += ring[k];
#pragma unroll
    for (int i = 0; i < SH; ++i) {
        if (i + AHEAD < SH) issue(i + AHEAD);
        const int r = s0 + i;
        const vf4* cur = sl[i % NS];
        const vf4* nxt = sl[(i + 1) % NS];
        float acc = cur[0].x + cur[1].y + cur[2].z + cur[3].w + nxt[0].y + nxt[1].z + nxt[2].w;
        acc += cur[0].w + cur[1].x + cur[2].y + cur[3].z + nxt[0].x + nxt[1].y + nxt[2].z;
        const uint32_t gnew = gn[i % (AHEAD + 1)];
        vsum += gnew - ring[i % NF];
        ring[i % NF] = gnew;
        const uint32_t x = vsum ^ vv[i % (AHEAD + 1)] ^ dd[i % (AHEAD + 1)];
        const uint32_t mix = (acc > 1e30f || x == 0x12345u) ? 1u : 0u;
        const uint32_t own = ring[(i + R + 1) % NF];
        const uint32_t lo = (uint32_t)(r * W + 4 * lane);
        st(own ^ mix, reinterpret_cast<uint32_t*>(go + (size_t)e * HW + lo), NT);
        vu2 aa = ag[i % (AHEAD + 1)];
        aa.x ^= mix;
        st(aa, reinterpret_cast<vu2*>(ao + (size_t)e * HW + lo), NT);
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
    uint8_t *g, *go, *vd;
    int16_t *a, *ao;
    uint16_t* db;
    vf4* es;
    if (hipMalloc(&g, N) || hipMalloc(&go, N) || hipMalloc(&vd, N) || hipMalloc(&a, 2 * N) || hipMalloc(&ao, 2 * N) ||
        hipMalloc(&db, N / 8) || hipMalloc(&es, 16 * N)) {
        printf("{\"error\": \"hipMalloc\"}\n");
        return 1;
    }
    (void)hipMemset(g, 1, N);
    (void)hipMemset(vd, 2, N);
    (void)hipMemset(a, 0, 2 * N);
    (void)hipMemset(db, 0, N / 8);
    (void)hipMemset(es, 0, 16 * N);
    printf("{\"cells\": %zu, \"bytes_per_cell\": 23.125", N);
#define P(NAME, SH, AH, OCC, NT, XCD) printf(", \"%s_p%d_ms\": %.4f", NAME, pass, \
        time_ms([&] { const int nw = E * (H / SH); hipLaunchKernelGGL((probe_k<SH, AH, OCC, NT, XCD>), dim3((nw + 3) / 4), \
                                    dim3(256), 0, 0, g, go, a, ao, vd, db, es, nw); }))
    for (int pass = 0; pass < 3; ++pass) {
        P("base", 16, 1, 3, true, true);
        P("ahead2", 16, 2, 3, true, true);
        P("occ4", 16, 1, 4, true, true);
        P("plain", 16, 1, 3, false, true);
        P("linear", 16, 1, 3, true, false);
        P("sh32", 32, 1, 3, true, true);
    }
    printf("}\n");
    return 0;
}
