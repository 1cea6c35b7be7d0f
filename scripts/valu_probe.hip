// valu_probe.hip — relative VALU issue cost of the instructions the CA kernels lean on (gfx950), measured, not
// assumed: every kernel runs 8 independent dependency chains per lane of one instruction kind at full occupancy
// (2048 blocks x 256 threads), 256 iterations x 8 ops; cost = time / time of the v_add_u32 kernel. Build:
// hipcc -O3 --offload-arch=gfx950 scripts/valu_probe.hip -o scripts/valu_probe. Prints one JSON line.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int IT = 256;

#define CHAINS8(T, init, body)                                                        \
    T x0 = init(0), x1 = init(1), x2 = init(2), x3 = init(3), x4 = init(4), x5 = init(5), \
      x6 = init(6), x7 = init(7);                                                     \
    for (int i = 0; i < IT; ++i) {                                                    \
        body(x0); body(x1); body(x2); body(x3); body(x4); body(x5); body(x6); body(x7);  \
    }

__global__ __launch_bounds__(256) void k_add(uint32_t* out, uint32_t s) {
    auto init = [&](int j) { return (uint32_t)(threadIdx.x + j); };
    auto body = [&](uint32_t& x) { asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "s"(s)); };
    CHAINS8(uint32_t, init, body)
    out[blockIdx.x * 256 + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
}
__global__ __launch_bounds__(256) void k_mad64(uint32_t* out, uint32_t s) {
    auto init = [&](int j) { return (uint64_t)(threadIdx.x + j); };
    auto body = [&](uint64_t& x) {
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(x) : "v"((uint32_t)x), "s"(s) : "vcc");
    };
    CHAINS8(uint64_t, init, body)
    out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7);
}
__global__ __launch_bounds__(256) void k_mullo(uint32_t* out, uint32_t s) {
    auto init = [&](int j) { return (uint32_t)(threadIdx.x + j); };
    auto body = [&](uint32_t& x) { asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "s"(s)); };
    CHAINS8(uint32_t, init, body)
    out[blockIdx.x * 256 + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
}
__global__ __launch_bounds__(256) void k_mulhi(uint32_t* out, uint32_t s) {
    auto init = [&](int j) { return (uint32_t)(threadIdx.x + j); };
    auto body = [&](uint32_t& x) { asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "s"(s)); };
    CHAINS8(uint32_t, init, body)
    out[blockIdx.x * 256 + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
}
__global__ __launch_bounds__(256) void k_mul24(uint32_t* out, uint32_t s) {
    auto init = [&](int j) { return (uint32_t)(threadIdx.x + j); };
    auto body = [&](uint32_t& x) { asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "s"(s)); };
    CHAINS8(uint32_t, init, body)
    out[blockIdx.x * 256 + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
}
__global__ __launch_bounds__(256) void k_bitop3(uint32_t* out, uint32_t s) {
    auto init = [&](int j) { return (uint32_t)(threadIdx.x + j); };
    auto body = [&](uint32_t& x) { asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(x) : "s"(s)); };
    CHAINS8(uint32_t, init, body)
    out[blockIdx.x * 256 + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
}
__global__ __launch_bounds__(256) void k_rcp(uint32_t* out, uint32_t s) {
    auto init = [&](int j) { return (float)(threadIdx.x + j + 1); };
    auto body = [&](float& x) { asm volatile("v_rcp_f32 %0, %0" : "+v"(x)); };
    CHAINS8(float, init, body)
    out[blockIdx.x * 256 + threadIdx.x] = __float_as_uint(x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7);
}
__global__ __launch_bounds__(256) void k_pkmul(uint32_t* out, uint32_t s) {
    auto init = [&](int j) { return (f2){(float)(threadIdx.x + j), 1.0f}; };
    auto body = [&](f2& x) { asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(x) : "v"((f2){1.0f, 1.0f})); };
    CHAINS8(f2, init, body)
    out[blockIdx.x * 256 + threadIdx.x] = __float_as_uint(x0.x + x1.x + x2.x + x3.x + x4.x + x5.x + x6.x + x7.x);
}
__global__ __launch_bounds__(256) void k_mulf(uint32_t* out, uint32_t s) {
    auto init = [&](int j) { return (float)(threadIdx.x + j); };
    auto body = [&](float& x) { asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x) : "s"(s)); };
    CHAINS8(float, init, body)
    out[blockIdx.x * 256 + threadIdx.x] = __float_as_uint(x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7);
}
__global__ __launch_bounds__(256) void k_dpp(uint32_t* out, uint32_t s) {
    auto init = [&](int j) { return (uint32_t)(threadIdx.x + j); };
    auto body = [&](uint32_t& x) {
        asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(x));
    };
    CHAINS8(uint32_t, init, body)
    out[blockIdx.x * 256 + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
}
__global__ __launch_bounds__(256) void k_cvtub(uint32_t* out, uint32_t s) {
    auto init = [&](int j) { return (float)(threadIdx.x + j); };
    auto body = [&](float& x) { asm volatile("v_cvt_f32_ubyte0 %0, %0" : "+v"(x)); };
    CHAINS8(float, init, body)
    out[blockIdx.x * 256 + threadIdx.x] = __float_as_uint(x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7);
}

template <class K>
static float time_ms(K k, uint32_t* out) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(k, dim3(2048), dim3(256), 0, 0, out, 3u);
    (void)hipEventRecord(a);
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(k, dim3(2048), dim3(256), 0, 0, out, 3u);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / 20;
}

int main() {
    uint32_t* out;
    if (hipMalloc(&out, 2048 * 256 * 4) != hipSuccess) return 1;
    const float base = time_ms(k_add, out);
    // wave-instructions per SIMD: 2048 blocks x 4 waves x IT x 8 / 1024 SIMDs; cycles from the v_add kernel at 2
    // cycles per wave64 instruction (SIMD-32)
    const double winst = 2048.0 * 4 * IT * 8 / 1024.0;
    printf("{\"v_add_u32_ms\": %.4f, \"clock_ghz_if_add_is_2cyc\": %.3f, \"rel\": {", base, winst * 2 / (base * 1e6));
    const char* names[] = {"v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mul_u32_u24", "v_bitop3_b32", "v_rcp_f32",
                           "v_pk_mul_f32", "v_mul_f32", "v_mov_b32_dpp", "v_cvt_f32_ubyte0"};
    const float t[] = {time_ms(k_mad64, out), time_ms(k_mullo, out), time_ms(k_mulhi, out), time_ms(k_mul24, out),
                       time_ms(k_bitop3, out), time_ms(k_rcp, out), time_ms(k_pkmul, out), time_ms(k_mulf, out),
                       time_ms(k_dpp, out), time_ms(k_cvtub, out)};
    for (int i = 0; i < 10; ++i) printf("%s\"%s\": %.3f", i ? ", " : "", names[i], t[i] / base);
    printf("}}\n");
    return 0;
}
