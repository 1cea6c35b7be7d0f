// fetch_calib.hip — what FETCH_SIZE reports on gfx950 for each load width the marching Alexandridis kernel issues
// (MI355X_MICROARCH.md: 16 B/lane streaming reads count at exactly 1/2; other widths uncalibrated). Each kernel
// streams one 1 GiB buffer (beyond the 256 MiB Infinity Cache) once with a fixed per-lane width, each wave reading one
// contiguous 64 x width span per instruction, and folds the data into one store per thread. Run under
// `rocprofv3 --pmc FETCH_SIZE -- scripts/fetch_calib`: FETCH_SIZE (KB) x 1024 / 2^30 = the counted fraction.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/fetch_calib.hip -o scripts/fetch_calib
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr size_t BYTES = size_t(1) << 30;

template <class T>
__global__ __launch_bounds__(256) void stream_k(const T* __restrict__ src, uint32_t* __restrict__ out, size_t n) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const T v = src[i];
        uint32_t w[(sizeof(T) + 3) / 4] = {};
        __builtin_memcpy(w, &v, sizeof(T));
        for (size_t k = 0; k < (sizeof(T) + 3) / 4; ++k) acc ^= w[k];
    }
    out[blockIdx.x * (size_t)blockDim.x + threadIdx.x] = acc;
}

int main() {
    void* buf;
    uint32_t* out;
    if (hipMalloc(&buf, BYTES) != hipSuccess || hipMalloc(&out, 8192 * 256 * 4) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, BYTES);
    const dim3 g(8192), b(256);
    hipLaunchKernelGGL((stream_k<uint16_t>), g, b, 0, 0, (const uint16_t*)buf, out, BYTES / 2);
    hipLaunchKernelGGL((stream_k<uint32_t>), g, b, 0, 0, (const uint32_t*)buf, out, BYTES / 4);
    hipLaunchKernelGGL((stream_k<uint2>), g, b, 0, 0, (const uint2*)buf, out, BYTES / 8);
    hipLaunchKernelGGL((stream_k<uint4>), g, b, 0, 0, (const uint4*)buf, out, BYTES / 16);
    (void)hipDeviceSynchronize();
    printf("{\"bytes_per_kernel\": %zu, \"kernels\": [\"u16\", \"u32\", \"u32x2\", \"u32x4\"]}\n", BYTES);
    return 0;
}
