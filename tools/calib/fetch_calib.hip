// FETCH_SIZE / WRITE_SIZE calibration for the access widths the step kernels use (round 5).
// MI355X_MICROARCH.md calibrates 16-B-per-lane streaming reads (FETCH_SIZE = half the bytes) and
// stores (exact); other widths are uncalibrated. Each kernel here moves a known byte count:
//   rd16: 16 B per lane loads, rd4: 4 B per lane loads, rd1: 1 B per lane loads,
//   wr16 / wr4 / wr1: the same widths stored.  1 GiB buffers (past the 256 MiB MALL).
// Build: hipcc -O3 --offload-arch=gfx950 -o fetch_calib fetch_calib.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <class T>
__global__ void __launch_bounds__(256) rd(const T* __restrict__ src, size_t n, uint32_t* sink) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const T v = src[i];
        if constexpr (sizeof(T) == 16) acc ^= v.x ^ v.y ^ v.z ^ v.w;
        else acc ^= (uint32_t)v;
    }
    if (acc == 0x12345678u) sink[0] = acc;  // (keeps the loads; never true for the zero-filled buffer)
}

template <class T>
__global__ void __launch_bounds__(256) wr(T* __restrict__ dst, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        T v{};
        if constexpr (sizeof(T) == 16) v.x = (uint32_t)i;
        else v = (T)i;
        dst[i] = v;
    }
}

int main() {
    const size_t bytes = (size_t)1 << 30;
    void *a = nullptr, *s = nullptr;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&s, 64) != hipSuccess) return 1;
    (void)hipMemset(a, 0, bytes);
    (void)hipDeviceSynchronize();
    const int g = 256 * 8 * 4;
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(rd<uint4>, dim3(g), dim3(256), 0, 0, (const uint4*)a, bytes / 16, (uint32_t*)s);
        hipLaunchKernelGGL(rd<uint32_t>, dim3(g), dim3(256), 0, 0, (const uint32_t*)a, bytes / 4, (uint32_t*)s);
        hipLaunchKernelGGL(rd<uint8_t>, dim3(g), dim3(256), 0, 0, (const uint8_t*)a, bytes, (uint32_t*)s);
        hipLaunchKernelGGL(wr<uint4>, dim3(g), dim3(256), 0, 0, (uint4*)a, bytes / 16);
        hipLaunchKernelGGL(wr<uint32_t>, dim3(g), dim3(256), 0, 0, (uint32_t*)a, bytes / 4);
        hipLaunchKernelGGL(wr<uint8_t>, dim3(g), dim3(256), 0, 0, (uint8_t*)a, bytes);
    }
    const hipError_t e = hipDeviceSynchronize();
    printf("calibration kernels done: %s (each moves %zu bytes)\n", hipGetErrorString(e), bytes);
    (void)hipFree(a);
    (void)hipFree(s);
    return e == hipSuccess ? 0 : 1;
}
