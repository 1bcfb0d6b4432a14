// Micro-benchmark: cost of one MT19937 raw draw per lane in the reset kernel's
// stream generator (ChainMT), alone and with the tile/raw bookkeeping.
// hipcc -O3 --offload-arch=gfx950 -I element-crush-gym_amd/csrc tools/ubench/chain_bench.hip -o /tmp/chain_bench
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "m3_rules.hpp"

using namespace m3;

template <int MODE>
__global__ void __launch_bounds__(64) k_chain(const uint32_t* seeds, uint32_t* out, uint8_t* raw, int draws) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    const uint32_t s = seeds[i];
    ChainMT g;
    g.init(s, mt_state397(s));
    uint32_t acc = 0, cur0 = 0, cur1 = 0, cur2 = 0, nt = 0, pk = 0;
    for (int k = 0; k < draws; ++k) {
        const uint32_t v = g.next32();
        if (MODE == 0) {
            acc ^= v;
        } else {
            const uint32_t t = v & 7u;
            const bool ok = t <= 5u;
            if (MODE >= 2) {
                pk |= (v & 0xFFu) << (8 * (k & 3));
                if ((k & 3) == 3) {
                    reinterpret_cast<uint32_t*>(raw)[(size_t)i * 64 + (k >> 2) % 64] = pk;
                    pk = 0;
                }
            }
            if (ok) {
                const uint32_t val = t + 1u, sh = nt & 31u;
                cur0 |= (val & 1u) << sh;
                cur1 |= ((val >> 1) & 1u) << sh;
                cur2 |= ((val >> 2) & 1u) << sh;
                ++nt;
                if ((nt & 31u) == 0u) {
                    acc ^= cur0 ^ (cur1 << 1) ^ (cur2 << 2);
                    cur0 = cur1 = cur2 = 0;
                }
            }
        }
    }
    out[i] = acc ^ cur0 ^ cur1 ^ cur2 ^ nt ^ g.k;
}

template <int MODE>
float run(int blocks, int draws, const uint32_t* d_seeds, uint32_t* d_out, uint8_t* d_raw) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(k_chain<MODE>, dim3(blocks), dim3(64), 0, 0, d_seeds, d_out, d_raw, draws);
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_chain<MODE>, dim3(blocks), dim3(64), 0, 0, d_seeds, d_out, d_raw, draws);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main() {
    const int maxb = 4096;
    uint32_t* d_seeds;
    uint32_t* d_out;
    uint8_t* d_raw;
    hipMalloc(&d_seeds, maxb * 64 * 4);
    hipMalloc(&d_out, maxb * 64 * 4);
    hipMalloc(&d_raw, (size_t)maxb * 64 * 256);
    uint32_t* h = new uint32_t[maxb * 64];
    for (int i = 0; i < maxb * 64; ++i) h[i] = 1000 + i;
    hipMemcpy(d_seeds, h, maxb * 64 * 4, hipMemcpyHostToDevice);
    for (int draws : {226, 624}) {
        for (int blocks : {256, 1024, 4096}) {
            const float m0 = run<0>(blocks, draws, d_seeds, d_out, d_raw);
            const float m1 = run<1>(blocks, draws, d_seeds, d_out, d_raw);
            const float m2 = run<2>(blocks, draws, d_seeds, d_out, d_raw);
            printf("draws %3d waves %5d: rng only %8.1f us (%6.1f ns/draw)  +tiles %8.1f us  +raw stores %8.1f us\n",
                   draws, blocks, m0 * 1e3, m0 * 1e6 / draws, m1 * 1e3, m2 * 1e3);
        }
    }
    return 0;
}
