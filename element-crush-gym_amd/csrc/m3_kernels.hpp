// m3_kernels.hpp -- the gfx950 kernels of libm3.so and their host-side launchers.
//
// Included by m3_api.hip (the C ABI) and by m3_inst.hip, which is compiled once
// per board configuration (-DM3_INST=<id>, see CF_<id> below) and explicitly
// instantiates that configuration's launchers -- and with them its kernels --
// so the configurations compile in parallel translation units. A single-TU
// build (m3_api.hip without -DM3_SPLIT_TU) instantiates everything implicitly.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/m3.h"
#include "m3_rules.hpp"

using namespace m3;

// defined in m3_api.hip: sets the thread-local m3_last_error() message, returns code
int set_err(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

namespace {


#define HIP_TRY(expr)                                                                            \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess)                                                                    \
            return set_err(M3_ERR_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                           __LINE__);                                                            \
    } while (0)

#define RCCL_TRY(expr)                                                                            \
    do {                                                                                          \
        ncclResult_t r_ = (expr);                                                                 \
        if (r_ != ncclSuccess) return set_err(M3_ERR_RCCL, "%s: %s", #expr, ncclGetErrorString(r_)); \
    } while (0)

#define CHECK_ARG(cond, msg)                                       \
    do {                                                           \
        if (!(cond)) return set_err(M3_ERR_INVALID, "%s", (msg)); \
    } while (0)

constexpr int BLOCK = 256;
constexpr int FIX_BLOCK = 64;
constexpr int FIX_GRID = 16;       // step fixup almost never has work: few blocks schedule fast
constexpr int INIT_FIX_BLOCK = 64;
constexpr int INIT_BLOCK = 64;
// active lanes of the one-board-per-lane fix / reset kernels (KS::BPW: one for the 32 x 32 frame)
// (M3_WIDE_FRAME_LANES: an experiment knob, 64 to run the 32 x 32 frame one board per LANE again)
#ifndef M3_WIDE_FRAME_LANES
#define M3_WIDE_FRAME_LANES 1
#endif
template <class CF>
constexpr uint32_t lanes_for() { return CF::W > 8 ? (uint32_t)M3_WIDE_FRAME_LANES : 64u; }
// 9x9: k_init redoes its few >= 624-draw resets in-wave (wave_reset); 16x16
// resets go straight to k_init_fix_lane (most need >= 624 draws)
template <class CF>
constexpr bool INIT_INLINE_FIX = CF::N <= 128;
constexpr int MAX_SHARDS = 8;  // env board shards (one HIP stream each)
// k_init's lockstep draw budget when it may defer (env prefetch): 9x9x6 resets
// past 454 draws (~4 %: the third chain level and the second block) go to
// k_init_coop, so a wave no longer runs to its slowest lane's ~600 draws
#ifndef M3_RESET_KCAP
#define M3_RESET_KCAP 454
#endif
constexpr uint32_t RESET_KCAP = M3_RESET_KCAP;
// grid caps of the env-prefetch reset kernels (0: sized by the queue's usual length), see launch_init
// The prefetch reset launches are sized for n / PF_DIV queued resets of the shard (grid-strided beyond
// that; blocks past the queue's length exit at once). Round 6: every board's episode ends on the same
// step (the bench's 20-move episodes all start together), so one step in 20 queues the whole shard;
// sized for n / 8 (round 5) that burst ran ~1 wave per SIMD for 1.3-1.8 ms and held the step that
// reuses the queue ~1 ms. A/B (driver command): 9x9 n / 1 2.53-2.55 vs 2.41-2.42 G env-steps/s,
// 16x16 n / 2 0.79-0.80 vs 0.78 (n / 1 0.76-0.79). Frame shapes keep n / 8.
#ifndef M3_PF_DIV
#define M3_PF_DIV 1
#endif
#ifndef M3_PF_DIV16
#define M3_PF_DIV16 2
#endif
#ifndef M3_COOP_GMAX  // most blocks of a prefetch k_init_coop launch (one deferred reset per wave at a time)
#define M3_COOP_GMAX 4096
#endif
#ifndef M3_PF_GRID
#define M3_PF_GRID 0
#endif
#ifndef M3_PF_COOP_GRID
#define M3_PF_COOP_GRID 0
#endif
// 16x16x8 resets: 1 = lane-per-board on the two-block register chain (k_init_chain2),
// 0 = lane-per-board FullMT in scratch (k_init_fix_lane)
#ifndef M3_RESET16_CHAIN2
#define M3_RESET16_CHAIN2 0
#endif
// A reset stops after this many rounds of BoardV2.__init__'s redraw loop (boardv2.py:23-27) and
// flags M3_FLAG_RESET_CAP: only two-colour boards get near it (a 16x16x2 reset can need more than
// 10,000 rounds; the reference keeps going), and a GPU lane must end.
constexpr uint32_t RESET_ROUND_CAP = 1u << 14;

// Per-shape step-kernel geometry: boards (lanes) per workgroup and the
// match-group table capacity, sized so staging + table fit the 160 KB LDS.
// One wave per workgroup: the boards of a wave are staged through its own LDS
// slice, so a wave that finishes early never waits at a barrier for the
// workgroup's slowest wave (cascade depth varies a lot between boards) and its
// slot is refilled at once.
template <class CF>
struct KS {
    static constexpr int B = 64;
    static_assert(B == 64, "one-wave workgroups: lds_sync() orders a single wave's LDS accesses");
    // match groups in LDS per lane (more spill to a global pool): 9x9 6 (9 KB per wave, +0.8 %,
    // gpurun_out/r05aj), 16x16 4 (past the staging area a larger table costs occupancy)
    static constexpr int GCAP = CF::N <= 128 ? 6 : 4;
    // boards per wave: 64 (one per lane), but ONE for the 32 x 32 frame. Those kernels carry
    // ~2,500 SGPR spills through VGPR lanes, and with several lanes active some boards came out
    // wrong only in company (32x32x8 steps: 92 of 689; each exact alone) -- the lane interference
    // DESIGN.md §4 describes for the 16 x 16 frame. One active lane per wave has no divergence.
    static constexpr int BPW = CF::W > 8 ? M3_WIDE_FRAME_LANES : B;
#ifndef M3_STEP_WPS
#define M3_STEP_WPS 4
#endif
    // k_env_step waves per SIMD the register allocation is bounded for (16x16:
    // 2, with 708 B of spill, +7 % over 1 once resets stopped binding)
#ifndef M3_STEP_WPS16
#define M3_STEP_WPS16 2
#endif
    // frame shapes (run-time board shape, FCfg): 1 wave/SIMD. Their uniform shape masks take
    // ~100 SGPRs and spill into VGPR lanes; at 2 waves/SIMD those VGPRs spilled to scratch in
    // turn and divergent lanes of a wave corrupted each other's results (rollouts at 10x8x9,
    // tools/dbg); with 512 registers per lane nothing reaches scratch.
#ifndef M3_STEP_WPS_FRAME
#define M3_STEP_WPS_FRAME 1
#endif
    static constexpr int STEP_WPS = CF::DYN ? M3_STEP_WPS_FRAME : (CF::N > 128 ? M3_STEP_WPS16 : M3_STEP_WPS);
    // k_env_cont: bounded like the step kernel it runs beside (a 2-waves/SIMD
    // build without spills measured 4 % slower overall: its waves take register
    // file the other shard's step waves need)
#ifndef M3_CONT_WPS
#define M3_CONT_WPS M3_STEP_WPS
#endif
    static constexpr int CONT_WPS = CF::N > 128 ? 1 : M3_CONT_WPS;
    // spill pool records per shard (32 x 32 frame: a record is 86 KB; fewer, the rest recompute)
    static constexpr uint32_t SPILL_RECORDS = CF::W > 8 ? 256 : 4096;
    // The env step's RNG is the register-only MT19937 chain from the board's
    // (seed, mt[397]) -- 4 B of per-board state (a per-board stream cache of
    // the first raw outputs, built by the reset, measured equal at 9x9 and 2x
    // slower at 16x16; removed in round 3).
    // 16x16: one chain level (draws < 227; a step needing more -- a near-full
    // board refill -- goes to k_env_fix), five fewer VGPRs live through the
    // cascade, +2.5 %. 9x9: the full three-level chain; the one-level build
    // came out 16 % slower (A/B gpurun_out/ab3), the register allocation of
    // the 3-waves/SIMD bound shifts with it.
    using Chain = std::conditional_t<(CF::N > 128), ChainMT1, ChainMT>;
    using Rng = Chain;
// Issue priorities against the prefetch resets that share the SIMDs (A/B knobs, off by default):
// M3_STEP_PRIO -- s_setprio of the k_env_step waves; M3_STREAM_PRIO -- the shard's step stream at
// the device's greatest stream priority and its prefetch stream at the least.
#ifndef M3_STEP_PRIO
#define M3_STEP_PRIO 0
#endif
#ifndef M3_STREAM_PRIO
#define M3_STREAM_PRIO 0
#endif
#ifndef M3_CASCADE_LIMIT
#define M3_CASCADE_LIMIT 2
#endif
    // k_env_step runs at most this many cascade iterations per step (-1: no
    // bound); longer steps are finished by k_env_cont (see there)
    // (16x16: off -- the continuation launch cost more than it saved:
    // 0.364 vs 0.337 G env-steps/s at 1 wave/SIMD, 0.391 vs 0.384 at 2)
#ifndef M3_CASCADE_LIMIT16
#define M3_CASCADE_LIMIT16 -1
#endif
    static constexpr int CASCADE_LIMIT = CF::N > 128 ? M3_CASCADE_LIMIT16 : M3_CASCADE_LIMIT;
};

// LDS pointers carry their address space, so table accesses compile to ds_*
// instructions: a generic pointer that may point at either the LDS table or
// the global spill pool made the compiler emit flat loads, and every wait on a
// flat load also waits for all of the wave's global memory traffic.
#ifdef __HIP_DEVICE_COMPILE__
#define M3_LDS_AS __attribute__((address_space(3)))
#else
#define M3_LDS_AS
#endif
typedef M3_LDS_AS uint32_t lds_u32;
__device__ __forceinline__ lds_u32* as_lds(uint32_t* p) { return (lds_u32*)p; }

// Per-lane match-group table (see m3_rules.hpp, match_scan): the first CAP
// groups in LDS, entry (g, h|v, word i) of lane l at tab[((g*2 + hv)*W + i)*LANES + l]
// (consecutive lanes hit consecutive dwords: conflict-free). A board that
// forms more groups in one scan (~1e-3 of steps at CAP 4) takes a record from
// a small global spill pool for groups CAP..MAXG-1; only a full pool (never in
// practice) sends the step to the exact recompute pass.
// LDS-only table (stateless kernels: a board with more groups is recomputed by k_apply_fix)
template <class CF, int CAP_, int LANES>
struct LdsTable {
    static constexpr int CAP = CAP_;
    static constexpr int W = CF::W;
    static constexpr int BLOCK = LANES;
    static constexpr int WORDS = CAP * 2 * W * BLOCK;
    lds_u32* tab;  // already offset by threadIdx.x
    __device__ __forceinline__ typename CF::Bd get_h(int g) const {
        typename CF::Bd r;
#pragma unroll
        for (int i = 0; i < W; ++i) r.w[i] = tab[((g * 2) * W + i) * BLOCK];
        return r;
    }
    __device__ __forceinline__ typename CF::Bd get_v(int g) const {
        typename CF::Bd r;
#pragma unroll
        for (int i = 0; i < W; ++i) r.w[i] = tab[((g * 2 + 1) * W + i) * BLOCK];
        return r;
    }
    __device__ __forceinline__ bool put(int g, const typename CF::Bd& h, const typename CF::Bd& v) {
#pragma unroll
        for (int i = 0; i < W; ++i) {
            tab[((g * 2) * W + i) * BLOCK] = h.w[i];
            tab[((g * 2 + 1) * W + i) * BLOCK] = v.w[i];
        }
        return true;
    }
};

template <class CF, int CAP_, int LANES>
struct LdsStore {
    static constexpr int CAP = CF::MAXG;     // logical capacity (spill included)
    static constexpr int LCAP = CAP_;        // groups held in LDS
    static constexpr int W = CF::W;
    static constexpr int BLOCK = LANES;
    static constexpr int WORDS = LCAP * 2 * W * BLOCK;
    static constexpr int SPILL_WORDS = (CF::MAXG - LCAP) * 2 * W;  // per pool record
    lds_u32* tab;         // already offset by threadIdx.x
    uint32_t* spill;      // nullable: pool of records
    uint32_t* pool_next;  // pool allocation counter
    uint32_t pool_cap;
    uint32_t rec = ~0u;   // this lane's record
    __device__ __forceinline__ typename CF::Bd get(int g, int hv) const {
        typename CF::Bd r;
        if (g < LCAP) {
#pragma unroll
            for (int i = 0; i < W; ++i) r.w[i] = tab[((g * 2 + hv) * W + i) * BLOCK];
        } else {
            const uint32_t* p = spill + (size_t)rec * SPILL_WORDS + ((g - LCAP) * 2 + hv) * W;
#pragma unroll
            for (int i = 0; i < W; ++i) r.w[i] = p[i];
        }
        return r;
    }
    __device__ __forceinline__ typename CF::Bd get_h(int g) const { return get(g, 0); }
    __device__ __forceinline__ typename CF::Bd get_v(int g) const { return get(g, 1); }
    __device__ __forceinline__ bool put(int g, const typename CF::Bd& h, const typename CF::Bd& v) {
        if (g < LCAP) {
#pragma unroll
            for (int i = 0; i < W; ++i) {
                tab[((g * 2) * W + i) * BLOCK] = h.w[i];
                tab[((g * 2 + 1) * W + i) * BLOCK] = v.w[i];
            }
            return true;
        }
        if (rec == ~0u) rec = atomicAdd(pool_next, 1u);
        const bool ok = rec < pool_cap;
        if (ok) {
            uint32_t* p = spill + (size_t)rec * SPILL_WORDS + (g - LCAP) * 2 * W;
#pragma unroll
            for (int i = 0; i < W; ++i) {
                p[i] = h.w[i];
                p[W + i] = v.w[i];
            }
        }
        return ok;
    }
};

// Phase profiling (profiling build only, -DM3_PHASE_PROF; tools/phase_prof.py).
// mark<K>() charges the wave's cycles since the previous mark to phase K; the
// first active lane keeps the per-wave accumulators in LDS, so the split is
// exact wave time even inside divergent loops.
#ifdef M3_PHASE_PROF
constexpr int PROF_SLOTS = PH_N + 2;  // phases, total cycles, waves
__device__ unsigned long long g_prof[2][PROF_SLOTS];  // [0] k_env_step, [1] k_init
template <class Base>
struct Prof : Base {
    static constexpr bool PROF = true;
    unsigned long long* w;  // this wave's LDS slot: PH_N accumulators, last, start
    template <int K>
    __device__ __forceinline__ void mark() {
        const unsigned long long now = clock64();
        if (__lane_id() == __builtin_amdgcn_readfirstlane(__lane_id())) {
            w[K] += now - w[PH_N];
            w[PH_N] = now;
        }
    }
    __device__ __forceinline__ void begin() {
        if (__lane_id() == 0) {
            for (int k = 0; k < PH_N; ++k) w[k] = 0;
            w[PH_N] = w[PH_N + 1] = clock64();
        }
        __builtin_amdgcn_wave_barrier();
    }
    __device__ __forceinline__ void end(int which) {
        mark<PH_STORE>();
        __builtin_amdgcn_wave_barrier();
        if (__lane_id() == 0) {
            for (int k = 0; k < PH_N; ++k) atomicAdd(&g_prof[which][k], w[k]);
            atomicAdd(&g_prof[which][PH_N], w[PH_N] - w[PH_N + 1]);
            atomicAdd(&g_prof[which][PH_N + 1], 1ull);
        }
    }
};
#define M3_PROF_LDS(LANES) __shared__ unsigned long long prof_s[(LANES) / 64][PH_N + 2];
// this translation unit's counters (read and optionally cleared)
inline int m3_prof_read_tu(uint64_t* out, int reset) {
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), sizeof(g_prof)));
    if (reset) {
        static const unsigned long long zero[2][PROF_SLOTS] = {};
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_prof), zero, sizeof(zero)));
    }
    return PH_N;
}
#endif

// profiling build: wait for the wave's outstanding memory operations, so the next mark charges their
// latency to the phase that issued them (no-op for every other Store)
template <class S>
__device__ __forceinline__ void prof_drain(S&) {
    if constexpr (HasProf<S>::value) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

// Staging barrier of the one-wave (64-lane) workgroups: it only has to order
// this wave's own LDS accesses (a wave's DS instructions execute in issue
// order), so a wavefront-scope fence suffices. __syncthreads() would also make
// the wave wait for every global store it has in flight (vmcnt(0) of the
// workgroup-scope release), i.e. a full memory round trip per kernel tail.
#ifndef M3_WAVE_SYNC
#define M3_WAVE_SYNC 0
#endif
__device__ __forceinline__ void lds_sync() {
#if M3_WAVE_SYNC
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
#else
    __syncthreads();
#endif
}

// ---------------------------------------------------------------------------
// LDS staging
// ---------------------------------------------------------------------------
// bytes = boards x cells (cells: the board's R*C, a compile-time constant
// except for frame shapes)
template <int BLOCK>
__device__ __forceinline__ void block_copy_in(const int8_t* __restrict__ g, uint8_t* lds, int bytes) {
    const int n16 = bytes >> 4;
    const uint4* s4 = reinterpret_cast<const uint4*>(g);
    uint4* d4 = reinterpret_cast<uint4*>(lds);
    for (int i = threadIdx.x; i < n16; i += BLOCK) d4[i] = s4[i];
    for (int i = (n16 << 4) + threadIdx.x; i < bytes; i += BLOCK) lds[i] = (uint8_t)g[i];
}

// the same copy for host-supplied boards: also reports whether any byte of the
// thread's share has bit 7 set (a cell value outside [0, 127], include/m3.h)
template <int BLOCK>
__device__ __forceinline__ bool block_copy_in_checked(const int8_t* __restrict__ g, uint8_t* lds, int bytes) {
    const int n16 = bytes >> 4;
    const uint4* s4 = reinterpret_cast<const uint4*>(g);
    uint4* d4 = reinterpret_cast<uint4*>(lds);
    uint32_t hi = 0u;
    for (int i = threadIdx.x; i < n16; i += BLOCK) {
        const uint4 v = s4[i];
        hi |= v.x | v.y | v.z | v.w;
        d4[i] = v;
    }
    for (int i = (n16 << 4) + threadIdx.x; i < bytes; i += BLOCK) {
        const uint8_t v = (uint8_t)g[i];
        hi |= v;
        lds[i] = v;
    }
    return (hi & 0x80808080u) != 0u;
}

// mark that some wave saw a bad cell: a plain store of 1 (the flag may live in host memory on the
// zero-copy path of small host-buffer calls, where device atomics are not an option)
__device__ __forceinline__ void flag_bad_cells(bool bad, uint32_t* flag) {
    if (flag && __any((int)bad) && __lane_id() == 0) *(volatile uint32_t*)flag = 1u;
}

template <int BLOCK>
__device__ __forceinline__ void block_copy_out(int8_t* __restrict__ g, const uint8_t* lds, int bytes) {
    const int n16 = bytes >> 4;
    const uint4* s4 = reinterpret_cast<const uint4*>(lds);
    uint4* d4 = reinterpret_cast<uint4*>(g);
    for (int i = threadIdx.x; i < n16; i += BLOCK) d4[i] = s4[i];
    for (int i = (n16 << 4) + threadIdx.x; i < bytes; i += BLOCK) g[i] = (int8_t)lds[i];
}

// The staging copies with PAD bytes after every ROW-byte board in LDS (ROW % 16 == 0): 16-byte
// chunks, each inside one row. A lane that reads or writes its own row then meets the other lanes
// 4-way on a bank instead of 64-way (ROW = 256: every row would start on bank 0).
template <int BLOCK, int ROW, int PAD>
__device__ __forceinline__ void block_copy_in_rows(const int8_t* __restrict__ g, uint8_t* lds, int bytes) {
    static_assert(ROW % 16 == 0 && PAD % 16 == 0, "whole 16-byte chunks");
    const int n16 = bytes >> 4;
    const uint4* s4 = reinterpret_cast<const uint4*>(g);
    for (int i = threadIdx.x; i < n16; i += BLOCK)
        *reinterpret_cast<uint4*>(lds + i * 16 + (i / (ROW / 16)) * PAD) = s4[i];
}
template <int BLOCK, int ROW, int PAD>
__device__ __forceinline__ void block_copy_out_rows(int8_t* __restrict__ g, const uint8_t* lds, int bytes) {
    static_assert(ROW % 16 == 0 && PAD % 16 == 0, "whole 16-byte chunks");
    const int n16 = bytes >> 4;
    uint4* d4 = reinterpret_cast<uint4*>(g);
    for (int i = threadIdx.x; i < n16; i += BLOCK)
        d4[i] = *reinterpret_cast<const uint4*>(lds + i * 16 + (i / (ROW / 16)) * PAD);
}

// N cell bytes (little-endian in cw[ceil(N/4)]) to dst of any alignment:
// up to 3 head bytes, aligned dwords (one funnel shift each), up to 3 tail
// bytes -- instead of N byte stores.
template <int N>
__device__ __forceinline__ void store_cells(uint8_t* dst, const uint32_t* cw) {
    constexpr int NW = (N + 3) / 4;
    const uint32_t head = (4u - ((uint32_t)(uintptr_t)dst & 3u)) & 3u;
    const uint32_t nd = ((uint32_t)N - head) >> 2;
    const uint32_t t0 = head + 4u * nd;
    const uint32_t s = 8u * head;
#pragma unroll
    for (int y = 0; y < 3; ++y)
        if ((uint32_t)y < head) dst[y] = (uint8_t)(cw[y >> 2] >> (8 * (y & 3)));
    uint32_t* d32 = reinterpret_cast<uint32_t*>(dst + head);
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        if ((uint32_t)i < nd) {
            const uint32_t lo = cw[i], hi = (i + 1 < NW) ? cw[i + 1] : 0u;
            d32[i] = s ? ((lo >> s) | (hi << (32u - s))) : lo;
        }
    }
#pragma unroll
    for (int y = N - 3; y < N; ++y)
        if ((uint32_t)y >= t0) dst[y] = (uint8_t)(cw[y >> 2] >> (8 * (y & 3)));
}

// lane's board (N bytes at lds + slot*N, any alignment) -> bit-planes.
// The dword window may reach into the neighbour's bytes; planes_from_words
// masks every bit >= N.
template <class CF>
__device__ __forceinline__ void lds_to_planes(const uint8_t* lds, int slot, typename CF::Bd* P,
                                              const typename CF::Dim& dm = typename CF::Dim{}) {
    if constexpr (CF::DYN) {
        frame_from_bytes<CF>(lds + slot * dm.cells(), P, dm);
        return;
    }
    constexpr int NW = (CF::N + 3) / 4;
    const int off = slot * CF::N;
    const uint32_t* d = reinterpret_cast<const uint32_t*>(lds + (off & ~3));
    const uint32_t sh = (uint32_t)(off & 3) * 8u;
    uint32_t cw[NW];
    uint32_t prev = d[0];
#pragma unroll
    for (int q = 0; q < NW; ++q) {
        const uint32_t next = d[q + 1];
        cw[q] = __builtin_amdgcn_alignbit(next, prev, sh);
        prev = next;
    }
    planes_from_words<CF>(cw, P);
}

template <class CF>
__device__ __forceinline__ void planes_to_bytes(const typename CF::Bd* P, uint8_t* dst,
                                                const typename CF::Dim& dm = typename CF::Dim{}) {
    if constexpr (CF::DYN) {
        frame_to_bytes<CF>(P, dst, dm);
        return;
    }
    constexpr int NW = (CF::N + 3) / 4;
    uint32_t cw[NW];
    words_from_planes<CF>(P, cw);
    store_cells<CF::N>(dst, cw);
}

template <class CF>
__device__ __forceinline__ void bytes_to_planes(const int8_t* src, typename CF::Bd* P,
                                                const typename CF::Dim& dm = typename CF::Dim{}) {
    if constexpr (CF::DYN) {
        frame_from_bytes<CF>(reinterpret_cast<const uint8_t*>(src), P, dm);
        return;
    }
    constexpr int NW = (CF::N + 3) / 4;
    uint32_t cw[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) {
        uint32_t v = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int x = 4 * q + k;
            if (x < CF::N) v |= (uint32_t)(uint8_t)src[x] << (8 * k);
        }
        cw[q] = v;
    }
    planes_from_words<CF>(cw, P);
}

template <class CF>
__device__ __forceinline__ void store_legal(uint32_t* out, const uint32_t* act,
                                            const typename CF::Dim& dm = typename CF::Dim{}) {
#pragma unroll
    for (int i = 0; i < CF::AW; ++i)
        if (i < dm.aw()) out[i] = act[i];
}

// words of one board's cells as packed little-endian words (env episode slots)
template <class CF>
__device__ __forceinline__ int cell_words(const typename CF::Dim& dm) {
    return (dm.cells() + 3) / 4;
}

// ---------------------------------------------------------------------------
// stateless kernels (BoardV2 facade): m3_apply_actions / m3_init_boards /
// m3_legal_actions
// ---------------------------------------------------------------------------
}  // namespace
// launcher signatures name this struct: it needs linkage (m3_inst.hip instantiates them)
namespace m3k {
struct ApplyArgs {
    Shape shape;  // the board (frame kernels; the specialised ones ignore it)
    int64_t n;
    const int8_t* boards;
    const uint32_t* seeds;
    const int32_t* n_actions;
    const int32_t* actions;
    int8_t* out_boards;
    int32_t* reward;
    uint32_t* draws;
    uint32_t* flags;
    uint32_t* legal;       // nullable
    int32_t* next_action;  // nullable
    uint32_t* ovf_count;
    uint32_t* ovf_list;
    uint32_t* bad_cells;   // nullable: set to 1 if a cell value lies outside [0, 127]
    int clear_ovf;         // k_apply_fix (one block) zeroes *ovf_count when done (zero-copy calls)
};
}  // namespace m3k
using m3k::ApplyArgs;
namespace {

// one full apply_action + outputs for board b; returns false on RNG overflow
template <class CF, class RNG, class Store>
__device__ __forceinline__ bool apply_and_emit(typename CF::Bd* P, const ApplyArgs& a, int64_t b, RNG& rng,
                                               Store& st, const typename CF::Dim& dm) {
    typename CF::Bd HL, VL;
    uint32_t f;
    const int r = apply_action<CF>(P, a.n_actions[b], a.actions[b], rng, f, HL, VL, st, dm);
    if (f & FLAG_RECOMPUTE) return false;
    const bool stepped = !(f & (FLAG_TERMINAL | FLAG_BAD_ACTION));
    a.reward[b] = r;
    a.draws[b] = stepped ? rng.draws() : 0u;
    uint32_t act[CF::AW];
    action_bits<CF>(HL, VL, act, dm);
    int na = -1;
    if (stepped) {
        na = random_action<CF>(act, rng);
        if (rng.overflow) return false;
        if (na < 0) f |= FLAG_NO_LEGAL;
    }
    mark<PH_NEXT>(st);
    a.flags[b] = f;
    if (a.next_action) a.next_action[b] = na;
    if (a.legal) store_legal<CF>(a.legal + b * dm.aw(), act, dm);
    return true;
}

template <class CF>
__global__ void __launch_bounds__(KS<CF>::B) k_apply(ApplyArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[KS<CF>::B * CF::N + 16];
    __shared__ uint32_t gtab[LdsStore<CF, KS<CF>::GCAP, KS<CF>::B>::WORDS];
    const typename CF::Dim dm(a.shape);
    const int NC = dm.cells();
    const int64_t b0 = (int64_t)blockIdx.x * KS<CF>::BPW;
    const int nb = (int)((a.n - b0) < KS<CF>::BPW ? (a.n - b0) : KS<CF>::BPW);
    flag_bad_cells(block_copy_in_checked<KS<CF>::B>(a.boards + b0 * NC, lds, nb * NC), a.bad_cells);
    lds_sync();
    const int t = threadIdx.x;
    if (t < nb) {
        const int64_t b = b0 + t;
        typename CF::Bd P[CF::NP];
        lds_to_planes<CF>(lds, t, P, dm);
        const uint32_t s = a.seeds[b];
        ChainMT rng;
        rng.init(s, mt_state397(s));
        LdsTable<CF, KS<CF>::GCAP, KS<CF>::B> st{as_lds(gtab + t)};  // overflow -> k_apply_fix
        if (!apply_and_emit<CF>(P, a, b, rng, st, dm)) {
            const uint32_t slot = atomicAdd(a.ovf_count, 1u);
            a.ovf_list[slot] = (uint32_t)b;
        }
        planes_to_bytes<CF>(P, lds + t * NC, dm);
    }
    lds_sync();
    block_copy_out<KS<CF>::B>(a.out_boards + b0 * NC, lds, nb * NC);
}

// redo overflowed boards with the full 624-word state (lane-private scratch)
template <class CF>
__global__ void __launch_bounds__(FIX_BLOCK) k_apply_fix(ApplyArgs a) {
    const uint32_t cnt = *a.ovf_count;
    const typename CF::Dim dm(a.shape);
    for (uint32_t i = blockIdx.x * lanes_for<CF>() + threadIdx.x; threadIdx.x < lanes_for<CF>() && i < cnt;
         i += gridDim.x * lanes_for<CF>()) {
        const int64_t b = a.ovf_list[i];
        typename CF::Bd P[CF::NP];
        bytes_to_planes<CF>(a.boards + b * dm.cells(), P, dm);
        FullMT mt;  // scratch: this pass almost never has work, and an LDS state would
                    // make even an empty launch wait for a whole free CU
        mt.init(a.seeds[b], 0u);
        ArrayStore<CF> st;
        apply_and_emit<CF>(P, a, b, mt, st, dm);
        planes_to_bytes<CF>(P, reinterpret_cast<uint8_t*>(a.out_boards + b * dm.cells()), dm);
    }
    if (a.clear_ovf) {  // a one-block launch: every thread has read the count
        __syncthreads();
        if (threadIdx.x == 0) *a.ovf_count = 0u;
    }
}

// M3_NSLOT: episode slots per board (A/B knob; at most 5: the counter blocks below). Round 6 A/B
// of 5 slots -- one more step of slack for the synchronised end-of-episode reset bursts: equal speed.
#ifndef M3_NSLOT
#define M3_NSLOT 4
#endif
constexpr int NSLOT = M3_NSLOT;     // episode slots per board (see EnvArgs)
static_assert(NSLOT >= 2 && NSLOT <= 255, "slot index is a byte");
constexpr int PF_LAG = NSLOT - 1;   // steps between a prefetch and its first use
// Per-shard counter blocks (8 words each), by step % CBLOCKS. Step t's block is read last by its
// prefetch chain, which step t + PF_LAG waits for; so when step t + PF_LAG's k_env_fix runs, the
// block of step t + PF_LAG + 1 (= step t's) is free and that kernel zeroes it -- no fill dispatch
// per shard-step and no cross-block ticket.
constexpr int CBLOCKS = PF_LAG + 1;
static_assert(8 * CBLOCKS <= 40, "the counter blocks end where a shard's stats begin (m3_env::counters, word 40)");
#ifndef M3_STAGE_PAD  // k_env_step's 16x16 staging rows 16 B apart (bank conflicts, see block_copy_in_rows)
#define M3_STAGE_PAD 1
#endif

// A reset launch processes "items". Item i is (board b, seed, slot): with a
// list (env prefetch) b = list[i], seed = list_seed[i], slot = list_slot[i];
// without, b = i, seed = seeds[i] + seed_add, slot = slot_of ? (slot_of[b] +
// slot0) % NSLOT : slot0. Per-board outputs go to index ob = slot * sstride + b
// (sstride 0 = the env's current state, n = one of the episode slots).
}  // namespace
// launcher signatures name this struct: it needs linkage (m3_inst.hip instantiates them)
namespace m3k {
struct InitArgs {
    Shape shape;
    int64_t n;
    const uint32_t* list;        // nullable
    const uint32_t* list_seed;
    const uint32_t* list_slot;
    const uint32_t* list_count;  // device count for list
    const uint32_t* seeds;       // implicit items
    uint32_t seed_add;
    uint32_t slot0;
    const uint8_t* slot_of;      // nullable
    int64_t sstride;
    int8_t* boards;              // cells as bytes at ob * N            (one of boards /
    uint32_t* board_words;       // cells as LE words at ob * NW         board_words)
    uint32_t* draws;             // nullable
    int32_t* first_action;       // nullable
    uint32_t* legal;             // nullable
    int32_t* score;              // nullable: zeroed episode state (explicit env reset)
    int32_t* moves;
    int32_t* reward;
    uint8_t* done;
    uint8_t* trunc;
    uint32_t* flags;
    uint32_t* slot_flags;        // nullable: M3_FLAG_RESET_CAP of the reset at ob (env episode slots), else 0
    uint32_t* stats;             // nullable: [0] resets, [1] reset recomputes (>= 624 draws)
    uint32_t* m397;              // nullable: mt[397] of the seed's init_genrand state at (slot, b)
    int64_t cstride;
    uint32_t* defer;             // nullable: items k_init leaves to k_init_coop (reset needs >= RESET_KCAP draws)
    uint32_t* defer_count;       // device count for defer (zeroed before k_init)
    uint32_t* tab;               // nullable: two-stage reset table rows [n][TwoStage::TW] (16x16x8 prefetch)
};
}  // namespace m3k
using m3k::InitArgs;
namespace {

__device__ __forceinline__ void init_item(const InitArgs& a, int64_t i, int64_t& b, uint32_t& seed, uint32_t& slot) {
    if (a.list) {
        b = (int64_t)a.list[i];
        seed = a.list_seed[i];
        slot = a.list_slot[i];
    } else {
        b = i;
        seed = a.seeds[b] + a.seed_add;
        slot = a.slot_of ? ((uint32_t)a.slot_of[b] + a.slot0) % (uint32_t)NSLOT : a.slot0;
    }
}

template <class CF>
__device__ __forceinline__ void init_store_board(const InitArgs& a, int64_t ob, const typename CF::Bd* P,
                                                 const typename CF::Dim& dm) {
    if constexpr (CF::DYN) {
        uint8_t* dst = a.board_words ? reinterpret_cast<uint8_t*>(a.board_words + ob * cell_words<CF>(dm))
                                     : reinterpret_cast<uint8_t*>(a.boards + ob * dm.cells());
        frame_to_bytes<CF>(P, dst, dm);
        return;
    }
    constexpr int NW = (CF::N + 3) / 4;
    uint32_t cw[NW];
    words_from_planes<CF>(P, cw);
    if (a.board_words) {
#pragma unroll
        for (int q = 0; q < NW; ++q) a.board_words[ob * NW + q] = cw[q];
    } else {
        store_cells<CF::N>(reinterpret_cast<uint8_t*>(a.boards + ob * CF::N), cw);
    }
}

// BoardV2.__init__ (boardv2.py:17-27) + first seeded random action
// (samplerTasks.py:11-13) for board b. Returns false if the stream overflowed.
// Everything a reset writes besides the cells: legal set, the first seeded
// random action (np.random.seed(cfg.seed) then choice(legal), samplerTasks.py:11-13),
// the cached mt[397] and the zeroed episode state.
template <class CF>
__device__ __forceinline__ void init_outputs(const InitArgs& a, int64_t b, int64_t ob, uint32_t seed, uint32_t m397,
                                             uint32_t draws, const typename CF::Bd* P,
                                             const typename CF::Dim& dm = typename CF::Dim{}) {
    typename CF::Bd HL, VL;
    legal_masks<CF>(P, special_mask<CF, CF::NP>(P), HL, VL, dm);
    uint32_t act[CF::AW];
    action_bits<CF>(HL, VL, act, dm);
    ChainMT rng;
    rng.init(seed, m397);
    const int fa = random_action<CF>(act, rng);
    if (a.draws) a.draws[ob] = draws;
    if (a.first_action) a.first_action[ob] = fa;
    if (a.legal) store_legal<CF>(a.legal + ob * dm.aw(), act, dm);
    if (a.score) a.score[b] = 0;
    if (a.moves) a.moves[b] = 0;
    if (a.reward) a.reward[b] = 0;
    if (a.done) a.done[b] = 0;
    if (a.trunc) a.trunc[b] = 0;
    if (a.flags) a.flags[b] = fa < 0 ? FLAG_NO_LEGAL : 0u;
    if (a.slot_flags) a.slot_flags[ob] = 0u;  // (k_init_fix_lane raises FLAG_RESET_CAP after this)
}

// Reset of board b on a tile stream generated in LDS (init_board_tiles).
// Returns false if the reset needs >= kcap draws (wave_reset redoes it).
template <class CF, class S = NoStore>
__device__ __forceinline__ bool init_emit(const InitArgs& a, int64_t b, uint32_t seed, uint32_t slot, uint32_t m397,
                                          uint32_t* tm, uint32_t* pos, S* ps = nullptr, uint32_t kcap = 624u) {
    typename CF::Bd P[CF::NP];
    ChainMT g;
    g.init(seed, m397);
    if (a.m397) a.m397[(int64_t)slot * a.cstride + b] = m397;
    uint32_t draws = 0;
    const bool ok = init_board_tiles<CF>(
        P, g, tm, pos, INIT_BLOCK, draws, 0u, [](uint32_t, uint32_t) {}, [](uint32_t, uint32_t) {}, ps, kcap);
    if (!ok) return false;
    const int64_t ob = (int64_t)slot * a.sstride + b;
    init_outputs<CF>(a, b, ob, seed, m397, draws, P);
    init_store_board<CF>(a, ob, P, typename CF::Dim{});
    return true;
}

// ---- wave-cooperative reset for boards whose reset needs >= 624 draws ----
// One board per wave. The 624-word MT19937 state sits in LDS; the twist runs
// on all 64 lanes (three dependency phases), and randint(1, T+1) over the
// board is a parallel filter: 64 raw outputs per trip, ballot of the accepted
// ones, prefix popcount for their cell. The bitboard logic (get_matches
// mask, legal, first action) runs redundantly on every lane, so control flow
// stays wave-uniform. Latency ~tens of us instead of ~1 ms for one lane
// walking the state.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ void wave_twist(uint32_t* key, int lane) {  // numpy mt19937_gen
    for (int base = 0; base < 227; base += 64) {  // mt'[i] = mt[i+397] ^ twist(mt[i], mt[i+1])
        const int i = base + lane;
        uint32_t a0 = 0, a1 = 0, x = 0;
        if (i < 227) { a0 = key[i]; a1 = key[i + 1]; x = key[i + 397]; }
        asm volatile("" ::: "memory");  // every lane's loads before any lane's store
        if (i < 227) key[i] = x ^ mt_twist(a0, a1);
        wave_sync();
    }
    for (int base = 227; base < 623; base += 64) {  // mt'[i] = mt'[i-227] ^ twist(mt[i], mt[i+1])
        const int i = base + lane;
        uint32_t a0 = 0, a1 = 0, x = 0;
        if (i < 623) { a0 = key[i]; a1 = key[i + 1]; x = key[i - 227]; }
        asm volatile("" ::: "memory");
        if (i < 623) key[i] = x ^ mt_twist(a0, a1);
        wave_sync();
    }
    if (lane == 0) key[623] = key[396] ^ mt_twist(key[623], key[0]);
    wave_sync();
}

__device__ __forceinline__ int select_bit64(uint64_t m, int k) {
    const uint32_t lo = (uint32_t)m;
    const int c = __builtin_popcount(lo);
    return k < c ? select_bit(lo, k) : 32 + select_bit((uint32_t)(m >> 32), k - c);
}

// RandomState.randint(1, T+1, (R, C)) into cells (only where `only` is set,
// if given); advances (pos, k) over the LDS state exactly as numpy would.
template <class CF>
__device__ __forceinline__ void wave_fill(uint32_t* key, uint8_t* cells, int lane, uint32_t& pos, uint32_t& k,
                                          const typename CF::Bd* only) {
    int filled = 0;
    while (filled < CF::N) {
        if constexpr (CF::TILE_RNG == 0u) {  // randint(1, 2): no draws consumed
            for (int c = lane; c < CF::N; c += 64)
                if (!only || only->test(c)) cells[c] = 1;
            break;
        }
        if (pos == 624u) {
            wave_twist(key, lane);
            pos = 0u;
        }
        const int take = (int)min(64u, 624u - pos);
        uint32_t v = 0;
        bool acc = false;
        if (lane < take) {
            v = mt_temper(key[pos + lane]) & CF::TILE_MASK;
            acc = v <= CF::TILE_RNG;
        }
        const uint64_t bal = __ballot(acc);
        const int rank = __builtin_popcountll(bal & ((1ull << lane) - 1ull));
        const int need = CF::N - filled, got = __builtin_popcountll(bal);
        if (acc && rank < need) {
            const int c = filled + rank;
            if (!only || only->test(c)) cells[c] = (uint8_t)(v + 1u);
        }
        const int used = got >= need ? select_bit64(bal, need - 1) + 1 : take;
        pos += (uint32_t)used;
        k += (uint32_t)used;
        filled += got >= need ? need : got;
    }
    wave_sync();
}

// init_genrand(seed) into key[0..623]. The recurrence is serial and the seed
// wave-uniform, so it runs on the scalar unit; v_writelane gathers 64
// consecutive values into one VGPR and a single LDS store writes them.
__device__ __forceinline__ void wave_init_key(uint32_t* key, uint32_t seed, int lane) {
    uint32_t x = __builtin_amdgcn_readfirstlane(seed);
    for (int blk = 0; blk < 9; ++blk) {  // 9 x 64 + 48 = 624
        uint32_t col = 0u;
#pragma unroll
        for (int j = 0; j < 64; ++j) {
            asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(col) : "s"(x), "n"(j));
            x = mt_init_next(x, (uint32_t)(blk * 64 + j) + 1u);
        }
        key[blk * 64 + lane] = col;
    }
    uint32_t col = 0u;
#pragma unroll
    for (int j = 0; j < 48; ++j) {
        asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(col) : "s"(x), "n"(j));
        x = mt_init_next(x, (uint32_t)(576 + j) + 1u);
    }
    if (lane < 48) key[576 + lane] = col;
}

// One reset (item of the launch) by the whole wave; key: 624 words of LDS,
// cells: N bytes of LDS. Returns the draws BoardV2.__init__ consumed.
template <class CF>
__device__ uint32_t wave_reset(const InitArgs& a, int64_t item, uint32_t* key, uint8_t* cells, int lane) {
    int64_t b;
    uint32_t seed, slot;
    init_item(a, item, b, seed, slot);
    wave_init_key(key, seed, lane);
    wave_sync();
    const uint32_t m397 = key[397];
    uint32_t pos = 624u, k = 0u;
    typename CF::Bd P[CF::NP], mask;
    const int64_t ob = (int64_t)slot * a.sstride + b;
    constexpr int NW = (CF::N + 3) / 4;
    wave_fill<CF>(key, cells, lane, pos, k, nullptr);               // boardv2.py:21
    planes_from_words<CF>(reinterpret_cast<const uint32_t*>(cells), P);
    while (get_match_mask<CF>(P, mask)) {                           // boardv2.py:23-27
        wave_fill<CF>(key, cells, lane, pos, k, &mask);
        planes_from_words<CF>(reinterpret_cast<const uint32_t*>(cells), P);
    }
    if (a.m397 && lane == 0) a.m397[(int64_t)slot * a.cstride + b] = m397;
    if (lane == 0) init_outputs<CF>(a, b, ob, seed, m397, k, P);
    if (a.board_words) {
        for (int q = lane; q < NW; q += 64)
            a.board_words[ob * NW + q] = reinterpret_cast<const uint32_t*>(cells)[q];
    } else {
        int8_t* dst = a.boards + ob * CF::N;
        for (int x = lane; x < CF::N; x += 64) dst[x] = (int8_t)cells[x];
    }
    wave_sync();
    return k;
}

// Reset on the register-only MT19937 chain; grid-strided over n (or *list_count).
// A reset that needs >= 624 draws (~0.7 % at 9x9x6) is redone by its own wave
// right away (wave_reset).
// REDO: the explicit-reset form, whose wave redoes its >= 624-draw resets itself (wave_reset, 2.5 KB
// of LDS for the MT state); the env prefetch (a.defer) defers them to k_init_coop instead and leaves
// that LDS out, so with the 10-word tile ring its wave takes ~10 KB -- what a CU full of k_env_step waves
// (16 x 9 KB) still has free.
template <class CF, bool REDO>
__global__ void __launch_bounds__(INIT_BLOCK) k_init(InitArgs a) {
    const int64_t cnt = a.list_count ? (int64_t)*a.list_count : a.n;
    if (a.stats && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&a.stats[0], (uint32_t)cnt);
    __shared__ uint32_t tm_s[CF::BITS * TileGen<CF>::TWMAX * INIT_BLOCK];
    __shared__ uint32_t pos_s[TileGen<CF>::MAXR * INIT_BLOCK];
    uint32_t* tm = tm_s + threadIdx.x;
    uint32_t* pos = pos_s + threadIdx.x;
#ifdef M3_PHASE_PROF
    M3_PROF_LDS(INIT_BLOCK)
    Prof<NoStore> ps;
    ps.w = prof_s[threadIdx.x >> 6];
    const bool live = (int64_t)blockIdx.x * INIT_BLOCK < cnt;
    if (live) ps.begin();
#else
    NoStore* const pp = nullptr;
#endif
    static_assert(INIT_INLINE_FIX<CF> && INIT_BLOCK == 64, "the in-wave redo is one wave's");
    __shared__ uint32_t key_s[REDO ? 624 : 1];
    __shared__ __attribute__((aligned(16))) uint8_t cell_s[REDO ? (CF::N + 3) / 4 * 4 + 16 : 16];
    for (int64_t base = (int64_t)blockIdx.x * INIT_BLOCK; base < cnt; base += (int64_t)gridDim.x * INIT_BLOCK) {
        const int64_t i = base + threadIdx.x;
        bool ok = true;
        if (i < cnt) {
            int64_t b;
            uint32_t seed, slot;
            init_item(a, i, b, seed, slot);
            const uint32_t m397 = mt_state397(seed);
            const uint32_t kcap = a.defer ? RESET_KCAP : 624u;
#ifdef M3_PHASE_PROF
            ok = init_emit<CF>(a, b, seed, slot, m397, tm, pos, &ps, kcap);
#else
            ok = init_emit<CF>(a, b, seed, slot, m397, tm, pos, pp, kcap);
#endif
        }
        uint64_t bad = __ballot(!ok);
        if (!REDO) {  // left to k_init_coop: one wave-aggregated append (a.defer is set)
            if (bad) {
                const int lane = (int)threadIdx.x;
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(a.defer_count, (uint32_t)__popcll(bad));
                base = __shfl(base, 0);
                if (!ok) a.defer[base + (uint32_t)__popcll(bad & ((1ull << lane) - 1ull))] = (uint32_t)i;
            }
            continue;
        }
        // this wave redoes its >= 624-draw resets at once
        if (bad && a.stats && threadIdx.x == 0) atomicAdd(&a.stats[1], (uint32_t)__builtin_popcountll(bad));
        if constexpr (REDO) {
            while (bad) {
                const int l = __builtin_ctzll(bad);
                bad &= bad - 1ull;
                wave_reset<CF>(a, __shfl(i, l), key_s, cell_s, (int)threadIdx.x);
            }
        }
    }
#ifdef M3_PHASE_PROF
    if (live) ps.end(1);
#endif
}

// The resets k_init deferred (>= RESET_KCAP draws), one wave per board
// (wave_reset), grid-strided over the device-side count.
template <class CF>
__global__ void __launch_bounds__(64) k_init_coop(InitArgs a) {
    __shared__ uint32_t key_s[624];
    __shared__ __attribute__((aligned(16))) uint8_t cell_s[(CF::N + 3) / 4 * 4 + 16];
    const uint32_t cnt = *a.defer_count;
    const int lane = (int)threadIdx.x;
    for (uint32_t q = blockIdx.x; q < cnt; q += gridDim.x) {
        wave_reset<CF>(a, a.defer[q], key_s, cell_s, lane);
        if (a.stats && lane == 0) atomicAdd(&a.stats[1], 1u);
    }
}

// ---- lane-per-board reset for boards that need >= 624 draws -------------
// One board per lane with the full 624-word MT19937 state in lane-private
// scratch (FullMT; scratch is swizzled per lane, so the state accesses of a
// wave are coalesced). At 9x9x6 ~0.7% of resets land here, at 16x16x8 ~60%
// (every round of randint(1, 9, (16, 16)) takes 256 draws), so this pass is
// throughput work: all 64 lanes of a wave run their own board.
//
// One round of BoardV2.__init__ (boardv2.py:21 / :25): randint(1, T+1, (R, C))
// draws a tile for EVERY cell in row-major order; cells outside `only` take
// their draw and drop it (array[mask] = new[mask]). A plane word collects 32
// tiles, then merges under the mask.
template <class R, class = void>
struct HasBulk : std::false_type {};
template <class R>
struct HasBulk<R, std::void_t<decltype(std::declval<R&>().bulk_ready(1u))>> : std::true_type {};

template <class CF, class RNG>
__device__ __forceinline__ void fill_round(typename CF::Bd* P, RNG& mt, const typename CF::Bd* only) {
#pragma unroll
    for (int w = 0; w < CF::W; ++w) {
        constexpr int BITS = CF::BITS;
        const int nbits = CF::N - 32 * w < 32 ? CF::N - 32 * w : 32;
        uint32_t t[BITS];
#pragma unroll
        for (int p = 0; p < BITS; ++p) t[p] = 0u;
        int bit = 0;
        if constexpr (CF::TILE_RNG != 0u && CF::TILE_RNG == CF::TILE_MASK && HasBulk<RNG>::value) {
            // T a power of two: every draw is a tile, so a word is nbits consecutive outputs
            if (mt.bulk_ready((uint32_t)nbits)) {
#pragma unroll
                for (int j = 0; j < nbits; ++j) {
                    const uint32_t v = (mt.bulk_out((uint32_t)j) & CF::TILE_MASK) + 1u;
#pragma unroll
                    for (int p = 0; p < BITS; ++p) t[p] |= ((v >> p) & 1u) << j;
                }
                mt.bulk_skip((uint32_t)nbits);
                bit = nbits;
            }
        }
        for (; bit < nbits; ++bit) {
            uint32_t v = 1u;
            if constexpr (CF::TILE_RNG != 0u) {
                do {
                    v = mt.next32() & CF::TILE_MASK;
                } while (v > CF::TILE_RNG);
                v += 1u;
            }
#pragma unroll
            for (int p = 0; p < BITS; ++p) t[p] |= ((v >> p) & 1u) << bit;
        }
        const uint32_t m = only ? only->w[w] : 0xFFFFFFFFu;
#pragma unroll
        for (int p = 0; p < BITS; ++p) P[p].w[w] = (P[p].w[w] & ~m) | (t[p] & m);
    }
}

// Every reset of the launch (k_init is skipped at 16x16x8: most resets
// overflow the chain anyway). stats[1] counts the resets that needed >= 624
// draws, as k_init's in-wave redo does at 9x9, so the counter means the same
// at both shapes.
template <class CF>
__global__ void __launch_bounds__(INIT_FIX_BLOCK) k_init_fix_lane(InitArgs a) {
    const typename CF::Dim dm(a.shape);
    const int64_t cnt = a.list_count ? (int64_t)*a.list_count : a.n;
    if (a.stats && blockIdx.x == 0 && threadIdx.x == 0 && cnt) atomicAdd(&a.stats[0], (uint32_t)cnt);
    constexpr int64_t L = lanes_for<CF>();
    for (int64_t base = (int64_t)blockIdx.x * L; base < cnt; base += (int64_t)gridDim.x * L) {
        const int64_t oi = base + threadIdx.x;
        bool long_reset = false;
        if (threadIdx.x < L && oi < cnt) {
            int64_t b;
            uint32_t seed, slot;
            init_item(a, oi, b, seed, slot);
            FullMT mt;
            mt.init(seed, 0u);
            const uint32_t m397 = mt.key[397];  // init_genrand state, before the first twist
            if (a.m397) a.m397[(int64_t)slot * a.cstride + b] = m397;
            typename CF::Bd P[CF::NP], mask;
#pragma unroll
            for (int p = 0; p < CF::NP; ++p) P[p] = CF::Bd::zero();
            uint32_t rounds = 0;
            if constexpr (CF::DYN) {
                fill_round_frame<CF>(P, mt, nullptr, dm);                              // boardv2.py:21
                while (get_match_mask<CF>(P, mask) && ++rounds < RESET_ROUND_CAP)    // :23-27
                    fill_round_frame<CF>(P, mt, &mask, dm);
            } else {
                fill_round<CF>(P, mt, nullptr);                              // boardv2.py:21
                while (get_match_mask<CF>(P, mask) && ++rounds < RESET_ROUND_CAP)  // boardv2.py:23-27
                    fill_round<CF>(P, mt, &mask);
            }
            const int64_t ob = (int64_t)slot * a.sstride + b;
            init_outputs<CF>(a, b, ob, seed, m397, mt.draws(), P, dm);
            if (rounds >= RESET_ROUND_CAP) {
                if (a.flags) a.flags[b] |= FLAG_RESET_CAP;
                if (a.slot_flags) a.slot_flags[ob] = FLAG_RESET_CAP;
            }
            init_store_board<CF>(a, ob, P, dm);
            long_reset = mt.draws() >= 624u;
        }
        const uint64_t m = __ballot(long_reset);
        if (m && a.stats && (threadIdx.x & 63) == 0) atomicAdd(&a.stats[1], (uint32_t)__popcll(m));
    }
}

// One round of randint(1, T+1, (R, C)) for a power-of-two T (every draw is a
// tile) as a rolled loop over the board's words: the RNG code appears once in
// the kernel instead of once per unrolled word (fill_round), which keeps a
// large generator such as ChainMT2 from multiplying the register peak.
template <class CF, class RNG>
__device__ __forceinline__ void fill_round_seq(typename CF::Bd* P, RNG& mt, const typename CF::Bd* only) {
    static_assert(CF::TILE_RNG != 0u && CF::TILE_RNG == CF::TILE_MASK && CF::N % 32 == 0, "N draws per round");
    constexpr int BITS = CF::BITS;
#pragma unroll 1
    for (int w = 0; w < CF::W; ++w) {
        uint32_t t[BITS];
#pragma unroll
        for (int p = 0; p < BITS; ++p) t[p] = 0u;
#pragma unroll 1
        for (int bit = 0; bit < 32; ++bit) {
            const uint32_t v = (mt.next32() & CF::TILE_MASK) + 1u;
#pragma unroll
            for (int p = 0; p < BITS; ++p) t[p] |= ((v >> p) & 1u) << bit;
        }
        const uint32_t m = only ? only->word_at(w) : 0xFFFFFFFFu;
#pragma unroll
        for (int p = 0; p < BITS; ++p) {
#pragma unroll
            for (int i = 0; i < CF::W; ++i)
                if (i == w) P[p].w[i] = (P[p].w[i] & ~m) | (t[p] & m);
        }
    }
}

// ---- lane-per-board reset on the two-block register chain (16x16x8) -------
// Every reset of the launch, one board per lane, on ChainMT2: the first 1248
// raw outputs of seed(s) from registers (m3_rng.hpp), so no reset walks a
// 2.5 KB lane-private state in scratch. With a power-of-two tile count every
// round of randint(1, T+1, (R, C)) takes exactly R*C draws (16x16x8: 256), so
// the lanes of a wave draw in lockstep and the chain's level changes are
// wave-uniform. A reset that would need a round past draw 1248 (16x16x8: a
// 5th round, ~2 % of resets) leaves the lane: appended to the defer list for
// k_init_coop (one wave per board; every launch of this kernel carries a defer
// list). stats[1] counts the resets the wave-cooperative pass finishes.
template <class CF>
__global__ void __launch_bounds__(INIT_BLOCK) k_init_chain2(InitArgs a) {
    static_assert(!CF::DYN && INIT_BLOCK == 64, "specialised shapes, one-wave blocks");
    constexpr bool LOCKSTEP = CF::TILE_RNG != 0u && CF::TILE_RNG == CF::TILE_MASK;  // N draws per round
    static_assert(LOCKSTEP, "power-of-two tile counts (16x16x8)");
    const int64_t cnt = a.list_count ? (int64_t)*a.list_count : a.n;
    if (a.stats && blockIdx.x == 0 && threadIdx.x == 0 && cnt) atomicAdd(&a.stats[0], (uint32_t)cnt);
    const typename CF::Dim dm{};
    for (int64_t base = (int64_t)blockIdx.x * INIT_BLOCK; base < cnt; base += (int64_t)gridDim.x * INIT_BLOCK) {
        const int64_t i = base + threadIdx.x;
        bool ok = true;
        if (i < cnt) {
            int64_t b;
            uint32_t seed, slot;
            init_item(a, i, b, seed, slot);
            const uint32_t m397 = mt_state397(seed);
            ChainMT2 mt;
            mt.init(seed, m397);
            typename CF::Bd P[CF::NP], mask;
#pragma unroll
            for (int p = 0; p < CF::NP; ++p) P[p] = CF::Bd::zero();
            fill_round_seq<CF>(P, mt, nullptr);                                 // boardv2.py:21
            for (;;) {                                                          // :23-27
                if (!get_match_mask<CF>(P, mask)) break;
                if (mt.k + (uint32_t)CF::N > ChainMT2::LIMIT) {  // the next round leaves the chain
                    ok = false;
                    break;
                }
                fill_round_seq<CF>(P, mt, &mask);
            }
            if (ok) {
                if (a.m397) a.m397[(int64_t)slot * a.cstride + b] = m397;
                const int64_t ob = (int64_t)slot * a.sstride + b;
                init_outputs<CF>(a, b, ob, seed, m397, mt.draws(), P, dm);
                init_store_board<CF>(a, ob, P, dm);
            }
        }
        const uint64_t bad = __ballot(!ok);
        if (bad) {  // left to k_init_coop (one wave per board): one wave-aggregated append
            const int lane = (int)threadIdx.x;
            uint32_t q = 0;
            if (lane == 0) q = atomicAdd(a.defer_count, (uint32_t)__popcll(bad));
            q = __shfl(q, 0);
            if (!ok) a.defer[q + (uint32_t)__popcll(bad & ((1ull << lane) - 1ull))] = (uint32_t)i;
        }
    }
}

// ---- two-stage reset (16x16x8 env prefetch) -----------------------------
// Each round of BoardV2.__init__'s redraw loop draws a whole (R, C) board
// (boardv2.py:21, :25), and with a power-of-two tile count every draw is a
// tile, so round k of a reset is raw outputs [k*N, (k+1)*N) of its seed's
// MT19937 stream, whatever the match masks turn out to be. The reset splits:
//   k_reset_stream: G resets per wave. Each lane runs init_genrand of one
//     board into LDS (VALU: the recurrence is serial per board), then the wave
//     twists each board's 624-word state and packs its first ROUNDS rounds of
//     tiles as raw-bit planes (one ballot per bit per 64 draws) into a table
//     row of TW words, written with one coalesced store;
//   k_reset_tiles: one board per lane, the match-mask loop of boardv2.py:23-27
//     over the table rounds (16-B loads), then the outputs of init_outputs.
// A reset that needs a round past ROUNDS (~2 %) goes to k_init_coop's defer
// list (one wave per board, from the seed). This replaces the lane-private
// 2.5 KB FullMT state that k_init_fix_lane walks in scratch.
#ifndef M3_RESET16_TWO_STAGE
#define M3_RESET16_TWO_STAGE 1
#endif
#ifndef M3_TS_BOARDS
#define M3_TS_BOARDS 4
#endif
#ifndef M3_TS_ROUNDS  // redraw rounds in the table (16x16x8: a fifth round for 1.7 % of resets, a sixth for 0.4 %)
#define M3_TS_ROUNDS 5
#endif
#ifndef M3_TS_INTERLEAVE
#define M3_TS_INTERLEAVE 4
#endif
template <class CF, bool DYN = CF::DYN>  // (frame configurations have no compile-time tile range)
struct TwoStageOk : std::false_type {};
template <class CF>
struct TwoStageOk<CF, false>
    : std::bool_constant<M3_RESET16_TWO_STAGE && (CF::N > 128) && CF::N % 64 == 0 && CF::TILE_RNG != 0u &&
                         CF::TILE_RNG == CF::TILE_MASK> {};
template <class CF>
constexpr bool RESET_TWO_STAGE = TwoStageOk<CF>::value;
template <class CF>
struct TwoStage {
    static constexpr int RB = __builtin_popcount(CF::TILE_MASK);  // raw bits per tile
    static constexpr int ROUNDS = M3_TS_ROUNDS;
    static constexpr int DRAWS = ROUNDS * CF::N;                  // 16x16x8: 1024
    static_assert(DRAWS > 624 && DRAWS - 1248 <= 227, "two blocks and at most a first-phase head of a third");
    static constexpr int GROUPS = DRAWS / 64;
    static constexpr int RW = CF::W * RB;                         // table words per round
    static constexpr int TW = (ROUNDS * RW + 1 + 3) / 4 * 4;      // + mt[397], rows 16-B aligned
    static_assert(ROUNDS * RW <= 128 && RW % 4 == 0, "row = two lane words; rounds on 16 B");
    static constexpr int G = M3_TS_BOARDS;                        // boards per wave
    static constexpr int U = M3_TS_INTERLEAVE;                    // boards twisted / packed together
    static_assert(G % U == 0, "whole interleave groups");
    static_assert(G >= 1 && G <= 64, "one lane per board in the init");
    static constexpr int KST = 625;  // LDS words per board: odd, so the init's lanes hit distinct banks
};

// The MT19937 twist of U boards' states at once (key + u * stride; the first nu
// are real), in place, so each trip's LDS latency is paid once for U boards.
// NW = 624: the whole block; NW < 624: only words [0, NW) of the next block
// (the draws past the table's last round are never made) -- words [NW, 624)
// keep the current block's values.
template <int U, int NW = 624>
__device__ __forceinline__ void wave_twist_u(uint32_t* key, int stride, int nu, int lane) {
    static_assert(NW == 624 || NW <= 576, "a whole block, or a head of the next");
    constexpr int E1 = NW < 227 ? NW : 227, E2 = NW == 624 ? 623 : (NW < 227 ? 227 : NW);
    for (int base = 0; base < E1; base += 64) {  // mt'[i] = mt[i+397] ^ twist(mt[i], mt[i+1])
        const int i = base + lane;
        uint32_t a0[U], a1[U], x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t* k = key + u * stride;
            a0[u] = a1[u] = x[u] = 0u;
            if (u < nu && i < E1) { a0[u] = k[i]; a1[u] = k[i + 1]; x[u] = k[i + 397]; }
        }
        asm volatile("" ::: "memory");  // every lane's loads before any lane's store
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (u < nu && i < E1) key[u * stride + i] = x[u] ^ mt_twist(a0[u], a1[u]);
        wave_sync();
    }
    for (int base = 227; base < E2; base += 64) {  // mt'[i] = mt'[i-227] ^ twist(mt[i], mt[i+1])
        const int i = base + lane;
        uint32_t a0[U], a1[U], x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t* k = key + u * stride;
            a0[u] = a1[u] = x[u] = 0u;
            if (u < nu && i < E2) { a0[u] = k[i]; a1[u] = k[i + 1]; x[u] = k[i - 227]; }
        }
        asm volatile("" ::: "memory");
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (u < nu && i < E2) key[u * stride + i] = x[u] ^ mt_twist(a0[u], a1[u]);
        wave_sync();
    }
    if constexpr (NW == 624) {
        if (lane < nu) {
            uint32_t* k = key + lane * stride;
            k[623] = k[396] ^ mt_twist(k[623], k[0]);
        }
        wave_sync();
    }
}

template <class CF>
__global__ void __launch_bounds__(64) k_reset_stream(InitArgs a) {
    using TS = TwoStage<CF>;
    constexpr int NX = TS::DRAWS <= 1248 ? TS::DRAWS - 624 : 624;  // words of the second block
    constexpr int G1 = 624 / 64;         // 64-draw groups wholly in the first block
    static_assert(TS::DRAWS > 1248 || NX <= G1 * 64, "the second twist must leave the straddling group's words");
    constexpr int U = TS::U;
    __shared__ uint32_t key_s[TS::G * TS::KST];
    const int lane = (int)threadIdx.x;
    const int64_t cnt = a.list_count ? (int64_t)*a.list_count : a.n;
    for (int64_t base = (int64_t)blockIdx.x * TS::G; base < cnt; base += (int64_t)gridDim.x * TS::G) {
        const int nb = (int)(cnt - base < TS::G ? cnt - base : TS::G);
        if (lane < nb) {  // init_genrand(seed), one board per lane
            int64_t b;
            uint32_t seed, slot;
            init_item(a, base + lane, b, seed, slot);
            uint32_t* k = key_s + lane * TS::KST;
            uint32_t x = seed;
            k[0] = x;
#pragma unroll 8
            for (uint32_t i = 1; i < 624u; ++i) {
                x = mt_init_next(x, i);
                k[i] = x;
            }
        }
        wave_sync();
#pragma unroll 1
        for (int j0 = 0; j0 < nb; j0 += U) {
            const int nu = nb - j0 < U ? nb - j0 : U;
            uint32_t* key = key_s + j0 * TS::KST;
            const uint32_t m397 = lane < nu ? key[lane * TS::KST + 397] : 0u;  // lane u: board j0 + u
            wave_sync();
            uint32_t o0[U], o1[U];  // row words lane and 64 + lane
#pragma unroll
            for (int u = 0; u < U; ++u) o0[u] = o1[u] = 0u;
            // draws 64g .. 64g + 63 into the row: one ballot per raw bit and board
            // (draw d sits at word d % 624 of the block last twisted, or of the one before it for the
            // straddling group's low lanes -- words the twist of a block head leaves alone; `prev`:
            // those words saved before a whole-block twist)
            auto pack = [&](int g, const uint32_t* prev) {
                const int d = g * 64 + lane;
                const bool low = prev && d % 624 >= 576;  // the previous block's words
                uint32_t y[U];
#pragma unroll
                for (int u = 0; u < U; ++u)  // randint - 1
                    y[u] = mt_temper(low ? prev[u] : key[u * TS::KST + d % 624]) & CF::TILE_MASK;
#pragma unroll
                for (int u = 0; u < U; ++u) {
#pragma unroll
                    for (int q = 0; q < TS::RB; ++q) {
                        const uint64_t bal = __ballot((y[u] >> q) & 1u);
                        const int idx = (g * TS::RB + q) * 2;  // words idx (draws 0-31) and idx + 1 (32-63)
                        const uint32_t val = (lane & 1) ? (uint32_t)(bal >> 32) : (uint32_t)bal;
                        if ((lane & ~1) == (idx & 63)) {
                            if (idx < 64) o0[u] = val;
                            else o1[u] = val;
                        }
                    }
                }
            };
            wave_twist_u<U>(key, TS::KST, nu, lane);  // draws 0 .. 623
#pragma unroll 1
            for (int g = 0; g < G1; ++g) pack(g, 0);
            wave_sync();
            if constexpr (TS::DRAWS <= 1248) {
                wave_twist_u<U, NX>(key, TS::KST, nu, lane);  // draws 624 .. DRAWS - 1, over words [0, NX)
#pragma unroll 1
                for (int g = G1; g < TS::GROUPS; ++g) pack(g, 0);
            } else {  // a whole second block and the head of a third
                constexpr int G2 = 1248 / 64;  // groups below the third block's first word
                uint32_t t9[U];                // the straddling group's first-block words (lanes < 48)
#pragma unroll
                for (int u = 0; u < U; ++u) t9[u] = key[u * TS::KST + (G1 * 64 + lane) % 624];
                wave_sync();
                wave_twist_u<U>(key, TS::KST, nu, lane);  // draws 624 .. 1247
                pack(G1, t9);
#pragma unroll 1
                for (int g = G1 + 1; g < G2; ++g) pack(g, 0);
                wave_sync();
                wave_twist_u<U, TS::DRAWS - 1248>(key, TS::KST, nu, lane);  // draws 1248 .. DRAWS - 1
#pragma unroll 1
                for (int g = G2; g < TS::GROUPS; ++g) pack(g, 0);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (u < nu) {
                    uint32_t* row = a.tab + (base + j0 + u) * TS::TW;
                    row[lane] = o0[u];
                    if (lane < TS::ROUNDS * TS::RW - 64) row[64 + lane] = o1[u];
                }
            }
            if (lane < nu) a.tab[(base + j0 + lane) * TS::TW + TS::ROUNDS * TS::RW] = m397;
            wave_sync();
        }
    }
}

// round k of the table row into the planes: value = raw + 1, under `only`
template <class CF>
__device__ __forceinline__ void tab_round(typename CF::Bd* P, const uint32_t* t, const typename CF::Bd* only) {
    using TS = TwoStage<CF>;
    uint32_t raw[TS::RW];
#pragma unroll
    for (int q = 0; q < TS::RW; q += 4) {
        const uint4 x = *reinterpret_cast<const uint4*>(t + q);
        raw[q] = x.x;
        raw[q + 1] = x.y;
        raw[q + 2] = x.z;
        raw[q + 3] = x.w;
    }
#pragma unroll
    for (int w = 0; w < CF::W; ++w) {
        uint32_t c = 0xFFFFFFFFu;  // + 1: a ripple carry over the bit planes
        const uint32_t m = only ? only->w[w] : 0xFFFFFFFFu;
#pragma unroll
        for (int p = 0; p < CF::BITS; ++p) {
            const uint32_t r = p < TS::RB ? raw[((w >> 1) * TS::RB + (p < TS::RB ? p : 0)) * 2 + (w & 1)] : 0u;
            const uint32_t vb = r ^ c;
            c &= r;
            P[p].w[w] = (P[p].w[w] & ~m) | (vb & m);
        }
    }
}

template <class CF>
__global__ void __launch_bounds__(64) k_reset_tiles(InitArgs a) {
    using TS = TwoStage<CF>;
    const typename CF::Dim dm{};
    const int64_t cnt = a.list_count ? (int64_t)*a.list_count : a.n;
    if (a.stats && blockIdx.x == 0 && threadIdx.x == 0 && cnt) atomicAdd(&a.stats[0], (uint32_t)cnt);
    for (int64_t base = (int64_t)blockIdx.x * 64; base < cnt; base += (int64_t)gridDim.x * 64) {
        const int64_t i = base + threadIdx.x;
        bool ok = true, long_reset = false;
        if (i < cnt) {
            int64_t b;
            uint32_t seed, slot;
            init_item(a, i, b, seed, slot);
            const uint32_t* t = a.tab + i * TS::TW;
            const uint32_t m397 = t[TS::ROUNDS * TS::RW];
            typename CF::Bd P[CF::NP], mask;
#pragma unroll
            for (int p = 0; p < CF::NP; ++p) P[p] = CF::Bd::zero();
            tab_round<CF>(P, t, nullptr);                                  // boardv2.py:21
            uint32_t rounds = 0;
            while (get_match_mask<CF>(P, mask)) {                          // :23-27
                if (++rounds >= (uint32_t)TS::ROUNDS) {
                    ok = false;
                    break;
                }
                tab_round<CF>(P, t + rounds * TS::RW, &mask);
            }
            if (ok) {
                if (a.m397) a.m397[(int64_t)slot * a.cstride + b] = m397;
                const int64_t ob = (int64_t)slot * a.sstride + b;
                const uint32_t draws = (rounds + 1u) * (uint32_t)CF::N;
                init_outputs<CF>(a, b, ob, seed, m397, draws, P, dm);
                init_store_board<CF>(a, ob, P, dm);
                long_reset = draws >= 624u;
            }
        }
        const uint64_t bad = __ballot(!ok);
        const int lane = (int)threadIdx.x;
        if (bad) {  // left to k_init_coop (one wave per board): one wave-aggregated append
            uint32_t q = 0;
            if (lane == 0) q = atomicAdd(a.defer_count, (uint32_t)__popcll(bad));
            q = __shfl(q, 0);
            if (!ok) a.defer[q + (uint32_t)__popcll(bad & ((1ull << lane) - 1ull))] = (uint32_t)i;
        }
        const uint64_t lm = __ballot(long_reset);
        if (lm && a.stats && lane == 0) atomicAdd(&a.stats[1], (uint32_t)__popcll(lm));
    }
}

#include "m3_reset9.hpp"

// mt[397] of init_genrand(seeds[b]): the chain word of each board's current
// episode (env resume, m3_env_set)
__global__ void __launch_bounds__(256) k_mt397(int64_t n, const uint32_t* seeds, uint32_t* out) {
    for (int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x; b < n; b += (int64_t)gridDim.x * 256)
        out[b] = mt_state397(seeds[b]);
}

template <class CF>
__global__ void __launch_bounds__(KS<CF>::B) k_legal(Shape shape, int64_t n, const int8_t* boards, uint32_t* legal) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[KS<CF>::B * CF::N + 16];
    const typename CF::Dim dm(shape);
    const int NC = dm.cells();
    const int64_t b0 = (int64_t)blockIdx.x * KS<CF>::BPW;
    const int nb = (int)((n - b0) < KS<CF>::BPW ? (n - b0) : KS<CF>::BPW);
    block_copy_in<KS<CF>::B>(boards + b0 * NC, lds, nb * NC);
    lds_sync();
    const int t = threadIdx.x;
    if (t < nb) {
        typename CF::Bd P[CF::NP], HL, VL;
        lds_to_planes<CF>(lds, t, P, dm);
        legal_masks<CF>(P, special_mask<CF, CF::NP>(P), HL, VL, dm);
        uint32_t act[CF::AW];
        action_bits<CF>(HL, VL, act, dm);
        store_legal<CF>(legal + (b0 + t) * dm.aw(), act, dm);
    }
}

// ---------------------------------------------------------------------------
// batched env (n x Match3Env, env.py:8-65)
// ---------------------------------------------------------------------------
// Autoreset keeps NSLOT episode slots per board: the current episode's stream
// cache is slot cur[b]; slots cur+1 .. cur+NSLOT-1 hold the next episodes
// (seed + k*stride) -- initial board, first action, legal set and stream
// cache -- computed ahead by the prefetch pass (k_init on its own stream). A
// finished board swaps in slot cur+1 inside the step and queues slot cur (now
// free) for the episode NSLOT-1 ahead; the prefetch of step t is only needed
// NSLOT-1 steps later, so resets never sit on the step's critical path.

}  // namespace
// launcher signatures name this struct: it needs linkage (m3_inst.hip instantiates them)
namespace m3k {
struct EnvArgs {
    Shape shape;
    int64_t n;
    int num_moves, goal;
    int autoreset;
    uint32_t stride;         // autoreset seed increment
    const int8_t* cur;
    int8_t* nxt;
    const int32_t* actions;  // nullable -> next_action
    uint32_t* seeds;
    int32_t* score;
    int32_t* moves;
    int32_t* next_action;
    int32_t* reward;
    uint8_t* done;
    uint8_t* trunc;
    uint32_t* flags;
    uint32_t* draws;
    uint32_t* legal;  // nullable
    int32_t* packed;  // nullable: reward<<2 | trunc<<1 | done for the RCCL gather
    uint32_t* counters;  // this step's block: [0] overflow count, [1] prefetch count, [2] prefetch overflow
                         // count, [3] spill records used, [4] continuation records
    uint32_t* spill;     // group-table spill pool of the shard
    uint32_t* stats;     // [0] step recomputes
    uint32_t* ovf_list;
    uint8_t* slot;       // current episode slot per board
    const uint32_t* ne_words;  // episode slots: initial cells (LE words) [3][n][NW]
    const int32_t* ne_first;   // [3][n] first seeded random action
    const uint32_t* ne_legal;  // [3][n][AW]
    const uint32_t* ne_flags;  // [NSLOT][n] FLAG_RESET_CAP of the slot's reset (0 otherwise)
    uint32_t* pf_list;   // prefetch queue of this step: board, seed, slot
    uint32_t* pf_seed;
    uint32_t* pf_slot;
    const uint32_t* m397;  // [NSLOT][cstride] mt[397] of each slot's seed
    int64_t cstride;
    uint32_t* cont;        // nullable: continuation records of paused steps (k_env_cont_grid), CONT_REC words each
    int64_t cont_stride;
    uint32_t* zero_next;   // the counter block of the next step, zeroed by k_env_fix (see CBLOCKS)
};
}  // namespace m3k
using m3k::EnvArgs;
namespace {

// Counter block words (8 per shard and step, see CBLOCKS): the continuation count and the
// prefetch queue length share one 64-bit word, so k_env_step's wave takes both of its slots with
// ONE atomic (low half: continuation records, high half: queue entries).
enum : int { CNT_OVF = 0, CNT_PF_DEFER = 2, CNT_SPILL = 3, CNT_CONT = 4, CNT_PF = 5 };

// Match3Env.step bookkeeping (env.py:48-56) after BoardV2.apply_action (r, f,
// HL/VL of the resulting board), and the same-step autoreset (the finished
// step's reward/done/flags stay visible, the observation and episode state
// become the next episode's). mv / sc0: the board's moves and score before the
// step. In three parts, so k_env_step can take the queue slots of its resets and
// the continuation records of its paused lanes with one atomic between the
// decisions and the stores:
//   env_fin_begin   the decisions (draw count, next seeded random action, done /
//                   truncated, autoreset) and every load the stores need (the next
//                   episode's slot -- first action, reset flags, legal set, cells);
//                   false if the next random action ran past the RNG (recompute;
//                   nothing has been stored then);
//   env_fin_store   the per-board stores and the reset swap;
//   env_fin_queue   the freed slot's entry in the prefetch queue (slot q).
// env_finish is the three in a row with its own queue atomic (k_env_cont_grid,
// k_env_fix).
//
// Memory order: every load and the atomic are issued BEFORE the first store. A
// wave's vector memory counter covers loads and stores, so a value returned behind
// stores is only usable once those stores are acknowledged too (round 5: one full
// memory round trip per load / store pair; round 6: the continuation atomic, issued
// after the step's stores, waited for all of them).
// row (nullable, k_env_step): the board's bytes go to this LDS staging row --
// the resulting board, or the next episode's cells on a reset -- and P is not
// needed afterwards. Without a row, P holds the board to write (the next
// episode's on a reset).
template <class CF>
struct EnvFin {
    static constexpr bool CELLS_IN_REGS = !CF::DYN;  // frame boards load their cells at the use
    static constexpr int NWS = (CF::N + 3) / 4;
    uint32_t ndraws, f, nflags, s_old, seed;
    int r, tr, dn, sc, mv1, na, first;
    bool reset;
    int64_t ob;
    uint32_t act[CF::AW];
    uint32_t lg[CF::AW];
    uint32_t cw[CELLS_IN_REGS ? NWS : 1];
};

template <class CF, class RNG, class Store>
__device__ __forceinline__ bool env_fin_begin(typename CF::Bd* P, const EnvArgs& a, int64_t b, RNG& rng, Store& st,
                                              int r, uint32_t f, const typename CF::Bd& HL, const typename CF::Bd& VL,
                                              int mv, int sc0, const typename CF::Dim& dm, uint8_t* row,
                                              EnvFin<CF>& e, const uint32_t* known_slot = nullptr,
                                              const uint32_t* known_seed = nullptr, bool cells = true) {
    const bool stepped = !(f & (FLAG_TERMINAL | FLAG_BAD_ACTION));
    e.r = r;
    e.sc = sc0 + r;
    e.mv1 = mv + 1;
    e.tr = e.sc >= a.goal;                          // env.py:53
    e.dn = e.tr || e.mv1 == a.num_moves;            // env.py:54
    e.ndraws = stepped ? rng.draws() : 0u;          // the step's own draws (before the next action's)
    action_bits<CF>(HL, VL, e.act, dm);
    e.na = -1;
    if (stepped) {
        e.na = random_action<CF>(e.act, rng);
        if (rng.overflow) return false;
        if (e.na < 0) f |= FLAG_NO_LEGAL;
    }
    e.f = f;
    mark<PH_NEXT>(st);
    e.reset = e.dn && a.autoreset;
    if (row) planes_to_bytes<CF>(P, row, dm);  // (LDS) P is dead from here on in k_env_step
    mark<PH_TBYTES>(st);
    // ---- loads: everything the stores need ----
    const int AW = dm.aw();
    e.s_old = 0u;
    e.seed = 0u;
    e.ob = 0;
    e.first = -1;
    e.nflags = 0u;  // the next episode's reset flags (FLAG_RESET_CAP)
    if (e.reset) {  // swap in the prefetched next episode (slot + 1)
        // (k_env_step passes the slot and seed it loaded before the cascade: no load, then a
        // dependent load of the slot's words, on the way to the stores)
        const uint32_t s_old = known_slot ? *known_slot : a.slot[b];
        e.seed = (known_seed ? *known_seed : a.seeds[b]) + a.stride;
        const uint32_t s_new = s_old + 1u == (uint32_t)NSLOT ? 0u : s_old + 1u;
        e.ob = (int64_t)s_new * a.cstride + b;  // slots are strided by the env's n
        e.first = a.ne_first[e.ob];
        e.nflags = a.ne_flags ? a.ne_flags[e.ob] : 0u;
        if (a.legal) {
#pragma unroll
            for (int i = 0; i < CF::AW; ++i) e.lg[i] = i < AW ? a.ne_legal[e.ob * AW + i] : 0u;
        }
        if constexpr (EnvFin<CF>::CELLS_IN_REGS) {
            if (cells) {
#pragma unroll
                for (int q = 0; q < EnvFin<CF>::NWS; ++q) e.cw[q] = a.ne_words[e.ob * EnvFin<CF>::NWS + q];
            }
        }
        e.s_old = s_new;  // (from here on: the new slot)
    }
    prof_drain(st);
    mark<PH_TLOAD>(st);
    return true;
}

template <class CF, class Store>
__device__ __forceinline__ void env_fin_store(typename CF::Bd* P, const EnvArgs& a, int64_t b, Store& st,
                                              const EnvFin<CF>& e, const typename CF::Dim& dm, uint8_t* row,
                                              bool cells = true) {
    const int AW = dm.aw();
    a.draws[b] = e.ndraws;
    a.reward[b] = e.r;
    a.trunc[b] = (uint8_t)e.tr;
    a.done[b] = (uint8_t)e.dn;
    a.flags[b] = e.f | e.nflags;  // (a reset that stopped at its round cap flags the step that swapped it in)
    if (a.packed) a.packed[b] = (e.r << 2) | (e.tr << 1) | e.dn;
    if (!e.reset) {
        a.score[b] = e.sc;
        a.moves[b] = e.mv1;
        a.next_action[b] = e.na;
        if (a.legal) store_legal<CF>(a.legal + b * AW, e.act, dm);
    } else {
        a.slot[b] = (uint8_t)e.s_old;
        a.seeds[b] = e.seed;
        a.score[b] = 0;
        a.moves[b] = 0;
        a.next_action[b] = e.first;
        if (a.legal) {
#pragma unroll
            for (int i = 0; i < CF::AW; ++i)
                if (i < AW) a.legal[b * AW + i] = e.lg[i];
        }
        if constexpr (EnvFin<CF>::CELLS_IN_REGS) {
            if (!cells) {
                // (k_env_step with M3_COOP_CELLS: the wave copies them, coop_reset_cells)
            } else if (row) {
                store_cells<CF::N>(row, e.cw);
            } else {
                planes_from_words<CF>(e.cw, P);
            }
        } else {
            const uint8_t* src = reinterpret_cast<const uint8_t*>(a.ne_words + e.ob * cell_words<CF>(dm));
            if (row) {
                for (int x = 0; x < dm.cells(); ++x) row[x] = src[x];
            } else {
                frame_from_bytes<CF>(src, P, dm);
            }
        }
    }
    mark<PH_RESET>(st);
}

// the freed slot (the one before the new current slot) takes the episode NSLOT - 1 ahead
__device__ __forceinline__ void env_fin_queue(const EnvArgs& a, int64_t b, uint32_t q, uint32_t seed, uint32_t s_new) {
    a.pf_list[q] = (uint32_t)b;
    a.pf_seed[q] = seed + (uint32_t)(NSLOT - 1) * a.stride;
    a.pf_slot[q] = s_new == 0u ? (uint32_t)(NSLOT - 1) : s_new - 1u;
}

// The next episode's cells of the wave's resetting lanes (mask m), copied into their LDS staging
// rows by the whole wave: NWS lanes per board, one dword each (64 / NWS boards per pass), instead of
// NWS words in every lane's registers across the atomic (M3_COOP_CELLS). ob: the lane's slot word
// offset (EnvFin::ob). Loads of every pass first, then the byte writes.
#ifndef M3_COOP_CELLS
#define M3_COOP_CELLS 1
#endif
template <class CF>
__device__ __forceinline__ void coop_reset_cells(const EnvArgs& a, uint64_t m, int64_t ob, uint8_t* lds, int row_stride) {
    constexpr int NWS = EnvFin<CF>::NWS;
    static_assert(NWS <= 64, "one word per lane per board");
    constexpr int PER = 64 / NWS;             // boards per pass (9x9: 3, 16x16: 1)
    constexpr int BATCH = PER >= 3 ? 1 : 4;   // passes whose loads go out together
    const int lane = (int)__lane_id(), j = lane / NWS, w = lane - j * NWS;
    while (m) {
        uint32_t v[BATCH];
        int src[BATCH];
#pragma unroll
        for (int u = 0; u < BATCH; ++u) {
            src[u] = -1;
#pragma unroll
            for (int k = 0; k < PER; ++k) {  // this lane's board of the pass: the j-th set lane of m
                const int l = m ? __ffsll((unsigned long long)m) - 1 : -1;
                if (k == j) src[u] = l;
                if (m) m &= m - 1ull;
            }
            const int64_t sob = __shfl(ob, src[u] < 0 ? 0 : src[u]);
            v[u] = (j < PER && src[u] >= 0) ? a.ne_words[sob * NWS + w] : 0u;
        }
#pragma unroll
        for (int u = 0; u < BATCH; ++u) {
            if (j < PER && src[u] >= 0) {
                uint8_t* dst = lds + src[u] * row_stride + 4 * w;
                if constexpr (CF::N % 4 == 0) {
                    *reinterpret_cast<uint32_t*>(dst) = v[u];  // (rows 16-B aligned: one dword)
                } else {
#pragma unroll
                    for (int y = 0; y < 4; ++y)
                        if (4 * w + y < CF::N) dst[y] = (uint8_t)(v[u] >> (8 * y));
                }
            }
        }
    }
}

// k_env_step's extras for the finish of a step: inputs it already holds, and the cooperative copy
// of the next episode's cells (the wave copies them after the step, coop_reset_cells)
struct FinOpts {
    const uint32_t* slot = nullptr;  // the board's current episode slot (else loaded again)
    const uint32_t* seed = nullptr;  // the board's seed (else loaded again)
    bool cells = true;               // false: leave the next episode's cells to coop_reset_cells
    bool* reset = nullptr;           // out: this lane swapped in its next episode
    int64_t* ob = nullptr;           // out: that episode's slot word offset
};

// rank of this lane among the set lanes of m
__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {
    return (uint32_t)__popcll(m & ((1ull << __lane_id()) - 1ull));
}

template <class CF, class RNG, class Store>
__device__ __forceinline__ bool env_finish(typename CF::Bd* P, const EnvArgs& a, int64_t b, RNG& rng, Store& st,
                                           int r, uint32_t f, const typename CF::Bd& HL, const typename CF::Bd& VL,
                                           int mv, int sc0, const typename CF::Dim& dm, uint8_t* row = nullptr,
                                           FinOpts o = FinOpts{}) {
    EnvFin<CF> e;
    if (!env_fin_begin<CF>(P, a, b, rng, st, r, f, HL, VL, mv, sc0, dm, row, e, o.slot, o.seed, o.cells)) return false;
    if (o.reset) *o.reset = e.reset;
    if (o.ob) *o.ob = e.ob;
    // the freed slot is queued for the episode after next: one atomic per wave, not per lane
    const uint64_t m = __ballot(e.reset);
    uint32_t qbase = 0u;
    int leader = 0;
    if (m) {
        leader = __ffsll((unsigned long long)m) - 1;
        if ((int)__lane_id() == leader) qbase = atomicAdd(&a.counters[CNT_PF], (uint32_t)__popcll(m));
    }
    prof_drain(st);
    mark<PH_TATOM>(st);
    env_fin_store<CF>(P, a, b, st, e, dm, row, o.cells);
    if (m) {
        qbase = __shfl(qbase, leader);
        if (e.reset) env_fin_queue(a, b, qbase + lane_rank(m), e.seed, e.s_old);
    }
    mark<PH_QUEUE>(st);
    return true;
}

enum : int { ENV_STEP_DONE = 0, ENV_STEP_RECOMPUTE = 1, ENV_STEP_PAUSED = 2 };

// internal: a continuation record of a settled board with no legal move (the
// row shuffle comes next), as opposed to one paused before a cascade iteration
constexpr uint32_t FLAG_CONT_DEAD = 0x80u;

// One Match3Env.step of board b. With DEFER (k_env_step), the cascade stops
// after `limit` inner iterations and at a dead board (the shuffle path is left
// out of the kernel): the step returns ENV_STEP_PAUSED with its state in P,
// rng, r, f (f & FLAG_CONT_DEAD: dead) and has written nothing yet; k_env_cont_grid
// finishes it. Without DEFER the whole step runs here.
template <class CF, bool DEFER, class RNG, class Store>
__device__ __forceinline__ int env_step_one(typename CF::Bd* P, const EnvArgs& a, int64_t b, RNG& rng, Store& st,
                                            int limit, int& r, uint32_t& f, const typename CF::Dim& dm,
                                            uint8_t* row = nullptr, FinOpts o = FinOpts{}) {
    // every per-board input is loaded before the cascade, so its latency hides behind it
    const int act_in = a.actions ? a.actions[b] : a.next_action[b];
    const int mv = a.moves[b];
    const int sc0 = a.score[b];
    typename CF::Bd HL, VL;
    if (apply_begin<CF>(P, a.num_moves - mv, act_in, rng, f, HL, VL, st, r, dm)) {
        const int c = apply_cascade_ex<CF, DEFER ? CASX_STOP_DEAD : 0>(P, rng, f, HL, VL, st, r, limit, false, dm);
        if (!(f & FLAG_RECOMPUTE)) {
            if (c == CAS_PAUSED) return ENV_STEP_PAUSED;
            if (c == CAS_DEAD) {
                f |= FLAG_CONT_DEAD;
                return ENV_STEP_PAUSED;
            }
        }
    }
    if (f & FLAG_RECOMPUTE) return ENV_STEP_RECOMPUTE;
    return env_finish<CF>(P, a, b, rng, st, r, f, HL, VL, mv, sc0, dm, row, o) ? ENV_STEP_DONE
                                                                                      : ENV_STEP_RECOMPUTE;
}

// Continuation records of paused steps (KS::CASCADE_LIMIT): word 0 the
// shard-local board index, words 1.. the Cont state, padded to CONT_REC words
// (9x9x6: 32 words, 128 B) so a lane writes and reads its record with 16-byte
// accesses -- 8 instructions each way instead of one per word (round 5 wrote them
// SoA, word w of record q at cont[w * n + q]: 31 stores per wave). Record q at
// cont[q * CONT_REC]; the step's counter block [CNT_CONT] counts them.
template <class CF>
using EnvCont = Cont<CF, typename KS<CF>::Rng>;
template <class CF>
constexpr int CONT_REC = (1 + EnvCont<CF>::WORDS + 3) & ~3;

template <class CF>
__device__ __forceinline__ void cont_store(uint32_t* rec, uint32_t b, const typename CF::Bd* P,
                                           const typename KS<CF>::Rng& rng, int r, uint32_t f) {
    constexpr int RW = CONT_REC<CF>;
    uint32_t w[RW];
    w[0] = b;
    EnvCont<CF>::save(P, rng, r, f, [&](int i, uint32_t x) { w[i + 1] = x; });
#pragma unroll
    for (int i = 1 + EnvCont<CF>::WORDS; i < RW; ++i) w[i] = 0u;
    uint4* d = reinterpret_cast<uint4*>(rec);
#pragma unroll
    for (int k = 0; k < RW / 4; ++k) d[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
}

template <class CF>
__device__ __forceinline__ int64_t cont_load(const uint32_t* rec, typename CF::Bd* P, typename KS<CF>::Rng& rng,
                                             int& r, uint32_t& f) {
    constexpr int RW = CONT_REC<CF>;
    uint32_t w[RW];
    const uint4* s = reinterpret_cast<const uint4*>(rec);
#pragma unroll
    for (int k = 0; k < RW / 4; ++k) {
        const uint4 v = s[k];
        w[4 * k] = v.x;
        w[4 * k + 1] = v.y;
        w[4 * k + 2] = v.z;
        w[4 * k + 3] = v.w;
    }
    EnvCont<CF>::load(P, rng, r, f, [&](int i) { return w[i + 1]; });
    return (int64_t)w[0];
}

template <class CF>
__global__ void __launch_bounds__(KS<CF>::B, KS<CF>::STEP_WPS) k_env_step(EnvArgs a) {
    // The board staging area is only live before the cascade (HBM -> LDS ->
    // planes) and after it (planes -> LDS -> HBM), the match-group table only
    // inside it; with one wave per workgroup nothing else can touch the LDS
    // in between, so the two share storage (9 KB per wave at 9x9: the 6-slot table).
    using K = KS<CF>;
    if constexpr (M3_STEP_PRIO > 0) __builtin_amdgcn_s_setprio(M3_STEP_PRIO);
    static_assert(K::B == 64, "staging/table aliasing assumes one wave per workgroup");
    // 16x16: staging rows padded by 16 B (block_copy_in_rows)
    constexpr int RPAD = (!CF::DYN && CF::N % 64 == 0 && M3_STAGE_PAD) ? 16 : 0;
    constexpr int STAGE_WORDS = (K::B * (CF::N + RPAD) + 16 + 3) / 4;
    constexpr int TAB_WORDS = LdsStore<CF, K::GCAP, K::B>::WORDS;
    __shared__ __attribute__((aligned(16))) uint32_t stage_tab[STAGE_WORDS > TAB_WORDS ? STAGE_WORDS : TAB_WORDS];
    uint8_t* const lds = reinterpret_cast<uint8_t*>(stage_tab);
    uint32_t* const gtab = stage_tab;
    const typename CF::Dim dm(a.shape);
    const int NC = dm.cells();
    const int64_t b0 = (int64_t)blockIdx.x * KS<CF>::BPW;
    const int nb = (int)((a.n - b0) < KS<CF>::BPW ? (a.n - b0) : KS<CF>::BPW);
    if constexpr (RPAD) block_copy_in_rows<KS<CF>::B, CF::N, RPAD>(a.cur + b0 * NC, lds, nb * NC);
    else block_copy_in<KS<CF>::B>(a.cur + b0 * NC, lds, nb * NC);
    const int t = threadIdx.x;
    const uint32_t cslot = t < nb ? a.slot[b0 + t] : 0u;
    lds_sync();
#ifdef M3_PHASE_PROF
    M3_PROF_LDS(KS<CF>::B)
    Prof<LdsStore<CF, KS<CF>::GCAP, KS<CF>::B>> st;
    st.tab = as_lds(gtab + t);
    st.w = prof_s[t >> 6];
    const bool live = ((t & ~63) < nb);
    if (live) st.begin();
#else
    LdsStore<CF, KS<CF>::GCAP, KS<CF>::B> st{as_lds(gtab + t)};
#endif
    st.spill = a.spill;
    st.pool_next = &a.counters[CNT_SPILL];
    st.pool_cap = K::SPILL_RECORDS;
    bool reset_lane = false;  // (M3_COOP_CELLS: the wave copies the resetting lanes' next cells below)
    int64_t reset_ob = 0;
    if (t < nb) {
        const int64_t b = b0 + t;
        typename CF::Bd P[CF::NP];
        lds_to_planes<CF>(lds + t * RPAD, t, P, dm);  // (every lane of the wave, before any group-table write)
        typename K::Rng rng;
        rng.init(a.seeds[b], a.m397[(int64_t)cslot * a.cstride + b]);
        int r;
        uint32_t f;
        int res;
        // a finished step leaves its board bytes (or the next episode's) in its staging row
        uint8_t* const row = lds + t * (NC + RPAD);
        if constexpr (K::CASCADE_LIMIT >= 0) {  // (a.cont is set)
            // env_step_one<CF, true> with the epilogue split round one atomic per wave: the
            // decisions of every lane (paused, or finished and resetting), then the wave's
            // continuation records and prefetch queue entries in one 64-bit atomicAdd, then the
            // stores (see env_finish)
            const int act_in = a.actions ? a.actions[b] : a.next_action[b];
            const int mv = a.moves[b];
            const int sc0 = a.score[b];
            typename CF::Bd HL, VL;
            res = ENV_STEP_DONE;
            if (apply_begin<CF>(P, a.num_moves - mv, act_in, rng, f, HL, VL, st, r, dm)) {
                const int c =
                    apply_cascade_ex<CF, CASX_STOP_DEAD>(P, rng, f, HL, VL, st, r, K::CASCADE_LIMIT, false, dm);
                if (!(f & FLAG_RECOMPUTE)) {
                    if (c == CAS_PAUSED) {
                        res = ENV_STEP_PAUSED;
                    } else if (c == CAS_DEAD) {
                        f |= FLAG_CONT_DEAD;
                        res = ENV_STEP_PAUSED;
                    }
                }
            }
            if (f & FLAG_RECOMPUTE) res = ENV_STEP_RECOMPUTE;
            EnvFin<CF> e;
            const uint32_t seed_in = rng.seed;
            if (res == ENV_STEP_DONE &&
                !env_fin_begin<CF>(P, a, b, rng, st, r, f, HL, VL, mv, sc0, dm, row, e, &cslot, &seed_in, !M3_COOP_CELLS))
                res = ENV_STEP_RECOMPUTE;
            const bool fin = res == ENV_STEP_DONE, paused = res == ENV_STEP_PAUSED;
            const bool reset = fin && e.reset;
            const uint64_t mp = __ballot(paused), mr = __ballot(reset);
            uint32_t cbase = 0u, qbase = 0u;
            int leader = 0;
            if (mp | mr) {
                leader = __ffsll((unsigned long long)(mp | mr)) - 1;
                if ((int)__lane_id() == leader) {
                    const unsigned long long add =
                        (unsigned long long)__popcll(mp) | ((unsigned long long)__popcll(mr) << 32);
                    const unsigned long long old =
                        atomicAdd(reinterpret_cast<unsigned long long*>(&a.counters[CNT_CONT]), add);
                    cbase = (uint32_t)old;
                    qbase = (uint32_t)(old >> 32);
                }
            }
            if (res == ENV_STEP_RECOMPUTE) {  // (rare; its row is rewritten by k_env_fix)
                const uint32_t slot = atomicAdd(&a.counters[CNT_OVF], 1u);
                a.ovf_list[slot] = (uint32_t)b;
            }
            prof_drain(st);
            mark<PH_TATOM>(st);
            if (fin) env_fin_store<CF>(P, a, b, st, e, dm, row, !M3_COOP_CELLS);
            reset_lane = reset;
            reset_ob = e.ob;
            if (mp | mr) {
                cbase = __shfl(cbase, leader);
                qbase = __shfl(qbase, leader);
                if (reset) env_fin_queue(a, b, qbase + lane_rank(mr), e.seed, e.s_old);
                // paused steps leave a continuation record; their rows are rewritten by k_env_cont_grid
                // (round 6 A/B: the record at the board's own index before the atomic and only the index
                // in the compacted list -- equal speed, one more dependent load in k_env_cont_grid)
                if (paused)
                    cont_store<CF>(a.cont + (int64_t)(cbase + lane_rank(mp)) * CONT_REC<CF>, (uint32_t)b, P, rng, r, f);
            }
            mark<PH_QUEUE>(st);
        } else {
            FinOpts o;
            const uint32_t seed_in = rng.seed;
            if constexpr (!CF::DYN) {
                o.slot = &cslot;
                o.seed = &seed_in;
                o.cells = !M3_COOP_CELLS;
                o.reset = &reset_lane;
                o.ob = &reset_ob;
            }
            res = env_step_one<CF, false>(P, a, b, rng, st, -1, r, f, dm, row, o);
            if (res == ENV_STEP_RECOMPUTE) {  // (its row is rewritten by k_env_fix)
                const uint32_t slot = atomicAdd(&a.counters[CNT_OVF], 1u);
                a.ovf_list[slot] = (uint32_t)b;
            }
        }
    }
    if constexpr (M3_COOP_CELLS && !CF::DYN) {
        const uint64_t mr = __ballot(reset_lane);  // (all 64 lanes: a ragged last wave too)
        if (mr) coop_reset_cells<CF>(a, mr, reset_ob, lds, NC + RPAD);
    }
    lds_sync();
    if constexpr (RPAD) block_copy_out_rows<KS<CF>::B, CF::N, RPAD>(a.nxt + b0 * NC, lds, nb * NC);
    else block_copy_out<KS<CF>::B>(a.nxt + b0 * NC, lds, nb * NC);
#ifdef M3_PHASE_PROF
    if (live) st.end(0);
#endif
}

// Finish the steps k_env_step paused (their cascade ran past KS::CASCADE_LIMIT
// inner iterations, or it settled on a board with no legal move: the row
// shuffle): the long cascades of a launch, packed densely into waves instead
// of holding every lane of their k_env_step wave idle. Grid-stride over the
// records; each board is written straight to nxt.
template <class CF>
__global__ void __launch_bounds__(KS<CF>::B, KS<CF>::CONT_WPS) k_env_cont_grid(EnvArgs a) {
    using K = KS<CF>;
    // The few waves of this kernel are the step's critical path; they share SIMDs with
    // the other shard's step waves and the resets: issue first (A/B: within noise).
    __builtin_amdgcn_s_setprio(3);
    __shared__ uint32_t tab[LdsStore<CF, K::GCAP, K::B>::WORDS];
    const uint32_t cnt = a.counters[CNT_CONT];
    LdsStore<CF, K::GCAP, K::B> st{as_lds(tab + threadIdx.x)};
    st.spill = a.spill;
    st.pool_next = &a.counters[CNT_SPILL];
    st.pool_cap = K::SPILL_RECORDS;
    for (uint32_t q = blockIdx.x * K::B + threadIdx.x; q < cnt; q += gridDim.x * K::B) {
        typename CF::Bd P[CF::NP];
        typename K::Rng rng;
        int r;
        uint32_t f;
        const int64_t b = cont_load<CF>(a.cont + (int64_t)q * CONT_REC<CF>, P, rng, r, f);
        const int mv = a.moves[b], sc0 = a.score[b];
        typename CF::Bd HL, VL;
        const bool dead = (f & FLAG_CONT_DEAD) != 0;  // settled with no legal move: continue at the shuffle
        f &= ~FLAG_CONT_DEAD;
        const typename CF::Dim dm(a.shape);
        apply_cascade_ex<CF, 0>(P, rng, f, HL, VL, st, r, -1, dead, dm);
        const bool ok = !(f & FLAG_RECOMPUTE) && env_finish<CF>(P, a, b, rng, st, r, f, HL, VL, mv, sc0, dm);
        if (!ok) {
            const uint32_t slot = atomicAdd(&a.counters[CNT_OVF], 1u);
            a.ovf_list[slot] = (uint32_t)b;
        } else {
            planes_to_bytes<CF>(P, reinterpret_cast<uint8_t*>(a.nxt + b * dm.cells()), dm);
        }
    }
}

// k_env_fix runs on the step stream between two steps of a shard and almost never has work
// (16x16x8: 7 recomputed boards in 50 steps of 262,144); at 512 VGPRs (16x16x8) its waves can only
// start on a SIMD with no other wave resident (31 us average launch duration in the trace).
// M3_FIX_LEAN=1: the specialised shapes run it one board per wave under a 128-VGPR bound (the rare
// recompute spills to scratch; one active lane, so no divergence under the spills). Measured OFF:
// 16x16x8 0.74-0.75 vs 0.80 G env-steps/s, 9x9 equal (gpurun_out/r05ac) -- the launch was not
// what held the shard's stream.
#ifndef M3_FIX_LEAN
#define M3_FIX_LEAN 0
#endif
template <class CF>
constexpr uint32_t env_fix_lanes() { return (!CF::DYN && M3_FIX_LEAN) ? 1u : lanes_for<CF>(); }
template <class CF>
constexpr int ENV_FIX_WPS = (!CF::DYN && M3_FIX_LEAN) ? 4 : 1;

template <class CF>
__global__ void __launch_bounds__(FIX_BLOCK, ENV_FIX_WPS<CF>) k_env_fix(EnvArgs a) {
    const uint32_t cnt = a.counters[CNT_OVF];
    if (blockIdx.x == 0 && threadIdx.x == 0 && cnt) atomicAdd(&a.stats[0], cnt);
    if (a.zero_next && blockIdx.x == 0 && threadIdx.x < 8) a.zero_next[threadIdx.x] = 0u;  // (CBLOCKS)
    const typename CF::Dim dm(a.shape);
    constexpr uint32_t L = env_fix_lanes<CF>();
    for (uint32_t i = blockIdx.x * L + threadIdx.x; threadIdx.x < L && i < cnt; i += gridDim.x * L) {
        const int64_t b = a.ovf_list[i];
        typename CF::Bd P[CF::NP];
        bytes_to_planes<CF>(a.cur + b * dm.cells(), P, dm);
        ArrayStore<CF> st;
        int r;
        uint32_t f;
        int res = ENV_STEP_RECOMPUTE;
        if constexpr (std::is_same_v<typename KS<CF>::Chain, ChainMT1>) {
            // the step ran out of the one-level chain (> 226 draws): the
            // three-level chain covers the whole first block in registers,
            // where FullMT would walk 2.5 KB of scratch state at memory
            // latency on the step's critical path
            ChainMT cm;
            cm.init(a.seeds[b], a.m397[(int64_t)a.slot[b] * a.cstride + b]);
            res = env_step_one<CF, false>(P, a, b, cm, st, -1, r, f, dm);
            if (res == ENV_STEP_RECOMPUTE) bytes_to_planes<CF>(a.cur + b * dm.cells(), P, dm);
        }
        if (res == ENV_STEP_RECOMPUTE) {  // >= 624 draws
            FullMT mt;  // scratch (see k_apply_fix)
            mt.init(a.seeds[b], 0u);
            env_step_one<CF, false>(P, a, b, mt, st, -1, r, f, dm);
        }
        planes_to_bytes<CF>(P, reinterpret_cast<uint8_t*>(a.nxt + b * dm.cells()), dm);
    }
}

// ---------------------------------------------------------------------------
// batched MCTS rollouts (mctslib/standard/mcts.py:14-19)
// ---------------------------------------------------------------------------
// One rollout per lane: np.random.seed(rseed); while n_actions >= 1:
// action = choice(legal_actions) from the global stream, state =
// apply_action(action). The first choice reads the stream of rseed; every
// later one reads the stream apply_action left behind (cfg.seed reseeded at
// boardv2.py:46, advanced by the step's draws), i.e. the same register chain
// the step just used. The match-group table is the env's LDS table + spill
// pool, and a lane keeps its spill record for the whole rollout; a rollout
// that overflows the chain (>= 624 draws in one step) or the pool is
// replayed from its first move by k_rollout_fix.
}  // namespace
// launcher signatures name this struct: it needs linkage (m3_inst.hip instantiates them)
namespace m3k {
struct RolloutArgs {
    Shape shape;
    int64_t n;
    const int8_t* boards;
    const uint32_t* seeds;     // cfg.seed of each state
    const int32_t* n_actions;
    const uint32_t* rseeds;    // rollout seed (random.randint(0, 2**31 - 1) or state.seed)
    int32_t* gain;             // sum of the step rewards of the rollout
    int32_t* steps;            // apply_action calls
    uint32_t* draws;           // global-stream draws since its last seed when the rollout ends
    uint32_t* flags;           // OR of the steps' M3_FLAG_*
    int8_t* out_boards;        // nullable: terminal boards
    uint32_t* counters;        // [0] overflow count, [1] spill records taken, [2] waves with a bad cell
    uint32_t* ovf_list;
    uint32_t* spill;
    uint32_t spill_cap;
};
}  // namespace m3k
using m3k::RolloutArgs;
namespace {

template <class CF, class RNG, class Store>
__device__ __forceinline__ bool rollout_one(typename CF::Bd* P, const RolloutArgs& a, int64_t b, RNG& first, RNG& rng,
                                            Store& st, const typename CF::Dim& dm) {
    int n = a.n_actions[b];
    int gain = 0, steps = 0;
    uint32_t fl = 0u, dr = 0u;
    if (n >= 1) {                                               // mcts.py:16 while not is_terminal
        typename CF::Bd HL, VL;
        legal_masks<CF>(P, special_mask<CF, CF::NP>(P), HL, VL, dm);
        uint32_t act[CF::AW];
        action_bits<CF>(HL, VL, act, dm);
        int x = random_action<CF>(act, first);                  // mcts.py:17, stream of the rollout seed
        dr = first.draws();
        for (;;) {
            if (x < 0) {                                        // np.random.choice([]) raises
                fl |= FLAG_NO_LEGAL;
                break;
            }
            uint32_t f;
            const int r = apply_action<CF>(P, n, x, rng, f, HL, VL, st, dm);  // mcts.py:18
            if (f & FLAG_RECOMPUTE) return false;
            fl |= f;
            gain += r;
            ++steps;
            --n;
            dr = rng.draws();
            if (n < 1) break;
            action_bits<CF>(HL, VL, act, dm);
            x = random_action<CF>(act, rng);                    // stream where apply_action left it
            if (rng.overflow) return false;
            dr = rng.draws();
        }
    }
    a.gain[b] = gain;
    a.steps[b] = steps;
    a.draws[b] = dr;
    a.flags[b] = fl;
    return true;
}

template <class CF>
__global__ void __launch_bounds__(KS<CF>::B, KS<CF>::STEP_WPS) k_rollout(RolloutArgs a) {
    using K = KS<CF>;
    static_assert(K::B == 64, "staging/table aliasing assumes one wave per workgroup");
    // staging and match-group table share the LDS (as in k_env_step)
    constexpr int STAGE_WORDS = (K::B * CF::N + 16 + 3) / 4;
    constexpr int TAB_WORDS = LdsStore<CF, K::GCAP, K::B>::WORDS;
    __shared__ __attribute__((aligned(16))) uint32_t stage_tab[STAGE_WORDS > TAB_WORDS ? STAGE_WORDS : TAB_WORDS];
    uint8_t* const lds = reinterpret_cast<uint8_t*>(stage_tab);
    const typename CF::Dim dm(a.shape);
    const int NC = dm.cells();
    const int64_t b0 = (int64_t)blockIdx.x * K::BPW;
    const int nb = (int)((a.n - b0) < K::BPW ? (a.n - b0) : K::BPW);
    flag_bad_cells(block_copy_in_checked<K::B>(a.boards + b0 * NC, lds, nb * NC), &a.counters[2]);
    lds_sync();
    const int t = threadIdx.x;
    typename CF::Bd P[CF::NP];
    if (t < nb) lds_to_planes<CF>(lds, t, P, dm);
    lds_sync();
    LdsStore<CF, K::GCAP, K::B> st{as_lds(stage_tab + t)};
    st.spill = a.spill;
    st.pool_next = &a.counters[1];
    st.pool_cap = a.spill_cap;
    if (t < nb) {
        const int64_t b = b0 + t;
        const uint32_t rs = a.rseeds[b], s = a.seeds[b];
        typename K::Chain first, rng;  // a step past the chain's reach replays the rollout in k_rollout_fix
        first.init(rs, mt_state397(rs));
        rng.init(s, mt_state397(s));
        if (!rollout_one<CF>(P, a, b, first, rng, st, dm)) {
            const uint32_t o = atomicAdd(&a.counters[0], 1u);
            a.ovf_list[o] = (uint32_t)b;
        }
    }
    if (!a.out_boards) return;
    lds_sync();
    if (t < nb) planes_to_bytes<CF>(P, lds + t * NC, dm);
    lds_sync();
    block_copy_out<K::B>(a.out_boards + b0 * NC, lds, nb * NC);
}

// exact replay of overflowed rollouts: 624-word MT19937 states and the full
// group table in lane-private scratch
template <class CF>
__global__ void __launch_bounds__(FIX_BLOCK) k_rollout_fix(RolloutArgs a) {
    const uint32_t cnt = a.counters[0];
    const typename CF::Dim dm(a.shape);
    for (uint32_t i = blockIdx.x * lanes_for<CF>() + threadIdx.x; threadIdx.x < lanes_for<CF>() && i < cnt;
         i += gridDim.x * lanes_for<CF>()) {
        const int64_t b = a.ovf_list[i];
        typename CF::Bd P[CF::NP];
        bytes_to_planes<CF>(a.boards + b * dm.cells(), P, dm);
        FullMT first, rng;
        first.init(a.rseeds[b], 0u);
        rng.init(a.seeds[b], 0u);
        ArrayStore<CF> st;
        rollout_one<CF>(P, a, b, first, rng, st, dm);
        if (a.out_boards) planes_to_bytes<CF>(P, reinterpret_cast<uint8_t*>(a.out_boards + b * dm.cells()), dm);
    }
}

// ---------------------------------------------------------------------------
// shape dispatch
// ---------------------------------------------------------------------------
#define M3_SHAPES(X) \
    X(9, 9, 6)       \
    X(16, 16, 8)

constexpr int N_SPECIALISED = 2;
// Specialised shapes first (ids 0..N_SPECIALISED-1), then the frame configs
// FCfg<2..5> (ids N_SPECIALISED + BITS - 2) for every other shape with rows
// and columns 3..16, and FCfg<2..5, 32> (ids N_SPECIALISED + 4 + BITS - 2)
// for rows and columns 3..32 with a side above 16; types 2..31. (types = 2: from about 7x7 up a refill
// of two colours almost always leaves a match, so the reference's cascade
// does not return -- steps here stop at CASCADE_CAP refills and flag it -- and
// a large board's reset can take millions of draws -- stopped at
// RESET_ROUND_CAP rounds and flagged; types = 1: the reset never ends.)
int shape_id(int r, int c, int t) {
    int id = 0;
#define X(R_, C_, T_)                                 \
    if (r == R_ && c == C_ && t == T_) return id; \
    ++id;
    M3_SHAPES(X)
#undef X
    if (r < 3 || c < 3 || r > MAX_FRAME || c > MAX_FRAME || t < 2 || t > 31) return -1;
    return N_SPECIALISED + (frame_side(r, c) == 32 ? 4 : 0) + bits_for_types(t) - 2;
}

}  // namespace

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
struct m3_ctx {
    int device = 0;
    int R = 0, C = 0, T = 0, N = 0, A = 0, AW = 0;
    int shape = -1;
    Shape sdesc{};  // kernel argument: the board shape (+ its id-reachable swaps)
    hipStream_t stream = nullptr;
    // stateless scratch
    void* dbuf = nullptr;
    size_t dcap = 0;
    // pinned host staging of the host-buffer calls: inputs go up as one image, outputs come back
    // as one image (one copy each way per call, include/m3.h "stateless batch calls")
    void* hbuf = nullptr;
    void* hdev = nullptr;  // hbuf as the device addresses it (zero-copy calls)
    size_t hcap = 0;
    uint32_t* counters = nullptr;  // rollouts: [0] overflow count, [1] spill records, [2] bad-cell waves
};

struct m3_env {
    m3_ctx* ctx = nullptr;
    int64_t n = 0;
    int num_moves = 20, goal = 500;
    int autoreset = 0;
    uint32_t stride = 0;
    bool ready = false;  // every state field holds a board's state (m3_env_reset, or m3_env_set of each)
    uint32_t loaded = 0; // bit `what` per field m3_env_set has loaded since create (ready once all are)
    // M3_ENV_LEGAL is derived from the boards: the step kernels write it only once a caller has
    // asked for its device pointer (a device consumer reads it every step); m3_env_get computes it
    // on request otherwise (20 B per board and step fewer writes)
    bool legal_eager = false;
    bool stale = false;  // fields were loaded with m3_env_set: rederive() before the next step
    int8_t* boards[2] = {nullptr, nullptr};
    int cur = 0;
    uint32_t *seeds = nullptr, *flags = nullptr, *draws = nullptr, *legal = nullptr;
    int32_t *score = nullptr, *moves = nullptr, *next_action = nullptr, *reward = nullptr;
    uint8_t *done = nullptr, *trunc = nullptr;
    // host-action steps (m3_env_step with actions): device copies and pinned
    // staging, double-buffered by step parity like `packed`, uploaded on
    // `ustream` (allocated on first use)
    int32_t* actions[2] = {nullptr, nullptr};
    int32_t* hstage[2] = {nullptr, nullptr};
    hipStream_t ustream = nullptr;
    hipEvent_t upload_ev[2] = {nullptr, nullptr};
    bool upload_pend[2] = {false, false};  // upload_ev[p] recorded and not yet waited on by the host
    bool upload_this = false;              // the step being enqueued reads actions[step & 1]
    // counters, 64 words per shard: [8q + CNT_*] (q = step % CBLOCKS): step overflow count,
    // deferred prefetch resets, spill records taken, continuation records | prefetch queue
    // length (one 64-bit word); stats
    // [40] step recomputes, [41] resets, [42] reset recomputes; [48 + k] the
    // reset / slot-fill overflow counts (shard 0's block)
    uint32_t* counters = nullptr;
    uint32_t* ovf_list = nullptr;
    uint32_t* spill = nullptr;  // group-table spill pools, one per shard slot
    // NSLOT episode slots per board (see EnvArgs): the current episode's
    // stream cache + the next episodes' initial state and cache
    uint8_t* slot = nullptr;
    uint32_t* ne_words = nullptr;
    int32_t* ne_first = nullptr;
    uint32_t* ne_legal = nullptr;
    uint32_t* ne_flags = nullptr;  // [NSLOT][n] M3_FLAG_RESET_CAP of each slot's reset
    uint32_t* m397 = nullptr;  // [NSLOT][n]
    uint32_t* cont = nullptr;  // continuation records of paused steps [n][CONT_REC] (k_env_cont_grid)
    uint32_t* defer = nullptr; // prefetch resets k_init leaves to k_init_coop [n]
    uint32_t* tab = nullptr;   // two-stage reset table rows [n][TwoStage::TW] (16x16x8)
    // prefetch queues and their overflow lists, by step % PF_LAG
    uint32_t *pf_list[PF_LAG] = {}, *pf_seed[PF_LAG] = {}, *pf_slot[PF_LAG] = {};
    int64_t steps = 0;
    int32_t* packed = nullptr;
    int32_t* gathered = nullptr;
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    // per-step kernel timing ring (bench.py roofline): event pair i brackets
    // the i-th k_env_step launch since m3_env_timing(enable)
    std::vector<hipEvent_t> tev;
    int tcap = 0, tn = 0;
    // Independent board shards, each with a step stream (step + fixup) and a
    // prefetch stream (next-episode resets). Step t of a shard waits only for
    // the prefetch of step t - PF_LAG, so resets overlap the following steps.
    struct Shard {
        int64_t off = 0, n = 0;
        hipStream_t stream = nullptr, pstream = nullptr;
        hipEvent_t ev = nullptr;       // last step work of this shard
        hipEvent_t aev[2] = {};        // step work of the last step of each parity (reads actions[parity])
        bool apending[2] = {};
        hipEvent_t pev[PF_LAG] = {};   // prefetch of queue q done
        bool ppending[PF_LAG] = {};
    };
    std::vector<Shard> shards;
    // `packed` is double-buffered by step parity, so the RCCL gather of step t
    // (context stream) overlaps step t+1; step t+2 waits for it (gev[buffer])
    hipEvent_t gev[2] = {nullptr, nullptr};
    bool gpend[2] = {false, false};
};

// The configurations by id (shape_id / with_shape in m3_api.hip).
using CF_0 = Cfg<9, 9, 6>;
using CF_1 = Cfg<16, 16, 8>;
using CF_2 = FCfg<2>;
using CF_3 = FCfg<3>;
using CF_4 = FCfg<4>;
using CF_5 = FCfg<5>;
using CF_6 = FCfg<2, 32>;
using CF_7 = FCfg<3, 32>;
using CF_8 = FCfg<4, 32>;
using CF_9 = FCfg<5, 32>;
constexpr int N_CONFIGS = 10;

namespace m3k {

// fix-pass blocks: FIX_GRID x 64 active lanes in all
template <class CF>
int fix_grid() { return (int)(FIX_GRID * 64 / lanes_for<CF>()); }

template <class CF>
int grid_for(int64_t n) { return (int)((n + KS<CF>::BPW - 1) / KS<CF>::BPW); }

template <class CF>
int launch_apply(m3_ctx* c, const ApplyArgs& a) {
    if (a.n == 0) return M3_OK;  // (*a.ovf_count and *a.bad_cells are zero: the caller's upload)
    hipLaunchKernelGGL(k_apply<CF>, dim3(grid_for<CF>(a.n)), dim3(KS<CF>::B), 0, c->stream, a);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_apply_fix<CF>, dim3(a.clear_ovf ? 1 : fix_grid<CF>()), dim3(FIX_BLOCK), 0, c->stream, a);
    HIP_TRY(hipGetLastError());
    return M3_OK;
}

template <class CF>
int launch_init(hipStream_t stream, const InitArgs& a, int64_t max_items) {
    if (max_items == 0) return M3_OK;
    int64_t g = (max_items + INIT_BLOCK - 1) / INIT_BLOCK;
    if (g > 4096) g = 4096;
    // env prefetch (a.defer): the reset kernels grid-stride over the queue, and their waves share the
    // CUs with the step kernels (k_init holds ~10 KB of LDS per wave, about one step wave's
    // worth); capping their grids bounds how many run at once. The queue is needed PF_LAG steps later.
    const int64_t pf_cap = a.defer ? (int64_t)M3_PF_GRID : 0, coop_cap = a.defer ? (int64_t)M3_PF_COOP_GRID : 0;
    if (pf_cap > 0 && g > pf_cap) g = pf_cap;
    if constexpr (INIT_INLINE_FIX<CF>) {
        if constexpr (RESET_TWO_STAGE_REJ<CF>) {
            if (a.tab && a.defer) {  // 9x9x6 env prefetch (m3_reset9.hpp)
                int64_t ga = (max_items + TwoStageRej<CF>::G - 1) / TwoStageRej<CF>::G;
                ga = ga > 2048 ? 2048 : ga;
                hipLaunchKernelGGL(k_reset_stream_rej<CF>, dim3((unsigned)ga), dim3(64), 0, stream, a);
                HIP_TRY(hipGetLastError());
                hipLaunchKernelGGL(k_reset_tiles_rej<CF>, dim3((unsigned)g), dim3(64), 0, stream, a);
                HIP_TRY(hipGetLastError());
                int64_t gc = max_items / 64 + 1;  // the few past the table's rounds
                gc = gc < 64 ? 64 : (gc > 4096 ? 4096 : gc);
                if (coop_cap > 0 && gc > coop_cap) gc = coop_cap;
                hipLaunchKernelGGL(k_init_coop<CF>, dim3((unsigned)gc), dim3(64), 0, stream, a);
                HIP_TRY(hipGetLastError());
                return M3_OK;
            }
        }
        if (a.defer) hipLaunchKernelGGL((k_init<CF, false>), dim3((unsigned)g), dim3(INIT_BLOCK), 0, stream, a);
        else hipLaunchKernelGGL((k_init<CF, true>), dim3((unsigned)g), dim3(INIT_BLOCK), 0, stream, a);
        if (a.defer) {  // sized for the usual ~4 % deferred share, grid-strided
            HIP_TRY(hipGetLastError());
            int64_t gc = max_items / 16 + 1;
            gc = gc < 64 ? 64 : (gc > M3_COOP_GMAX ? M3_COOP_GMAX : gc);
            if (coop_cap > 0 && gc > coop_cap) gc = coop_cap;
            hipLaunchKernelGGL(k_init_coop<CF>, dim3((unsigned)gc), dim3(64), 0, stream, a);
        }
    } else if constexpr (!CF::DYN && M3_RESET16_CHAIN2) {  // 16x16x8: ~60 % of resets need the second MT block
        hipLaunchKernelGGL(k_init_chain2<CF>, dim3((unsigned)g), dim3(INIT_BLOCK), 0, stream, a);
        if (a.defer) {  // the ~2 % past draw 1248, one wave per board
            HIP_TRY(hipGetLastError());
            int64_t gc = max_items / 32 + 1;
            gc = gc < 64 ? 64 : (gc > 4096 ? 4096 : gc);
            hipLaunchKernelGGL(k_init_coop<CF>, dim3((unsigned)gc), dim3(64), 0, stream, a);
        }
    } else if (RESET_TWO_STAGE<CF> && a.tab && a.defer) {  // 16x16x8 env prefetch (see k_reset_stream)
        if constexpr (RESET_TWO_STAGE<CF>) {
            const InitArgs& s = a;
            int64_t ga = (max_items + TwoStage<CF>::G - 1) / TwoStage<CF>::G;
            ga = ga > 2048 ? 2048 : ga;
            if (pf_cap > 0 && ga > pf_cap) ga = pf_cap;
            hipLaunchKernelGGL(k_reset_stream<CF>, dim3((unsigned)ga), dim3(64), 0, stream, s);
            HIP_TRY(hipGetLastError());
            hipLaunchKernelGGL(k_reset_tiles<CF>, dim3((unsigned)(g > 4096 ? 4096 : g)), dim3(64), 0, stream, s);
            HIP_TRY(hipGetLastError());
            int64_t gc = max_items / 32 + 1;  // the ~2 % past the table's rounds
            gc = gc < 64 ? 64 : (gc > M3_COOP_GMAX ? M3_COOP_GMAX : gc);
            if (coop_cap > 0 && gc > coop_cap) gc = coop_cap;
            hipLaunchKernelGGL(k_init_coop<CF>, dim3((unsigned)gc), dim3(64), 0, stream, a);
        }
    } else {  // frame shapes: FullMT (lane-private scratch); 32 x 32 frame: one board per wave
        const int64_t gl = (max_items + lanes_for<CF>() - 1) / lanes_for<CF>();
        hipLaunchKernelGGL(k_init_fix_lane<CF>, dim3((unsigned)(gl > 4096 ? 4096 : gl)), dim3(INIT_FIX_BLOCK), 0,
                           stream, a);
    }
    HIP_TRY(hipGetLastError());
    return M3_OK;
}

template <class CF>
int launch_legal(m3_ctx* c, int64_t n, const int8_t* boards, uint32_t* legal) {
    if (n == 0) return M3_OK;
    hipLaunchKernelGGL(k_legal<CF>, dim3(grid_for<CF>(n)), dim3(KS<CF>::B), 0, c->stream, c->sdesc, n, boards, legal);
    HIP_TRY(hipGetLastError());
    return M3_OK;
}

// InitArgs of the prefetch (next-episode slots) of the boards from offset o.
template <class CF>
void prefetch_args(const m3_env* e, int64_t o, InitArgs& r) {
    r.shape = e->ctx->sdesc;
    r.sstride = e->n;
    r.board_words = e->ne_words + o * ((e->ctx->N + 3) / 4);
    r.first_action = e->ne_first + o;
    r.legal = e->ne_legal + o * e->ctx->AW;
    r.m397 = e->m397 + o;
    r.slot_flags = e->ne_flags + o;
    r.cstride = e->n;
    if constexpr (RESET_TWO_STAGE<CF>) r.tab = e->tab ? e->tab + o * TwoStage<CF>::TW : nullptr;
    if constexpr (RESET_TWO_STAGE_REJ<CF>) r.tab = e->tab ? e->tab + o * TwoStageRej<CF>::TW : nullptr;
}

// Enqueue one env step of shard s: on the step stream, wait for the prefetch
// of step t - PF_LAG (the queue and slots this step reuses), for the RCCL
// gather of step t - 2 (same `packed` buffer) and, for host actions, for
// their upload; zero this parity's counters, k_env_step (cur -> nxt, with
// the in-step autoreset swap) and k_env_fix (exact recompute of overflowed
// boards); on the prefetch stream, k_init + k_init_fix over the queued slots.
// Every pointer is offset to the shard, so kernels see shard-local indices.
template <class CF>
int launch_env_shard(m3_env* e, int s, const int32_t* d_actions) {
    m3_ctx* c = e->ctx;
    m3_env::Shard& sh = e->shards[s];
    if (sh.n == 0) return M3_OK;
    const int64_t o = sh.off;
    const int N = c->N, AW = c->AW;
    const int par = (int)(e->steps % PF_LAG);
    uint32_t* base = e->counters + 64 * s;
    uint32_t* cnt = base + 8 * (e->steps % CBLOCKS);
    hipStream_t st = sh.stream;
    const int pb = (int)(e->steps & 1);  // packed buffer of this step
    if (e->upload_this) HIP_TRY(hipStreamWaitEvent(st, e->upload_ev[pb], 0));  // host actions in actions[pb]
#ifndef M3_TEST_NO_GATHER_WAIT  // negative-control build for tests/test_gpu_dist.py only
    if (e->gpend[pb]) HIP_TRY(hipStreamWaitEvent(st, e->gev[pb], 0));          // gather of step t-2 still reading
#endif
    if (sh.ppending[par]) HIP_TRY(hipStreamWaitEvent(st, sh.pev[par], 0));  // queue + slots of step t - PF_LAG
    EnvArgs a{};
    a.shape = c->sdesc;
    a.n = sh.n;
    a.num_moves = e->num_moves;
    a.goal = e->goal;
    a.autoreset = e->autoreset;
    a.stride = e->stride;
    a.cur = e->boards[e->cur] + o * N;
    a.nxt = e->boards[e->cur ^ 1] + o * N;
    a.actions = d_actions ? d_actions + o : nullptr;
    a.seeds = e->seeds + o;
    a.score = e->score + o;
    a.moves = e->moves + o;
    a.next_action = e->next_action + o;
    a.reward = e->reward + o;
    a.done = e->done + o;
    a.trunc = e->trunc + o;
    a.flags = e->flags + o;
    a.draws = e->draws + o;
    a.legal = e->legal_eager ? e->legal + o * AW : nullptr;
    a.packed = e->comm ? e->packed + (size_t)pb * e->n + o : nullptr;  // only the RCCL gather reads it
    a.counters = cnt;
    a.spill = e->spill + (size_t)s * KS<CF>::SPILL_RECORDS * LdsStore<CF, KS<CF>::GCAP, KS<CF>::B>::SPILL_WORDS;
    a.stats = base + 40;
    a.ovf_list = e->ovf_list + o;
    a.slot = e->slot + o;
    a.ne_words = e->ne_words + o * ((N + 3) / 4);
    a.ne_first = e->ne_first + o;
    a.ne_legal = e->ne_legal + o * AW;
    a.ne_flags = e->ne_flags + o;
    a.pf_list = e->pf_list[par] + o;
    a.pf_seed = e->pf_seed[par] + o;
    a.pf_slot = e->pf_slot[par] + o;
    a.m397 = e->m397 + o;
    a.cstride = e->n;
    a.cont = KS<CF>::CASCADE_LIMIT >= 0 ? e->cont + o * CONT_REC<CF> : nullptr;
    a.cont_stride = CONT_REC<CF>;
    a.zero_next = base + 8 * ((e->steps + 1) % CBLOCKS);
    const bool timed = e->tn < e->tcap;
    if (timed) HIP_TRY(hipEventRecord(e->tev[3 * e->tn], st));
    hipLaunchKernelGGL(k_env_step<CF>, dim3(grid_for<CF>(sh.n)), dim3(KS<CF>::B), 0, st, a);
    HIP_TRY(hipGetLastError());
    if (timed) HIP_TRY(hipEventRecord(e->tev[3 * e->tn + 1], st));  // k_env_step alone (the dominant kernel)
    if constexpr (KS<CF>::CASCADE_LIMIT >= 0) {
        // grid-strides over the device-side count of paused steps: sized for their usual share (~20 % at limit 2)
        const int64_t g = ((int64_t)(sh.n * 0.25) + KS<CF>::B - 1) / KS<CF>::B;
        hipLaunchKernelGGL(k_env_cont_grid<CF>, dim3((unsigned)(g > 0 ? g : 1)), dim3(KS<CF>::B), 0, st, a);
        HIP_TRY(hipGetLastError());
    }
    // (one board per wave: 64 waves; else FIX_GRID x 64 lanes)
    hipLaunchKernelGGL(k_env_fix<CF>, dim3(env_fix_lanes<CF>() == 1u ? 64 : fix_grid<CF>()), dim3(FIX_BLOCK), 0, st, a);
    HIP_TRY(hipGetLastError());
    if (timed) {  // the whole step pipeline of the shard, fixup pass included
        HIP_TRY(hipEventRecord(e->tev[3 * e->tn + 2], st));
        e->tn++;
    }
    HIP_TRY(hipEventRecord(sh.ev, st));
    if (e->upload_this) {  // the upload two steps ahead rewrites actions[pb] once this shard has read it
        HIP_TRY(hipEventRecord(sh.aev[pb], st));
        sh.apending[pb] = true;
    }
    if (e->autoreset) {
        HIP_TRY(hipStreamWaitEvent(sh.pstream, sh.ev, 0));
        InitArgs r{};
        r.n = sh.n;
        r.list = e->pf_list[par] + o;
        r.list_seed = e->pf_seed[par] + o;
        r.list_slot = e->pf_slot[par] + o;
        r.list_count = &cnt[CNT_PF];
        r.stats = base + 41;
        if constexpr (INIT_INLINE_FIX<CF> || (!CF::DYN && M3_RESET16_CHAIN2) || RESET_TWO_STAGE<CF>) {
            r.defer = e->defer + o;
            r.defer_count = &cnt[CNT_PF_DEFER];  // zeroed with the block
        }
        prefetch_args<CF>(e, o, r);
        // the grid is sized for n / PF_DIV finished boards and grid-strides (M3_PF_DIV)
#ifndef M3_DEBUG_NO_PREFETCH  // timing experiment only: the next episodes are never built (not bit-exact)
        constexpr int64_t PF_DIV = CF::DYN ? 8 : (CF::N > 128 ? M3_PF_DIV16 : M3_PF_DIV);
        int rc = launch_init<CF>(sh.pstream, r, sh.n / PF_DIV + 1);
        if (rc) return rc;
#endif
        HIP_TRY(hipEventRecord(sh.pev[par], sh.pstream));
        sh.ppending[par] = true;
    }
    return M3_OK;
}

template <class CF>
int launch_env_step(m3_env* e, const int32_t* d_actions) {
    for (int s = 0; s < (int)e->shards.size(); ++s) {
        int rc = launch_env_shard<CF>(e, s, d_actions);
        if (rc) return rc;
    }
    e->upload_this = false;
    e->gpend[e->steps & 1] = false;
    e->cur ^= 1;
    e->steps++;
    return M3_OK;
}

// Episode slots cur + 1 .. cur + NSLOT - 1 of every board from its current
// seed (explicit reset, or autoreset switched on later).
template <class CF>
int fill_next_slots(m3_env* e) {
    m3_ctx* c = e->ctx;
    for (uint32_t k = 1; k < (uint32_t)NSLOT; ++k) {
        InitArgs r{};
        r.n = e->n;
        r.seeds = e->seeds;
        r.seed_add = k * e->stride;
        r.slot0 = k;
        r.slot_of = e->slot;
        prefetch_args<CF>(e, 0, r);
        int rc = launch_init<CF>(c->stream, r, e->n);
        if (rc) return rc;
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    return M3_OK;
}

// After m3_env_set: rebuild what the env derives from the loaded fields --
// every board back in episode slot 0, the chain word mt[397] of its seed, the
// legal set of its board, the queued next episodes -- and restart the step
// counter, exactly the state m3_env_reset leaves behind for those fields.
template <class CF>
int rederive(m3_env* e) {
    m3_ctx* c = e->ctx;
    HIP_TRY(hipMemsetAsync(e->counters, 0, 64 * 4 * MAX_SHARDS, c->stream));
    HIP_TRY(hipMemsetAsync(e->slot, 0, e->n, c->stream));
    const int64_t g = std::min<int64_t>((e->n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_mt397, dim3((unsigned)g), dim3(256), 0, c->stream, e->n, e->seeds, e->m397);
    HIP_TRY(hipGetLastError());
    int rc = launch_legal<CF>(c, e->n, e->boards[e->cur], e->legal);
    if (rc) return rc;
    e->steps = 0;
    e->gpend[0] = e->gpend[1] = false;
    if (e->autoreset) {
        rc = fill_next_slots<CF>(e);
        if (rc) return rc;
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    e->stale = false;
    return M3_OK;
}

// MCTS rollouts (k_rollout + its exact replay pass) of one launch
template <class CF>
int launch_rollouts(m3_ctx* c, const RolloutArgs& a) {
    hipLaunchKernelGGL(k_rollout<CF>, dim3(grid_for<CF>(a.n)), dim3(KS<CF>::B), 0, c->stream, a);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_rollout_fix<CF>, dim3(fix_grid<CF>()), dim3(FIX_BLOCK), 0, c->stream, a);
    HIP_TRY(hipGetLastError());
    return M3_OK;
}

// explicit instantiation (m3_inst.hip: M3_INSTANTIATE(template, CF)) or declaration
// (m3_api.hip: M3_INSTANTIATE(extern template, CF)) of one configuration's launchers
#define M3_INSTANTIATE(KW, CF)                                                     \
    KW int launch_apply<CF>(m3_ctx*, const ApplyArgs&);                            \
    KW int launch_init<CF>(hipStream_t, const InitArgs&, int64_t);                 \
    KW int launch_legal<CF>(m3_ctx*, int64_t, const int8_t*, uint32_t*);           \
    KW int launch_env_step<CF>(m3_env*, const int32_t*);                           \
    KW int fill_next_slots<CF>(m3_env*);                                           \
    KW int rederive<CF>(m3_env*);                                                  \
    KW int launch_rollouts<CF>(m3_ctx*, const RolloutArgs&);

}  // namespace m3k
