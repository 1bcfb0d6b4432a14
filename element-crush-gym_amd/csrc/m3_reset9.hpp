// m3_reset9.hpp -- the two-stage autoreset prefetch for tile counts that are not a power of two
// (9x9x6). Included by m3_kernels.hpp after k_reset_stream (it reuses wave_twist_u, init_item,
// init_outputs, init_store_board).
#pragma once

// ---- two-stage reset with rejection sampling (9x9x6 env prefetch) ----------
// randint(1, T+1) for a T that is not a power of two draws a raw output per
// tile and rejects (raw & TILE_MASK) > TILE_RNG (9x9x6: 6 and 7, a quarter):
// round k of BoardV2.__init__ (boardv2.py:21, :25) is accepted tiles
// [k*N, (k+1)*N) of the seed's stream, whatever the match masks turn out to
// be. k_reset_stream_rej: 4 resets per wave, as k_reset_stream, but the
// accepted tiles are compacted through LDS (ballot + mbcnt) and packed as raw
// bit planes over the tile index, with the raw position after each round (the
// draw count __init__ reports); k_reset_tiles_rej: one board per lane, the
// match-mask loop over the rounds (funnel shifts out of the tile planes).
// A reset needing more rounds than the table holds goes to k_init_coop.
#ifndef M3_RESET9_TWO_STAGE
#define M3_RESET9_TWO_STAGE 0
#endif
template <class CF, bool DYN = CF::DYN>
struct TwoStageRejOk : std::false_type {};
template <class CF>
struct TwoStageRejOk<CF, false>
    : std::bool_constant<M3_RESET9_TWO_STAGE && (CF::N <= 128) && CF::TILE_RNG != 0u &&
                         CF::TILE_RNG != CF::TILE_MASK> {};
template <class CF>
constexpr bool RESET_TWO_STAGE_REJ = TwoStageRejOk<CF>::value;
template <class CF>
struct TwoStageRej {
    static constexpr int RB = __builtin_popcount(CF::TILE_MASK);  // raw bits per tile
    static constexpr int DRAWS = 832;                             // raw outputs made per reset (13 groups)
    static constexpr int NX = DRAWS - 624;                        // words of the second block
    static constexpr int GROUPS = DRAWS / 64;
    static constexpr int TMAX = DRAWS;                            // accepted tiles at most
    static constexpr int TWORDS = (TMAX + 31) / 32 + 1;           // plane words (+1: funnel pad)
    static constexpr int ROUNDS = (TMAX / CF::N) < 8 ? (TMAX / CF::N) : 8;  // rounds whose draw count is kept
    // row: RB planes x TWORDS | raw position after rounds 1..ROUNDS | tiles made | mt[397]
    static constexpr int O_POS = RB * TWORDS, O_CNT = O_POS + ROUNDS, O_M397 = O_CNT + 1;
    static constexpr int TW = (O_M397 + 1 + 3) / 4 * 4;
    static constexpr int G = 4, U = 4;
    static constexpr int KST = 625;
    static constexpr int TST = TMAX + 64;  // LDS tile bytes per board (a whole group past the last)
    static_assert(NX <= 576 && DRAWS % 64 == 0, "second block head, whole groups");
};

template <class CF>
__global__ void __launch_bounds__(64) k_reset_stream_rej(InitArgs a) {
    using TS = TwoStageRej<CF>;
    constexpr int U = TS::U;
    __shared__ uint32_t key_s[TS::G * TS::KST];
    __shared__ uint8_t tile_s[U * TS::TST];
    __shared__ uint32_t pos_s[U * TS::ROUNDS];
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
            const uint32_t m397 = lane < nu ? key[lane * TS::KST + 397] : 0u;
            wave_sync();
            uint32_t nt[U];  // accepted tiles so far, per board (wave-uniform)
#pragma unroll
            for (int u = 0; u < U; ++u) nt[u] = 0u;
            // accept / compact the draws of group g into each board's LDS tile bytes
            auto take = [&](int g) {
                const int d = g * 64 + lane;
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t y = mt_temper(key[u * TS::KST + d % 624]) & CF::TILE_MASK;
                    const bool acc = y <= CF::TILE_RNG;
                    const uint64_t bal = __ballot(acc);
                    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
                    const uint32_t idx = nt[u] + rank;
                    if (acc) {
                        tile_s[u * TS::TST + idx] = (uint8_t)y;
                        // the draw that completes a round: __init__ has consumed d + 1 raw outputs
                        const uint32_t r = (idx + 1u) / (uint32_t)CF::N;
                        if ((idx + 1u) % (uint32_t)CF::N == 0u && r >= 1u && r <= (uint32_t)TS::ROUNDS)
                            pos_s[u * TS::ROUNDS + r - 1] = (uint32_t)d + 1u;
                    }
                    nt[u] += (uint32_t)__popcll(bal);
                }
            };
            wave_twist_u<U>(key, TS::KST, nu, lane);  // draws 0 .. 623
#pragma unroll 1
            for (int g = 0; g < 624 / 64; ++g) take(g);
            wave_sync();
            wave_twist_u<U, TS::NX>(key, TS::KST, nu, lane);  // draws 624 .. DRAWS - 1, over words [0, NX)
#pragma unroll 1
            for (int g = 624 / 64; g < TS::GROUPS; ++g) take(g);
            wave_sync();
            // the compacted tiles as raw-bit planes over the tile index
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (u >= nu) continue;
                uint32_t* row = a.tab + (base + j0 + u) * TS::TW;
#pragma unroll 1
                for (int c = 0; c < (TS::TWORDS + 1) / 2; ++c) {  // 64 tiles per trip
                    const uint32_t i = (uint32_t)(c * 64 + lane);
                    const uint32_t y = i < nt[u] ? tile_s[u * TS::TST + i] : 0u;
#pragma unroll
                    for (int q = 0; q < TS::RB; ++q) {
                        const uint64_t bal = __ballot((y >> q) & 1u);
                        const int w = 2 * c + (lane & 1);
                        if (lane < 2 && w < TS::TWORDS)
                            row[q * TS::TWORDS + w] = (lane & 1) ? (uint32_t)(bal >> 32) : (uint32_t)bal;
                    }
                }
                const uint32_t mu = __shfl(m397, u);  // (every lane: lane u holds board j0 + u's)
                if (lane < TS::ROUNDS) row[TS::O_POS + lane] = pos_s[u * TS::ROUNDS + lane];
                if (lane == 0) {
                    row[TS::O_CNT] = nt[u];
                    row[TS::O_M397] = mu;
                }
            }
            wave_sync();
        }
    }
}

// round k of a rejection table row into the planes (value = raw + 1, under `only`)
template <class CF>
__device__ __forceinline__ void tab_round_rej(typename CF::Bd* P, const uint32_t* t, int k,
                                              const typename CF::Bd* only) {
    using TS = TwoStageRej<CF>;
#pragma unroll
    for (int w = 0; w < CF::W; ++w) {
        const int o = k * CF::N + 32 * w;
        const int nbits = CF::N - 32 * w < 32 ? CF::N - 32 * w : 32;
        const uint32_t valid = nbits == 32 ? 0xFFFFFFFFu : (1u << nbits) - 1u;
        uint32_t c = 0xFFFFFFFFu;  // + 1: a ripple carry over the bit planes
        const uint32_t m = (only ? only->w[w] : 0xFFFFFFFFu) & valid;
#pragma unroll
        for (int p = 0; p < CF::BITS; ++p) {
            uint32_t r = 0u;
            if (p < TS::RB) {
                const uint32_t* pl = t + (p < TS::RB ? p : 0) * TS::TWORDS;
                r = __builtin_amdgcn_alignbit(pl[(o >> 5) + 1], pl[o >> 5], (uint32_t)(o & 31));
            }
            const uint32_t vb = r ^ c;
            c &= r;
            P[p].w[w] = (P[p].w[w] & ~m) | (vb & m);
        }
    }
}

template <class CF>
__global__ void __launch_bounds__(64) k_reset_tiles_rej(InitArgs a) {
    using TS = TwoStageRej<CF>;
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
            const uint32_t m397 = t[TS::O_M397];
            const uint32_t have = t[TS::O_CNT] / (uint32_t)CF::N;  // whole rounds in the row
            const int kmax = (int)(have < (uint32_t)TS::ROUNDS ? have : (uint32_t)TS::ROUNDS);
            typename CF::Bd P[CF::NP], mask;
#pragma unroll
            for (int p = 0; p < CF::NP; ++p) P[p] = CF::Bd::zero();
            int rounds = 0;
            if (kmax < 1) {
                ok = false;
            } else {
                tab_round_rej<CF>(P, t, 0, nullptr);                        // boardv2.py:21
                while (get_match_mask<CF>(P, mask)) {                       // :23-27
                    if (++rounds >= kmax) {
                        ok = false;
                        break;
                    }
                    tab_round_rej<CF>(P, t, rounds, &mask);
                }
            }
            if (ok) {
                if (a.m397) a.m397[(int64_t)slot * a.cstride + b] = m397;
                const int64_t ob = (int64_t)slot * a.sstride + b;
                const uint32_t draws = t[TS::O_POS + rounds];
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
