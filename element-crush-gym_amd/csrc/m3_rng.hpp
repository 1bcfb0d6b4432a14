// m3_rng.hpp -- numpy legacy RandomState (MT19937) streams, one per lane.
//
// The reference reseeds numpy's global MT19937 with the board's fixed seed at
// the start of every step (match3tile/boardv2.py:46) and on every dead-board
// shuffle (match3tile/boardFunctions.py:17), so a step only ever reads the
// first few dozen outputs of the stream seed(s). MT19937's first block of 624
// outputs is
//     out[k] = temper(mt'[k]),  mt'[k] = X[k] ^ twist(mt[k], mt[k+1])
// with X[k] = mt[k+397] for k < 227 and X[k] = mt'[k-227] afterwards, where
// mt[] is the init_genrand sequence mt[i] = 1812433253*(mt[i-1]^(mt[i-1]>>30))+i.
//
// ChainMT walks that definition directly: one "chain" keeps (mt[i], mt[i+397])
// and advances both by one init_genrand step per draw, so a draw costs two
// integer multiplies and no memory at all. Draw k >= 227 needs mt'[k-227],
// provided by a second chain started at 0 (and a third for k >= 454). The
// only per-board state is seed and mt[397] (computed once at reset). Draws
// k >= 624 (a second twist) are beyond ChainMT and raise `overflow`; the caller
// recomputes such a step with FullMT.
//
// FullMT is the textbook 624-word state (numpy mt19937_seed/mt19937_gen) kept
// in lane-private memory; it serves reset (BoardV2.__init__ draws up to ~1300
// values, boardv2.py:20-27) and the rare overflowing step.
#pragma once

#include <type_traits>

#include "m3_bitboard.hpp"

namespace m3 {

constexpr uint32_t MT_MATRIX_A = 0x9908b0dfu;
constexpr uint32_t MT_UPPER = 0x80000000u;
constexpr uint32_t MT_LOWER = 0x7fffffffu;

M3_HD uint32_t mt_init_next(uint32_t x, uint32_t i) { return 1812433253u * (x ^ (x >> 30)) + i; }
M3_HD uint32_t mt_twist(uint32_t lo, uint32_t lo1) {
    const uint32_t y = (lo & MT_UPPER) | (lo1 & MT_LOWER);
    return (y >> 1) ^ ((0u - (y & 1u)) & MT_MATRIX_A);
}
M3_HD uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}
// mt[397] of init_genrand(seed): the only cached per-board RNG state.
M3_HD uint32_t mt_state397(uint32_t seed) {
    uint32_t x = seed;
    for (uint32_t i = 1; i <= 397; ++i) x = mt_init_next(x, i);
    return x;
}

// LIMIT = 624: three chain levels, every draw of the first MT block.
// LIMIT = 227: one level; draw 227 raises `overflow` (the step kernels use
// this: a step needs > 226 draws essentially never, and one level keeps five
// fewer VGPRs live through the cascade).
template <uint32_t LIMIT>
struct ChainMTT {
    static_assert(LIMIT == 227u || LIMIT == 624u, "chain depth");
    uint32_t seed, mt397;
    uint32_t k;           // raw outputs since the last reseed
    uint32_t a_lo, a_hi;  // mt[k], mt[k+397]
    uint32_t b_lo, b_hi;  // chain at k-227
    uint32_t c_lo, c_hi;  // chain at k-454
    uint32_t overflow;

    M3_HD void init(uint32_t s, uint32_t s397) {
        seed = s;
        mt397 = s397;
        overflow = 0;
        reseed();
    }
    M3_HD void reseed() {
        k = 0;
        a_lo = seed;
        a_hi = mt397;
    }
    M3_HD uint32_t next32() {
        const uint32_t i = k;
        uint32_t v;
        if (i < 227u) {
            const uint32_t lo1 = mt_init_next(a_lo, i + 1u);
            v = a_hi ^ mt_twist(a_lo, lo1);
            a_hi = mt_init_next(a_hi, i + 398u);
            a_lo = lo1;
        } else {
            v = slow(i);
        }
        k = i + 1u;
        return mt_temper(v);
    }
    M3_HD uint32_t draws() const { return k; }

  private:
    M3_HD uint32_t slow(uint32_t i) {
        if (i >= LIMIT) {
            overflow = 1u;
            return 0u;
        }
        // level 0 at index i (i >= 227): X = mt'[i-227]
        uint32_t lo1a;
        if (i == 623u) {  // mt[624] wraps to the already-twisted mt'[0]
            lo1a = mt397 ^ mt_twist(seed, mt_init_next(seed, 1u));
        } else {
            lo1a = mt_init_next(a_lo, i + 1u);
        }
        const uint32_t twa = mt_twist(a_lo, lo1a);
        a_lo = lo1a;
        // level 1 at j = i-227 gives mt'[j]
        const uint32_t j = i - 227u;
        if (j == 0u) {
            b_lo = seed;
            b_hi = mt397;
        }
        const uint32_t lo1b = mt_init_next(b_lo, j + 1u);
        const uint32_t twb = mt_twist(b_lo, lo1b);
        b_lo = lo1b;
        uint32_t vb;
        if (j < 227u) {
            vb = b_hi ^ twb;
            b_hi = mt_init_next(b_hi, j + 398u);
        } else {  // level 2 at jj = i-454 gives mt'[jj]
            const uint32_t jj = j - 227u;
            if (jj == 0u) {
                c_lo = seed;
                c_hi = mt397;
            }
            const uint32_t lo1c = mt_init_next(c_lo, jj + 1u);
            const uint32_t vc = c_hi ^ mt_twist(c_lo, lo1c);
            c_hi = mt_init_next(c_hi, jj + 398u);
            c_lo = lo1c;
            vb = vc ^ twb;
        }
        return vb ^ twa;
    }
};
using ChainMT = ChainMTT<624u>;
using ChainMT1 = ChainMTT<227u>;

// Textbook MT19937 (numpy mt19937_seed / mt19937_gen / mt19937_next32).
// Key is the state's storage: KeyArray = lane-private scratch (an LDS column
// per lane, one wave per CU, measured slower in k_init_fix_lane). The twist
// carries key[i+1] to the next index and is unrolled so a batch of state
// loads is in flight at once; bulk_* hand out a run of outputs the same way.
struct KeyArray {
    uint32_t w[624];
    M3_HD uint32_t& operator[](uint32_t p) { return w[p]; }
    M3_HD uint32_t operator[](uint32_t p) const { return w[p]; }
};

template <class Key>
struct MT19937 {
    Key key;
    uint32_t pos;
    uint32_t k;  // raw outputs since the last reseed
    uint32_t seed;
    uint32_t overflow;

    M3_HD void init(uint32_t s, uint32_t /*s397*/) {
        seed = s;
        overflow = 0;
        reseed();
    }
    M3_HD void reseed() {
        uint32_t x = seed;
        for (uint32_t p = 0; p < 624u; ++p) {
            key[p] = x;
            x = mt_init_next(x, p + 1u);
        }
        pos = 624u;
        k = 0u;
    }
    M3_HD void gen() {
        uint32_t i = 0, cur = key[0];
#pragma unroll 8
        for (; i < 624u - 397u; ++i) {
            const uint32_t nx = key[i + 1u];
            key[i] = key[i + 397u] ^ mt_twist(cur, nx);
            cur = nx;
        }
#pragma unroll 8
        for (; i < 623u; ++i) {
            const uint32_t nx = key[i + 1u];
            key[i] = key[i - 227u] ^ mt_twist(cur, nx);
            cur = nx;
        }
        key[623] = key[396] ^ mt_twist(cur, key[0]);
        pos = 0u;
    }
    M3_HD uint32_t next32() {
        if (pos == 624u) gen();
        const uint32_t y = key[pos];
        pos += 1u;
        k += 1u;
        return mt_temper(y);
    }
    // n consecutive outputs without a twist between them: out(j) = temper(key[pos + j]).
    M3_HD bool bulk_ready(uint32_t n) {
        if (pos == 624u) gen();
        return pos + n <= 624u;
    }
    M3_HD uint32_t bulk_out(uint32_t j) { return mt_temper(key[pos + j]); }
    M3_HD void bulk_skip(uint32_t n) {
        pos += n;
        k += n;
    }
    M3_HD uint32_t draws() const { return k; }
};
using FullMT = MT19937<KeyArray>;

// --------------------------------------------------------------------------
// Per-board stream cache (batched env). Because the reference reseeds with the
// board's fixed seed at every step, every step of an episode reads the SAME
// stream, so reset stores it once (k_init):
//   raw[k]   low bits of raw output k, k < RAWN (RawT is wide enough for every
//            mask a step applies: 2^BITS-1 for tiles, the shuffle's <= 15 and
//            the random action's < 2^ceil(log2 A));
//   ts[p][w] tile stream as bit-planes: tile j = (j-th accepted masked draw)+1
//            = randint(1, T+1) value j, bit p of tile j at bit j of plane p;
//   acc[w]   acceptance bitmap of the raw draws (bit k: raw k became a tile).
// A step then never runs MT19937: the refill deposits whole columns of tiles
// (m3_rules.hpp, refill_tiles), and the few raw draws of a shuffle or of the
// next random action are byte loads. Position bookkeeping: in tile mode the
// raw position after tile j-1 is max(kb, position of the (j-1)-th accepted
// draw + 1); in raw mode it is k. Anything beyond the cache raises `overflow`
// and the step is recomputed exactly (FullMT).
template <class RawT, int RAWN, int BITS, int TSW, int ACCW>
struct CachedRNG {
    static constexpr bool TILES = true;
    static constexpr int TCAP = TSW * 32;
    static constexpr uint32_t WE = 16u / sizeof(RawT);  // raw entries per 16-byte window
    const RawT* raw;       // this board's RAWN-entry row (16-byte aligned)
    const uint32_t* ts;    // plane p, word w at ts[(p * (TSW + 1) + w) * stride] (word TSW is a zero pad)
    const uint32_t* acc;   // word w at acc[w * stride]
    int stride;
    uint32_t cap;          // tiles available: min(TCAP, accepted draws below RAWN)
    uint32_t kb, j, k, in_tiles, overflow;
    uint32_t win[4], wlo;  // raw entries [wlo, wlo + WE), one 16-byte load

    M3_HD void load_window(uint32_t at) {
        wlo = at & ~(WE - 1u);
        const uint32_t* src = reinterpret_cast<const uint32_t*>(raw + wlo);
#pragma unroll
        for (int i = 0; i < 4; ++i) win[i] = src[i];
    }
    M3_HD void init(const RawT* r, const uint32_t* t, const uint32_t* a, int st) {
        raw = r;
        ts = t;
        acc = a;
        stride = st;
        load_window(0u);  // issued early: the random action usually reads the first few entries
        uint32_t n = 0;
#pragma unroll
        for (int w = 0; w < ACCW; ++w) n += (uint32_t)__builtin_popcount(acc[w * stride]);
        cap = n < (uint32_t)TCAP ? n : (uint32_t)TCAP;
        overflow = 0u;
        reseed();
    }
    M3_HD void reseed() {
        kb = 0u;
        j = 0u;
        k = 0u;
        in_tiles = 1u;
    }
    // raw position of the draw after the (jj-1)-th accepted one (jj >= 1)
    M3_HD uint32_t after_tile(uint32_t jj) const {
        uint32_t r = jj - 1u, word = 0u, wi = (uint32_t)ACCW;
        bool found = false;
#pragma unroll
        for (int w = 0; w < ACCW; ++w) {
            const uint32_t a = acc[w * stride];
            const uint32_t c = (uint32_t)__builtin_popcount(a);
            const bool here = !found && r < c;
            word = here ? a : word;
            wi = here ? (uint32_t)w : wi;
            r = (found || here) ? r : r - c;
            found = found || here;
        }
        if (!found) return (uint32_t)RAWN + 1u;
        return 32u * wi + (uint32_t)select_bit(word, (int)r) + 1u;
    }
    M3_HD uint32_t draws() const {
        if (!in_tiles) return k;
        if (j == 0u) return kb;
        const uint32_t p = after_tile(j);
        return p > kb ? p : kb;
    }
    M3_HD uint32_t next32() {
        if (in_tiles) {
            k = draws();
            in_tiles = 0u;
        }
        if (k >= (uint32_t)RAWN) {
            overflow = 1u;
            return 0u;
        }
        if (k - wlo >= WE) load_window(k);
        const uint32_t e = k - wlo;
        k += 1u;
        constexpr uint32_t PER = 4u / sizeof(RawT), SH = 8u * sizeof(RawT);
        const uint32_t q = e / PER;
        uint32_t wv = 0u;
#pragma unroll
        for (int i = 0; i < 4; ++i) wv |= win[i] & (0u - (uint32_t)(q == (uint32_t)i));
        return (wv >> (SH * (e % PER))) & ((1u << SH) - 1u);
    }
    // switch to tile mode at the current raw position
    M3_HD void begin_tiles() {
        if (in_tiles) return;
        kb = k;
        uint32_t n = 0;
#pragma unroll
        for (int w = 0; w < ACCW; ++w) {
            const int lo = 32 * w;
            const uint32_t a = acc[w * stride];
            uint32_t m = 0xFFFFFFFFu;
            if ((int)k < lo) m = 0u;
            else if ((int)k < lo + 32) m = (1u << (k - (uint32_t)lo)) - 1u;
            n += (uint32_t)__builtin_popcount(a & m);
        }
        j = n;
        in_tiles = 1u;
    }
    // 32 bits of tile plane p starting at tile jj (jj < TCAP)
    M3_HD uint32_t tile_bits(int p, uint32_t jj) const {
        const uint32_t q = jj >> 5, s = jj & 31u;
        const uint32_t lo = ts[(p * (TSW + 1) + (int)q) * stride];
        const uint32_t hi = ts[(p * (TSW + 1) + (int)q + 1) * stride];
        return s ? ((lo >> s) | (hi << (32u - s))) : lo;
    }
};

template <class G, class = void>
struct HasTiles {
    static constexpr bool value = false;
};
template <class G>
struct HasTiles<G, std::void_t<decltype(G::TILES)>> {
    static constexpr bool value = true;
};

// Fill a stream cache from seed s (RAWN raw outputs of seed(s)); used by reset.
// raw_out(k, v) receives every raw output; ts/acc words are returned through
// the callbacks so the caller chooses the memory layout.
template <int RAWN, int BITS, int TSW, int ACCW, uint32_t TILE_MASK, uint32_t TILE_RNG, class RawF, class TsF,
          class AccF>
M3_HD void build_stream_cache(uint32_t seed, uint32_t m397, RawF raw_out, TsF ts_out, AccF acc_out) {
    static_assert(TILE_RNG > 0u, "randint(1, 2) consumes no draws: no tile stream");
    static_assert(RAWN == 32 * ACCW && RAWN <= 624, "cache geometry");
    ChainMTT<624u> g;
    g.init(seed, m397);
    uint32_t tp[BITS];
#pragma unroll
    for (int p = 0; p < BITS; ++p) tp[p] = 0u;
    uint32_t accw = 0u, nt = 0u;
    for (int k = 0; k < RAWN; ++k) {
        const uint32_t v = g.next32();
        raw_out(k, v);
        const uint32_t t = v & TILE_MASK;
        if (t <= TILE_RNG) {
            accw |= 1u << (k & 31);
            if (nt < (uint32_t)(TSW * 32)) {
                const uint32_t val = t + 1u;
#pragma unroll
                for (int p = 0; p < BITS; ++p) tp[p] |= ((val >> p) & 1u) << (nt & 31u);
                ++nt;
                if ((nt & 31u) == 0u) {
#pragma unroll
                    for (int p = 0; p < BITS; ++p) {
                        ts_out(p, (int)(nt >> 5) - 1, tp[p]);
                        tp[p] = 0u;
                    }
                }
            }
        }
        if ((k & 31) == 31) {
            acc_out(k >> 5, accw);
            accw = 0u;
        }
    }
    if (nt < (uint32_t)(TSW * 32)) {
#pragma unroll
        for (int p = 0; p < BITS; ++p) ts_out(p, (int)(nt >> 5), tp[p]);
        for (int w = (int)(nt >> 5) + 1; w < TSW; ++w)
#pragma unroll
            for (int p = 0; p < BITS; ++p) ts_out(p, w, 0u);
    }
#pragma unroll
    for (int p = 0; p < BITS; ++p) ts_out(p, TSW, 0u);  // pad
}

// RandomState.randint(low, low+rng+1) for one element (legacy masked rejection):
// returns v in [0, rng]. rng == 0 consumes no draw (numpy's rng == 0 fast path).
template <class G>
M3_HD uint32_t rand_masked(G& g, uint32_t rng) {
    if (rng == 0u) return 0u;
    uint32_t mask = rng;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    uint32_t v;
    do {
        v = g.next32() & mask;
    } while (v > rng && !g.overflow);
    return v;
}

}  // namespace m3
