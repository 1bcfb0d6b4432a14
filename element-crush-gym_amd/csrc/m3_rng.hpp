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
    static constexpr bool DRAW_BOUNDED = true;  // overflow after LIMIT draws (bounds the cascade)
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
