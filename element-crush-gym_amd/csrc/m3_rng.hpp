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
#ifndef __HIP_DEVICE_COMPILE__
        // b_* / c_* are only read after slow() set them (draws 227 / 454), but a paused step copies
        // the whole struct into its Cont record (m3_rules.hpp); the host build defines them so
        // MemorySanitizer sees no copy of an unset word (tests/hostcore msan). The device code
        // leaves them unset: zeroing would hold 4 more VGPRs from the first draw on.
        b_lo = b_hi = c_lo = c_hi = 0u;
#endif
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

// --------------------------------------------------------------------------
// ChainMT2: the first TWO MT19937 blocks (raw outputs k < 1248) from registers.
// Resets of 16x16x8 boards draw 256 tiles a round and most need 3-4 rounds
// (768-1024 draws), past the first block that ChainMT covers.
//
// The second twist is mt''[m] = Y ^ twist(mt'[m], mt'[m+1]) with Y =
// mt'[m+397] (m < 227) or mt''[m-227] (m >= 227), and mt''[623] uses mt''[0]
// in place of mt'[624]. Every mt' value is again a chain walk (MtpChain, the
// level structure of ChainMT), so block 2 runs the recursion
//     L1(m)  = Y1 ^ twist(A1 at m, A1 at m+1),  Y1 = B at 397+m  | L2(m-227)
//     L2(m') = Y2 ^ twist(A2 at m', ...),        Y2 = B at 397+m' | L3(m'-227)
//     L3(m") = B at 397+m" ^ twist(A3 at m", ...)
// with three "A" walks over mt'[0..] (started as block 2, L2 and L3 begin)
// and ONE "B" walk over mt'[397..623], restarted at each level change (its
// previous use ends exactly there). B starts mid-sequence, so it needs the
// init_genrand words s[170] and s[567] besides s[397] (computed once, when a
// reset first reaches block 2). ~27 registers, no memory; draw 1248 raises
// `overflow` (the caller hands the board to the wave-cooperative reset).
// --------------------------------------------------------------------------
// mt'[i] for consecutive i, over index range [.., LV * 227) (LV = chain levels)
template <int LV>
struct MtpChain {
    uint32_t a_lo, a_hi, b_lo, b_hi, c_lo, c_hi;  // fields of unused levels are never touched
    M3_HD void start0(uint32_t seed, uint32_t s397) {
        a_lo = seed;
        a_hi = s397;
    }
    M3_HD void start397(uint32_t s397, uint32_t s170, uint32_t s567) {  // position at i = 397 (LV 3)
        a_lo = s397;
        b_lo = s170;
        b_hi = s567;
    }
    // returns mt'[i] and advances to i + 1 (i < 624; i == 623 wraps to mt'[0] as ChainMT)
    M3_HD uint32_t step(uint32_t i, uint32_t seed, uint32_t s397) {
        if (LV == 1 || i < 227u) {
            const uint32_t lo1 = mt_init_next(a_lo, i + 1u);
            const uint32_t v = a_hi ^ mt_twist(a_lo, lo1);
            a_hi = mt_init_next(a_hi, i + 398u);
            a_lo = lo1;
            return v;
        }
        uint32_t lo1a;
        if (LV >= 3 && i == 623u) lo1a = s397 ^ mt_twist(seed, mt_init_next(seed, 1u));
        else lo1a = mt_init_next(a_lo, i + 1u);
        const uint32_t twa = mt_twist(a_lo, lo1a);
        a_lo = lo1a;
        const uint32_t j = i - 227u;
        if (j == 0u) {
            b_lo = seed;
            b_hi = s397;
        }
        const uint32_t lo1b = mt_init_next(b_lo, j + 1u);
        const uint32_t twb = mt_twist(b_lo, lo1b);
        b_lo = lo1b;
        uint32_t vb;
        if (LV == 2 || j < 227u) {
            vb = b_hi ^ twb;
            b_hi = mt_init_next(b_hi, j + 398u);
        } else {
            const uint32_t jj = j - 227u;
            if (jj == 0u) {
                c_lo = seed;
                c_hi = s397;
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

struct ChainMT2 {
    static constexpr bool DRAW_BOUNDED = true;  // overflow after 1248 draws
    static constexpr uint32_t LIMIT = 1248u;
    uint32_t seed, mt397, s170, s567;
    uint32_t k;
    uint32_t overflow;
    MtpChain<3> A1, B;
    MtpChain<2> A2;
    MtpChain<1> A3;
    uint32_t p1, p2, p3, q0;  // previous A1 / A2 / A3 value; mt''[0]

    M3_HD void init(uint32_t s, uint32_t s397) {
        seed = s;
        mt397 = s397;
        overflow = 0u;
        reseed();
    }
    M3_HD void reseed() {
        k = 0u;
        A1.start0(seed, mt397);
    }
    M3_HD uint32_t draws() const { return k; }
    M3_HD uint32_t next32() {
        const uint32_t i = k;
        uint32_t v;
        if (i < 624u) {
            v = A1.step(i, seed, mt397);
        } else if (i < LIMIT) {
            v = block2(i - 624u);
        } else {
            overflow = 1u;
            v = 0u;
        }
        k = i + 1u;
        return mt_temper(v);
    }

  private:
    M3_HD uint32_t lvl3(uint32_t m) {  // mt''[m], m < 170 (inside L2)
        if (m == 0u) {
            A3.start0(seed, mt397);
            p3 = A3.step(0u, seed, mt397);
            B.start397(mt397, s170, s567);
        }
        const uint32_t c = A3.step(m + 1u, seed, mt397);
        const uint32_t v = B.step(397u + m, seed, mt397) ^ mt_twist(p3, c);
        p3 = c;
        return v;
    }
    M3_HD uint32_t lvl2(uint32_t m) {  // mt''[m], m < 397 (inside L1)
        if (m == 0u) {
            A2.start0(seed, mt397);
            p2 = A2.step(0u, seed, mt397);
            B.start397(mt397, s170, s567);
        }
        const uint32_t c = A2.step(m + 1u, seed, mt397);
        const uint32_t y = m < 227u ? B.step(397u + m, seed, mt397) : lvl3(m - 227u);
        const uint32_t v = y ^ mt_twist(p2, c);
        p2 = c;
        return v;
    }
    M3_HD uint32_t block2(uint32_t m) {  // mt''[m], m < 624
        if (m == 0u) {
            uint32_t x = seed;
            for (uint32_t i = 1; i <= 170u; ++i) x = mt_init_next(x, i);
            s170 = x;
            x = mt397;
            for (uint32_t i = 398; i <= 567u; ++i) x = mt_init_next(x, i);
            s567 = x;
            A1.start0(seed, mt397);
            p1 = A1.step(0u, seed, mt397);
            B.start397(mt397, s170, s567);
        }
        const uint32_t c = m < 623u ? A1.step(m + 1u, seed, mt397) : q0;
        const uint32_t y = m < 227u ? B.step(397u + m, seed, mt397) : lvl2(m - 227u);
        const uint32_t v = y ^ mt_twist(p1, c);
        p1 = c;
        if (m == 0u) q0 = v;
        return v;
    }
};

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
