// m3_bitboard.hpp -- multi-word bitboards for one R x C board per lane.
//
// A board of N = R*C cells is one bit per cell, row-major (bit x = r*C + c),
// stored in W = ceil(N/32) 32-bit words that live in VGPRs. All shifts are by
// compile-time amounts, so each one lowers to W v_alignbit_b32 (funnel
// shifts); every index into `w[]` is compile-time, so nothing spills to
// scratch. Dynamic (per-lane) cell positions only appear in bit_at()/test()/
// range_mask(), which lower to W v_cndmask selects.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define M3_HD __host__ __device__ __forceinline__

namespace m3 {

template <int W>
struct BB {
    uint32_t w[W];

    static constexpr M3_HD BB zero() {
        BB b{};
        for (int i = 0; i < W; ++i) b.w[i] = 0u;
        return b;
    }
    M3_HD BB operator&(const BB& o) const { BB r; _Pragma("unroll") for (int i = 0; i < W; ++i) r.w[i] = w[i] & o.w[i]; return r; }
    M3_HD BB operator|(const BB& o) const { BB r; _Pragma("unroll") for (int i = 0; i < W; ++i) r.w[i] = w[i] | o.w[i]; return r; }
    M3_HD BB operator^(const BB& o) const { BB r; _Pragma("unroll") for (int i = 0; i < W; ++i) r.w[i] = w[i] ^ o.w[i]; return r; }
    M3_HD BB operator~() const { BB r; _Pragma("unroll") for (int i = 0; i < W; ++i) r.w[i] = ~w[i]; return r; }
    M3_HD BB& operator&=(const BB& o) { _Pragma("unroll") for (int i = 0; i < W; ++i) w[i] &= o.w[i]; return *this; }
    M3_HD BB& operator|=(const BB& o) { _Pragma("unroll") for (int i = 0; i < W; ++i) w[i] |= o.w[i]; return *this; }
    M3_HD BB& operator^=(const BB& o) { _Pragma("unroll") for (int i = 0; i < W; ++i) w[i] ^= o.w[i]; return *this; }
    // a & ~b in one op per word (v_bfi / s_andn2 friendly)
    M3_HD BB andnot(const BB& o) const { BB r; _Pragma("unroll") for (int i = 0; i < W; ++i) r.w[i] = w[i] & ~o.w[i]; return r; }

    M3_HD bool any() const {
        uint32_t a = 0;
        _Pragma("unroll") for (int i = 0; i < W; ++i) a |= w[i];
        return a != 0u;
    }
    M3_HD int popc() const {
        int n = 0;
        _Pragma("unroll") for (int i = 0; i < W; ++i) n += __builtin_popcount(w[i]);
        return n;
    }
    // index of the lowest set bit; caller guarantees any()
    M3_HD int lowest() const {
        int idx = 0;
        bool found = false;
        _Pragma("unroll") for (int i = 0; i < W; ++i) {
            if (!found && w[i] != 0u) { idx = i * 32 + __builtin_ctz(w[i]); found = true; }
        }
        return idx;
    }
    // one-hot board with cell x set (x dynamic)
    static M3_HD BB bit_at(int x) {
        BB r;
        const uint32_t b = 1u << (x & 31);
        const int q = x >> 5;
        _Pragma("unroll") for (int i = 0; i < W; ++i) r.w[i] = (q == i) ? b : 0u;
        return r;
    }
    // Dynamic word select written as masks, not a select chain: LLVM turns a
    // select chain over several boards into a stack array + indexed scratch
    // load, which costs a memory round trip on the GPU.
    M3_HD uint32_t word_at(int q) const {
        uint32_t v = 0u;
        _Pragma("unroll") for (int i = 0; i < W; ++i) v |= w[i] & (0u - (uint32_t)(q == i));
        return v;
    }
    M3_HD uint32_t test(int x) const { return (word_at(x >> 5) >> (x & 31)) & 1u; }
    // clear the lowest set bit (caller guarantees any())
    M3_HD void pop_lowest() {
        bool done = false;
        _Pragma("unroll") for (int i = 0; i < W; ++i) {
            if (!done && w[i] != 0u) { w[i] &= w[i] - 1u; done = true; }
        }
    }
};

// the low n bits (0 <= n <= 32; a plain (1u << 32) - 1 would be 0 on the GPU)
M3_HD constexpr uint32_t low_bits(int n) { return n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u); }

M3_HD int select_bit(uint32_t u, int k) {  // position of the k-th (0-based) set bit of u
    int pos = 0;
#pragma unroll
    for (int half = 16; half >= 1; half >>= 1) {
        const uint32_t lo = u & ((1u << half) - 1u);
        const int c = __builtin_popcount(lo);
        if (k >= c) {
            k -= c;
            u >>= half;
            pos += half;
        } else {
            u = lo;
        }
    }
    return pos;
}

// out[y] = a[y + D]   (D > 0 looks "ahead" to higher cells, D < 0 looks back)
template <int D, int W>
M3_HD BB<W> at(const BB<W>& a) {
    BB<W> r;
    if constexpr (D == 0) {
        return a;
    } else if constexpr (D > 0) {
        constexpr int q = D / 32, s = D % 32;
        _Pragma("unroll") for (int i = 0; i < W; ++i) {
            const uint32_t lo = (i + q < W) ? a.w[i + q] : 0u;
            const uint32_t hi = (i + q + 1 < W) ? a.w[i + q + 1] : 0u;
            r.w[i] = s == 0 ? lo : ((lo >> s) | (hi << ((32 - s) & 31)));
        }
    } else {
        constexpr int E = -D;
        constexpr int q = E / 32, s = E % 32;
        _Pragma("unroll") for (int i = 0; i < W; ++i) {
            const uint32_t hi = (i - q >= 0) ? a.w[i - q] : 0u;
            const uint32_t lo = (i - q - 1 >= 0) ? a.w[i - q - 1] : 0u;
            r.w[i] = s == 0 ? hi : ((hi << s) | (lo >> ((32 - s) & 31)));
        }
    }
    return r;
}

// bits [a, b) set (a, b dynamic, 0 <= a, b <= 32*W)
template <int W>
M3_HD BB<W> range_mask(int a, int b) {
    BB<W> r;
    _Pragma("unroll") for (int i = 0; i < W; ++i) {
        int lo = a - 32 * i, hi = b - 32 * i;
        lo = lo < 0 ? 0 : (lo > 32 ? 32 : lo);
        hi = hi < 0 ? 0 : (hi > 32 ? 32 : hi);
        const uint32_t mhi = hi >= 32 ? 0xFFFFFFFFu : ((1u << hi) - 1u);
        const uint32_t mlo = lo >= 32 ? 0xFFFFFFFFu : ((1u << lo) - 1u);
        r.w[i] = hi > lo ? (mhi & ~mlo) : 0u;
    }
    return r;
}

// Compile-time cell masks for an R x C board.
template <int R, int C, int W>
struct Geo {
    static constexpr int N = R * C;

    template <class Pred>
    static constexpr BB<W> build(Pred pred) {
        BB<W> b = BB<W>::zero();
        for (int x = 0; x < N; ++x)
            if (pred(x / C, x % C)) b.w[x >> 5] |= (1u << (x & 31));
        return b;
    }
    static constexpr BB<W> valid() { return build([](int, int) { return true; }); }
    static constexpr BB<W> col_ge(int k) { return build([k](int, int c) { return c >= k; }); }
    static constexpr BB<W> col_le(int k) { return build([k](int, int c) { return c <= k; }); }
    static constexpr BB<W> row_ge(int k) { return build([k](int r, int) { return r >= k; }); }
    static constexpr BB<W> row_le(int k) { return build([k](int r, int) { return r <= k; }); }
    static constexpr BB<W> col_eq(int k) { return build([k](int, int c) { return c == k; }); }

    // Column band [c0, c1) for dynamic c0 <= c1 <= C: replicate the C-bit row
    // pattern into every row. Rows starting inside word i are placed with one
    // carry-free multiply; the row that straddles into word i from below is
    // one shift.
    static constexpr uint32_t rep_mul(int i) {
        uint32_t m = 0;
        for (int r = 0; r < R; ++r) {
            const int off = r * C - 32 * i;
            if (off >= 0 && off < 32) m |= 1u << off;
        }
        return m;
    }
    static constexpr int straddle_shift(int i) {  // 0 = none
        for (int r = 0; r < R; ++r) {
            const int s = r * C, e = r * C + C;
            if (s < 32 * i && e > 32 * i) return 32 * i - s;
        }
        return 0;
    }
    static M3_HD BB<W> col_band(int c0, int c1) {
        const uint32_t pat = (c1 > c0) ? (low_bits(c1) & ~low_bits(c0)) : 0u;
        BB<W> r;
        _Pragma("unroll") for (int i = 0; i < W; ++i) {
            uint32_t v = pat * rep_mul(i);
            const int sh = straddle_shift(i);
            if (sh) v |= pat >> sh;
            r.w[i] = v;
        }
        constexpr BB<W> V = valid();
        return r & V;
    }
    static M3_HD BB<W> row_band(int r0, int r1) { return range_mask<W>(r0 * C, r1 * C); }
};

}  // namespace m3
