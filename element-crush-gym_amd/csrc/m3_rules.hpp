// m3_rules.hpp -- the env step of ThorLL/Element-Crush-Gym as bitboard code.
//
// One board per lane. A board is NP=7 bit-planes (cell values are int8 in
// [0, 127]; plane p holds bit p of every cell), each plane a W-word bitboard
// in registers. Everything the reference does cell-by-cell in Python/numpy is
// restated as whole-board word operations:
//   * TB = board & TM is planes [0, BITS); "TB == TB[x+d]" for every cell is
//     one XOR/OR pass over BITS planes (eq<d>);
//   * legal_actions (boardFunctions.py:26-112) is ~25 such comparisons;
//   * get_matches (boardFunctions.py:121-156) is a sequential scan whose
//     result depends on scan order; it is reproduced exactly by visiting only
//     the run starts (cells that begin a horizontal or vertical triple) in
//     ascending bit order and flood-filling runs with doubling shifts;
//   * gravity (boardv2.py:166-173) is a few whole-board "drop everything
//     above a hole by one row" passes;
//   * scoring / merge / clip (boardv2.py:157-163) are popcounts and masks.
// Cross-references to the reference are file:line in each function.
#pragma once

#include <type_traits>

#include "m3_bitboard.hpp"
#include "m3_rng.hpp"

namespace m3 {

// Phase-profiling hooks. A Store type that defines PROF receives mark<K>() at
// phase boundaries (m3_api.hip builds such a variant with -DM3_PHASE_PROF);
// for every other Store the calls compile to nothing.
enum : int { PH_LOAD, PH_SWAP, PH_MATCH, PH_CLEAR, PH_DROP, PH_REFILL, PH_LEGAL, PH_NEXT, PH_RESET, PH_QUEUE,
             PH_STORE, PH_TBYTES, PH_TLOAD, PH_TATOM, PH_N };
template <class S, class = void>
struct HasProf : std::false_type {};
template <class S>
struct HasProf<S, std::void_t<decltype(S::PROF)>> : std::true_type {};
template <int K, class S>
M3_HD void mark(S& st) {
    if constexpr (HasProf<S>::value) st.template mark<K>();
}

constexpr int ceil_log2(int v) {
    int b = 0;
    while ((1 << b) < v) ++b;
    return b;
}

// Flags, mirrored in include/m3.h.
enum : uint32_t {
    FLAG_TERMINAL = 0x01u,     // n_actions < 1: board returned unchanged (boardv2.py:44-45)
    FLAG_BAD_ACTION = 0x02u,   // action id outside [0, A) (KeyError at boardv2.py:48)
    FLAG_SHUFFLE_CAP = 0x04u,  // dead-board shuffle did not terminate within the cap (reference hangs)
    FLAG_NO_LEGAL = 0x08u,     // no legal action to sample (np.random.choice([]) raises)
    FLAG_SHUFFLED = 0x10u,     // the dead-board shuffle ran at least once
    FLAG_RNG_OVERFLOW = 0x20u, // internal: step needed >= 624 draws; recomputed with FullMT
    FLAG_GROUP_OVERFLOW = 0x40u, // internal: more match groups than the fast table holds; recomputed
    FLAG_RECOMPUTE = FLAG_RNG_OVERFLOW | FLAG_GROUP_OVERFLOW,
    FLAG_CASCADE_CAP = 0x100u, // cascade stopped after CASCADE_CAP refills (reference: unbounded)
    FLAG_RESET_CAP = 0x200u,   // reset stopped after RESET_ROUND_CAP redraw rounds (reference: unbounded)
};
// Refill-and-rematch passes one step may run. The reference loops until a
// refill leaves no match (boardv2.py:138-202); with two tile types on a board
// of about 7x7 or more that practically never happens (tests/golden/types2.npz
// records it), and a GPU lane must end.
// Steps of the headline shapes use 1-10 passes, two-colour 6x6
// steps up to ~10,000 (types2.npz); the cap is a safety bound above those,
// flagged when hit (parity undefined there, as at the shuffle cap).
constexpr int CASCADE_CAP = 1 << 16;
// An RNG that raises `overflow` after a fixed number of draws (ChainMT: 624)
// bounds the cascade by itself -- every pass that continues refills >= 3
// cleared cells -- so the specialised shapes on such a stream skip the pass
// counter: it would be one more register live through the step kernels'
// cascade (measured: 5 % / 11 % slower at 9x9x6 / 16x16x8 from the spills).
template <class R, class = void>
struct DrawBounded : std::false_type {};
template <class R>
struct DrawBounded<R, std::void_t<decltype(R::DRAW_BOUNDED)>> : std::bool_constant<R::DRAW_BOUNDED> {};

template <class CF>
struct StaticDim;
template <class CF>
struct FrameDim;

// BoardConfig (match3tile/boardConfig.py:26-43) as compile-time constants.
template <int R_, int C_, int T_>
struct Cfg {
    static constexpr bool DYN = false;  // shape fixed at compile time (see FCfg)
    static constexpr int R = R_, C = C_, T = T_;
    static constexpr int N = R * C;
    static constexpr int W = (N + 31) / 32;
    static constexpr int BITS = ceil_log2(T + 1);
    static constexpr int TM = (1 << BITS) - 1;
    static constexpr int STM = (1 << (BITS + 1)) + 1 + TM;
    static constexpr int H = TM + 1;
    static constexpr int V = 2 * H;
    static constexpr int B = STM;
    static constexpr int M = TM + STM + 1;
    static constexpr int A = R * (C - 1) * 2;
    static constexpr int AW = (A + 31) / 32;
    static constexpr int NP = 7;                 // value planes for int8 cells in [0, 127]
    static constexpr int MAXG = N / 3 + 1;       // run-disjoint group creators, >= 3 cells each
    static constexpr int SHUFFLE_CAP = 1024;
    // randint(1, T+1) = 1 + masked-rejection draw on [0, T-1]
    static constexpr uint32_t TILE_RNG = (uint32_t)(T - 1);
    static constexpr uint32_t TILE_MASK = (1u << ceil_log2(T)) - 1u;
    static_assert(R >= 4 && C >= 4 && R <= 16 && C <= 16, "board size");
    static_assert(T >= 2 && BITS <= 4, "tile types must fit 4 bits");
    using Bd = BB<W>;
    using G = Geo<R, C, W>;
    using Dim = StaticDim<Cfg>;
};

// Any other BoardConfig(rows, columns, types) with 3 <= rows, columns <= 16
// and 2 <= types <= 15 runs in a 16 x 16 FRAME: cell (r, c) is bit r*16 + c,
// so the row stride -- every shift the rule code uses -- is a compile-time 16
// for every board width, and only BITS (the token layout, boardConfig.py:29-33)
// is a template parameter. Boards with more than 16 rows or columns (up to
// 32 x 32) run the same code in a 32 x 32 frame (FS = 32: one row per 32-bit
// word; 1024-bit planes, so those kernels trade speed for reach). The board's own rows / columns / types / action
// count are run-time values (FrameDim). Cells outside the board ("walls")
// hold 0 in every plane: they never start or extend a run (get_matches skips
// 0, boardFunctions.py:136), never equal a non-zero token in the legal-move
// patterns (so the reference's bounds checks, boardFunctions.py:42-92, hold
// by construction), and are kept out of every cleared / empty / refilled set
// by the board mask. (Rows < columns are accepted for reset only: the
// reference's action ids then reach past the last row and legal_actions /
// apply_action raise IndexError, boardConfig.py:27,45-59.)
template <int BITS_, int FS_ = 16>
struct FCfg {
    static constexpr bool DYN = true;
    static constexpr int FS = FS_;
    static_assert(FS == 16 || FS == 32, "frame side");
    static constexpr int R = FS, C = FS;  // the frame (row stride FS)
    static constexpr int N = R * C;
    static constexpr int W = N / 32;
    static constexpr int BITS = BITS_;
    static constexpr int TM = (1 << BITS) - 1;
    static constexpr int STM = (1 << (BITS + 1)) + 1 + TM;
    static constexpr int H = TM + 1;
    static constexpr int V = 2 * H;
    static constexpr int B = STM;
    static constexpr int M = TM + STM + 1;
    static constexpr int A = R * (C - 1) * 2;    // upper bounds: the board's are FrameDim's
    static constexpr int AW = (A + 31) / 32;
    // value planes: 7 for int8 cells in [0, 127]; with 5 token bits (types 16..31) an 8th, for
    // the mega token 128 a 5-in-a-row spawns before the clip to 32 (boardv2.py:163-164)
    static constexpr int NP = BITS >= 5 ? 8 : 7;
    static constexpr int MAXG = N / 3 + 1;
    static constexpr int SHUFFLE_CAP = 1024;
    static_assert(BITS >= 2 && BITS <= 5, "types 2..31");
    using Bd = BB<W>;
    using G = Geo<R, C, W>;
    using Dim = FrameDim<FCfg>;
};

constexpr int bits_for_types(int t) { return ceil_log2(t + 1); }

// A board shape at run time (kernel argument of the frame kernels): the
// BoardConfig fields plus, per frame cell x, whether the swap (x, x+1) /
// (x, x+FS) is the decode of some action id < A. Those are the only swaps
// legal_actions can return (boardFunctions.py:97 iterates cfg.actions), and
// on most non-square boards they are not all of them: with C = 3 the literal
// 3 of boardConfig.py:50 sends the vertical ids of row r to row r-1, and when
// rows > columns the id range A = R(C-1)*2 (boardConfig.py:27) ends inside a
// row. The dead-board test (boardv2.py:188) is "no legal id", so it must see
// exactly these swaps.
constexpr int MAX_FRAME = 32;  // largest board side
struct Shape {
    int rows, cols, types;
    int fs;  // frame side: 16, or 32 for a board with a side > 16
    uint32_t hreach[MAX_FRAME * MAX_FRAME / 32], vreach[MAX_FRAME * MAX_FRAME / 32];
};

M3_HD constexpr int frame_side(int rows, int cols) { return (rows > 16 || cols > 16) ? 32 : 16; }

// decode (boardConfig.py:45-59) -> the first cell of the swap, and whether it is vertical
M3_HD void decode_action(int action, int cols, int& r, int& c, bool& vertical) {
    const int AR = 2 * cols - 1, BR = cols - 1;
    if (action % AR >= BR) {
        c = action % AR - BR;
        r = (action - 3 - c) / AR;  // C / C++ division truncates toward 0, as Python's int()
        vertical = true;
    } else {
        c = action % AR;
        r = (action - c) / AR;
        vertical = false;
    }
}

M3_HD Shape make_shape(int rows, int cols, int types) {
    Shape s;
    s.rows = rows;
    s.cols = cols;
    s.types = types;
    s.fs = frame_side(rows, cols);
    for (int i = 0; i < MAX_FRAME * MAX_FRAME / 32; ++i) s.hreach[i] = s.vreach[i] = 0u;
    const int A = rows * (cols - 1) * 2;
    for (int a = 0; a < A; ++a) {
        int r, c;
        bool v;
        decode_action(a, cols, r, c, v);
        const int x = r * s.fs + c;
        if (r < 0 || x < 0 || x >= s.fs * s.fs) continue;
        (v ? s.vreach : s.hreach)[x >> 5] |= 1u << (x & 31);
    }
    return s;
}

// The board shape as the rule code reads it. For a Cfg every accessor is a
// compile-time constant (the specialised kernels compile exactly as if the
// constants were written in place); for an FCfg they are the run-time values
// of the board in its frame.
template <class CF>
struct StaticDim {
    M3_HD constexpr StaticDim() {}
    M3_HD constexpr StaticDim(const Shape&) {}
    M3_HD static constexpr int rows() { return CF::R; }
    M3_HD static constexpr int cols() { return CF::C; }
    M3_HD static constexpr int cells() { return CF::N; }
    M3_HD static constexpr int actions() { return CF::A; }
    M3_HD static constexpr int aw() { return CF::AW; }
    M3_HD static constexpr uint32_t tile_rng() { return CF::TILE_RNG; }
    M3_HD static constexpr uint32_t tile_mask() { return CF::TILE_MASK; }
    M3_HD static constexpr typename CF::Bd valid() { return CF::G::valid(); }
};

// A copy of x that lives in a VGPR: the frame shape's masks are wave-uniform,
// so the compiler keeps them (and everything derived from them) in SGPRs,
// runs out of the ~100 a wave has and spills thousands of SGPRs through VGPR
// lanes; held per lane they cost 3*W VGPRs instead.
M3_HD uint32_t in_vgpr(uint32_t x) {
#ifdef __HIP_DEVICE_COMPILE__
    uint32_t r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(x));
    return r;
#else
    return x;
#endif
}

template <class CF>
struct FrameDim {
    using Bd = typename CF::Bd;
    int r, c, a;
    uint32_t trng, tmask;
    Bd vmask;      // board cells
    Bd hl, vl;     // swaps (x, x+1) / (x, x+FS) that some action id decodes to (Shape)
    M3_HD FrameDim(const Shape& s) : r(s.rows), c(s.cols), a(s.rows * (s.cols - 1) * 2) {
        trng = (uint32_t)(s.types - 1);                      // randint(1, T+1)
        uint32_t m = trng;
        m |= m >> 1; m |= m >> 2; m |= m >> 4;
        tmask = m;
        const uint32_t row = low_bits(c);
#pragma unroll
        for (int i = 0; i < CF::W; ++i) {
            if constexpr (CF::FS == 16) {  // two rows per word
                const int r0 = 2 * i, r1 = 2 * i + 1;
                vmask.w[i] = (r0 < r ? row : 0u) | (r1 < r ? row << 16 : 0u);
            } else {                       // one row per word
                vmask.w[i] = i < r ? row : 0u;
            }
            hl.w[i] = in_vgpr(s.hreach[i]);
            vl.w[i] = in_vgpr(s.vreach[i]);
            vmask.w[i] = in_vgpr(vmask.w[i]);
        }
    }
    M3_HD int rows() const { return r; }
    M3_HD int cols() const { return c; }
    M3_HD int cells() const { return r * c; }
    M3_HD int actions() const { return a; }
    M3_HD int aw() const { return (a + 31) / 32; }
    M3_HD uint32_t tile_rng() const { return trng; }
    M3_HD uint32_t tile_mask() const { return tmask; }
    M3_HD Bd valid() const { return vmask; }
};

// wave-wide "any" (host build: the lane itself)
M3_HD bool wave_any(bool p) {
#ifdef __HIP_DEVICE_COMPILE__
    return __any((int)p) != 0;
#else
    return p;
#endif
}

// The cascade loop of apply_cascade_ex with a wave-uniform exit (see there): 1 everywhere, 2 in the
// frame configurations only (the specialised 16x16x8 step measured 9 % slower with it, 9x9 1-2 %),
// 0 nowhere
#ifndef M3_UNIFORM_CASCADE
#define M3_UNIFORM_CASCADE 2
#endif

// boards of at least this many words take the word-sliced legal_masks (0: never)
#ifndef M3_LEGAL_SLICED_W
#define M3_LEGAL_SLICED_W 5
#endif

// --------------------------------------------------------------------------
// small helpers
// --------------------------------------------------------------------------
template <class CF>
M3_HD typename CF::Bd tb_nonzero(const typename CF::Bd* P) {
    typename CF::Bd r = P[0];
#pragma unroll
    for (int p = 1; p < CF::BITS; ++p) r |= P[p];
    return r;
}

template <class CF, int NPU>
M3_HD typename CF::Bd special_mask(const typename CF::Bd* P) {  // board > TM
    typename CF::Bd r = P[CF::BITS];
#pragma unroll
    for (int p = CF::BITS + 1; p < NPU; ++p) r |= P[p];
    return r;
}

// bit y set iff TB[y] != TB[y + D]
template <class CF, int D>
M3_HD typename CF::Bd tb_ne(const typename CF::Bd* P) {
    typename CF::Bd r = P[0] ^ at<D>(P[0]);
#pragma unroll
    for (int p = 1; p < CF::BITS; ++p) r |= P[p] ^ at<D>(P[p]);
    return r;
}
template <class CF, int D>
M3_HD typename CF::Bd tb_eq(const typename CF::Bd* P) {
    return ~tb_ne<CF, D>(P);
}

template <class CF, int NPU>
M3_HD int cell_value(const typename CF::Bd* P, int x) {
    const typename CF::Bd bm = CF::Bd::bit_at(x);
    int v = 0;
#pragma unroll
    for (int p = 0; p < NPU; ++p) v |= (int)((P[p] & bm).any()) << p;
    return v;
}

// write value v (< 2^NPU) into cell x, overwriting
template <class CF, int NPU>
M3_HD void set_cell(typename CF::Bd* P, int x, int v) {
    const typename CF::Bd bm = CF::Bd::bit_at(x);
#pragma unroll
    for (int p = 0; p < NPU; ++p) {
        const uint32_t on = 0u - (uint32_t)((v >> p) & 1);
#pragma unroll
        for (int i = 0; i < CF::W; ++i) P[p].w[i] = (P[p].w[i] & ~bm.w[i]) | (bm.w[i] & on);
    }
}

// compile-time extraction of LEN (<= 32) bits starting at bit POS
template <int POS, int LEN, int W>
M3_HD uint32_t extract_bits(const BB<W>& b) {
    constexpr int q = POS >> 5, s = POS & 31;
    uint32_t lo = b.w[q] >> s;
    if constexpr (s != 0 && q + 1 < W) lo |= b.w[q + 1] << (32 - s);
    return LEN >= 32 ? lo : (lo & ((1u << (LEN & 31)) - 1u));
}

// --------------------------------------------------------------------------
// legal_actions (boardFunctions.py:26-112), all 2*R*(C-1) candidates at once.
// HL bit x: horizontal swap (x, x+1) is legal; VL bit x: vertical swap (x, x+C).
// --------------------------------------------------------------------------
// Word-sliced form of the same predicate for wide boards (16x16: W = 8).
// Every shifted equality at<S>(tb_eq<D>) is rewritten as one comparison of
// two offsets, [TB[y+S] == TB[y+S+D]], and evaluated one output word at a
// time straight from the tile planes, so only a few words are live at once:
// the whole-board form holds ~13 equality boards (104 VGPRs at W = 8) next
// to the planes and spilled to scratch. Where a shifted offset leaves the
// board the two forms differ (zero fill of the board vs of the comparison),
// but every such cell is cleared by the row/column mask its term carries.
template <int K, int W>
M3_HD uint32_t wget(const BB<W>& a) {
    if constexpr (K >= 0 && K < W) return a.w[K];
    else return 0u;
}
// word I of at<D>(a)
template <int D, int I, int W>
M3_HD uint32_t wat(const BB<W>& a) {
    if constexpr (D == 0) {
        return wget<I>(a);
    } else if constexpr (D > 0) {
        constexpr int q = D / 32, s = D % 32;
        if constexpr (s == 0) return wget<I + q>(a);
        else return (wget<I + q>(a) >> s) | (wget<I + q + 1>(a) << (32 - s));
    } else {
        constexpr int q = (-D) / 32, s = (-D) % 32;
        if constexpr (s == 0) return wget<I - q>(a);
        else return (wget<I - q>(a) << s) | (wget<I - q - 1>(a) >> (32 - s));
    }
}
// word I of [TB[y+A] == TB[y+B]]
template <class CF, int A, int B, int I>
M3_HD uint32_t weq(const typename CF::Bd* P) {
    uint32_t r = 0u;
#pragma unroll
    for (int p = 0; p < CF::BITS; ++p) r |= wat<A, I>(P[p]) ^ wat<B, I>(P[p]);
    return ~r;
}
template <class CF, int I>
M3_HD void legal_word(const typename CF::Bd* P, const typename CF::Bd& z0, const typename CF::Bd& spec,
                      typename CF::Bd& HL, typename CF::Bd& VL) {
    using G = typename CF::G;
    constexpr int C = CF::C, R = CF::R;
    constexpr uint32_t RGE1 = G::row_ge(1).w[I], RGE2 = G::row_ge(2).w[I];
    constexpr uint32_t RLE2 = G::row_le(R - 2).w[I], RLE3 = G::row_le(R - 3).w[I], RLE4 = G::row_le(R - 4).w[I];
    constexpr uint32_t CGE1 = G::col_ge(1).w[I], CGE2 = G::col_ge(2).w[I];
    constexpr uint32_t CLE2 = G::col_le(C - 2).w[I], CLE3 = G::col_le(C - 3).w[I], CLE4 = G::col_le(C - 4).w[I];
    {   // horizontal (see legal_masks)
        const uint32_t spc = z0.w[I] | wat<1, I>(z0) | (spec.w[I] & wat<1, I>(spec));
        const uint32_t condA = CGE2 & weq<CF, -2, 1, I>(P) & weq<CF, -1, 1, I>(P);
        const uint32_t condB = CLE4 & weq<CF, 0, 2, I>(P) & weq<CF, 0, 3, I>(P);
        const uint32_t up = RGE1 & weq<CF, -C, 1, I>(P), dn = RLE2 & weq<CF, 1, C, I>(P);
        const uint32_t up2 = RGE2 & weq<CF, -2 * C, 1, I>(P), dn2 = RLE3 & weq<CF, 1, 2 * C, I>(P);
        const uint32_t ab1 = (up & dn) | (up & ~dn & up2) | (dn & ~up & dn2);
        const uint32_t upb = RGE1 & weq<CF, 1 - C, 0, I>(P), dnb = RLE2 & weq<CF, 0, C + 1, I>(P);
        const uint32_t up2b = RGE2 & weq<CF, 1 - 2 * C, 0, I>(P), dn2b = RLE3 & weq<CF, 0, 2 * C + 1, I>(P);
        const uint32_t ab2 = (upb & dnb) | (upb & ~dnb & up2b) | (dnb & ~upb & dn2b);
        HL.w[I] = CLE2 & (spc | ((condA | condB | ab1 | ab2) & ~weq<CF, 0, 1, I>(P)));
    }
    {   // vertical
        const uint32_t spc = z0.w[I] | wat<C, I>(z0) | (spec.w[I] & wat<C, I>(spec));
        const uint32_t condA = RLE4 & weq<CF, 0, 2 * C, I>(P) & weq<CF, 0, 3 * C, I>(P);
        const uint32_t condB = RGE2 & weq<CF, -2 * C, C, I>(P) & weq<CF, -C, C, I>(P);
        const uint32_t l1 = CGE1 & weq<CF, 0, C - 1, I>(P), r1 = CLE2 & weq<CF, 0, C + 1, I>(P);
        const uint32_t l2 = CGE2 & weq<CF, 0, C - 2, I>(P), r2 = CLE3 & weq<CF, 0, C + 2, I>(P);
        const uint32_t lr1 = (l1 & r1) | (l1 & ~r1 & l2) | (r1 & ~l1 & r2);
        const uint32_t l1b = CGE1 & weq<CF, -1, C, I>(P), r1b = CLE2 & weq<CF, 1, C, I>(P);
        const uint32_t l2b = CGE2 & weq<CF, -2, C, I>(P), r2b = CLE3 & weq<CF, 2, C, I>(P);
        const uint32_t lr2 = (l1b & r1b) | (l1b & ~r1b & l2b) | (r1b & ~l1b & r2b);
        VL.w[I] = RLE2 & (spc | ((condA | condB | lr1 | lr2) & ~weq<CF, 0, C, I>(P)));
    }
}
template <class CF, int I = 0>
M3_HD void legal_words(const typename CF::Bd* P, const typename CF::Bd& z0, const typename CF::Bd& spec,
                       typename CF::Bd& HL, typename CF::Bd& VL) {
    if constexpr (I < CF::W) {
        legal_word<CF, I>(P, z0, spec, HL, VL);
        legal_words<CF, I + 1>(P, z0, spec, HL, VL);
    }
}

template <class CF>
M3_HD void legal_masks_all(const typename CF::Bd* P, const typename CF::Bd& spec,
                           typename CF::Bd& HL, typename CF::Bd& VL) {
    using Bd = typename CF::Bd;
    using G = typename CF::G;
    constexpr int C = CF::C, R = CF::R;
    constexpr Bd VALID = G::valid();
    const Bd z0 = VALID.andnot(tb_nonzero<CF>(P));  // TB == 0
    if constexpr (M3_LEGAL_SLICED_W > 0 && CF::W >= M3_LEGAL_SLICED_W) {
        legal_words<CF>(P, z0, spec, HL, VL);
        return;
    }

    // equalities shared by both directions
    const Bd e1 = tb_eq<CF, 1>(P), e2 = tb_eq<CF, 2>(P), e3 = tb_eq<CF, 3>(P);
    const Bd ecm1 = tb_eq<CF, C - 1>(P), ecp1 = tb_eq<CF, C + 1>(P);
    const Bd e2cm1 = tb_eq<CF, 2 * C - 1>(P), e2cp1 = tb_eq<CF, 2 * C + 1>(P);
    const Bd ec = tb_eq<CF, C>(P), e2c = tb_eq<CF, 2 * C>(P), e3c = tb_eq<CF, 3 * C>(P);
    const Bd ecm2 = tb_eq<CF, C - 2>(P), ecp2 = tb_eq<CF, C + 2>(P);

    constexpr Bd RGE1 = G::row_ge(1), RGE2 = G::row_ge(2), RLE2 = G::row_le(R - 2), RLE3 = G::row_le(R - 3);
    constexpr Bd CGE1 = G::col_ge(1), CGE2 = G::col_ge(2), CLE2 = G::col_le(C - 2), CLE3 = G::col_le(C - 3);

    {   // horizontal: cell1 = x, cell2 = x+1; token1 = TB[x], token2 = TB[x+1]
        const Bd spc = z0 | at<1>(z0) | (spec & at<1>(spec));                       // :100-102
        const Bd condA = G::col_ge(2) & at<-2>(e3) & at<-1>(e2);                     // :42-43
        const Bd condB = G::col_le(C - 4) & e2 & e3;                                  // :45-46
        // check_above_and_below(row, c, token2)                                       :48-59
        const Bd up = RGE1 & at<-C>(ecp1), dn = RLE2 & at<1>(ecm1);
        const Bd up2 = RGE2 & at<-2 * C>(e2cp1), dn2 = RLE3 & at<1>(e2cm1);
        const Bd ab1 = (up & dn) | (up.andnot(dn) & up2) | (dn.andnot(up) & dn2);
        // check_above_and_below(row, c+1, token1)
        const Bd upb = RGE1 & at<1 - C>(ecm1), dnb = RLE2 & ecp1;
        const Bd up2b = RGE2 & at<1 - 2 * C>(e2cm1), dn2b = RLE3 & e2cp1;
        const Bd ab2 = (upb & dnb) | (upb.andnot(dnb) & up2b) | (dnb.andnot(upb) & dn2b);
        HL = CLE2 & (spc | ((condA | condB | ab1 | ab2).andnot(e1)));                 // :103-104
    }
    {   // vertical: cell1 = x (upper), cell2 = x+C; token1 = TB[x], token2 = TB[x+C]
        const Bd spc = z0 | at<C>(z0) | (spec & at<C>(spec));
        const Bd condA = G::row_le(R - 4) & e2c & e3c;                               // :75-76
        const Bd condB = RGE2 & at<-2 * C>(e3c) & at<-C>(e2c);                       // :78-79
        // check_left_and_right(r+1, c, token1)                                        :81-92
        const Bd l1 = CGE1 & ecm1, r1 = CLE2 & ecp1, l2 = CGE2 & ecm2, r2 = CLE3 & ecp2;
        const Bd lr1 = (l1 & r1) | (l1.andnot(r1) & l2) | (r1.andnot(l1) & r2);
        // check_left_and_right(r, c, token2)
        const Bd l1b = CGE1 & at<-1>(ecp1), r1b = CLE2 & at<1>(ecm1);
        const Bd l2b = CGE2 & at<-2>(ecp2), r2b = CLE3 & at<2>(ecm2);
        const Bd lr2 = (l1b & r1b) | (l1b.andnot(r1b) & l2b) | (r1b.andnot(l1b) & r2b);
        VL = RLE2 & (spc | ((condA | condB | lr1 | lr2).andnot(ec)));
    }
}

// In a frame (FCfg) the patterns above run over the whole 16 x 16 frame; only
// swaps with both cells on the board are actions.
template <class CF>
M3_HD void legal_masks(const typename CF::Bd* P, const typename CF::Bd& spec, typename CF::Bd& HL,
                       typename CF::Bd& VL, const typename CF::Dim& dm = typename CF::Dim{}) {
    legal_masks_all<CF>(P, spec, HL, VL);
    if constexpr (CF::DYN) {
        HL &= dm.hl;
        VL &= dm.vl;
    }
}

// legal bits in action-id order (BoardConfig.actions, boardConfig.py:37,45-59):
// row r owns ids r*(2C-1) .. ; first C-1 horizontal (r,c)-(r,c+1), then C vertical.
template <class CF, int ROW = 0>
M3_HD void action_bits_rows(const typename CF::Bd& HL, const typename CF::Bd& VL, uint32_t* act) {
    if constexpr (ROW < CF::R) {
        constexpr int C = CF::C;
        constexpr int POS = ROW * (2 * C - 1);
        const uint32_t h = extract_bits<ROW * C, C - 1>(HL);
        const uint32_t v = extract_bits<ROW * C, C>(VL);
        const uint32_t f = h | (v << (C - 1));  // 2C-1 <= 31 bits
        constexpr int q = POS >> 5, s = POS & 31;
        act[q] |= f << s;
        if constexpr (s != 0 && s + 2 * C - 1 > 32 && q + 1 < CF::AW) act[q + 1] |= f >> (32 - s);
        action_bits_rows<CF, ROW + 1>(HL, VL, act);
    }
}
// Frame form: the board's row length L = 2C-1 is a run-time value, so output
// word i collects, for every id-row r, the bits of its field f_r that land in
// [32i, 32i+32) (compile-time indices only: no dynamic register indexing).
// Vertical ids of id-row r decode to cell row int((r*L + C-1 - 3) / L)
// (boardConfig.py:50's literal 3): r for C >= 4, r - 1 (0 for r = 0) for C = 3.
// Ids >= A (the last row's missing swaps, boardConfig.py:27) are dropped.
template <class CF>
M3_HD void action_bits_frame(const typename CF::Bd& HL, const typename CF::Bd& VL, uint32_t* act,
                             const typename CF::Dim& dm) {
    // One rolled pass over the board's rows: a row's field (2C-1 <= 63 bits)
    // spans up to three output words. (Unrolled over rows x words, the shift
    // amounts -- all wave-uniform -- were hoisted into ~240 SGPRs and spilled.)
    const int C = dm.cols(), L = 2 * C - 1, A = dm.actions();
    const uint64_t hm = ((uint64_t)1 << (C - 1)) - 1u, vm = ((uint64_t)1 << C) - 1u;
    auto row = [&](const typename CF::Bd& b, int r) -> uint64_t {
        if constexpr (CF::FS == 16) return (b.word_at(r >> 1) >> ((r & 1) * 16)) & 0xFFFFu;
        else return b.word_at(r);
    };
#pragma unroll
    for (int i = 0; i < CF::AW; ++i) act[i] = 0u;
    for (int r = 0; r < dm.rows(); ++r) {
        const int rv = C == 3 ? (r > 0 ? r - 1 : 0) : r;
        const uint64_t f = (row(HL, r) & hm) | ((row(VL, rv) & vm) << (C - 1));
        const int pos = r * L, q = pos >> 5, sh = pos & 31;
        const uint64_t lo = f << sh;
        const uint32_t w0 = (uint32_t)lo, w1 = (uint32_t)(lo >> 32), w2 = sh ? (uint32_t)(f >> (64 - sh)) : 0u;
#pragma unroll
        for (int i = 0; i < CF::AW; ++i)
            act[i] |= (i == q ? w0 : 0u) | (i == q + 1 ? w1 : 0u) | (i == q + 2 ? w2 : 0u);
    }
#pragma unroll
    for (int i = 0; i < CF::AW; ++i) {
        const int lim = A - 32 * i;
        act[i] = lim >= 32 ? act[i] : (lim <= 0 ? 0u : (act[i] & ((1u << lim) - 1u)));
    }
}

template <class CF>
M3_HD void action_bits(const typename CF::Bd& HL, const typename CF::Bd& VL, uint32_t* act,
                       const typename CF::Dim& dm = typename CF::Dim{}) {
    if constexpr (CF::DYN) {
        action_bits_frame<CF>(HL, VL, act, dm);
    } else {
#pragma unroll
        for (int i = 0; i < CF::AW; ++i) act[i] = 0u;
        action_bits_rows<CF, 0>(HL, VL, act);
    }
}


// np.random.choice(legal_actions) (samplerTasks.py:13): legal[randint(0, len)]
template <class CF, class RNG>
M3_HD int random_action(const uint32_t* act, RNG& rng) {
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < CF::AW; ++i) cnt += __builtin_popcount(act[i]);
    if (cnt == 0) return -1;
    int k = (int)rand_masked(rng, (uint32_t)(cnt - 1));
    int res = 0;
    bool found = false;
#pragma unroll
    for (int i = 0; i < CF::AW; ++i) {
        const int c = __builtin_popcount(act[i]);
        if (!found) {
            if (k < c) {
                res = i * 32 + select_bit(act[i], k);
                found = true;
            } else {
                k -= c;
            }
        }
    }
    return res;
}

// --------------------------------------------------------------------------
// get_matches (boardFunctions.py:121-156) + get_match_spawn_mask (:159-169)
//
// The reference scans cells row-major, skips cells already in a group, and for
// a start with a horizontal and/or vertical triple appends the maximal run(s)
// to the FIRST group sharing a cell (duplicates kept). Facts used here (each
// follows from the scan order): h-runs are disjoint, v-runs are disjoint, a
// run's vertical part never meets an earlier run, and its horizontal part can
// only meet earlier vertical runs. So a group is (Hg = union of its h-runs,
// Vg = union of its v-runs), cell multiplicity is Hg[x] + Vg[x], and the merge
// target is the first group with Vg & run_h != 0.
//
// Spawn: group with len = |Hg| + |Vg| > 3 gets, at the (len/2)-th cell of its
// sorted multiset, V/M if it is one h-run (rows equal), H/M if one v-run
// (cols equal), else B; later groups overwrite. The spawn map is returned as
// the three value planes BITS..BITS+2 (H = bit BITS, V = bit BITS+1, B = both,
// M = bit BITS+2).
// --------------------------------------------------------------------------
// Group tables. get_matches only touches a group through get_h/get_v/put, so
// the storage is pluggable: the HIP kernels keep a small per-lane table in LDS
// (m3_api.hip, LdsStore) and report overflow; the fallback pass and the host
// harness use ArrayStore, which can hold every group a board can form.
template <class CF>
struct ArrayStore {
    static constexpr int CAP = CF::MAXG;
    typename CF::Bd h[CAP];
    typename CF::Bd v[CAP];
    M3_HD typename CF::Bd get_h(int g) const { return h[g]; }
    M3_HD typename CF::Bd get_v(int g) const { return v[g]; }
    M3_HD bool put(int g, const typename CF::Bd& hh, const typename CF::Bd& vv) {
        h[g] = hh;
        v[g] = vv;
        return true;
    }
};

// A deliberately tiny table (test harness): forces the overflow path.
template <class CF, int CAP_>
struct SmallStore {
    static constexpr int CAP = CAP_;
    typename CF::Bd h[CAP];
    typename CF::Bd v[CAP];
    M3_HD typename CF::Bd get_h(int g) const { return h[g]; }
    M3_HD typename CF::Bd get_v(int g) const { return v[g]; }
    M3_HD bool put(int g, const typename CF::Bd& hh, const typename CF::Bd& vv) {
        h[g] = hh;
        v[g] = vv;
        return true;
    }
};

enum : int { MATCH_NONE = 0, MATCH_FOUND = 1, MATCH_OVERFLOW = -1 };

template <class CF>
M3_HD int multiset_select(const typename CF::Bd& hg, const typename CF::Bd& vg, int k) {
#pragma unroll
    for (int i = 0; i < CF::W; ++i) {
        const int c = __builtin_popcount(hg.w[i]) + __builtin_popcount(vg.w[i]);
        if (k < c) {
            uint32_t u = hg.w[i] | vg.w[i];
            while (u) {
                const int b = __builtin_ctz(u);
                const int m = (int)((hg.w[i] >> b) & 1u) + (int)((vg.w[i] >> b) & 1u);
                if (k < m) return i * 32 + b;
                k -= m;
                u &= u - 1u;
            }
        }
        k -= c;
    }
    return 0;
}

struct NoStore {
    static constexpr int CAP = 0;
};

// Returns MATCH_NONE / MATCH_FOUND, or MATCH_OVERFLOW when SPAWN needs more
// groups than Store::CAP (the caller then recomputes with ArrayStore).
template <class CF, bool SPAWN, class Store>
M3_HD int match_scan(const typename CF::Bd* P, typename CF::Bd& mask, typename CF::Bd* sw, Store& st) {
    using Bd = typename CF::Bd;
    using G = typename CF::G;
    constexpr int C = CF::C, R = CF::R;
    constexpr Bd CLE2 = G::col_le(C - 2), RLE2 = G::row_le(R - 2);

    const Bd nz = tb_nonzero<CF>(P);
    const Bd e1h = CLE2 & tb_eq<CF, 1>(P);   // TB[x] == TB[x+1], same row
    const Bd e1v = RLE2 & tb_eq<CF, C>(P);   // TB[x] == TB[x+C]
    const Bd h3 = nz & e1h & at<1>(e1h);     // :138 horizontal triple starts here
    const Bd v3 = nz & e1v & at<C>(e1v);     // :147 vertical triple starts here
    Bd cand = h3 | v3;
    mask = Bd::zero();
    if constexpr (SPAWN) {
        sw[0] = Bd::zero();
        sw[1] = Bd::zero();
        sw[2] = Bd::zero();
    }
    if (!cand.any()) return MATCH_NONE;

    // doubling link masks for run floods (runs are <= 16 long; <= 32 in the 32 x 32 frame)
    const Bd dh2 = e1h & at<1>(e1h), dh4 = dh2 & at<2>(dh2), dh8 = dh4 & at<4>(dh4);
    const Bd dv2 = e1v & at<C>(e1v), dv4 = dv2 & at<2 * C>(dv2), dv8 = dv4 & at<4 * C>(dv4);
    Bd dh16, dv16;
    if constexpr (C > 16) dh16 = dh8 & at<8>(dh8);
    if constexpr (R > 16) dv16 = dv8 & at<8 * C>(dv8);

    int ng = 0;
    Bd vruns = Bd::zero();
    while (cand.any()) {                                       // row-major scan over run starts
        const int x = cand.lowest();
        const Bd bx = Bd::bit_at(x);
        Bd rh = Bd::zero(), rv = Bd::zero();
        if ((h3 & bx).any()) {                                 // :138-144 extend right
            rh = bx;
            rh |= at<-1>(rh & e1h);
            rh |= at<-2>(rh & dh2);
            rh |= at<-4>(rh & dh4);
            if constexpr (C > 8) rh |= at<-8>(rh & dh8);
            if constexpr (C > 16) rh |= at<-16>(rh & dh16);
        }
        if ((v3 & bx).any()) {                                 // :147-153 extend down
            rv = bx;
            rv |= at<-C>(rv & e1v);
            rv |= at<-2 * C>(rv & dv2);
            rv |= at<-4 * C>(rv & dv4);
            if constexpr (R > 8) rv |= at<-8 * C>(rv & dv8);
            if constexpr (R > 16) rv |= at<-16 * C>(rv & dv16);
        }
        const Bd run = rh | rv;
        mask |= run;
        cand = cand.andnot(run | bx);                           // later starts inside a run are skipped (:136)
        if constexpr (SPAWN) {
            int g = -1;
            if ((rh & vruns).any()) {                          // add_to_matches (:126-131)
                for (int gi = 0; gi < ng; ++gi) {
                    if ((st.get_v(gi) & rh).any()) { g = gi; break; }
                }
            }
            if (g < 0) {
                if (ng == Store::CAP || !st.put(ng, rh, rv)) return MATCH_OVERFLOW;
                ++ng;
            } else if (!st.put(g, st.get_h(g) | rh, st.get_v(g) | rv)) {
                return MATCH_OVERFLOW;
            }
            vruns |= rv;
        }
    }
    if constexpr (SPAWN) {
        for (int gi = 0; gi < ng; ++gi) {                      // get_match_spawn_mask (:159-169)
            const Bd hg = st.get_h(gi), vg = st.get_v(gi);
            const int len = hg.popc() + vg.popc();
            if (len <= 3) continue;
            int centre, kind;  // kind bits: 1 = plane BITS, 2 = BITS+1, 4 = BITS+2
            if (!vg.any()) {                                   // all rows equal
                centre = hg.lowest() + len / 2;
                kind = len > 4 ? 4 : 2;                        // M : V
            } else if (!hg.any()) {                            // all cols equal
                centre = vg.lowest() + (len / 2) * C;
                kind = len > 4 ? 4 : 1;                        // M : H
            } else {
                centre = multiset_select<CF>(hg, vg, len / 2);
                kind = 3;                                      // B
            }
            const Bd bm = Bd::bit_at(centre);
            sw[0] = sw[0].andnot(bm);
            sw[1] = sw[1].andnot(bm);
            sw[2] = sw[2].andnot(bm);
            if (kind & 1) sw[0] |= bm;
            if (kind & 2) sw[1] |= bm;
            if (kind & 4) sw[2] |= bm;
        }
    }
    return MATCH_FOUND;
}

// get_matches without the per-start loop when that is provably equal (round 6). If no cell lies in
// both a horizontal and a vertical run of three or more, the scan visits exactly the first cell of
// every maximal run (a first cell can only be covered by a run of the other direction), takes that
// run whole and never merges (a run meets no earlier group): every maximal run is its own group,
// the mask is the union of the runs, and a group's length is its run's. Spawns (groups longer than
// 3): an h-run of 4 puts V, of 5 M, at its first cell + 2; a v-run of 4 puts H, of 5 M, two rows
// below its top (boardFunctions.py:159-169, get_center :8-13 on a sorted straight run). Runs of 6 or
// more (centre past + 2) and crossing runs (L / T groups, merged arms, duplicates) take the scan.
// Whole-board operations only: no loop, no group table, no overflow. Host-checked equal to the scan
// on every fixture and on random boards (tests/test_hostcore_cpu.py::test_fast_matches_equal_scan).
#ifndef M3_FAST_MATCH
#define M3_FAST_MATCH 1
#endif
template <class CF, class Store>
M3_HD int get_matches(const typename CF::Bd* P, typename CF::Bd& mask, typename CF::Bd* sw, Store& st) {
    if constexpr (M3_FAST_MATCH) {
        using Bd = typename CF::Bd;
        using G = typename CF::G;
        constexpr int C = CF::C, R = CF::R;
        constexpr Bd CLE2 = G::col_le(C - 2), RLE2 = G::row_le(R - 2);
        const Bd nz = tb_nonzero<CF>(P);
        const Bd e1h = CLE2 & tb_eq<CF, 1>(P);   // TB[x] == TB[x+1], same row
        const Bd e1v = RLE2 & tb_eq<CF, C>(P);   // TB[x] == TB[x+C]
        const Bd h3 = nz & e1h & at<1>(e1h);     // a horizontal triple starts here
        const Bd v3 = nz & e1v & at<C>(e1v);     // a vertical triple starts here
        if (!(h3 | v3).any()) {
            mask = Bd::zero();
            sw[0] = sw[1] = sw[2] = Bd::zero();
            return MATCH_NONE;
        }
        const Bd hc = h3 | at<-1>(h3) | at<-2>(h3);      // every cell of a horizontal run
        const Bd vc = v3 | at<-C>(v3) | at<-2 * C>(v3);  // every cell of a vertical run
        const Bd h4 = h3 & at<1>(h3), v4 = v3 & at<C>(v3);  // a run of >= 4 starts here
        const bool six = (h4 & at<2>(h4)).any() || (v4 & at<2 * C>(v4)).any();
        if (!(hc & vc).any() && !six) {
            const Bd hf = h4.andnot(at<-1>(e1h));          // first cells of h-runs of 4 or 5
            const Bd vf = v4.andnot(at<-C>(e1v));          // top cells of v-runs of 4 or 5
            const Bd hf5 = hf & at<2>(h3), vf5 = vf & at<2 * C>(v3);
            mask = hc | vc;
            sw[0] = at<-2 * C>(vf.andnot(vf5));                // H (v-run of 4)
            sw[1] = at<-2>(hf.andnot(hf5));                    // V (h-run of 4)
            sw[2] = at<-2>(hf5) | at<-2 * C>(vf5);             // M (runs of 5)
            return MATCH_FOUND;
        }
    }
    return match_scan<CF, true>(P, mask, sw, st);
}

// mask only (BoardV2.__init__ only asks "any match?" and which cells,
// boardv2.py:23-27), by the sequential scan
template <class CF>
M3_HD bool get_match_mask_scan(const typename CF::Bd* P, typename CF::Bd& mask) {
    NoStore ns;
    return match_scan<CF, false>(P, mask, nullptr, ns) != MATCH_NONE;
}

// The same mask without the per-start loop whenever that is provably equal.
// The scan visits each maximal run's first start (leftmost / top cell) unless
// an EARLIER run already covers it: an h-run start inside a v-run from above,
// or a v-run start inside an h-run from its left (the dropped-arm quirk). If no
// start cell is covered by a run of the other direction that began before it,
// every maximal run is added whole and the mask is just the union of all runs
// of three or more; otherwise fall back to the scan. Uniform cost, a handful of
// whole-board operations (no loop over run starts).
template <class CF>
M3_HD bool get_match_mask(const typename CF::Bd* P, typename CF::Bd& mask) {
    using Bd = typename CF::Bd;
    using G = typename CF::G;
    constexpr int C = CF::C, R = CF::R;
    constexpr Bd CLE2 = G::col_le(C - 2), RLE2 = G::row_le(R - 2);
    const Bd nz = tb_nonzero<CF>(P);
    const Bd e1h = CLE2 & tb_eq<CF, 1>(P);
    const Bd e1v = RLE2 & tb_eq<CF, C>(P);
    const Bd h3 = nz & e1h & at<1>(e1h);        // a horizontal triple starts here
    const Bd v3 = nz & e1v & at<C>(e1v);        // a vertical triple starts here
    if (!(h3 | v3).any()) {
        mask = Bd::zero();
        return false;
    }
    const Bd hc = h3 | at<-1>(h3) | at<-2>(h3);             // every cell of a horizontal run
    const Bd vc = v3 | at<-C>(v3) | at<-2 * C>(v3);         // every cell of a vertical run
    const Bd hin = hc.andnot(h3.andnot(at<-1>(h3)));        // run cells right of the run's first start
    const Bd vin = vc.andnot(v3.andnot(at<-C>(v3)));        // run cells below the run's top
    if (!((h3 & vin) | (v3 & hin)).any()) {
        mask = hc | vc;
        return true;
    }
    return get_match_mask_scan<CF>(P, mask);
}

// --------------------------------------------------------------------------
// cascade pieces (boardv2.py:138-202)
// --------------------------------------------------------------------------
// Python slice a[start:stop] on an axis of length n (start may be -1)
M3_HD void py_slice(int start, int stop, int n, int& lo, int& hi) {
    if (start < 0) {
        start += n;
        if (start < 0) start = 0;
    }
    if (start > n) start = n;
    if (stop > n) stop = n;
    lo = start;
    hi = stop > start ? stop : start;
}

// special tokens whose TB is zero fire (:141-154); SP is not refreshed inside
// the pass, so the effects are a union and order does not matter.
template <class CF, int NPU>
M3_HD typename CF::Bd fire_specials(const typename CF::Bd* P, typename CF::Bd z,
                                   const typename CF::Dim& dm = typename CF::Dim{}) {
    using Bd = typename CF::Bd;
    using G = typename CF::G;
    constexpr int BITS = CF::BITS, C = CF::C;
    const int R = dm.rows(), CB = dm.cols();  // slice lengths: the board's
    const Bd spz = z & special_mask<CF, NPU>(P);
    const Bd kh = P[BITS].andnot(P[BITS + 1]);   // (x & STM) == H
    const Bd kv = P[BITS + 1].andnot(P[BITS]);   // (x & STM) == V
    const Bd kb = P[BITS] & P[BITS + 1];         // (x & STM) == B
    Bd trig = spz & (kh | kv | kb);
    Bd add = Bd::zero();
    while (trig.any()) {
        const int x = trig.lowest();
        trig.pop_lowest();
        const int i = x / C, j = x % C;
        if (kh.test(x)) {
            add |= G::row_band(i, i + 1);                   // token_board[i, :] = 0
        } else if (kv.test(x)) {
            add |= G::col_band(j, j + 1);                   // token_board[:, j] = 0
        } else {                                            // token_board[j-1:j+1, i-1:i+1] = 0
            int rl, rh, cl, ch;
            py_slice(j - 1, j + 1, R, rl, rh);
            py_slice(i - 1, i + 1, CB, cl, ch);
            add |= G::row_band(rl, rh) & G::col_band(cl, ch);
        }
    }
    if constexpr (CF::DYN) return (z | add) & dm.valid();  // frame rows / columns reach into the walls
    return z | add;
}

// reward += sum(points[TB == 0]) with point_board_vec (:58-65, :157-158)
template <class CF, int NPU>
M3_HD int score(const typename CF::Bd* P, const typename CF::Bd& z) {
    using Bd = typename CF::Bd;
    constexpr int BITS = CF::BITS;
    const Bd spec = special_mask<CF, NPU>(P);
    Bd hi2 = P[BITS + 2];
#pragma unroll
    for (int p = BITS + 3; p < NPU; ++p) hi2 |= P[p];
    Bd other = P[0];
#pragma unroll
    for (int p = 1; p < NPU; ++p)
        if (p != BITS + 2) other |= P[p];
    const Bd eqm = P[BITS + 2].andnot(other);                  // x == M
    const Bd kb = P[BITS] & P[BITS + 1];
    const Bd lt = spec.andnot(hi2 | kb);                       // TM < x < STM
    const Bd zs = z & spec;
    const int n_all = z.popc(), n_spec = zs.popc();
    const int n_m = (z & eqm).popc(), n_lt = (z & lt).popc();
    return 2 * (n_all - n_spec) + 250 * n_m + 25 * n_lt + 50 * (n_spec - n_m - n_lt);
}

// next_state[TB==0] = 0; next_state += spawn; clip(0, 32)   (:161-163)
template <class CF, int NPU>
M3_HD void merge_clip(typename CF::Bd* P, const typename CF::Bd& z, const typename CF::Bd* sw) {
    using Bd = typename CF::Bd;
    constexpr int BITS = CF::BITS;
#pragma unroll
    for (int p = 0; p < NPU; ++p) P[p] = P[p].andnot(z);
    P[BITS] |= sw[0];
    P[BITS + 1] |= sw[1];
    P[BITS + 2] |= sw[2];
    // > 32: bit 5 with any lower bit, or bit 6 (or 7)
    Bd low = P[0];
#pragma unroll
    for (int p = 1; p < 5; ++p) low |= P[p];
    // plane 6 holds input values >= 64 (first pass) or a spawned M = 64 on
    // 4-bit-type boards (V = 64 on 5-bit ones); plane 7 (5-bit types only) a
    // spawned M = 128; all clip to 32
    Bd hi = P[6];
#pragma unroll
    for (int p = 7; p < CF::NP; ++p) hi |= P[p];
    const Bd cl = (P[5] & low) | hi;
#pragma unroll
    for (int p = 0; p < 5; ++p) P[p] = P[p].andnot(cl);
    P[5] |= cl;
#pragma unroll
    for (int p = 6; p < CF::NP; ++p) P[p] = Bd::zero();
}

// gravity + refill (:166-173). Columns left to right, new tiles on top in draw
// order (new[0] at row 0). Tiles come from randint(1, T+1).
// gravity: returns the (top-aligned) empty cells
//
// Round 5: by the binary decomposition of every tile's drop distance (the number of holes below
// it in its column), low bits first -- stage i moves the tiles whose distance has bit i set by
// 2^i rows. This is Hacker's Delight's `compress` (7-4) run down every column at once: the bit i
// of each distance is a column-wise suffix parity of the holes still counted (mp), and moving
// the low bits first never lets two tiles meet. A stage no lane of the wave needs is skipped as
// a whole (wave-uniform branch): the wave runs ceil(log2 R) fixed stages at most instead of the
// row-by-row loop's max-drop + 1 passes, with no divergence (M3_GRAVITY_LOOP=1: the loop).
#ifndef M3_GRAVITY_LOOP
#define M3_GRAVITY_LOOP 0
#endif
template <class CF>
M3_HD typename CF::Bd gravity_decomp(typename CF::Bd* P, const typename CF::Dim& dm = typename CF::Dim{}) {
    using Bd = typename CF::Bd;
    constexpr int C = CF::C, R = CF::R, NPU = 6;
    constexpr int STAGES = ceil_log2(R);           // drop distances < R
    const Bd VALID = dm.valid();                   // walls are neither holes nor tiles
    Bd m = P[0];
#pragma unroll
    for (int p = 1; p < NPU; ++p) m |= P[p];
    Bd mk = at<C>(VALID.andnot(m));                // a hole right below
    auto stage = [&](auto S) {
        constexpr int D = (1 << decltype(S)::value) * C;  // rows moved in this stage, as bits
        Bd mp = mk ^ at<C>(mk);                    // holes below, counted mod 2 down the column
        if constexpr (R > 3) mp ^= at<2 * C>(mp);  // (a suffix over the R - 1 cells below)
        if constexpr (R > 5) mp ^= at<4 * C>(mp);
        if constexpr (R > 9) mp ^= at<8 * C>(mp);
        if constexpr (R > 17) mp ^= at<16 * C>(mp);
        const Bd mv = mp & m;                      // tiles whose distance has this bit
        if (wave_any(mv.any())) {
            m = m.andnot(mv) | at<-D>(mv);
#pragma unroll
            for (int p = 0; p < NPU; ++p) {
                const Bd t = P[p] & mv;
                P[p] = P[p].andnot(mv) | at<-D>(t);
            }
        }
        mk = mk.andnot(mp);
    };
    stage(std::integral_constant<int, 0>{});
    if constexpr (STAGES > 1) if (wave_any(mk.any())) {
        stage(std::integral_constant<int, 1>{});
        if constexpr (STAGES > 2) if (wave_any(mk.any())) {
            stage(std::integral_constant<int, 2>{});
            if constexpr (STAGES > 3) if (wave_any(mk.any())) {
                stage(std::integral_constant<int, 3>{});
                if constexpr (STAGES > 4) if (wave_any(mk.any())) stage(std::integral_constant<int, 4>{});
            }
        }
    }
    return VALID.andnot(m);
}

template <class CF>
M3_HD typename CF::Bd gravity(typename CF::Bd* P, const typename CF::Dim& dm = typename CF::Dim{}) {
    if constexpr (!M3_GRAVITY_LOOP) return gravity_decomp<CF>(P, dm);
    using Bd = typename CF::Bd;
    constexpr int C = CF::C, R = CF::R, NPU = 6;
    const Bd VALID = dm.valid();  // walls are neither holes nor tiles
    Bd occ = P[0];
#pragma unroll
    for (int p = 1; p < NPU; ++p) occ |= P[p];
    for (;;) {  // drop every tile that has a hole somewhere below it by one row
        const Bd e = VALID.andnot(occ);
        Bd s = at<C>(e);
        s |= at<C>(s);
        s |= at<2 * C>(s);
        s |= at<4 * C>(s);
        if constexpr (R > 9) s |= at<8 * C>(s);
        if constexpr (R > 17) s |= at<16 * C>(s);
        const Bd mv = occ & s;
        if (!mv.any()) break;
#pragma unroll
        for (int p = 0; p < NPU; ++p) {
            const Bd m = P[p] & mv;
            P[p] = P[p].andnot(mv) | at<-C>(m);
        }
        occ = occ.andnot(mv) | at<-C>(mv);
    }
    return VALID.andnot(occ);
}

// refill of the top-aligned empty cells em
template <class CF, class RNG>
M3_HD void refill(typename CF::Bd* P, const typename CF::Bd& em, RNG& rng,
                  const typename CF::Dim& dm = typename CF::Dim{}) {
    using Bd = typename CF::Bd;
    constexpr int C = CF::C, R = CF::R;
    if (!em.any()) return;
    uint32_t tops = em.w[0] & low_bits(C);  // columns with at least one empty cell
    int c = __builtin_ctz(tops);
    int r = 0;
    // One raw draw per loop trip (the masked-rejection of randint(1, T+1) is
    // folded into the trip count): with a nested rejection loop per tile the
    // wave would wait for its unluckiest lane on every tile.
    const uint32_t tmask = dm.tile_mask(), trng = dm.tile_rng();
    for (;;) {
        uint32_t v = rng.next32() & tmask;
        if (rng.overflow) break;
        if (v > trng) continue;
        v += 1u;                                           // randint(1, T+1)
        const int x = r * C + c;
        const Bd bm = Bd::bit_at(x);
#pragma unroll
        for (int p = 0; p < CF::BITS; ++p) {
            const uint32_t on = 0u - ((v >> p) & 1u);
#pragma unroll
            for (int i = 0; i < CF::W; ++i) P[p].w[i] |= bm.w[i] & on;
        }
        if (r + 1 < R && em.test(x + C)) {
            ++r;
        } else {
            tops &= ~(1u << c);
            if (!tops) break;
            c = __builtin_ctz(tops);
            r = 0;
        }
    }
}

// shuffle (boardFunctions.py:16-23): reseed, Fisher-Yates over rows with
// random_interval, then put every special back at its original cell.
template <class CF, class RNG>
M3_HD void shuffle_rows(typename CF::Bd* P, RNG& rng, const typename CF::Dim& dm = typename CF::Dim{}) {
    using Bd = typename CF::Bd;
    constexpr int C = CF::C, R = CF::R, NPU = 6;
    rng.reseed();
    const Bd sp = special_mask<CF, NPU>(P);
    if constexpr (R > 16) {  // 32 x 32 frame: one row per word, the permutation in a small array
        static_assert(C == 32, "one row per word");
        uint8_t perm[R];
#pragma unroll
        for (int i = 0; i < R; ++i) perm[i] = (uint8_t)i;
        for (int i = dm.rows() - 1; i >= 1; --i) {
            const int j = (int)rand_masked(rng, (uint32_t)i);
            const uint8_t a = perm[i];
            perm[i] = perm[j];
            perm[j] = a;
        }
        Bd out[NPU];
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int src = perm[i];
#pragma unroll
            for (int p = 0; p < NPU; ++p) out[p].w[i] = P[p].word_at(src);
        }
#pragma unroll
        for (int p = 0; p < NPU; ++p) P[p] = out[p].andnot(sp) | (P[p] & sp);
        return;
    }
    uint64_t idx = 0;  // nibble i = source row of row i
#pragma unroll
    for (int i = 0; i < R; ++i) idx |= (uint64_t)i << (4 * i);
    for (int i = dm.rows() - 1; i >= 1; --i) {  // the board's rows; frame rows below stay in place
        const int j = (int)rand_masked(rng, (uint32_t)i);
        const uint64_t a = (idx >> (4 * i)) & 0xFull, b = (idx >> (4 * j)) & 0xFull;
        idx &= ~((0xFull << (4 * i)) | (0xFull << (4 * j)));
        idx |= (b << (4 * i)) | (a << (4 * j));
    }
    Bd out[NPU];
#pragma unroll
    for (int p = 0; p < NPU; ++p) out[p] = Bd::zero();
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const int src = (int)((idx >> (4 * i)) & 0xFull);
        const int sb = src * C;
        const int q = sb >> 5, s = sb & 31;
#pragma unroll
        for (int p = 0; p < NPU; ++p) {
            const uint32_t lo = P[p].word_at(q), hi = P[p].word_at(q + 1);
            uint32_t f = s ? ((lo >> s) | (hi << ((32 - s) & 31))) : lo;
            f &= low_bits(C);
            const int dpos = i * C;
            const int dq = dpos >> 5, ds = dpos & 31;
            out[p].w[dq] |= f << ds;
            if (ds + C > 32 && dq + 1 < CF::W) out[p].w[dq + 1] |= f >> (32 - ds);
        }
    }
#pragma unroll
    for (int p = 0; p < NPU; ++p) P[p] = out[p].andnot(sp) | (P[p] & sp);
}

// --------------------------------------------------------------------------
// BoardV2.apply_action (boardv2.py:43-207), in two parts so a batched kernel
// can bound the divergent cascade (apply_begin + apply_cascade == apply_action):
//   apply_begin   :44-136 + the first clear pass (:141-163 on the swap's
//                 matches / combo window). Returns false when the step is
//                 complete already (terminal board, bad action: HL/VL set;
//                 group-table overflow: flagged for recompute).
//   apply_cascade the fixed point :138-202 from the top of its inner loop.
//                 With limit >= 0 it stops before starting inner iteration
//                 limit + 1 and returns false: the whole state is then P
//                 (planes 0..5; 6 is clear after the first pass), rng, reward
//                 and flags, and a later apply_cascade(limit = -1) on that
//                 state finishes the step exactly as one uninterrupted call
//                 would (the spawn planes are rewritten before each use).
// P: NP planes in/out; sets flags, the reward and the legal masks of the
// resulting board.
// --------------------------------------------------------------------------
template <class CF, class RNG, class Store>
M3_HD bool apply_begin(typename CF::Bd* P, int n_actions, int action, RNG& rng, uint32_t& flags,
                       typename CF::Bd& HL, typename CF::Bd& VL, Store& st, int& reward,
                       const typename CF::Dim& dm = typename CF::Dim{}) {
    using Bd = typename CF::Bd;
    using G = typename CF::G;
    constexpr int C = CF::C, TM = CF::TM;  // C: the row stride of the bit layout
    constexpr int H = CF::H, V = CF::V, B = CF::B, M = CF::M;
    const int R = dm.rows(), CB = dm.cols();  // the board (== R, C unless in a frame)
    const Bd VALID = dm.valid();
    flags = 0u;
    reward = 0;
    mark<PH_LOAD>(st);
    if (n_actions < 1 || action < 0 || action >= dm.actions()) {  // :44-45, KeyError at :48
        flags = (n_actions < 1) ? FLAG_TERMINAL : FLAG_BAD_ACTION;
        legal_masks<CF>(P, special_mask<CF, CF::NP>(P), HL, VL, dm);
        return false;
    }
    rng.reseed();                                               // :46
    // decode (boardConfig.py:45-59)
    const int AR = 2 * CB - 1, BR = CB - 1;
    int sr, sc, tr, tc;
    if (action % AR >= BR) {
        sc = action % AR - BR;
        sr = (action - 3 - sc) / AR;
        tr = sr + 1;
        tc = sc;
    } else {
        sc = action % AR;
        sr = (action - sc) / AR;
        tr = sr;
        tc = sc + 1;
    }
    const int s = sr * C + sc, t = tr * C + tc;
    const int tok1 = cell_value<CF, CF::NP>(P, s), tok2 = cell_value<CF, CF::NP>(P, t);  // :73
    {   // swap (:51, boardFunctions.py:115-118)
        const Bd st = Bd::bit_at(s) | Bd::bit_at(t);
        const int d = tok1 ^ tok2;
#pragma unroll
        for (int p = 0; p < CF::NP; ++p)
            if ((d >> p) & 1) P[p] ^= st;
    }
    const int ty1 = tok2 > TM ? tok2 : 0, ty2 = tok1 > TM ? tok1 : 0;  // special_tokens[source/target] :74
    auto are = [&](int a, int b) { return (ty1 == a && ty2 == b) || (ty2 == a && ty1 == b); };  // :76-77

    Bd sw[3] = {Bd::zero(), Bd::zero(), Bd::zero()};
    Bd zr;
    if (are(M, M)) {                                            // :81-82
        zr = VALID;
    } else if (are(M, B) || are(M, H) || are(M, V) || are(M, 0)) {
        zr = Bd::zero();  // :84-103 select TB == max(token1, token2) == M: empty by construction
    } else if (are(B, B)) {                                     // :112-116
        const int r0 = tr - 2 < 0 ? 0 : tr - 2, r1 = tr + 2 > R ? R : tr + 2;
        const int c0 = tc - 2 < 0 ? 0 : tc - 2, c1 = tc + 2 > CB ? CB : tc + 2;
        zr = G::row_band(r0, r1) & G::col_band(c0, c1);
    } else if (are(B, H) || are(B, V)) {                        // :123-125
        const int r0 = tr - 2 < 0 ? 0 : tr - 2, r1 = tr + 2 > R ? R : tr + 2;
        const int c0 = tc - 2 < 0 ? 0 : tc - 2, c1 = tc + 2 > CB ? CB : tc + 2;
        zr = G::col_band(c0, c1) | G::row_band(r0, r1);
    } else if (are(H, V)) {                                     // :130-132 rows < t.col, rows >= t.row
        zr = G::row_band(0, tc < R ? tc : R) | G::row_band(tr, R);
    } else {                                                    // :133-136
        mark<PH_SWAP>(st);
        if (get_matches<CF>(P, zr, sw, st) == MATCH_OVERFLOW) {
            flags |= FLAG_GROUP_OVERFLOW;
            return false;
        }
        mark<PH_MATCH>(st);
    }
    mark<PH_SWAP>(st);
    // first pass with all 7 planes (input values may exceed 32 until the clip)
    Bd z = zr | VALID.andnot(tb_nonzero<CF>(P));
    z = fire_specials<CF, CF::NP>(P, z, dm);  // (in a frame: also clips the windows above to the board)
    reward += score<CF, CF::NP>(P, z);
    merge_clip<CF, CF::NP>(P, z, sw);
    mark<PH_CLEAR>(st);
    return true;
}

// apply_cascade_ex: the fixed point with more exit/entry points, so batched
// kernels can leave rare or long work to another launch (m3_api.hip):
//   OPTS & CASX_STOP_SETTLED  return CAS_SETTLED as soon as the board has no
//                  match left, before its legal set (the caller computes it);
//   OPTS & CASX_STOP_DEAD     return CAS_DEAD when the settled board has no
//                  legal move, before the row shuffle (:188-194) -- the
//                  shuffle path is then not even compiled into the caller,
//                  which keeps its register allocation small;
//   start_settled  the state is a settled board (CAS_SETTLED / CAS_DEAD):
//                  continue at its legal set.
// Returns CAS_PAUSED (limit reached), CAS_SETTLED, CAS_DEAD, or CAS_DONE
// (HL/VL set; or flags ask for a recompute).
enum : int { CAS_PAUSED = 0, CAS_DONE = 1, CAS_SETTLED = 2, CAS_DEAD = 3 };
enum : int { CASX_STOP_SETTLED = 1, CASX_STOP_DEAD = 2 };

template <class CF, int OPTS, class RNG, class Store>
M3_HD int apply_cascade_ex(typename CF::Bd* P, RNG& rng, uint32_t& flags, typename CF::Bd& HL,
                           typename CF::Bd& VL, Store& st, int& reward, int limit, bool start_settled,
                           const typename CF::Dim& dm = typename CF::Dim{}) {
    using Bd = typename CF::Bd;
    const Bd VALID = dm.valid();
    Bd sw[3];
    int it = 0;
    bool settled = start_settled;
    for (;;) {                                                  // :138
        Bd mask;
        bool found = false;
        if (!settled) {
            if constexpr (M3_UNIFORM_CASCADE == 1 || (M3_UNIFORM_CASCADE == 2 && CF::DYN)) {
                // cascade: refill, rematch, clear while matches remain -- with a wave-UNIFORM loop exit:
                // the wave runs its longest lane's trip count (as the divergent loop does) with the
                // body predicated per lane, so no value leaves the loop from a lane that quit early.
                // Values live out of a divergent loop came back stale (or garbage) for such lanes
                // whenever the kernel spilled VGPRs (the frame-kernel lane
                // interference; tools/dbg/lanes*.py).
                int xr = -1;  // an early return (paused, group overflow)
                bool live = true;
                for (;;) {
                    if (!wave_any(live)) break;
                    if (!live) continue;
                    if (it == limit) {                              // paused before iteration limit + 1
                        xr = CAS_PAUSED;
                        live = false;
                        continue;
                    }
                    if constexpr (CF::DYN || !DrawBounded<RNG>::value) {
                        if (it >= CASCADE_CAP) {
                            flags |= FLAG_CASCADE_CAP;
                            live = false;
                            continue;
                        }
                    }
                    ++it;
                    const Bd em = gravity<CF>(P, dm);               // :166-173
                    mark<PH_DROP>(st);
                    refill<CF>(P, em, rng, dm);
                    mark<PH_REFILL>(st);
                    if (rng.overflow) {
                        live = false;
                        continue;
                    }
                    const int mr = get_matches<CF>(P, mask, sw, st);  // :176-181
                    mark<PH_MATCH>(st);
                    if (mr == MATCH_OVERFLOW) {
                        flags |= FLAG_GROUP_OVERFLOW;
                        xr = CAS_DONE;
                        live = false;
                        continue;
                    }
                    if (mr != MATCH_FOUND) {
                        live = false;
                        continue;
                    }
                    Bd z = mask | VALID.andnot(tb_nonzero<CF>(P));  // :199 + TB==0 cells
                    z = fire_specials<CF, 6>(P, z, dm);
                    reward += score<CF, 6>(P, z);
                    merge_clip<CF, 6>(P, z, sw);
                    mark<PH_CLEAR>(st);
                }
                if (xr >= 0) return xr;
            } else {
            for (;;) {  // cascade: refill, rematch, clear while matches remain
                if (it == limit) return CAS_PAUSED;             // paused before iteration limit + 1
                if constexpr (CF::DYN || !DrawBounded<RNG>::value) {
                    if (it >= CASCADE_CAP) {
                        flags |= FLAG_CASCADE_CAP;
                        break;
                    }
                }
                ++it;
                const Bd em = gravity<CF>(P, dm);               // :166-173
                mark<PH_DROP>(st);
                refill<CF>(P, em, rng, dm);
                mark<PH_REFILL>(st);
                if (rng.overflow) break;
                const int mr = get_matches<CF>(P, mask, sw, st);  // :176-181
                mark<PH_MATCH>(st);
                if (mr == MATCH_OVERFLOW) {
                    flags |= FLAG_GROUP_OVERFLOW;
                    return CAS_DONE;
                }
                if (mr != MATCH_FOUND) break;
                Bd z = mask | VALID.andnot(tb_nonzero<CF>(P));  // :199 + TB==0 cells
                z = fire_specials<CF, 6>(P, z, dm);
                reward += score<CF, 6>(P, z);
                merge_clip<CF, 6>(P, z, sw);
                mark<PH_CLEAR>(st);
            }
            }
            if (rng.overflow) break;
            if constexpr ((OPTS & CASX_STOP_SETTLED) != 0) return CAS_SETTLED;
        }
        settled = false;
        // no match left: the legal set of the settled board, computed once
        // after the (divergent) cascade so the wave runs it once
        legal_masks<CF>(P, special_mask<CF, 6>(P), HL, VL, dm);
        mark<PH_LEGAL>(st);
        if (HL.any() || VL.any()) break;
        if constexpr ((OPTS & CASX_STOP_DEAD) != 0) return CAS_DEAD;
        int shuffles = 0;                                       // :188-194 dead board
        while (!found && !(HL.any() || VL.any())) {
            if (shuffles >= CF::SHUFFLE_CAP) {
                flags |= FLAG_SHUFFLE_CAP;
                break;
            }
            shuffle_rows<CF>(P, rng, dm);
            flags |= FLAG_SHUFFLED;
            ++shuffles;
            const int mr = get_matches<CF>(P, mask, sw, st);
            if (mr == MATCH_OVERFLOW) {
                flags |= FLAG_GROUP_OVERFLOW;
                return CAS_DONE;
            }
            found = mr == MATCH_FOUND;
            if (!found) legal_masks<CF>(P, special_mask<CF, 6>(P), HL, VL, dm);
        }
        if (!found) break;                                      // :195-196
        Bd z = mask | VALID.andnot(tb_nonzero<CF>(P));         // :199 + TB==0 cells
        z = fire_specials<CF, 6>(P, z, dm);
        reward += score<CF, 6>(P, z);
        merge_clip<CF, 6>(P, z, sw);
        mark<PH_CLEAR>(st);
    }
    if (rng.overflow) flags |= FLAG_RNG_OVERFLOW;
    return CAS_DONE;
}

// true when the step is finished (HL/VL set, or flagged for recompute),
// false when paused (see apply_begin)
template <class CF, class RNG, class Store>
M3_HD bool apply_cascade(typename CF::Bd* P, RNG& rng, uint32_t& flags, typename CF::Bd& HL,
                         typename CF::Bd& VL, Store& st, int& reward, int limit,
                         const typename CF::Dim& dm = typename CF::Dim{}) {
    return apply_cascade_ex<CF, 0>(P, rng, flags, HL, VL, st, reward, limit, false, dm) != CAS_PAUSED;
}

// A paused cascade's live state as Cont<CF, RNG>::WORDS 32-bit words: planes
// 0..5, the RNG struct, reward, flags. put(i, w) / get(i) choose the memory
// layout (the env kernel writes them SoA, one word column per index).
template <class CF, class RNG>
struct Cont {
    static_assert(std::is_trivially_copyable<RNG>::value && sizeof(RNG) % 4 == 0, "RNG state must be words");
    static constexpr int PW = 6 * CF::W;
    static constexpr int RW = (int)(sizeof(RNG) / 4);
    static constexpr int WORDS = PW + RW + 2;
    template <class Put>
    static M3_HD void save(const typename CF::Bd* P, const RNG& rng, int reward, uint32_t flags, Put put) {
#pragma unroll
        for (int p = 0; p < 6; ++p)
#pragma unroll
            for (int i = 0; i < CF::W; ++i) put(p * CF::W + i, P[p].w[i]);
        uint32_t r[RW];
        __builtin_memcpy(r, &rng, sizeof(RNG));
#pragma unroll
        for (int i = 0; i < RW; ++i) put(PW + i, r[i]);
        put(PW + RW, (uint32_t)reward);
        put(PW + RW + 1, flags);
    }
    template <class Get>
    static M3_HD void load(typename CF::Bd* P, RNG& rng, int& reward, uint32_t& flags, Get get) {
#pragma unroll
        for (int p = 0; p < 6; ++p)
#pragma unroll
            for (int i = 0; i < CF::W; ++i) P[p].w[i] = get(p * CF::W + i);
#pragma unroll
        for (int p = 6; p < CF::NP; ++p) P[p] = CF::Bd::zero();
        uint32_t r[RW];
#pragma unroll
        for (int i = 0; i < RW; ++i) r[i] = get(PW + i);
        __builtin_memcpy(&rng, r, sizeof(RNG));
        reward = (int)get(PW + RW);
        flags = get(PW + RW + 1);
    }
};

// Returns the step reward (0 when flags ask for a recompute).
template <class CF, class RNG, class Store>
M3_HD int apply_action(typename CF::Bd* P, int n_actions, int action, RNG& rng, uint32_t& flags,
                       typename CF::Bd& HL, typename CF::Bd& VL, Store& st,
                       const typename CF::Dim& dm = typename CF::Dim{}) {
    int reward;
    if (apply_begin<CF>(P, n_actions, action, rng, flags, HL, VL, st, reward, dm))
        apply_cascade<CF>(P, rng, flags, HL, VL, st, reward, -1, dm);
    return (flags & FLAG_RECOMPUTE) ? 0 : reward;
}

// --------------------------------------------------------------------------
// BoardV2.__init__ with array=None (boardv2.py:17-27). mt must be freshly
// seeded. Writes the planes (values 1..T).
// --------------------------------------------------------------------------
template <class CF, class RNG, class S>
M3_HD void init_board(typename CF::Bd* P, RNG& mt, S& st, const typename CF::Dim& dm = typename CF::Dim{}) {
    using Bd = typename CF::Bd;
#pragma unroll
    for (int p = 0; p < CF::NP; ++p) P[p] = Bd::zero();
    const int RB = dm.rows(), CB = dm.cols();
    const uint32_t tmask = dm.tile_mask(), trng = dm.tile_rng();
    // randint(1, T+1, (R, C)) fills cells in row-major order; as in the
    // refill, one raw draw per loop trip so lanes never wait on each other's
    // rejections. An accepted value belongs to cell (r, c).
    auto fill = [&](const Bd* only) {
        int r = 0, c = 0;
        while (r < RB) {
            uint32_t v = mt.next32() & tmask;
            if (mt.overflow) return;
            if (v > trng) continue;
            v += 1u;
            const int x = r * CF::C + c;
            if (!only || only->test(x)) set_cell<CF, CF::BITS>(P, x, (int)v);
            if (++c == CB) {
                c = 0;
                ++r;
            }
        }
    };
    mark<PH_LOAD>(st);
    fill(nullptr);                                             // :21
    mark<PH_REFILL>(st);
    Bd mask;
    for (;;) {                                                 // :23-27
        if (mt.overflow) break;
        const bool any = get_match_mask<CF>(P, mask);
        mark<PH_MATCH>(st);
        if (!any) break;
        fill(&mask);
        mark<PH_REFILL>(st);
    }
}


// --------------------------------------------------------------------------
// BoardV2.__init__ (boardv2.py:17-27) on a tile stream: every round of the
// reference draws randint(1, T+1, (R, C)), i.e. the next N tiles of the
// stream in row-major order, so a round is "take N tiles as bit-planes" (a
// funnel shift of the stream's plane words) plus one masked merge. The
// stream is generated as it is needed (one raw draw per loop trip, tiles
// appended to plane words in `tm`, plane p word w at tm[(p*TWMAX + w)*stride]).
// Raw outputs k < rawn and their acceptance bits go to the sinks (the
// kernels pass rawn = 0; the host harness uses them to check the stream).
// Returns false if the board needs more than the first kcap draws (at most
// the first MT block, 624): the caller recomputes it. `draws` = raw outputs
// consumed by __init__.
// --------------------------------------------------------------------------
// The stream is kept as a RING of TWMAX plane words (round 6; was the whole 624-tile stream, 21
// words): a round only reads its own N tiles, and every live lane of a wave is at the same round, so
// a lane's unread tiles span about N + one 64-draw chunk + the acceptance spread between lanes (9x9:
// 192 usable tiles in the 10-word ring below are enough for all but a few). A lane whose unread tiles would overrun the ring
// stops (its reset reports the cap: the exact fallback redoes it), so the ring never loses a tile.
// 9x9: 10 words per plane (192 usable tiles; indexed modulo 10): tm 7.5 KB + pos 2.3 KB per wave,
// so more reset waves fit a CU beside the step waves (k_init is LDS-bound). A/B on the driver
// command: 16 words 2.50-2.51, 12 2.53-2.57, 10 2.60, 8 2.25-2.29 G env-steps/s (too small: resets
// overrun the ring and go to the wave-per-board fallback).
template <class CF>
struct TileGen {
#ifndef M3_TW9
#define M3_TW9 10
#endif
    static constexpr int TWMAX = CF::N <= 128 ? M3_TW9 : 32;  // ring words per plane
    static constexpr int MAXR = 624 / CF::N + 2;             // rounds one MT block can feed
    static_assert(TWMAX > CF::W + 1, "a round's read window fits the ring");
    // ring slot of stream word q (a mask for a power of two, else a modulo by a constant)
    static M3_HD uint32_t slot(uint32_t q) {
        if constexpr ((TWMAX & (TWMAX - 1)) == 0) return q & (uint32_t)(TWMAX - 1);
        else return q % (uint32_t)TWMAX;
    }
};


template <class CF, class RNG, class RawSink, class AccSink, class S = NoStore>
M3_HD bool init_board_tiles(typename CF::Bd* P, RNG& g, uint32_t* tm, uint32_t* pos, int stride, uint32_t& draws,
                            uint32_t rawn, RawSink raw_sink, AccSink acc_sink, S* ps = nullptr,
                            uint32_t kcap = 624u) {
    using Bd = typename CF::Bd;
    using G = typename CF::G;
    constexpr int TW = TileGen<CF>::TWMAX, N = CF::N, MAXR = TileGen<CF>::MAXR;
    constexpr Bd VALID = G::valid();
    static_assert(!CF::DYN, "frame boards reset on FullMT (k_init_fix_lane)");
    static_assert(CF::TILE_RNG > 0u, "randint(1, 2) consumes no draws");
    uint32_t cur[CF::BITS];
#pragma unroll
    for (int p = 0; p < CF::BITS; ++p) cur[p] = 0u;
    uint32_t nt = 0u, accw = 0u;
    uint32_t floor_tile = 0u;  // first tile this lane still has to read (its current round's)
    bool ring_full = false;    // the unread tiles would overrun the ring (the reset goes to the fallback)
    constexpr uint32_t RING_TILES = 32u * (uint32_t)(TW - CF::W - 1);  // (take reads W + 1 words)
    // Every lane draws raw outputs [g.k, kend): the trip count is the same on
    // all lanes (one draw per trip), so the MT19937 chain runs without
    // divergence; tiles are appended to the lane's own stream. pos[r] records
    // the raw position after tile r*N - 1 (what __init__ has consumed after r rounds).
    auto gen_to = [&](uint32_t kend) {
        for (uint32_t k = g.k; k < kend; ++k) {
            const uint32_t v = g.next32();
            const uint32_t t = v & CF::TILE_MASK;
            const bool ok = t <= CF::TILE_RNG;
            if (k < rawn) {
                raw_sink(k, v);
                accw |= (uint32_t)ok << (k & 31u);
                if ((k & 31u) == 31u) {
                    acc_sink(k >> 5, accw);
                    accw = 0u;
                }
            }
            if (ok && nt - floor_tile >= RING_TILES) ring_full = true;
            if (ok && !ring_full) {
                const uint32_t val = t + 1u, sh = nt & 31u;
#pragma unroll
                for (int p = 0; p < CF::BITS; ++p) cur[p] |= ((val >> p) & 1u) << sh;
                ++nt;
                if ((nt & 31u) == 0u) {
#pragma unroll
                    for (int p = 0; p < CF::BITS; ++p) {
                        tm[(p * TW + (int)TileGen<CF>::slot((nt >> 5) - 1u)) * stride] = cur[p];
                        cur[p] = 0u;
                    }
                }
                if (nt % (uint32_t)N == 0u && nt / (uint32_t)N < (uint32_t)MAXR) pos[(nt / N) * stride] = k + 1u;
            }
        }
#pragma unroll
        for (int p = 0; p < CF::BITS; ++p)  // the partial word, so a round can read it
            tm[(p * TW + (int)TileGen<CF>::slot(nt >> 5)) * stride] = cur[p];
    };
    // make sure every lane that still needs them has `need` tiles (or the block is exhausted)
    auto ensure = [&](uint32_t need, bool want) {
        while (wave_any(want && !ring_full && nt < need) && g.k < kcap) {
            const uint32_t kend = g.k + 64u < kcap ? g.k + 64u : kcap;
            gen_to(kend);
        }
        return !want || nt >= need;
    };
    auto take = [&](uint32_t j, Bd* T) {  // tiles [j, j + N) as planes
        const uint32_t q = j >> 5;
        const uint32_t sh = j & 31u;
#pragma unroll
        for (int p = 0; p < CF::BITS; ++p) {
            uint32_t lo = tm[(p * TW + (int)TileGen<CF>::slot(q)) * stride];
#pragma unroll
            for (int i = 0; i < CF::W; ++i) {
                const uint32_t hi = tm[(p * TW + (int)TileGen<CF>::slot(q + (uint32_t)i + 1u)) * stride];
                T[p].w[i] = sh ? ((lo >> sh) | (hi << (32u - sh))) : lo;
                lo = hi;
            }
            T[p] &= VALID;
        }
    };
    if constexpr (HasProf<S>::value) ps->template mark<PH_LOAD>();
#pragma unroll
    for (int p = 0; p < CF::NP; ++p) P[p] = Bd::zero();
    bool ok = ensure((uint32_t)N, true);                       // :21
    if (ok) take(0u, P);
    floor_tile = (uint32_t)N;
    if constexpr (HasProf<S>::value) ps->template mark<PH_REFILL>();
    uint32_t rounds = 1u;
    bool live = ok;
    Bd mask;
    for (;;) {                                                 // :23-27
        const bool any = live && get_match_mask<CF>(P, mask);
        if constexpr (HasProf<S>::value) ps->template mark<PH_MATCH>();
        live = any;
        const uint32_t need = (rounds + 1u) * (uint32_t)N;
        const bool have = ensure(need, live);
        if (live && !have) ok = false;
        live = live && have;
        if (!wave_any(live)) break;
        if (live) {
            Bd T[CF::BITS];
            take(rounds * (uint32_t)N, T);
#pragma unroll
            for (int p = 0; p < CF::BITS; ++p) P[p] = P[p].andnot(mask) | (T[p] & mask);
            ++rounds;
            floor_tile = rounds * (uint32_t)N;  // (earlier tiles are never read again)
        } else {
            floor_tile = nt;  // (a finished lane reads nothing more: no ring limit)
        }
        if constexpr (HasProf<S>::value) ps->template mark<PH_REFILL>();
    }
    draws = ok ? pos[rounds * stride] : 0u;
    if (g.k < rawn) gen_to(rawn);  // complete the step's stream cache: raw draws [0, rawn)
    if (rawn & 31u) acc_sink(rawn >> 5, accw);
    if constexpr (HasProf<S>::value) ps->template mark<PH_NEXT>();
    return ok;
}

// --------------------------------------------------------------------------
// planes <-> int8 cells. Eight cells at a time: an 8x8 bit-matrix transpose
// turns 8 bytes (cell-major) into 8 plane bytes (plane-major) and back.
// --------------------------------------------------------------------------
M3_HD void transpose8(uint32_t& lo, uint32_t& hi) {
    uint32_t t;
    t = (lo ^ (lo >> 7)) & 0x00AA00AAu; lo ^= t ^ (t << 7);
    t = (hi ^ (hi >> 7)) & 0x00AA00AAu; hi ^= t ^ (t << 7);
    t = (lo ^ (lo >> 14)) & 0x0000CCCCu; lo ^= t ^ (t << 14);
    t = (hi ^ (hi >> 14)) & 0x0000CCCCu; hi ^= t ^ (t << 14);
    t = (lo ^ (hi << 4)) & 0xF0F0F0F0u; lo ^= t; hi ^= t >> 4;
}

// cells: N bytes as little-endian 32-bit words, cw[q] holds cells 4q..4q+3
template <class CF>
M3_HD void planes_from_words(const uint32_t* cw, typename CF::Bd* P) {
    constexpr int NW = (CF::N + 3) / 4;
#pragma unroll
    for (int p = 0; p < CF::NP; ++p) P[p] = CF::Bd::zero();
#pragma unroll
    for (int g = 0; g < (CF::N + 7) / 8; ++g) {
        uint32_t lo = (2 * g < NW) ? cw[2 * g] : 0u;
        uint32_t hi = (2 * g + 1 < NW) ? cw[2 * g + 1] : 0u;
        transpose8(lo, hi);
        const int q = (8 * g) >> 5, sh = (8 * g) & 31;
#pragma unroll
        for (int p = 0; p < CF::NP; ++p) {
            const uint32_t byte = ((p < 4 ? lo : hi) >> (8 * (p & 3))) & 0xFFu;
            P[p].w[q] |= byte << sh;
        }
    }
    constexpr typename CF::Bd VALID = CF::G::valid();
#pragma unroll
    for (int p = 0; p < CF::NP; ++p) P[p] &= VALID;
}

template <class CF>
M3_HD void words_from_planes(const typename CF::Bd* P, uint32_t* cw) {
    constexpr int NW = (CF::N + 3) / 4;
#pragma unroll
    for (int g = 0; g < (CF::N + 7) / 8; ++g) {
        const int q = (8 * g) >> 5, sh = (8 * g) & 31;
        uint32_t lo = 0u, hi = 0u;
#pragma unroll
        for (int p = 0; p < CF::NP; ++p) {
            const uint32_t byte = (P[p].w[q] >> sh) & 0xFFu;
            if (p < 4) lo |= byte << (8 * p);
            else hi |= byte << (8 * (p - 4));
        }
        transpose8(lo, hi);
        if (2 * g < NW) cw[2 * g] = lo;
        if (2 * g + 1 < NW) cw[2 * g + 1] = hi;
    }
}


// --------------------------------------------------------------------------
// Frame boards (FCfg) <-> the board's own int8 cells (R*C bytes, row-major,
// any alignment): board row r is C bytes, cells (r, 0..C-1) sit at frame
// bits r*FS .. r*FS + C-1; one 8x8 transpose per 8 cells of a row.
// --------------------------------------------------------------------------
// a frame row's bits (r compile-time in the unrolled callers)
template <class CF>
M3_HD uint32_t frame_row(const typename CF::Bd& b, int r) {
    if constexpr (CF::FS == 16) return (b.w[r >> 1] >> ((r & 1) * 16)) & 0xFFFFu;
    else return b.w[r];
}
// bits m of frame row r := the same bits of v
template <class CF>
M3_HD void frame_row_merge(typename CF::Bd& b, int r, uint32_t v, uint32_t m) {
    if constexpr (CF::FS == 16) {
        const int sh = (r & 1) * 16;
        b.w[r >> 1] = (b.w[r >> 1] & ~(m << sh)) | ((v & m) << sh);
    } else {
        b.w[r] = (b.w[r] & ~m) | (v & m);
    }
}

template <class CF>
M3_HD void frame_from_bytes(const uint8_t* src, typename CF::Bd* P, const typename CF::Dim& dm) {
    static_assert(CF::DYN, "frame layout");
    constexpr int FS = CF::FS, NG = FS / 8;  // 8-cell groups per row
    const int RB = dm.rows(), CB = dm.cols();
#pragma unroll
    for (int p = 0; p < CF::NP; ++p) P[p] = CF::Bd::zero();
#pragma unroll
    for (int r = 0; r < CF::R; ++r) {
        if (r < RB) {
            const uint8_t* row = src + r * CB;
            uint32_t w[2 * NG];
#pragma unroll
            for (int k = 0; k < 2 * NG; ++k) w[k] = 0u;
#pragma unroll
            for (int k = 0; k < FS; ++k)
                if (k < CB) w[k >> 2] |= (uint32_t)row[k] << (8 * (k & 3));
#pragma unroll
            for (int g = 0; g < NG; ++g) transpose8(w[2 * g], w[2 * g + 1]);
#pragma unroll
            for (int p = 0; p < CF::NP; ++p) {
                uint32_t v = 0u;
#pragma unroll
                for (int g = 0; g < NG; ++g) v |= ((w[2 * g + (p < 4 ? 0 : 1)] >> (8 * (p & 3))) & 0xFFu) << (8 * g);
                frame_row_merge<CF>(P[p], r, v, 0xFFFFFFFFu >> (32 - FS));
            }
        }
    }
}

template <class CF>
M3_HD void frame_to_bytes(const typename CF::Bd* P, uint8_t* dst, const typename CF::Dim& dm) {
    static_assert(CF::DYN, "frame layout");
    constexpr int FS = CF::FS, NG = FS / 8;
    const int RB = dm.rows(), CB = dm.cols();
#pragma unroll
    for (int r = 0; r < CF::R; ++r) {
        if (r < RB) {
            uint32_t w[2 * NG];
#pragma unroll
            for (int k = 0; k < 2 * NG; ++k) w[k] = 0u;
#pragma unroll
            for (int p = 0; p < CF::NP; ++p) {
                const uint32_t bits = frame_row<CF>(P[p], r);
#pragma unroll
                for (int g = 0; g < NG; ++g) w[2 * g + (p < 4 ? 0 : 1)] |= ((bits >> (8 * g)) & 0xFFu) << (8 * (p & 3));
            }
#pragma unroll
            for (int g = 0; g < NG; ++g) transpose8(w[2 * g], w[2 * g + 1]);
            uint8_t* row = dst + r * CB;
#pragma unroll
            for (int k = 0; k < FS; ++k)
                if (k < CB) row[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
        }
    }
}

// One round of BoardV2.__init__ on a frame board (boardv2.py:21 / :25):
// randint(1, T+1, (R, C)) draws a tile for EVERY cell in row-major order;
// cells outside `only` take their draw and drop it (array[mask] = new[mask]).
template <class CF, class RNG>
M3_HD void fill_round_frame(typename CF::Bd* P, RNG& mt, const typename CF::Bd* only, const typename CF::Dim& dm) {
    const int RB = dm.rows(), CB = dm.cols();
    const uint32_t tmask = dm.tile_mask(), trng = dm.tile_rng(), rowm = low_bits(CB);
#pragma unroll
    for (int r = 0; r < CF::R; ++r) {
        if (r < RB) {
            uint32_t t[CF::BITS];
#pragma unroll
            for (int p = 0; p < CF::BITS; ++p) t[p] = 0u;
            for (int c = 0; c < CB; ++c) {
                uint32_t v;
                do {
                    v = mt.next32() & tmask;
                } while (v > trng);
                v += 1u;
#pragma unroll
                for (int p = 0; p < CF::BITS; ++p) t[p] |= ((v >> p) & 1u) << c;
            }
            const uint32_t m = only ? frame_row<CF>(*only, r) & rowm : rowm;
#pragma unroll
            for (int p = 0; p < CF::BITS; ++p) frame_row_merge<CF>(P[p], r, t[p], m);
        }
    }
}

}  // namespace m3
