// asan_main.hip -- TEST INFRASTRUCTURE ONLY: the device rule code's host build
// (hostcore.hip: m3_rules.hpp / m3_bitboard.hpp / m3_rng.hpp compiled for the
// CPU) under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5
// sanitizer row). Every hostcore entry point runs over the specialised shapes
// and frame shapes (tiny, columns = 3, rows > columns, 16 types) on seeded
// boards with sprinkled specials, typed values and holes, every action id (legal
// or not, plus out-of-range ids), the tiny group tables that force the
// overflow fallback, and the paused/resumed cascade. The small-table and
// paused runs must also agree with the plain run. Built and run by
// tests/test_sanitizers_cpu.py; any sanitizer report exits non-zero.
#include "hostcore.hip"

#include <stdio.h>
#include <stdlib.h>

#include <vector>

static constexpr int FRAME = 2;  // any shape in the 16 x 16 frame (hc_set_frame), as hostcore.py

static uint32_t lcg(uint32_t* s) {
    *s = *s * 1664525u + 1013904223u;
    return *s >> 8;
}

static int fail(const char* what, int cfg, long i) {
    fprintf(stderr, "mismatch: %s (cfg %d, item %ld)\n", what, cfg, i);
    return 1;
}

// one configuration: cfg id (0, 1 or FRAME after hc_set_frame), board R x C, T types, BITS
static int run(int cfg, int R, int C, int T, int BITS, uint32_t& rs, long& checks) {
    const long n = getenv("HC_N") ? atol(getenv("HC_N")) : 96;  // (the MemorySanitizer run uses fewer)
    const int N = R * C, A = R * (C - 1) * 2, AW = (A + 31) / 32;
    const int TM = (1 << BITS) - 1, H = TM + 1, V = 2 * H, STM = (1 << (BITS + 1)) + 1 + TM, M = TM + STM + 1;
    std::vector<uint32_t> seeds(n), m397(n);
    std::vector<int8_t> boards(n * N), out(n * N), out2(n * N);
    std::vector<int32_t> draws(n), first(n), na(n), act(n), rew(n), rew2(n), d2(n), fl(n), fl2(n), nx(n), nx2(n);
    std::vector<uint32_t> legal(n * AW), legal2(n * AW);
    for (long i = 0; i < n; ++i) seeds[i] = lcg(&rs) * 977u + 1u;
    hc_init(cfg, n, seeds.data(), boards.data(), draws.data(), m397.data(), first.data());
    std::vector<int32_t> dsc(n);
    std::vector<int8_t> bsc(n * N);
    hc_init_scalar(cfg, n, seeds.data(), bsc.data(), dsc.data());
    for (long i = 0; i < n * N; ++i)
        if (bsc[i] != boards[i]) return fail("init: tile stream vs scalar", cfg, i / N);
    const int vals[] = {H, V, STM, M, H | 3, V | 3, STM | 3, 0, M + 8, 127};
    for (long i = 0; i < n * N; ++i)
        if (lcg(&rs) % 100 < 6) boards[i] = (int8_t)vals[lcg(&rs) % 10];
    for (long i = 0; i < n; ++i) {
        na[i] = (int32_t)(lcg(&rs) % 22);  // includes terminal boards (n_actions 0)
        const uint32_t r = lcg(&rs) % 100;
        act[i] = r < 3 ? -1 : (r < 6 ? A + (int)(lcg(&rs) % 7) : (int)(lcg(&rs) % A));
    }
    hc_apply(cfg, n, boards.data(), seeds.data(), na.data(), act.data(), out.data(), rew.data(), draws.data(),
             fl.data(), legal.data(), nx.data(), 0);
    for (int small : {1, 4, 8, 32}) {
        hc_apply(cfg, n, boards.data(), seeds.data(), na.data(), act.data(), out2.data(), rew2.data(), d2.data(),
                 fl2.data(), legal2.data(), nx2.data(), small);
        for (long i = 0; i < n; ++i) {
            if (rew[i] != rew2[i] || d2[i] != draws[i] || nx[i] != nx2[i]) return fail("small table", cfg, i);
            for (int x = 0; x < N; ++x)
                if (out[i * N + x] != out2[i * N + x]) return fail("small table board", cfg, i);
        }
    }
    for (int pause = 0; pause < 3; ++pause) {  // the k_env_step -> k_env_cont hand-over (specialised only)
        if (cfg == FRAME) break;
        hc_apply(cfg, n, boards.data(), seeds.data(), na.data(), act.data(), out2.data(), rew2.data(), d2.data(),
                 fl2.data(), legal2.data(), nx2.data(), 100 + pause);
        for (long i = 0; i < n; ++i)
            if (rew[i] != rew2[i] || nx[i] != nx2[i]) return fail("paused cascade", cfg, i);
    }
    std::vector<uint8_t> mask(n * N);
    std::vector<int32_t> spawn(n * N), found(n);
    hc_matches(cfg, n, out.data(), mask.data(), spawn.data(), found.data());
    hc_legal(cfg, n, out.data(), legal2.data());
    for (long i = 0; i < n * AW; ++i)
        if (legal[i] != legal2[i]) return fail("legal vs stateless legal", cfg, i / AW);
    hc_roundtrip(cfg, n, boards.data(), out2.data());
    std::vector<int32_t> rounds(n);
    hc_rounds(cfg, n, boards.data(), seeds.data(), na.data(), act.data(), rounds.data());
    for (int k = 0; k < 700; k += 37) (void)hc_chain_draw(seeds[k % n], k);
    {   // MCTS.rollout as k_rollout's rollout_one composes the rules (the round-4/5 lane-interference
        // path): 1 and 20 moves from the stepped boards; n_actions 1 must equal the one step + choice
        std::vector<uint32_t> rsd(n), dr(n), fg(n);
        std::vector<int32_t> gain(n), steps(n);
        for (long i = 0; i < n; ++i) rsd[i] = lcg(&rs);
        for (int k : {1, 20}) {
            std::vector<int32_t> nk(n, k);
            hc_rollout(cfg, n, out.data(), seeds.data(), nk.data(), rsd.data(), gain.data(), steps.data(), dr.data(),
                       fg.data());
            for (long i = 0; i < n; ++i)
                if (gain[i] >= 0 && steps[i] > k) return fail("rollout steps", cfg, i);
        }
    }
    checks += n;
    return 0;
}

int main() {
    uint32_t rs = 2024u;
    long checks = 0;
    if (run(0, 9, 9, 6, 3, rs, checks)) return 1;
    if (run(1, 16, 16, 8, 4, rs, checks)) return 1;
    static const int frames[][3] = {{3, 3, 3}, {5, 3, 3}, {7, 7, 4}, {10, 8, 5}, {12, 12, 7}, {16, 3, 4},
                                    {6, 5, 15}, {9, 9, 2}, {9, 9, 6}, {10, 8, 9}};
    for (const auto& f : frames) {
        if (hc_set_frame(f[0], f[1], f[2]) != 0) return 1;
        int bits = 0;
        while ((1 << bits) <= f[2]) ++bits;
        if (run(FRAME, f[0], f[1], f[2], bits, rs, checks)) return 1;
        printf("frame %dx%dx%d done\n", f[0], f[1], f[2]);
        fflush(stdout);
    }
    printf("hostcore asan: %ld boards through every entry point, no sanitizer report\n", checks);
    return 0;
}
