/*
 * asan_main.c -- TEST INFRASTRUCTURE ONLY: the C oracle under AddressSanitizer +
 * UndefinedBehaviorSanitizer (SURVEY.md §5 sanitizer row). Drives every oracle
 * entry point over many board shapes (tiny, columns = 3, rows > columns,
 * 16x16) with seeded boards, sprinkled specials / typed values / holes, every
 * action id (legal or not, plus out-of-range ids), episodes and rollouts.
 * Built by `make -C oracle asan`, run by tests/test_sanitizers_cpu.py; any
 * sanitizer report makes the process exit non-zero.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "m3_oracle.h"

static uint32_t lcg(uint32_t *s) {
    *s = *s * 1664525u + 1013904223u;
    return *s >> 8;
}

int main(void) {
    static const int shapes[][3] = {{3, 3, 3}, {5, 3, 3}, {4, 4, 3}, {7, 7, 4}, {10, 8, 5}, {9, 9, 6},
                                    {12, 12, 7}, {16, 3, 4}, {6, 5, 15}, {16, 16, 8}};
    uint32_t rs = 12345u;
    long checks = 0;
    m3o_set_episode_shuffle_cap(1024);
    for (size_t si = 0; si < sizeof(shapes) / sizeof(shapes[0]); ++si) {
        m3o_cfg cfg;
        m3o_cfg_init(&cfg, shapes[si][0], shapes[si][1], shapes[si][2]);
        const int N = cfg.R * cfg.C;
        int32_t *board = malloc(sizeof(int32_t) * N), *out = malloc(sizeof(int32_t) * N);
        int32_t *legal = malloc(sizeof(int32_t) * (cfg.A + 1));
        uint8_t *mask = malloc(N);
        int32_t *spawn = malloc(sizeof(int32_t) * N);
        const int specials[] = {cfg.H, cfg.V, cfg.B, cfg.M, 0, cfg.H + 1, cfg.M + 3 > 127 ? 127 : cfg.M + 3};
        for (int it = 0; it < 60; ++it) {
            const uint32_t seed = lcg(&rs) | 1u;
            m3o_mt mt;
            m3o_init_board(&cfg, seed, board, &mt);
            for (int k = 0; k < N; ++k)
                if (lcg(&rs) % 100 < 7) board[k] = specials[lcg(&rs) % 7];
            m3o_legal_actions(&cfg, board, legal);
            m3o_matches_and_spawn(&cfg, board, mask, spawn);
            for (int a = -1; a <= cfg.A; a += (cfg.A > 60 ? 7 : 1)) {
                int f = 0;
                m3o_apply_action(&cfg, seed, 20, board, a, out, &mt, &f, 1024);
                ++checks;
            }
            int f = 0;
            m3o_apply_action(&cfg, seed, 0, board, 0, out, &mt, &f, 1024);  // terminal
            int r1, c1, r2, c2;
            for (int a = 0; a < cfg.A; ++a) m3o_decode(&cfg, a, &r1, &c1, &r2, &c2);
        }
        enum { E = 24, MV = 20 };
        uint32_t seeds[E];
        for (int i = 0; i < E; ++i) seeds[i] = lcg(&rs) | 1u;
        int32_t *acts = malloc(sizeof(int32_t) * E * MV), *rews = malloc(sizeof(int32_t) * E * MV);
        int32_t *drws = malloc(sizeof(int32_t) * E * MV), *fin = malloc(sizeof(int32_t) * E * N);
        uint8_t *dn = malloc(E * MV);
        int32_t moves[E], flg[E];
        m3o_batch_episodes(&cfg, E, seeds, MV, 300, 2, acts, rews, drws, dn, fin, moves, flg);
        int32_t nact[E], gain[E], steps[E];
        int64_t draws[E];
        for (int i = 0; i < E; ++i) nact[i] = (int32_t)(lcg(&rs) % 21);
        m3o_batch_rollouts(&cfg, E, fin, seeds, nact, seeds, 2, gain, steps, draws, flg, fin);
        int64_t tot[E];
        m3o_run_episodes(&cfg, E, seeds, MV, 500, 2, tot);
        free(acts); free(rews); free(drws); free(fin); free(dn);
        free(board); free(out); free(legal); free(mask); free(spawn);
    }
    printf("asan oracle ok: %ld apply_action calls\n", checks);
    return 0;
}
