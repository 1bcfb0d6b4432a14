/*
 * m3_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Scalar C restatement of the reference hot path (ThorLL/Element-Crush-Gym,
 * match3tile/boardv2.py + match3tile/boardFunctions.py + numpy's legacy
 * RandomState). It is the *checker* for the HIP path: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product library (libm3.so) never links or calls it.
 *
 * Parity of this oracle is pinned by golden vectors generated from the real
 * reference in this container (tests/golden/gen_golden.py).
 */
#ifndef M3_ORACLE_H
#define M3_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* numpy legacy MT19937 (numpy/random/src/mt19937/mt19937.c, legacy seeding). */
typedef struct {
    uint32_t key[624];
    int pos;
    int64_t draws; /* raw u32 outputs consumed since the last seed() */
} m3o_mt;

void     m3o_mt_seed(m3o_mt *mt, uint32_t seed);
uint32_t m3o_mt_next32(m3o_mt *mt);
/* RandomState.randint(low, high) for one element (legacy masked rejection). */
int64_t  m3o_randint(m3o_mt *mt, int64_t low, int64_t high);
/* random_interval(max): used by the legacy shuffle. */
uint64_t m3o_random_interval(m3o_mt *mt, uint64_t max);

/* BoardConfig (match3tile/boardConfig.py:5-43). */
typedef struct {
    int R, C, T;
    int TM, STM, H, V, B, M, A;
} m3o_cfg;

void m3o_cfg_init(m3o_cfg *cfg, int rows, int columns, int types);
void m3o_decode(const m3o_cfg *cfg, int action, int *r1, int *c1, int *r2, int *c2);
int  m3o_encode(const m3o_cfg *cfg, int r1, int c1, int r2, int c2);

/* Flags (mirrors include/m3.h). */
#define M3O_FLAG_TERMINAL     0x01
#define M3O_FLAG_BAD_ACTION   0x02
#define M3O_FLAG_SHUFFLE_CAP  0x04
#define M3O_FLAG_NO_LEGAL     0x08
#define M3O_FLAG_SHUFFLED     0x10

/* get_matches (boardFunctions.py:121-156) mask only; returns number of groups. */
int m3o_get_matches(const m3o_cfg *cfg, const int32_t *tb, uint8_t *mask);
/* get_match_spawn_mask over get_matches groups; returns number of groups. */
int m3o_matches_and_spawn(const m3o_cfg *cfg, const int32_t *tb, uint8_t *mask, int32_t *spawn);
/* legal_actions (boardFunctions.py:26-112); returns count, writes ascending ids. */
int m3o_legal_actions(const m3o_cfg *cfg, const int32_t *board, int32_t *out_actions);

/* BoardV2.__init__ with array=None (boardv2.py:17-27). Returns raw draws. */
int64_t m3o_init_board(const m3o_cfg *cfg, uint32_t seed, int32_t *board, m3o_mt *mt);

/* BoardV2.apply_action (boardv2.py:43-207). `mt` is numpy's global RNG; it is
 * reseeded with `seed` exactly as the reference does. Returns the step reward;
 * *flags gets M3O_FLAG_*; on return mt->draws = draws since the last reseed. */
int64_t m3o_apply_action(const m3o_cfg *cfg, uint32_t seed, int n_actions,
                         const int32_t *board, int action, int32_t *out_board,
                         m3o_mt *mt, int *flags, int shuffle_cap);

/* samplerTasks.random_task (samplerTasks.py:9-14) generalised to the
 * Match3Env bookkeeping (env.py:48-56): init, reseed, then per move
 * choice(legal) -> apply_action. Writes per-move actions/rewards/draws and the
 * final board. Returns number of moves executed. */
void m3o_set_episode_shuffle_cap(int cap);
int m3o_random_episode(const m3o_cfg *cfg, uint32_t seed, int num_moves, int env_goal,
                       int32_t *actions, int32_t *rewards, int32_t *draws,
                       uint8_t *done, int32_t *final_board, int *flags);

/* Threaded: n seeded episodes with every per-move output kept
 * (actions/rewards/draws/done are [n][num_moves], final_boards [n][R*C]). */
void m3o_batch_episodes(const m3o_cfg *cfg, int64_t n, const uint32_t *seeds, int num_moves, int env_goal,
                        int nthreads, int32_t *actions, int32_t *rewards, int32_t *draws, uint8_t *done,
                        int32_t *final_boards, int32_t *moves_out, int32_t *flags_out);

/* MCTS.rollout (mctslib/standard/mcts.py:14-19) from state (board, seed = cfg.seed,
 * n_actions): np.random.seed(rollout_seed); while n_actions >= 1: action =
 * choice(legal_actions) on the global stream; board = apply_action(action).
 * Writes the terminal board (nullable), the step count, the global stream's
 * draws since its last seed and the OR of the step flags; returns the summed
 * step rewards (the rollout's return minus state.reward). */
int64_t m3o_rollout(const m3o_cfg *cfg, const int32_t *board, uint32_t seed, int n_actions,
                    uint32_t rollout_seed, int32_t *final_board, int *steps, int64_t *draws, int *flags);

/* Threaded: n rollouts (boards [n][R*C]); gain/steps/draws/flags [n], final [n][R*C] nullable. */
void m3o_batch_rollouts(const m3o_cfg *cfg, int64_t n, const int32_t *boards, const uint32_t *seeds,
                        const int32_t *n_actions, const uint32_t *rollout_seeds, int nthreads,
                        int32_t *gain, int32_t *steps, int64_t *draws, int32_t *flags, int32_t *final_boards);

/* Threaded CPU baseline: run n episodes (seeds[i]) of num_moves moves with
 * random actions; returns total env steps; writes per-episode total reward. */
int64_t m3o_run_episodes(const m3o_cfg *cfg, int64_t n, const uint32_t *seeds,
                         int num_moves, int env_goal, int nthreads, int64_t *out_total);

#ifdef __cplusplus
}
#endif
#endif
