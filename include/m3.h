/*
 * m3.h -- C ABI of libm3.so, the MI355X-native batched Match3 env step.
 *
 * Plain C types only (no torch, no HIP types): the reference is Python, and a
 * Python maintainer binds this with ctypes. Every entry
 * point names the reference interface it replaces (paths relative to the
 * ThorLL/Element-Crush-Gym checkout).
 *
 * Conventions
 *   - Return value: 0 (M3_OK) on success, a negative M3_ERR_* code otherwise;
 *     m3_last_error() then returns a thread-local message.
 *   - Boards are int8 row-major [n][rows][columns], cell values in [0, 127]
 *     (the reference stores int64; every value reachable from env play or
 *     dataset.py's type_switch fits).
 *   - Legal-action bitsets are uint32 words [n][ceil(A/32)], bit a = action a
 *     (A = rows*(columns-1)*2, ids as BoardConfig.decode, boardConfig.py:45-59).
 *   - "draws" = raw MT19937 outputs consumed since the last reseed, i.e. numpy's
 *     global RandomState after the call equals seed(cfg.seed) advanced by draws
 *     (boardv2.py:46, boardFunctions.py:17) -- the facade uses it to keep the
 *     reference's global-RNG side effect.
 *   - All calls on one context are serialised on that context's HIP stream;
 *     use one context per host thread. Host-buffer calls block until done.
 *   - No CPU fallback: on a machine without a usable gfx950 device, context
 *     creation fails with M3_ERR_NO_DEVICE.
 */
#ifndef M3_H
#define M3_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define M3_ABI_VERSION 1

#define M3_OK 0
#define M3_ERR_INVALID (-1)     /* bad argument */
#define M3_ERR_UNSUPPORTED (-2) /* board shape not compiled in */
#define M3_ERR_HIP (-3)         /* HIP runtime error */
#define M3_ERR_RCCL (-4)        /* RCCL error */
#define M3_ERR_NO_DEVICE (-5)   /* no usable GPU */
#define M3_ERR_STATE (-6)       /* call out of order (e.g. step before reset) */
#define M3_ERR_CAP (-7)         /* a safety cap stopped a reset the reference would keep running (see flags) */

/* Per-board flags (uint32 out_flags). */
#define M3_FLAG_TERMINAL 0x01u    /* n_actions < 1: board returned unchanged (boardv2.py:44-45) */
#define M3_FLAG_BAD_ACTION 0x02u  /* action id not in [0, A): reference raises KeyError (boardv2.py:48) */
#define M3_FLAG_SHUFFLE_CAP 0x04u /* dead-board shuffle cycled past the cap: reference hangs (boardv2.py:188-194) */
#define M3_FLAG_NO_LEGAL 0x08u    /* no legal action to sample: reference raises in np.random.choice */
#define M3_FLAG_SHUFFLED 0x10u    /* the dead-board shuffle ran */
#define M3_FLAG_CASCADE_CAP 0x100u /* cascade stopped after 65536 refills: the reference keeps going (types = 2 boards) */
#define M3_FLAG_RESET_CAP 0x200u   /* reset stopped after 16384 redraw rounds: the reference keeps going (large types = 2 boards) */

typedef struct m3_ctx m3_ctx;
typedef struct m3_env m3_env;

int m3_abi_version(void);
const char *m3_last_error(void);
/* Number of visible HIP devices (0 when none). Never initialises a context. */
int m3_device_count(int *out_count);
/* 1 if kernels for BoardConfig(rows, columns, types) are compiled in, else 0. */
int m3_supported(int rows, int columns, int types);
/* Action-space size and bitset words for a shape (BoardConfig.action_space, boardConfig.py:27). */
int m3_action_space(int rows, int columns, int *out_actions, int *out_words);

/* One context per (device, board shape): owns a HIP stream and scratch. */
int m3_ctx_create(int device, int rows, int columns, int types, m3_ctx **out);
int m3_ctx_destroy(m3_ctx *ctx);
int m3_ctx_synchronize(m3_ctx *ctx);

/* Device memory on the context's device, through the HIP runtime libm3 itself
 * runs on (host tools and benches need no second runtime, e.g. torch, in the
 * process). m3_dev_copy blocks; kind 1 = host to device, 2 = device to host. */
int m3_dev_alloc(m3_ctx *ctx, int64_t bytes, void **out);
int m3_dev_free(m3_ctx *ctx, void *ptr);
int m3_dev_copy(m3_ctx *ctx, void *dst, const void *src, int64_t bytes, int kind);

/* ---- stateless batch calls on host buffers (BoardV2 facade) ------------- */

/* BoardV2(n_actions, cfg) with array=None: seeded initial board (boardv2.py:17-27).
 * out_first_action: np.random.seed(cfg.seed); np.random.choice(legal_actions)
 * (samplerTasks.py:11-13), -1 if the board has no legal action. Nullable outs. */
int m3_init_boards(m3_ctx *ctx, int64_t n, const uint32_t *seeds, int8_t *out_boards,
                   uint32_t *out_draws, int32_t *out_first_action);
/* The same, with out_flags[i] (nullable): M3_FLAG_RESET_CAP when reset i stopped after 16384 redraw
 * rounds (large types = 2 boards; the reference keeps drawing), M3_FLAG_NO_LEGAL when it has no legal
 * action. m3_init_boards itself returns M3_ERR_CAP (outputs written) if any reset hit the cap. */
int m3_init_boards_ex(m3_ctx *ctx, int64_t n, const uint32_t *seeds, int8_t *out_boards,
                      uint32_t *out_draws, int32_t *out_first_action, uint32_t *out_flags);

/* BoardV2.apply_action (boardv2.py:43-207) for n independent (board, seed,
 * n_actions, action) tuples. out_next_action = choice(legal_actions(next))
 * drawn from the stream where apply_action left it (samplerTasks.py:12-13).
 * out_legal_bits / out_next_action are nullable. */
int m3_apply_actions(m3_ctx *ctx, int64_t n, const int8_t *boards, const uint32_t *seeds,
                     const int32_t *n_actions, const int32_t *actions, int8_t *out_boards,
                     int32_t *out_reward, uint32_t *out_draws, uint32_t *out_flags,
                     uint32_t *out_legal_bits, int32_t *out_next_action);

/* legal_actions(cfg, board) (boardFunctions.py:26-112) as bitsets. */
int m3_legal_actions(m3_ctx *ctx, int64_t n, const int8_t *boards, uint32_t *out_legal_bits);

/* ---- batched MCTS rollouts (mctslib/standard/mcts.py:14-19) ------------- */

/* MCTS.rollout(state) for n independent states (board, cfg.seed, n_actions):
 * np.random.seed(rollout_seeds[i]); while n_actions >= 1: action =
 * np.random.choice(legal_actions); state = state.apply_action(action).
 * The first choice reads rollout_seeds[i]'s stream, later ones the stream
 * apply_action left (cfg.seed + draws), exactly as the reference's global RNG.
 * out_gain = sum of the step rewards (rollout return = state.reward + gain),
 * out_steps = apply_action calls, out_draws = raw draws of the global stream
 * since its last seed at the end (seed = cfg.seed if out_steps > 0, else
 * rollout_seeds[i]), out_flags = OR of the steps' M3_FLAG_* (M3_FLAG_NO_LEGAL:
 * the reference raises in np.random.choice; the rollout stops there).
 * out_boards (nullable) = terminal boards. Host buffers; blocks until done. */
int m3_rollouts(m3_ctx *ctx, int64_t n, const int8_t *boards, const uint32_t *seeds,
                const int32_t *n_actions, const uint32_t *rollout_seeds, int32_t *out_gain,
                int32_t *out_steps, uint32_t *out_draws, uint32_t *out_flags, int8_t *out_boards);
/* Same on device buffers, enqueued on the context stream (no sync). Inputs
 * must stay valid until the stream reaches the launch. */
int m3_rollouts_device(m3_ctx *ctx, int64_t n, const int8_t *boards, const uint32_t *seeds,
                       const int32_t *n_actions, const uint32_t *rollout_seeds, int32_t *out_gain,
                       int32_t *out_steps, uint32_t *out_draws, uint32_t *out_flags, int8_t *out_boards);

/* ---- device-resident batched env: n x Match3Env (env.py:8-65) ----------- */

/* num_moves / env_goal as Match3Env(num_moves=20, env_goal=500) (env.py:15-16). */
int m3_env_create(m3_ctx *ctx, int64_t n, int num_moves, int env_goal, m3_env **out);
int m3_env_destroy(m3_env *env);

/* Match3Env.reset (env.py:58-65) for every board. seeds: host uint32[n], or
 * NULL for seeds seed_base + i. Draws each board's first seeded random action. */
int m3_env_reset(m3_env *env, const uint32_t *seeds, uint32_t seed_base);

/* Split the boards into nshards (1..8) contiguous shards, each stepped on its
 * own HIP stream (plus one prefetch stream per shard for the autoreset
 * launches). Results do not depend on it. Default: 1. Each shard adds two
 * streams; with GPU_MAX_HW_QUEUES >= 8 in the process, 2 shards are fastest
 * (the shards' step kernels fill each other's tails); with HIP's default 4
 * queues, 1. */
int m3_env_set_shards(m3_env *env, int nshards);
/* Wait for all work of the env (every shard stream). */
int m3_env_synchronize(m3_env *env);

/* After a step, boards that are done are reset in place with seed += stride
 * (gymnasium vector-env autoreset; same-step semantics). Default: off. */
int m3_env_set_autoreset(m3_env *env, int enabled, uint32_t seed_stride);

/* Match3Env.step (env.py:48-56) on every board. actions: host int32[n], or
 * NULL to play each board's seeded env.board.random_action() (README.md:23,
 * samplerTasks.py:13) drawn on device at the end of the previous step.
 * Host actions are copied into pinned staging before the call returns (the
 * caller may reuse `actions` at once) and uploaded on a stream of their own;
 * the call blocks at most until the upload of two steps earlier is done. */
int m3_env_step(m3_env *env, const int32_t *actions);
/* Same with actions already in device memory (int32[n]); NULL = random. */
int m3_env_step_device(m3_env *env, const int32_t *d_actions);

/* What to copy out. */
#define M3_ENV_BOARDS 0      /* int8  [n][rows*columns]  observation (env.py:56) */
#define M3_ENV_REWARD 1      /* int32 [n]  reward of the last step           */
#define M3_ENV_DONE 2        /* uint8 [n]  done (env.py:54)                  */
#define M3_ENV_TRUNCATED 3   /* uint8 [n]  truncated: score >= env_goal (env.py:53) */
#define M3_ENV_SCORE 4       /* int32 [n]  episode score                      */
#define M3_ENV_MOVES 5       /* int32 [n]  moves taken in the episode         */
#define M3_ENV_FLAGS 6       /* uint32[n]  M3_FLAG_* of the last step         */
#define M3_ENV_NEXT_ACTION 7 /* int32 [n]  pre-drawn seeded random action     */
#define M3_ENV_LEGAL 8       /* uint32[n][words] legal bitset of the current board (derived: m3_env_get
                                computes it from the boards; after m3_env_device_ptr of this field every
                                step writes it, for device consumers) */
#define M3_ENV_SEEDS 9       /* uint32[n]  current episode seed               */
#define M3_ENV_DRAWS 10      /* uint32[n]  raw MT draws of the last step      */
#define M3_ENV_GATHERED 11   /* int32 [nranks][n] the env's all-gather buffer (after m3_env_comm_init) */
int m3_env_get(m3_env *env, int what, void *host_out);
int m3_env_device_ptr(m3_env *env, int what, void **out);

/* Checkpoint / resume of the batched env (the reference state is
 * (array, cfg.seed, n_actions, _reward), boardv2.py:12-16, plus Match3Env's
 * score and moves_taken, env.py:34). Overwrites one field of every board from
 * host memory laid out as m3_env_get returns it. Settable: M3_ENV_BOARDS,
 * SEEDS, SCORE, MOVES, NEXT_ACTION and the last step's REWARD, DONE,
 * TRUNCATED, FLAGS, DRAWS; LEGAL and GATHERED are derived (M3_ERR_INVALID).
 * The per-board state the env derives from these -- the legal set of the
 * board, the MT19937 chain word mt[397] of the seed, the queued autoreset
 * episodes -- is rebuilt before the next step / get / synchronize, so an env
 * loaded with another env's fields steps exactly as that env would have. A
 * freshly created env may be loaded instead of reset. */
int m3_env_set(m3_env *env, int what, const void *host_in);

/* ---- multi-GPU: RCCL over xGMI, one process per GPU --------------------- */
/* 128-byte ncclUniqueId; rank 0 creates it, the caller ships it to all ranks. */
int m3_comm_unique_id(uint8_t out_id[128]);
/* One communicator per env; a second call returns M3_ERR_STATE. */
int m3_env_comm_init(m3_env *env, const uint8_t id[128], int nranks, int rank);
/* Ranks of the env's communicator as RCCL reports them (ncclCommCount); 1 before m3_env_comm_init. */
int m3_env_comm_size(m3_env *env, int *out_nranks);
/* ncclAllGather of the last step's packed (reward << 2 | truncated << 1 | done)
 * int32 words of every board of every rank into the env's device buffer
 * M3_ENV_GATHERED ([nranks][n], rank-major); host_out (nullable, int32[nranks*n])
 * receives a copy and the call then blocks until it is there. The step kernel
 * writes the packed words only once a communicator exists, so gather the
 * outcomes of steps taken after m3_env_comm_init. No counterpart in the
 * reference (single host, no collectives): SURVEY.md §8(e). */
int m3_env_gather(m3_env *env, int32_t *host_out);
/* Same, into a caller-owned device buffer d_out (int32[nranks][n]; NULL = the
 * env's buffer), enqueued on the env's context stream without blocking. d_out
 * holds the step's outcomes once that stream reaches the gather: after
 * m3_env_synchronize, or for any later m3_env_get / m3_env_gather. Steps keep
 * running meanwhile (the packed words are double-buffered by step parity). */
int m3_env_gather_device(m3_env *env, int32_t *d_out);
/* Test hook: enqueue ~usec of idle GPU time on the env's context stream (the
 * stream the gathers run on), to hold a gather in flight while later steps run. */
int m3_env_debug_stall(m3_env *env, uint32_t usec);

/* Cumulative counters since the last m3_env_reset: out[0] steps recomputed on
 * the exact fallback pass (>= 624 MT draws or more match groups than the LDS
 * table), out[1] resets recomputed by the wave-cooperative pass (>= 624 draws),
 * out[2] autoresets, out[3] number of shards. */
int m3_env_stats(m3_env *env, uint64_t out[4]);

/* ---- timing helpers for bench.py ---------------------------------------- */
/* Kernel-side timing: after m3_env_timing(env, cap), each of the next cap
 * shard-step launches records HIP events on its shard's stream before
 * k_env_step, after it, and after the pipeline's last kernel (k_env_cont_grid,
 * k_env_fix). m3_env_kernel_ms waits for them and returns the per-launch
 * durations of the whole pipeline in ms (out_n of them); m3_env_step_kernel_ms
 * the same for k_env_step alone (the dominant kernel, bench.py's roofline). */
int m3_env_timing(m3_env *env, int capacity);
int m3_env_kernel_ms(m3_env *env, float *out_ms, int max_n, int *out_n);
int m3_env_step_kernel_ms(m3_env *env, float *out_ms, int max_n, int *out_n);

#ifdef __cplusplus
}
#endif
#endif /* M3_H */
