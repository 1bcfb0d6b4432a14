/*
 * m3_oracle.c -- TEST INFRASTRUCTURE ONLY (see m3_oracle.h).
 *
 * A literal, scalar restatement of the reference's env-step path. Each
 * function cites the reference lines it follows (paths relative to the
 * ThorLL/Element-Crush-Gym checkout). Data structures deliberately follow the
 * reference (Python lists of (row, col) tuples for match groups, row-major
 * argwhere order, Python slice semantics) rather than the GPU design, so the
 * two implementations share no code and no shortcuts.
 */
#include "m3_oracle.h"

#include <stdlib.h>
#include <string.h>

#define MT_N 624
#define MT_M 397
#define MT_MATRIX_A 0x9908b0dfU
#define MT_UPPER 0x80000000U
#define MT_LOWER 0x7fffffffU

/* ---- numpy legacy RandomState (MT19937) ------------------------------------
 * numpy/random/src/mt19937/mt19937.c: mt19937_seed (legacy int seeding via
 * RandomState._legacy_seeding), mt19937_gen, mt19937_next32.
 * Called from boardv2.py:20,21,25,46,172 and boardFunctions.py:17,22. */
void m3o_mt_seed(m3o_mt *mt, uint32_t seed) {
    for (int pos = 0; pos < MT_N; pos++) {
        mt->key[pos] = seed;
        seed = 1812433253U * (seed ^ (seed >> 30)) + (uint32_t)(pos + 1);
    }
    mt->pos = MT_N;
    mt->draws = 0;
}

static void mt_gen(m3o_mt *mt) {
    uint32_t y;
    int i;
    for (i = 0; i < MT_N - MT_M; i++) {
        y = (mt->key[i] & MT_UPPER) | (mt->key[i + 1] & MT_LOWER);
        mt->key[i] = mt->key[i + MT_M] ^ (y >> 1) ^ ((0U - (y & 1U)) & MT_MATRIX_A);
    }
    for (; i < MT_N - 1; i++) {
        y = (mt->key[i] & MT_UPPER) | (mt->key[i + 1] & MT_LOWER);
        mt->key[i] = mt->key[i + (MT_M - MT_N)] ^ (y >> 1) ^ ((0U - (y & 1U)) & MT_MATRIX_A);
    }
    y = (mt->key[MT_N - 1] & MT_UPPER) | (mt->key[0] & MT_LOWER);
    mt->key[MT_N - 1] = mt->key[MT_M - 1] ^ (y >> 1) ^ ((0U - (y & 1U)) & MT_MATRIX_A);
    mt->pos = 0;
}

uint32_t m3o_mt_next32(m3o_mt *mt) {
    if (mt->pos == MT_N) mt_gen(mt);
    uint32_t y = mt->key[mt->pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680U;
    y ^= (y << 15) & 0xefc60000U;
    y ^= (y >> 18);
    mt->draws++;
    return y;
}

static uint64_t gen_mask(uint64_t max) {
    uint64_t m = max;
    m |= m >> 1; m |= m >> 2; m |= m >> 4; m |= m >> 8; m |= m >> 16; m |= m >> 32;
    return m;
}

/* RandomState.randint -> _rand_int64(..., use_masked=True) ->
 * random_bounded_uint64_fill -> buffered_bounded_masked_uint32 (32-bit ranges). */
int64_t m3o_randint(m3o_mt *mt, int64_t low, int64_t high) {
    uint64_t rng = (uint64_t)(high - low) - 1U;
    if (rng == 0) return low;
    if (rng == 0xFFFFFFFFULL) return low + (int64_t)m3o_mt_next32(mt);
    /* every range on this path is < 2^32 */
    uint32_t mask = (uint32_t)gen_mask(rng);
    uint32_t v;
    while ((v = (m3o_mt_next32(mt) & mask)) > rng) {}
    return low + (int64_t)v;
}

/* numpy/random/src/distributions/distributions.c: random_interval (legacy shuffle). */
uint64_t m3o_random_interval(m3o_mt *mt, uint64_t max) {
    if (max == 0) return 0;
    uint32_t mask = (uint32_t)gen_mask(max);
    uint32_t v;
    while ((v = (m3o_mt_next32(mt) & mask)) > max) {}
    return v;
}

/* ---- BoardConfig (match3tile/boardConfig.py:26-69) ------------------------- */
void m3o_cfg_init(m3o_cfg *cfg, int rows, int columns, int types) {
    cfg->R = rows;
    cfg->C = columns;
    cfg->T = types;
    cfg->A = rows * (columns - 1) * 2;                 /* :27 */
    int bits = 0;                                      /* :29 ceil(log2(types+1)) */
    while ((1 << bits) < types + 1) bits++;
    cfg->TM = (1 << bits) - 1;                         /* :30 */
    cfg->STM = (1 << (bits + 1)) + 1 + cfg->TM;        /* :31 */
    cfg->H = cfg->TM + 1;                              /* :32 */
    cfg->V = 2 * cfg->H;                               /* :41 */
    cfg->B = cfg->STM;                                 /* :42 */
    cfg->M = cfg->TM + cfg->STM + 1;                   /* :43 */
}

/* decode (boardConfig.py:45-59), including int() truncation toward zero. */
void m3o_decode(const m3o_cfg *cfg, int action, int *r1, int *c1, int *r2, int *c2) {
    int a = 2 * cfg->C - 1;
    int b = cfg->C - 1;
    int q = action / a; /* int(action / a) for action >= 0 */
    if (action - a * q >= b) {
        int col1 = action % a - b;
        int num = action - 3 - col1;
        int row1 = num / a; /* C division truncates toward zero == Python int() */
        *r1 = row1; *c1 = col1; *r2 = row1 + 1; *c2 = col1;
    } else {
        int col1 = action % a;
        *r1 = (action - col1) / a; *c1 = col1; *r2 = *r1; *c2 = col1 + 1;
    }
}

/* encode (boardConfig.py:61-69) */
int m3o_encode(const m3o_cfg *cfg, int r1, int c1, int r2, int c2) {
    int a = 2 * cfg->C - 1;
    int b = (c1 == c2) ? cfg->C - 1 : 0;
    return (r1 < r2 ? r1 : r2) * a + b + (c1 < c2 ? c1 : c2);
}

/* ---- get_matches (boardFunctions.py:121-156) --------------------------------
 * `matches` is a Python list of lists of (row, col) tuples. Here every group
 * is a growable int array of cell ids (r*C+c), duplicates kept. */
typedef struct {
    int n;
    int *len;
    int *cap;
    int **items;
} groups_t;

static void groups_init(groups_t *g) { memset(g, 0, sizeof(*g)); }
static void groups_free(groups_t *g) {
    for (int i = 0; i < g->n; i++) free(g->items[i]);
    free(g->items); free(g->len); free(g->cap);
    memset(g, 0, sizeof(*g));
}
static int group_has(const groups_t *g, int gi, int cell) {
    for (int k = 0; k < g->len[gi]; k++) if (g->items[gi][k] == cell) return 1;
    return 0;
}
static void group_push(groups_t *g, int gi, int cell) {
    if (g->len[gi] == g->cap[gi]) {
        g->cap[gi] = g->cap[gi] ? 2 * g->cap[gi] : 16;
        g->items[gi] = (int *)realloc(g->items[gi], sizeof(int) * (size_t)g->cap[gi]);
    }
    g->items[gi][g->len[gi]++] = cell;
}
static int group_new(groups_t *g) {
    int gi = g->n++;
    g->items = (int **)realloc(g->items, sizeof(int *) * (size_t)g->n);
    g->len = (int *)realloc(g->len, sizeof(int) * (size_t)g->n);
    g->cap = (int *)realloc(g->cap, sizeof(int) * (size_t)g->n);
    g->items[gi] = NULL; g->len[gi] = 0; g->cap[gi] = 0;
    return gi;
}

/* add_to_matches (boardFunctions.py:126-131): merge into the FIRST group that
 * shares any cell; `item not in matches` compares a tuple against lists and is
 * always true, so every item (duplicates included) is appended. */
static void add_to_matches(groups_t *g, const int *run, int n) {
    for (int gi = 0; gi < g->n; gi++) {
        int hit = 0;
        for (int k = 0; k < n && !hit; k++) hit = group_has(g, gi, run[k]);
        if (hit) {
            for (int k = 0; k < n; k++) group_push(g, gi, run[k]);
            return;
        }
    }
    int gi = group_new(g);
    for (int k = 0; k < n; k++) group_push(g, gi, run[k]);
}

static int in_any_group(const groups_t *g, int cell) {
    for (int gi = 0; gi < g->n; gi++) if (group_has(g, gi, cell)) return 1;
    return 0;
}

static void get_matches_groups(const m3o_cfg *cfg, const int32_t *a, uint8_t *mask, groups_t *g) {
    const int R = cfg->R, C = cfg->C;
    int *run = (int *)malloc(sizeof(int) * (size_t)(R + C + 2));
    memset(mask, 0, (size_t)(R * C));
    for (int r = 0; r < R; r++) {
        for (int c = 0; c < C; c++) {
            int32_t v = a[r * C + c];
            if (v == 0 || in_any_group(g, r * C + c)) continue;           /* :136 */
            int n = 0;
            if (c <= C - 3 && a[r * C + c] == a[r * C + c + 1] && a[r * C + c + 1] == a[r * C + c + 2]) {
                for (int k = c; k < C && a[r * C + k] == v; k++) {       /* :140-145 */
                    run[n++] = r * C + k;
                    mask[r * C + k] = 1;
                }
            }
            if (r <= R - 3 && a[r * C + c] == a[(r + 1) * C + c] && a[(r + 1) * C + c] == a[(r + 2) * C + c]) {
                for (int k = r; k < R && a[k * C + c] == v; k++) {       /* :148-153 */
                    run[n++] = k * C + c;
                    mask[k * C + c] = 1;
                }
            }
            if (n > 2) add_to_matches(g, run, n);                         /* :154-155 */
        }
    }
    free(run);
}

int m3o_get_matches(const m3o_cfg *cfg, const int32_t *tb, uint8_t *mask) {
    groups_t g;
    groups_init(&g);
    get_matches_groups(cfg, tb, mask, &g);
    int n = g.n;
    groups_free(&g);
    return n;
}

static int cmp_int(const void *x, const void *y) {
    int a = *(const int *)x, b = *(const int *)y;
    return (a > b) - (a < b);
}

/* get_match_spawn_mask + get_center (boardFunctions.py:159-169, 8-13).
 * Sorting by (row, col) == sorting by cell id r*C+c. */
static void spawn_mask(const m3o_cfg *cfg, groups_t *g, int32_t *spawn) {
    const int C = cfg->C;
    memset(spawn, 0, sizeof(int32_t) * (size_t)(cfg->R * C));
    for (int gi = 0; gi < g->n; gi++) {
        int n = g->len[gi];
        if (n <= 3) continue;                                             /* :161 */
        qsort(g->items[gi], (size_t)n, sizeof(int), cmp_int);             /* :10 */
        int center = g->items[gi][n / 2];                                 /* :13 */
        int r0 = g->items[gi][0] / C, c0 = g->items[gi][0] % C;
        int rows_eq = 1, cols_eq = 1;
        for (int k = 0; k < n; k++) {
            if (g->items[gi][k] / C != r0) rows_eq = 0;
            if (g->items[gi][k] % C != c0) cols_eq = 0;
        }
        if (rows_eq) spawn[center] = n > 4 ? cfg->M : cfg->V;             /* :163-164 */
        else if (cols_eq) spawn[center] = n > 4 ? cfg->M : cfg->H;        /* :165-166 */
        else spawn[center] = cfg->B;                                      /* :167-168 */
    }
}

int m3o_matches_and_spawn(const m3o_cfg *cfg, const int32_t *tb, uint8_t *mask, int32_t *spawn) {
    groups_t g;
    groups_init(&g);
    get_matches_groups(cfg, tb, mask, &g);
    spawn_mask(cfg, &g, spawn);
    int n = g.n;
    groups_free(&g);
    return n;
}

/* ---- legal_actions (boardFunctions.py:26-112) ------------------------------- */
static int check_above_and_below(const m3o_cfg *cfg, const int32_t *arr, int r, int c, int32_t token) {
    const int R = cfg->R, C = cfg->C;                                     /* :48-59 */
    int above = r - 1 >= 0 && arr[(r - 1) * C + c] == token;
    int below = r + 1 < R && arr[(r + 1) * C + c] == token;
    if (!(above || below)) return 0;
    if (above && below) return 1;
    if (above && !below) return r - 2 >= 0 && arr[(r - 2) * C + c] == token;
    return r + 2 < R && arr[(r + 2) * C + c] == token;
}

static int check_left_and_right(const m3o_cfg *cfg, const int32_t *arr, int r, int c, int32_t token) {
    const int C = cfg->C;                                                 /* :81-92 */
    int left = c - 1 >= 0 && arr[r * C + c - 1] == token;
    int right = c + 1 < C && arr[r * C + c + 1] == token;
    if (!(left || right)) return 0;
    if (left && right) return 1;
    if (left && !right) return c - 2 >= 0 && arr[r * C + c - 2] == token;
    return c + 2 < C && arr[r * C + c + 2] == token;
}

/* horizontal_check(left_token, right_token, left, right, arr)  (:30-61) */
static int horizontal_check(const m3o_cfg *cfg, const int32_t *arr, int32_t lt, int32_t rt,
                            int lr, int lc, int rr, int rc) {
    const int C = cfg->C;
    if (lc - 2 >= 0 && arr[lr * C + lc - 2] == arr[lr * C + lc - 1] && arr[lr * C + lc - 1] == lt) return 1;
    if (rc + 2 < C && arr[rr * C + rc + 1] == arr[rr * C + rc + 2] && arr[rr * C + rc + 2] == rt) return 1;
    return check_above_and_below(cfg, arr, lr, lc, lt) || check_above_and_below(cfg, arr, rr, rc, rt);
}

/* vertical_check(above_token, below_token, above, below, arr)  (:63-94) */
static int vertical_check(const m3o_cfg *cfg, const int32_t *arr, int32_t at, int32_t bt,
                          int ar, int ac, int br, int bc) {
    const int R = cfg->R, C = cfg->C;
    if (br + 2 < R && arr[(br + 1) * C + bc] == arr[(br + 2) * C + bc] && arr[(br + 2) * C + bc] == bt) return 1;
    if (ar - 2 >= 0 && arr[(ar - 2) * C + ac] == arr[(ar - 1) * C + ac] && arr[(ar - 1) * C + ac] == at) return 1;
    return check_left_and_right(cfg, arr, br, bc, bt) || check_left_and_right(cfg, arr, ar, ac, at);
}

int m3o_legal_actions(const m3o_cfg *cfg, const int32_t *board, int32_t *out_actions) {
    const int R = cfg->R, C = cfg->C, N = R * C;
    int32_t *tb = (int32_t *)malloc(sizeof(int32_t) * (size_t)N);
    for (int i = 0; i < N; i++) tb[i] = board[i] & cfg->TM;                /* :96 */
    int n = 0;
    for (int action = 0; action < cfg->A; action++) {                      /* :97 */
        int r1, c1, r2, c2;
        m3o_decode(cfg, action, &r1, &c1, &r2, &c2);
        int32_t t1 = tb[r1 * C + c1], t2 = tb[r2 * C + c2];
        if (t1 == 0 || t2 == 0 || (board[r1 * C + c1] > cfg->TM && board[r2 * C + c2] > cfg->TM)) {
            out_actions[n++] = action;                                     /* :100-102 */
            continue;
        }
        if (t1 == t2) continue;                                            /* :103-104 */
        int is_vertical = (c1 == c2);                                      /* :105 */
        int ok;
        if (is_vertical)  /* vertical_check(token2, token1, cell1, cell2) -> above=cell1, below=cell2 */
            ok = vertical_check(cfg, tb, t2, t1, r1, c1, r2, c2);
        else              /* horizontal_check(token2, token1, cell1, cell2) */
            ok = horizontal_check(cfg, tb, t2, t1, r1, c1, r2, c2);
        if (ok) out_actions[n++] = action;
    }
    free(tb);
    return n;
}

/* ---- BoardV2.__init__ (boardv2.py:12-29) ------------------------------------ */
int64_t m3o_init_board(const m3o_cfg *cfg, uint32_t seed, int32_t *board, m3o_mt *mt) {
    const int N = cfg->R * cfg->C;
    m3o_mt local;
    if (!mt) mt = &local;
    m3o_mt_seed(mt, seed);                                                 /* :20 */
    for (int i = 0; i < N; i++) board[i] = (int32_t)m3o_randint(mt, 1, cfg->T + 1); /* :21 */
    uint8_t *mask = (uint8_t *)malloc((size_t)N);
    int32_t *fresh = (int32_t *)malloc(sizeof(int32_t) * (size_t)N);
    int ng = m3o_get_matches(cfg, board, mask);                            /* :23 */
    while (ng > 0) {                                                       /* :24 */
        for (int i = 0; i < N; i++) fresh[i] = (int32_t)m3o_randint(mt, 1, cfg->T + 1); /* :25 */
        for (int i = 0; i < N; i++) if (mask[i]) board[i] = fresh[i];    /* :26 */
        ng = m3o_get_matches(cfg, board, mask);                            /* :27 */
    }
    free(mask);
    free(fresh);
    return mt->draws;
}

/* Python slice normalisation a[start:stop] on an axis of length n. */
static void pyslice(int start, int stop, int n, int *lo, int *hi) {
    if (start < 0) { start += n; if (start < 0) start = 0; }
    if (start > n) start = n;
    if (stop < 0) { stop += n; if (stop < 0) stop = 0; }
    if (stop > n) stop = n;
    *lo = start;
    *hi = stop > start ? stop : start;
}

static int32_t point_of(const m3o_cfg *cfg, int32_t x) {                   /* boardv2.py:58-65 */
    if (x <= cfg->TM) return 2;
    if (x == cfg->M) return 250;
    if (x < cfg->STM) return 25;
    return 50;
}

static int lower_clamp(int v) { return v < 0 ? 0 : v; }                    /* util/quickMath.py:1-2 */
static int upper_clamp(int v, int m) { return v > m ? m : v; }             /* util/quickMath.py:5-6 */

/* shuffle (boardFunctions.py:16-23): reseed, save specials, legacy
 * RandomState.shuffle of the rows (Fisher-Yates with random_interval), restore. */
static void oracle_shuffle(const m3o_cfg *cfg, uint32_t seed, int32_t *arr, m3o_mt *mt) {
    const int R = cfg->R, C = cfg->C, N = R * C;
    m3o_mt_seed(mt, seed);
    uint8_t *sp = (uint8_t *)malloc((size_t)N);
    int32_t *saved = (int32_t *)malloc(sizeof(int32_t) * (size_t)N);
    int32_t *buf = (int32_t *)malloc(sizeof(int32_t) * (size_t)C);
    for (int i = 0; i < N; i++) { sp[i] = arr[i] > cfg->TM; saved[i] = sp[i] ? arr[i] : 0; }
    for (int i = R - 1; i >= 1; i--) {
        int j = (int)m3o_random_interval(mt, (uint64_t)i);
        if (i == j) continue;
        memcpy(buf, arr + j * C, sizeof(int32_t) * (size_t)C);
        memcpy(arr + j * C, arr + i * C, sizeof(int32_t) * (size_t)C);
        memcpy(arr + i * C, buf, sizeof(int32_t) * (size_t)C);
    }
    for (int i = 0; i < N; i++) if (sp[i]) arr[i] = saved[i];
    free(sp); free(saved); free(buf);
}

/* ---- BoardV2.apply_action (boardv2.py:43-207) ------------------------------- */
int64_t m3o_apply_action(const m3o_cfg *cfg, uint32_t seed, int n_actions,
                         const int32_t *board, int action, int32_t *out_board,
                         m3o_mt *mt, int *flags, int shuffle_cap) {
    const int R = cfg->R, C = cfg->C, N = R * C;
    const int TM = cfg->TM, STM = cfg->STM, H = cfg->H, V = cfg->V, B = cfg->B, M = cfg->M;
    *flags = 0;
    if (n_actions < 1) {                                                   /* :44-45 */
        memcpy(out_board, board, sizeof(int32_t) * (size_t)N);
        *flags |= M3O_FLAG_TERMINAL;
        return 0;
    }
    if (action < 0 || action >= cfg->A) {                                  /* :48 KeyError */
        memcpy(out_board, board, sizeof(int32_t) * (size_t)N);
        *flags |= M3O_FLAG_BAD_ACTION;
        return 0;
    }
    m3o_mt_seed(mt, seed);                                                 /* :46 */
    int64_t reward = 0;
    int sr, sc, tr, tc;
    m3o_decode(cfg, action, &sr, &sc, &tr, &tc);                           /* :48 */
    const int s = sr * C + sc, t = tr * C + tc;

    int32_t *ns = out_board;                                               /* next_state */
    memcpy(ns, board, sizeof(int32_t) * (size_t)N);
    ns[s] = board[t]; ns[t] = board[s];                                    /* :51 swap */

    int32_t *pts = (int32_t *)malloc(sizeof(int32_t) * (size_t)N);
    int32_t *sp = (int32_t *)malloc(sizeof(int32_t) * (size_t)N);
    int32_t *tb = (int32_t *)malloc(sizeof(int32_t) * (size_t)N);
    int32_t *spawn = (int32_t *)calloc((size_t)N, sizeof(int32_t));
    uint8_t *mask = (uint8_t *)malloc((size_t)N);
    int32_t *legal = (int32_t *)malloc(sizeof(int32_t) * (size_t)(cfg->A > 0 ? cfg->A : 1));
    int *trig = (int *)malloc(sizeof(int) * (size_t)N);

    for (int i = 0; i < N; i++) {                                          /* :68-71 */
        pts[i] = point_of(cfg, ns[i]);
        sp[i] = ns[i] > TM ? ns[i] : 0;
        tb[i] = ns[i] & TM;
    }
    const int32_t token1 = board[s], token2 = board[t];                    /* :73 */
    const int32_t ty1 = sp[s], ty2 = sp[t];                                /* :74 */
#define ARE(x, y) ((ty1 == (x) && ty2 == (y)) || (ty2 == (x) && ty1 == (y)))  /* :76-77 */
    if (ARE(M, M)) {                                                       /* :81-82 */
        for (int i = 0; i < N; i++) tb[i] = 0;
    } else if (ARE(M, B)) {                                                /* :84-89 */
        int32_t token = token1 > token2 ? token1 : token2;
        for (int i = 0; i < N; i++)
            if (tb[i] == token && sp[i] == 0) sp[i] = token + B;
    } else if (ARE(M, H) || ARE(M, V)) {                                   /* :91-99 */
        int32_t token = token1 > token2 ? token1 : token2;
        int n = 0;
        for (int i = 0; i < N; i++) {                                      /* argwhere order */
            if (tb[i] == token && sp[i] == 0) {
                tb[i] = 0;
                if (sp[i] == 0) sp[i] = (n % 2 == 0) ? V : H;
                n++;
            }
        }
    } else if (ARE(M, 0)) {                                                /* :101-103 */
        int32_t token = token1 > token2 ? token1 : token2;
        for (int i = 0; i < N; i++) if (tb[i] == token) tb[i] = 0;
    } else if (ARE(B, B)) {                                                /* :112-116 */
        int r0 = lower_clamp(tr - 2), r1 = upper_clamp(tr + 2, R);
        int c0 = lower_clamp(tc - 2), c1 = upper_clamp(tc + 2, C);
        for (int r = r0; r < r1; r++) for (int c = c0; c < c1; c++) tb[r * C + c] = 0;
    } else if (ARE(B, H) || ARE(B, V)) {                                   /* :123-125 */
        int c0 = lower_clamp(tc - 2), c1 = upper_clamp(tc + 2, C);
        for (int r = 0; r < R; r++) for (int c = c0; c < c1; c++) tb[r * C + c] = 0;
        int r0 = lower_clamp(tr - 2), r1 = upper_clamp(tr + 2, R);
        for (int r = r0; r < r1; r++) for (int c = 0; c < C; c++) tb[r * C + c] = 0;
    } else if (ARE(H, V) || ARE(V, H)) {                                   /* :130-132 */
        int lo, hi;
        pyslice(0, tc, R, &lo, &hi);                                       /* token_board[:target[1]] (rows) */
        for (int r = lo; r < hi; r++) for (int c = 0; c < C; c++) tb[r * C + c] = 0;
        pyslice(tr, R, R, &lo, &hi);                                       /* token_board[target[0]:] */
        for (int r = lo; r < hi; r++) for (int c = 0; c < C; c++) tb[r * C + c] = 0;
    } else {                                                               /* :133-136 */
        m3o_matches_and_spawn(cfg, tb, mask, spawn);
        for (int i = 0; i < N; i++) if (mask[i]) tb[i] = 0;
    }
#undef ARE

    for (;;) {                                                             /* :138 */
        for (int i = 0; i < N; i++) if (tb[i] != 0) sp[i] = 0;             /* :141 */
        int nt = 0;
        for (int i = 0; i < N; i++) if (sp[i] != 0) trig[nt++] = i;       /* :142 argwhere */
        for (int k = 0; k < nt; k++) {
            int i = trig[k] / C, j = trig[k] % C;
            int32_t st = sp[trig[k]] & STM;                                /* :144 */
            if (st == H) {                                                 /* :147-148 */
                for (int c = 0; c < C; c++) tb[i * C + c] = 0;
            } else if (st == V) {                                          /* :149-150 */
                for (int r = 0; r < R; r++) tb[r * C + j] = 0;
            } else if (st == B) {                                          /* :151-154 transposed slice */
                int rl, rh, cl, ch;
                pyslice(j - 1, j + 1, R, &rl, &rh);
                pyslice(i - 1, i + 1, C, &cl, &ch);
                for (int r = rl; r < rh; r++) for (int c = cl; c < ch; c++) tb[r * C + c] = 0;
            }
        }
        for (int i = 0; i < N; i++) if (tb[i] == 0) reward += pts[i];     /* :157-158 */
        for (int i = 0; i < N; i++) if (tb[i] == 0) ns[i] = 0;            /* :161 */
        for (int i = 0; i < N; i++) if (spawn[i] != 0) ns[i] += spawn[i]; /* :162 */
        for (int i = 0; i < N; i++) ns[i] = ns[i] < 0 ? 0 : (ns[i] > 32 ? 32 : ns[i]); /* :163 */
        for (int c = 0; c < C; c++) {                                      /* :166-173 gravity */
            int keep[64];
            int nk = 0;
            for (int r = 0; r < R; r++) if (ns[r * C + c] > 0) keep[nk++] = ns[r * C + c];
            if (nk == R) continue;
            int k = R - nk;
            for (int r = 0; r < k; r++) ns[r * C + c] = (int32_t)m3o_randint(mt, 1, cfg->T + 1);
            for (int r = 0; r < nk; r++) ns[(k + r) * C + c] = keep[r];
        }
        for (int i = 0; i < N; i++) {                                      /* :176-178 */
            pts[i] = point_of(cfg, ns[i]);
            sp[i] = ns[i] > TM ? ns[i] : 0;
            tb[i] = ns[i] & TM;
        }
        int ng = m3o_matches_and_spawn(cfg, tb, mask, spawn);              /* :181 */
        int shuffles = 0;
        while (ng == 0 && m3o_legal_actions(cfg, ns, legal) == 0) {       /* :188 */
            if (shuffles >= shuffle_cap) { *flags |= M3O_FLAG_SHUFFLE_CAP; break; }
            oracle_shuffle(cfg, seed, ns, mt);                             /* :189 */
            shuffles++;
            *flags |= M3O_FLAG_SHUFFLED;
            for (int i = 0; i < N; i++) {                                  /* :191-193 */
                pts[i] = point_of(cfg, ns[i]);
                sp[i] = ns[i] > TM ? ns[i] : 0;
                tb[i] = ns[i] & TM;
            }
            ng = m3o_matches_and_spawn(cfg, tb, mask, spawn);              /* :194 */
        }
        if (ng == 0) break;                                                /* :195-196 */
        for (int i = 0; i < N; i++) if (mask[i]) tb[i] = 0;               /* :199 */
        /* spawn already holds get_match_spawn_mask(matches)                  :202 */
    }
    free(pts); free(sp); free(tb); free(spawn); free(mask); free(legal); free(trig);
    return reward;
}

/* ---- seeded random episode (samplerTasks.py:9-14 + env.py:48-56 bookkeeping) */
/* Shuffle cap of the episode / rollout drivers below. The reference has none
 * (a cycling dead board hangs it, boardv2.py:188-194); the default 2^20 is
 * "never" for boards that terminate. Tests on tiny boards, where cycling dead
 * boards are common, lower it to the GPU's 1024 and compare the flag. */
static int g_episode_cap = 1 << 20;
void m3o_set_episode_shuffle_cap(int cap) { g_episode_cap = cap; }

int m3o_random_episode(const m3o_cfg *cfg, uint32_t seed, int num_moves, int env_goal,
                       int32_t *actions, int32_t *rewards, int32_t *draws,
                       uint8_t *done, int32_t *final_board, int *flags) {
    const int N = cfg->R * cfg->C;
    m3o_mt mt;
    int32_t *a = (int32_t *)malloc(sizeof(int32_t) * (size_t)N);
    int32_t *b = (int32_t *)malloc(sizeof(int32_t) * (size_t)N);
    int32_t *legal = (int32_t *)malloc(sizeof(int32_t) * (size_t)cfg->A);
    m3o_init_board(cfg, seed, a, &mt);                                     /* samplerTasks.py:10 */
    m3o_mt_seed(&mt, seed);                                                /* samplerTasks.py:11 */
    int64_t score = 0;
    int moves = 0;
    *flags = 0;
    int n_actions = num_moves;
    while (moves < num_moves) {
        int nl = m3o_legal_actions(cfg, a, legal);
        if (nl == 0) { *flags |= M3O_FLAG_NO_LEGAL; break; }              /* choice([]) raises */
        int act = legal[m3o_randint(&mt, 0, nl)];                          /* samplerTasks.py:13 */
        int f = 0;
        int64_t r = m3o_apply_action(cfg, seed, n_actions, a, act, b, &mt, &f, g_episode_cap);
        *flags |= f;
        n_actions--;
        memcpy(a, b, sizeof(int32_t) * (size_t)N);
        score += r;
        actions[moves] = act;
        rewards[moves] = (int32_t)r;
        draws[moves] = (int32_t)mt.draws;
        int d = (score >= env_goal) || (moves + 1 == num_moves);           /* env.py:53-54 */
        done[moves] = (uint8_t)d;
        moves++;
        if (d) break;
    }
    if (final_board) memcpy(final_board, a, sizeof(int32_t) * (size_t)N);
    free(a); free(b); free(legal);
    return moves;
}

/* n independent seeded episodes, all per-move outputs kept (parity checks). */
void m3o_batch_episodes(const m3o_cfg *cfg, int64_t n, const uint32_t *seeds, int num_moves, int env_goal,
                        int nthreads, int32_t *actions, int32_t *rewards, int32_t *draws, uint8_t *done,
                        int32_t *final_boards, int32_t *moves_out, int32_t *flags_out) {
    const int N = cfg->R * cfg->C;
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 16)
    for (int64_t i = 0; i < n; i++) {
        int f = 0;
        moves_out[i] = m3o_random_episode(cfg, seeds[i], num_moves, env_goal, actions + i * num_moves,
                                          rewards + i * num_moves, draws + i * num_moves, done + i * num_moves,
                                          final_boards + i * N, &f);
        flags_out[i] = f;
    }
}

/* mctslib/standard/mcts.py:14-19. The global RNG is seeded once with the
 * rollout seed (:15); apply_action reseeds it with cfg.seed every step
 * (boardv2.py:46), so every choice after the first reads cfg.seed's stream
 * where the step left it. A terminal state (n_actions < 1) returns at once. */
int64_t m3o_rollout(const m3o_cfg *cfg, const int32_t *board, uint32_t seed, int n_actions,
                    uint32_t rollout_seed, int32_t *final_board, int *steps, int64_t *draws, int *flags) {
    const int N = cfg->R * cfg->C;
    m3o_mt mt;
    int32_t *a = (int32_t *)malloc(sizeof(int32_t) * (size_t)N);
    int32_t *b = (int32_t *)malloc(sizeof(int32_t) * (size_t)N);
    int32_t *legal = (int32_t *)malloc(sizeof(int32_t) * (size_t)cfg->A);
    memcpy(a, board, sizeof(int32_t) * (size_t)N);
    m3o_mt_seed(&mt, rollout_seed);                                         /* mcts.py:15 */
    int64_t gain = 0;
    *steps = 0;
    *flags = 0;
    while (n_actions >= 1) {                                                /* mcts.py:16 */
        int nl = m3o_legal_actions(cfg, a, legal);
        if (nl == 0) { *flags |= M3O_FLAG_NO_LEGAL; break; }               /* choice([]) raises */
        int act = legal[m3o_randint(&mt, 0, nl)];                           /* mcts.py:17 */
        int f = 0;
        gain += m3o_apply_action(cfg, seed, n_actions, a, act, b, &mt, &f, g_episode_cap);  /* mcts.py:18 */
        *flags |= f;
        n_actions--;
        (*steps)++;
        memcpy(a, b, sizeof(int32_t) * (size_t)N);
    }
    *draws = mt.draws;
    if (final_board) memcpy(final_board, a, sizeof(int32_t) * (size_t)N);
    free(a); free(b); free(legal);
    return gain;
}

void m3o_batch_rollouts(const m3o_cfg *cfg, int64_t n, const int32_t *boards, const uint32_t *seeds,
                        const int32_t *n_actions, const uint32_t *rollout_seeds, int nthreads,
                        int32_t *gain, int32_t *steps, int64_t *draws, int32_t *flags, int32_t *final_boards) {
    const int N = cfg->R * cfg->C;
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 16)
    for (int64_t i = 0; i < n; i++) {
        int st = 0, f = 0;
        int64_t d = 0;
        gain[i] = (int32_t)m3o_rollout(cfg, boards + i * N, seeds[i], n_actions[i], rollout_seeds[i],
                                       final_boards ? final_boards + i * N : NULL, &st, &d, &f);
        steps[i] = st;
        draws[i] = d;
        flags[i] = f;
    }
}

int64_t m3o_run_episodes(const m3o_cfg *cfg, int64_t n, const uint32_t *seeds,
                         int num_moves, int env_goal, int nthreads, int64_t *out_total) {
    int64_t steps = 0;
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 4) reduction(+ : steps)
    for (int64_t i = 0; i < n; i++) {
        int32_t acts[1024], rews[1024], drw[1024];
        uint8_t dn[1024];
        int f;
        int mv = num_moves > 1024 ? 1024 : num_moves;
        int k = m3o_random_episode(cfg, seeds[i], mv, env_goal, acts, rews, drw, dn, NULL, &f);
        int64_t tot = 0;
        for (int j = 0; j < k; j++) tot += rews[j];
        if (out_total) out_total[i] = tot;
        steps += k;
    }
    return steps;
}
