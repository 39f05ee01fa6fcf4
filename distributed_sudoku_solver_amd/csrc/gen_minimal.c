/*
 * gen_minimal.c -- deterministic generator of distinct MINIMAL unique Sudoku puzzles:
 * synthetic workload data for tests and the bench (libsudoku_gen.so, host CPU only,
 * loaded by synth.make_minimal).  It is not part of the solve path: libsudoku_hip.so
 * does not link it and nothing here computes an answer that is returned to a caller.
 *
 * Puzzle k of a run with seed S:
 *   1. a random complete grid: randomized backtracking (digits tried in a random
 *      order per cell) from an empty board, PRNG splitmix64(S, k);
 *   2. clue removal: cells in a random order; a clue is removed when the board
 *      still has exactly one completion (counted up to 2 with a bitmask MRV
 *      search).  Every clue left is needed, so the puzzle is minimal and unique.
 * The answer of every puzzle is its generating grid (unique by construction);
 * tests re-check a sample against the oracle's naive DFS (the reference's answer).
 *
 * Hard subset (gen_minimal_nodes_batch): the search nodes a lowest-open-cell DFS with
 * naked + hidden singles propagation takes on puzzle k (the propagating solvers'
 * branching, SDK_ORDER_LEX); tools/make_hard_set.py keeps the puzzles that need >= 20
 * and commits their indices and clue masks.  gen_grid_batch rebuilds the grids of
 * given indices (step 1 alone), so a puzzle is grid & mask without a removal pass.
 *
 * build: csrc/Makefile (gcc -O2 -shared -fPIC -pthread -> ../libsudoku_gen.so)
 */
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <string.h>

#define ALL 0x3FEu

static inline uint64_t splitmix(uint64_t *s)
{
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

typedef struct { uint16_t row[9], col[9], box[9]; uint8_t cell[81]; } st_t;

static inline int bx(int i) { return (i / 27) * 3 + (i % 9) / 3; }

static void st_init(st_t *s, const uint8_t *b)
{
    memset(s, 0, sizeof *s);
    for (int i = 0; i < 81; ++i) {
        s->cell[i] = b[i];
        if (b[i]) {
            uint16_t m = (uint16_t)(1u << b[i]);
            s->row[i / 9] |= m; s->col[i % 9] |= m; s->box[bx(i)] |= m;
        }
    }
}

/* completions up to `limit` (MRV branching) */
static int count(st_t *s, int limit)
{
    int best = -1, bn = 10;
    uint16_t bc = 0;
    for (int i = 0; i < 81; ++i) {
        if (s->cell[i]) continue;
        uint16_t c = (uint16_t)(ALL & ~(s->row[i / 9] | s->col[i % 9] | s->box[bx(i)]));
        int n = __builtin_popcount(c);
        if (n < bn) { bn = n; best = i; bc = c; if (n == 0) return 0; if (n == 1) break; }
    }
    if (best < 0) return 1;
    int total = 0, r = best / 9, c = best % 9, b = bx(best);
    while (bc) {
        int d = __builtin_ctz(bc);
        bc &= (uint16_t)(bc - 1);
        uint16_t m = (uint16_t)(1u << d);
        s->row[r] |= m; s->col[c] |= m; s->box[b] |= m; s->cell[best] = (uint8_t)d;
        total += count(s, limit - total);
        s->row[r] &= (uint16_t)~m; s->col[c] &= (uint16_t)~m; s->box[b] &= (uint16_t)~m; s->cell[best] = 0;
        if (total >= limit) break;
    }
    return total;
}

static int fill(st_t *s, int i, uint64_t *rng)
{
    if (i == 81) return 1;
    uint16_t c = (uint16_t)(ALL & ~(s->row[i / 9] | s->col[i % 9] | s->box[bx(i)]));
    uint8_t d[9];
    int n = 0;
    while (c) { d[n++] = (uint8_t)__builtin_ctz(c); c &= (uint16_t)(c - 1); }
    for (int k = n - 1; k > 0; --k) {          /* random digit order */
        int j = (int)(splitmix(rng) % (uint64_t)(k + 1));
        uint8_t t = d[k]; d[k] = d[j]; d[j] = t;
    }
    for (int k = 0; k < n; ++k) {
        uint16_t m = (uint16_t)(1u << d[k]);
        s->row[i / 9] |= m; s->col[i % 9] |= m; s->box[bx(i)] |= m; s->cell[i] = d[k];
        if (fill(s, i + 1, rng)) return 1;
        s->row[i / 9] &= (uint16_t)~m; s->col[i % 9] &= (uint16_t)~m; s->box[bx(i)] &= (uint16_t)~m; s->cell[i] = 0;
    }
    return 0;
}

void gen_minimal_one(uint64_t seed, uint64_t k, uint8_t *puzzle, uint8_t *solution)
{
    uint64_t rng = seed * 0x100000001B3ull ^ (k + 1) * 0x9E3779B97F4A7C15ull;
    st_t s;
    uint8_t zero[81] = {0};
    st_init(&s, zero);
    fill(&s, 0, &rng);
    memcpy(solution, s.cell, 81);
    uint8_t b[81], order[81];
    memcpy(b, s.cell, 81);
    for (int i = 0; i < 81; ++i) order[i] = (uint8_t)i;
    for (int i = 80; i > 0; --i) {
        int j = (int)(splitmix(&rng) % (uint64_t)(i + 1));
        uint8_t t = order[i]; order[i] = order[j]; order[j] = t;
    }
    for (int q = 0; q < 81; ++q) {
        int i = order[q];
        uint8_t v = b[i];
        b[i] = 0;
        st_t t;
        st_init(&t, b);
        if (count(&t, 2) != 1) b[i] = v;
    }
    memcpy(puzzle, b, 81);
}

/* the grid of puzzle k (step 1 of gen_minimal_one, same PRNG stream) */
void gen_grid_one(uint64_t seed, uint64_t k, uint8_t *solution)
{
    uint64_t rng = seed * 0x100000001B3ull ^ (k + 1) * 0x9E3779B97F4A7C15ull;
    st_t s;
    uint8_t zero[81] = {0};
    st_init(&s, zero);
    fill(&s, 0, &rng);
    memcpy(solution, s.cell, 81);
}

/* ---- search nodes of a singles-propagating lowest-open-cell DFS (the hard filter) ---- */
static int g_unit[27][9];
static pthread_once_t g_unit_once = PTHREAD_ONCE_INIT;

static void unit_init(void)
{
    for (int u = 0; u < 9; ++u)
        for (int k = 0; k < 9; ++k) {
            g_unit[u][k] = 9 * u + k;
            g_unit[9 + u][k] = 9 * k + u;
            g_unit[18 + u][k] = ((u / 3) * 3 + k / 3) * 9 + (u % 3) * 3 + k % 3;
        }
}

/* candidate masks (bits 0..8) to a fixpoint of naked and hidden singles:
   -1 contradiction, 0 open cells left, 1 solved */
static int propagate(uint16_t *c)
{
    for (;;) {
        int changed = 0;
        for (int u = 0; u < 27; ++u) {
            uint16_t once = 0, twice = 0, fixed = 0;
            for (int k = 0; k < 9; ++k) {
                const uint16_t m = c[g_unit[u][k]];
                if (__builtin_popcount(m) == 1) {
                    if (fixed & m) return -1;
                    fixed |= m;
                }
                twice |= once & m;
                once |= m;
            }
            if (once != 0x1FF) return -1;
            const uint16_t hidden = once & ~twice & ~fixed;
            for (int k = 0; k < 9; ++k) {
                const int i = g_unit[u][k];
                const uint16_t m = c[i];
                if (__builtin_popcount(m) == 1) continue;
                uint16_t v = m & ~fixed;
                if (v & hidden) {
                    if (__builtin_popcount(v & hidden) > 1) return -1;
                    v &= hidden;
                }
                if (!v) return -1;
                if (v != m) { c[i] = v; changed = 1; }
            }
        }
        if (!changed) break;
    }
    for (int i = 0; i < 81; ++i)
        if (__builtin_popcount(c[i]) > 1) return 0;
    return 1;
}

static int lex_dfs(uint16_t *c, uint64_t *nodes, uint64_t cap)
{
    if (++*nodes >= cap) return 1;          /* stop counting (the caller only thresholds) */
    const int r = propagate(c);
    if (r != 0) return r > 0;
    int i = 0;
    while (__builtin_popcount(c[i]) == 1) ++i;
    uint16_t m = c[i];
    while (m) {
        const uint16_t d = m & (uint16_t)-m;
        m ^= d;
        uint16_t t[81];
        memcpy(t, c, sizeof t);
        t[i] = d;
        if (lex_dfs(t, nodes, cap)) return 1;
    }
    return 0;
}

uint32_t lex_singles_nodes(const uint8_t *puzzle, uint32_t cap)
{
    pthread_once(&g_unit_once, unit_init);
    uint16_t c[81];
    for (int i = 0; i < 81; ++i) c[i] = puzzle[i] ? (uint16_t)(1u << (puzzle[i] - 1)) : 0x1FF;
    uint64_t nodes = 0;
    lex_dfs(c, &nodes, cap);
    return (uint32_t)nodes;
}

enum { JOB_MINIMAL, JOB_NODES, JOB_GRIDS };
typedef struct {
    int kind;
    uint64_t seed, first;
    const uint64_t *idx;
    size_t n;
    uint8_t *p, *s;
    uint32_t *nodes;
    _Atomic size_t next;
} job_t;

static void *worker(void *arg)
{
    job_t *j = (job_t *)arg;
    for (;;) {
        size_t i = atomic_fetch_add(&j->next, 1);
        if (i >= j->n) break;
        if (j->kind == JOB_GRIDS) {
            gen_grid_one(j->seed, j->idx[i], j->s + 81 * i);
        } else if (j->kind == JOB_MINIMAL) {
            gen_minimal_one(j->seed, j->first + i, j->p + 81 * i, j->s + 81 * i);
        } else {
            uint8_t sol[81];
            gen_minimal_one(j->seed, j->first + i, j->p + 81 * i, sol);
            j->nodes[i] = lex_singles_nodes(j->p + 81 * i, 1u << 20);
        }
    }
    return NULL;
}

static int run(job_t *j, int threads)
{
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    for (int t = 1; t < threads; ++t) pthread_create(&tid[t], NULL, worker, j);
    worker(j);
    for (int t = 1; t < threads; ++t) pthread_join(tid[t], NULL);
    return 0;
}

/* puzzles k = first .. first+n-1 of seed `seed`, `threads` threads */
int gen_minimal_batch(uint64_t seed, uint64_t first, size_t n, uint8_t *puzzles, uint8_t *solutions, int threads)
{
    job_t j = {JOB_MINIMAL, seed, first, NULL, n, puzzles, solutions, NULL, 0};
    return run(&j, threads);
}

/* puzzles k = first .. first+n-1 and the singles-DFS search nodes of each (capped at 2^20) */
int gen_minimal_nodes_batch(uint64_t seed, uint64_t first, size_t n, uint8_t *puzzles, uint32_t *nodes, int threads)
{
    job_t j = {JOB_NODES, seed, first, NULL, n, puzzles, NULL, nodes, 0};
    return run(&j, threads);
}

/* the grids of puzzles idx[0..n-1] */
int gen_grid_batch(uint64_t seed, const uint64_t *idx, size_t n, uint8_t *grids, int threads)
{
    job_t j = {JOB_GRIDS, seed, 0, idx, n, NULL, grids, NULL, 0};
    return run(&j, threads);
}
