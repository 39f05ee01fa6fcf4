/*
 * sudoku_hip.h -- C-ABI of libsudoku_hip.so, the MI355X (gfx950) Sudoku engine.
 *
 * The reference (jsturm-11/distributed_sudoku_solver) has no FFI: its hot path
 * is two Python call contracts, which this ABI replaces (see INTEGRATION.md for
 * the ctypes binding the reference side would add):
 *
 *   DHTNode.solve_sudoku(puzzle, uuid, arr=range(1,10)) -> bool
 *       DHT_Node.py:474-538 (twin main.py:301-354), with find_next_empty
 *       utils.py:14-25, is_valid utils.py:27-56 and the TASK digit range that
 *       split_array_in_middle (utils.py:1-9) produces.
 *       -> sdk_solve_batch / sdk_solve_batch_dev
 *   Sudoku(grid).check() -> bool            sudoku.py:43-94
 *       -> sdk_check_batch / sdk_check_batch_dev
 *   (no reference counterpart)
 *       -> sdk_count_solutions
 *   DFS subtree split across ring nodes (NEEDWORK/TASK, DHT_Node.py:491-510,
 *   225-250; utils.py:1-9) -- within one node of GPUs:
 *       -> sdk_frontier_* + sdk_comm_* (RCCL over xGMI)
 *
 * Conventions
 *   - Boards are uint8_t[81], row-major, 0 = empty, 1..9 = given digit,
 *     10..255 = an out-of-domain given that (as in the reference, where only
 *     `== guess` comparisons happen) never conflicts with a digit.
 *   - Every function returns SDK_OK (0) or a negative SDK_E* code; the message
 *     of the last failure on the calling thread is sdk_last_error().  No C++
 *     exception and no abort() crosses this boundary.
 *   - An sdk_ctx binds one HIP device and one HIP stream.  Calls on one context
 *     are serialised by an internal mutex; distinct contexts may be used from
 *     different threads concurrently.
 *   - Host-pointer calls are synchronous.  *_dev calls take device pointers,
 *     enqueue on the context stream and return immediately (sdk_synchronize).
 *     Device boards must be 16-byte aligned.
 */
#ifndef SUDOKU_HIP_H
#define SUDOKU_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDK_ABI_VERSION 2   /* 2: sdk_solve_batch_ex, frontier records, p2p send/recv */

/* return codes */
#define SDK_OK        0
#define SDK_EINVAL   -1   /* bad argument */
#define SDK_EHIP     -2   /* HIP runtime failure (message in sdk_last_error) */
#define SDK_ENOMEM   -3   /* device or host allocation failed */
#define SDK_ECOMM    -4   /* RCCL failure (message in sdk_last_error) */

/* per-board solve status (int8_t) */
#define SDK_SOLVED        1   /* out = lexicographically first completion          */
#define SDK_UNSOLVABLE    0   /* out = input (the reference restores the grid)     */
#define SDK_BUDGET_HIT   -2   /* node budget exhausted; out = input                */

/* check verdict bits (uint8_t) */
#define SDK_CHECK_OK        1u  /* intended Sudoku.check(): all 27 units pass     */
#define SDK_CHECK_RAW_NAMEERROR 2u /* reference check() would raise NameError      */
                                   /* (sudoku.py:68): rows ok, cols ok, box00 sum 45 */

/* options for sdk_set_option */
#define SDK_OPT_ORDER        1  /* SDK_ORDER_* (default LEX)                           */
#define SDK_OPT_NODE_BUDGET  2  /* max search nodes per board, 0 = unlimited          */
#define SDK_OPT_WAVES_PER_CU 3  /* solver residency, 1..32 (default 32)               */
#define SDK_OPT_CHECK_BLOCKS_PER_CU 4 /* checker grid = CUs x this, 1..16 (default 3)  */
#define SDK_OPT_WORK_COUNTER 5  /* what solve `work` counts: SDK_WORK_* (default nodes) */
#define SDK_OPT_DEVICE_CUS   6  /* read-only: compute units of the context's GPU        */
#define SDK_OPT_SOLVER       7  /* solve kernel: SDK_SOLVER_* (default QUAD)             */
#define SDK_OPT_WAVES_PER_CU2 8 /* grid of the HALFWAVE / QUAD solver per CU, 1..32 (default 28) */
#define SDK_OPT_CHECK_VARIANT 9 /* checker tile pipeline: SDK_CHECK_* (default REG1) */
#define SDK_OPT_SOLVE_CHUNK  10  /* boards per solver dequeue, 0 = automatic (default)  */
#define SDK_OPT_TIMING       11  /* 1 = bracket every kernel with HIP events for        */
                                 /* sdk_timer_read (default 0: no events are created)    */
#define SDK_OPT_TIMER_EVENTS 12  /* read-only: HIP event pairs the context holds         */
#define SDK_OPT_LOCKED       13  /* QUAD solver: locked-candidates pass (pointing /      */
                                 /* claiming) at propagation fixpoints before branching: */
                                 /* 0 never, 1 at the root node only (default), 2 at     */
                                 /* every node; same answers, fewer search nodes         */
#define SDK_OPT_XCD_HEADS    14  /* QUAD solver: 1 = one dequeue head per XCD segment of */
                                 /* the batch (default), 0 = one shared head             */
#define SDK_OPT_DONATE       15  /* QUAD solver (LEX or MRV_UNIQUE order): phased solve  */
                                 /* with subtree donation.  1 (default) or a split       */
                                 /* budget >= 2: every board first gets at most that     */
                                 /* many search nodes (1: 128); the boards that need     */
                                 /* more are solved again by the donation kernel, where  */
                                 /* idle waves take a heavy board's shallowest untried   */
                                 /* branches.  Same boards and statuses; `work` adds up  */
                                 /* both phases and the board's parts.  0 = off: one     */
                                 /* launch, every board searched by one slot             */
#define SDK_OPT_DONATED      16  /* read-only: branches handed to idle waves by the last */
                                 /* solve's donation phase (waits for it)                */
#define SDK_OPT_SPLIT_BOARDS 17  /* read-only: boards the last solve passed to its       */
                                 /* donation phase                                       */
#define SDK_OPT_DONATE_MODE  18  /* the donation phase's order: 1 (default) exhaustive:  */
                                 /* MRV, at most two completions per board (a unique one */
                                 /* is the lex-first), boards with several are solved    */
                                 /* again in LEX with donation; 0: LEX directly          */
#define SDK_OPT_LEX_BOARDS   19  /* read-only: boards of the last solve's donation phase */
                                 /* that needed the LEX re-solve                         */
#define SDK_OPT_DONATE_MAX   20  /* largest batch solved in phases with donation         */
                                 /* (default 2^19; 0 = any size): a larger batch is one  */
                                 /* launch, where its heavy boards are a small share of  */
                                 /* the time (1M minimal puzzles: the phases cost 6 %)   */
#define SDK_OPT_DN_FAULT     21  /* test only: 1 = idle waves of the donation kernel skip */
                                 /* writing their registration entry, so a donor's       */
                                 /* bounded wait for it runs out: the solve then fails   */
                                 /* with SDK_EHIP (every wait on another wave inside a   */
                                 /* launch is bounded and reports this way)              */
#define SDK_OPT_DONATE_HELPERS 22 /* waves of a donation launch per board it re-solves   */
                                 /* (plus 64; default 2, at most the resident grid)      */
#define SDK_OPT_DONATE_RESUME 23 /* 1 (default): a board the split phase stops resumes  */
                                 /* in the donation launch from its open subtrees (the   */
                                 /* split phase leaves its DFS stack); 0: it restarts    */
#define SDK_OPT_RESUMED      24  /* read-only: boards of the last phased solve resumed   */
                                 /* from their saved stacks (its last pass; waits)       */
#define SDK_OPT_PROP32       25  /* QUAD solver: 1 (default) = a batch is first run      */
                                 /* through bit-sliced root propagation (32 boards per   */
                                 /* half-wave: singles + locked candidates); boards it   */
                                 /* does not decide are searched by solve4 and scattered */
                                 /* back -- same answers and statuses.  Plain solves     */
                                 /* only (no masks, work counters or strided inputs)     */
#define SDK_OPT_PROP32_LC    26  /* ... a locked-candidates pass every N steps (low byte),  */
                                 /* the first after step F (N | F << 8; F = 0: after step */
                                 /* N); default 5 | 3 << 8: after steps 3, 8, 13, ...     */
#define SDK_OPT_PROP32_MIN   27  /* ... for batches of at least N boards (default 4096)   */
#define SDK_OPT_PROP32_UNDECIDED 28 /* read-only: boards the last solve's propagation pass */
                                 /* left to the search (waits)                           */
#define SDK_OPT_PROP32_HANDOVER 29 /* ... 1 (default): with no node budget the search     */
                                 /* starts from a board's propagated grid (same          */
                                 /* completions); 0: from its input                      */
#define SDK_OPT_PROP32_TAIL  30  /* ... live | step << 8: from `step` on, a 64-board     */
                                 /* group with at most `live` boards still open hands     */
                                 /* them to the search (0 = never)                       */

#define SDK_CHECK_REG1       0  /* 1 tile ahead, staged in VGPRs (check_kernel)        */
#define SDK_CHECK_REG2       1  /* 2 tiles ahead, VGPR ring (check_kernel_rr2)         */
#define SDK_CHECK_GLDS2      2  /* LDS-DMA ring of 2 tiles (check_kernel_glds<2>)      */
#define SDK_CHECK_GLDS3      3  /* LDS-DMA ring of 3 tiles (check_kernel_glds<3>)      */
#define SDK_CHECK_GLDS4      4  /* LDS-DMA ring of 4 tiles (check_kernel_glds<4>)      */
#define SDK_CHECK_WAVE1      5  /* per-wave 64-board tiles, no barrier, 1 ahead       */
#define SDK_CHECK_WAVE2      6  /* ... 2 tiles ahead per wave (check_kernel_wave<2>)   */

#define SDK_SOLVER_WAVE      0  /* one board per wavefront (solve_kernel)              */
#define SDK_SOLVER_HALFWAVE  1  /* two boards per wavefront, 27 lanes x 3 cells each   */
#define SDK_SOLVER_QUAD      2  /* four boards per wavefront: HALFWAVE's layout with two */
                                /* boards packed in the 16-bit halves of every word      */
#define SDK_SOLVER_LANE      3  /* one board per lane: the reference's naive DFS itself  */
                                /* (LDS-resident stack); `work` = the reference's        */
                                /* validations, SDK_OPT_NODE_BUDGET counts validations;  */
                                /* SDK_ORDER_LEX only; counts use WAVE                   */

#define SDK_WORK_NODES       0  /* search nodes (propagation fixpoints)                */
#define SDK_WORK_ROUNDS      1  /* propagation rounds (profiling)                      */
#define SDK_WORK_DEPTH       2  /* deepest DFS level reached (profiling, tests)         */

#define SDK_ORDER_MRV_UNIQUE 0  /* MRV search for <=2 solutions; lex re-search if >=2 */
#define SDK_ORDER_LEX        1  /* lowest-index branching after propagation            */

typedef struct sdk_ctx sdk_ctx;

int         sdk_abi_version(void);
const char *sdk_last_error(void);
int         sdk_device_count(int *count);

int sdk_create(int device, sdk_ctx **out);
int sdk_destroy(sdk_ctx *ctx);
int sdk_set_option(sdk_ctx *ctx, int key, int64_t value);
int sdk_get_option(sdk_ctx *ctx, int key, int64_t *value);

/* ---- host-pointer batch API (synchronous) ------------------------------- */

/* Replaces Sudoku.check() (sudoku.py:43-94) for n boards: verdict[i] gets
 * SDK_CHECK_* bits, evaluated with the reference's literal per-unit rule
 * `sum == 45 and len(set) == 9`. */
int sdk_check_batch(sdk_ctx *ctx, const uint8_t *boards, uint8_t *verdict, size_t n);

/* The same for int64 cells (the reference's check() takes any Python int):
 * |value| < 2^59 (else SDK_EINVAL), so a unit's sum is exact. */
int sdk_check_batch_i64(sdk_ctx *ctx, const int64_t *boards, uint8_t *verdict, size_t n);

/* Replaces DHTNode.solve_sudoku (DHT_Node.py:474-538) for n boards.
 *   first_cell_mask  nullable; bit d (1..9) = digit d may be tried at the
 *                    lowest-index empty input cell (the TASK `range`); NULL =
 *                    range(1,10) for every board.
 *   out              lexicographically first completion (= the reference's
 *                    row-major ascending-digit DFS result) when status == 1,
 *                    else a copy of the input.
 *   status           SDK_SOLVED / SDK_UNSOLVABLE / SDK_BUDGET_HIT.
 *   work             nullable; search nodes spent per board (engine counter, not
 *                    the reference's naive-DFS `validations`). */
int sdk_solve_batch(sdk_ctx *ctx, const uint8_t *in, const uint16_t *first_cell_mask,
                    uint8_t *out, int8_t *status, uint64_t *work, size_t n);

/* sdk_solve_batch with the node budget of THIS call (search nodes per board, 0 =
 * unlimited, SDK_BUDGET_CONTEXT = the context's SDK_OPT_NODE_BUDGET): callers that
 * share a context (several ring nodes on one GPU) bound their own launches without
 * touching the shared option.  A board that runs out is SDK_BUDGET_HIT -- never
 * SDK_UNSOLVABLE: its subtree is unexplored, not empty (the reference would still be
 * searching, DHT_Node.py:474-538).  Its launch ends anyway, so one hard board cannot
 * hold back the rest of its batch. */
#define SDK_BUDGET_CONTEXT UINT64_MAX
int sdk_solve_batch_budget(sdk_ctx *ctx, const uint8_t *in, const uint16_t *first_cell_mask,
                           uint8_t *out, int8_t *status, uint64_t *work, size_t n, uint64_t node_budget);

/* sdk_solve_batch_budget with this call's SDK_OPT_DONATE as well (SDK_DONATE_CONTEXT = the
 * context's; 0 = one launch, one slot per board; 1 or a split budget >= 2 = the phased
 * solve with subtree donation).  Threads sharing a context (ring nodes on one GPU, a node's
 * batch and search threads) pick the launch shape per call without touching the shared
 * option. */
#define SDK_DONATE_CONTEXT -1
int sdk_solve_batch_ex(sdk_ctx *ctx, const uint8_t *in, const uint16_t *first_cell_mask,
                       uint8_t *out, int8_t *status, uint64_t *work, size_t n, uint64_t node_budget,
                       int64_t donate);

/* The worklist step of a resumable lex-first search of a board whose solve hit the
 * budget (distributed_sudoku_solver_amd/search.py; the in-node form of handing a
 * subtree on, DHT_Node.py:491-510): expand n boards -- board i with first-cell mask
 * first_cell_masks[i] (nullable = range(1,10) everywhere) -- breadth-first in the
 * reference's DFS order (lowest open cell after propagation, digits ascending, solved
 * boards kept, contradicted ones dropped), at least one level deep and on until the
 * frontier holds >= target boards or nothing branches.  The frontier goes to `out`
 * (*out_n boards, uint8[*out_n][81]); children keep their parents' order, so board k's
 * completions all precede board k+1's in lex order, and the union of their completions
 * is exactly the seeds'.  cap = capacity of `out` in boards; cap >= 9 * max(n, target)
 * always suffices (SDK_EINVAL if the frontier does not fit). */
int sdk_expand_boards(sdk_ctx *ctx, const uint8_t *boards, const uint16_t *first_cell_masks, size_t n,
                      uint64_t target, uint8_t *out, size_t cap, uint64_t *out_n);

/* Counts completions of one board (same constraint as the solver), stopping
 * at `limit` (0 = no limit).  status as above. */
int sdk_count_solutions(sdk_ctx *ctx, const uint8_t *board, uint64_t limit,
                        uint64_t *count, int8_t *status);

/* Multi-GPU form (one context per GPU, one call per rank): every rank expands
 * the same deterministic breadth-first frontier of `board` and counts the
 * subtrees of its contiguous slice; rank 0 also counts the completions met
 * during expansion.  The sum of `count` over ranks is the total (callers
 * all-reduce it).  frontier_size (nullable) = boards in the split frontier. */
int sdk_count_solutions_slice(sdk_ctx *ctx, const uint8_t *board, uint64_t limit, int rank, int world,
                              uint64_t *count, uint64_t *frontier_size, int8_t *status);

/* ---- multi-GPU searches of ONE board ---------------------
 *
 * Every rank builds the same deterministic breadth-first frontier of the board
 * on its own GPU (no exchange), works on its share of it, and combines results
 * with RCCL collectives on device memory, enqueued on the context stream.
 *
 *   SDK_FRONTIER_COUNT  MRV branching; completions met while expanding are
 *                       counted in *leaves (identical on every rank) and dropped.
 *   SDK_FRONTIER_FIRST  lowest-open-cell branching, digits ascending, solved
 *                       boards kept: frontier index order = the reference's DFS
 *                       order (DHT_Node.py:522), so the first frontier board with
 *                       a completion holds the reference's answer.  The digit
 *                       mask (nullable) restricts the lowest empty cell of
 *                       `board`, like a TASK `range`.
 * target = frontier size to reach (0 = 8 boards per resident solver wave). */
#define SDK_FRONTIER_COUNT 0
#define SDK_FRONTIER_FIRST 1
int sdk_frontier_build(sdk_ctx *ctx, const uint8_t *board, const uint16_t *first_cell_mask, int mode,
                       uint64_t target, uint64_t *size, uint64_t *leaves);

/* Count mode: completions below frontier boards first, first+step, ... < end,
 * written to d_result (device, 2 x uint64): {count, boards that hit the node
 * budget}.  The per-board search stops the batch once count >= limit (0 = none). */
/* Second, rank-local stage of a frontier split (count mode): keep boards first,
 * first+step, ... of the frontier built last and expand them further on this device
 * until they number `target` (or nothing branches); *size / *leaves = the refined
 * frontier and the completions met while refining (this rank's alone).  A rank can so
 * take its share of a small replicated frontier and grow it locally, instead of every
 * rank expanding a world-sized frontier. */
int sdk_frontier_refine(sdk_ctx *ctx, uint64_t first, uint64_t step, uint64_t target, uint64_t *size,
                        uint64_t *leaves);
int sdk_frontier_count_dev(sdk_ctx *ctx, uint64_t first, uint64_t step, uint64_t end, uint64_t limit,
                           void *d_result);

/* First mode: solve frontier boards [lo, hi) (each to its lex-first completion)
 * and write the lowest index whose status is not SDK_UNSOLVABLE to d_found
 * (device int64; INT64_MAX if none) and that board's output + status to d_best
 * (device, 82 bytes: board[81], int8 status).  d_found is also the launch's found
 * word: a board that ends solved or at the node budget lowers it, and boards above
 * it stop at their next check ("shards whose index is above the
 * minimum may stop"), so the launch ends once every board below the lowest hit is
 * decided.  The result is the one a launch that solves every board would give. */
int sdk_frontier_first_dev(sdk_ctx *ctx, uint64_t lo, uint64_t hi, void *d_found, void *d_best);

/* Frontier records, for moving live subtrees between ranks (SURVEY §8(e) rebalance; the
 * device form of the reference handing a partial board on mid-search, DHT_Node.py:502-509):
 *   sdk_frontier_boards_dev   *d_boards = device address of the current frontier's
 *                             uint8[*size][81] records (valid until the next frontier call
 *                             on this context); send a range of it with sdk_comm_send_dev.
 *   sdk_frontier_load_dev     the n records at d_boards (device, e.g. received with
 *                             sdk_comm_recv_dev) become the current frontier, in the mode
 *                             of the frontier built last (copied; 0 leaves).
 *   sdk_frontier_refine_range keep frontier boards [lo, hi) and expand them on this device
 *                             until they number `target` (or nothing branches): a rank splits
 *                             its last heavy subtree into second-level records.  The mode is
 *                             the frontier's: count mode counts the completions met while
 *                             refining in *leaves; first mode keeps them in place (lex order,
 *                             *leaves = 0), so the refined range is still sorted by completion. */
int sdk_frontier_boards_dev(sdk_ctx *ctx, void **d_boards, uint64_t *size);
int sdk_frontier_load_dev(sdk_ctx *ctx, const void *d_boards, uint64_t n);
int sdk_frontier_refine_range(sdk_ctx *ctx, uint64_t lo, uint64_t hi, uint64_t target, uint64_t *size,
                              uint64_t *leaves);
/* Keep boards [lo, mid) refined as sdk_frontier_refine_range does, followed by boards
 * [mid, hi) unchanged (the new frontier: refined([lo, mid)) ++ [mid, hi)).  A first-solution
 * search splits the one board that hit its node budget (mid = lo + 1) and keeps the rest of
 * its live range as it is; in first mode the frontier stays sorted by completion. */
int sdk_frontier_refine_head(sdk_ctx *ctx, uint64_t lo, uint64_t mid, uint64_t hi, uint64_t target,
                             uint64_t *size, uint64_t *leaves);

/* RCCL communicator bound to a context (one rank per GPU).  Rank 0 makes the
 * id, the caller distributes it (e.g. over torch.distributed/gloo), every rank
 * calls sdk_comm_init (collective, blocks until all ranks joined). */
#define SDK_COMM_ID_BYTES 128
#define SDK_COMM_U64 0
#define SDK_COMM_I64 1
#define SDK_COMM_U8  2
#define SDK_COMM_SUM 0
#define SDK_COMM_MIN 1
#define SDK_COMM_MAX 2
int sdk_comm_unique_id(uint8_t *id /* SDK_COMM_ID_BYTES */);
int sdk_comm_init(sdk_ctx *ctx, const uint8_t *id, int rank, int world);
/* Single-process form: creates one context per device of
 * `devices` (distinct GPUs) and ONE RCCL clique over them (ncclCommInitAll);
 * ctxs[k] is rank k.  Collectives on the contexts must then be issued from one
 * host thread per context (each call enqueues on its own stream).  On failure
 * no context is left behind (ctxs[k] = NULL).  Release with sdk_destroy. */
int sdk_comm_init_all(const int *devices, int ndev, sdk_ctx **ctxs);
int sdk_comm_destroy(sdk_ctx *ctx);
/* In place, on device memory, enqueued on the context stream. */
int sdk_comm_allreduce_dev(sdk_ctx *ctx, void *d_buf, size_t count, int dtype, int op);
int sdk_comm_broadcast_dev(sdk_ctx *ctx, void *d_buf, size_t bytes, int root);
/* d_recv[r*bytes .. (r+1)*bytes) = rank r's d_send (ncclAllGather): the live-range
 * exchange of the rebalanced frontier count (shard.sharded_count_rebalanced). */
int sdk_comm_allgather_dev(sdk_ctx *ctx, const void *d_send, void *d_recv, size_t bytes);
/* Point-to-point on device memory (ncclSend / ncclRecv inside one ncclGroupStart/End):
 * the frontier-record moves of the rebalanced count.  sdk_comm_p2p_dev issues `nops`
 * operations as one group: ops[k] = SDK_COMM_SEND (bufs[k] -> rank peers[k]) or
 * SDK_COMM_RECV (rank peers[k] -> bufs[k]), bytes[k] each (a matching pair of calls on
 * the two ranks must agree on the size). */
#define SDK_COMM_SEND 0
#define SDK_COMM_RECV 1
int sdk_comm_send_dev(sdk_ctx *ctx, const void *d_buf, size_t bytes, int peer);
int sdk_comm_recv_dev(sdk_ctx *ctx, void *d_buf, size_t bytes, int peer);
int sdk_comm_p2p_dev(sdk_ctx *ctx, int nops, const int *ops, const int *peers, void *const *bufs,
                     const size_t *bytes);

/* ---- device-pointer API (asynchronous on the context stream) ------------ */
int sdk_dev_alloc(sdk_ctx *ctx, size_t bytes, void **dptr);
int sdk_dev_free(sdk_ctx *ctx, void *dptr);
int sdk_memcpy_h2d(sdk_ctx *ctx, void *dst, const void *src, size_t bytes);
int sdk_memcpy_d2h(sdk_ctx *ctx, void *dst, const void *src, size_t bytes);
int sdk_synchronize(sdk_ctx *ctx);

int sdk_check_batch_dev(sdk_ctx *ctx, const void *d_boards, void *d_verdict, size_t n);
int sdk_solve_batch_dev(sdk_ctx *ctx, const void *d_in, const void *d_first_cell_mask,
                        void *d_out, void *d_status, void *d_work, size_t n);

/* Kernel time accounting (HIP events on the context stream, bracketing every
 * kernel launched by the *_dev / host calls since the last reset).  Only with
 * SDK_OPT_TIMING = 1; at most 65536 timed launches between resets (further
 * launches fail with SDK_EINVAL).  Valid after sdk_synchronize. */
int sdk_timer_reset(sdk_ctx *ctx);
int sdk_timer_read(sdk_ctx *ctx, double *total_ms, int64_t *launches);

#ifdef __cplusplus
}
#endif
#endif /* SUDOKU_HIP_H */
