/* fu.h — C ABI of libfu.so, the MI355X-native Flow Updating engine.
 *
 * Drop-in boundary. The reference (AvilaAndre/simgrid-flow-updating-implementation) has no
 * library API. Its "operator API" is the SimGrid actor contract of
 * flowupdating-collectall.py (CA) and flowupdating-pairwise.py (PW):
 *   e.load_platform(...)            CA:154 / PW:143
 *   e.register_actor("peer", Peer)  CA:156 / PW:145
 *   e.load_deployment(...)          CA:157 / PW:146
 *   e.run_until(10000)              CA:164 / PW:153
 *   the watcher + global_values     CA:131-148 / PW:120-137
 * Every `peer` actor and the SimGrid engine behind it are replaced by the entry points
 * below. Host-side Python (the `fu` package) binds them with ctypes, mirroring the
 * Engine/Peer surface. The integration stub is in INTEGRATION.md.
 *
 * Conventions: every function returns int status, 0 = FU_OK and < 0 = error;
 * fu_last_error() returns a thread-local message. All pointers are plain host pointers
 * owned by the caller unless stated. fp64 everywhere (Python float). Indices are int32
 * (n < 2^31, E < 2^31). Each handle owns one HIP stream. Calls on one handle are
 * stream-ordered and not reentrant.
 */
#ifndef FU_H_
#define FU_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FU_OK 0
#define FU_ERR_ARG (-1)
#define FU_ERR_HIP (-2)
#define FU_ERR_ALLOC (-3)
#define FU_ERR_STATE (-4)
#define FU_ERR_GRAPH (-5)
#define FU_ERR_NCCL (-6)

/* Thread-local message for the last failing call on this thread. */
const char *fu_last_error(void);
/* ABI version (bumped when a signature changes). */
int fu_version(void);
/* Number of visible HIP devices (0 without a GPU; never an error on a CPU-only host). */
int fu_device_count(int32_t *out);
/* Free and total bytes of HBM on `device` (hipMemGetInfo): how large a graph still fits. */
int fu_mem_info(int32_t device, int64_t *free_bytes, int64_t *total_bytes);

/* ======================================================================================
 * Host graphs (native C++; no GPU needed)
 * Replaces the deployment parsing SimGrid does for `peer` actors: neighbour lists from
 * actors.xml (ACT:4-27) parsed by Peer.__init__ (CA:29-31, CA:38-40). CSR rows keep the
 * caller's neighbour order, because that order fixes the summation order (CA:106, 110).
 * Generators provide the synthetic BASELINE configs. All are seeded and deterministic
 * (SplitMix64 counter streams, independent of thread count).
 * ==================================================================================== */
typedef struct fu_graph fu_graph;

/* Undirected edge list -> symmetric CSR: drop self-loops, dedup, rows sorted by id. */
int fu_graph_from_edges(int32_t n, int64_t m, const int32_t *src, const int32_t *dst,
                        fu_graph **out);
/* CSR as given (row order kept). If require_symmetric, fails unless every i->j has j->i. */
int fu_graph_from_csr(int32_t n, const int64_t *rowptr, const int32_t *col,
                      int32_t require_symmetric, fu_graph **out);
/* Erdos-Renyi G(n, m): m uniform pairs, self-loops dropped, deduplicated, symmetrised. */
int fu_graph_gen_er(int32_t n, int64_t m, uint64_t seed, fu_graph **out);
/* Random d-regular graph (pairing model + edge switches). n*d must be even. */
int fu_graph_gen_rr(int32_t n, int32_t d, uint64_t seed, fu_graph **out);
/* R-MAT (scale, edge factor, a, b, c; d = 1-a-b-c), symmetrised and deduplicated. */
int fu_graph_gen_rmat(int32_t scale, int32_t edge_factor, double a, double b, double c,
                      uint64_t seed, fu_graph **out);
/* Random geometric graph: n points in the unit square, edge iff distance < radius.
 * Nodes are numbered in cell (x-major) order, which gives locality. */
int fu_graph_gen_rgg(int32_t n, double radius, uint64_t seed, fu_graph **out);
/* n, directed edge count, max degree, 1 if symmetric. */
int fu_graph_info(const fu_graph *g, int32_t *n, int64_t *e, int32_t *max_deg,
                  int32_t *symmetric);
/* Copy out; any output may be NULL. rev[e] = index of the reverse edge (symmetric only). */
int fu_graph_export(const fu_graph *g, int64_t *rowptr, int32_t *col, int32_t *rev);
int fu_graph_free(fu_graph *g);
/* Node relabelling for gather locality: node i of g becomes node new_of_old[i] of *out.
 * Rows move as blocks and keep their neighbour order (the summation order of
 * avg_and_send, CA:106 / CA:110), so a round on *out computes, per node, the same bits.
 * order 0: new_of_old is given (must be a permutation); order 1: degree descending, ties
 * by id (the nodes most gathered first), written to new_of_old. rev follows the rows. */
int fu_graph_relabel(const fu_graph *g, int32_t order, int32_t *new_of_old, fu_graph **out);
/* value[i] = lo + (hi - lo) * U_i, U_i = (splitmix64(seed + (i+1)*0x9E3779B97F4A7C15) >> 11) * 2^-53 */
int fu_values_uniform(int64_t n, uint64_t seed, double lo, double hi, double *out);

/* ======================================================================================
 * Synchronous collect-all engine — THE HOT PATH.
 * One call to fu_run_collectall(h, R, ...) = R generation-synchronous rounds. Each round
 * is Peer.on_receive (CA:93-103) for every directed edge, then Peer.avg_and_send
 * (CA:105-128) for every node, as one data-parallel pass in HBM.
 * Round 0 = the timeout fire on zero state (CA:33-34, CA:87-91). The graph must be
 * symmetric (rev index). Results are bitwise equal to the reference's Python floats.
 * ==================================================================================== */
typedef struct fu_handle fu_handle;

/* rowptr[n+1], col[e], rev[e] (rev may be NULL: computed natively), value[n]. */
int fu_create(int32_t n, int64_t e, const int64_t *rowptr, const int32_t *col,
              const int32_t *rev, const double *value, int32_t device, fu_handle **out);
int fu_create_from_graph(const fu_graph *g, const double *value, int32_t device,
                         fu_handle **out);
/* layout 0 = as fu_create_from_graph; 1 = the device graph is relabelled by degree
 * (fu_graph_relabel order 1) so the most-gathered estimates share cache lines. value,
 * targets, estimates and flows stay in the caller's numbering: the handle maps them. */
int fu_create_from_graph_ex(const fu_graph *g, const double *value, int32_t device,
                            int32_t layout, fu_handle **out);
/* Options (fu_set_option; FU_ERR_ARG for an unknown key or value):
 * "kernel"        0 = auto (fu_tune / autotuned between rounds), 4 = recon (LDS tiles, flow
 *                 reconstruction, direct estimate gathers), 8 = stage (estimates staged slice
 *                 by slice through LDS; single GPU, needs a slice layout), 9 = pregather
 *                 (stage + per-bucket transpose into edge order; single GPU, <= 2^25 nodes).
 *                 All kernels are bitwise equal. On an RCCL rank (fu_dist_create) this
 *                 option is collective: every rank sets it, and a kernel whose layout fails
 *                 on one rank (the slice limits count ghost slots, so they are rank-local)
 *                 fails with FU_ERR_STATE on every rank, so no rank starts rounds alone.
 *                 Kernel 9 on partitions sends its halo after the round (no overlap): it is
 *                 meant for the in-process transport and power-law graphs; auto never picks it.
 * "tile_edges"    kernel 4 tile edges: 2048, 1024 (default) or 512; "tile_nodes" 0/128/256.
 * "hub_threshold" rows of higher degree run as heavy rows, one wave each (default 128).
 * "mega_hub"      rows of higher degree run as mega hubs: one chain-only block each, their
 *                 (fr, er) staged by many blocks (default 8192).
 * "wave_heavy"    heavy rows one per wave (1, default) or one per block (0).
 * "fork_heavy"    kernel 4: heavy tiles on a side stream beside the light tiles (default 1).
 * "split_hubs"    kernel 4: only the mega-hub tiles on the side stream (default 1).
 * "mid_heavy"     kernel 9: heavy rows of 257-1024 edges in a launch of their own that keeps
 *                 the whole row in registers (default 1).
 * "tr_bpx"        kernel 9: transpose blocks per XCD, each looping over buckets (default 32;
 *                 0 = one block per bucket).
 * "multi_heavy"   kernel 9: rows of more than 256 edges as multi-row chain blocks (default 1);
 *                 "multi_mid" 0 keeps the rows of 257-1024 edges in the register launch.
 * "lag"           kernel 9: the multi-row heavy rows leave f_r unwritten and write f_{r-2}
 *                 from f_{r-4} and their kept a_{r-4}, two rounds later (default 1); the
 *                 lagged flows are finalized before fu_get_flows, other kernels and rebuilds.
 * "iso_rows"      kernel 9: the trailing run of degree-0 rows (the degree layout's last rows)
 *                 runs as one thread per row (k_isolated, 1, default) or as light tiles (0).
 * "multi_short"   kernel 9: the rows of 129-256 edges run in the multi-row blocks too (default 1;
 *                 0: one row per wave, four per block).
 * "tr_nt"         kernel 9: k_transpose's G_B stores non-temporal (default 1; its G_A loads are plain
 *                 since round 5: non-temporal loads measured slower, profiles/r05/u).
 * "c16"           kernel 4: 2-byte column offsets for light tiles whose columns lie within
 *                 32K ids of their 1024-edge block's first row (default 1).
 * "pack"          gather lossless 8/16/32-bit codes of the estimates once they cluster
 *                 (default 1); "pack_every" rounds between encoding plans (default 16).
 * "stage_layout"  kernel 8, tests: -1 = by packing width, 0..3 = the 1/2/4/8-byte layout.
 * "staged_lo"     kernel 8: staged indices loaded ahead of the flows (1, default) or
 *                 interleaved with them (0; the round-1 order, kept for A/B and tests).
 * Removed after measurement (FU_ERR_ARG; the numbers are in DESIGN.md §4 and
 * profiles/MEASUREMENTS.md): "tr_pipe", "hub_prio", "side_tiles", "split_tr", "hub_multi",
 * "hub_blocks", "fuse", "light_geo", "tr_hot" (kernel 9), "hub_cus" / "hub_cu_stride" (the
 * hub path on CU-masked streams, profiles/r05/b), "st_split" (kernel 8's next stage beside
 * this round's tiles, profiles/r05/c), "nt" (kernel 4's non-temporal column loads) and "g56"
 * (kernel 8's 7-byte staged codes, profiles/r06/g). */
int fu_set_option(fu_handle *h, const char *key, int64_t value);
/* Zero the state: the next round run is round 0. */
int fu_reset(fu_handle *h);
/* Per-node convergence targets (e.g. exact component means) for the error check. */
int fu_set_targets(fu_handle *h, const double *target);
/* Run `rounds` rounds. If err_every > 0 (targets required), err_trace receives
 * max_i |a_i - target_i| after every err_every-th round (rounds / err_every entries).
 * Asynchronous unless err_trace != NULL. */
int fu_run_collectall(fu_handle *h, int32_t rounds, int32_t err_every, double *err_trace);
/* Same, timed with HIP events on the handle's stream: *ms = elapsed device time of the
 * whole region (synchronises). */
int fu_run_collectall_timed(fu_handle *h, int32_t rounds, float *ms);
/* Kernel "auto": one autotune pass now, at the current packing width, on real rounds
 * (1 warm + 8 timed per candidate, 2 more to confirm a slow warm round before the candidate
 * is dropped; ~45-55 rounds; round 0 first if none ran; packing plans wait). The rounds
 * advance the state: call fu_reset before a run that must start from zero. The winner is
 * kept across fu_reset. Synchronises. Lets a caller tune outside a timed region. */
int fu_tune(fu_handle *h);
/* A timed window in one call: runs rounds_at[n_marks - 1] rounds and records mark k (the
 * event of fu_mark slot k) once rounds_at[k] of them are queued (non-decreasing, rounds_at[0]
 * = 0 marks the start; n_marks <= 64). A single-GPU window that starts at round 0 takes mark 0
 * from round 0's own kernel start and, when rounds_at[1] == 1, mark 1 from its end (events of
 * the launch itself: an event on the idle stream ahead of it would hold the dispatch latency).
 * Asynchronous; read the times with fu_mark_elapsed. bench.py times its windows with it. */
int fu_run_collectall_marked(fu_handle *h, int32_t n_marks, const int32_t *rounds_at);
/* Record HIP event `slot` (0..63) on the handle's stream (asynchronous). */
int fu_mark(fu_handle *h, int32_t slot);
/* *ms = device time between two recorded marks (waits for `to`). */
int fu_mark_elapsed(fu_handle *h, int32_t from, int32_t to, float *ms);
/* max_i |a_i - target_i| on the current estimates (synchronises). */
int fu_max_err(fu_handle *h, double *out);
/* Per-node estimate = last_avg (CA:114, CA:56-63). */
int fu_get_estimates(fu_handle *h, double *a_out);
/* Per-directed-edge flow f[e] = flows[col[e]] of node i (CA:117-118), CSR order. */
int fu_get_flows(fu_handle *h, double *f_out);
int fu_get_round(fu_handle *h, int64_t *rounds_done);
/* info[0] = kernel in use, [1] = nt, [2] = autotune (0 off, 1 pending, 2 done),
 * [3] = rounds done, [4]/[5] = kernel 4 tile geometry (edges / nodes), [6] = autotune
 * passes, [7] = packing width of the last pass, [8..12] = the last pass's ns per round for
 * its candidates (kernel 4 at 2048x256, kernel 4 at 512x64, kernel 8, kernel 4 at
 * 1024x128, kernel 9; 0 = not run), [20] = mega hubs, [23..26] = the autotune winner per
 * packing width 0, 8, 16, 32 (kernel * 10 + kernel-4 geometry index, -1 = not tuned yet),
 * [27..30] = kernel 8 slices per layout (element bytes 1, 2, 4, 8; 0 = not built).
 * With kernel "auto" (the default) fu_tune, or a run with enough rounds left, times the
 * candidates on real rounds (they share state and are bitwise identical) and keeps the
 * fastest; the pass re-runs when the packing plan changes width. */
int fu_get_info(fu_handle *h, int64_t info[32]);  /* ABI 2: 32 entries */
/* Packed estimate table widths (0 = doubles): [0]/[1] = the code tables of the last
 * even/odd round, [2] = the current encoding plan (synchronises). */
int fu_get_pack(fu_handle *h, int32_t width[3]);
int fu_synchronize(fu_handle *h);
int fu_destroy(fu_handle *h);
/* Measurement helper (no reference counterpart): the device's streaming rate, a float4
 * copy of `bytes` bytes (read + write counted) repeated `iters` times on `device`, best of
 * the repetitions in GB/s. bench.py reports it beside the roofline (roofline.copy_GBs) so a
 * slow box reads as a slow copy too. */
int fu_copy_bandwidth(int32_t device, int64_t bytes, int32_t iters, double *gbs);

/* ======================================================================================
 * Tick-level replay (pairwise mode, and faithful collect-all on small platforms).
 * Replaces the SimGrid maestro + Peer.loop (CA:70-85 / PW:69-84): the loop's control flow
 * never depends on fp values, so the whole schedule is precomputed on the host as a trace.
 * The GPU then replays one tick per batch. Events of one tick are on distinct nodes and
 * touch only their own row and message slots, so they commute. Mailbox model: SURVEY.md
 * App. B.
 * ==================================================================================== */
#define FU_MODE_COLLECTALL 0
#define FU_MODE_PAIRWISE 1

#define FU_EV_RECV 0    /* {0, slot, msg_in, 0}     est[slot]=msg.a; flow[slot]=-msg.f (CA:98-99, PW:98-99) */
#define FU_EV_FIRE_CA 1 /* {1, k, out_off, 0}       avg over slots [0,k), k msgs to out_ids[out_off..] (CA:105-125) */
#define FU_EV_FIRE_PW 2 /* {2, slot, k, msg_out}    pairwise avg with slot; flows summed over [0,k) (PW:102-117) */

typedef struct fu_trace fu_trace;

/* Declared neighbour lists (ACT:4-27) in CSR: decl_rowptr[n+1], decl_col. ticks = number
 * of ticks simulated (t = 0 .. ticks-1). order: "fwd" | "rev" | "rand:<seed>" (intra-tick
 * actor order; SimGrid's real tie order is not observable offline). */
int fu_trace_build(int32_t n, const int64_t *decl_rowptr, const int32_t *decl_col,
                   int32_t mode, int32_t ticks, const char *order, fu_trace **out);
/* Same, with fault injection (not in the reference): faults =
 * "drop=P,delay=D:Q,seed=S" (any subset; NULL or "" = none). Each put is lost with
 * probability P or delayed by D ticks with probability Q (SplitMix64 stream in put order).
 * Lost messages exercise the timeouts (CA:87-91, PW:86-91). */
int fu_trace_build_ex(int32_t n, const int64_t *decl_rowptr, const int32_t *decl_col,
                      int32_t mode, int32_t ticks, const char *order, const char *faults,
                      fu_trace **out);
/* Same, with route transfer times: route_s[src * n + dst] = seconds
 * a message from src to dst takes (SimGrid's LV08 model: 13.01 * sum(latency) +
 * size / (0.97 * min bandwidth), fu/platform.py; no link sharing: fu_trace_build_links). A message
 * matched at tick t is consumed from tick t + floor(T) + 1 (t + 1 for T < 1 s, the only
 * case on the reference platform, CA:76). route_s NULL = every route under one tick. */
int fu_trace_build_routes(int32_t n, const int64_t *decl_rowptr, const int32_t *decl_col,
                          int32_t mode, int32_t ticks, const char *order, const char *faults,
                          const double *route_s, fu_trace **out);
/* Same, with link sharing (parity-unpinned against SimGrid): the
 * platform's links (bandwidth B/s, latency s, shared = 0 for FATPIPE) and every route
 * (route_links[route_off[src * n + dst] .. route_off[src * n + dst + 1]), n * n + 1 offsets;
 * an empty route = same host, or a pair the platform does not route: delivery within one
 * tick). A message matched at tick t starts a transfer at time t: lat_factor * sum(latency)
 * with no bandwidth, then msg_bytes at the max-min fair share of bw_factor * bandwidth on
 * every shared link it crosses (capped by its FATPIPE links); it is consumed at the first tick
 * after its end. Alone, a transfer takes the per-route time above (SimGrid LV08: lat_factor
 * 13.01, bw_factor 0.97, 154-byte messages). Every flow on a link gets an EQUAL max-min
 * share here; fu_trace_build_links_ex adds LV08's weighting by sharing penalty and the TCP
 * window bound (the drop-in Engine uses it). The reference platform's 154-byte transfers all
 * end within one tick, where every variant gives the plain schedule. */
int fu_trace_build_links(int32_t n, const int64_t *decl_rowptr, const int32_t *decl_col, int32_t mode,
                         int32_t ticks, const char *order, const char *faults, int32_t n_links,
                         const double *link_bw, const double *link_lat, const int32_t *link_shared,
                         const int64_t *route_off, const int32_t *route_links, double msg_bytes,
                         double lat_factor, double bw_factor, fu_trace **out);
/* fu_trace_build_links with SimGrid LV08's weighted sharing: a transfer's share of a shared
 * link is proportional to 1 / its sharing penalty, the route's latency sum + weight_S /
 * bandwidth of each of its links (LV08: weight_S = 20537), and with tcp_gamma > 0 its rate
 * is capped at tcp_gamma / (2 * latency sum), the TCP window (LV08: 4194304). weight_S = 0
 * and tcp_gamma = 0 are fu_trace_build_links. Parity-unpinned (SimGrid is not installable
 * offline); oracle/oracle.py's LinkNet restates it operation for operation. */
int fu_trace_build_links_ex(int32_t n, const int64_t *decl_rowptr, const int32_t *decl_col, int32_t mode,
                            int32_t ticks, const char *order, const char *faults, int32_t n_links,
                            const double *link_bw, const double *link_lat, const int32_t *link_shared,
                            const int64_t *route_off, const int32_t *route_links, double msg_bytes,
                            double lat_factor, double bw_factor, double weight_S, double tcp_gamma,
                            fu_trace **out);
/* fu_trace_build_links_ex with SimGrid's network/crosstraffic: every transfer also loads each
 * shared link of its reverse route (route dst -> src) with crosstraffic x its rate (the TCP
 * acknowledgements; SimGrid: 0.05), and a FATPIPE link of the reverse route alone caps it at
 * bw_factor * bandwidth / crosstraffic. crosstraffic = 0 is fu_trace_build_links_ex. SimGrid
 * enables it by default, but this repository keeps it OFF by default (the drop-in Engine
 * turns it on with --cfg=network/crosstraffic:1): its effect on a schedule cannot be pinned
 * offline, and on the reference platform every 154-byte transfer ends within its tick with or
 * without it. Parity-unpinned; oracle/oracle.py's LinkNet restates it operation for operation. */
int fu_trace_build_links_cross(int32_t n, const int64_t *decl_rowptr, const int32_t *decl_col, int32_t mode,
                               int32_t ticks, const char *order, const char *faults, int32_t n_links,
                               const double *link_bw, const double *link_lat, const int32_t *link_shared,
                               const int64_t *route_off, const int32_t *route_links, double msg_bytes,
                               double lat_factor, double bw_factor, double weight_S, double tcp_gamma,
                               double crosstraffic, fu_trace **out);
int fu_trace_fault_stats(const fu_trace *t, int64_t *dropped, int64_t *delayed);
/* info[0]=union edges, [1]=tasks, [2]=events, [3]=out_ids, [4]=message slots,
 * [5]=ticks, [6]=dynamic neighbour additions (CA:94-96 errors), [7]=messages sent. */
int fu_trace_info(const fu_trace *t, int64_t info[8]);
/* union_rowptr[n+1] / union_col: neighbour slots in insertion order (declared, then first
 * arrival). tick_task_off[ticks+1]; tasks[3*n_tasks] = (node, ev_begin, ev_end);
 * events[4*n_events]; out_ids[n_out_ids]; first_avg_seq[n] (order of first average:
 * key order of global_values["last_avg"], -1 = never averaged); fires[n]. Any may be NULL. */
int fu_trace_export(const fu_trace *t, int64_t *union_rowptr, int32_t *union_col,
                    int64_t *tick_task_off, int32_t *tasks, int32_t *events,
                    int32_t *out_ids, int64_t *first_avg_seq, int32_t *fires);
int fu_trace_free(fu_trace *t);

typedef struct fu_replay fu_replay;
/* Raw-array form (the trace arrays above, caller-owned). */
int fu_replay_create(int32_t n, const int64_t *rowptr, const double *value, int32_t ticks,
                     const int64_t *tick_task_off, int64_t n_tasks, const int32_t *tasks,
                     int64_t n_events, const int32_t *events, int64_t n_out_ids,
                     const int32_t *out_ids, int64_t n_msgs, int32_t device,
                     fu_replay **out);
int fu_replay_create_from_trace(const fu_trace *t, const double *value, int32_t device,
                                fu_replay **out);
/* Run ticks [current, tick_end). snaps[k*n .. ] receives last_avg after tick
 * snap_ticks[k] (ascending, within the range); snaps may be NULL if n_snap == 0. */
int fu_replay_run(fu_replay *r, int32_t tick_end, int32_t n_snap, const int32_t *snap_ticks,
                  double *snaps);
/* Timed variant: *ms = device time of the tick kernels (synchronises). */
int fu_replay_run_timed(fu_replay *r, int32_t tick_end, float *ms);
int fu_replay_get(fu_replay *r, double *last_avg, double *flows, double *est);
/* "persistent" = 1: one launch for all ticks in dataflow order (per-node event streams,
 * unique message slots tagged by a sentinel); 0 = one launch per tick (default). Same bits.
 * "persistent_reg" = 1 (default): in persistent mode, when every node's thread can be
 * resident and the degree is <= 16, each thread keeps its node's state in registers. */
int fu_replay_set_option(fu_replay *r, const char *key, int64_t value);
int fu_replay_destroy(fu_replay *r);

/* ======================================================================================
 * Multi-GPU (one process per GPU, RCCL over xGMI). The graph is partitioned into
 * contiguous node ranges. Each rank holds its rows plus ghost slots for the reverse flows
 * and estimates of cut edges. One halo exchange per round (ncclSend/ncclRecv to each
 * neighbouring part in one group) replaces the simulated mailboxes (CA:74, CA:124).
 * ==================================================================================== */
#define FU_UNIQUE_ID_BYTES 128
int fu_dist_unique_id(uint8_t *id_out /* FU_UNIQUE_ID_BYTES */);
/* Local part, in local numbering:
 *   n_local rows (global ids [row_begin, row_begin + n_local)), rowptr[n_local+1];
 *   col[e]: < n_local = local node, >= n_local = ghost estimate slot (n_local + g);
 *   rev[e]: < e_local = local edge, >= e_local = ghost flow slot (e_local + q).
 * Halo plan (per peer rank, CSR over peers):
 *   send_f_off[nranks+1] / send_f_idx: local edges whose flow goes to each peer, in the
 *     order that peer stores them in its ghost flow slots;
 *   recv_f_off[nranks+1]: ghost flow slots per peer (contiguous, peer order);
 *   send_a_off / send_a_idx, recv_a_off: the same for estimates of boundary nodes.
 * The round kernels rebuild the neighbours' flows from estimates (flow reconstruction), so
 * the halo carries estimates only: rev must be NULL, n_ghost_f 0 and the flow plan empty
 * (send_f_off / recv_f_off all zero; the parameters stay for ABI stability). */
int fu_dist_create(int32_t n_local, int64_t e_local, const int64_t *rowptr,
                   const int32_t *col, const int32_t *rev, const double *value,
                   int32_t n_ghost_a, int64_t n_ghost_f, int32_t nranks, int32_t rank,
                   const int64_t *send_f_off, const int32_t *send_f_idx,
                   const int64_t *recv_f_off, const int64_t *send_a_off,
                   const int32_t *send_a_idx, const int64_t *recv_a_off,
                   const uint8_t *unique_id, int32_t device, fu_handle **out);

/* In-process transport (one process, e.g. all ranks on one GPU): the same rank handle
 * without a communicator, and the same comm-stream / event chain as RCCL. Each round packs
 * the rank's boundary estimates on its comm stream behind the boundary tiles; after every
 * rank has launched round r, fu_dist_exchange_local(hs, nranks) queues, on each receiver's
 * comm stream, device copies of its peers' packed slots into its ghost slots (the order
 * RCCL uses), beside the interior tiles of round r; round r + 1 waits for them. No host
 * synchronisation. Errors: FU_ERR_STATE if the ranks have run different numbers of rounds
 * or round r's halo was already exchanged. fu_dist_run_local runs `rounds` rounds of every
 * rank, each followed by the exchange. The error all-reduce is left to the caller. This
 * exercises the ghost-slot reads, the pack kernel and the overlapped halo ordering without
 * a multi-GPU box (two RCCL ranks cannot share one GPU). */
int fu_dist_create_local(int32_t n_local, int64_t e_local, const int64_t *rowptr,
                         const int32_t *col, const double *value, int32_t n_ghost_a,
                         int32_t nranks, int32_t rank, const int64_t *send_a_off,
                         const int32_t *send_a_idx, const int64_t *recv_a_off, int32_t device,
                         fu_handle **out);
int fu_dist_exchange_local(fu_handle **hs, int32_t nranks);
int fu_dist_run_local(fu_handle **hs, int32_t nranks, int32_t rounds);
/* Device time (ms) of the last round's halo on the rank's communication stream: from the
 * start of the pack (boundary tiles done) to the ghost slots written. The halo overlaps the
 * round's interior tiles. Waits for that halo. FU_ERR_STATE before the first exchange; 0 for
 * an RCCL rank with nothing to send or receive (one rank), whose rounds skip the
 * communication stream altogether. */
int fu_dist_halo_time(fu_handle *h, float *ms);

/* Partition-aware random geometric graph: rank `part` of `nparts` generates only its slab
 * of cell columns (plus the two halo columns) of the graph fu_graph_gen_rgg(n_total, radius,
 * seed) would build, with the same global node ids and row order. Output: local CSR in
 * ghost numbering and the estimates-only halo plan for fu_dist_create (rev = NULL). */
typedef struct fu_part fu_part;
int fu_part_gen_rgg(int64_t n_total, double radius, uint64_t seed, int32_t nparts,
                    int32_t part, fu_part **out);
/* info[0]=n_local [1]=e_local [2]=lo [3]=hi (global ids) [4]=ghost estimates
 * [5]=boundary sends [6]=max degree [7]=n_total */
int fu_part_info(const fu_part *p, int64_t info[8]);
int fu_part_export(const fu_part *p, int64_t *rowptr, int32_t *col, int64_t *ghost_gid,
                   int64_t *send_a_off, int32_t *send_a_idx, int64_t *recv_a_off);
int fu_part_free(fu_part *p);
/* out[k] = lo + (hi - lo) * U_{first+k}: a slice of the fu_values_uniform stream. */
int fu_values_uniform_range(int64_t first, int64_t count, uint64_t seed, double lo, double hi,
                            double *out);

#ifdef __cplusplus
}
#endif

#endif /* FU_H_ */
