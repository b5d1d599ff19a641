// Host-side launch plans of the collect-all round kernels (fu_engine.hip), as pure C++ with no
// HIP dependency: the kernel 4 tile lists per geometry (mega hubs, heavy rows, light tiles, the
// trailing degree-0 rows), the mega-hub side tables, kernel 8's slice layouts and kernel 9's
// staging and transpose tables, and the launch partition of a kernel-9 round (which launch
// computes which rows, CA:105-128).
//
// libfu.so uploads these tables as they are built here. tools/plan_check.cpp builds the same
// plans under AddressSanitizer / UndefinedBehaviorSanitizer and replays every kernel's index
// arithmetic on the CPU (tests/test_plan_check.py): each load and store in range, each row
// computed by exactly one launch, each staged estimate the neighbour the edge names.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "fu_tuning.h"

namespace fu {
namespace plan {

struct I4 {  // the layout of HIP's int4 (16 bytes)
  int32_t x, y, z, w;
};
static_assert(sizeof(I4) == 16, "I4 must match int4");

// geometry and class constants shared with the kernels
constexpr int kR0E = 1024;                       // round-0 flow blocks; c16 blocks
constexpr int kGeoEdges[4] = {2048, 1024, 1024, 512};
constexpr int kGeoNodes[4] = {256, 128, 256, 64};
constexpr int kStageLds = 131072;                // bytes of estimate table per slice
using ::kStageTE;                                // csrc/fu_tuning.h
using ::kStageTN;
using ::kTrBE;
using ::kHeavyRL;
constexpr int kStageRuns = 64;                   // slice runs per tile the u16 index addresses
constexpr int kStageMaxP = 512;                  // slices per kernel 8 layout
static_assert(kTrBE <= 32768 && kTrBE % 1024 == 0 && kTrBE / 64 <= 1024, "u16 positions, coarse table");
constexpr int kTrMaxP = 2048;                    // kernel 9: slices of 16K nodes (n <= 2^25)
constexpr int kMidRL = 16;                       // kernel 9 register launch: rows of <= 64 x kMidRL
constexpr int kMR = 16;                          // k_heavy_multi: rows per block
constexpr int kHubBlk = 256;                     // k_hub_stage / k_hub_flows threads per block

// The graph as the handle holds it: na = n + ghost estimate slots (multi-GPU).
struct Graph {
  int32_t n = 0, na = 0;
  int64_t E = 0;
  const int64_t *rowptr = nullptr;
  const int32_t *col = nullptr;
  const int32_t *cbase = nullptr;  // per kR0E-edge block: narrow base row or -1 (c16)
  int64_t deg(int32_t i) const { return rowptr[i + 1] - rowptr[i]; }
};

// Round 0 (k_round0_flows) and kernel 4's 2-byte columns, per kR0E-edge block b: blk_row[b]
// = the row of edge b kR0E (blk_row[nblk] = the row of edge E - 1); cbase[b] = that row when
// every column of the block lies within 32K ids of it (col16[e] = col[e] - cbase + 32768),
// else -1 (the block's tiles read the 4-byte columns).
void build_blocks(int32_t n, int64_t E, const int64_t *rowptr, const int32_t *col, std::vector<int32_t> &blk_row,
                  std::vector<int32_t> &cbase, std::vector<uint16_t> &col16);

struct TileOpts {
  int hub_threshold = 128;  // rows above it are heavy rows
  int mega_hub = 8192;      // rows above it are mega hubs
  int wave_heavy = 1;       // heavy rows one per wave, four per tile (else one per block)
};

// Tile list of one geometry: mega hubs {i, -3, b, e}, heavy rows ({hrows offset, -4, count, 0}
// with wave_heavy, else {i, -1, b, e}), then light tiles {first row, end row, first edge,
// end edge}; the boundary light tiles (ghost neighbours) lead the light ones.
struct Tiles {
  std::vector<I4> all;
  std::vector<int32_t> narrow;  // per tile: every kR0E block narrow (c16)
  int nheavy = 0, nbound = 0;
  int mid[2] = {0, 0};          // heavy tiles [mid0, mid1) lead with a row of 64 x (kHeavyRL, kMidRL] edges
  int multi[2] = {0, 0};        // this geometry's sorted heavy rows: offset in hrows, count
  int niso = 0, iso0 = 0;       // trailing light tiles of the last degree-0 rows: [iso0, n)
};
// hrows: the heavy rows of every geometry, appended (this geometry's list at multi[0]).
// Returns false with *why set if a mega hub fell into a light tile.
bool build_tiles_geom(const Graph &g, int te, int tn, const TileOpts &o, std::vector<int32_t> &hrows,
                      Tiles &out, std::string *why);

// Mega hubs (degree > mega_hub): {node, row begin, row end, offset in the hub edge list},
// their offsets, and per kHubBlk-thread block of the hub edges the hub of its first edge.
struct Hubs {
  std::vector<I4> rows;
  std::vector<int32_t> off, blk;
  int64_t total = 0;
};
void build_hubs(const Graph &g, int mega_hub, Hubs &out);

// Kernel 8: light tiles (kStageTE x kStageTN; rows above min(hub_threshold, kStageTE) are
// heavy rows {i, -1, b, e}) and one slice layout per table element width (1, 2, 4, 8 B).
struct StageLight {
  std::vector<I4> light, heavy;
  int nbound = 0;
};
void build_stage_light(const Graph &g, int hub_threshold, StageLight &out);
struct StageLayout {
  int P = 0, Q = 0, SN = 0, NB = 0;  // P = 0: not built
  int64_t total = 0;                 // G elements
  std::vector<I4> brange;            // per stage block: {begin, end} in G, slice, 0
  std::vector<uint16_t> colS;        // per G element: column offset in its slice (pads: 0)
  std::vector<uint16_t> sidx16;      // per light-tile edge, slice order: position | run << 10
  std::vector<int32_t> dtab;         // per light tile: kStageRuns run offsets (G index - m)
};
// Builds the layouts that fit; returns the number built (0: *why says why).
int build_stage_layouts(const Graph &g, const std::vector<I4> &light, int n_cu, StageLayout L[4], std::string *why);

// Kernel 9 (pregather): slices of kStageLds / 8 nodes, buckets of kTrBE edges.
struct TransPlan {
  int P = 0, Q = 0, NB = 0, B = 0, Bh = 0, Bm = 0;
  int64_t total = 0;              // G_A elements (each slice's region padded to 16)
  std::vector<int64_t> reg;       // P + 1: slice regions in G_A
  std::vector<I4> brange;         // stage blocks: {begin, end} in G_A, slice, 0
  std::vector<uint16_t> colS;     // per G_A element: column offset in its slice
  std::vector<uint16_t> pos;      // per G_A element: position in its bucket
  std::vector<int32_t> offT;      // (B + 1) x P: G_A index where bucket b's run of slice s starts
};
// multi_rows: the k_heavy_multi rows of geometry 1 (hrows + multi[0], multi[1] of them).
bool build_transpose(const Graph &g, int mega_hub, int n_cu, const int32_t *multi_rows, int n_multi_rows,
                     TransPlan &out, std::string *why);

// Which launch of a kernel-9 round computes which rows (launch_k9): mega-hub chains
// (tiles [0, nmega)), k_heavy_multi (the first n_multi sorted heavy rows), the heavy tiles
// [m0, m1) in registers when !multi_mid, [nmega, m0) / [m0, m1) when !multi, one row per wave
// [m1s, nh), k_isolated [iso0, n) when niso, the light tiles [nh, nh + nl).
struct K9Opts {
  int mid_heavy = 1, multi_mid = 1, multi_short = 1, multi_heavy = 1, wave_heavy = 1, iso_rows = 1;
};
struct K9Sched {
  int nmega = 0, nh = 0, niso = 0, nl = 0, m0 = 0, m1 = 0, m1s = 0, n_multi = 0;
  bool multi = false;
};
K9Sched k9_schedule(const Tiles &t1, int n_hub, const K9Opts &o);

// Autotune candidates (fixed order: fu_get_info reports per index) and one pass's steps
// (autotune_kernel). Per candidate: skipped, run (a warm round + kTimed timed rounds; on one
// GPU a slow warm round may end the candidate early), or stand-in: a multi-GPU rank on which
// kernel 8 has no slice layout runs kernel 4 rounds in its place, so that every rank runs the
// same rounds (each is a halo exchange: a rank running fewer would hang RCCL, not fail).
struct TuneCand {
  int kernel, geo;
};
constexpr TuneCand kCands[] = {{4, 0}, {4, 3}, {8, 1}, {4, 1}, {9, 1}};
constexpr int kNCands = (int)(sizeof(kCands) / sizeof(kCands[0]));
constexpr int kTimed = 8;  // timed rounds per candidate
enum TuneStep : int { kTuneSkip = 0, kTuneRun = 1, kTuneStandIn = 2 };
struct TuneRank {
  bool dist = false;           // a partitioned (multi-GPU) handle
  int width = 0;               // packing width of the pass (multi-GPU handles never pack)
  int tune_out[kNCands] = {};  // passes in which the candidate was > 1.3x the best (rank-local)
  bool k8_ok = true;           // kernel 8 has a slice layout on this rank's graph
  bool k9_ok = true;           // kernel 9 has a staging layout
};
void tune_steps(const TuneRank &r, int steps[kNCands]);
int tune_need(const TuneRank &r);          // rounds a pass may take (the budget it waits for)
int tune_rounds_fixed(const TuneRank &r);  // rounds of a pass without warm-round drops (multi-GPU)

}  // namespace plan
}  // namespace fu
