// plan_check: test infrastructure (not linked into libfu). Builds the host-side launch plans
// of the collect-all kernels with the engine's own code (csrc/fu_plan.cpp) and replays every
// kernel's index arithmetic on the CPU, so that an index a kernel would compute from a host
// table is checked without a GPU. Built with -fsanitize=address,undefined (tools/Makefile), so
// the builders themselves run under ASan/UBSan too. Run by tests/test_plan_check.py.
//
// Checked, per graph and option set (the kernels' reads and writes, fu_engine.hip):
//   * k_round0_flows: blk_row, the row search of every 4-edge group;
//   * kernel 4 tiles of the four geometries: every row computed by exactly one launch (mega-hub
//     chains, heavy tiles, light tiles), every flow written once (k_hub_flows for the hubs),
//     light tiles within their geometry, the clamped loads in range, c16 offsets decoding to
//     the column;
//   * kernel 8: the light tiles and heavy rows own every row once; per slice layout the stage
//     blocks (LDS lookups < the slice's nodes, 16-element alignment, disjoint regions) and the
//     tiles' u16 {position, run} and run offsets: every edge's staged element is its neighbour;
//   * kernel 9: the staging launch (as kernel 8), every transpose bucket through the block's
//     own run scan / coarse table / binary search (u16 run starts, nst <= kTrBE), positions
//     written exactly once, the transposed value of edge e equal to
//     col[e] for every e (values = node ids), every bucket visited once per grid (tr_bpx);
//     the launch partition of a round (FP::k9_schedule) for every option combination: each row
//     computed once, each flow written once, k_heavy_multi's rows and history slots in range;
//   * the mega-hub tables: every hub edge's thread finds its hub.
//
//   plan_check --csr FILE | --rmat SCALE EF SEED | --er N M SEED
//              [--layout given|degree] [--mega M]... [--ht T]... [--ghosts K]
// FILE: int64 n, int64 E, int64 rowptr[n + 1], int32 col[E]. Exit 0 = every check passed.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "fu_common.h"
#include "fu_plan.h"

namespace FP = fu::plan;
using FP::I4;

namespace {

long g_fail = 0;
long g_checks = 0;
std::string g_ctx;

#define CHECK(cond, ...)                                                  \
  do {                                                                    \
    ++g_checks;                                                           \
    if (!(cond)) {                                                        \
      if (g_fail < 40) {                                                  \
        std::fprintf(stderr, "FAIL [%s] %s:%d: ", g_ctx.c_str(), __FILE__, __LINE__); \
        std::fprintf(stderr, __VA_ARGS__);                                \
        std::fprintf(stderr, "\n");                                       \
      }                                                                   \
      ++g_fail;                                                           \
    }                                                                     \
  } while (0)

struct Csr {
  int32_t n = 0;
  int32_t na = 0;  // estimate slots (n + ghosts); 0 = n
  int64_t E = 0;
  std::vector<int64_t> rowptr;
  std::vector<int32_t> col;
  int64_t deg(int32_t i) const { return rowptr[i + 1] - rowptr[i]; }
};

constexpr int kBlock = 256;
constexpr int kTrThreads = 1024;

int64_t fe_of(int64_t E) { return std::max<int64_t>(32, (E + 31) / 32 * 32); }  // split-word flow slots

// ---- k_round0_flows ------------------------------------------------------------------
void check_round0(const Csr &g, const std::vector<int32_t> &blk_row) {
  const int64_t nblk = (g.E + FP::kR0E - 1) / FP::kR0E;
  CHECK((int64_t)blk_row.size() == nblk + 1, "blk_row size %zu, want %lld", blk_row.size(), (long long)nblk + 1);
  for (int64_t b = 0; b < nblk; ++b) {
    const int r0 = blk_row[b], span = blk_row[b + 1] - blk_row[b] + 1;
    CHECK(r0 >= 0 && r0 < g.n && span >= 1 && r0 + span <= g.n, "round0 block %lld rows %d +%d", (long long)b, r0, span);
    if (!(r0 >= 0 && span >= 1 && r0 + span <= g.n)) continue;
    auto rp = [&](int q) { return g.rowptr[r0 + q]; };  // the kernel's rowptr[r0 + q], q <= span
    for (int t = 0; t < kBlock; ++t) {
      const int64_t k0 = b * FP::kR0E + 4 * t;
      if (k0 >= g.E) break;
      int lo = 0, hi = span - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (rp(mid) <= k0) lo = mid;
        else hi = mid - 1;
      }
      for (int u = 0; u < 4; ++u) {
        const int64_t k = k0 + u;
        while (lo + 1 < span && rp(lo + 1) <= k) ++lo;
        if (k < g.E) CHECK(g.rowptr[r0 + lo] <= k && k < g.rowptr[r0 + lo + 1], "round0 edge %lld row %d", (long long)k, r0 + lo);
      }
      CHECK(k0 + 3 < fe_of(g.E), "round0 store past the flows at edge %lld", (long long)k0);
    }
  }
}

// ---- kernel 4 tiles (k_round_recon) ----------------------------------------------------
struct Own {
  std::vector<int> row, edge;
  Own(const Csr &g) : row(g.n, 0), edge(g.E, 0) {}
  void add_row(const Csr &g, int32_t i, bool flows) {
    CHECK(i >= 0 && i < g.n, "row %d out of range", i);
    if (i < 0 || i >= g.n) return;
    row[i]++;
    if (flows)
      for (int64_t e = g.rowptr[i]; e < g.rowptr[i + 1]; ++e) edge[e]++;
  }
  void expect_once(const char *what) {
    long bad = 0, first = -1;
    for (size_t i = 0; i < row.size(); ++i)
      if (row[i] != 1) {
        if (first < 0) first = (long)i;
        ++bad;
      }
    CHECK(bad == 0, "%s: %ld rows not computed exactly once (first %ld: %d times)", what, bad, first,
          first >= 0 ? row[first] : 0);
    bad = 0, first = -1;
    for (size_t e = 0; e < edge.size(); ++e)
      if (edge[e] != 1) {
        if (first < 0) first = (long)e;
        ++bad;
      }
    CHECK(bad == 0, "%s: %ld flows not written exactly once (first edge %ld: %d times)", what, bad, first,
          first >= 0 ? edge[first] : 0);
  }
};

// the light-tile path's loads for one tile (PRE: G_B instead of col / col16 + gather)
void light_tile_loads(const Csr &g, const FP::Tiles &t, const std::vector<int32_t> &cbase,
                      const std::vector<uint16_t> &col16, size_t k, int te, int tn, bool pre) {
  const I4 tl = t.all[k];
  const int nb = tl.x, nn = tl.y - tl.x, e0 = tl.z, ne = tl.w - tl.z;
  CHECK(nn >= 1 && nn <= tn, "light tile %zu: %d rows (max %d)", k, nn, tn);
  CHECK(ne >= 0 && ne <= te, "light tile %zu: %d edges (max %d)", k, ne, te);
  CHECK(nb >= 0 && tl.y <= g.n, "light tile %zu rows [%d, %d)", k, nb, tl.y);
  if (nn < 1 || nb < 0 || tl.y > g.n) return;
  CHECK(g.rowptr[nb] == e0 && g.rowptr[tl.y] == tl.w, "light tile %zu: edges [%d, %d) are not its rows'", k, e0, tl.w);
  const int64_t fe = fe_of(g.E);
  for (int tt = 0; tt < kBlock; ++tt) {
    const int tnn = std::min(tt, nn - 1);
    CHECK(nb + std::min(tt, nn) <= g.n && nb + tnn < g.n, "light tile %zu: rowptr / v index", k);
    if (tn == kBlock && tt == 0 && nn == kBlock) CHECK(nb + kBlock <= g.n, "light tile %zu: rl0", k);
  }
  const bool narrow = !pre && t.narrow[k];
  for (int q = 0; q < te; ++q) {
    const int64_t ci = q < ne ? e0 + q : (ne > 0 ? e0 : 0);
    if (!pre) {
      CHECK(ci < std::max<int64_t>(g.E, 1), "light tile %zu: col index %lld", k, (long long)ci);
      if (narrow) {
        CHECK((size_t)ci < col16.size() && (size_t)(ci >> 10) < cbase.size(), "light tile %zu: c16 index", k);
        if (q < ne && (size_t)(ci >> 10) < cbase.size()) {
          const int64_t c = (int64_t)cbase[ci >> 10] + col16[ci] - 32768;
          CHECK(cbase[ci >> 10] >= 0 && c == g.col[ci], "light tile %zu: c16 edge %lld decodes to %lld, col %d", k,
                (long long)ci, (long long)c, g.col[ci]);
        }
      }
      if (q < ne) CHECK(g.col[ci] >= 0 && g.col[ci] < (g.na ? g.na : g.n), "gather index");
    }
    const int64_t fi = q < ne ? e0 + q : 0;
    CHECK(fi < fe, "light tile %zu: flow index %lld", k, (long long)fi);
  }
}

// rows of a heavy tile (-4: four sorted rows; -1: one row), -3: a mega hub
void heavy_tile_rows(const Csr &g, const FP::Tiles &t, const std::vector<int32_t> &hrows, size_t k,
                     std::vector<int32_t> &rows) {
  rows.clear();
  const I4 tl = t.all[k];
  if (tl.y == -4) {
    CHECK(tl.z >= 1 && tl.z <= 4 && tl.x >= t.multi[0] && tl.x + tl.z <= t.multi[0] + t.multi[1] &&
              (size_t)(tl.x + tl.z) <= hrows.size(),
          "heavy tile %zu: hrows [%d, +%d) outside [%d, +%d)", k, tl.x, tl.z, t.multi[0], t.multi[1]);
    for (int w = 0; w < tl.z && (size_t)(tl.x + w) < hrows.size(); ++w) rows.push_back(hrows[tl.x + w]);
  } else {
    CHECK(tl.y == -1 || tl.y == -3, "heavy tile %zu: kind %d", k, tl.y);
    rows.push_back(tl.x);
    if (tl.x >= 0 && tl.x < g.n)
      CHECK(tl.z == g.rowptr[tl.x] && tl.w == g.rowptr[tl.x + 1], "heavy tile %zu: edges of row %d", k, tl.x);
  }
}

void check_hubs(const Csr &g, const FP::Hubs &hb, int mega) {
  const int nhub = (int)hb.rows.size();
  int64_t tot = 0;
  for (int q = 0; q < nhub; ++q) {
    const I4 r = hb.rows[q];
    CHECK(r.x >= 0 && r.x < g.n && g.rowptr[r.x] == r.y && g.rowptr[r.x + 1] == r.z && r.w == tot &&
              hb.off[q] == r.w && r.z - r.y > mega,
          "hub %d: {%d, %d, %d, %d}", q, r.x, r.y, r.z, r.w);
    tot += r.z - r.y;
  }
  CHECK(tot == hb.total, "hub total %lld vs %lld", (long long)tot, (long long)hb.total);
  CHECK((int64_t)hb.blk.size() == (hb.total + FP::kHubBlk - 1) / FP::kHubBlk, "hub_blk size");
  for (int64_t q = 0; q < hb.total; ++q) {  // k_hub_stage / k_hub_flows thread q
    const int64_t b = q / FP::kHubBlk;
    if ((size_t)b >= hb.blk.size()) break;
    int lo = hb.blk[b];
    CHECK(lo >= 0 && lo < nhub, "hub_blk[%lld] = %d", (long long)b, lo);
    if (lo < 0 || lo >= nhub) break;
    while (lo + 1 < nhub && hb.rows[lo + 1].w <= q) ++lo;
    const I4 r = hb.rows[lo];
    const int64_t k = r.y + (q - r.w);
    CHECK(q >= r.w && k >= r.y && k < r.z, "hub edge thread %lld finds hub %d (edge %lld)", (long long)q, lo, (long long)k);
  }
}

// kernel 4 launch (launch_k4_geo): heavy tiles [0, nh) (mega hubs as chains + k_hub_flows),
// light tiles [nh, ntiles)
void check_k4(const Csr &g, const FP::Tiles &t, const std::vector<int32_t> &hrows, const FP::Hubs &hb,
              const std::vector<int32_t> &cbase, const std::vector<uint16_t> &col16, int geo, const FP::TileOpts &o) {
  const int te = FP::kGeoEdges[geo], tn = FP::kGeoNodes[geo];
  Own own(g);
  std::vector<int32_t> rows;
  const int nhub = (int)hb.rows.size();
  CHECK(t.nheavy >= nhub && t.nheavy <= (int)t.all.size(), "nheavy %d, hubs %d, tiles %zu", t.nheavy, nhub, t.all.size());
  for (int k = 0; k < t.nheavy && k < (int)t.all.size(); ++k) {
    const I4 tl = t.all[k];
    if (k < nhub) {
      CHECK(tl.y == -3 && tl.x == hb.rows[k].x, "tile %d is not hub %d", k, k);
      own.add_row(g, tl.x, false);  // chain; k_hub_flows writes its flows
      continue;
    }
    CHECK(tl.y != -3, "mega hub tile %d after the hub tiles", k);
    heavy_tile_rows(g, t, hrows, k, rows);
    for (int32_t i : rows) {
      if (i < 0 || i >= g.n) continue;
      const int64_t d = g.deg(i);
      CHECK((d > o.hub_threshold || d > te) && d <= o.mega_hub, "heavy row %d of degree %lld (threshold %d, te %d)", i,
            (long long)d, o.hub_threshold, te);
      own.add_row(g, i, true);
    }
  }
  for (int q = 0; q < nhub; ++q)
    for (int64_t e = hb.rows[q].y; e < hb.rows[q].z; ++e) own.edge[e]++;  // k_hub_flows
  for (size_t k = t.nheavy; k < t.all.size(); ++k) {
    light_tile_loads(g, t, cbase, col16, k, te, tn, false);
    const I4 tl = t.all[k];
    for (int32_t i = std::max(tl.x, 0); i < std::min(tl.y, g.n); ++i) {
      const int64_t d = g.deg(i);
      CHECK(d <= o.hub_threshold && d <= te && d <= o.mega_hub, "light row %d of degree %lld", i, (long long)d);
      own.add_row(g, i, true);
    }
  }
  own.expect_once("kernel 4");
  // mid ranges, the trailing degree-0 rows
  CHECK(t.mid[0] <= t.mid[1] && t.mid[1] <= t.nheavy && (t.mid[0] >= nhub || t.mid[0] == t.mid[1]),
        "mid [%d, %d), nheavy %d", t.mid[0], t.mid[1], t.nheavy);
  const int nl = (int)t.all.size() - t.nheavy;
  CHECK(t.niso >= 0 && t.niso <= nl, "niso %d of %d light tiles", t.niso, nl);
  if (t.niso) {
    CHECK(t.iso0 == t.all[t.all.size() - t.niso].x, "iso0 %d is not the first isolated tile's row", t.iso0);
    for (int32_t i = t.iso0; i < g.n; ++i) CHECK(g.deg(i) == 0, "k_isolated row %d has degree %lld", i, (long long)g.deg(i));
    int32_t next = t.iso0;  // the isolated tiles cover [iso0, n) contiguously
    for (size_t k = t.all.size() - t.niso; k < t.all.size(); ++k) {
      CHECK(t.all[k].x == next && t.all[k].z == t.all[k].w, "isolated tile %zu", k);
      next = t.all[k].y;
    }
    CHECK(next == g.n, "isolated tiles end at %d, n %d", next, g.n);
  }
}

// kernel 9 launch partition (launch_k9 with FP::k9_schedule)
void check_k9_schedule(const Csr &g, const FP::Tiles &t, const std::vector<int32_t> &hrows, const FP::Hubs &hb,
                       const FP::K9Opts &ko) {
  const FP::K9Sched s = FP::k9_schedule(t, (int)hb.rows.size(), ko);
  Own own(g);
  std::vector<int32_t> rows;
  CHECK(s.nl >= 0 && s.nh + s.nl + s.niso == (int)t.all.size(), "k9: nh %d nl %d niso %d tiles %zu", s.nh, s.nl,
        s.niso, t.all.size());
  for (int k = 0; k < s.nmega; ++k) {  // chains (a_r); k_hub_flows (flows)
    own.add_row(g, t.all[k].x, false);
    for (int64_t e = t.all[k].z; e < t.all[k].w; ++e) own.edge[e]++;
  }
  auto heavy = [&](int t0, int t1) {
    CHECK(t0 >= s.nmega && t1 <= s.nh, "k9 heavy launch [%d, %d) outside [%d, %d)", t0, t1, s.nmega, s.nh);
    for (int k = t0; k < t1; ++k) {
      heavy_tile_rows(g, t, hrows, k, rows);
      for (int32_t i : rows) own.add_row(g, i, true);
    }
  };
  if (s.multi) {
    CHECK(s.n_multi >= 1 && s.n_multi <= t.multi[1], "k9: n_multi %d of %d sorted rows", s.n_multi, t.multi[1]);
    for (int q = 0; q < s.n_multi; ++q) {  // k_heavy_multi block q / kMR, thread q % kMR; hist[q]
      const int32_t i = hrows[t.multi[0] + q];
      own.add_row(g, i, true);
      const int64_t b = g.rowptr[i], d = g.deg(i);
      for (int c = 0; c < (int)((d + 63) / 64) + 2; ++c)  // the clamped loads of every chunk (two ahead)
        for (int lane = 0; lane < 64; lane += 63) {
          const int64_t kk = std::min<int64_t>((int64_t)c * 64 + lane, std::max<int64_t>(d - 1, 0));
          CHECK(b + kk < std::max<int64_t>(g.E, 1), "k_heavy_multi row %d load %lld", i, (long long)(b + kk));
        }
    }
    CHECK(s.n_multi + 1 <= t.multi[1] + 1, "hist slots");
    if (!ko.multi_mid) heavy(s.m0, s.m1);
  } else {
    heavy(s.nmega, s.m0);
    heavy(s.m0, s.m1);
  }
  heavy(s.m1s, s.nh);
  if (s.niso)
    for (int32_t i = t.iso0; i < g.n; ++i) own.add_row(g, i, true);
  for (int k = s.nh; k < s.nh + s.nl; ++k)
    for (int32_t i = std::max(t.all[k].x, 0); i < std::min(t.all[k].y, g.n); ++i) own.add_row(g, i, true);
  char what[160];
  std::snprintf(what, sizeof what, "kernel 9 (mid %d multi_mid %d short %d multi %d wave %d iso %d)", ko.mid_heavy,
                ko.multi_mid, ko.multi_short, ko.multi_heavy, ko.wave_heavy, ko.iso_rows);
  own.expect_once(what);
}

// ---- the staging launch (k_stage), kernels 8 and 9 ------------------------------------
// G element -> slice (from the stage blocks); returns false on a malformed block list
void check_stage_blocks(const std::vector<I4> &br, int NB, int P, int SN, int32_t nslots, int64_t total,
                        std::vector<int32_t> &slice_of, const char *what) {
  CHECK((int)br.size() == NB, "%s: %zu stage blocks, NB %d", what, br.size(), NB);
  slice_of.assign(total, -1);
  for (int bid = 0; bid < NB && bid < (int)br.size(); ++bid) {
    const I4 rg = br[bid];
    if (rg.x >= rg.y) continue;  // an empty region or a grid pad
    CHECK(rg.x >= 0 && rg.y <= total && rg.x % 16 == 0 && (rg.y % 16 == 0 || rg.y == total), "%s: block %d [%d, %d) of %lld",
          what, bid, rg.x, rg.y, (long long)total);
    CHECK(rg.z >= 0 && rg.z < P, "%s: block %d slice %d of %d", what, bid, rg.z, P);
    if (rg.x < 0 || rg.y > total || rg.z < 0 || rg.z >= P) continue;
    const int64_t nb = (int64_t)rg.z * SN;
    const int64_t cnt = std::min<int64_t>(SN, nslots - nb);
    CHECK(cnt >= 1, "%s: block %d slice %d has no nodes", what, bid, rg.z);
    for (int64_t q = rg.x; q < rg.y; ++q) {
      CHECK(slice_of[q] < 0, "%s: G element %lld staged twice", what, (long long)q);
      slice_of[q] = rg.z;
    }
  }
}

void check_k8(const Csr &g, const FP::Graph &pg, int hub_threshold) {
  FP::StageLight sl;
  FP::build_stage_light(pg, hub_threshold, sl);
  Own own(g);
  for (const I4 &hv : sl.heavy) {
    CHECK(hv.y == -1 && g.deg(hv.x) > std::min(hub_threshold, FP::kStageTE), "kernel 8 heavy row %d", hv.x);
    own.add_row(g, hv.x, true);
  }
  for (const I4 &tl : sl.light)
    for (int32_t i = tl.x; i < tl.y; ++i) own.add_row(g, i, true);
  own.expect_once("kernel 8");
  FP::StageLayout L[4];
  std::string why;
  const int built = FP::build_stage_layouts(pg, sl.light, 256, L, &why);
  if (!built) return;  // kernel 8 unavailable (too many slices or runs): nothing launches
  for (int li = 0; li < 4; ++li) {
    const FP::StageLayout &S = L[li];
    if (!S.P) continue;
    char what[32];
    std::snprintf(what, sizeof what, "kernel 8 layout %d", li);
    std::vector<int32_t> slice_of;
    check_stage_blocks(S.brange, S.NB, S.P, S.SN, pg.na, S.total, slice_of, what);
    for (int64_t q = 0; q < S.total; ++q)
      if (slice_of[q] >= 0) {
        const int64_t cnt = std::min<int64_t>(S.SN, pg.na - (int64_t)slice_of[q] * S.SN);
        CHECK(S.colS[q] < cnt, "%s: element %lld LDS offset %u of %lld", what, (long long)q, S.colS[q], (long long)cnt);
      }
    // k_round_staged, every tile
    std::vector<int> seen;
    for (size_t t = 0; t < sl.light.size(); ++t) {
      const I4 tl = sl.light[t];
      const int nn = tl.y - tl.x, e0 = tl.z, ne = tl.w - tl.z;
      CHECK(nn >= 1 && nn <= FP::kStageTN && ne <= FP::kStageTE, "%s: tile %zu %d rows %d edges", what, t, nn, ne);
      seen.assign(ne, 0);
      for (int q = 0; q < ne; ++q) {
        const unsigned c = S.sidx16[e0 + q];
        const int pos = (int)(c & 1023u), run = (int)(c >> 10);
        CHECK(pos < ne && run < FP::kStageRuns, "%s: tile %zu edge %d: pos %d run %d", what, t, q, pos, run);
        if (pos >= ne || run >= FP::kStageRuns) continue;
        seen[pos]++;
        const int64_t gi = q + (int64_t)S.dtab[t * FP::kStageRuns + run];
        CHECK(gi >= 0 && gi < S.total && slice_of[gi] >= 0, "%s: tile %zu edge %d: G index %lld", what, t, q, (long long)gi);
        if (gi < 0 || gi >= S.total || slice_of[gi] < 0) continue;
        const int64_t nbr = (int64_t)slice_of[gi] * S.SN + S.colS[gi];
        CHECK(nbr == g.col[e0 + pos], "%s: tile %zu edge %d stages node %lld, col %d", what, t, e0 + pos,
              (long long)nbr, g.col[e0 + pos]);
      }
      for (int q = 0; q < ne; ++q) CHECK(seen[q] == 1, "%s: tile %zu position %d read %d times", what, t, q, seen[q]);
    }
  }
}

// k_transpose over buckets [b0, b0 + nbk) with tr_bpx blocks per XCD; vals: G_A values (node
// ids), gb: G_B written (checked once per edge by the caller)
void run_transpose(const Csr &g, const FP::TransPlan &T, const std::vector<int64_t> &ga_val, int b0, int nbk, int bpx,
                   std::vector<int64_t> &gb, std::vector<int> &bucket_seen) {
  const int P = T.P;
  const int per = (nbk + 7) / 8;
  const int nj = bpx > 0 ? std::min(per, bpx) : per;  // gridDim.x / 8 (tr_grid)
  std::vector<int32_t> s_m(FP::kTrMaxP + 1), s_o(FP::kTrMaxP), s_c(FP::kTrBE / 64 + 1);
  std::vector<int64_t> s_v(FP::kTrBE);
  std::vector<int> s_hit(FP::kTrBE);
  for (int blk = 0; blk < 8 * nj; ++blk) {
    int bk = (blk & 7) * per + (blk >> 3);
    const int bend = std::min((blk & 7) * per + per, nbk);
    for (; bk < bend; bk += nj) {
      const int bb = b0 + bk;
      CHECK(bb >= 0 && bb < T.B, "transpose bucket %d of %d", bb, T.B);
      if (bb < 0 || bb >= T.B) return;
      bucket_seen[bb]++;
      const int64_t e0 = (int64_t)bb * FP::kTrBE;
      const int ne = (int)std::min<int64_t>(FP::kTrBE, g.E - e0);
      CHECK(P <= 2 * kTrThreads, "transpose: %d slices for %d threads", P, kTrThreads);
      int tot = 0;
      for (int s = 0; s < P; ++s) {  // load_runs + the block scan
        const size_t i0 = (size_t)bb * P + s, i1 = (size_t)(bb + 1) * P + s;
        CHECK(i1 < T.offT.size(), "offT index %zu of %zu", i1, T.offT.size());
        const int o = T.offT[i0], len = T.offT[i1] - o;
        CHECK(len >= 0 && o >= T.reg[s] && o + len <= T.reg[s + 1], "bucket %d slice %d run [%d, +%d) outside [%lld, %lld)",
              bb, s, o, len, (long long)T.reg[s], (long long)T.reg[s + 1]);
        s_m[s] = tot;
        s_o[s] = o;
        tot += len;
      }
      CHECK(tot <= ne && tot <= 65535, "bucket %d: %d staged elements for %d edges", bb, tot, ne);
      s_m[P] = tot;
      const int nst = (int)(uint16_t)tot;  // s_m is u16 in the kernel
      for (int t = 0; t < FP::kTrBE / 64; ++t) {  // coarse table
        const int m = t * 64;
        int lo = 1, hi = P;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if ((int)(uint16_t)s_m[mid] > m) hi = mid;
          else lo = mid + 1;
        }
        s_c[t] = lo;
      }
      s_c[FP::kTrBE / 64] = P;
      std::fill(s_hit.begin(), s_hit.end(), 0);
      for (int m = 0; m < nst && m < FP::kTrBE; ++m) {
        int lo = s_c[m >> 6], hi = s_c[(m >> 6) + 1];
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if ((int)(uint16_t)s_m[mid] > m) hi = mid;
          else lo = mid + 1;
        }
        const int run = lo - 1;
        CHECK(run >= 0 && run < P, "bucket %d element %d: run %d", bb, m, run);
        if (run < 0 || run >= P) continue;
        const int64_t gi = s_o[run] + (m - (int)(uint16_t)s_m[run]);
        CHECK(gi >= 0 && gi < T.total, "bucket %d element %d: G_A index %lld", bb, m, (long long)gi);
        if (gi < 0 || gi >= T.total) continue;
        const int pos = T.pos[gi];
        CHECK(pos < ne, "bucket %d: position %d of %d", bb, pos, ne);
        if (pos >= ne) continue;
        s_v[pos] = ga_val[gi];
        s_hit[pos]++;
      }
      for (int q = 0; q < ne; ++q) {
        CHECK(s_hit[q] == 1, "bucket %d position %d written %d times", bb, q, s_hit[q]);
        CHECK(e0 + q < g.E, "G_B store %lld", (long long)(e0 + q));
        gb[e0 + q] = s_v[q];
      }
    }
  }
}

void check_k9_tables(const Csr &g, const FP::Graph &pg, const FP::Tiles &t1, const std::vector<int32_t> &hrows,
                     int mega, bool hubs) {
  FP::TransPlan T;
  std::string why;
  const int32_t *mrows = hrows.empty() ? nullptr : hrows.data() + t1.multi[0];
  if (!FP::build_transpose(pg, mega, 256, mrows, t1.multi[1], T, &why)) return;  // kernel 9 unavailable
  const char *what = "kernel 9 stage";
  const int SN = FP::kStageLds / 8;
  std::vector<int32_t> slice_of;
  check_stage_blocks(T.brange, T.NB, T.P, SN, pg.na, T.total, slice_of, what);  // k_stage reads a_{r-1}[0, na)
  CHECK((int64_t)T.offT.size() == (int64_t)(T.B + 1) * T.P, "offT size");
  std::vector<int64_t> ga_val(T.total, -1);
  for (int s = 0; s < T.P; ++s) {
    const int64_t used = T.offT[(size_t)T.B * T.P + s];  // end of slice s's elements
    CHECK(used >= T.reg[s] && used <= T.reg[s + 1], "slice %d end %lld", s, (long long)used);
    for (int64_t q = T.reg[s]; q < T.reg[s + 1]; ++q) {
      CHECK(slice_of[q] == s, "%s: G_A element %lld not staged by its slice (%d)", what, (long long)q, slice_of[q]);
      const int64_t cnt = std::min<int64_t>(SN, pg.na - (int64_t)s * SN);
      CHECK(T.colS[q] < cnt, "%s: element %lld LDS offset %u of %lld", what, (long long)q, T.colS[q], (long long)cnt);
      ga_val[q] = (int64_t)s * SN + T.colS[q];  // the stage writes a_{r-1}[s SN + colS]: here the node id
    }
  }
  // the transposes as launch_k9 issues them: the mega-hub buckets [0, Bh), then the rest
  for (int bpx : {32, 3, 0}) {
    std::vector<int64_t> gb(g.E, -1);
    std::vector<int> seen(T.B, 0);
    const int bh = hubs ? T.Bh : 0;
    CHECK(bh >= 0 && bh <= T.B, "Bh %d of %d", bh, T.B);
    if (bh) run_transpose(g, T, ga_val, 0, bh, bpx, gb, seen);
    if (T.B > bh) run_transpose(g, T, ga_val, bh, T.B - bh, bpx, gb, seen);
    for (int b = 0; b < T.B; ++b) CHECK(seen[b] == 1, "tr_bpx %d: bucket %d transposed %d times", bpx, b, seen[b]);
    long bad = 0, first = -1;
    for (int64_t e = 0; e < g.E; ++e)
      if (gb[e] != g.col[e]) {
        if (first < 0) first = (long)e;
        ++bad;
      }
    CHECK(bad == 0, "tr_bpx %d: %ld edges get the wrong estimate (first %ld: %lld, col %d)", bpx, bad, first,
          first >= 0 ? (long long)gb[first] : 0LL, first >= 0 ? g.col[first] : 0);
  }
}

// ---- one option set ----------------------------------------------------------------------
// ghosts > 0: a multi-GPU rank's view: the last `ghosts` node ids become ghost estimate slots
// (rows [0, n - ghosts) local, na = n), as fu_part.cpp numbers them
void check_all(const Csr &g, int mega, int ht, int ghosts = 0) {
  char ctx[112];
  std::snprintf(ctx, sizeof ctx, "n=%d E=%lld mega=%d ht=%d ghosts=%d", g.n, (long long)g.E, mega, ht, ghosts);
  g_ctx = ctx;
  std::vector<int32_t> blk_row, cbase;
  std::vector<uint16_t> col16;
  FP::build_blocks(g.n, g.E, g.rowptr.data(), g.col.data(), blk_row, cbase, col16);
  check_round0(g, blk_row);
  FP::Graph pg;
  pg.n = g.n;
  pg.na = g.n + ghosts;
  pg.E = g.E;
  pg.rowptr = g.rowptr.data();
  pg.col = g.col.data();
  pg.cbase = cbase.data();
  FP::Hubs hb;
  FP::build_hubs(pg, mega, hb);
  check_hubs(g, hb, mega);
  for (int wave : {1, 0}) {
    FP::TileOpts o;
    o.hub_threshold = ht;
    o.mega_hub = mega;
    o.wave_heavy = wave;
    std::vector<int32_t> hrows;
    FP::Tiles tg[4];
    bool ok = true;
    for (int geo = 0; geo < 4; ++geo) {
      std::string why;
      ok = FP::build_tiles_geom(pg, FP::kGeoEdges[geo], FP::kGeoNodes[geo], o, hrows, tg[geo], &why) && ok;
      CHECK(ok, "build_tiles_geom: %s", why.c_str());
    }
    if (!ok) continue;
    for (int geo = 0; geo < 4; ++geo) check_k4(g, tg[geo], hrows, hb, cbase, col16, geo, o);
    // kernel 9 runs geometry 1; its light tiles read G_B (PRE)
    for (size_t k = tg[1].nheavy; k < tg[1].all.size(); ++k)
      light_tile_loads(g, tg[1], cbase, col16, k, FP::kGeoEdges[1], FP::kGeoNodes[1], true);
    for (int mid : {1, 0})
      for (int mm : {1, 0})
        for (int sh : {1, 0})
          for (int mh : {1, 0})
            for (int iso : {1, 0}) {
              FP::K9Opts ko;
              ko.mid_heavy = mid;
              ko.multi_mid = mm;
              ko.multi_short = sh;
              ko.multi_heavy = mh;
              ko.wave_heavy = wave;
              ko.iso_rows = iso;
              check_k9_schedule(g, tg[1], hrows, hb, ko);
            }
    if (wave) check_k9_tables(g, pg, tg[1], hrows, mega, !hb.rows.empty());
    if (ghosts)  // the boundary light tiles (a ghost neighbour) lead the light ones
      for (int geo = 0; geo < 4; ++geo)
        for (size_t k = tg[geo].nheavy; k < tg[geo].all.size(); ++k) {
          bool gh = false;
          for (int32_t e = tg[geo].all[k].z; e < tg[geo].all[k].w; ++e) gh |= g.col[e] >= g.n;
          CHECK(gh == ((int)k < tg[geo].nheavy + tg[geo].nbound), "geometry %d tile %zu: boundary order", geo, k);
        }
  }
  check_k8(g, pg, ht);
}

// the rank view of a graph: rows [0, n - ghosts), columns kept (ids >= n - ghosts are ghosts)
Csr local_view(const Csr &g, int ghosts) {
  Csr l;
  l.n = g.n - ghosts;
  l.na = g.n;
  l.rowptr.assign(g.rowptr.begin(), g.rowptr.begin() + l.n + 1);
  l.E = l.rowptr[l.n];
  l.col.assign(g.col.begin(), g.col.begin() + l.E);
  return l;
}

// ---- the autotune pass (--tune) -----------------------------------------------------------
// Multi-GPU: every rank runs the same rounds in a pass whatever its rank-local state (tune_out
// from its own timings, whether kernel 8 / 9 have layouts on its graph): each round is a halo
// exchange, so a rank running fewer would hang RCCL. Every combination of forced candidate
// drops (tune_out 0..3 per candidate) and missing layouts, per width.
void check_tune() {
  g_ctx = "tune";
  for (int width : {0, 8, 16, 32}) {
    int want_rounds = -1, want_need = -1;
    long combos = 0;
    for (int code = 0; code < (1 << (2 * FP::kNCands)); ++code)
      for (int k8 : {1, 0})
        for (int k9 : {1, 0}) {
          FP::TuneRank r;
          r.dist = true;
          r.width = width;
          r.k8_ok = k8;
          r.k9_ok = k9;
          for (int c = 0; c < FP::kNCands; ++c) r.tune_out[c] = (code >> (2 * c)) & 3;
          const int rounds = FP::tune_rounds_fixed(r), need = FP::tune_need(r);
          if (want_rounds < 0) want_rounds = rounds, want_need = need;
          CHECK(rounds == want_rounds && need == want_need, "width %d tune_out code %d k8 %d k9 %d: %d rounds / need %d, "
                "other ranks %d / %d", width, code, k8, k9, rounds, need, want_rounds, want_need);
          CHECK(rounds <= need, "a pass runs more rounds (%d) than it waits for (%d)", rounds, need);
          int st[FP::kNCands];
          FP::tune_steps(r, st);
          CHECK(st[4] == FP::kTuneSkip, "multi-GPU pass runs kernel 9");
          ++combos;
        }
    std::printf("plan_check --tune: width %d, %ld rank states, %d rounds per multi-GPU pass\n", width, combos,
                want_rounds);
  }
  // one GPU: a dropped candidate (tune_out >= 2) is skipped, kernel 9 only at width 0
  FP::TuneRank r;
  r.tune_out[1] = 2;
  int st[FP::kNCands];
  FP::tune_steps(r, st);
  CHECK(st[1] == FP::kTuneSkip && st[0] == FP::kTuneRun && st[4] == FP::kTuneRun, "single-GPU steps");
  r.width = 8;
  FP::tune_steps(r, st);
  CHECK(st[4] == FP::kTuneSkip, "kernel 9 at a packed width");
}

bool read_csr(const char *path, Csr &g) {
  FILE *f = std::fopen(path, "rb");
  if (!f) return false;
  int64_t hdr[2];
  bool ok = std::fread(hdr, 8, 2, f) == 2;
  if (ok) {
    g.n = (int32_t)hdr[0];
    g.E = hdr[1];
    g.rowptr.resize(g.n + 1);
    g.col.resize(g.E);
    ok = std::fread(g.rowptr.data(), 8, g.n + 1, f) == (size_t)g.n + 1 &&
         std::fread(g.col.data(), 4, g.E, f) == (size_t)g.E;
  }
  std::fclose(f);
  return ok;
}

bool from_handle(fu_graph *h, Csr &g) {
  int32_t n, md, sym;
  int64_t e;
  if (fu_graph_info(h, &n, &e, &md, &sym)) return false;
  g.n = n;
  g.E = e;
  g.rowptr.resize(n + 1);
  g.col.resize(std::max<int64_t>(e, 1));
  if (fu_graph_export(h, g.rowptr.data(), g.col.data(), nullptr)) return false;
  g.col.resize(e);
  return true;
}

}  // namespace

int main(int argc, char **argv) {
  Csr g;
  std::string layout = "given";
  std::vector<int> megas, hts;
  int ghosts = 0;
  fu_graph *gh = nullptr;
  for (int a = 1; a < argc; ++a)
    if (!std::strcmp(argv[a], "--tune")) {
      check_tune();
      std::printf("plan_check --tune: %ld checks, %ld failed\n", g_checks, g_fail);
      return g_fail ? 1 : 0;
    }
  // --tune-rank WIDTH K8_OK K9_OK CODE: the rounds of one multi-GPU autotune pass for one rank
  // state (tune_out of candidate c = (CODE >> 2c) & 3), as the engine runs it
  // (tests/test_bench_cli.py drives bench.py's N > 1 sequence with these counts)
  if (argc == 6 && !std::strcmp(argv[1], "--tune-rank")) {
    FP::TuneRank r;
    r.dist = true;
    r.width = std::atoi(argv[2]);
    r.k8_ok = std::atoi(argv[3]) != 0;
    r.k9_ok = std::atoi(argv[4]) != 0;
    const int code = std::atoi(argv[5]);
    for (int c = 0; c < FP::kNCands; ++c) r.tune_out[c] = (code >> (2 * c)) & 3;
    std::printf("tune_rounds %d need %d\n", FP::tune_rounds_fixed(r), FP::tune_need(r));
    return 0;
  }
  for (int a = 1; a < argc; ++a) {
    const std::string k = argv[a];
    auto need = [&](int cnt) {
      if (a + cnt >= argc) {
        std::fprintf(stderr, "plan_check: %s needs %d values\n", k.c_str(), cnt);
        std::exit(2);
      }
    };
    if (k == "--csr") {
      need(1);
      if (!read_csr(argv[++a], g)) {
        std::fprintf(stderr, "plan_check: cannot read %s\n", argv[a]);
        return 2;
      }
    } else if (k == "--rmat") {
      need(3);
      const int sc = std::atoi(argv[a + 1]), ef = std::atoi(argv[a + 2]);
      const uint64_t seed = std::strtoull(argv[a + 3], nullptr, 10);
      a += 3;
      if (fu_graph_gen_rmat(sc, ef, 0.57, 0.19, 0.19, seed, &gh) || !from_handle(gh, g)) return 2;
    } else if (k == "--er") {
      need(3);
      const int n = std::atoi(argv[a + 1]);
      const int64_t m = std::atoll(argv[a + 2]);
      const uint64_t seed = std::strtoull(argv[a + 3], nullptr, 10);
      a += 3;
      if (fu_graph_gen_er(n, m, seed, &gh) || !from_handle(gh, g)) return 2;
    } else if (k == "--layout") {
      need(1);
      layout = argv[++a];
    } else if (k == "--mega") {
      need(1);
      megas.push_back(std::atoi(argv[++a]));
    } else if (k == "--ht") {
      need(1);
      hts.push_back(std::atoi(argv[++a]));
    } else if (k == "--ghosts") {
      need(1);
      ghosts = std::atoi(argv[++a]);
    } else {
      std::fprintf(stderr, "plan_check: unknown argument %s\n", k.c_str());
      return 2;
    }
  }
  if (g.n <= 0) {
    std::fprintf(stderr, "plan_check: no graph\n");
    return 2;
  }
  if (layout == "degree") {  // the device numbering of fu_create_from_graph_ex(layout 1)
    fu_graph *src = nullptr, *rel = nullptr;
    if (fu_graph_from_csr(g.n, g.rowptr.data(), g.col.data(), 0, &src)) return 2;
    std::vector<int32_t> nofo(g.n);
    if (fu_graph_relabel(src, 1, nofo.data(), &rel) || !from_handle(rel, g)) return 2;
    fu_graph_free(src);
    fu_graph_free(rel);
  }
  if (megas.empty()) megas = {8192};
  if (hts.empty()) hts = {128};
  if (ghosts < 0 || ghosts >= g.n) {
    std::fprintf(stderr, "plan_check: --ghosts must be in [0, n)\n");
    return 2;
  }
  const Csr lv = ghosts ? local_view(g, ghosts) : Csr{};
  for (int mega : megas)
    for (int ht : hts) check_all(ghosts ? lv : g, mega, ht, ghosts);
  if (gh) fu_graph_free(gh);
  std::printf("plan_check: n=%d E=%lld layout=%s: %ld checks, %ld failed\n", g.n, (long long)g.E, layout.c_str(),
              g_checks, g_fail);
  return g_fail ? 1 : 0;
}
