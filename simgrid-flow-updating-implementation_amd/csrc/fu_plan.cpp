// Host-side launch plans of the collect-all round kernels (see fu_plan.h). No HIP here: the
// engine (fu_engine.hip) uploads what these functions build, and tools/plan_check.cpp runs
// them under ASan/UBSan against a CPU replay of the kernels' indexing.
#include "fu_plan.h"

#include <algorithm>

namespace fu {
namespace plan {

namespace {
I4 i4(int64_t x, int64_t y, int64_t z, int64_t w) { return I4{(int32_t)x, (int32_t)y, (int32_t)z, (int32_t)w}; }
}  // namespace

void build_blocks(int32_t n, int64_t E, const int64_t *rowptr, const int32_t *col, std::vector<int32_t> &blk_row,
                  std::vector<int32_t> &cbase, std::vector<uint16_t> &col16) {
  const int64_t nblk = (E + kR0E - 1) / kR0E;
  blk_row.assign(nblk + 1, 0);
  int32_t i = 0;
  for (int64_t b = 0; b <= nblk; ++b) {
    const int64_t k = b < nblk ? b * kR0E : E - 1;
    while (i + 1 < n && rowptr[i + 1] <= k) ++i;  // last row with rowptr[i] <= k
    blk_row[b] = i;
  }
  // narrow blocks: every column within 32K ids of the block's first row (graphs with
  // locality: RGG in cell order); a wide block keeps cbase -1
  col16.assign(std::max<int64_t>(E, 1), 0);
  cbase.assign(std::max<int64_t>(nblk, 1), -1);
  for (int64_t b = 0; b < nblk; ++b) {
    const int32_t base = blk_row[b];
    bool ok = true;
    const int64_t k1 = std::min<int64_t>(E, (b + 1) * kR0E);
    for (int64_t k = b * kR0E; k < k1 && ok; ++k) {
      const int64_t d = (int64_t)col[k] - base + 32768;
      ok = d >= 0 && d <= 65535;
    }
    if (!ok) continue;
    cbase[b] = base;
    for (int64_t k = b * kR0E; k < k1; ++k) col16[k] = (uint16_t)((int64_t)col[k] - base + 32768);
  }
}

bool build_tiles_geom(const Graph &g, int te, int tn, const TileOpts &o, std::vector<int32_t> &hrows, Tiles &out,
                      std::string *why) {
  out = Tiles{};
  std::vector<I4> heavy, light, hubs;
  const int32_t n = g.n;
  int32_t i = 0;
  while (i < n) {
    const int64_t d = g.deg(i);
    if (d > o.mega_hub) {
      hubs.push_back(i4(i, -3, g.rowptr[i], g.rowptr[i + 1]));
      ++i;
      continue;
    }
    if (d > o.hub_threshold || d > te) {
      heavy.push_back(i4(i, -1, g.rowptr[i], g.rowptr[i + 1]));
      ++i;
      continue;
    }
    const int32_t b = i;
    const int64_t eb = g.rowptr[b];
    while (i < n && i - b < tn) {
      const int64_t di = g.deg(i);
      if (di > o.hub_threshold || di > te || di > o.mega_hub) break;  // (mega_hub may be < hub_threshold)
      if (g.rowptr[i + 1] - eb > te) break;
      ++i;
    }
    light.push_back(i4(b, i, g.rowptr[b], g.rowptr[i]));
  }
  // every mega hub must lead the list: its tile index is its hub_off / hubxy slot
  int64_t n_mega = 0;
  for (int32_t r = 0; r < n; ++r) n_mega += g.deg(r) > o.mega_hub;
  if ((int64_t)hubs.size() != n_mega) {
    if (why) *why = "build_tiles: a mega hub fell into a light tile";
    return false;
  }
  // mega hubs, then heavy tiles first so their long sequential chains start early
  std::vector<I4> &all = out.all;
  all = hubs;
  if (o.wave_heavy && !heavy.empty()) {
    std::vector<int32_t> rows;
    for (const I4 &hv : heavy) rows.push_back(hv.x);
    std::stable_sort(rows.begin(), rows.end(), [&](int32_t x, int32_t y) { return g.deg(x) > g.deg(y); });
    const size_t base = hrows.size();  // each geometry appends its own list
    hrows.insert(hrows.end(), rows.begin(), rows.end());
    out.multi[0] = (int)base;  // this geometry's sorted heavy rows (k_heavy_multi takes a prefix)
    out.multi[1] = (int)rows.size();
    // tiles whose longest (first) row fits kMidRL registers per lane but not kHeavyRL
    out.mid[0] = out.mid[1] = (int)all.size();
    for (size_t q = 0; q < rows.size(); q += 4) {
      const int64_t d0 = g.deg(rows[q]);
      if (d0 > 64 * kMidRL) out.mid[0] = out.mid[1] = (int)all.size() + 1;
      else if (d0 > 64 * kHeavyRL) out.mid[1] = (int)all.size() + 1;
      all.push_back(i4((int64_t)(base + q), -4, (int64_t)std::min<size_t>(4, rows.size() - q), 0));
    }
  } else {
    out.mid[0] = out.mid[1] = (int)hubs.size();
    out.multi[0] = out.multi[1] = 0;
    all.insert(all.end(), heavy.begin(), heavy.end());
  }
  out.nheavy = (int)all.size();
  // the trailing degree-0 rows (the degree layout's isolated rows: R-MAT-24 has 7.9 M, 62 K
  // tiles of 128) run as k_isolated, one thread per row, which writes every row of
  // [iso0, n): so iso0 must lie in the trailing run of degree-0 rows. Trailing edge-less light
  // tiles before a heavy row or a mega hub (layout "given") stay light tiles.
  out.niso = 0;
  out.iso0 = n;
  if (g.na == g.n) {
    int32_t z = n;  // rows [z, n) have degree 0 (never heavy rows or hubs)
    while (z > 0 && g.rowptr[z] == g.rowptr[z - 1]) --z;
    size_t q = light.size();
    while (q > 0 && light[q - 1].x >= z) --q;
    out.niso = (int)(light.size() - q);
    if (out.niso) out.iso0 = light[q].x;
  }
  // multi-GPU (ghost estimate slots exist): light tiles that read a ghost go first, so the
  // halo exchange can start once they are done, beside the interior tiles
  out.nbound = 0;
  if (g.na > g.n) {
    auto has_ghost = [&](const I4 &tl) {
      for (int32_t e = tl.z; e < tl.w; ++e)
        if (g.col[e] >= g.n) return true;
      return false;
    };
    auto mid = std::stable_partition(light.begin(), light.end(), has_ghost);
    out.nbound = (int)(mid - light.begin());
  }
  const size_t nlead = all.size();
  all.insert(all.end(), light.begin(), light.end());
  // light tiles whose kR0E-edge blocks are all narrow read the 2-byte column offsets
  out.narrow.assign(all.size(), 0);
  for (size_t q = nlead; q < all.size() && g.cbase; ++q) {
    const int64_t a0 = all[q].z, a1 = all[q].w;
    bool ok = a1 > a0;
    for (int64_t b = a0 / kR0E; ok && b <= (a1 - 1) / kR0E; ++b) ok = g.cbase[b] >= 0;
    out.narrow[q] = ok ? 1 : 0;
  }
  return true;
}

void build_hubs(const Graph &g, int mega_hub, Hubs &out) {
  out = Hubs{};
  int64_t tot = 0;
  for (int32_t i = 0; i < g.n; ++i) {
    const int64_t d = g.deg(i);
    if (d > mega_hub) {
      out.rows.push_back(i4(i, g.rowptr[i], g.rowptr[i + 1], tot));
      out.off.push_back((int32_t)tot);
      tot += d;
    }
  }
  out.total = tot;
  out.blk.resize((size_t)((tot + kHubBlk - 1) / kHubBlk));
  for (size_t b = 0, hh = 0; b < out.blk.size(); ++b) {
    const int64_t q0 = (int64_t)b * kHubBlk;
    while (hh + 1 < out.off.size() && out.off[hh + 1] <= q0) ++hh;
    out.blk[b] = (int32_t)hh;
  }
}

void build_stage_light(const Graph &g, int hub_threshold, StageLight &out) {
  out = StageLight{};
  const int32_t n = g.n;
  const int64_t lim = std::min<int64_t>(hub_threshold, kStageTE);
  for (int32_t i = 0; i < n;) {
    const int64_t d = g.deg(i);
    if (d > lim) {
      out.heavy.push_back(i4(i, -1, g.rowptr[i], g.rowptr[i + 1]));
      ++i;
      continue;
    }
    const int32_t b = i;
    while (i < n && i - b < kStageTN) {
      const int64_t di = g.deg(i);
      if (di > lim || g.rowptr[i + 1] - g.rowptr[b] > kStageTE) break;
      ++i;
    }
    out.light.push_back(i4(b, i, g.rowptr[b], g.rowptr[i]));
  }
  // multi-GPU (ghost estimate slots exist): light tiles that read a ghost go first, so the
  // halo exchange can start once they are done, beside the interior tiles (as kernel 4)
  if (g.na > g.n) {
    auto has_ghost = [&](const I4 &tl) {
      for (int32_t e = tl.z; e < tl.w; ++e)
        if (g.col[e] >= n) return true;
      return false;
    };
    out.nbound = (int)(std::stable_partition(out.light.begin(), out.light.end(), has_ghost) - out.light.begin());
  }
}

// G is slice-major: for slice s and block part q (the light tiles cut into Q contiguous parts,
// one stage block each), the tiles' edges whose neighbour lies in slice s, tile by tile, in
// position order; each (s, q) region padded to 16 elements (a lane stores 16 bytes) with
// column offset 0 (never read). A tile's edges of one slice are one contiguous run of G: per
// edge the round kernel reads u16 {position, run} and per tile the run offsets D (G index =
// m + D[run], m = index in slice order). A layout is built only if every light tile touches
// at most kStageRuns slices.
int build_stage_layouts(const Graph &g, const std::vector<I4> &light, int n_cu, StageLayout L[4], std::string *why) {
  const int T = (int)light.size();
  std::string w = "kernel 8 (staged slices): no light tiles";
  int built = 0;
  for (int li = 0; li < 4; ++li) L[li] = StageLayout{};
  for (int li = 0; li < 4 && T > 0; ++li) {
    const int64_t SN = std::min<int64_t>(kStageLds >> li, 65536);  // column offsets are u16
    const int64_t P = ((int64_t)g.na + SN - 1) / SN;                 // multi-GPU: the ghost slots are slices too
    if (P > kStageMaxP) {
      w = "kernel 8 (staged slices): more than " + std::to_string(kStageMaxP) + " slices";
      continue;
    }
    const int64_t Q = std::max<int64_t>(1, std::min<int64_t>(T, (n_cu + P / 2) / P));
    auto part = [&](int t) { return (int64_t)t * Q / T; };
    // elements per (slice, part) and runs per tile
    std::vector<int64_t> cnt(P * Q, 0);
    std::vector<int32_t> stamp(P, -1);
    bool ok = true;
    for (int t = 0; t < T && ok; ++t) {
      int runs = 0;
      const int64_t q = part(t);
      for (int32_t e = light[t].z; e < light[t].w; ++e) {
        const int32_t s = g.col[e] / (int32_t)SN;
        if (stamp[s] != t) {
          stamp[s] = t;
          ++runs;
        }
        cnt[s * Q + q]++;
      }
      ok = runs <= kStageRuns;
    }
    if (!ok) {
      w = "kernel 8 (staged slices): a tile touches more than " + std::to_string(kStageRuns) + " slices";
      continue;
    }
    std::vector<int64_t> off(P * Q + 1, 0);
    for (int64_t k = 0; k < P * Q; ++k) off[k + 1] = off[k] + (cnt[k] + 15) / 16 * 16;
    const int64_t total = off[P * Q];
    if (total >= (int64_t)INT32_MAX - 16) {
      w = "kernel 8 (staged slices): staged index exceeds 2^31";
      continue;
    }
    StageLayout &S = L[li];
    S.colS.assign(std::max<int64_t>(total, 16), 0);
    S.sidx16.assign(g.E > 0 ? g.E : 1, 0);
    S.dtab.assign((size_t)T * kStageRuns, 0);
    std::vector<int64_t> cur(off.begin(), off.end() - 1);
    std::vector<int32_t> ord;
    for (int t = 0; t < T; ++t) {
      const int32_t e0 = light[t].z, ne = light[t].w - light[t].z;
      const int64_t q = part(t);
      ord.resize(ne);
      for (int32_t m = 0; m < ne; ++m) ord[m] = m;
      std::stable_sort(ord.begin(), ord.end(),
                       [&](int32_t x, int32_t y) { return g.col[e0 + x] / SN < g.col[e0 + y] / SN; });
      int run = -1;
      int64_t sprev = -1;
      for (int32_t m = 0; m < ne; ++m) {
        const int32_t pos = ord[m];
        const int32_t c = g.col[e0 + pos];
        const int64_t s = c / SN;
        const int64_t gidx = cur[s * Q + q]++;
        S.colS[gidx] = (uint16_t)(c % SN);
        if (s != sprev) {
          ++run;
          sprev = s;
          S.dtab[(size_t)t * kStageRuns + run] = (int32_t)(gidx - m);
        }
        S.sidx16[e0 + m] = (uint16_t)(pos | (run << 10));
      }
    }
    // stage block of region (s, q) at b = 8 (Q (s / 8) + q) + s % 8: the Q blocks of slice s run
    // on one XCD (blocks are dealt round-robin over the 8 XCDs; placement only, never
    // correctness), so the slice's Q - 1 re-reads hit that XCD's L2
    const int64_t NB = 8 * Q * ((P + 7) / 8);
    S.brange.assign(NB, I4{0, 0, 0, 0});
    for (int64_t s2 = 0; s2 < P; ++s2)
      for (int64_t q = 0; q < Q; ++q) {
        const int64_t k = s2 * Q + q, b = 8 * (Q * (s2 / 8) + q) + s2 % 8;
        S.brange[b] = i4(off[k], off[k + 1], s2, 0);
      }
    S.P = (int)P;
    S.Q = (int)Q;
    S.SN = (int)SN;
    S.NB = (int)NB;
    S.total = std::max<int64_t>(total, 16);
    ++built;
  }
  if (!built && why) *why = w;
  return built;
}

// G_A: slice-major, within a slice in edge order, each slice's region starting at a multiple
// of 16 (the stage launch stores 16 bytes per lane); offT[b * P + s] = where bucket b's run of
// slice s starts (offT[B * P + s]: the end of slice s's elements); stage blocks cut each
// slice's region into pieces of about equal element count.
bool build_transpose(const Graph &g, int mega_hub, int n_cu, const int32_t *multi_rows, int n_multi_rows,
                     TransPlan &out, std::string *why) {
  out = TransPlan{};
  const int64_t E = g.E;
  const int64_t SN = kStageLds / 8;
  const int64_t P = ((int64_t)g.na + SN - 1) / SN;  // multi-GPU: the ghost slots are slices too
  if (E == 0 || P > kTrMaxP) {
    if (why) *why = E == 0 ? "kernel 9 (pregather): no edges" : "kernel 9 (pregather): more than 2^25 nodes";
    return false;
  }
  const int64_t B = (E + kTrBE - 1) / kTrBE;
  // buckets [0, Bh) hold every mega-hub edge: transposed first, so the hub chains can start
  int64_t hub_end = 0;
  for (int32_t i = 0; i < g.n; ++i)
    if (g.deg(i) > mega_hub) hub_end = g.rowptr[i + 1];
  std::vector<int64_t> cnt(P, 0);
  for (int64_t e = 0; e < E; ++e) cnt[g.col[e] / SN]++;
  out.reg.assign(P + 1, 0);
  for (int64_t s2 = 0; s2 < P; ++s2) out.reg[s2 + 1] = out.reg[s2] + (cnt[s2] + 15) / 16 * 16;
  const int64_t total = out.reg[P];
  if (total >= (int64_t)INT32_MAX) {
    if (why) *why = "kernel 9 (pregather): more than 2^31 staged elements";
    return false;
  }
  out.colS.assign(total, 0);
  out.pos.assign(total, 0);
  out.offT.assign((size_t)(B + 1) * P, 0);
  std::vector<int64_t> cur(out.reg.begin(), out.reg.end() - 1);
  for (int64_t b = 0; b < B; ++b) {
    for (int64_t s2 = 0; s2 < P; ++s2) out.offT[(size_t)b * P + s2] = (int32_t)cur[s2];
    const int64_t e1 = std::min<int64_t>(E, (b + 1) * kTrBE);
    for (int64_t e = b * kTrBE; e < e1; ++e) {
      const int32_t c = g.col[e];
      const int64_t gi = cur[c / SN]++;
      out.colS[gi] = (uint16_t)(c % SN);
      out.pos[gi] = (uint16_t)(e - b * kTrBE);
    }
  }
  for (int64_t s2 = 0; s2 < P; ++s2) out.offT[(size_t)B * P + s2] = (int32_t)cur[s2];
  // stage pieces by element count, not per slice: under the degree layout the hottest slice
  // holds ~40% of all elements (R-MAT-24), so a slice gets as many blocks as its share
  // (each re-reads the 128 KB slice, mostly from L2)
  const int64_t piece = std::max<int64_t>(16384, (total / (4 * (int64_t)n_cu) + 15) / 16 * 16);
  for (int64_t s2 = 0; s2 < P; ++s2)
    for (int64_t p0 = out.reg[s2]; p0 < out.reg[s2 + 1] || p0 == out.reg[s2]; p0 += piece)
      out.brange.push_back(i4(p0, std::min(out.reg[s2 + 1], p0 + piece), s2, 0));
  out.P = (int)P;
  out.Q = (int)((int64_t)out.brange.size() / P);
  out.NB = (int)out.brange.size();
  out.B = (int)B;
  out.total = total;
  out.Bh = (int)((hub_end + kTrBE - 1) / kTrBE);
  // the multi-row heavy rows of geometry 1 (contiguous after the hubs under the degree layout)
  int64_t mend = hub_end;
  for (int q = 0; q < n_multi_rows; ++q) mend = std::max<int64_t>(mend, g.rowptr[multi_rows[q] + 1]);
  out.Bm = (int)std::max<int64_t>(out.Bh, (mend + kTrBE - 1) / kTrBE);
  return true;
}

K9Sched k9_schedule(const Tiles &t1, int n_hub, const K9Opts &o) {
  K9Sched s;
  s.nmega = n_hub;
  s.nh = t1.nheavy;
  s.niso = o.iso_rows ? t1.niso : 0;  // the trailing degree-0 rows: k_isolated
  s.nl = (int)t1.all.size() - s.nh - s.niso;
  // heavy tiles [m0, m1): the register-resident launch (mid_heavy)
  s.m0 = o.mid_heavy ? std::max(s.nmega, t1.mid[0]) : s.nh;
  s.m1 = o.mid_heavy ? std::max(s.m0, t1.mid[1]) : s.nh;
  // multi_short: the rows of 129-256 edges (heavy tiles [m1, nh)) join the multi-row blocks
  const int mend = o.multi_mid ? (o.multi_short ? s.nh : s.m1) : s.m0;
  s.n_multi = std::min(t1.multi[1], 4 * (mend - s.nmega));
  s.multi = o.multi_heavy && o.mid_heavy && o.wave_heavy && s.n_multi > 0;
  s.m1s = s.multi && o.multi_mid && o.multi_short ? s.nh : s.m1;  // one-row-per-wave tiles [m1s, nh)
  return s;
}

// multi-GPU: no candidate is dropped (tune_out) and none stops early on rank-local timings;
// kernel 9 is single-GPU. Kernel 9 stages the doubles whatever the packing: a candidate of the
// unpacked table only.
static bool tune_active(const TuneRank &r, int c) {
  const bool on = (r.dist || r.tune_out[c] < 2) && !(r.dist && kCands[c].kernel == 9);
  return on && !(kCands[c].kernel == 9 && r.width != 0);
}

void tune_steps(const TuneRank &r, int steps[kNCands]) {
  for (int c = 0; c < kNCands; ++c) {
    steps[c] = kTuneSkip;
    if (!tune_active(r, c)) continue;
    if (kCands[c].kernel == 8 && !r.k8_ok) steps[c] = r.dist ? kTuneStandIn : kTuneSkip;
    else if (kCands[c].kernel == 9 && !r.k9_ok) steps[c] = kTuneSkip;
    else steps[c] = kTuneRun;
  }
}

int tune_need(const TuneRank &r) {
  int need = 0;
  for (int c = 0; c < kNCands; ++c) need += tune_active(r, c) ? 3 + kTimed : 0;  // warm + a confirmation pair + timed
  return need;
}

int tune_rounds_fixed(const TuneRank &r) {
  int st[kNCands];
  tune_steps(r, st);
  int n = 0;
  for (int c = 0; c < kNCands; ++c) n += st[c] != kTuneSkip ? 1 + kTimed : 0;
  return n;
}

}  // namespace plan
}  // namespace fu
