// Partition-aware random geometric graph: one rank's slab, built without the global graph.
//
// BASELINE config 5 is RGG with 2^26 nodes over 2/4/8 GPUs. fu_graph_gen_rgg numbers
// nodes in cell order (x-major cells of side >= radius, then generation index). So a
// contiguous range of cell columns is a contiguous range of node ids, and an edge can only
// join adjacent columns. Rank p therefore needs only
//   * the column histogram of all points (one streaming pass over the counter-based RNG),
//     which gives its columns [c_lo, c_hi) balanced by node count and their global id offset;
//   * its own points, plus the points of columns c_lo-1 and c_hi (the halo).
// From these it builds its rows: global neighbour ids, sorted, the same rows as the global
// generator, which the tests check. It also builds the ghost numbering and the halo plan of
// fu_dist_create for the estimates-only halo (kernel 4: flows are rebuilt locally, so
// there are no ghost flows).
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>

#include "fu_common.h"

struct fu_part {
  int32_t nparts = 0, part = 0;
  int64_t n_total = 0, lo = 0, hi = 0;  // global ids [lo, hi)
  std::vector<int64_t> rowptr;          // local rows
  std::vector<int32_t> col;             // ghost-extended: < n_local local, else n_local + g
  std::vector<int64_t> ghost_gid;       // global id of each ghost estimate slot
  std::vector<int64_t> send_a_off, recv_a_off;  // [nparts + 1]
  std::vector<int32_t> send_a_idx;
  int32_t max_deg = 0;
};

namespace {
using namespace fu;

struct Pt {
  double x, y;
  int64_t cell, idx;
};
}  // namespace

extern "C" {

int fu_part_gen_rgg(int64_t n_total, double radius, uint64_t seed, int32_t nparts, int32_t part,
                    fu_part **out) {
  FU_TRY_BEGIN
  if (!out || n_total <= 1 || n_total >= (int64_t)INT32_MAX || !(radius > 0.0) || radius >= 0.5 ||
      nparts < 1 || part < 0 || part >= nparts)
    return fail(FU_ERR_ARG, "fu_part_gen_rgg: bad arguments");
  int64_t G = (int64_t)std::floor(1.0 / radius);
  if (G < 1) G = 1;
  if (G > 65536) G = 65536;
  if (G < nparts) return fail(FU_ERR_ARG, "fu_part_gen_rgg: fewer cell columns than parts (radius too large)");
  auto gen = [&](int64_t i, double &x, double &y, int64_t &cx, int64_t &cy) {
    x = u01(splitmix_at(seed, 2 * (uint64_t)i));
    y = u01(splitmix_at(seed, 2 * (uint64_t)i + 1));
    cx = std::min<int64_t>(G - 1, (int64_t)(x * G));
    cy = std::min<int64_t>(G - 1, (int64_t)(y * G));
  };
  // 1. column histogram (all points)
  std::vector<int64_t> colcnt(G, 0);
#pragma omp parallel
  {
    std::vector<int64_t> loc(G, 0);
#pragma omp for schedule(static)
    for (int64_t i = 0; i < n_total; ++i) {
      double x, y;
      int64_t cx, cy;
      gen(i, x, y, cx, cy);
      loc[cx]++;
    }
#pragma omp critical
    for (int64_t c = 0; c < G; ++c) colcnt[c] += loc[c];
  }
  std::vector<int64_t> colpre(G + 1, 0);
  for (int64_t c = 0; c < G; ++c) colpre[c + 1] = colpre[c] + colcnt[c];
  // 2. column ranges balanced by node count: part q owns [cb[q], cb[q+1])
  std::vector<int64_t> cb(nparts + 1, 0);
  for (int32_t q = 1; q < nparts; ++q) {
    const int64_t target = n_total * q / nparts;
    int64_t c = std::lower_bound(colpre.begin(), colpre.end(), target) - colpre.begin();
    c = std::max<int64_t>(cb[q - 1] + 1, std::min<int64_t>(c, G - (nparts - q)));
    cb[q] = c;
  }
  cb[nparts] = G;
  const int64_t clo = cb[part], chi = cb[part + 1];
  const int64_t hlo = std::max<int64_t>(0, clo - 1), hhi = std::min<int64_t>(G, chi + 1);
  // 3. points of columns [hlo, hhi): own + halo, in global cell order
  std::vector<Pt> pts;
  {
    std::vector<std::vector<Pt>> loc(omp_get_max_threads());
#pragma omp parallel
    {
      auto &mine = loc[omp_get_thread_num()];
#pragma omp for schedule(static)
      for (int64_t i = 0; i < n_total; ++i) {
        double x, y;
        int64_t cx, cy;
        gen(i, x, y, cx, cy);
        if (cx >= hlo && cx < hhi) mine.push_back({x, y, cx * G + cy, i});
      }
    }
    for (auto &v : loc) pts.insert(pts.end(), v.begin(), v.end());
  }
  std::sort(pts.begin(), pts.end(), [](const Pt &a, const Pt &b) {
    return a.cell != b.cell ? a.cell < b.cell : a.idx < b.idx;
  });
  // global id of pts[k] = colpre[hlo] + k (columns are contiguous in cell order)
  const int64_t gbase = colpre[hlo];
  const int64_t lo = colpre[clo], hi = colpre[chi];
  const int64_t own_b = lo - gbase, own_e = hi - gbase;  // own points are pts[own_b, own_e)
  // cell start index inside pts (columns hlo..hhi-1)
  const int64_t ncols = hhi - hlo;
  std::vector<int64_t> cstart(ncols * G + 1, 0);
  for (const Pt &p : pts) cstart[(p.cell / G - hlo) * G + p.cell % G + 1]++;
  for (int64_t q = 0; q < ncols * G; ++q) cstart[q + 1] += cstart[q];
  const double r2 = radius * radius;
  const int64_t n_local = hi - lo;
  std::vector<int64_t> deg(n_local, 0);
  auto scan = [&](int64_t k, std::vector<int64_t> *dst) {
    const Pt &p = pts[k];
    const int64_t cx = p.cell / G, cy = p.cell % G;
    int64_t cnt = 0;
    for (int64_t dx = -1; dx <= 1; ++dx) {
      const int64_t ex = cx + dx;
      if (ex < hlo || ex >= hhi) continue;
      for (int64_t dy = -1; dy <= 1; ++dy) {
        const int64_t ey = cy + dy;
        if (ey < 0 || ey >= G) continue;
        const int64_t q = (ex - hlo) * G + ey;
        for (int64_t j = cstart[q]; j < cstart[q + 1]; ++j) {
          if (j == k) continue;
          const double ddx = p.x - pts[j].x, ddy = p.y - pts[j].y;
          if (ddx * ddx + ddy * ddy < r2) {
            if (dst) dst->push_back(gbase + j);
            ++cnt;
          }
        }
      }
    }
    return cnt;
  };
  auto *P = new fu_part();
  P->nparts = nparts;
  P->part = part;
  P->n_total = n_total;
  P->lo = lo;
  P->hi = hi;
#pragma omp parallel for schedule(dynamic, 4096)
  for (int64_t k = own_b; k < own_e; ++k) deg[k - own_b] = scan(k, nullptr);
  P->rowptr.assign(n_local + 1, 0);
  for (int64_t i = 0; i < n_local; ++i) P->rowptr[i + 1] = P->rowptr[i] + deg[i];
  if (P->rowptr[n_local] >= (int64_t)INT32_MAX) { delete P; return fail(FU_ERR_ARG, "fu_part_gen_rgg: too many local edges"); }
  std::vector<int64_t> gcol(P->rowptr[n_local]);
  int32_t md = 0;
#pragma omp parallel reduction(max : md)
  {
    std::vector<int64_t> buf;
#pragma omp for schedule(dynamic, 4096)
    for (int64_t k = own_b; k < own_e; ++k) {
      buf.clear();
      scan(k, &buf);
      std::sort(buf.begin(), buf.end());
      std::copy(buf.begin(), buf.end(), gcol.begin() + P->rowptr[k - own_b]);
      md = std::max<int32_t>(md, (int32_t)buf.size());
    }
  }
  P->max_deg = md;
  // 4. ghost numbering: remote neighbours grouped by owner part, sorted by global id
  std::vector<int64_t> ghosts;
  for (int64_t g : gcol)
    if (g < lo || g >= hi) ghosts.push_back(g);
  std::sort(ghosts.begin(), ghosts.end());
  ghosts.erase(std::unique(ghosts.begin(), ghosts.end()), ghosts.end());
  P->ghost_gid = ghosts;
  auto owner = [&](int64_t gid) {
    // part q owns global ids [colpre[cb[q]], colpre[cb[q+1]])
    int32_t q = 0;
    while (q + 1 < nparts && gid >= colpre[cb[q + 1]]) ++q;
    return q;
  };
  P->recv_a_off.assign(nparts + 1, 0);
  for (int64_t g : ghosts) P->recv_a_off[owner(g) + 1]++;
  for (int32_t q = 0; q < nparts; ++q) P->recv_a_off[q + 1] += P->recv_a_off[q];
  P->col.resize(gcol.size());
  for (size_t e = 0; e < gcol.size(); ++e) {
    const int64_t g = gcol[e];
    P->col[e] = (g >= lo && g < hi) ? (int32_t)(g - lo)
                                     : (int32_t)(n_local + (std::lower_bound(ghosts.begin(), ghosts.end(), g) - ghosts.begin()));
  }
  // 5. send lists: my nodes adjacent to part q, ascending (== q's ghost order for me)
  P->send_a_off.assign(nparts + 1, 0);
  std::vector<std::vector<int32_t>> sends(nparts);
  for (int64_t i = 0; i < n_local; ++i) {
    int32_t lastq = -1;
    std::vector<int32_t> qs;
    for (int64_t e = P->rowptr[i]; e < P->rowptr[i + 1]; ++e) {
      const int64_t g = gcol[e];
      if (g >= lo && g < hi) continue;
      const int32_t q = owner(g);
      if (std::find(qs.begin(), qs.end(), q) == qs.end()) qs.push_back(q);
    }
    (void)lastq;
    for (int32_t q : qs) sends[q].push_back((int32_t)i);
  }
  for (int32_t q = 0; q < nparts; ++q) {
    P->send_a_off[q + 1] = P->send_a_off[q] + (int64_t)sends[q].size();
    P->send_a_idx.insert(P->send_a_idx.end(), sends[q].begin(), sends[q].end());
  }
  *out = P;
  return FU_OK;
  FU_TRY_END
}

// info: [0] n_local, [1] e_local, [2] lo, [3] hi, [4] n_ghost_a, [5] sends, [6] max_deg, [7] n_total
int fu_part_info(const fu_part *p, int64_t info[8]) {
  if (!p || !info) return fail(FU_ERR_ARG, "fu_part_info: NULL argument");
  info[0] = p->hi - p->lo;
  info[1] = p->rowptr.back();
  info[2] = p->lo;
  info[3] = p->hi;
  info[4] = (int64_t)p->ghost_gid.size();
  info[5] = (int64_t)p->send_a_idx.size();
  info[6] = p->max_deg;
  info[7] = p->n_total;
  return FU_OK;
}

int fu_part_export(const fu_part *p, int64_t *rowptr, int32_t *col, int64_t *ghost_gid,
                   int64_t *send_a_off, int32_t *send_a_idx, int64_t *recv_a_off) {
  if (!p) return fail(FU_ERR_ARG, "fu_part_export: NULL part");
  auto cp = [](void *dst, const void *src, size_t bytes) {
    if (dst && bytes) std::memcpy(dst, src, bytes);
  };
  cp(rowptr, p->rowptr.data(), sizeof(int64_t) * p->rowptr.size());
  cp(col, p->col.data(), sizeof(int32_t) * p->col.size());
  cp(ghost_gid, p->ghost_gid.data(), sizeof(int64_t) * p->ghost_gid.size());
  cp(send_a_off, p->send_a_off.data(), sizeof(int64_t) * p->send_a_off.size());
  cp(send_a_idx, p->send_a_idx.data(), sizeof(int32_t) * p->send_a_idx.size());
  cp(recv_a_off, p->recv_a_off.data(), sizeof(int64_t) * p->recv_a_off.size());
  return FU_OK;
}

int fu_part_free(fu_part *p) {
  delete p;
  return FU_OK;
}

// value[k] = lo + (hi - lo) * U_{first + k} (same stream as fu_values_uniform, any range)
int fu_values_uniform_range(int64_t first, int64_t count, uint64_t seed, double lo, double hi,
                            double *out) {
  if (count < 0 || first < 0 || (count > 0 && !out)) return fail(FU_ERR_ARG, "fu_values_uniform_range: bad arguments");
  const double w = hi - lo;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < count; ++i) out[i] = lo + w * u01(splitmix_at(seed, (uint64_t)(first + i)));
  return FU_OK;
}

}  // extern "C"
