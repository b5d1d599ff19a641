// Host graph construction: CSR + reverse-edge index, seeded synthetic generators.
//
// The reference builds its topology from actors.xml: each Peer splits its neighbour string
// (flowupdating-collectall.py:29-31) into an insertion-ordered dict (CA:38-40). That order
// is the summation order of avg_and_send (CA:106, CA:110), so fu_graph_from_csr keeps row
// order exactly. Generated graphs use rows sorted by neighbour id; the oracle and the
// fixtures use the same CSR, so the order is shared.
//
// Everything here is deterministic for a given seed, whatever the OpenMP thread count:
// random numbers come from SplitMix64 in counter form (splitmix_at(seed, i)), and rows are
// sorted after any parallel scatter.
#include <omp.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <numeric>
#include <unordered_set>

#include "fu_common.h"

namespace fu {

static thread_local std::string g_err;

void set_error(const std::string &msg) { g_err = msg; }
int fail(int code, const std::string &msg) {
  g_err = msg;
  return code;
}

// Symmetric CSR from directed pairs (both directions must already be present or are added
// by the caller). Rows sorted and deduplicated; self-loops dropped.
static void csr_from_directed(int32_t n, const std::vector<uint32_t> &src,
                              const std::vector<uint32_t> &dst, fu_graph &g) {
  const int64_t m = (int64_t)src.size();
  std::vector<std::atomic<int64_t>> cnt(n);
  for (int32_t i = 0; i < n; ++i) cnt[i].store(0, std::memory_order_relaxed);
#pragma omp parallel for schedule(static)
  for (int64_t k = 0; k < m; ++k)
    if (src[k] != dst[k]) cnt[src[k]].fetch_add(1, std::memory_order_relaxed);
  std::vector<int64_t> off(n + 1, 0);
  for (int32_t i = 0; i < n; ++i) off[i + 1] = off[i] + cnt[i].load(std::memory_order_relaxed);
  std::vector<int32_t> tmp(off[n]);
#pragma omp parallel for schedule(static)
  for (int32_t i = 0; i < n; ++i) cnt[i].store(off[i], std::memory_order_relaxed);
#pragma omp parallel for schedule(static)
  for (int64_t k = 0; k < m; ++k)
    if (src[k] != dst[k]) tmp[cnt[src[k]].fetch_add(1, std::memory_order_relaxed)] = (int32_t)dst[k];
  std::vector<int64_t> deg(n);
#pragma omp parallel for schedule(dynamic, 4096)
  for (int32_t i = 0; i < n; ++i) {
    auto b = tmp.begin() + off[i], e = tmp.begin() + off[i + 1];
    std::sort(b, e);
    deg[i] = std::unique(b, e) - b;
  }
  g.n = n;
  g.rowptr.assign(n + 1, 0);
  for (int32_t i = 0; i < n; ++i) g.rowptr[i + 1] = g.rowptr[i] + deg[i];
  g.col.resize(g.rowptr[n]);
  int32_t md = 0;
#pragma omp parallel for schedule(static) reduction(max : md)
  for (int32_t i = 0; i < n; ++i) {
    std::memcpy(g.col.data() + g.rowptr[i], tmp.data() + off[i], sizeof(int32_t) * deg[i]);
    md = std::max<int32_t>(md, (int32_t)deg[i]);
  }
  g.max_deg = md;
}

static void symmetric_from_pairs(int32_t n, const std::vector<uint32_t> &u,
                                 const std::vector<uint32_t> &v, fu_graph &g) {
  std::vector<uint32_t> s(u.size() * 2), d(u.size() * 2);
  const int64_t m = (int64_t)u.size();
#pragma omp parallel for schedule(static)
  for (int64_t k = 0; k < m; ++k) {
    s[2 * k] = u[k];
    d[2 * k] = v[k];
    s[2 * k + 1] = v[k];
    d[2 * k + 1] = u[k];
  }
  csr_from_directed(n, s, d, g);
}

int build_rev(fu_graph &g) {
  const int32_t n = g.n;
  const int64_t E = g.rowptr[n];
  if (E > (int64_t)INT32_MAX)  // rev is int32 (fu_graph_export): no silent truncation
    return fail(FU_ERR_GRAPH, "graph has " + std::to_string(E) +
                                  " directed edges, more than an int32 reverse index holds; run it as partitions "
                                  "(fu_part_gen_rgg + fu_dist_create_local)");
  // sorted view of every row: perm[rowptr[i]..] = positions sorted by neighbour id
  std::vector<int32_t> perm(E);
  bool all_sorted = true;
#pragma omp parallel for schedule(dynamic, 4096) reduction(&& : all_sorted)
  for (int32_t i = 0; i < n; ++i) {
    int64_t b = g.rowptr[i], e = g.rowptr[i + 1];
    for (int64_t k = b; k < e; ++k) perm[k] = (int32_t)(k - b);
    bool sorted = true;
    for (int64_t k = b + 1; k < e; ++k)
      if (g.col[k - 1] >= g.col[k]) { sorted = false; break; }
    if (!sorted) {
      std::sort(perm.begin() + b, perm.begin() + e,
                [&](int32_t x, int32_t y) { return g.col[b + x] < g.col[b + y]; });
      all_sorted = false;
    }
  }
  g.rev.assign(E, -1);
  std::atomic<int64_t> bad{-1};
#pragma omp parallel for schedule(dynamic, 4096)
  for (int32_t i = 0; i < n; ++i) {
    for (int64_t k = g.rowptr[i]; k < g.rowptr[i + 1]; ++k) {
      int32_t j = g.col[k];
      int64_t b = g.rowptr[j], e = g.rowptr[j + 1];
      int64_t lo = 0, hi = e - b;
      while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (g.col[b + perm[b + mid]] < i) lo = mid + 1;
        else hi = mid;
      }
      if (lo < e - b && g.col[b + perm[b + lo]] == i) g.rev[k] = (int32_t)(b + perm[b + lo]);
      else bad.store(k, std::memory_order_relaxed);
    }
  }
  (void)all_sorted;
  if (bad.load() >= 0) {
    g.rev.clear();
    return fail(FU_ERR_GRAPH, "graph is not symmetric (edge " + std::to_string(bad.load()) +
                                  " has no reverse edge)");
  }
  return FU_OK;
}

}  // namespace fu

using namespace fu;

extern "C" {

const char *fu_last_error(void) { return fu::g_err.c_str(); }
int fu_version(void) { return 2; }

int fu_graph_from_edges(int32_t n, int64_t m, const int32_t *src, const int32_t *dst,
                        fu_graph **out) {
  FU_TRY_BEGIN
  if (!out || n <= 0 || m < 0 || (m > 0 && (!src || !dst))) return fail(FU_ERR_ARG, "fu_graph_from_edges: bad arguments");
  std::vector<uint32_t> u(m), v(m);
  for (int64_t k = 0; k < m; ++k) {
    if (src[k] < 0 || src[k] >= n || dst[k] < 0 || dst[k] >= n)
      return fail(FU_ERR_ARG, "fu_graph_from_edges: node id out of range");
    u[k] = (uint32_t)src[k];
    v[k] = (uint32_t)dst[k];
  }
  auto *g = new fu_graph();
  symmetric_from_pairs(n, u, v, *g);
  int rc = build_rev(*g);
  if (rc) { delete g; return rc; }
  *out = g;
  return FU_OK;
  FU_TRY_END
}

int fu_graph_from_csr(int32_t n, const int64_t *rowptr, const int32_t *col,
                      int32_t require_symmetric, fu_graph **out) {
  FU_TRY_BEGIN
  if (!out || n <= 0 || !rowptr || rowptr[0] != 0) return fail(FU_ERR_ARG, "fu_graph_from_csr: bad arguments");
  const int64_t E = rowptr[n];
  if (E > 0 && !col) return fail(FU_ERR_ARG, "fu_graph_from_csr: col is NULL");
  if (E >= (int64_t)INT32_MAX) return fail(FU_ERR_ARG, "fu_graph_from_csr: more than 2^31-1 edges");
  auto *g = new fu_graph();
  g->n = n;
  g->rowptr.assign(rowptr, rowptr + n + 1);
  g->col.assign(col, col + E);
  int32_t md = 0;
  for (int32_t i = 0; i < n; ++i) {
    if (rowptr[i + 1] < rowptr[i]) { delete g; return fail(FU_ERR_ARG, "fu_graph_from_csr: rowptr not monotone"); }
    md = std::max<int32_t>(md, (int32_t)(rowptr[i + 1] - rowptr[i]));
    for (int64_t k = rowptr[i]; k < rowptr[i + 1]; ++k) {
      if (col[k] < 0 || col[k] >= n) { delete g; return fail(FU_ERR_ARG, "fu_graph_from_csr: neighbour id out of range"); }
      if (col[k] == i) { delete g; return fail(FU_ERR_GRAPH, "fu_graph_from_csr: self-loop at node " + std::to_string(i)); }
    }
  }
  g->max_deg = md;
  // duplicates inside a row are not allowed (the reference's dict keys are unique, CA:38-40)
  {
    std::vector<int32_t> tmp;
    for (int32_t i = 0; i < n; ++i) {
      tmp.assign(col + rowptr[i], col + rowptr[i + 1]);
      std::sort(tmp.begin(), tmp.end());
      if (std::adjacent_find(tmp.begin(), tmp.end()) != tmp.end()) {
        delete g;
        return fail(FU_ERR_GRAPH, "fu_graph_from_csr: duplicate neighbour in row " + std::to_string(i));
      }
    }
  }
  int rc = build_rev(*g);
  if (rc) {
    if (require_symmetric) { delete g; return rc; }
    set_error("");
  }
  *out = g;
  return FU_OK;
  FU_TRY_END
}

int fu_graph_gen_er(int32_t n, int64_t m, uint64_t seed, fu_graph **out) {
  FU_TRY_BEGIN
  if (!out || n <= 1 || m < 0) return fail(FU_ERR_ARG, "fu_graph_gen_er: bad arguments");
  std::vector<uint32_t> u(m), v(m);
#pragma omp parallel for schedule(static)
  for (int64_t k = 0; k < m; ++k) {
    u[k] = (uint32_t)(splitmix_at(seed, 2 * (uint64_t)k) % (uint64_t)n);
    v[k] = (uint32_t)(splitmix_at(seed, 2 * (uint64_t)k + 1) % (uint64_t)n);
  }
  auto *g = new fu_graph();
  symmetric_from_pairs(n, u, v, *g);
  int rc = build_rev(*g);
  if (rc) { delete g; return rc; }
  *out = g;
  return FU_OK;
  FU_TRY_END
}

int fu_graph_gen_rr(int32_t n, int32_t d, uint64_t seed, fu_graph **out) {
  FU_TRY_BEGIN
  if (!out || n <= 1 || d < 0 || d >= n || ((int64_t)n * d) % 2) return fail(FU_ERR_ARG, "fu_graph_gen_rr: need 0 <= d < n and n*d even");
  const int64_t m = (int64_t)n * d / 2;
  std::vector<uint32_t> stubs((size_t)n * d);
  for (int64_t k = 0; k < (int64_t)n * d; ++k) stubs[k] = (uint32_t)(k / d);
  uint64_t st = seed;
  for (int64_t i = (int64_t)stubs.size() - 1; i > 0; --i) {
    uint64_t j = splitmix_next(st) % (uint64_t)(i + 1);
    std::swap(stubs[i], stubs[j]);
  }
  std::vector<uint32_t> u(m), v(m);
  auto key = [](uint32_t a, uint32_t b) { return a < b ? ((uint64_t)a << 32) | b : ((uint64_t)b << 32) | a; };
  std::unordered_multiset<uint64_t> have;
  have.reserve(m * 2);
  for (int64_t k = 0; k < m; ++k) {
    u[k] = stubs[2 * k];
    v[k] = stubs[2 * k + 1];
    have.insert(key(u[k], v[k]));
  }
  auto is_bad = [&](int64_t k) { return u[k] == v[k] || have.count(key(u[k], v[k])) > 1; };
  std::vector<int64_t> bad;
  for (int64_t k = 0; k < m; ++k)
    if (is_bad(k)) bad.push_back(k);
  // edge switching: (u,v) bad, (x,y) random -> (u,x), (v,y)
  int64_t guard = 0;
  while (!bad.empty()) {
    if (++guard > 1000 * (m + 10)) { return fail(FU_ERR_GRAPH, "fu_graph_gen_rr: did not converge"); }
    int64_t b = bad.back();
    if (!is_bad(b)) { bad.pop_back(); continue; }
    int64_t o = (int64_t)(splitmix_next(st) % (uint64_t)m);
    if (o == b) continue;
    uint32_t a1 = u[b], b1 = v[b], x = u[o], y = v[o];
    if (splitmix_next(st) & 1) std::swap(x, y);
    if (a1 == x || b1 == y) continue;
    if (have.count(key(a1, x)) || have.count(key(b1, y))) continue;
    have.erase(have.find(key(a1, b1)));
    have.erase(have.find(key(u[o], v[o])));
    u[b] = a1; v[b] = x;
    u[o] = b1; v[o] = y;
    have.insert(key(u[b], v[b]));
    have.insert(key(u[o], v[o]));
    if (!is_bad(b)) bad.pop_back();
    if (is_bad(o)) bad.push_back(o);
  }
  auto *g = new fu_graph();
  symmetric_from_pairs(n, u, v, *g);
  int rc = build_rev(*g);
  if (rc) { delete g; return rc; }
  *out = g;
  return FU_OK;
  FU_TRY_END
}

int fu_graph_gen_rmat(int32_t scale, int32_t edge_factor, double a, double b, double c,
                      uint64_t seed, fu_graph **out) {
  FU_TRY_BEGIN
  if (!out || scale < 1 || scale > 30 || edge_factor < 1 || a < 0 || b < 0 || c < 0 || a + b + c > 1.0)
    return fail(FU_ERR_ARG, "fu_graph_gen_rmat: bad arguments");
  const int32_t n = (int32_t)(1u << scale);
  const int64_t m = (int64_t)n * edge_factor;
  std::vector<uint32_t> u(m), v(m);
  const double ab = a + b, abc = a + b + c;
#pragma omp parallel for schedule(static)
  for (int64_t k = 0; k < m; ++k) {
    uint32_t x = 0, y = 0;
    for (int32_t l = 0; l < scale; ++l) {
      double r = u01(splitmix_at(seed, (uint64_t)k * 64 + l));
      x <<= 1;
      y <<= 1;
      if (r < a) {
      } else if (r < ab) {
        y |= 1;
      } else if (r < abc) {
        x |= 1;
      } else {
        x |= 1;
        y |= 1;
      }
    }
    u[k] = x;
    v[k] = y;
  }
  auto *g = new fu_graph();
  symmetric_from_pairs(n, u, v, *g);
  int rc = build_rev(*g);
  if (rc) { delete g; return rc; }
  *out = g;
  return FU_OK;
  FU_TRY_END
}

int fu_graph_gen_rgg(int32_t n, double radius, uint64_t seed, fu_graph **out) {
  FU_TRY_BEGIN
  if (!out || n <= 1 || !(radius > 0.0) || radius >= 0.5) return fail(FU_ERR_ARG, "fu_graph_gen_rgg: bad arguments");
  int64_t G = (int64_t)std::floor(1.0 / radius);
  if (G < 1) G = 1;
  if (G > 65536) G = 65536;
  std::vector<double> x(n), y(n);
  std::vector<int64_t> cell(n);
#pragma omp parallel for schedule(static)
  for (int32_t i = 0; i < n; ++i) {
    x[i] = u01(splitmix_at(seed, 2 * (uint64_t)i));
    y[i] = u01(splitmix_at(seed, 2 * (uint64_t)i + 1));
    int64_t cx = std::min<int64_t>(G - 1, (int64_t)(x[i] * G));
    int64_t cy = std::min<int64_t>(G - 1, (int64_t)(y[i] * G));
    cell[i] = cx * G + cy;
  }
  // node numbering: by cell (x-major), ties by generation index
  std::vector<int32_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int32_t p, int32_t q) { return cell[p] < cell[q]; });
  std::vector<double> xs(n), ys(n);
  std::vector<int64_t> cs(n);
  for (int32_t k = 0; k < n; ++k) {
    xs[k] = x[order[k]];
    ys[k] = y[order[k]];
    cs[k] = cell[order[k]];
  }
  std::vector<int64_t> cstart(G * G + 1, 0);
  for (int32_t k = 0; k < n; ++k) cstart[cs[k] + 1]++;
  for (int64_t q = 0; q < G * G; ++q) cstart[q + 1] += cstart[q];
  const double r2 = radius * radius;
  std::vector<int64_t> deg(n, 0);
  auto scan = [&](int32_t k, int32_t *dst) {
    int64_t cx = cs[k] / G, cy = cs[k] % G, cnt = 0;
    for (int64_t dx = -1; dx <= 1; ++dx) {
      int64_t ex = cx + dx;
      if (ex < 0 || ex >= G) continue;
      for (int64_t dy = -1; dy <= 1; ++dy) {
        int64_t ey = cy + dy;
        if (ey < 0 || ey >= G) continue;
        int64_t q = ex * G + ey;
        for (int64_t j = cstart[q]; j < cstart[q + 1]; ++j) {
          if (j == k) continue;
          double ddx = xs[k] - xs[j], ddy = ys[k] - ys[j];
          if (ddx * ddx + ddy * ddy < r2) {
            if (dst) dst[cnt] = (int32_t)j;
            ++cnt;
          }
        }
      }
    }
    return cnt;
  };
#pragma omp parallel for schedule(dynamic, 4096)
  for (int32_t k = 0; k < n; ++k) deg[k] = scan(k, nullptr);
  auto *g = new fu_graph();
  g->n = n;
  g->rowptr.assign(n + 1, 0);
  for (int32_t k = 0; k < n; ++k) g->rowptr[k + 1] = g->rowptr[k] + deg[k];
  if (g->rowptr[n] >= (int64_t)INT32_MAX) { delete g; return fail(FU_ERR_ARG, "fu_graph_gen_rgg: too many edges"); }
  g->col.resize(g->rowptr[n]);
  int32_t md = 0;
#pragma omp parallel for schedule(dynamic, 4096) reduction(max : md)
  for (int32_t k = 0; k < n; ++k) {
    int32_t *row = g->col.data() + g->rowptr[k];
    scan(k, row);
    std::sort(row, row + deg[k]);
    md = std::max<int32_t>(md, (int32_t)deg[k]);
  }
  g->max_deg = md;
  int rc = build_rev(*g);
  if (rc) { delete g; return rc; }
  *out = g;
  return FU_OK;
  FU_TRY_END
}

int fu_graph_info(const fu_graph *g, int32_t *n, int64_t *e, int32_t *max_deg,
                  int32_t *symmetric) {
  if (!g) return fail(FU_ERR_ARG, "fu_graph_info: NULL graph");
  if (n) *n = g->n;
  if (e) *e = g->rowptr[g->n];
  if (max_deg) *max_deg = g->max_deg;
  if (symmetric) *symmetric = g->rev.empty() && g->rowptr[g->n] > 0 ? 0 : 1;
  return FU_OK;
}

int fu_graph_export(const fu_graph *g, int64_t *rowptr, int32_t *col, int32_t *rev) {
  if (!g) return fail(FU_ERR_ARG, "fu_graph_export: NULL graph");
  const int64_t E = g->rowptr[g->n];
  if (rowptr) std::memcpy(rowptr, g->rowptr.data(), sizeof(int64_t) * (g->n + 1));
  if (col && E) std::memcpy(col, g->col.data(), sizeof(int32_t) * E);
  if (rev && E) {
    if ((int64_t)g->rev.size() != E) return fail(FU_ERR_GRAPH, "fu_graph_export: graph is not symmetric (no rev)");
    std::memcpy(rev, g->rev.data(), sizeof(int32_t) * E);
  }
  return FU_OK;
}

int fu_graph_free(fu_graph *g) {
  delete g;
  return FU_OK;
}

int fu_graph_relabel(const fu_graph *g, int32_t order, int32_t *new_of_old, fu_graph **out) {
  FU_TRY_BEGIN
  if (!g || !new_of_old || !out || order < 0 || order > 1) return fail(FU_ERR_ARG, "fu_graph_relabel: bad arguments");
  const int32_t n = g->n;
  const int64_t E = g->rowptr[n];
  const bool sym = (int64_t)g->rev.size() == E;
  std::vector<int32_t> old_of_new(n);
  if (order == 1) {  // degree descending, ties by old id: the gather-hot nodes first
    std::iota(old_of_new.begin(), old_of_new.end(), 0);
    std::stable_sort(old_of_new.begin(), old_of_new.end(), [&](int32_t x, int32_t y) {
      return g->rowptr[x + 1] - g->rowptr[x] > g->rowptr[y + 1] - g->rowptr[y];
    });
    for (int32_t p = 0; p < n; ++p) new_of_old[old_of_new[p]] = p;
  } else {
    std::vector<char> seen(n, 0);
    for (int32_t i = 0; i < n; ++i) {
      const int32_t p = new_of_old[i];
      if (p < 0 || p >= n || seen[p]) return fail(FU_ERR_ARG, "fu_graph_relabel: new_of_old is not a permutation");
      seen[p] = 1;
      old_of_new[p] = i;
    }
  }
  auto *h = new fu_graph();
  h->n = n;
  h->max_deg = g->max_deg;
  h->rowptr.assign(n + 1, 0);
  for (int32_t p = 0; p < n; ++p) {
    const int32_t i = old_of_new[p];
    h->rowptr[p + 1] = h->rowptr[p] + (g->rowptr[i + 1] - g->rowptr[i]);
  }
  h->col.resize(E);
  // rows move as blocks and keep their neighbour order (the summation order, CA:106/110)
#pragma omp parallel for schedule(dynamic, 4096)
  for (int32_t p = 0; p < n; ++p) {
    const int32_t i = old_of_new[p];
    const int64_t b = g->rowptr[i], d = g->rowptr[i + 1] - b, nb = h->rowptr[p];
    for (int64_t k = 0; k < d; ++k) h->col[nb + k] = new_of_old[g->col[b + k]];
  }
  if (sym) {  // new position of old edge k: rows moved as blocks, so rev maps through it
    std::vector<int32_t> pos(E);
#pragma omp parallel for schedule(dynamic, 4096)
    for (int32_t i = 0; i < n; ++i) {
      const int64_t b = g->rowptr[i], d = g->rowptr[i + 1] - b, nb = h->rowptr[new_of_old[i]];
      for (int64_t k = 0; k < d; ++k) pos[b + k] = (int32_t)(nb + k);
    }
    h->rev.resize(E);
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < E; ++k) h->rev[pos[k]] = pos[g->rev[k]];
  }
  *out = h;
  return FU_OK;
  FU_TRY_END
}

int fu_values_uniform(int64_t n, uint64_t seed, double lo, double hi, double *out) {
  if (n < 0 || (n > 0 && !out)) return fail(FU_ERR_ARG, "fu_values_uniform: bad arguments");
  const double w = hi - lo;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) out[i] = lo + w * u01(splitmix_at(seed, (uint64_t)i));
  return FU_OK;
}

}  // extern "C"
