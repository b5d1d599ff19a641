// libfu device engine for MI355X (gfx950): collect-all round kernels, tick replay kernels,
// convergence check, handle management. C ABI declared in include/fu.h.
//
// Arithmetic spec (bitwise parity with the reference's Python floats):
//   receive  (flowupdating-collectall.py:98-99):  fr[e] = -f_old[rev e], er[e] = a_old[col e]
//   fire     (CA:106-119):  S = 0.0 + fr[e0] + fr[e1] + ...  (left to right, row order)
//                           T = 0.0 + er[e0] + er[e1] + ...
//                           a = ((v - S) + T) / (deg + 1)
//                           f_new[e] = (fr[e] + a) - er[e]
// Compiled with -ffp-contract=off and without fast-math. There are no multiplies to
// contract, and `/` is the correctly rounded IEEE fp64 division. Every sum is a sequential
// dependency chain in row order, including for hubs (see k_round_tile's heavy path).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "fu_common.h"

using namespace fu;

#define HIP_TRY(expr)                                                                     \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess)                                                                 \
      return fu::fail(FU_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));     \
  } while (0)

namespace {

constexpr int kBlock = 256;      // threads per block (4 waves of 64)
constexpr int kTileEdges = 2048;  // max edges staged in LDS per light tile
constexpr int kTileNodes = kBlock;

// ------------------------------------------------------------------------------------
// error reduction: max over |a - target| as uint64 bit patterns (non-negative doubles
// order like their bits; a NaN (sign cleared) is larger than +inf, so NaN propagates)
// ------------------------------------------------------------------------------------
__device__ inline unsigned long long err_bits(double a, double t) {
  return (unsigned long long)__double_as_longlong(fabs(a - t));
}

__device__ inline void block_max_to(unsigned long long x, unsigned long long *dst) {
  for (int off = 32; off > 0; off >>= 1) {
    unsigned long long y = __shfl_xor(x, off, 64);
    x = x > y ? x : y;
  }
  __shared__ unsigned long long s_w[kBlock / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) s_w[w] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long m = s_w[0];
    for (int k = 1; k < kBlock / 64; ++k) m = m > s_w[k] ? m : s_w[k];
    // a plain read first: only blocks that raise the running max issue the atomic (a stale
    // read only costs an extra atomic, never a wrong max). Without it 16K blocks serialise
    // on one address.
    if (m && m > __hip_atomic_load(dst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(dst, m);
  }
}

// ------------------------------------------------------------------------------------
// Round 0: the timeout fire on zero state (CA:33-34, CA:87-91 -> CA:105-128)
// ------------------------------------------------------------------------------------
// SPLIT: kernels >= 4 keep flows as split words (see st_f); kernels 1-3 as doubles
template <bool SPLIT>
__global__ __launch_bounds__(kBlock) void k_round0(int n, const int *__restrict__ rowptr,
                                                   const double *__restrict__ v,
                                                   double *__restrict__ f,
                                                   double *__restrict__ a) {
  int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  int b = rowptr[i], e = rowptr[i + 1];
  double ai = ((v[i] - 0.0) + 0.0) / (double)(e - b + 1);
  a[i] = ai;
  double fv = (0.0 + ai) - 0.0;
  if constexpr (!SPLIT)
    for (int k = b; k < e; ++k) f[k] = fv;  // kernels 1-3 (split flows: k_round0_flows)
}

// Round 0's flows of kernels >= 4, one thread per edge (a hub's row is not one thread's
// loop): f[k] = (0.0 + a_0[row of k]) - 0.0 (CA:117 on zero state), split words.
__global__ __launch_bounds__(kBlock) void k_round0_flows(int n, long long E, const int *__restrict__ rowptr,
                                                         const double *__restrict__ a, double *__restrict__ f) {
  const long long k = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (k >= E) return;
  int lo = 0, hi = n - 1;  // row i with rowptr[i] <= k < rowptr[i + 1] (non-empty rows only)
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (rowptr[mid] <= k) lo = mid; else hi = mid - 1;
  }
  const double fv = (0.0 + a[lo]) - 0.0;
  unsigned *w = reinterpret_cast<unsigned *>(f);
  const long long j = ((k & ~31LL) << 1) | (k & 31);
  w[j] = (unsigned)__double2hiint(fv);
  w[j + 32] = (unsigned)__double2loint(fv);
}

// ------------------------------------------------------------------------------------
// Variant 1: one thread per node, gathers straight from global memory
// ------------------------------------------------------------------------------------
template <bool CHECK>
__global__ __launch_bounds__(kBlock) void k_round_tpn(
    int n, const int *__restrict__ rowptr, const int *__restrict__ col,
    const int *__restrict__ rev, const double *__restrict__ v,
    const double *__restrict__ f_old, const double *__restrict__ a_old,
    double *__restrict__ f_new, double *__restrict__ a_new,
    const double *__restrict__ target, unsigned long long *__restrict__ err) {
  int i = blockIdx.x * kBlock + threadIdx.x;
  unsigned long long eb = 0;
  if (i < n) {
    int b = rowptr[i], e = rowptr[i + 1];
    double S = 0.0, T = 0.0;
    for (int k = b; k < e; ++k) {
      S = S + (-f_old[rev[k]]);
      T = T + a_old[col[k]];
    }
    double a = ((v[i] - S) + T) / (double)(e - b + 1);
    a_new[i] = a;
    for (int k = b; k < e; ++k) f_new[k] = ((-f_old[rev[k]]) + a) - a_old[col[k]];
    if (CHECK) eb = err_bits(a, target[i]);
  }
  if (CHECK) block_max_to(eb, err);
}

// ------------------------------------------------------------------------------------
// Variant 2: LDS tiles. A light tile = a contiguous node range with <= kTileNodes nodes
// and <= kTileEdges edges. Its edges are gathered edge-parallel into LDS (coalesced
// col/rev, independent gathers), then each node sums its row sequentially from LDS, and
// the new flows are written edge-parallel (coalesced). A heavy tile = one node with more
// than hub_threshold edges. The whole block gathers it in chunks, and wave 0 keeps the
// exact left-to-right sum in a lane-uniform dependency chain (bitwise parity for hubs).
// tiles[t] = {node_begin, node_end}; node_end < 0 marks a heavy tile (node = begin).
// ------------------------------------------------------------------------------------
template <bool CHECK>
__global__ __launch_bounds__(kBlock) void k_round_tile(
    const int4 *__restrict__ tiles, const int *__restrict__ rowptr,
    const int *__restrict__ col, const int *__restrict__ rev, const double *__restrict__ v,
    const double *__restrict__ f_old, const double *__restrict__ a_old,
    double *__restrict__ f_new, double *__restrict__ a_new,
    const double *__restrict__ target, unsigned long long *__restrict__ err) {
  __shared__ double s_fr[kTileEdges];
  __shared__ double s_er[kTileEdges];
  __shared__ unsigned char s_own[kTileEdges];
  __shared__ int s_rp[kTileNodes + 1];
  __shared__ double s_a[kTileNodes];
  const int t = threadIdx.x;
  const int4 tl = tiles[blockIdx.x];
  unsigned long long eb = 0;

  if (tl.y < 0) {
    // ---------------- heavy node: block-chunked gather, wave-0 sequential chain ----------
    const int i = tl.x;
    const int b = rowptr[i], e = rowptr[i + 1];
    double S = 0.0, T = 0.0;
    for (int c0 = b; c0 < e; c0 += kTileEdges) {
      const int cn = min(kTileEdges, e - c0);
      for (int q = t; q < cn; q += kBlock) {
        s_fr[q] = -f_old[rev[c0 + q]];
        s_er[q] = a_old[col[c0 + q]];
      }
      __syncthreads();
      if (t < 64) {
        for (int q = 0; q < cn; ++q) {  // lane-uniform LDS broadcast reads
          S = S + s_fr[q];
          T = T + s_er[q];
        }
      }
      __syncthreads();
    }
    if (t == 0) {
      double a = ((v[i] - S) + T) / (double)(e - b + 1);
      s_a[0] = a;
      a_new[i] = a;
      if (CHECK) eb = err_bits(a, target[i]);
    }
    __syncthreads();
    const double a = s_a[0];
    for (int k = b + t; k < e; k += kBlock) f_new[k] = ((-f_old[rev[k]]) + a) - a_old[col[k]];
    if (CHECK) block_max_to(eb, err);
    return;
  }

  // ---------------- light tile ----------------
  const int nb = tl.x, nn = tl.y - tl.x;
  for (int q = t; q <= nn; q += kBlock) s_rp[q] = rowptr[nb + q];
  __syncthreads();
  const int e0 = s_rp[0];
  const int ne = s_rp[nn] - e0;
#pragma unroll 4
  for (int q = t; q < ne; q += kBlock) {
    const int k = e0 + q;
    s_fr[q] = -f_old[rev[k]];
    s_er[q] = a_old[col[k]];
  }
  if (t < nn) {
    for (int q = s_rp[t] - e0; q < s_rp[t + 1] - e0; ++q) s_own[q] = (unsigned char)t;
  }
  __syncthreads();
  if (t < nn) {
    const int qb = s_rp[t] - e0, qe = s_rp[t + 1] - e0;
    double S = 0.0, T = 0.0;
    for (int q = qb; q < qe; ++q) {
      S = S + s_fr[q];
      T = T + s_er[q];
    }
    const double a = ((v[nb + t] - S) + T) / (double)(qe - qb + 1);
    s_a[t] = a;
    a_new[nb + t] = a;
    if (CHECK) eb = err_bits(a, target[nb + t]);
  }
  __syncthreads();
  for (int q = t; q < ne; q += kBlock) f_new[e0 + q] = (s_fr[q] + s_a[s_own[q]]) - s_er[q];
  if (CHECK) block_max_to(eb, err);
}

// ------------------------------------------------------------------------------------
// Variant 3: push / inbox. Message (flow, estimate) from j to i lives at i's own row slot
// for j (the FlowUpdatingMsg of CA:121, stored where its receiver reads it). A node reads
// its inbox row contiguously and scatters its new messages to inbox_new[rev[e]]. No col
// and no random reads; one random 16-byte store per directed edge.
// ------------------------------------------------------------------------------------
template <bool CHECK>
__global__ __launch_bounds__(kBlock) void k_round_push(
    const int4 *__restrict__ tiles, const int *__restrict__ rowptr,
    const int *__restrict__ rev, const double *__restrict__ v,
    const double2 *__restrict__ in_old, double2 *__restrict__ in_new,
    double *__restrict__ a_new, const double *__restrict__ target,
    unsigned long long *__restrict__ err) {
  __shared__ double2 s_m[kTileEdges];
  __shared__ unsigned char s_own[kTileEdges];
  __shared__ int s_rp[kTileNodes + 1];
  __shared__ double s_a[kTileNodes];
  const int t = threadIdx.x;
  const int4 tl = tiles[blockIdx.x];
  unsigned long long eb = 0;

  if (tl.y < 0) {
    const int i = tl.x;
    const int b = rowptr[i], e = rowptr[i + 1];
    double S = 0.0, T = 0.0;
    for (int c0 = b; c0 < e; c0 += kTileEdges) {
      const int cn = min(kTileEdges, e - c0);
      for (int q = t; q < cn; q += kBlock) s_m[q] = in_old[c0 + q];
      __syncthreads();
      if (t < 64) {
        for (int q = 0; q < cn; ++q) {
          const double2 m = s_m[q];
          S = S + (-m.x);
          T = T + m.y;
        }
      }
      __syncthreads();
    }
    if (t == 0) {
      double a = ((v[i] - S) + T) / (double)(e - b + 1);
      s_a[0] = a;
      a_new[i] = a;
      if (CHECK) eb = err_bits(a, target[i]);
    }
    __syncthreads();
    const double a = s_a[0];
    for (int k = b + t; k < e; k += kBlock) {
      const double2 m = in_old[k];
      in_new[rev[k]] = make_double2(((-m.x) + a) - m.y, a);
    }
    if (CHECK) block_max_to(eb, err);
    return;
  }

  const int nb = tl.x, nn = tl.y - tl.x;
  for (int q = t; q <= nn; q += kBlock) s_rp[q] = rowptr[nb + q];
  __syncthreads();
  const int e0 = s_rp[0];
  const int ne = s_rp[nn] - e0;
  for (int q = t; q < ne; q += kBlock) s_m[q] = in_old[e0 + q];
  if (t < nn) {
    for (int q = s_rp[t] - e0; q < s_rp[t + 1] - e0; ++q) s_own[q] = (unsigned char)t;
  }
  __syncthreads();
  if (t < nn) {
    const int qb = s_rp[t] - e0, qe = s_rp[t + 1] - e0;
    double S = 0.0, T = 0.0;
    for (int q = qb; q < qe; ++q) {
      const double2 m = s_m[q];
      S = S + (-m.x);
      T = T + m.y;
    }
    const double a = ((v[nb + t] - S) + T) / (double)(qe - qb + 1);
    s_a[t] = a;
    a_new[nb + t] = a;
    if (CHECK) eb = err_bits(a, target[nb + t]);
  }
  __syncthreads();
  for (int q = t; q < ne; q += kBlock) {
    const double2 m = s_m[q];
    const double a = s_a[s_own[q]];
    in_new[rev[e0 + q]] = make_double2(((-m.x) + a) - m.y, a);
  }
  if (CHECK) block_max_to(eb, err);
}

// ------------------------------------------------------------------------------------
// Packed estimate table (kernel 4). Once the estimates have converged into a narrow
// cluster, the neighbour gather reads a W-bit code per node (W = 8, 16 or 32) instead of
// the 8-byte double: a 1-4 MB table instead of 8 MB for ER-1M, so the random gathers hit
// the XCD's L2. The code is a LOSSLESS offset of the double's order-preserving 64-bit key
// from a per-table base: key(x) - base in [0, 2^W - 2]. Any estimate outside that window
// is stored as the escape code 2^W - 1, and its reader gathers the double instead. Every
// decoded value is the exact bit pattern, so the results are unchanged. Each round writes
// the doubles (coalesced, always) and, when packing is on, the codes under the parameters
// pack_plan chose from a sample of gather targets. Slots: ctl[r & 1] describes the code
// table written in round r (copied by block 0 from ctl[2], the current encoding plan);
// width 0 = no codes (the reader gathers the doubles).
// ------------------------------------------------------------------------------------
struct PackCtl {
  unsigned long long base;
  int width;
  int pad;
};

// Write-through store (global_store ... sc1): the line leaves the XCD's L2 at once instead
// of staying dirty there. A kernel's end writes back every dirty L2 line before the next
// launch may start, so round kernels that leave their output (flows, estimates, codes,
// staged words) dirty pay that writeback serially at each boundary (MI355X_MICROARCH.md:
// + bytes / 6 TB/s per boundary); streamed through, it overlaps the kernel's own work.
// Byte and short sc1 stores go out as one fabric write each (MI355X_MICROARCH.md: 6-12x the
// per-byte cost of wide ones), so 1- and 2-byte elements keep plain (write-back) stores.
// Measured on ER-1M: write-through did not shorten the round kernels (kernel 4 lost 4.5 us,
// kernel 8 gained nothing), so it is off unless built with -DFU_WT=1.
#ifndef FU_WT
#define FU_WT 0
#endif
template <typename T>
__device__ __forceinline__ void st_wt(T *p, T v) {
  if constexpr (FU_WT && sizeof(T) >= 4) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

__device__ inline unsigned long long dkey(double x) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(x);
  return (b >> 63) ? ~b : (b | (1ull << 63));
}
__device__ inline double dkey_inv(unsigned long long k) {
  const unsigned long long b = (k >> 63) ? (k & ~(1ull << 63)) : ~k;
  return __longlong_as_double((long long)b);
}
template <int W>
__device__ inline unsigned ld_code(const void *tab, int i) {
  if constexpr (W == 8) return reinterpret_cast<const unsigned char *>(tab)[i];
  else if constexpr (W == 16) return reinterpret_cast<const unsigned short *>(tab)[i];
  else return reinterpret_cast<const unsigned *>(tab)[i];
}
__device__ inline void put_code(const PackCtl &pc, void *tab, int i, double a) {
  const unsigned long long off = dkey(a) - pc.base;
  const unsigned esc = pc.width == 32 ? 0xFFFFFFFFu : (1u << pc.width) - 1u;
  const unsigned cd = off < (unsigned long long)esc ? (unsigned)off : esc;
  if (pc.width == 8) st_wt(reinterpret_cast<unsigned char *>(tab) + i, (unsigned char)cd);
  else if (pc.width == 16) st_wt(reinterpret_cast<unsigned short *>(tab) + i, (unsigned short)cd);
  else st_wt(reinterpret_cast<unsigned *>(tab) + i, cd);
}
template <int W>
__device__ inline double decode_or(unsigned cd, unsigned long long base, const double *a_prev, int j) {
  constexpr unsigned esc = W == 32 ? 0xFFFFFFFFu : (1u << W) - 1u;
  return cd == esc ? a_prev[j] : dkey_inv(base + cd);
}
// One neighbour estimate a_{r-1}[j] under the table's packing (uniform branch).
__device__ inline double ld_est(const PackCtl &pp, const void *codes, const double *a_prev, int j) {
  if (pp.width == 8) return decode_or<8>(ld_code<8>(codes, j), pp.base, a_prev, j);
  if (pp.width == 16) return decode_or<16>(ld_code<16>(codes, j), pp.base, a_prev, j);
  if (pp.width == 32) return decode_or<32>(ld_code<32>(codes, j), pp.base, a_prev, j);
  return a_prev[j];
}
// The light tile's kPer neighbour estimates: all code loads first, then decode (escapes
// gather the double).
template <int W, int KP>
__device__ inline void gather_packed(const int (&c)[KP], double (&g)[KP], int t, int ne,
                                     const void *codes, unsigned long long base,
                                     const double *a_prev) {
  unsigned cd[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) cd[k] = t + k * kBlock < ne ? ld_code<W>(codes, c[k]) : 0u;
#pragma unroll
  for (int k = 0; k < KP; ++k) g[k] = t + k * kBlock < ne ? decode_or<W>(cd[k], base, a_prev, c[k]) : 0.0;
}
// Encoding plan from the estimates a_r of a fixed sample of kPlanSamples gather targets:
// the centre is the median of the first 64 sampled keys; the width is the smallest W whose
// window [centre - 2^(W-1), centre + 2^(W-1) - 2] holds >= 99.5 % of the sample; else 0.
constexpr int kPlanSamples = 4096;

__global__ __launch_bounds__(kBlock) void k_pack_plan(const double *__restrict__ a,
                                                      const int *__restrict__ sample,
                                                      PackCtl *__restrict__ ctl) {
  constexpr int kPer = kPlanSamples / kBlock;
  __shared__ unsigned long long s_centre;
  __shared__ int s_cnt[3];
  const int t = threadIdx.x;
  if (t < 3) s_cnt[t] = 0;
  int idx[kPer];
  unsigned long long key[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) idx[k] = sample[t + k * kBlock];  // all loads in flight
#pragma unroll
  for (int k = 0; k < kPer; ++k) key[k] = dkey(a[idx[k]]);
  if (t < 64) {  // median of samples 0..63: rank by comparison against every lane
    int below = 0;
    for (int l = 0; l < 64; ++l) {
      const unsigned long long o = __shfl(key[0], l, 64);
      below += (o < key[0]) || (o == key[0] && l < t);
    }
    if (below == 32) s_centre = key[0];
  }
  __syncthreads();
  const unsigned long long c = s_centre;
  int n8 = 0, n16 = 0, n32 = 0;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const unsigned long long d = key[k] >= c ? key[k] - c : c - key[k];
    n8 += d + 2 <= (1ull << 7);
    n16 += d + 2 <= (1ull << 15);
    n32 += d + 2 <= (1ull << 31);
  }
  atomicAdd(&s_cnt[0], n8);
  atomicAdd(&s_cnt[1], n16);
  atomicAdd(&s_cnt[2], n32);
  __syncthreads();
  if (t == 0) {
    const int need = kPlanSamples - kPlanSamples / 200;
    const int w = s_cnt[0] >= need ? 8 : s_cnt[1] >= need ? 16 : s_cnt[2] >= need ? 32 : 0;
    PackCtl p;
    p.base = w ? c - (1ull << (w - 1)) : 0;
    p.width = w;
    p.pad = 0;
    ctl[2] = p;
  }
}

// ------------------------------------------------------------------------------------
// Flow storage of kernels >= 4 (state shared by kernels 4-10): split words. The flow of
// edge e is stored as its double's high and low 32-bit words in separate 128-byte lines:
// block e / 32 holds 32 high words, then 32 low words. Each round rewrites every low word,
// but a high word (sign, exponent, top 20 mantissa bits) only when it changes. Once the
// estimates have converged the flows move by a few ulps per round and their high words
// stay put, so a round writes 4 instead of 8 bytes per edge (the store of an identical
// word is skipped; the value in memory is always the exact f_r).
// ------------------------------------------------------------------------------------
__device__ __forceinline__ long long fhi_idx(int e) { return ((long long)(e & ~31) << 1) | (e & 31); }
__device__ __forceinline__ double ld_f(const double *F, int e) {
  const unsigned *w = reinterpret_cast<const unsigned *>(F);
  const long long i = fhi_idx(e);
  return __hiloint2double((int)w[i], (int)w[i + 32]);
}
// store f_r over f_old (the value the slot held)
__device__ __forceinline__ void st_f(double *F, int e, double v, double f_old) {
  unsigned *w = reinterpret_cast<unsigned *>(F);
  const long long i = fhi_idx(e);
  st_wt(w + i + 32, (unsigned)__double2loint(v));
  if (__double2hiint(v) != __double2hiint(f_old)) st_wt(w + i, (unsigned)__double2hiint(v));
}
__device__ __forceinline__ void st_f_full(double *F, int e, double v) {
  unsigned *w = reinterpret_cast<unsigned *>(F);
  const long long i = fhi_idx(e);
  st_wt(w + i + 32, (unsigned)__double2loint(v));
  st_wt(w + i, (unsigned)__double2hiint(v));
}

// ------------------------------------------------------------------------------------
// Variant 4: flow reconstruction ("recon"). Node j computed, in round r-1,
//     f_{r-1}[j->i] = ((-f_{r-2}[i->j]) + a_{r-1}[j]) - a_{r-2}[i]        (CA:99, CA:117)
// from three operands that node i also holds: its own previous flow f_{r-2}[i->j] (its
// own row), its own estimate a_{r-2}[i], and j's estimate a_{r-1}[j]. So i recomputes the
// reverse flow with the same IEEE operations on the same operands, and gets the same bits,
// instead of gathering f_old[rev[e]] from a 64 MB array. Per edge, the only random access
// left is a_{r-1}[col e] (8 B from an 8 MB array). Flows are updated in place: round r
// reads f_{r-2} and writes f_r in the same rows, owned by the same block. Buffers:
// F[r & 1], A[r % 3] (see launch_round). Round 1 reads f_{-1} = -0.0, a_{-1} = 0.0, which
// reproduces round 0's (0.0 + a) - 0.0 exactly.
// ------------------------------------------------------------------------------------
__device__ inline double recon_fr(double f_own_old, double a_nb, double a_own_old2) {
  const double f_rev = ((-f_own_old) + a_nb) - a_own_old2;  // j's f_{r-1}[j->i], bitwise
  return -f_rev;                                            // CA:99 flows[j] = -msg.flow
}

__device__ inline void wave_sync() {
  // LDS traffic of one wave is processed in order; this only stops the compiler from moving
  // LDS accesses across the hand-off between lanes
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Exact left-to-right chains S += xs[q], T += es[q] over q = 0 .. cn-1 (one whole wave;
// S and T lane-uniform in and out). Even lanes run the S chain, odd lanes the T chain, so
// one fp64 add per element advances both sums: a wave64 v_add_f64 occupies the SIMD for the
// same cycles whatever the EXEC mask, and two separate chains cost two. The LDS reads of
// the next B elements are issued before the dependent adds of the current B (B = 16: the adds
// of one batch cover the LDS latency of the next).
#ifndef FU_CHAIN_B
#define FU_CHAIN_B 16  // measured: 8 -> 8.75, 16 -> 7.2, 32 -> 6.4 ns per element (32 costs registers)
#endif
__device__ __forceinline__ void chain_sum(const double *xs, const double *es, int cn, double &S, double &T) {
  constexpr int B = FU_CHAIN_B;
  const bool odd = threadIdx.x & 1;
  const double *src = odd ? es : xs;
  double acc = odd ? T : S;
  int q = 0;
  if (cn >= B) {
    double a[B];
#pragma unroll
    for (int k = 0; k < B; ++k) a[k] = src[k];
    for (q = B; q + B <= cn; q += B) {
      double a2[B];
#pragma unroll
      for (int k = 0; k < B; ++k) a2[k] = src[q + k];
#pragma unroll
      for (int k = 0; k < B; ++k) acc = acc + a[k];
#pragma unroll
      for (int k = 0; k < B; ++k) a[k] = a2[k];
    }
#pragma unroll
    for (int k = 0; k < B; ++k) acc = acc + a[k];
  }
  for (; q < cn; ++q) acc = acc + src[q];
  S = __shfl(acc, 0);
  T = __shfl(acc, 1);
}

// ------------------------------------------------------------------------------------
// Mega hubs: the exact left-to-right sums of avg_and_send (CA:106, CA:110) in parallel.
// Python's sum is the chain s_{k+1} = fl(s_k + x_k) from s_0 = 0: inherently sequential,
// and one wave running it for a 406K-edge R-MAT hub needs ~3 ms per round. The chain is
// decomposed instead (host prototype and adversarial checks: tools/exact_scan_proto.c):
//   * an approximate prefix p_k (any summation order) gives a speculative key of s_{k+1}:
//     its ulp exponent ue (u = 2^ue) and sign;
//   * a step whose key differs from the previous step's is a BOUNDARY: it is done later as
//     one exact fp64 add in a short serial pass;
//   * every other step keeps s a multiple of u, so s_{k+1} = u (m_k + t_k) with
//     t_k = round(x_k / u), ties to the even m_k + t_k: t_k depends on m_k only through its
//     parity. A step is a 2-state transducer (t0, t1, q0, q1); compositions stay in that form,
//     plus the min / max of the partial increments, so a RUN of such steps is one RunSum;
//   * the serial pass walks pieces of 2048 elements: head run, then per boundary its exact
//     add and the run after it, VERIFYING each run in O(1): every result must satisfy
//     2^52 < |m| < 2^53 (the exact sum was inside the binade, so fl rounded at u). A piece
//     that fails (speculation wrong, > kMaxBnd boundaries, zeros / subnormals) is redone
//     element by element. The result is the chain's bits in every case.
// ------------------------------------------------------------------------------------
constexpr int kPieceT = 8;                // elements per thread
constexpr int kPiece = kBlock * kPieceT;  // elements per piece (one block)
constexpr int kMaxBnd = 32;               // boundaries listed per piece and chain
constexpr int kKeySpecial = -1000000;     // zero, subnormal, inf, nan
constexpr long long kRunLim = 1LL << 56;  // |t|, |mn|, |mx| bound of a verifiable run

struct RunSum {
  long long t0, t1, mn, mx;  // increment for start parity 0 / 1; min / max partial increment
  int len, q;                // steps; q bit0 / bit1 = end parity for start parity 0 / 1, bit2 = bad
};
struct BndSum {
  double x;  // the boundary element
  int key, pad;
  RunSum run;  // the run after it (up to the next boundary or the piece end)
};
struct PieceSum {
  int first_key, nb, pad0, pad1;  // key the head run assumes; boundaries (> kMaxBnd: dense)
  RunSum head;
  BndSum b[kMaxBnd];
  long long pad_end;
};
static_assert(sizeof(PieceSum) % 16 == 0, "PieceSum is copied in 16-byte words");
constexpr int kPieceWords = (int)(sizeof(PieceSum) / 16);

__device__ __forceinline__ int ulp_key(double x) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(x);
  const int E = (int)((b >> 52) & 0x7ff);
  return (E == 0 || E == 0x7ff) ? kKeySpecial : ((E - 1075) * 2) | (int)(b >> 63);
}
__device__ __forceinline__ RunSum run_id() { return RunSum{0, 0, 0, 0, 0, 2}; }
__device__ __forceinline__ RunSum run_cat(const RunSum &a, const RunSum &b) {  // a, then b
  if (b.len == 0) return a;
  if (a.len == 0) return b;
  const int a0 = a.q & 1, a1 = (a.q >> 1) & 1, b0 = b.q & 1, b1 = (b.q >> 1) & 1;
  RunSum r;
  r.t0 = a.t0 + (a0 ? b.t1 : b.t0);
  r.t1 = a.t1 + (a1 ? b.t1 : b.t0);
  // b's partial increments start at a.t0 or a.t1: conservative bounds over both
  r.mn = min(a.mn, min(a.t0, a.t1) + b.mn);
  r.mx = max(a.mx, max(a.t0, a.t1) + b.mx);
  r.len = a.len + b.len;
  r.q = (a0 ? b1 : b0) | ((a1 ? b1 : b0) << 1) | ((a.q | b.q) & 4);
  // |values| <= 2^56 in, <= 2^57 out: no overflow; a run that large can never verify
  if (r.mn < -kRunLim || r.mx > kRunLim) r.q |= 4;
  return r;
}
__device__ __forceinline__ RunSum run_step(double x, int ue) {
  const double y = ldexp(x, -ue);  // exact (a power-of-two scaling)
  RunSum r;
  r.len = 1;
  if (!(fabs(y) < 0x1p54)) {  // the result cannot stay in the binade
    r.t0 = r.t1 = r.mn = r.mx = 0;
    r.q = 2 | 4;
    return r;
  }
  const double fl = floor(y), fr = y - fl;  // both exact
  const long long f = (long long)fl;
  long long t0, t1;
  if (fr < 0.5) t0 = t1 = f;
  else if (fr > 0.5) t0 = t1 = f + 1;
  else {  // tie: the even m + t
    t0 = (f & 1) ? f + 1 : f;
    t1 = (f & 1) ? f : f + 1;
  }
  r.t0 = t0;
  r.t1 = t1;
  r.mn = min(t0, t1);
  r.mx = max(t0, t1);
  r.q = (int)(t0 & 1) | ((int)((t1 + 1) & 1) << 1);
  return r;
}
// Applies a run to m (units 2^ue), verifying every result stays strictly inside the binade.
__device__ __forceinline__ bool run_apply(const RunSum &r, long long &m) {
  if (r.len == 0) return true;
  if (r.q & 4) return false;
  constexpr long long lo = 1LL << 52, hi = 1LL << 53;
  if (m > 0) {
    if (!(m + r.mn > lo && m + r.mx < hi)) return false;
  } else {
    if (!(m + r.mx < -lo && m + r.mn > -hi)) return false;
  }
  m += (m & 1) ? r.t1 : r.t0;
  return true;
}
__device__ __forceinline__ long long key_m(double s, int key) {
  return key == kKeySpecial ? 0 : (long long)ldexp(s, -(key >> 1));
}

// Serial pass of one chain over pieces [p0, p1) of a hub (one wave, lane-uniform). buf:
// this wave's LDS buffer (a PieceSum, reused as 64 doubles by the element-wise fallback).
// comp: 0 = fr (S), 1 = er (T); xy: the hub's (fr, er) pairs; d: its degree.
__device__ double hub_serial_pass(const PieceSum *__restrict__ hsum, int p0, int p1, int comp,
                                  const double2 *__restrict__ xy, int d, PieceSum *buf,
                                  unsigned long long *__restrict__ redo) {
  const int lane = threadIdx.x & 63;
  double s = 0.0;
  int key = kKeySpecial;
  long long m = 0;
  const int4 *src = reinterpret_cast<const int4 *>(hsum);
  int4 *dst = reinterpret_cast<int4 *>(buf);
  int4 w0 = make_int4(0, 0, 0, 0), w1 = w0;
  auto fetch = [&](int p) {
    const int4 *q = src + ((size_t)p * 2 + comp) * kPieceWords;
    w0 = q[lane];
    if (lane + 64 < kPieceWords) w1 = q[lane + 64];
  };
  if (p0 < p1) fetch(p0);
  for (int p = p0; p < p1; ++p) {
    wave_sync();
    dst[lane] = w0;
    if (lane + 64 < kPieceWords) dst[lane + 64] = w1;
    wave_sync();
    if (p + 1 < p1) fetch(p + 1);
    const double s0 = s;
    const int nb = buf->nb;
    bool ok = nb <= kMaxBnd;
    if (ok && buf->head.len) {
      ok = key != kKeySpecial && key == buf->first_key && run_apply(buf->head, m);
      if (ok) s = ldexp((double)m, key >> 1);
    }
    for (int j = 0; ok && j < nb; ++j) {
      s = s + buf->b[j].x;  // the boundary step: one exact fp64 add
      key = ulp_key(s);
      m = key_m(s, key);
      if (buf->b[j].run.len) {
        ok = key != kKeySpecial && key == buf->b[j].key && run_apply(buf->b[j].run, m);
        if (ok) s = ldexp((double)m, key >> 1);
      }
    }
    if (!ok) {  // element by element from the piece start (64 at a time through LDS)
      if (lane == 0) atomicAdd(redo, 1ull);
      s = s0;
      double *xs = reinterpret_cast<double *>(buf);
      const int kb = (p - p0) * kPiece, ke = min(d, kb + kPiece);
      for (int c0 = kb; c0 < ke; c0 += 64) {
        const int k = c0 + lane;
        const double2 v2 = k < ke ? xy[k] : make_double2(0.0, 0.0);
        wave_sync();
        xs[lane] = comp ? v2.y : v2.x;
        wave_sync();
        const int cn = min(64, ke - c0);
        for (int q = 0; q < cn; ++q) s = s + xs[q];
      }
      key = ulp_key(s);
      m = key_m(s, key);
    }
  }
  return s;
}

template <typename T>
__device__ inline T ld_stream(const T *p) {
  return __builtin_nontemporal_load(p);
}

// DIAG (timing-only builds selected by fu_set_option("diag", k); results are WRONG):
//   1 = the a_{r-1}[col e] gather replaced by a coalesced read (prices the gather);
//   2 = no flow load/store (prices the flow stream);
//   3 / 4 = the gather folded into the first n/2 / n/4 estimates (prices a smaller table);
//   5 = hub chains skipped (prices the exact sequential hub sums);
//   6 = the flow pass of multi-chunk heavy rows skips its estimate gathers;
//   12 = 1 and 2 together (prices col + the per-node arrays alone).
template <bool CHECK, bool NT, int DIAG = 0, int TE = kTileEdges, int TN = kTileNodes, int PART = 0>
__global__ __launch_bounds__(kBlock) void k_round_recon(
    const int4 *__restrict__ tiles, const int *__restrict__ rowptr,
    const int *__restrict__ col, const double *__restrict__ v, double *__restrict__ F,
    const double *__restrict__ a_prev, const double *__restrict__ a_prev2,
    double *__restrict__ a_new, const double *__restrict__ target,
    unsigned long long *__restrict__ err, const int *__restrict__ perm,
    const void *__restrict__ code_prev, void *__restrict__ code_new, PackCtl *__restrict__ ctl,
    int rslot, const double2 *__restrict__ hubxy, const int *__restrict__ hub_off,
    const int *__restrict__ hrows, const PieceSum *__restrict__ hsum, const int *__restrict__ hub_p0,
    unsigned long long *__restrict__ hub_redo, int hub_sep) {
  static_assert(TE % kBlock == 0 && TN <= kBlock && TN <= 256, "tile geometry");
  const PackCtl pp = ctl[rslot ^ 1];  // packing of a_{r-1} (the table gathered here)
  const PackCtl pc = ctl[2];          // packing of a_r (the table written here)
  if (blockIdx.x == 0 && threadIdx.x == 0) ctl[rslot] = pc;
  __shared__ double s_x[TE];   // f_{r-2} on load, fr after phase B
  __shared__ double s_er[TE];  // a_{r-1}[col e]
  __shared__ unsigned char s_own[TE];
  __shared__ int s_rp[TN + 1];
  __shared__ double s_a[TN];
  const int t = threadIdx.x;
  const int4 tl = tiles[blockIdx.x];
  unsigned long long eb = 0;

  if constexpr (PART != 1 && TE == kTileEdges && TN == kTileNodes) {
  if (tl.y == -2) {
    // ---------------- degree bin: R rows of similar degree, one chain per row ----------
    // Rows perm[tl.x .. tl.x + R) (sorted by degree, longest first). Each iteration stages
    // C = TE / R positions of every row in LDS, loaded along row segments (coalesced).
    // Then thread r runs row r's exact left-to-right chain over its C values. Element
    // (r, k) lives at r*C + (k ^ sw(r)): the XOR swizzle keeps the column reads of the
    // chain conflict-free without padding.
    const int R = tl.z, C = tl.w;
    const int lgC = 31 - __clz(C);
    // LDS reuse (no extra footprint): node ids and degrees in s_own's 2 KB, row starts in
    // s_rp, a_{r-2} of each row in s_a until the chains end, then a_r.
    int *s_node = reinterpret_cast<int *>(s_own);
    int *s_deg = s_node + kBlock;
    int *s_rb = s_rp;
    double *s_own2 = s_a;
    if (t < R) {
      const int node = perm[tl.x + t];
      s_node[t] = node;
      const int rb = rowptr[node];
      s_rb[t] = rb;
      s_deg[t] = rowptr[node + 1] - rb;
      s_own2[t] = a_prev2[node];
    }
    __syncthreads();
    auto sw = [&](int r) { return C >= 32 ? (r & 31) : ((r >> (5 - lgC)) & (C - 1)); };
    const int maxd = s_deg[0];
    const int my_deg = t < R ? s_deg[t] : 0;
    double S = 0.0, T = 0.0;
    for (int c0 = 0; c0 < maxd; c0 += C) {
#pragma unroll 4
      for (int q = t; q < R * C; q += kBlock) {
        const int r = q >> lgC, k = q & (C - 1);
        if (c0 + k < s_deg[r]) {
          const int e = s_rb[r] + c0 + k;
          const double er = ld_est(pp, code_prev, a_prev, col[e]);
          const int slot = (r << lgC) + (k ^ sw(r));
          s_x[slot] = recon_fr(ld_f(F, e), er, s_own2[r]);
          s_er[slot] = er;
        }
      }
      __syncthreads();
      if (t < R) {
        const int kend = min(C, my_deg - c0);
        const int base = t << lgC, x = sw(t);
        for (int k = 0; k < kend; ++k) {
          S = S + s_x[base + (k ^ x)];
          T = T + s_er[base + (k ^ x)];
        }
      }
      __syncthreads();
    }
    double a_mine = 0.0;
    if (t < R) {
      const int node = s_node[t];
      a_mine = ((v[node] - S) + T) / (double)(my_deg + 1);
      st_wt(a_new + node, a_mine);
      if (pc.width) put_code(pc, code_new, node, a_mine);
      if (CHECK) eb = err_bits(a_mine, target[node]);
    }
    __syncthreads();  // every read of s_own2 (aliases s_a) is done
    if (t < R) s_a[t] = a_mine;
    __syncthreads();
    if (maxd <= C) {  // one iteration: fr and er are still in LDS
      for (int q = t; q < R * C; q += kBlock) {
        const int r = q >> lgC, k = q & (C - 1);
        if (k < s_deg[r]) {
          const int slot = (r << lgC) + (k ^ sw(r));
          st_f_full(F, s_rb[r] + k, (s_x[slot] + s_a[r]) - s_er[slot]);
        }
      }
    } else {  // long rows: re-read the flow, re-gather the estimate (L2-warm)
      for (int r = 0; r < R; ++r) {
        const int rb = s_rb[r], d = s_deg[r];
        const double own2 = a_prev2[s_node[r]], a = s_a[r];
        for (int k = t; k < d; k += kBlock) {
          const double er = ld_est(pp, code_prev, a_prev, col[rb + k]);
          const double fo = ld_f(F, rb + k);
          st_f(F, rb + k, (recon_fr(fo, er, own2) + a) - er, fo);
        }
      }
    }
    if (CHECK) block_max_to(eb, err);
    return;
  }
  }  // if constexpr (default geometry)

  if constexpr (PART != 1) {  // heavy tiles (PART 1: light tiles only, 64 VGPRs)
  if (tl.y == -4) {
    // ---------------- heavy rows, one per wave ----------------
    // Rows hrows[tl.x .. tl.x + tl.z) (degree > hub_threshold, <= mega_hub, sorted by
    // degree so a block's waves finish together): wave w owns one row and its quarter of
    // s_x / s_er, stages the row chunk by chunk (each lane TE / 256 elements), runs the
    // exact left-to-right chain (lane-uniform) and rewrites the row's flows. No block
    // barrier: 4 rows per block progress independently.
    constexpr int CH = TE / 4, PL = CH / 64;
    const int w = t >> 6, lane = t & 63;
    if (w < tl.z) {
      const int i = hrows[tl.x + w];
      const int b = rowptr[i], e = rowptr[i + 1], d = e - b;
      const double own2 = a_prev2[i];
      double *xs = s_x + w * CH, *es = s_er + w * CH;
      double S = 0.0, T = 0.0;
      double fo[PL], er[PL];  // the last chunk's operands (a one-chunk row writes its flows from them)
      for (int c0 = 0; c0 < d; c0 += CH) {
        int cc[PL];
#pragma unroll
        for (int u = 0; u < PL; ++u) {
          const int k = c0 + lane + 64 * u;
          cc[u] = k < d ? col[b + k] : 0;
          fo[u] = k < d ? ld_f(F, b + k) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < PL; ++u) er[u] = c0 + lane + 64 * u < d ? ld_est(pp, code_prev, a_prev, cc[u]) : 0.0;
        wave_sync();  // the previous chunk's chain is done with the buffer
#pragma unroll
        for (int u = 0; u < PL; ++u) {
          xs[lane + 64 * u] = recon_fr(fo[u], er[u], own2);
          es[lane + 64 * u] = er[u];
        }
        wave_sync();
        if (DIAG != 5) chain_sum(xs, es, min(CH, d - c0), S, T);
      }
      const double a = ((v[i] - S) + T) / (double)(d + 1);
      if (lane == 0) {
        st_wt(a_new + i, a);
        if (pc.width) put_code(pc, code_new, i, a);
        if (CHECK) eb = err_bits(a, target[i]);
      }
      if (d <= CH) {  // flows (CA:117-118) from the registers that staged the row
#pragma unroll
        for (int u = 0; u < PL; ++u) {
          const int k = lane + 64 * u;
          if (k < d) st_f(F, b + k, (recon_fr(fo[u], er[u], own2) + a) - er[u], fo[u]);
        }
      } else
      for (int k0 = 0; k0 < d; k0 += 4 * 64) {  // flows (CA:117-118), 4 loads in flight per lane
        int cc[4];
        double fo[4], er[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int k = k0 + lane + 64 * u;
          cc[u] = k < d ? col[b + k] : 0;
          fo[u] = k < d ? ld_f(F, b + k) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          er[u] = k0 + lane + 64 * u < d ? (DIAG == 6 ? 0.0 : ld_est(pp, code_prev, a_prev, cc[u])) : 0.0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int k = k0 + lane + 64 * u;
          if (k < d) st_f(F, b + k, (recon_fr(fo[u], er[u], own2) + a) - er[u], fo[u]);
        }
      }
    }
    if (CHECK) block_max_to(eb, err);
    return;
  }

  if (tl.y == -3) {
    // ---------------- mega hub (degree > mega_hub, default 8192) ----------------
    // k_hub_stage has already put (fr, er) of every edge of the row into hubxy (many
    // blocks, coalesced), so the exact left-to-right chain is all that is left: wave 0
    // streams the pairs through two LDS halves (the loads of chunk c + 1 in flight while
    // chunk c is summed), with no block barrier and no gather on the chain's path.
    const int i = tl.x, b = tl.z, e = tl.w;
    const double2 *xy = hubxy + hub_off[blockIdx.x];
    const int d = e - b;
    double S = 0.0, T = 0.0;
    constexpr int CH = TE / 2, PL = CH / 64;  // pairs per chunk, per lane
    if (hsum) {
      // parallel exact sums: k_hub_sum summarised the pieces; wave 0 runs the serial pass
      // of S, wave 1 that of T, each in its own LDS buffer
      static_assert(2 * sizeof(PieceSum) <= sizeof(double) * TE, "LDS for the serial pass");
      PieceSum *bufs = reinterpret_cast<PieceSum *>(s_x);
      if (t < 128 && DIAG != 5) {
        const double r = hub_serial_pass(hsum, hub_p0[blockIdx.x], hub_p0[blockIdx.x + 1], t >> 6, xy, d,
                                         bufs + (t >> 6), hub_redo);
        if ((t & 63) == 0) s_a[t >> 6] = r;
      }
      __syncthreads();
      S = s_a[0];
      T = s_a[1];
      if (DIAG == 5) S = T = 0.0;
      __syncthreads();
    } else if (t < 64) {
      double2 nx[PL];
#pragma unroll
      for (int u = 0; u < PL; ++u) nx[u] = t + 64 * u < d ? xy[t + 64 * u] : make_double2(0.0, 0.0);
      for (int c0 = 0; c0 < d; c0 += CH) {
        double *xs = s_x + ((c0 / CH) & 1) * CH, *es = s_er + ((c0 / CH) & 1) * CH;
#pragma unroll
        for (int u = 0; u < PL; ++u) {
          xs[t + 64 * u] = nx[u].x;
          es[t + 64 * u] = nx[u].y;
        }
        const int c1 = c0 + CH;
#pragma unroll
        for (int u = 0; u < PL; ++u) {
          const int k = c1 + t + 64 * u;
          nx[u] = k < d ? xy[k] : make_double2(0.0, 0.0);
        }
        wave_sync();
        if (DIAG != 5) chain_sum(xs, es, min(CH, d - c0), S, T);
        wave_sync();
      }
    }
    if (t == 0) {
      const double a = ((v[i] - S) + T) / (double)(d + 1);
      s_a[0] = a;
      st_wt(a_new + i, a);
      if (pc.width) put_code(pc, code_new, i, a);
      if (CHECK) eb = err_bits(a, target[i]);
    }
    if (!hub_sep) {  // else k_hub_flows writes the row's flows with many blocks
      __syncthreads();
      const double a = s_a[0];
      for (int k = t; k < d; k += kBlock) {
        const double2 p2 = xy[k];
        const double fo = ld_f(F, b + k);
        st_f(F, b + k, (p2.x + a) - p2.y, fo);
      }
    }
    if (CHECK) block_max_to(eb, err);
    return;
  }

  if (tl.y < 0) {
    // ---------------- heavy node ----------------
    // chunks of CH = TE / 2 in the two halves of s_x / s_er: wave 0 runs the exact
    // left-to-right chain of chunk c (lane-uniform) while waves 1-3 stage chunk c + 1
    const int i = tl.x;
    const int b = rowptr[i], e = rowptr[i + 1];
    const double own2 = a_prev2[i];
    double S = 0.0, T = 0.0;
    constexpr int CH = TE / 2;
    const int nch = (e - b + CH - 1) / CH;
    auto stage = [&](int c, int tid, int nthr) {
      const int c0 = b + c * CH, cn = min(CH, e - c0);
      double *xs = s_x + (c & 1) * CH, *es = s_er + (c & 1) * CH;
      for (int q = tid; q < cn; q += nthr) {
        const double er = ld_est(pp, code_prev, a_prev, col[c0 + q]);
        xs[q] = recon_fr(ld_f(F, c0 + q), er, own2);
        es[q] = er;
      }
    };
    if (nch > 0) stage(0, t, kBlock);
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
      if (t >= 64) {
        if (c + 1 < nch) stage(c + 1, t - 64, kBlock - 64);
      } else if (DIAG != 5) {
        chain_sum(s_x + (c & 1) * CH, s_er + (c & 1) * CH, min(CH, e - (b + c * CH)), S, T);
      }
      __syncthreads();
    }
    if (t == 0) {
      const double a = ((v[i] - S) + T) / (double)(e - b + 1);
      s_a[0] = a;
      st_wt(a_new + i, a);
      if (pc.width) put_code(pc, code_new, i, a);
      if (CHECK) eb = err_bits(a, target[i]);
    }
    __syncthreads();
    const double a = s_a[0];
    for (int k = b + t; k < e; k += kBlock) {
      const double er = ld_est(pp, code_prev, a_prev, col[k]);
      const double fo = ld_f(F, k);
      st_f(F, k, (recon_fr(fo, er, own2) + a) - er, fo);
    }
    if (CHECK) block_max_to(eb, err);
    return;
  }
  }  // PART != 1
  if constexpr (PART != 2) {  // light tiles

  // ---------------- light tile ----------------
  // Every global load of the tile is issued up front with no dependence on an earlier load
  // except the a_{r-1}[col] gathers (one hop): 2 serial memory latencies per tile.
  const int nb = tl.x, nn = tl.y - tl.x;
  const int e0 = tl.z, ne = tl.w - tl.z;
  constexpr int kPer = TE / kBlock;
  int c[kPer];
  double x[kPer], g[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int q = t + k * kBlock;
    c[k] = 0;
    x[k] = 0.0;
    if (q < ne) {
      if (NT) {
        c[k] = ld_stream(col + e0 + q);
        x[k] = (DIAG == 2 || DIAG == 12) ? 0.0 : ld_f(F, e0 + q);
      } else {
        c[k] = col[e0 + q];
        x[k] = (DIAG == 2 || DIAG == 12) ? 0.0 : ld_f(F, e0 + q);
      }
    }
  }
  const int rp = t <= nn ? rowptr[nb + t] : 0;
  int rp_last = 0;
  if constexpr (TN == kBlock) rp_last = (t == 0 && nn == kBlock) ? rowptr[nb + kBlock] : 0;
  const double vv = t < nn ? v[nb + t] : 0.0;
  const double own2 = t < nn ? a_prev2[nb + t] : 0.0;
  if (DIAG != 0 || pp.width == 0) {
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int q = t + k * kBlock;
      g[k] = 0.0;
      if (q < ne) {
        const int gi = (DIAG == 1 || DIAG == 12) ? nb + (q % (nn + 1)) : DIAG == 3 ? (c[k] >> 1) : DIAG == 4 ? (c[k] >> 2) : c[k];
        g[k] = a_prev[gi];
      }
    }
  } else if (pp.width == 8) {
    gather_packed<8>(c, g, t, ne, code_prev, pp.base, a_prev);
  } else if (pp.width == 16) {
    gather_packed<16>(c, g, t, ne, code_prev, pp.base, a_prev);
  } else {
    gather_packed<32>(c, g, t, ne, code_prev, pp.base, a_prev);
  }
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int q = t + k * kBlock;
    if (q < ne) {
      s_x[q] = x[k];
      s_er[q] = g[k];
    }
  }
  if (t <= nn) s_rp[t] = rp;
  if constexpr (TN == kBlock) {
    if (t == 0 && nn == kBlock) s_rp[kBlock] = rp_last;
  }
  __syncthreads();
  // phase B: per node, reconstruct fr and sum in row order (CA:106-113)
  if (t < nn) {
    const int qb = s_rp[t] - e0, qe = s_rp[t + 1] - e0;
    double S = 0.0, T = 0.0;
    for (int q = qb; q < qe; ++q) {
      const double er = s_er[q];
      const double fr = recon_fr(s_x[q], er, own2);
      s_x[q] = fr;
      s_own[q] = (unsigned char)t;
      S = S + fr;
      T = T + er;
    }
    const double a = ((vv - S) + T) / (double)(qe - qb + 1);
    s_a[t] = a;
    st_wt(a_new + nb + t, a);
    if (pc.width) put_code(pc, code_new, nb + t, a);
    if (CHECK) eb = err_bits(a, target[nb + t]);
  }
  __syncthreads();
  // phase C: new flows, coalesced, in place (CA:117-118)
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int q = t + k * kBlock;
    if (q < ne) {
      const double fnew = (s_x[q] + s_a[s_own[q]]) - s_er[q];
      if (DIAG == 2 || DIAG == 12) {
        if (fnew == 12345.678) st_f_full(F, e0 + q, fnew);  // keep the value live, store ~never
      } else {
        st_f(F, e0 + q, fnew, x[k]);
      }
    }
  }
  if (CHECK) block_max_to(eb, err);
  }  // PART != 2
}

// ------------------------------------------------------------------------------------
// Variant 7: kernel 4's light tiles at WAVE granularity ("wave"). Same arithmetic and
// state as kernel 4 (flow reconstruction, packed gathers); each 64-lane wave owns one tile
// of <= TN nodes / <= TE edges and its own LDS slice, so there is no block barrier: a wave
// that finishes its loads proceeds without waiting for the other three, and more tiles are
// in flight per CU. Phase C keeps each edge's er and f_{r-2} in the registers that loaded
// them. Heavy rows (degree > min(hub_threshold, TE)) run through kernel 4's heavy path in
// a separate launch before this one.
// ------------------------------------------------------------------------------------

__device__ inline void wave_max_to(unsigned long long x, unsigned long long *dst) {
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long y = __shfl_xor(x, off, 64);
    x = x > y ? x : y;
  }
  if ((threadIdx.x & 63) == 0 && x && x > __hip_atomic_load(dst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
    atomicMax(dst, x);
}

template <bool CHECK, int TE, int TN>
__global__ __launch_bounds__(kBlock) void k_round_wave(
    const int4 *__restrict__ wtiles, int nwt, const int *__restrict__ rowptr,
    const int *__restrict__ col, const double *__restrict__ v, double *__restrict__ F,
    const double *__restrict__ a_prev, const double *__restrict__ a_prev2,
    double *__restrict__ a_new, const double *__restrict__ target,
    unsigned long long *__restrict__ err, const void *__restrict__ code_prev,
    void *__restrict__ code_new, PackCtl *__restrict__ ctl, int rslot) {
  static_assert(TE % 64 == 0 && TN <= 64 && TE <= 512, "wave tile geometry");
  constexpr int kW = kBlock / 64;
  constexpr int kPer = TE / 64;
  __shared__ double s_x[kW][TE];   // f_{r-2}, then fr after phase B
  __shared__ double s_er[kW][TE];  // a_{r-1}[col e]
  __shared__ unsigned short s_own[kW][TE];
  __shared__ int s_rp[kW][TN + 1];
  __shared__ double s_a[kW][TN];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const PackCtl pp = ctl[rslot ^ 1];
  const PackCtl pc = ctl[2];
  if (blockIdx.x == 0 && threadIdx.x == 0) ctl[rslot] = pc;
  const int tile = blockIdx.x * kW + w;
  if (tile >= nwt) return;  // no block barrier below: waves are independent
  const int4 tl = wtiles[tile];
  const int nb = tl.x, nn = tl.y - tl.x;
  const int e0 = tl.z, ne = tl.w - tl.z;
  int c[kPer];
  double x[kPer], g[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int q = lane + k * 64;
    c[k] = q < ne ? col[e0 + q] : 0;
    x[k] = q < ne ? ld_f(F, e0 + q) : 0.0;
  }
  const int rp = lane <= nn ? rowptr[nb + lane] : 0;
  const int rp_last = (TN == 64 && lane == 0 && nn == 64) ? rowptr[nb + 64] : 0;
  const double vv = lane < nn ? v[nb + lane] : 0.0;
  const double own2 = lane < nn ? a_prev2[nb + lane] : 0.0;
  if (pp.width == 0) {
#pragma unroll
    for (int k = 0; k < kPer; ++k) g[k] = lane + k * 64 < ne ? a_prev[c[k]] : 0.0;
  } else {
    unsigned cd[kPer];
    if (pp.width == 8) {
#pragma unroll
      for (int k = 0; k < kPer; ++k) cd[k] = lane + k * 64 < ne ? ld_code<8>(code_prev, c[k]) : 0u;
#pragma unroll
      for (int k = 0; k < kPer; ++k) g[k] = lane + k * 64 < ne ? decode_or<8>(cd[k], pp.base, a_prev, c[k]) : 0.0;
    } else if (pp.width == 16) {
#pragma unroll
      for (int k = 0; k < kPer; ++k) cd[k] = lane + k * 64 < ne ? ld_code<16>(code_prev, c[k]) : 0u;
#pragma unroll
      for (int k = 0; k < kPer; ++k) g[k] = lane + k * 64 < ne ? decode_or<16>(cd[k], pp.base, a_prev, c[k]) : 0.0;
    } else {
#pragma unroll
      for (int k = 0; k < kPer; ++k) cd[k] = lane + k * 64 < ne ? ld_code<32>(code_prev, c[k]) : 0u;
#pragma unroll
      for (int k = 0; k < kPer; ++k) g[k] = lane + k * 64 < ne ? decode_or<32>(cd[k], pp.base, a_prev, c[k]) : 0.0;
    }
  }
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int q = lane + k * 64;
    if (q < ne) {
      s_x[w][q] = x[k];
      s_er[w][q] = g[k];
    }
  }
  if (lane <= nn && lane <= TN) s_rp[w][lane] = rp;
  if (TN == 64 && lane == 0 && nn == 64) s_rp[w][64] = rp_last;
  wave_sync();
  // phase B: one lane per node, its row in order (CA:106-113)
  unsigned long long eb = 0;
  if (lane < nn) {
    const int qb = s_rp[w][lane] - e0, qe = s_rp[w][lane + 1] - e0;
    double S = 0.0, T = 0.0;
    for (int q = qb; q < qe; ++q) {
      const double er = s_er[w][q];
      const double fr = recon_fr(s_x[w][q], er, own2);
      s_x[w][q] = fr;
      s_own[w][q] = (unsigned short)lane;
      S = S + fr;
      T = T + er;
    }
    const double a = ((vv - S) + T) / (double)(qe - qb + 1);
    s_a[w][lane] = a;
    st_wt(a_new + nb + lane, a);
    if (pc.width) put_code(pc, code_new, nb + lane, a);
    if (CHECK) eb = err_bits(a, target[nb + lane]);
  }
  wave_sync();
  // phase C: new flows, coalesced, in place (CA:117-118); er from the loading registers
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int q = lane + k * 64;
    if (q < ne) st_f(F, e0 + q, (s_x[w][q] + s_a[w][s_own[w][q]]) - g[k], x[k]);
  }
  if (CHECK) wave_max_to(eb, err);
}

// ------------------------------------------------------------------------------------
// Variant 8: LDS-staged slices ("stage"). The a_{r-1}[col e] gather is the part of a round
// that does not stream: on ER every gather is a random L2 request (8 M per round), and the
// fp64 table (8 MB) does not fit an XCD's 4 MB L2. Kernel 8 splits it into two launches:
//   * k_stage: the estimate table (codes, or doubles while unpacked) is cut into slices of
//     64 KB; a block copies slice s into LDS, then streams the slice-s column offsets of its
//     edge groups (u16) and writes the looked-up table elements to G, in the same
//     (group, slice, tile, position) order: coalesced reads and writes, gathers from LDS.
//   * k_round_staged: kernel 4's light tile (flow reconstruction, CA:98-99 + CA:105-128),
//     where each edge's estimate comes from G (contiguous runs of the tile) through a u32
//     {index in the group's G region, position in the tile} instead of col + gather.
// The layout depends on the table's element width (slice = 65536 / bytes nodes). The host
// builds it for the width it last saw; a table wider than the layout is still handled (the
// stage launch gathers it from global memory), so correctness never depends on the host's
// view of the device-side packing plan. Rows above the tile limit run as kernel 4 heavy
// tiles in a launch of their own. Results are bitwise those of kernel 4.
// ------------------------------------------------------------------------------------
constexpr int kStageThreads = 512;
constexpr int kStageLds = 65536;  // bytes of table per slice
constexpr int kStageTE = 1024, kStageTN = 128;

// The slice layouts (element bytes 1, 2, 4, 8) passed by value to the stage and round
// launches; the device picks the layout from the table's actual packing width, so the
// choice never depends on the host having seen the (asynchronous) packing plan.
struct StageArgs {
  int P[4], Q[4];
  const int *aoff[4];
  const int2 *aitem[4];
  const unsigned short *colS[4];
  const unsigned *sidx[4];
  const int *gbase[4];
  const unsigned short *sidx16[4];  // compact sidx (null: use sidx)
  const int *dtab[4];
  int sel[4];  // layout used for tables of width 8, 16, 32, 0 (0..3)
};
constexpr int kStageRuns = 64;  // slice runs per tile the compact sidx can address
__device__ __forceinline__ int width_index(int width) {
  return width == 8 ? 0 : width == 16 ? 1 : width == 32 ? 2 : 3;
}

constexpr int kStagePad = 8;      // segment padding: 8 consecutive elements per lane access
constexpr int kStageItem = 1024;  // elements per stage item (one wave: 2 x 8 per lane)
constexpr int kStageIU = kStageItem / (64 * kStagePad);
constexpr int kStageChunk = 256;  // item descriptors staged in LDS at a time

// One stage item (<= 1024 consecutive elements of one padded segment, one wave): lane l
// loads the column offsets of elements x + 8 (l + 64 u) .. + 7 with one 16-byte load each.
template <typename T>
__device__ __forceinline__ void stage_item_load(uint4 (&o)[kStageIU], int2 itm, int lane,
                                                const unsigned short *__restrict__ colS) {
#pragma unroll
  for (int u = 0; u < kStageIU; ++u) {
    const int k = itm.x + kStagePad * (lane + 64 * u);
    o[u] = *reinterpret_cast<const uint4 *>(colS + (k < itm.x + itm.y ? k : itm.x));
  }
}
template <typename T, bool LDS>
__device__ __forceinline__ void stage_item_store(const uint4 (&o)[kStageIU], int2 itm, int lane,
                                                 const unsigned char *s_tab, const T *__restrict__ tab,
                                                 int nb, T *__restrict__ G) {
#pragma unroll
  for (int u = 0; u < kStageIU; ++u) {
    const int k = itm.x + kStagePad * (lane + 64 * u);
    const unsigned w4[4] = {o[u].x, o[u].y, o[u].z, o[u].w};
    T val[kStagePad];
#pragma unroll
    for (int j = 0; j < kStagePad; ++j) {
      const unsigned off = (w4[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
      if constexpr (LDS) val[j] = reinterpret_cast<const T *>(s_tab)[off];
      else val[j] = tab[nb + (int)off];
    }
    if (k < itm.x + itm.y) {  // 8 consecutive elements, 16-byte aligned stores
      if constexpr (sizeof(T) == 1) {
        uint2 v;
        v.x = val[0] | (val[1] << 8) | (val[2] << 16) | ((unsigned)val[3] << 24);
        v.y = val[4] | (val[5] << 8) | (val[6] << 16) | ((unsigned)val[7] << 24);
        *reinterpret_cast<uint2 *>(G + k) = v;
      } else if constexpr (sizeof(T) == 2) {
        uint4 v;
        v.x = val[0] | ((unsigned)val[1] << 16);
        v.y = val[2] | ((unsigned)val[3] << 16);
        v.z = val[4] | ((unsigned)val[5] << 16);
        v.w = val[6] | ((unsigned)val[7] << 16);
        *reinterpret_cast<uint4 *>(G + k) = v;
      } else {
#pragma unroll
        for (int j = 0; j < kStagePad; j += 16 / (int)sizeof(T)) {
          uint4 v;
          __builtin_memcpy(&v, &val[j], 16);
          *reinterpret_cast<uint4 *>(G + k + j) = v;
        }
      }
    }
  }
}

// One stage block: slice s of the table (element type T) -> LDS (LDS = false: read from
// global memory, the table being wider than the layout), then its items, wave w taking
// items ib + w, ib + w + 8, ... Every load of an item is issued before any of its uses, and
// the next item's loads are issued before the current item is looked up and stored
// (two register sets, unrolled by two so no in-flight register is copied).
template <typename T, bool LDS>
__device__ __forceinline__ void stage_body(unsigned char *s_tab, int2 *s_items, int nb, int cnt,
                                           const int2 *__restrict__ items, int ib, int ie,
                                           const unsigned short *__restrict__ colS,
                                           const T *__restrict__ tab, T *__restrict__ G) {
  constexpr int kW = kStageLds / 16 / kStageThreads;
  constexpr int NW = kStageThreads / 64;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint4 buf[kW];
  const int bytes = LDS ? cnt * (int)sizeof(T) : 0;
  const int w16 = bytes >> 4;
  const uint4 *s16 = reinterpret_cast<const uint4 *>(tab + nb);
  if constexpr (LDS) {
#pragma unroll
    for (int u = 0; u < kW; ++u) {
      const int k = t + u * kStageThreads;
      buf[u] = k < w16 ? s16[k] : make_uint4(0u, 0u, 0u, 0u);
    }
  }
  const int2 z = make_int2(0, 0);
  bool filled = !LDS;
  // the block's item descriptors go through LDS in chunks of kStageChunk (one chunk on
  // ER-1M), so a wave never waits on a descriptor load behind its own column loads
  for (int cb = ib; cb < ie || !filled; cb += kStageChunk) {
    const int ce = min(ie, cb + kStageChunk);
    if (cb > ib) __syncthreads();  // previous chunk consumed
    for (int i = t; i < ce - cb; i += kStageThreads) s_items[i] = items[cb + i];
    __syncthreads();
    int it = w;
    const int nit = ce - cb;
    int2 i0 = it < nit ? s_items[it] : z;
    uint4 o0[kStageIU], o1[kStageIU];
    stage_item_load<T>(o0, i0, lane, colS);
    if (!filled) {  // slice stores after the first item's loads are in flight
#pragma unroll
      for (int u = 0; u < kW; ++u) {
        const int k = t + u * kStageThreads;
        if (k < w16) reinterpret_cast<uint4 *>(s_tab)[k] = buf[u];
      }
      const int tb = w16 << 4;
      if (t < bytes - tb) s_tab[tb + t] = reinterpret_cast<const unsigned char *>(tab + nb)[tb + t];
      __syncthreads();
      filled = true;
    }
    while (it < nit) {
      const int2 i1 = it + NW < nit ? s_items[it + NW] : z;
      stage_item_load<T>(o1, i1, lane, colS);
      stage_item_store<T, LDS>(o0, i0, lane, s_tab, tab, nb, G);
      it += NW;
      if (it >= nit) break;
      i0 = it + NW < nit ? s_items[it + NW] : z;
      stage_item_load<T>(o0, i0, lane, colS);
      stage_item_store<T, LDS>(o1, i1, lane, s_tab, tab, nb, G);
      it += NW;
    }
  }
}

__global__ __launch_bounds__(kStageThreads) void k_stage(StageArgs sa, int n,
                                                        const double *__restrict__ a_prev,
                                                        const void *__restrict__ code_prev,
                                                        const PackCtl *__restrict__ ctl, int rslot,
                                                        void *__restrict__ G) {
  __shared__ __align__(16) unsigned char s_tab[kStageLds];
  __shared__ int2 s_items[kStageChunk];
  const PackCtl pp = ctl[rslot ^ 1];
  const int wb = pp.width ? pp.width / 8 : 8;  // bytes per element of the table gathered
  const int li = sa.sel[width_index(pp.width)];
  const int P = sa.P[li];
  if ((int)blockIdx.x >= P * sa.Q[li]) return;
  const int LB = 1 << li;  // bytes per element the layout was built for
  const int SN = kStageLds >> li;
  const int s = blockIdx.x % P;
  const int nb = s * SN;
  const int cnt = min(SN, n - nb);
  const void *src = pp.width ? code_prev : static_cast<const void *>(a_prev);
  const unsigned short *colS = sa.colS[li];
  const int2 *aitem = sa.aitem[li];
  // this block's items {first element, count <= kStageItem}
  const int ib = sa.aoff[li][blockIdx.x], ie = sa.aoff[li][blockIdx.x + 1];
#define FU_BODY(T)                                                                                  \
  do {                                                                                              \
    if ((int)sizeof(T) <= LB)                                                                       \
      stage_body<T, true>(s_tab, s_items, nb, cnt, aitem, ib, ie, colS, reinterpret_cast<const T *>(src), \
                          reinterpret_cast<T *>(G));                                                \
    else                                                                                            \
      stage_body<T, false>(s_tab, s_items, nb, cnt, aitem, ib, ie, colS, reinterpret_cast<const T *>(src), \
                           reinterpret_cast<T *>(G));                                               \
  } while (0)
  if (wb == 1) FU_BODY(unsigned char);
  else if (wb == 2) FU_BODY(unsigned short);
  else if (wb == 4) FU_BODY(unsigned);
  else FU_BODY(unsigned long long);
#undef FU_BODY
}

// DIAG (timing only, wrong results): 1 = G read at the edge's own index (prices the runs),
// 2 = no stage launch and G read as in 1 (prices the round without staging), 3 = 2 without
// the XCD tile order; 4 = no stage launch, G read as usual (prices the round launch alone).
template <bool CHECK, int TE, int TN, int DIAG = 0>
__global__ __launch_bounds__(kBlock) void k_round_staged(
    const int4 *__restrict__ tiles, const int *__restrict__ tgbase, int ntl,
    const int *__restrict__ rowptr, const int *__restrict__ col,
    const StageArgs sa, const void *__restrict__ G, const double *__restrict__ v,
    double *__restrict__ F, const double *__restrict__ a_prev, const double *__restrict__ a_prev2,
    double *__restrict__ a_new, const double *__restrict__ target,
    unsigned long long *__restrict__ err, void *__restrict__ code_new, PackCtl *__restrict__ ctl,
    int rslot) {
  static_assert(TE % kBlock == 0 && TN <= kBlock, "tile geometry");
  const PackCtl pp = ctl[rslot ^ 1];
  const int lsel = sa.sel[width_index(pp.width)];
  const unsigned *__restrict__ sidx = sa.sidx[lsel];
  const PackCtl pc = ctl[2];
  if (blockIdx.x == 0 && threadIdx.x == 0) ctl[rslot] = pc;
  __shared__ double s_x[TE];
  __shared__ double s_er[TE];
  __shared__ unsigned char s_own[TE];
  __shared__ int s_rp[TN + 1];
  __shared__ double s_a[TN];
  const int t = threadIdx.x;
  unsigned long long eb = 0;
  // XCD-aware order: block b runs on XCD b % 8; consecutive tiles (one edge group, whose G
  // region the tiles share) go to the same XCD, so that region is fetched into one L2
  const int xcd = blockIdx.x & 7, per = ntl >> 3, rem = ntl & 7;
  const int tile = DIAG == 3 ? (int)blockIdx.x : xcd * per + min(xcd, rem) + (int)(blockIdx.x >> 3);
  const int4 tl = tiles[tile];
  const int gb = sa.gbase[lsel][tile];
  const int nb = tl.x, nn = tl.y - tl.x;
  const int e0 = tl.z, ne = tl.w - tl.z;
  constexpr int kPer = TE / kBlock;
  const unsigned short *__restrict__ s16 = sa.sidx16[lsel];
  unsigned si[kPer];  // position in the tile (low 16 bits) | G index in the group (high 16)
  double x[kPer], g[kPer];
  int gi[kPer];
  if (s16) {  // compact: u16 position | run << 10; G index = gbase + m + D[run] (lane run holds D)
    const int dl = sa.dtab[lsel][(size_t)tile * kStageRuns + (t & 63)];
    unsigned short c16[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int q = t + k * kBlock;
      c16[k] = q < ne ? s16[e0 + q] : (unsigned short)0;
      x[k] = q < ne ? ld_f(F, e0 + q) : 0.0;
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int q = t + k * kBlock;
      const int dd = __shfl(dl, (int)(c16[k] >> 10));
      si[k] = c16[k] & 1023u;
      gi[k] = q < ne ? ((DIAG >= 1 && DIAG <= 3) ? e0 + q : gb + q + dd) : -1;
    }
  } else {
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int q = t + k * kBlock;
      si[k] = q < ne ? sidx[e0 + q] : 0u;
      x[k] = q < ne ? ld_f(F, e0 + q) : 0.0;
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k)
      gi[k] = t + k * kBlock < ne ? ((DIAG >= 1 && DIAG <= 3) ? e0 + t + k * kBlock : gb + (int)(si[k] >> 16)) : -1;
  }
  const int rp = t <= nn ? rowptr[nb + t] : 0;
  const double vv = t < nn ? v[nb + t] : 0.0;
  const double own2 = t < nn ? a_prev2[nb + t] : 0.0;
  // every G load of the tile first, then decode (escapes gather the double via col)
  if (pp.width == 0) {
#pragma unroll
    for (int k = 0; k < kPer; ++k) g[k] = gi[k] >= 0 ? reinterpret_cast<const double *>(G)[gi[k]] : 0.0;
  } else {
    unsigned cd[kPer];
    unsigned esc;
    if (pp.width == 8) {
      esc = 0xFFu;
#pragma unroll
      for (int k = 0; k < kPer; ++k) cd[k] = gi[k] >= 0 ? reinterpret_cast<const unsigned char *>(G)[gi[k]] : 0u;
    } else if (pp.width == 16) {
      esc = 0xFFFFu;
#pragma unroll
      for (int k = 0; k < kPer; ++k) cd[k] = gi[k] >= 0 ? reinterpret_cast<const unsigned short *>(G)[gi[k]] : 0u;
    } else {
      esc = 0xFFFFFFFFu;
#pragma unroll
      for (int k = 0; k < kPer; ++k) cd[k] = gi[k] >= 0 ? reinterpret_cast<const unsigned *>(G)[gi[k]] : 0u;
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k)
      g[k] = gi[k] < 0 ? 0.0 : cd[k] == esc ? a_prev[col[e0 + (int)(si[k] & 0xFFFFu)]] : dkey_inv(pp.base + cd[k]);
  }
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int q = t + k * kBlock;
    if (q < ne) {
      s_x[q] = x[k];
      s_er[si[k] & 0xFFFFu] = g[k];
    }
  }
  if (t <= nn) s_rp[t] = rp;
  __syncthreads();
  if (t < nn) {  // phase B (CA:106-113)
    const int qb = s_rp[t] - e0, qe = s_rp[t + 1] - e0;
    double S = 0.0, T = 0.0;
    for (int q = qb; q < qe; ++q) {
      const double er = s_er[q];
      const double fr = recon_fr(s_x[q], er, own2);
      s_x[q] = fr;
      s_own[q] = (unsigned char)t;
      S = S + fr;
      T = T + er;
    }
    const double a = ((vv - S) + T) / (double)(qe - qb + 1);
    s_a[t] = a;
    st_wt(a_new + nb + t, a);
    if (pc.width) put_code(pc, code_new, nb + t, a);
    if (CHECK) eb = err_bits(a, target[nb + t]);
  }
  __syncthreads();
  // phase C: new flows, coalesced, in place (CA:117-118)
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int q = t + k * kBlock;
    if (q < ne) {
      st_f(F, e0 + q, (s_x[q] + s_a[s_own[q]]) - s_er[q], x[k]);
    }
  }
  if (CHECK) block_max_to(eb, err);
}

// ------------------------------------------------------------------------------------
// Variant 9: persistent, software-pipelined round ("pipe"). Kernels 4 and 8 run one tile
// per block through load -> gather -> LDS -> row chains -> store, so a block's memory
// latency is exposed once per tile and the chip runs short of bytes in flight (kernel 4
// without its gather still only streams 5.4 TB/s). Here a block owns a list of light tiles
// (1024 edges / 128 nodes, on its XCD) and keeps two of them ahead of the one it computes:
// while tile i is staged in LDS and summed, the estimate loads of tile i+1 and the stream
// loads (edges, flows, node arrays) of tile i+2 are in flight. LDS is double-buffered by
// tile parity, so two barriers per tile suffice. Rows above the tile limit (hubs) get
// blocks of their own at the front of the grid (kernel 4's exact chunked chain).
// MODE 0: per edge col -> a_{r-1}[col] (or its packed code); MODE 1: the staged runs of
// kernel 8 (sidx -> G). Arithmetic identical to kernel 4 (CA:98-99, CA:105-128).
// ------------------------------------------------------------------------------------
constexpr int kPipeTE = 1024, kPipeTN = 128, kPipeKP = kPipeTE / kBlock;
constexpr int kPipeChunk = 64;  // max tiles per block (host sizes the grid accordingly)

struct PipeStream {
  int nb, nn, e0, ne, gb;
  unsigned c[kPipeKP];  // MODE 0: col; MODE 1: sidx
  double x[kPipeKP];    // f_{r-2}
  int rp;
  double vv, own2;
};

// Every load of the pipeline is unconditional, with indices clamped into the arrays, so
// the loop body is straight-line code and the compiler can wait for exactly the loads an
// instruction consumes (a guarded load makes it fall back to waiting for all of them,
// prefetches included). Lanes past the tile read valid but unused elements.
template <int MODE>
__device__ inline void pipe_load(PipeStream &s, int it, int m, const int4 *s_tl, const int *s_gb,
                                 const int *__restrict__ rowptr, const unsigned *__restrict__ cidx,
                                 const double *__restrict__ F, const double *__restrict__ v,
                                 const double *__restrict__ a_prev2, int elast) {
  const int t = threadIdx.x;
  const int itc = it < m ? it : 0;
  const int4 tl = s_tl[itc];
  const bool live = it < m;
  s.nb = tl.x;
  s.nn = live ? tl.y - tl.x : -1;
  s.e0 = tl.z;
  s.ne = live ? tl.w - tl.z : 0;
  s.gb = MODE ? s_gb[itc] : 0;
#pragma unroll
  for (int k = 0; k < kPipeKP; ++k) {
    const int e = min(s.e0 + t + k * kBlock, elast);
    s.c[k] = cidx[e];
    s.x[k] = ld_f(F, e);
  }
  const int nn = tl.y - tl.x;
  s.rp = rowptr[s.nb + min(t, nn)];
  const int i = s.nb + min(t, max(nn - 1, 0));
  s.vv = v[i];
  s.own2 = a_prev2[i];
}

// raw estimate words of one tile (W = 0: the double's bits; else the W-bit code)
template <int MODE, int W>
__device__ inline void pipe_gather(unsigned long long (&raw)[kPipeKP], const PipeStream &s,
                                   const void *__restrict__ tab, const double *__restrict__ a_prev) {
#pragma unroll
  for (int k = 0; k < kPipeKP; ++k) {
    const int gi = MODE ? s.gb + (int)(s.c[k] >> 16) : (int)s.c[k];
    if constexpr (W == 0) raw[k] = reinterpret_cast<const unsigned long long *>(MODE ? tab : a_prev)[gi];
    else if constexpr (W == 8) raw[k] = reinterpret_cast<const unsigned char *>(tab)[gi];
    else if constexpr (W == 16) raw[k] = reinterpret_cast<const unsigned short *>(tab)[gi];
    else raw[k] = reinterpret_cast<const unsigned *>(tab)[gi];
  }
}

struct PipeLds {
  double x[2][kPipeTE];
  double er[2][kPipeTE];
  unsigned char own[2][kPipeTE];
  int rp[2][kPipeTN + 1];
  double a[2][kPipeTN];
  int4 tl[kPipeChunk];
  int gb[kPipeChunk];
};

// One pipeline step: compute tile `it` (stream registers sa, estimate words ga) while the
// estimates of tile it+1 (stream sb, into gb) and the stream of tile it+2 (into sc) load.
// The caller unrolls the step over the 3 x 2 register sets (period 6), so no register is
// ever copied while a load into it is in flight (a copy would wait for that load).
template <bool CHECK, int MODE, int W>
__device__ inline void pipe_step(
    PipeLds &L, int it, int m, PipeStream &sa, const PipeStream &sb, PipeStream &sc,
    unsigned long long (&ga)[kPipeKP], unsigned long long (&gb)[kPipeKP], unsigned long long &eb,
    const int *__restrict__ rowptr, const int *__restrict__ col, const unsigned *__restrict__ cidx,
    const void *__restrict__ tab, const double *__restrict__ v, double *__restrict__ F,
    const double *__restrict__ a_prev, const double *__restrict__ a_prev2, double *__restrict__ a_new,
    const double *__restrict__ target, void *__restrict__ code_new, const PackCtl &pp,
    const PackCtl &pc, int elast) {
  constexpr int KP = kPipeKP;
  const int t = threadIdx.x;
  const int bf = it & 1;
  pipe_gather<MODE, W>(gb, sb, tab, a_prev);                                       // tile it+1
  pipe_load<MODE>(sc, it + 2, m, L.tl, L.gb, rowptr, cidx, F, v, a_prev2, elast);  // tile it+2
  bool any_esc = false;
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    const int q = t + k * kBlock;
    double er;
    if constexpr (W == 0) {
      er = __longlong_as_double((long long)ga[k]);
    } else {
      constexpr unsigned long long esc = W == 32 ? 0xFFFFFFFFull : (1ull << W) - 1ull;
      er = dkey_inv(pp.base + ga[k]);
      any_esc |= q < sa.ne && ga[k] == esc;
    }
    if (q < sa.ne) {
      L.x[bf][q] = sa.x[k];
      L.er[bf][MODE ? (int)(sa.c[k] & 0xFFFFu) : q] = er;
    }
  }
  if constexpr (W != 0) {
    // escapes (rare): the double, through the edge's column, written over the LDS slot. The
    // load completes inside the branch (explicit wait), so the common path never waits for
    // it, and with it for every prefetch issued before it.
    if (__builtin_expect(__any(any_esc), 0)) {
      constexpr unsigned long long esc = W == 32 ? 0xFFFFFFFFull : (1ull << W) - 1ull;
#pragma unroll
      for (int k = 0; k < KP; ++k) {
        const int q = t + k * kBlock;
        if (q < sa.ne && ga[k] == esc) {
          const int pos = MODE ? (int)(sa.c[k] & 0xFFFFu) : q;
          L.er[bf][pos] = a_prev[MODE ? col[sa.e0 + pos] : (int)sa.c[k]];
        }
      }
      __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) expcnt(0) lgkmcnt(0)
    }
  }
  if (t <= sa.nn) L.rp[bf][t] = sa.rp;
  __syncthreads();
  if (t < sa.nn) {  // phase B (CA:106-113)
    const int qb = L.rp[bf][t] - sa.e0, qe = L.rp[bf][t + 1] - sa.e0;
    double S = 0.0, T = 0.0;
    for (int q = qb; q < qe; ++q) {
      const double e_ = L.er[bf][q];
      const double fr = recon_fr(L.x[bf][q], e_, sa.own2);
      L.x[bf][q] = fr;
      L.own[bf][q] = (unsigned char)t;
      S = S + fr;
      T = T + e_;
    }
    const double a = ((sa.vv - S) + T) / (double)(qe - qb + 1);
    L.a[bf][t] = a;
    st_wt(a_new + sa.nb + t, a);
    if (pc.width) put_code(pc, code_new, sa.nb + t, a);
    if (CHECK) {
      const unsigned long long b2 = err_bits(a, target[sa.nb + t]);
      eb = b2 > eb ? b2 : eb;
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < KP; ++k) {  // phase C (CA:117-118)
    const int q = t + k * kBlock;
    if (q < sa.ne) {
      st_f(F, sa.e0 + q, (L.x[bf][q] + L.a[bf][L.own[bf][q]]) - L.er[bf][q], sa.x[k]);
    }
  }
}

template <bool CHECK, int MODE, int W>
__device__ inline unsigned long long pipe_tiles(
    PipeLds &L, int m, const int *__restrict__ rowptr, const int *__restrict__ col,
    const unsigned *__restrict__ cidx, const void *__restrict__ tab, const double *__restrict__ v,
    double *__restrict__ F, const double *__restrict__ a_prev, const double *__restrict__ a_prev2,
    double *__restrict__ a_new, const double *__restrict__ target, void *__restrict__ code_new,
    const PackCtl &pp, const PackCtl &pc, int elast) {
  unsigned long long eb = 0;
  PipeStream s0, s1, s2;
  unsigned long long g0[kPipeKP], g1[kPipeKP];
  pipe_load<MODE>(s0, 0, m, L.tl, L.gb, rowptr, cidx, F, v, a_prev2, elast);
  pipe_load<MODE>(s1, 1, m, L.tl, L.gb, rowptr, cidx, F, v, a_prev2, elast);
  pipe_gather<MODE, W>(g0, s0, tab, a_prev);
#define FU_STEP(K, SA, SB, SC, GA, GB)                                                             \
  if (it + K >= m) break;                                                                          \
  pipe_step<CHECK, MODE, W>(L, it + K, m, SA, SB, SC, GA, GB, eb, rowptr, col, cidx, tab, v, F,    \
                            a_prev, a_prev2, a_new, target, code_new, pp, pc, elast)
  for (int it = 0; it < m; it += 6) {
    FU_STEP(0, s0, s1, s2, g0, g1);
    FU_STEP(1, s1, s2, s0, g1, g0);
    FU_STEP(2, s2, s0, s1, g0, g1);
    FU_STEP(3, s0, s1, s2, g1, g0);
    FU_STEP(4, s1, s2, s0, g0, g1);
    FU_STEP(5, s2, s0, s1, g1, g0);
  }
#undef FU_STEP
  return eb;
}

template <bool CHECK, int MODE>
__global__ __launch_bounds__(kBlock) void k_round_pipe(
    const int4 *__restrict__ tiles, const int *__restrict__ tgbase, int ntl,
    const int4 *__restrict__ heavy, int nheavy, const int *__restrict__ rowptr,
    const int *__restrict__ col, const StageArgs sa, const void *__restrict__ G,
    const double *__restrict__ v, double *__restrict__ F, const double *__restrict__ a_prev,
    const double *__restrict__ a_prev2, double *__restrict__ a_new,
    const double *__restrict__ target, unsigned long long *__restrict__ err,
    const void *__restrict__ code_prev, void *__restrict__ code_new, PackCtl *__restrict__ ctl,
    int rslot, int elast) {
  constexpr int TE = kPipeTE;
  __shared__ PipeLds L;
  const PackCtl pp = ctl[rslot ^ 1];
  const PackCtl pc = ctl[2];
  if (blockIdx.x == 0 && threadIdx.x == 0) ctl[rslot] = pc;
  const int t = threadIdx.x;
  unsigned long long eb = 0;

  if ((int)blockIdx.x < nheavy) {
    // ---------------- heavy row: kernel 4's exact chunked chain ----------------
    // chunks of TE in the two LDS buffers: wave 0 chains chunk c while waves 1-3 stage c + 1
    const int4 tl = heavy[blockIdx.x];
    const int i = tl.x, b = tl.z, e = tl.w;
    const double own2 = a_prev2[i];
    double S = 0.0, T = 0.0;
    const int nch = (e - b + TE - 1) / TE;
    auto stage = [&](int c, int tid, int nthr) {
      const int c0 = b + c * TE, cn = min(TE, e - c0);
      for (int q = tid; q < cn; q += nthr) {
        const double er = ld_est(pp, code_prev, a_prev, col[c0 + q]);
        L.x[c & 1][q] = recon_fr(ld_f(F, c0 + q), er, own2);
        L.er[c & 1][q] = er;
      }
    };
    if (nch > 0) stage(0, t, kBlock);
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
      if (t >= 64) {
        if (c + 1 < nch) stage(c + 1, t - 64, kBlock - 64);
      } else {
        chain_sum(L.x[c & 1], L.er[c & 1], min(TE, e - (b + c * TE)), S, T);
      }
      __syncthreads();
    }
    if (t == 0) {
      const double a = ((v[i] - S) + T) / (double)(e - b + 1);
      L.a[0][0] = a;
      st_wt(a_new + i, a);
      if (pc.width) put_code(pc, code_new, i, a);
      if (CHECK) eb = err_bits(a, target[i]);
    }
    __syncthreads();
    const double a = L.a[0][0];
    for (int k = b + t; k < e; k += kBlock) {
      const double er = ld_est(pp, code_prev, a_prev, col[k]);
      const double fo = ld_f(F, k);
      st_f(F, k, (recon_fr(fo, er, own2) + a) - er, fo);
    }
    if (CHECK) block_max_to(eb, err);
    return;
  }

  // ---------------- light tiles: this block's list (XCD-aware) ----------------
  const int bid = (int)blockIdx.x - nheavy, nbl = (int)gridDim.x - nheavy;  // nbl % 8 == 0
  const int x = bid & 7, j = bid >> 3, nbx = nbl >> 3;
  const int per = ntl >> 3, rem = ntl & 7;
  const int lo = x * per + min(x, rem), hi = lo + per + (x < rem ? 1 : 0);
  const int m = j < hi - lo ? (hi - lo - j + nbx - 1) / nbx : 0;
  if (t < m) {
    L.tl[t] = tiles[lo + j + t * nbx];
    if (MODE) L.gb[t] = sa.gbase[sa.sel[width_index(pp.width)]][lo + j + t * nbx];
  }
  if (t == 0 && m == 0) {  // keep the clamped prefetch of an empty list in bounds
    L.tl[0] = make_int4(0, 0, 0, 0);
    L.gb[0] = 0;
  }
  __syncthreads();
  const unsigned *cidx = MODE ? sa.sidx[sa.sel[width_index(pp.width)]] : reinterpret_cast<const unsigned *>(col);
  const void *tab = MODE ? G : code_prev;
#define FU_TILES(W_)                                                                                  \
  pipe_tiles<CHECK, MODE, W_>(L, m, rowptr, col, cidx, tab, v, F, a_prev, a_prev2, a_new, target,     \
                              code_new, pp, pc, elast)
  if (pp.width == 0) eb = FU_TILES(0);
  else if (pp.width == 8) eb = FU_TILES(8);
  else if (pp.width == 16) eb = FU_TILES(16);
  else eb = FU_TILES(32);
#undef FU_TILES
  if (CHECK) block_max_to(eb, err);
}

// Mega hubs: (fr, er) of every hub edge into hubxy, hub-major (CA:98-99 + the flow
// reconstruction of kernel 4), so k_round_recon's hub block only runs the chain.
__global__ __launch_bounds__(kBlock) void k_hub_stage(int nhub, const int4 *__restrict__ hubs,
                                                      long long total, const int *__restrict__ col,
                                                      const double *__restrict__ F,
                                                      const double *__restrict__ a_prev,
                                                      const double *__restrict__ a_prev2,
                                                      const void *__restrict__ code_prev,
                                                      const PackCtl *__restrict__ ctl, int rslot,
                                                      double2 *__restrict__ hubxy) {
  const long long q = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (q >= total) return;
  int lo = 0, hi = nhub - 1;  // hubs[h] = {node, row begin, row end, offset}
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (hubs[mid].w <= q) lo = mid; else hi = mid - 1;
  }
  const int4 hb = hubs[lo];
  const int k = hb.y + (int)(q - hb.w);
  const PackCtl pp = ctl[rslot ^ 1];
  const double er = ld_est(pp, code_prev, a_prev, col[k]);
  hubxy[q] = make_double2(recon_fr(ld_f(F, k), er, a_prev2[hb.x]), er);
}

// Mega hubs, parallel exact sums: stage launch. One block per piece of kPiece elements of a
// hub row ({hub, offset in hubxy, length, first edge}): (fr, er) of every edge into hubxy
// (CA:98-99 + kernel 4's flow reconstruction, coalesced), and the piece's approximate sums
// (any order: they only steer the speculation) into psum.
__global__ __launch_bounds__(kBlock) void k_hub_stage_p(
    const int4 *__restrict__ piece, const int4 *__restrict__ hubs, const int *__restrict__ col,
    const double *__restrict__ F, const double *__restrict__ a_prev, const double *__restrict__ a_prev2,
    const void *__restrict__ code_prev, const PackCtl *__restrict__ ctl, int rslot,
    double2 *__restrict__ hubxy, double2 *__restrict__ psum) {
  __shared__ double2 s_w[kBlock / 64];
  const int4 pc = piece[blockIdx.x];
  const int t = threadIdx.x;
  const double own2 = a_prev2[hubs[pc.x].x];
  const PackCtl pp = ctl[rslot ^ 1];
  int cc[kPieceT];
  double fo[kPieceT], er[kPieceT];
#pragma unroll
  for (int i = 0; i < kPieceT; ++i) {
    const int o = t + kBlock * i;
    cc[i] = o < pc.z ? col[pc.w + o] : 0;
    fo[i] = o < pc.z ? ld_f(F, pc.w + o) : 0.0;
  }
#pragma unroll
  for (int i = 0; i < kPieceT; ++i) er[i] = t + kBlock * i < pc.z ? ld_est(pp, code_prev, a_prev, cc[i]) : 0.0;
  double sx = 0.0, sy = 0.0;
#pragma unroll
  for (int i = 0; i < kPieceT; ++i) {
    const int o = t + kBlock * i;
    if (o < pc.z) {
      const double fr = recon_fr(fo[i], er[i], own2);
      hubxy[pc.y + o] = make_double2(fr, er[i]);
      sx += fr;
      sy += er[i];
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    sx += __shfl_down(sx, off);
    sy += __shfl_down(sy, off);
  }
  if ((t & 63) == 0) s_w[t >> 6] = make_double2(sx, sy);
  __syncthreads();
  if (t == 0) {
    double2 r = s_w[0];
    for (int w = 1; w < kBlock / 64; ++w) {
      r.x += s_w[w].x;
      r.y += s_w[w].y;
    }
    psum[blockIdx.x] = r;
  }
}

// (hasb, run) element of the reverse segmented scan over threads: the composition from a
// thread's start up to (and including the head of) the first thread with a boundary.
struct SegRun {
  RunSum r;
  int f;
};
__device__ __forceinline__ SegRun seg_cat(const SegRun &x, const SegRun &y) {  // x earlier
  if (x.f) return x;
  return SegRun{run_cat(x.r, y.r), y.f};
}
__device__ __forceinline__ SegRun shfl_down_seg(const SegRun &a, int off) {
  SegRun b;
  b.r.t0 = __shfl_down(a.r.t0, off);
  b.r.t1 = __shfl_down(a.r.t1, off);
  b.r.mn = __shfl_down(a.r.mn, off);
  b.r.mx = __shfl_down(a.r.mx, off);
  b.r.len = __shfl_down(a.r.len, off);
  b.r.q = __shfl_down(a.r.q, off);
  b.f = __shfl_down(a.f, off);
  return b;
}

// Mega hubs, parallel exact sums: summary launch. One block per piece; for each chain
// (comp 0 = fr -> S, 1 = er -> T) it writes the piece's PieceSum (see the helpers above).
__global__ __launch_bounds__(kBlock) void k_hub_sum(const int4 *__restrict__ piece,
                                                    const int *__restrict__ hub_p0,
                                                    const double2 *__restrict__ psum,
                                                    const double2 *__restrict__ hubxy,
                                                    PieceSum *__restrict__ hsum) {
  __shared__ double2 s_pre;
  __shared__ double s_wd[kBlock / 64];
  __shared__ int s_wi[kBlock / 64];
  __shared__ SegRun s_agg[kBlock / 64];
  __shared__ int s_lastkey[kBlock];
  const int4 pc = piece[blockIdx.x];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t < 64) {  // approximate sum of the hub's earlier pieces
    double ax = 0.0, ay = 0.0;
    for (int q = hub_p0[pc.x] + t; q < (int)blockIdx.x; q += 64) {
      const double2 v = psum[q];
      ax += v.x;
      ay += v.y;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      ax += __shfl_down(ax, off);
      ay += __shfl_down(ay, off);
    }
    if (t == 0) s_pre = make_double2(ax, ay);
  }
  const int nv = max(0, min(kPieceT, pc.z - t * kPieceT));
  double2 v[kPieceT];
#pragma unroll
  for (int i = 0; i < kPieceT; ++i) v[i] = i < nv ? hubxy[pc.y + t * kPieceT + i] : make_double2(0.0, 0.0);
  __syncthreads();
  for (int comp = 0; comp < 2; ++comp) {
    PieceSum *out = hsum + (size_t)blockIdx.x * 2 + comp;
    const double pre = comp ? s_pre.y : s_pre.x;
    double x[kPieceT];
#pragma unroll
    for (int i = 0; i < kPieceT; ++i) x[i] = comp ? v[i].y : v[i].x;
    // approximate prefix: thread sums, block exclusive scan, then in-thread order
    double ls = 0.0;
#pragma unroll
    for (int i = 0; i < kPieceT; ++i)
      if (i < nv) ls += x[i];
    double inc = ls;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const double y = __shfl_up(inc, off);
      if (lane >= off) inc += y;
    }
    if (lane == 63) s_wd[w] = inc;
    __syncthreads();
    double p = pre + (inc - ls);
    for (int u = 0; u < w; ++u) p += s_wd[u];
    int key[kPieceT];
#pragma unroll
    for (int i = 0; i < kPieceT; ++i) {
      p += x[i];
      key[i] = ulp_key(p);
    }
    if (nv) s_lastkey[t] = key[nv - 1];
    __syncthreads();
    const int key_in = t ? s_lastkey[t - 1] : ulp_key(pre);
    // first walk: boundaries, the head run (before the thread's first boundary)
    SegRun g{run_id(), 0};
    int nbl = 0;
    {
      int prev = key_in;
#pragma unroll
      for (int i = 0; i < kPieceT; ++i) {
        if (i < nv) {
          const bool bnd = key[i] == kKeySpecial || prev == kKeySpecial || key[i] != prev;
          if (bnd) {
            g.f = 1;
            ++nbl;
          } else if (!g.f) {
            g.r = run_cat(g.r, run_step(x[i], key[i] >> 1));
          }
          prev = key[i];
        }
      }
    }
    // reverse segmented scan: g = this thread's start up to the first boundary at or after it
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const SegRun y = shfl_down_seg(g, off);
      if (lane + off < 64) g = seg_cat(g, y);
    }
    // boundary counts: exclusive scan
    int ninc = nbl;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(ninc, off);
      if (lane >= off) ninc += y;
    }
    if (lane == 0) s_agg[w] = g;
    if (lane == 63) s_wi[w] = ninc;
    __syncthreads();
    SegRun suf{run_id(), 0};  // later waves, combined
    for (int u = kBlock / 64 - 1; u > w; --u) suf = seg_cat(s_agg[u], suf);
    g = seg_cat(g, suf);
    SegRun gnext = shfl_down_seg(g, 1);  // the next thread's g (exclusive)
    if (lane == 63) gnext = suf;
    int jb = ninc - nbl, nbt = 0;
    for (int u = 0; u < kBlock / 64; ++u) {
      if (u < w) jb += s_wi[u];
      nbt += s_wi[u];
    }
    if (t == 0) {
      out->first_key = ulp_key(pre);
      out->nb = nbt;
      out->head = g.r;  // the piece start up to its first boundary
    }
    if (nbl && nbt <= kMaxBnd) {  // second walk: each boundary and the run after it
      int prev = key_in, j = jb - 1;
      RunSum rr = run_id();
#pragma unroll
      for (int i = 0; i < kPieceT; ++i) {
        if (i < nv) {
          const bool bnd = key[i] == kKeySpecial || prev == kKeySpecial || key[i] != prev;
          if (bnd) {
            if (j >= jb) out->b[j].run = rr;
            ++j;
            out->b[j].x = x[i];
            out->b[j].key = key[i];
            rr = run_id();
          } else if (j >= jb) {
            rr = run_cat(rr, run_step(x[i], key[i] >> 1));
          }
          prev = key[i];
        }
      }
      out->b[j].run = run_cat(rr, gnext.r);
    }
    __syncthreads();  // s_wd / s_wi / s_agg / s_lastkey are reused by the next chain
  }
}

// Mega hubs: the flows of every hub edge (CA:117-118) once the hub blocks have written a_r,
// with many blocks (the hub block's own loop would hold one CU for d / 256 iterations on
// the round's critical path).
__global__ __launch_bounds__(kBlock) void k_hub_flows(int nhub, const int4 *__restrict__ hubs, long long total,
                                                      const double2 *__restrict__ hubxy,
                                                      const double *__restrict__ a_new, double *__restrict__ F) {
  const long long q = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (q >= total) return;
  int lo = 0, hi = nhub - 1;  // hubs[h] = {node, row begin, row end, offset}
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (hubs[mid].w <= q) lo = mid; else hi = mid - 1;
  }
  const int4 hb = hubs[lo];
  const int k = hb.y + (int)(q - hb.w);
  const double a = a_new[hb.x];
  const double2 p2 = hubxy[q];
  st_f(F, k, (p2.x + a) - p2.y, ld_f(F, k));
}

__global__ void k_fill_split(long long cnt, double val, double *__restrict__ p) {
  long long q = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (q < cnt) st_f_full(p, (int)q, val);
}
// split-word flows -> doubles (fu_get_flows of kernels >= 4)
__global__ void k_unsplit(long long cnt, const double *__restrict__ src, double *__restrict__ dst) {
  long long q = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (q < cnt) dst[q] = ld_f(src, (int)q);
}
__global__ void k_fill(long long cnt, double val, double *__restrict__ p) {
  long long q = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (q < cnt) p[q] = val;
}

// ------------------------------------------------------------------------------------
// Variant 5: column split ("split"). Identical arithmetic to variant 4. The neighbour
// estimates a_{r-1}[col e] are gathered by a separate launch in which each group of XCDs
// owns one half of the estimate table (4 MB instead of 8 MB for ER-1M, so it stays in the
// XCD's L2). The gather launch reads a part-major copy of col: the edges of every row with
// col < split first, then the rest, so each part's stream is contiguous. It writes G in the
// same part-major order. The compute launch then reads G coalesced and never gathers.
// Rows must be sorted by neighbour id, so that the part-0 edges of a row are its prefix
// and the row order of the sums is unchanged. Placement (blockIdx % 8 -> XCD) is used
// for locality only, never for correctness.
// ------------------------------------------------------------------------------------
constexpr int kGatherChunk = 2048;  // edges per gather block (8 per thread)

__global__ __launch_bounds__(kBlock) void k_gather_split(const int *__restrict__ col_pm,
                                                         long long e0_count, long long e_total,
                                                         const double *__restrict__ a_prev,
                                                         double *__restrict__ G) {
  const int b = blockIdx.x;
  const int part = (b & 7) >> 2;              // XCD group 0..3 -> part 0, 4..7 -> part 1
  const long long chunk = (long long)(b >> 3) * 4 + (b & 3);
  const long long pb = part ? e0_count : 0, pe = part ? e_total : e0_count;
  const long long base = pb + chunk * kGatherChunk;
  if (base >= pe) return;
  constexpr int kPer = kGatherChunk / kBlock;
  int c[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const long long e = base + threadIdx.x + k * kBlock;
    c[k] = e < pe ? ld_stream(col_pm + e) : -1;
  }
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const long long e = base + threadIdx.x + k * kBlock;
    if (c[k] >= 0) G[e] = a_prev[c[k]];
  }
}

// Kernel 6: gather only part 0 (low half of the estimate table), every block, every XCD.
__global__ __launch_bounds__(kBlock) void k_gather_part0(const int *__restrict__ col_pm,
                                                         long long e0_count,
                                                         const double *__restrict__ a_prev,
                                                         double *__restrict__ G) {
  constexpr int kPer = kGatherChunk / kBlock;
  const long long base = (long long)blockIdx.x * kGatherChunk;
  int c[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const long long e = base + threadIdx.x + k * kBlock;
    c[k] = e < e0_count ? ld_stream(col_pm + e) : -1;
  }
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const long long e = base + threadIdx.x + k * kBlock;
    if (c[k] >= 0) G[e] = a_prev[c[k]];
  }
}

// part-major index of canonical edge k (0-based position inside row t of the tile)
__device__ inline int split_index(int k, int split_t, int p0, int p1) {
  return k < split_t ? p0 + k : p1 + (k - split_t);
}

// GATHER1 (kernel 6): part-1 estimates are gathered here from a_prev (high half of the
// table, 4 MB for ER-1M) instead of being read from G; only part 0 went through G.
template <bool CHECK, bool GATHER1 = false>
__global__ __launch_bounds__(kBlock) void k_round_split(
    const int4 *__restrict__ tiles, const int2 *__restrict__ tiles_g, const int *__restrict__ rowptr,
    const int *__restrict__ rowptr0, long long e0_count, const double *__restrict__ v,
    double *__restrict__ F, const double *__restrict__ G, const double *__restrict__ a_prev2,
    double *__restrict__ a_new, const double *__restrict__ target,
    unsigned long long *__restrict__ err, PackCtl *__restrict__ ctl, int rslot,
    const int *__restrict__ col_pm = nullptr, const double *__restrict__ a_prev = nullptr) {
  if (blockIdx.x == 0 && threadIdx.x == 0) ctl[rslot].width = 0;  // a_r is not packed
  __shared__ double s_x[kTileEdges];  // f_{r-2} on load, fr after phase B (canonical order)
  __shared__ double s_g[kTileEdges];  // a_{r-1}[col] in part-major order: part 0 | part 1
  __shared__ unsigned char s_own[kTileEdges];
  __shared__ int s_rp[kTileNodes + 1];
  __shared__ int s_rp0[kTileNodes + 1];
  __shared__ double s_a[kTileNodes];
  const int t = threadIdx.x;
  const int4 tl = tiles[blockIdx.x];
  const int2 tg = tiles_g[blockIdx.x];  // {rowptr0[node_begin], rowptr0[node_end]}
  unsigned long long eb = 0;

  if (tl.y < 0) {
    // ---------------- heavy node ----------------
    const int i = tl.x;
    const int b = tl.z, e = tl.w;
    const int split_i = tg.y - tg.x;
    const int p0 = tg.x, p1 = (int)(e0_count + (b - tg.x));
    const double own2 = a_prev2[i];
    double S = 0.0, T = 0.0;
    for (int c0 = b; c0 < e; c0 += kTileEdges) {
      const int cn = min(kTileEdges, e - c0);
      for (int q = t; q < cn; q += kBlock) {
        const int gi = split_index(c0 - b + q, split_i, p0, p1);
        const double er = (GATHER1 && c0 - b + q >= split_i) ? a_prev[col_pm[gi]] : G[gi];
        s_x[q] = recon_fr(ld_f(F, c0 + q), er, own2);
        s_g[q] = er;
      }
      __syncthreads();
      if (t < 64) chain_sum(s_x, s_g, cn, S, T);
      __syncthreads();
    }
    if (t == 0) {
      const double a = ((v[i] - S) + T) / (double)(e - b + 1);
      s_a[0] = a;
      st_wt(a_new + i, a);
      if (CHECK) eb = err_bits(a, target[i]);
    }
    __syncthreads();
    const double a = s_a[0];
    for (int k = b + t; k < e; k += kBlock) {
      const int gi = split_index(k - b, split_i, p0, p1);
      const double er = (GATHER1 && k - b >= split_i) ? a_prev[col_pm[gi]] : G[gi];
      const double fo = ld_f(F, k);
      st_f(F, k, (recon_fr(fo, er, own2) + a) - er, fo);
    }
    if (CHECK) block_max_to(eb, err);
    return;
  }

  // ---------------- light tile ----------------
  const int nb = tl.x, nn = tl.y - tl.x;
  const int e0 = tl.z, ne = tl.w - tl.z;
  const int g0b = tg.x, n0 = tg.y - tg.x;   // part-0 edges of the tile: G[g0b, g0b + n0)
  const long long g1b = e0_count + (e0 - g0b);  // part-1 edges: G[g1b, g1b + ne - n0)
  constexpr int kPer = kTileEdges / kBlock;
  double x[kPer], g[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int q = t + k * kBlock;
    x[k] = 0.0;
    g[k] = 0.0;
    if (q < ne) {
      x[k] = ld_f(F, e0 + q);
      if (GATHER1) g[k] = q < n0 ? G[g0b + q] : a_prev[col_pm[g1b + (q - n0)]];
      else g[k] = q < n0 ? G[g0b + q] : G[g1b + (q - n0)];
    }
  }
  const int rp = t <= nn ? rowptr[nb + t] : 0;
  const int rp0 = t <= nn ? rowptr0[nb + t] : 0;
  const int rp_last = (t == 0 && nn == kBlock) ? rowptr[nb + kBlock] : 0;
  const int rp0_last = (t == 0 && nn == kBlock) ? rowptr0[nb + kBlock] : 0;
  const double vv = t < nn ? v[nb + t] : 0.0;
  const double own2 = t < nn ? a_prev2[nb + t] : 0.0;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int q = t + k * kBlock;
    if (q < ne) {
      s_x[q] = x[k];
      s_g[q] = g[k];
    }
  }
  if (t <= nn) {
    s_rp[t] = rp;
    s_rp0[t] = rp0;
  }
  if (t == 0 && nn == kBlock) {
    s_rp[kBlock] = rp_last;
    s_rp0[kBlock] = rp0_last;
  }
  __syncthreads();
  if (t < nn) {
    const int qb = s_rp[t] - e0, qe = s_rp[t + 1] - e0;
    const int split_t = s_rp0[t + 1] - s_rp0[t];
    const int p0 = s_rp0[t] - g0b;                         // LDS index of the row's part 0
    const int p1 = n0 + ((s_rp[t] - s_rp0[t]) - (e0 - g0b));  // LDS index of the row's part 1
    double S = 0.0, T = 0.0;
    for (int q = qb; q < qe; ++q) {
      const double er = s_g[split_index(q - qb, split_t, p0, p1)];
      const double fr = recon_fr(s_x[q], er, own2);
      s_x[q] = fr;
      s_own[q] = (unsigned char)t;
      S = S + fr;
      T = T + er;
    }
    const double a = ((vv - S) + T) / (double)(qe - qb + 1);
    s_a[t] = a;
    st_wt(a_new + nb + t, a);
    if (CHECK) eb = err_bits(a, target[nb + t]);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int q = t + k * kBlock;
    if (q < ne) {
      const int o = s_own[q];
      const int qb = s_rp[o] - e0;
      const int split_t = s_rp0[o + 1] - s_rp0[o];
      const int p0 = s_rp0[o] - g0b;
      const int p1 = n0 + ((s_rp[o] - s_rp0[o]) - (e0 - g0b));
      const double er = s_g[split_index(q - qb, split_t, p0, p1)];
      st_f(F, e0 + q, (s_x[q] + s_a[o]) - er, x[k]);
    }
  }
  if (CHECK) block_max_to(eb, err);
}

// round 0 for the push layout: message i->j = (a_i, a_i) stored at inbox[rev[e]]
__global__ __launch_bounds__(kBlock) void k_round0_push(int n, const int *__restrict__ rowptr,
                                                        const int *__restrict__ rev,
                                                        const double *__restrict__ v,
                                                        double2 *__restrict__ in_new,
                                                        double *__restrict__ a) {
  int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  int b = rowptr[i], e = rowptr[i + 1];
  double ai = ((v[i] - 0.0) + 0.0) / (double)(e - b + 1);
  a[i] = ai;
  double fv = (0.0 + ai) - 0.0;
  for (int k = b; k < e; ++k) in_new[rev[k]] = make_double2(fv, ai);
}

// flows of the push layout in CSR order: f[e] = inbox[rev[e]].x
__global__ void k_push_flows(long long E, const int *__restrict__ rev,
                             const double2 *__restrict__ in, double *__restrict__ f) {
  long long e = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (e < E) f[e] = in[rev[e]].x;
}

__global__ __launch_bounds__(kBlock) void k_max_err(int n, const double *__restrict__ a,
                                                    const double *__restrict__ target,
                                                    unsigned long long *__restrict__ err) {
  unsigned long long eb = 0;
  for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    unsigned long long x = err_bits(a[i], target[i]);
    eb = x > eb ? x : eb;
  }
  block_max_to(eb, err);
}

// ------------------------------------------------------------------------------------
// Tick replay: one thread per task (= one node's events in one tick, in program order).
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_replay_tick(
    long long task_begin, int ntasks, const int *__restrict__ tasks,
    const long long *__restrict__ rowptr, const int *__restrict__ events,
    const int *__restrict__ out_ids, const double *__restrict__ v, double *__restrict__ flow,
    double *__restrict__ est, double *__restrict__ last, double2 *__restrict__ msg) {
  int q = blockIdx.x * kBlock + threadIdx.x;
  if (q >= ntasks) return;
  const int *tk = tasks + 3 * (task_begin + q);
  const int node = tk[0], evb = tk[1], eve = tk[2];
  double *fl = flow + rowptr[node];
  double *es = est + rowptr[node];
  const double val = v[node];
  for (int p = evb; p < eve; ++p) {
    const int4 ev = *reinterpret_cast<const int4 *>(events + 4 * (long long)p);
    if (ev.x == FU_EV_RECV) {  // CA:98-99 / PW:98-99
      const double2 m = msg[ev.z];
      es[ev.y] = m.y;
      fl[ev.y] = -m.x;
    } else if (ev.x == FU_EV_FIRE_CA) {  // CA:105-125
      const int k = ev.y;
      double S = 0.0, T = 0.0;
      for (int j = 0; j < k; ++j) S = S + fl[j];
      const double estimate = val - S;
      for (int j = 0; j < k; ++j) T = T + es[j];
      const double avg = (estimate + T) / (double)(k + 1);
      last[node] = avg;
      for (int j = 0; j < k; ++j) {
        const double nf = (fl[j] + avg) - es[j];
        fl[j] = nf;
        es[j] = avg;
        msg[out_ids[ev.z + j]] = make_double2(nf, avg);
      }
    } else {  // FIRE_PW, PW:102-117
      const int s = ev.y, k = ev.z;
      double S = 0.0;
      for (int j = 0; j < k; ++j) S = S + fl[j];
      const double estimate = val - S;
      const double avg = (es[s] + estimate) / 2.0;
      last[node] = avg;
      const double nf = (fl[s] + avg) - es[s];
      fl[s] = nf;
      es[s] = avg;
      msg[ev.w] = make_double2(nf, avg);
    }
  }
}

// ------------------------------------------------------------------------------------
// Persistent replay: one launch for all ticks, dataflow order. Each thread owns nodes
// {gtid, gtid + G, ...} and walks each node's events in program order (events regrouped
// per node on the host). A RECV waits until its message exists. Messages have unique slots
// (no recycling), so a slot is written once: it starts as a signalling-NaN sentinel that
// arithmetic never produces, and each 8-byte half is its own readiness tag (data-tagged
// granule: agent-scope relaxed sc1 store, sc1 load; MI355X_MICROARCH.md "hand-off"). Per-node
// order + produce-before-consume is exactly the dependence structure of the tick batches,
// so the results are the same bits. A thread never blocks on one node: it polls once and
// moves on. The globally earliest pending event is always ready, so a fully resident grid
// always makes progress. The grid is sized below the occupancy bound.
// ------------------------------------------------------------------------------------
constexpr unsigned long long kMsgSentinel = 0x7FF7A5A5A5A5A5A5ull;

__device__ inline unsigned long long ld_tag(const unsigned long long *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st_tag(unsigned long long *p, double v) {
  __hip_atomic_store(p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kBlock) void k_replay_persist(
    int n, int tick_end, const long long *__restrict__ node_off, const int4 *__restrict__ node_ev,
    const int *__restrict__ node_tick, const int *__restrict__ out_uid,
    const long long *__restrict__ rowptr, const double *__restrict__ v, double *__restrict__ flow,
    double *__restrict__ est, double *__restrict__ last, unsigned long long *__restrict__ pay,
    long long *__restrict__ cursor, int *__restrict__ scur, int n_snap,
    const int *__restrict__ snap_ticks, double *__restrict__ snaps, int *__restrict__ status,
    long long max_iters) {
  const int G = gridDim.x * kBlock;
  const int g = blockIdx.x * kBlock + threadIdx.x;
  long long it = 0;
  bool left = true;
  while (left) {
    left = false;
    bool progressed = false;
    for (int node = g; node < n; node += G) {
      long long p = cursor[node];
      const long long pe = node_off[node + 1];
      int sc = scur[node];
      double *fl = flow + rowptr[node];
      double *es = est + rowptr[node];
      const double val = v[node];
      double lst = last[node];
      while (p < pe) {
        const int tk = node_tick[p];
        if (tk >= tick_end) break;
        while (sc < n_snap && snap_ticks[sc] < tk) snaps[(long long)sc++ * n + node] = lst;
        const int4 ev = node_ev[p];
        if (ev.x == FU_EV_RECV) {
          const unsigned long long fx = ld_tag(pay + 2 * (long long)ev.z);
          const unsigned long long fy = ld_tag(pay + 2 * (long long)ev.z + 1);
          if (fx == kMsgSentinel || fy == kMsgSentinel) break;  // not sent yet
          es[ev.y] = __longlong_as_double((long long)fy);
          fl[ev.y] = -__longlong_as_double((long long)fx);
        } else if (ev.x == FU_EV_FIRE_CA) {
          const int k = ev.y;
          double S = 0.0, T = 0.0;
          for (int j = 0; j < k; ++j) S = S + fl[j];
          const double estimate = val - S;
          for (int j = 0; j < k; ++j) T = T + es[j];
          const double avg = (estimate + T) / (double)(k + 1);
          lst = avg;
          for (int j = 0; j < k; ++j) {
            const double nf = (fl[j] + avg) - es[j];
            fl[j] = nf;
            es[j] = avg;
            const long long m = out_uid[ev.z + j];
            st_tag(pay + 2 * m, nf);
            st_tag(pay + 2 * m + 1, avg);
          }
        } else {
          const int sl = ev.y, k = ev.z;
          double S = 0.0;
          for (int j = 0; j < k; ++j) S = S + fl[j];
          const double estimate = val - S;
          const double avg = (es[sl] + estimate) / 2.0;
          lst = avg;
          const double nf = (fl[sl] + avg) - es[sl];
          fl[sl] = nf;
          es[sl] = avg;
          st_tag(pay + 2 * (long long)ev.w, nf);
          st_tag(pay + 2 * (long long)ev.w + 1, avg);
        }
        ++p;
        progressed = true;
      }
      const bool done = p == pe || node_tick[p] >= tick_end;
      if (done)
        while (sc < n_snap && snap_ticks[sc] < tick_end) snaps[(long long)sc++ * n + node] = lst;
      cursor[node] = p;
      scur[node] = sc;
      last[node] = lst;
      if (!done) left = true;
    }
    if (left && !progressed) __builtin_amdgcn_s_sleep(2);
    if (++it > max_iters) {  // bounded spin: a bug must end the kernel, not hang the GPU
      atomicExch(status, 1);
      break;
    }
  }
}

template <typename T>
int dmalloc(T **p, size_t count) {
  if (count == 0) count = 1;
  hipError_t e = hipMalloc((void **)p, sizeof(T) * count);
  if (e != hipSuccess) {
    *p = nullptr;
    return fail(FU_ERR_ALLOC, std::string("hipMalloc(") + std::to_string(sizeof(T) * count) + "): " + hipGetErrorString(e));
  }
  return FU_OK;
}

}  // namespace

// ======================================================================================
// handle
// ======================================================================================
struct fu_handle {
  int device = 0;
  // layout 1 (fu_create_from_graph_ex): device node p = caller node old_of_new[p]; the
  // caller's row pointer maps flows back (rows moved as blocks)
  std::vector<int32_t> h_new_of_old;
  std::vector<int64_t> h_orig_rowptr;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;  // autotune timing
  hipEvent_t ev2 = nullptr, ev3 = nullptr;  // fu_run_collectall_timed
  hipEvent_t marks[64] = {};                // fu_mark slots (created on first use)
  int32_t n = 0;
  int64_t E = 0;
  int32_t na = 0;  // estimate slots: n local + ghost estimates (multi-GPU)
  int32_t max_deg = 0;
  int *rowptr = nullptr, *col = nullptr, *rev = nullptr;
  double *v = nullptr;
  double *f[2] = {nullptr, nullptr};
  double *a[3] = {nullptr, nullptr, nullptr};  // a[2]: third estimate buffer (kernel 4)
  double2 *inbox[2] = {nullptr, nullptr};
  double *target = nullptr;
  unsigned long long *err = nullptr;
  int errcap = 0;
  double *ftmp = nullptr;
  int cur = 0;
  int64_t rounds = 0;
  int kernel = 4;
  int hub_threshold = 64;
  int nt = 0;  // non-temporal loads/stores for streamed arrays (kernel 4)
  bool autotune = true;  // kernel "auto": time kernels 4 (+nt), 6, 5 on real rounds, keep the best
  bool tuned = false;
  float tune_ms[12] = {};  // per candidate (autotune_kernel order)
  int tune_out[12] = {};   // passes in which the candidate was > 1.3x the best (2: dropped)
  int n_tunes = 0;        // autotune passes so far (re-run when the packing width changes)
  int tuned_width = 0;    // packing width the last pass ran under
  int tune_cache[4] = {-1, -1, -1, -1};  // winner per packing width (0, 8, 16, 32), kept across fu_reset
  int *h_pw = nullptr;    // pinned copy of the plan's width, refreshed after each plan
  hipEvent_t ev_pw = nullptr;
  bool pw_pending = false;
  int diag = 0;  // timing-only ablations of kernel 4 (wrong results; tools/ only)
  std::vector<int64_t> h_rowptr;
  std::vector<int32_t> h_col;  // host copy (column-split preparation)
  // kernel 5 (column split)
  int *colpm = nullptr, *rowptr0 = nullptr;
  double *G = nullptr;
  int4 *tiles_s = nullptr;
  int2 *tiles_g = nullptr;
  int ntiles_s = 0;
  int64_t e0_count = 0;
  int4 *tiles = nullptr;  // 2048-edge tiles (kernels 2, 3)
  int ntiles = 0;
  // kernel 4 tiles per geometry (0 = 2048x256, 1 = 1024x128, 2 = 1024x256, 3 = 512x64 edges x
  // nodes); all four are built up front so autotuning can switch geometry between rounds
  int4 *tiles_geo[4] = {nullptr, nullptr, nullptr, nullptr};
  int ntiles_geo[4] = {0, 0, 0, 0};
  int nheavy_geo[4] = {0, 0, 0, 0};  // leading non-light tiles (hubs, heavy rows, bins)
  int fork_heavy = 1;                 // option "fork_heavy": heavy tiles on stream2, concurrently
  hipStream_t stream2 = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  int geo = 0;
  // kernel 7 (wave tiles): per wave geometry (0 = 256 edges x 32 nodes, 1 = 512 x 64) the
  // light wave tiles and the heavy rows (kernel 4 heavy-path tiles) of that geometry
  int4 *wtiles[2] = {nullptr, nullptr};
  int nwtiles[2] = {0, 0};
  int4 *wheavy[2] = {nullptr, nullptr};
  int nwheavy[2] = {0, 0};
  int wgeo = 1;
  int *perm = nullptr;  // degree-sorted heavy rows (kernel 4 bins)
  // kernel 4 mega hubs (degree > mega_hub): first tiles of every geometry ({i, -3, b, e})
  int mega_hub = 8192;  // degree above which a row is a mega hub (option "mega_hub")
  int wave_heavy = 1;   // kernel 4: heavy rows one per wave (option "wave_heavy")
  std::vector<int32_t> h_hrows;
  int *hrows = nullptr;  // heavy rows of the wave-per-row tiles, longest first
  int n_hub = 0;
  int64_t hub_total = 0;
  // parallel exact hub sums (option "hub_scan", default off: on converged R-MAT rounds the
  // flow sums wander across binades, ~10% of their steps are boundaries, and the serial
  // pass loses to the one-wave chain): pieces of kPiece edges
  int hub_scan = 0;
  int n_piece = 0;
  int4 *hub_piece = nullptr;  // {hub, offset in hubxy, length, first edge}
  int *hub_p0 = nullptr;      // first piece of each hub (n_hub + 1)
  double2 *psum = nullptr;    // approximate (fr, er) sums per piece
  PieceSum *hsum = nullptr;   // run summaries per piece and chain
  unsigned long long *hub_redo = nullptr;  // pieces the serial pass redid element by element
  int4 *hub_rows = nullptr;  // {node, row begin, row end, offset in hubxy}
  int *hub_off = nullptr;    // per mega tile: offset in hubxy
  double2 *hubxy = nullptr;  // (fr, er) per hub edge, staged each round
  int bins = 0;         // kernel 4 (geometry 0): degree bins for rows above hub_threshold
  // kernel 4 packed estimate table (see PackCtl): code[r & 1] = codes of a_r
  unsigned char *code[2] = {nullptr, nullptr};
  PackCtl *pctl = nullptr;  // [0], [1]: per code table; [2]: current encoding plan
  int *psample = nullptr;   // gather targets sampled for the plan
  int n_psample = 0;
  int pack = 1;             // 0 = off
  int pack_every = 16;      // rounds between encoding plans
  int tile_edges = 2048;  // 2048 (256 nodes), 1024 (128 or 256 nodes), 512 (64 nodes)
  int tile_nodes = 0;
  bool has_target = false;
  // kernel 8 (LDS-staged slices): light tiles of kStageTE x kStageTN in edge groups, heavy
  // rows as kernel 4 heavy tiles, and one slice layout per table element width
  struct StageLayout {
    int P = 0, Q = 0;              // slices, blocks per slice
    int *aoff = nullptr;           // per stage block: first entry in aitem
    int2 *aitem = nullptr;         // stage items {first element, count}, grouped by block
    unsigned short *colS = nullptr;  // per staged element: column offset within its slice
    unsigned *sidx = nullptr;      // per tile edge (slice order): G index in group << 16 | position
    // compact form (when every tile's edges fall into <= 64 slice runs): per edge u16 =
    // position | run << 10, and per tile the run offsets D (G index = gbase + m + D[run])
    unsigned short *sidx16 = nullptr;
    int *dtab = nullptr;           // kStageRuns per light tile
    int *gbase = nullptr;          // per light tile: its group's first staged element
  };
  StageLayout st[4];            // element bytes 1, 2, 4, 8
  bool st_ready = false;
  int st_ngroups = 0;
  int4 *st_tiles = nullptr;     // light tiles
  int *st_gbase = nullptr;      // per light tile: first edge of its group
  int st_ntiles = 0;
  int4 *st_heavy = nullptr;     // rows above the tile limit ({i, -1, b, e})
  int st_nheavy = 0;
  void *stG = nullptr;          // staged estimates, 8 B per light edge
  int seen_width = 0;           // packing width the host last saw (layout choice)
  int st_force = -1;            // tests: force layout 0..3 (element bytes 1, 2, 4, 8)
  int st_compact = 1;           // option "stage_compact": kernel 8 reads the u16 sidx
  std::vector<int4> h_light;    // host copies (layout construction)
  std::vector<int32_t> h_gstart;
  int n_cu = 256;               // compute units (kernel 9 grid)
  int pipe_bpc = 4;             // kernel 9/10: persistent blocks per CU (4 fit at 1024x128 tiles)
  // multi-GPU (fu_dist.hip)
  void *dist = nullptr;
};

extern "C" int fu__dist_round_hook(fu_handle *h, int phase);
extern "C" void fu__dist_free(fu_handle *h);

namespace {


int build_tiles_geom(fu_handle *h, int te, int tn, int4 **dst, int *count,
                     std::vector<int4> *host_out = nullptr, bool mega = false, int *nheavy = nullptr) {
  std::vector<int4> heavy, light, hubs;
  const int32_t n = h->n;
  int32_t i = 0;
  while (i < n) {
    int64_t d = h->h_rowptr[i + 1] - h->h_rowptr[i];
    if (mega && d > h->mega_hub) {
      hubs.push_back(make_int4(i, -3, (int)h->h_rowptr[i], (int)h->h_rowptr[i + 1]));
      ++i;
      continue;
    }
    if (d > h->hub_threshold || d > te) {
      heavy.push_back(make_int4(i, -1, (int)h->h_rowptr[i], (int)h->h_rowptr[i + 1]));
      ++i;
      continue;
    }
    int32_t b = i;
    int64_t eb = h->h_rowptr[b];
    while (i < n && i - b < tn) {
      int64_t di = h->h_rowptr[i + 1] - h->h_rowptr[i];
      if (di > h->hub_threshold || di > te) break;
      if (h->h_rowptr[i + 1] - eb > te) break;
      ++i;
    }
    light.push_back(make_int4(b, i, (int)h->h_rowptr[b], (int)h->h_rowptr[i]));
  }
  // mega hubs, then heavy tiles first so their long sequential chains start early; heavy
  // rows of up to mega_hub go four to a block (one per wave) when wave_heavy is on, longest
  // first (the row list hrows is shared by every geometry)
  std::vector<int4> all(hubs);
  if (mega && h->wave_heavy && !heavy.empty()) {
    std::vector<int32_t> rows;
    for (const int4 &hv : heavy) rows.push_back(hv.x);
    std::stable_sort(rows.begin(), rows.end(), [&](int32_t x, int32_t y) {
      return h->h_rowptr[x + 1] - h->h_rowptr[x] > h->h_rowptr[y + 1] - h->h_rowptr[y];
    });
    const size_t base = h->h_hrows.size();  // each geometry appends its own list
    h->h_hrows.insert(h->h_hrows.end(), rows.begin(), rows.end());
    for (size_t q = 0; q < rows.size(); q += 4)
      all.push_back(make_int4((int)(base + q), -4, (int)std::min<size_t>(4, rows.size() - q), 0));
  } else {
    all.insert(all.end(), heavy.begin(), heavy.end());
  }
  if (nheavy) *nheavy = (int)all.size();
  all.insert(all.end(), light.begin(), light.end());
  if (host_out) *host_out = all;
  if (*dst) hipFree(*dst);
  *dst = nullptr;
  *count = (int)all.size();
  if (int rc = dmalloc(dst, all.size())) return rc;
  HIP_TRY(hipMemcpy(*dst, all.data(), sizeof(int4) * all.size(), hipMemcpyHostToDevice));
  return FU_OK;
}

// Kernel 4 tiles with degree bins: rows of degree > hub_threshold sorted by degree
// (descending, ties by id) and grouped R per block (R = TE / C, C = the power of two >= the
// bin's first degree, capped at TE); then light tiles of contiguous low-degree rows.
int build_tiles_binned(fu_handle *h) {
  const int32_t n = h->n;
  std::vector<int32_t> heavy;
  for (int32_t i = 0; i < n; ++i)
    if (h->h_rowptr[i + 1] - h->h_rowptr[i] > h->hub_threshold) heavy.push_back(i);
  auto deg = [&](int32_t i) { return h->h_rowptr[i + 1] - h->h_rowptr[i]; };
  std::stable_sort(heavy.begin(), heavy.end(), [&](int32_t x, int32_t y) { return deg(x) > deg(y); });
  std::vector<int4> all;
  size_t q = 0;
  while (q < heavy.size()) {
    const int64_t d = deg(heavy[q]);
    int C = 1;
    while (C < d && C < kTileEdges) C <<= 1;
    const int R = std::max(1, std::min(kBlock, kTileEdges / C));
    const int r = (int)std::min<size_t>(R, heavy.size() - q);
    all.push_back(make_int4((int)q, -2, r, kTileEdges / R));
    q += r;
  }
  // light tiles over the remaining rows (heavy rows are skipped inside build_tiles_geom)
  std::vector<int4> light;
  int32_t i = 0;
  while (i < n) {
    if (deg(i) > h->hub_threshold) { ++i; continue; }
    int32_t b = i;
    int64_t eb = h->h_rowptr[b];
    while (i < n && i - b < kTileNodes && deg(i) <= h->hub_threshold && h->h_rowptr[i + 1] - eb <= kTileEdges) ++i;
    light.push_back(make_int4(b, i, (int)h->h_rowptr[b], (int)h->h_rowptr[i]));
  }
  all.insert(all.end(), light.begin(), light.end());
  if (h->tiles_geo[0]) hipFree(h->tiles_geo[0]);
  if (h->perm) hipFree(h->perm);
  h->tiles_geo[0] = nullptr;
  h->perm = nullptr;
  h->ntiles_geo[0] = (int)all.size();
  h->nheavy_geo[0] = (int)(all.size() - light.size());
  if (int rc = dmalloc(&h->tiles_geo[0], all.size())) return rc;
  if (int rc = dmalloc(&h->perm, std::max<size_t>(1, heavy.size()))) return rc;
  HIP_TRY(hipMemcpy(h->tiles_geo[0], all.data(), sizeof(int4) * all.size(), hipMemcpyHostToDevice));
  if (!heavy.empty()) HIP_TRY(hipMemcpy(h->perm, heavy.data(), sizeof(int32_t) * heavy.size(), hipMemcpyHostToDevice));
  return FU_OK;
}

constexpr int kGeoEdges[4] = {2048, 1024, 1024, 512};
constexpr int kGeoNodes[4] = {256, 128, 256, 64};

constexpr int kWaveEdges[2] = {256, 512};
constexpr int kWaveNodes[2] = {32, 64};

// Kernel 7 tiles: light rows (degree <= min(hub_threshold, TE)) in contiguous wave tiles of
// <= TN nodes / <= TE edges; the other rows as kernel 4 heavy-path tiles {i, -1, b, e}.
int build_wave_tiles(fu_handle *h, int wg) {
  const int te = kWaveEdges[wg], tn = kWaveNodes[wg];
  const int64_t lim = std::min<int64_t>(h->hub_threshold, te);
  std::vector<int4> light, heavy;
  const int32_t n = h->n;
  int32_t i = 0;
  while (i < n) {
    const int64_t d = h->h_rowptr[i + 1] - h->h_rowptr[i];
    if (d > lim) {
      heavy.push_back(make_int4(i, -1, (int)h->h_rowptr[i], (int)h->h_rowptr[i + 1]));
      ++i;
      continue;
    }
    const int32_t b = i;
    const int64_t eb = h->h_rowptr[b];
    while (i < n && i - b < tn) {
      const int64_t di = h->h_rowptr[i + 1] - h->h_rowptr[i];
      if (di > lim || h->h_rowptr[i + 1] - eb > te) break;
      ++i;
    }
    light.push_back(make_int4(b, i, (int)h->h_rowptr[b], (int)h->h_rowptr[i]));
  }
  for (int4 **p : {&h->wtiles[wg], &h->wheavy[wg]}) {
    if (*p) hipFree(*p);
    *p = nullptr;
  }
  h->nwtiles[wg] = (int)light.size();
  h->nwheavy[wg] = (int)heavy.size();
  if (int rc = dmalloc(&h->wtiles[wg], std::max<size_t>(1, light.size()))) return rc;
  if (int rc = dmalloc(&h->wheavy[wg], std::max<size_t>(1, heavy.size()))) return rc;
  if (!light.empty()) HIP_TRY(hipMemcpy(h->wtiles[wg], light.data(), sizeof(int4) * light.size(), hipMemcpyHostToDevice));
  if (!heavy.empty()) HIP_TRY(hipMemcpy(h->wheavy[wg], heavy.data(), sizeof(int4) * heavy.size(), hipMemcpyHostToDevice));
  return FU_OK;
}

// Mega-hub side arrays (same rows, same order as the -3 tiles of build_tiles_geom).
int build_hubs(fu_handle *h) {
  for (void *p : {(void *)h->hub_rows, (void *)h->hub_off, (void *)h->hubxy, (void *)h->hub_piece,
                  (void *)h->hub_p0, (void *)h->psum, (void *)h->hsum})
    if (p) hipFree(p);
  h->hub_rows = nullptr;
  h->hub_off = nullptr;
  h->hubxy = nullptr;
  h->hub_piece = nullptr;
  h->hub_p0 = nullptr;
  h->psum = nullptr;
  h->hsum = nullptr;
  h->n_piece = 0;
  if (!h->hub_redo) {
    if (int rc = dmalloc(&h->hub_redo, 1)) return rc;
    HIP_TRY(hipMemset(h->hub_redo, 0, sizeof(unsigned long long)));
  }
  std::vector<int4> rows;
  std::vector<int32_t> off;
  int64_t tot = 0;
  for (int32_t i = 0; i < h->n; ++i) {
    const int64_t d = h->h_rowptr[i + 1] - h->h_rowptr[i];
    if (d > h->mega_hub) {
      rows.push_back(make_int4(i, (int)h->h_rowptr[i], (int)h->h_rowptr[i + 1], (int)tot));
      off.push_back((int32_t)tot);
      tot += d;
    }
  }
  h->n_hub = (int)rows.size();
  h->hub_total = tot;
  if (rows.empty()) return FU_OK;
  if (int rc = dmalloc(&h->hub_rows, rows.size())) return rc;
  if (int rc = dmalloc(&h->hub_off, off.size())) return rc;
  if (int rc = dmalloc(&h->hubxy, (size_t)tot)) return rc;
  HIP_TRY(hipMemcpy(h->hub_rows, rows.data(), sizeof(int4) * rows.size(), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(h->hub_off, off.data(), sizeof(int32_t) * off.size(), hipMemcpyHostToDevice));
  std::vector<int4> pcs;
  std::vector<int32_t> p0;
  for (size_t q = 0; q < rows.size(); ++q) {
    p0.push_back((int32_t)pcs.size());
    const int d = rows[q].z - rows[q].y;
    for (int k = 0; k < d; k += kPiece)
      pcs.push_back(make_int4((int)q, rows[q].w + k, std::min(kPiece, d - k), rows[q].y + k));
  }
  p0.push_back((int32_t)pcs.size());
  h->n_piece = (int)pcs.size();
  if (int rc = dmalloc(&h->hub_piece, pcs.size())) return rc;
  if (int rc = dmalloc(&h->hub_p0, p0.size())) return rc;
  if (int rc = dmalloc(&h->psum, pcs.size())) return rc;
  if (int rc = dmalloc(&h->hsum, 2 * pcs.size())) return rc;
  HIP_TRY(hipMemcpy(h->hub_piece, pcs.data(), sizeof(int4) * pcs.size(), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(h->hub_p0, p0.data(), sizeof(int32_t) * p0.size(), hipMemcpyHostToDevice));
  return FU_OK;
}

int build_tiles(fu_handle *h) {
  h->h_hrows.clear();
  if (int rc = build_tiles_geom(h, kTileEdges, kTileNodes, &h->tiles, &h->ntiles)) return rc;
  for (int wg = 0; wg < 2; ++wg)
    if (int rc = build_wave_tiles(h, wg)) return rc;
  for (int g = 0; g < 4; ++g) {
    if (g == 0 && h->bins) {
      if (int rc = build_tiles_binned(h)) return rc;
      continue;
    }
    if (int rc = build_tiles_geom(h, kGeoEdges[g], kGeoNodes[g], &h->tiles_geo[g], &h->ntiles_geo[g], nullptr, true,
                                  &h->nheavy_geo[g]))
      return rc;
  }
  if (h->hrows) hipFree(h->hrows);
  h->hrows = nullptr;
  if (int rc = dmalloc(&h->hrows, std::max<size_t>(1, h->h_hrows.size()))) return rc;
  if (!h->h_hrows.empty())
    HIP_TRY(hipMemcpy(h->hrows, h->h_hrows.data(), sizeof(int32_t) * h->h_hrows.size(), hipMemcpyHostToDevice));
  return build_hubs(h);
}

// Current estimate / flow buffers (kernel 4 rotates A[r % 3] and F[r & 1]).
inline double *cur_a(fu_handle *h) {
  if (h->kernel >= 4) return h->a[(int)((h->rounds + 2) % 3)];
  return h->a[h->cur];
}
inline double *cur_f(fu_handle *h) {
  if (h->kernel >= 4) return h->f[(int)((h->rounds + 1) & 1)];
  return h->f[h->cur];
}

// Kernel 5 preparation: split node id (edge-balanced), part-major col, rowptr0, tiles.
int ensure_split(fu_handle *h) {
  if (h->G) return FU_OK;
  const int32_t n = h->n;
  const int64_t E = h->E;
  for (int32_t i = 0; i < n; ++i)
    for (int64_t k = h->h_rowptr[i] + 1; k < h->h_rowptr[i + 1]; ++k)
      if (h->h_col[k - 1] >= h->h_col[k])
        return fail(FU_ERR_GRAPH, "kernel 5 (column split) needs rows sorted by neighbour id");
  // split id: smallest s with rowptr[s] >= E/2 (symmetric graph: in-degree == degree)
  int32_t split = (int32_t)(std::lower_bound(h->h_rowptr.begin(), h->h_rowptr.end(), E / 2) - h->h_rowptr.begin());
  if (split > n) split = n;
  std::vector<int32_t> rp0(n + 1, 0);
  for (int32_t i = 0; i < n; ++i) {
    auto b = h->h_col.begin() + h->h_rowptr[i], e = h->h_col.begin() + h->h_rowptr[i + 1];
    rp0[i + 1] = rp0[i] + (int32_t)(std::lower_bound(b, e, split) - b);
  }
  const int64_t E0 = rp0[n];
  std::vector<int32_t> pm(E > 0 ? E : 1);
  for (int32_t i = 0; i < n; ++i) {
    const int64_t b = h->h_rowptr[i], s0 = rp0[i + 1] - rp0[i];
    for (int64_t k = 0; k < s0; ++k) pm[rp0[i] + k] = h->h_col[b + k];
    const int64_t d = h->h_rowptr[i + 1] - b, p1 = E0 + (b - rp0[i]);
    for (int64_t k = s0; k < d; ++k) pm[p1 + (k - s0)] = h->h_col[b + k];
  }
  std::vector<int4> tv;
  if (int rc = build_tiles_geom(h, kTileEdges, kTileNodes, &h->tiles_s, &h->ntiles_s, &tv)) return rc;
  std::vector<int2> tg(tv.size());
  for (size_t q = 0; q < tv.size(); ++q) {
    const int4 t = tv[q];
    tg[q] = t.y < 0 ? make_int2(rp0[t.x], rp0[t.x + 1]) : make_int2(rp0[t.x], rp0[t.y]);
  }
  if (int rc = dmalloc(&h->colpm, (size_t)E)) return rc;
  if (int rc = dmalloc(&h->rowptr0, (size_t)n + 1)) return rc;
  if (int rc = dmalloc(&h->tiles_g, tg.size())) return rc;
  if (int rc = dmalloc(&h->G, (size_t)E)) return rc;
  if (E) HIP_TRY(hipMemcpy(h->colpm, pm.data(), sizeof(int32_t) * E, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(h->rowptr0, rp0.data(), sizeof(int32_t) * (n + 1), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(h->tiles_g, tg.data(), sizeof(int2) * tg.size(), hipMemcpyHostToDevice));
  h->e0_count = E0;
  return FU_OK;
}

// Kernel 8 preparation: light tiles, edge groups and the four slice layouts.
constexpr int kStageMaxP = 512;      // slices per layout (more: layout not built)
constexpr int kStageGroupEdges = 60000;  // G index within a group is u16 (room for padding)

// Light tiles (kStageTE x kStageTN), their edge groups and the heavy rows (kernels 8-10).
int ensure_light(fu_handle *h) {
  if (h->st_tiles) return FU_OK;
  const int32_t n = h->n;
  const auto &rp = h->h_rowptr;
  const int64_t lim = std::min<int64_t>(h->hub_threshold, kStageTE);
  std::vector<int4> light, heavy;
  std::vector<int32_t> gstart;  // per group: first light tile
  int64_t gedges = 0;
  bool prev_light = false;
  for (int32_t i = 0; i < n;) {
    const int64_t d = rp[i + 1] - rp[i];
    if (d > lim) {
      heavy.push_back(make_int4(i, -1, (int)rp[i], (int)rp[i + 1]));
      ++i;
      prev_light = false;
      continue;
    }
    const int32_t b = i;
    while (i < n && i - b < kStageTN) {
      const int64_t di = rp[i + 1] - rp[i];
      if (di > lim || rp[i + 1] - rp[b] > kStageTE) break;
      ++i;
    }
    const int64_t te = rp[i] - rp[b];
    if (!prev_light || gedges + te > kStageGroupEdges) {
      gstart.push_back((int32_t)light.size());
      gedges = 0;
    }
    light.push_back(make_int4(b, i, (int)rp[b], (int)rp[i]));
    gedges += te;
    prev_light = true;
  }
  const int ng = (int)gstart.size();
  gstart.push_back((int32_t)light.size());
  std::vector<int32_t> gbase(light.size());
  for (int g = 0; g < ng; ++g)
    for (int t = gstart[g]; t < gstart[g + 1]; ++t) gbase[t] = light[gstart[g]].z;
  auto up = [&](auto **dst, const auto *src, size_t cnt) -> int {
    if (int rc = dmalloc(dst, std::max<size_t>(1, cnt))) return rc;
    if (cnt) HIP_TRY(hipMemcpy(*dst, src, sizeof(**dst) * cnt, hipMemcpyHostToDevice));
    return FU_OK;
  };
  h->h_light = light;
  h->h_gstart = gstart;
  if (int rc = up(&h->st_tiles, light.data(), light.size())) return rc;
  if (int rc = up(&h->st_gbase, gbase.data(), gbase.size())) return rc;
  if (int rc = up(&h->st_heavy, heavy.data(), heavy.size())) return rc;
  h->st_ntiles = (int)light.size();
  h->st_nheavy = (int)heavy.size();
  h->st_ngroups = ng;
  return FU_OK;
}

// Kernel 8 / 10: the staged-estimate buffer and the four slice layouts.
int ensure_stage(fu_handle *h) {
  if (h->st_ready) return FU_OK;
  if (int rc = ensure_light(h)) return rc;
  const int32_t n = h->n;
  const int ng = h->st_ngroups;
  const std::vector<int4> &light = h->h_light;
  const std::vector<int32_t> &gstart = h->h_gstart;
  auto up = [&](auto **dst, const auto *src, size_t cnt) -> int {
    if (int rc = dmalloc(dst, std::max<size_t>(1, cnt))) return rc;
    if (cnt) HIP_TRY(hipMemcpy(*dst, src, sizeof(**dst) * cnt, hipMemcpyHostToDevice));
    return FU_OK;
  };
  // Staged index space per layout: group g's region holds its (slice, tile, position)
  // ordered elements, each (group, slice) segment padded to a multiple of kStagePad so the
  // stage launch moves 8 consecutive elements per lane with 16-byte column loads; a pad
  // element's column offset is 0 and its staged word is never read.
  int64_t gmax = 1;
  for (int li = 0; li < 4; ++li) {
    const int64_t SN = kStageLds >> li;
    const int64_t P = (n + SN - 1) / SN;
    auto &L = h->st[li];
    if (P > kStageMaxP) continue;
    std::vector<int32_t> segs((size_t)ng * (P + 1));
    std::vector<int32_t> gpos(ng + 1, 0);
    std::vector<int32_t> cur(P + 1);
    for (int g = 0; g < ng; ++g) {  // padded segment sizes -> group regions
      const int32_t ge0 = light[gstart[g]].z, ge1 = light[gstart[g + 1] - 1].w;
      std::fill(cur.begin(), cur.end(), 0);
      for (int32_t e = ge0; e < ge1; ++e) cur[h->h_col[e] / SN + 1]++;
      int32_t acc = 0;
      for (int64_t s = 0; s < P; ++s) {
        segs[(size_t)g * (P + 1) + s] = acc;
        acc += (cur[s + 1] + kStagePad - 1) / kStagePad * kStagePad;
      }
      segs[(size_t)g * (P + 1) + P] = acc;
      if (acc > 65536) return fail(FU_ERR_GRAPH, "kernel 8: staged group region exceeds 2^16 elements");
      gpos[g + 1] = gpos[g] + acc;
    }
    const int64_t total = gpos[ng];
    gmax = std::max<int64_t>(gmax, total);
    std::vector<uint16_t> colS(std::max<int64_t>(total, kStagePad), 0);  // >= one 16-B load
    std::vector<uint32_t> sidx(h->E > 0 ? h->E : 1);
    std::vector<int32_t> gbase(light.size());
    std::vector<int32_t> kpos;
    for (int g = 0; g < ng; ++g) {
      const int t0 = gstart[g], t1 = gstart[g + 1];
      const int32_t ge0 = light[t0].z, ge1 = light[t1 - 1].w;
      for (int64_t s = 0; s <= P; ++s) cur[s] = segs[(size_t)g * (P + 1) + s];
      kpos.assign(ge1 - ge0, 0);
      for (int32_t e = ge0; e < ge1; ++e) {  // stable: (slice, tile, position) order
        const int32_t c = h->h_col[e];
        const int32_t k = cur[c / SN]++;
        colS[gpos[g] + k] = (uint16_t)(c % SN);
        kpos[e - ge0] = k;
      }
      for (int t = t0; t < t1; ++t) {  // tile elements in slice order (stable in position)
        gbase[t] = gpos[g];
        const int32_t e0 = light[t].z, ne = light[t].w - light[t].z;
        std::vector<int32_t> ord(ne);
        for (int32_t m = 0; m < ne; ++m) ord[m] = m;
        std::stable_sort(ord.begin(), ord.end(), [&](int32_t x, int32_t y) {
          return h->h_col[e0 + x] / SN < h->h_col[e0 + y] / SN;
        });
        for (int32_t m = 0; m < ne; ++m)
          sidx[e0 + m] = ((uint32_t)kpos[e0 + ord[m] - ge0] << 16) | (uint32_t)ord[m];
      }
      for (int64_t s = 0; s <= P; ++s) segs[(size_t)g * (P + 1) + s] += gpos[g];  // absolute
    }
    // stage blocks (s, q), blockIdx = s + P * q (slice s on XCD s % 8 when 8 | P); slice
    // s's padded segments are cut into items of <= kStageItem elements (one wave each), and
    // its Q blocks take equal shares of the item list
    const int64_t Q = std::max<int64_t>(1, 512 / P);
    std::vector<int32_t> aoff(P * Q + 1, 0);
    std::vector<int2> aitem;
    std::vector<std::vector<int2>> per_s(P);
    for (int64_t s = 0; s < P; ++s)
      for (int g = 0; g < ng; ++g) {
        const int32_t kb = segs[(size_t)g * (P + 1) + s], ke = segs[(size_t)g * (P + 1) + s + 1];
        for (int32_t k = kb; k < ke; k += kStageItem) per_s[s].push_back(make_int2(k, std::min(kStageItem, ke - k)));
      }
    for (int64_t q = 0; q < Q; ++q)
      for (int64_t s = 0; s < P; ++s) {  // q outer, s inner: b = s + P q in order
        const int64_t b = s + P * q, ni = (int64_t)per_s[s].size();
        aoff[b] = (int32_t)aitem.size();
        for (int64_t i = ni * q / Q; i < ni * (q + 1) / Q; ++i) aitem.push_back(per_s[s][i]);
      }
    aoff[P * Q] = (int32_t)aitem.size();
    // compact sidx: within a tile's slice-order list, the elements of one slice are
    // consecutive in the group region, so G index - m is constant per run
    std::vector<uint16_t> s16;
    std::vector<int32_t> dt;
    bool compact = kStageTE <= 1024;
    if (compact) {
      s16.assign(h->E > 0 ? h->E : 1, 0);
      dt.assign(light.size() * kStageRuns, 0);
      for (size_t t = 0; t < light.size() && compact; ++t) {
        const int32_t e0 = light[t].z, ne = light[t].w - light[t].z;
        int run = -1;
        int32_t dprev = 0;
        int64_t sprev = -1;
        for (int32_t m = 0; m < ne; ++m) {
          const uint32_t v = sidx[e0 + m];
          const int32_t pos = (int32_t)(v & 0xFFFFu), kp = (int32_t)(v >> 16);
          const int64_t sl = h->h_col[e0 + pos] / SN;
          if (sl != sprev) {
            if (++run >= kStageRuns) { compact = false; break; }
            sprev = sl;
            dprev = kp - m;
            dt[t * kStageRuns + run] = dprev;
          } else if (kp - m != dprev) {
            compact = false;
            break;
          }
          s16[e0 + m] = (uint16_t)(pos | (run << 10));
        }
      }
    }
    if (L.sidx16) hipFree(L.sidx16);
    if (L.dtab) hipFree(L.dtab);
    L.sidx16 = nullptr;
    L.dtab = nullptr;
    if (compact) {
      if (int rc = up(&L.sidx16, s16.data(), s16.size())) return rc;
      if (int rc = up(&L.dtab, dt.data(), dt.size())) return rc;
    }
    L.P = (int)P;
    L.Q = (int)Q;
    if (int rc = up(&L.aoff, aoff.data(), aoff.size())) return rc;
    if (int rc = up(&L.aitem, aitem.data(), aitem.size())) return rc;
    if (int rc = up(&L.colS, colS.data(), colS.size())) return rc;
    if (int rc = up(&L.sidx, sidx.data(), sidx.size())) return rc;
    if (int rc = up(&L.gbase, gbase.data(), gbase.size())) return rc;
  }
  if (int rc = dmalloc(reinterpret_cast<unsigned long long **>(&h->stG), (size_t)gmax)) return rc;
  HIP_TRY(hipMemset(h->stG, 0, sizeof(unsigned long long) * (size_t)gmax));
  bool any = false;
  for (int li = 0; li < 4; ++li) any |= h->st[li].P > 0;
  if (!any) return fail(FU_ERR_GRAPH, "kernel 8 (staged slices): graph has too many nodes for a slice layout");
  h->st_ready = true;
  return FU_OK;
}

// Layout per table width (device-side choice): the narrowest built layout whose elements
// hold the width's (the table sits in LDS), else the widest built one (the stage launch
// then reads the table from global memory); a forced layout (tests) for every width.
StageArgs stage_args(fu_handle *h, unsigned *grid) {
  StageArgs sa{};
  unsigned g = 1;
  for (int li = 0; li < 4; ++li) {
    const auto &L = h->st[li];
    sa.P[li] = L.P ? L.P : 1;
    sa.Q[li] = L.P ? L.Q : 0;
    sa.aoff[li] = L.aoff;
    sa.aitem[li] = L.aitem;
    sa.colS[li] = L.colS;
    sa.sidx[li] = L.sidx;
    sa.gbase[li] = L.gbase;
    sa.sidx16[li] = h->st_compact ? L.sidx16 : nullptr;
    sa.dtab[li] = L.dtab;
    if (L.P) g = std::max<unsigned>(g, (unsigned)(L.P * L.Q));
  }
  for (int want = 0; want < 4; ++want) {
    int pick = -1;
    if (h->st_force >= 0 && h->st[h->st_force].P) pick = h->st_force;
    for (int li = want; li < 4 && pick < 0; ++li)
      if (h->st[li].P) pick = li;
    for (int li = want; li >= 0 && pick < 0; --li)
      if (h->st[li].P) pick = li;
    sa.sel[want] = pick < 0 ? 0 : pick;
  }
  if (grid) *grid = g;
  return sa;
}

int ensure_a2(fu_handle *h) {
  if (h->a[2]) return FU_OK;
  if (int rc = dmalloc(&h->a[2], (size_t)h->na)) return rc;
  HIP_TRY(hipMemset(h->a[2], 0, sizeof(double) * h->na));
  return FU_OK;
}

int ensure_inbox(fu_handle *h) {
  if (h->inbox[0]) return FU_OK;
  for (int k = 0; k < 2; ++k)
    if (int rc = dmalloc(&h->inbox[k], (size_t)h->E)) return rc;
  return FU_OK;
}

inline unsigned grid_for(long long work) { return (unsigned)((work + kBlock - 1) / kBlock); }

// One round: state in buffer `cur` -> buffer `cur ^ 1`. err_slot: nullptr = no check.
int launch_round(fu_handle *h, unsigned long long *err_slot) {
  const int src = h->cur, dst = h->cur ^ 1;
  const bool check = err_slot != nullptr;
  if (h->dist) {
    if (int rc = fu__dist_round_hook(h, 0)) return rc;
  }
  if (h->kernel >= 4) {
    const int64_t r = h->rounds;
    if (r == 0) {
      hipLaunchKernelGGL(k_round0<true>, dim3(grid_for(h->n)), dim3(kBlock), 0, h->stream, h->n,
                         h->rowptr, h->v, h->f[0], h->a[0]);
      if (h->E)
        hipLaunchKernelGGL(k_round0_flows, dim3(grid_for(h->E)), dim3(kBlock), 0, h->stream, h->n,
                           (long long)h->E, h->rowptr, h->a[0], h->f[0]);
      if (h->E)  // f_{-1} = -0.0 (split words) so that round 1 reproduces (0.0 + a) - 0.0
        hipLaunchKernelGGL(k_fill_split, dim3(grid_for(h->E)), dim3(kBlock), 0, h->stream, (long long)h->E,
                           -0.0, h->f[1]);
      HIP_TRY(hipMemsetAsync(h->a[2], 0, sizeof(double) * h->na, h->stream));  // a_{-1} = 0.0
      HIP_TRY(hipMemsetAsync(h->pctl, 0, sizeof(PackCtl) * 3, h->stream));      // no codes yet
      if (check)
        hipLaunchKernelGGL(k_max_err, dim3(std::min(1024u, grid_for(h->n))), dim3(kBlock), 0,
                           h->stream, h->n, h->a[0], h->target, err_slot);
    } else if (h->kernel == 6) {
      double *F = h->f[r & 1];
      const double *ap = h->a[(r - 1) % 3], *ap2 = h->a[(r + 1) % 3];
      double *an = h->a[r % 3];
      const unsigned gblocks = (unsigned)((h->e0_count + kGatherChunk - 1) / kGatherChunk);
      if (gblocks)
        hipLaunchKernelGGL(k_gather_part0, dim3(gblocks), dim3(kBlock), 0, h->stream, h->colpm,
                           (long long)h->e0_count, ap, h->G);
      if (check)
        hipLaunchKernelGGL((k_round_split<true, true>), dim3(h->ntiles_s), dim3(kBlock), 0, h->stream,
                           h->tiles_s, h->tiles_g, h->rowptr, h->rowptr0, (long long)h->e0_count, h->v, F,
                           h->G, ap2, an, h->target, err_slot, h->pctl, (int)(r & 1), h->colpm, ap);
      else
        hipLaunchKernelGGL((k_round_split<false, true>), dim3(h->ntiles_s), dim3(kBlock), 0, h->stream,
                           h->tiles_s, h->tiles_g, h->rowptr, h->rowptr0, (long long)h->e0_count, h->v, F,
                           h->G, ap2, an, h->target, err_slot, h->pctl, (int)(r & 1), h->colpm, ap);
    } else if (h->kernel == 5) {
      double *F = h->f[r & 1];
      const double *ap = h->a[(r - 1) % 3], *ap2 = h->a[(r + 1) % 3];
      double *an = h->a[r % 3];
      const long long E1 = h->E - h->e0_count;
      const long long mx = std::max<long long>(h->e0_count, E1);
      const unsigned gblocks = (unsigned)(8 * ((mx + 4LL * kGatherChunk - 1) / (4LL * kGatherChunk)));
      if (gblocks)
        hipLaunchKernelGGL(k_gather_split, dim3(gblocks), dim3(kBlock), 0, h->stream, h->colpm,
                           (long long)h->e0_count, (long long)h->E, ap, h->G);
      if (check)
        hipLaunchKernelGGL(k_round_split<true>, dim3(h->ntiles_s), dim3(kBlock), 0, h->stream, h->tiles_s,
                           h->tiles_g, h->rowptr, h->rowptr0, (long long)h->e0_count, h->v, F, h->G, ap2, an,
                           h->target, err_slot, h->pctl, (int)(r & 1));
      else
        hipLaunchKernelGGL(k_round_split<false>, dim3(h->ntiles_s), dim3(kBlock), 0, h->stream, h->tiles_s,
                           h->tiles_g, h->rowptr, h->rowptr0, (long long)h->e0_count, h->v, F, h->G, ap2, an,
                           h->target, err_slot, h->pctl, (int)(r & 1));
    } else if (h->kernel == 9 || h->kernel == 10) {
      double *F = h->f[r & 1];
      const double *ap = h->a[(r - 1) % 3], *ap2 = h->a[(r + 1) % 3];
      double *an = h->a[r % 3];
      const void *cp = h->code[(r - 1) & 1];
      const bool staged = h->kernel == 10;
      unsigned sgrid = 1;
      const StageArgs sa = staged ? stage_args(h, &sgrid) : StageArgs{};
      if (staged && h->st_ngroups)
        hipLaunchKernelGGL(k_stage, dim3(sgrid), dim3(kStageThreads), 0, h->stream, sa, h->n, ap, cp, h->pctl,
                           (int)(r & 1), h->stG);
      long long nbl = std::max<long long>((h->st_ntiles + kPipeChunk - 1) / kPipeChunk, (long long)h->pipe_bpc * h->n_cu);
      nbl = std::min<long long>(nbl, ((long long)h->st_ntiles + 7) / 8 * 8);
      nbl = std::max<long long>(8, (nbl + 7) / 8 * 8);
      const dim3 grid((unsigned)(nbl + h->st_nheavy));
#define FU_PIPE(C, M)                                                                                  \
  hipLaunchKernelGGL((k_round_pipe<C, M>), grid, dim3(kBlock), 0, h->stream, h->st_tiles, h->st_gbase,       \
                     h->st_ntiles, h->st_heavy, h->st_nheavy, h->rowptr, h->col, sa, h->stG, h->v, F, ap,     \
                     ap2, an, h->target, err_slot, cp, h->code[r & 1], h->pctl, (int)(r & 1),           \
                     (int)std::max<int64_t>(0, h->E - 1))
      if (check) {
        if (staged) FU_PIPE(true, 1); else FU_PIPE(true, 0);
      } else {
        if (staged) FU_PIPE(false, 1); else FU_PIPE(false, 0);
      }
#undef FU_PIPE
    } else if (h->kernel == 8) {
      double *F = h->f[r & 1];
      const double *ap = h->a[(r - 1) % 3], *ap2 = h->a[(r + 1) % 3];
      double *an = h->a[r % 3];
      unsigned sgrid = 1;
      const StageArgs sa = stage_args(h, &sgrid);
      const void *cp = h->code[(r - 1) & 1];
      if (h->st_ngroups && h->diag < 2)
        hipLaunchKernelGGL(k_stage, dim3(sgrid), dim3(kStageThreads), 0, h->stream, sa, h->n, ap, cp, h->pctl,
                           (int)(r & 1), h->stG);
      if (h->st_nheavy) {
        if (check)
          hipLaunchKernelGGL((k_round_recon<true, false, 0, kStageTE, kStageTN>), dim3(h->st_nheavy), dim3(kBlock), 0,
                             h->stream, h->st_heavy, h->rowptr, h->col, h->v, F, ap, ap2, an, h->target, err_slot,
                             h->perm, cp, h->code[r & 1], h->pctl, (int)(r & 1), nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0);
        else
          hipLaunchKernelGGL((k_round_recon<false, false, 0, kStageTE, kStageTN>), dim3(h->st_nheavy), dim3(kBlock), 0,
                             h->stream, h->st_heavy, h->rowptr, h->col, h->v, F, ap, ap2, an, h->target, err_slot,
                             h->perm, cp, h->code[r & 1], h->pctl, (int)(r & 1), nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0);
      }
#ifdef FU_DIAG
      if (h->st_ntiles && h->diag == 4) {  // round launch alone (stale G: timing only)
        hipLaunchKernelGGL((k_round_staged<false, kStageTE, kStageTN, 4>), dim3(h->st_ntiles), dim3(kBlock), 0,
                           h->stream, h->st_tiles, h->st_gbase, h->st_ntiles, h->rowptr, h->col, sa, h->stG,
                           h->v, F, ap, ap2, an, h->target, err_slot, h->code[r & 1], h->pctl, (int)(r & 1));
      } else if (h->st_ntiles && h->diag) {
        if (h->diag == 3)
          hipLaunchKernelGGL((k_round_staged<false, kStageTE, kStageTN, 3>), dim3(h->st_ntiles), dim3(kBlock), 0,
                             h->stream, h->st_tiles, h->st_gbase, h->st_ntiles, h->rowptr, h->col, sa, h->stG,
                             h->v, F, ap, ap2, an, h->target, err_slot, h->code[r & 1], h->pctl, (int)(r & 1));
        else
          hipLaunchKernelGGL((k_round_staged<false, kStageTE, kStageTN, 1>), dim3(h->st_ntiles), dim3(kBlock), 0,
                             h->stream, h->st_tiles, h->st_gbase, h->st_ntiles, h->rowptr, h->col, sa, h->stG,
                             h->v, F, ap, ap2, an, h->target, err_slot, h->code[r & 1], h->pctl, (int)(r & 1));
      } else
#endif
      if (h->st_ntiles) {
        if (check)
          hipLaunchKernelGGL((k_round_staged<true, kStageTE, kStageTN>), dim3(h->st_ntiles), dim3(kBlock), 0,
                             h->stream, h->st_tiles, h->st_gbase, h->st_ntiles, h->rowptr, h->col, sa, h->stG,
                             h->v, F, ap, ap2, an, h->target, err_slot, h->code[r & 1], h->pctl, (int)(r & 1));
        else
          hipLaunchKernelGGL((k_round_staged<false, kStageTE, kStageTN>), dim3(h->st_ntiles), dim3(kBlock), 0,
                             h->stream, h->st_tiles, h->st_gbase, h->st_ntiles, h->rowptr, h->col, sa, h->stG,
                             h->v, F, ap, ap2, an, h->target, err_slot, h->code[r & 1], h->pctl, (int)(r & 1));
      }
    } else if (h->kernel == 7) {
      double *F = h->f[r & 1];
      const double *ap = h->a[(r - 1) % 3], *ap2 = h->a[(r + 1) % 3];
      double *an = h->a[r % 3];
      const int wg = h->wgeo;
      if (h->nwheavy[wg]) {
        if (check)
          hipLaunchKernelGGL((k_round_recon<true, false, 0, 2048, 256>), dim3(h->nwheavy[wg]), dim3(kBlock), 0,
                             h->stream, h->wheavy[wg], h->rowptr, h->col, h->v, F, ap, ap2, an, h->target, err_slot,
                             h->perm, h->code[(r - 1) & 1], h->code[r & 1], h->pctl, (int)(r & 1), nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0);
        else
          hipLaunchKernelGGL((k_round_recon<false, false, 0, 2048, 256>), dim3(h->nwheavy[wg]), dim3(kBlock), 0,
                             h->stream, h->wheavy[wg], h->rowptr, h->col, h->v, F, ap, ap2, an, h->target, err_slot,
                             h->perm, h->code[(r - 1) & 1], h->code[r & 1], h->pctl, (int)(r & 1), nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0);
      }
      if (h->nwtiles[wg]) {
        const unsigned blocks = (unsigned)((h->nwtiles[wg] + kBlock / 64 - 1) / (kBlock / 64));
#define FU_WAVE(C, TE, TN)                                                                          \
  hipLaunchKernelGGL((k_round_wave<C, TE, TN>), dim3(blocks), dim3(kBlock), 0, h->stream, h->wtiles[wg], \
                     h->nwtiles[wg], h->rowptr, h->col, h->v, F, ap, ap2, an, h->target, err_slot,         \
                     h->code[(r - 1) & 1], h->code[r & 1], h->pctl, (int)(r & 1))
        if (wg == 0) {
          if (check) FU_WAVE(true, 256, 32); else FU_WAVE(false, 256, 32);
        } else {
          if (check) FU_WAVE(true, 512, 64); else FU_WAVE(false, 512, 64);
        }
#undef FU_WAVE
      }
    } else {
      double *F = h->f[r & 1];
      const double *ap = h->a[(r - 1) % 3], *ap2 = h->a[(r + 1) % 3];
      double *an = h->a[r % 3];
      // heavy tiles (hubs, heavy rows, bins) lead the tile list: they run as their own launch
      // on the side stream, concurrently with the light tiles' launch (which then keeps
      // kernel 4's light-path register budget: 64 VGPRs, 8 waves per SIMD)
      const int nh = h->nheavy_geo[h->geo], nl = h->ntiles_geo[h->geo] - nh;
      const int hub_sep = h->n_hub && !(h->geo == 0 && h->bins) ? 1 : 0;  // k_hub_flows after
      const bool fork = nh > 0 && h->fork_heavy;
      hipStream_t hs = fork ? h->stream2 : h->stream;
      if (fork) {
        HIP_TRY(hipEventRecord(h->ev_fork, h->stream));
        HIP_TRY(hipStreamWaitEvent(h->stream2, h->ev_fork, 0));
      }
      if (h->n_hub && !(h->geo == 0 && h->bins)) {
        if (h->hub_scan) {  // pieces: (fr, er) + approximate sums, then the run summaries
          hipLaunchKernelGGL(k_hub_stage_p, dim3(h->n_piece), dim3(kBlock), 0, hs, h->hub_piece, h->hub_rows,
                             h->col, F, ap, ap2, h->code[(r - 1) & 1], h->pctl, (int)(r & 1), h->hubxy, h->psum);
          hipLaunchKernelGGL(k_hub_sum, dim3(h->n_piece), dim3(kBlock), 0, hs, h->hub_piece, h->hub_p0,
                             h->psum, h->hubxy, h->hsum);
        } else {
          hipLaunchKernelGGL(k_hub_stage, dim3(grid_for(h->hub_total)), dim3(kBlock), 0, hs, h->n_hub,
                             h->hub_rows, (long long)h->hub_total, h->col, F, ap, ap2, h->code[(r - 1) & 1],
                             h->pctl, (int)(r & 1), h->hubxy);
        }
      }
#define FU_RECON_G(C, N, D, TE, TN)                                                         \
  do {                                                                                      \
    if (nh)                                                                                 \
      hipLaunchKernelGGL((k_round_recon<C, false, (D == 5 || D == 6 ? D : 0), TE, TN, 2>), dim3(nh), dim3(kBlock), 0, hs, \
                         h->tiles_geo[h->geo], h->rowptr, h->col, h->v, F, ap, ap2, an, h->target, err_slot, h->perm, \
                         h->code[(r - 1) & 1], h->code[r & 1], h->pctl, (int)(r & 1), h->hubxy, h->hub_off, \
                         h->hrows, h->hub_scan ? h->hsum : nullptr, h->hub_p0, h->hub_redo, hub_sep); \
    if (nl)                                                                                 \
      hipLaunchKernelGGL((k_round_recon<C, N, D, TE, TN, 1>), dim3(nl), dim3(kBlock), 0, h->stream, \
                         h->tiles_geo[h->geo] + nh, h->rowptr, h->col, h->v, F, ap, ap2, an, h->target, err_slot, \
                         h->perm, h->code[(r - 1) & 1], h->code[r & 1], h->pctl, (int)(r & 1), nullptr, nullptr, \
                         nullptr, nullptr, nullptr, nullptr, 0);                             \
  } while (0)
#define FU_RECON(C, N, D)                                                                   \
  do {                                                                                      \
    if (h->geo == 0) FU_RECON_G(C, N, D, 2048, 256);                                        \
    else if (h->geo == 2) FU_RECON_G(C, N, D, 1024, 256);                                   \
    else if (h->geo == 1) FU_RECON_G(C, N, D, 1024, 128);                                   \
    else FU_RECON_G(C, N, D, 512, 64);                                                      \
  } while (0)
#ifdef FU_DIAG
      if (h->diag == 1) FU_RECON(false, false, 1);
      else if (h->diag == 2) FU_RECON(false, false, 2);
      else if (h->diag == 3) FU_RECON(false, false, 3);
      else if (h->diag == 4) FU_RECON(false, false, 4);
      else if (h->diag == 5) FU_RECON(false, false, 5);
      else if (h->diag == 6) FU_RECON(false, false, 6);
      else if (h->diag == 12) FU_RECON(false, false, 12);
      else
#endif
      if (check) {
        if (h->nt) FU_RECON(true, true, 0); else FU_RECON(true, false, 0);
      } else {
        if (h->nt) FU_RECON(false, true, 0); else FU_RECON(false, false, 0);
      }
#undef FU_RECON
#undef FU_RECON_G
      if (hub_sep)
        hipLaunchKernelGGL(k_hub_flows, dim3(grid_for(h->hub_total)), dim3(kBlock), 0, hs, h->n_hub, h->hub_rows,
                           (long long)h->hub_total, h->hubxy, an, F);
      if (fork) {
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(h->ev_join, h->stream2));
        HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_join, 0));
      }
    }
  } else if (h->rounds == 0) {
    if (h->kernel == 3) {
      hipLaunchKernelGGL(k_round0_push, dim3(grid_for(h->n)), dim3(kBlock), 0, h->stream, h->n,
                         h->rowptr, h->rev, h->v, h->inbox[dst], h->a[dst]);
    } else {
      hipLaunchKernelGGL(k_round0<false>, dim3(grid_for(h->n)), dim3(kBlock), 0, h->stream, h->n,
                         h->rowptr, h->v, h->f[dst], h->a[dst]);
    }
    if (check) {
      hipLaunchKernelGGL(k_max_err, dim3(std::min(1024u, grid_for(h->n))), dim3(kBlock), 0,
                         h->stream, h->n, h->a[dst], h->target, err_slot);
    }
  } else if (h->kernel == 1) {
    if (check)
      hipLaunchKernelGGL(k_round_tpn<true>, dim3(grid_for(h->n)), dim3(kBlock), 0, h->stream,
                         h->n, h->rowptr, h->col, h->rev, h->v, h->f[src], h->a[src], h->f[dst],
                         h->a[dst], h->target, err_slot);
    else
      hipLaunchKernelGGL(k_round_tpn<false>, dim3(grid_for(h->n)), dim3(kBlock), 0, h->stream,
                         h->n, h->rowptr, h->col, h->rev, h->v, h->f[src], h->a[src], h->f[dst],
                         h->a[dst], h->target, err_slot);
  } else if (h->kernel == 2) {
    if (check)
      hipLaunchKernelGGL(k_round_tile<true>, dim3(h->ntiles), dim3(kBlock), 0, h->stream,
                         h->tiles, h->rowptr, h->col, h->rev, h->v, h->f[src], h->a[src],
                         h->f[dst], h->a[dst], h->target, err_slot);
    else
      hipLaunchKernelGGL(k_round_tile<false>, dim3(h->ntiles), dim3(kBlock), 0, h->stream,
                         h->tiles, h->rowptr, h->col, h->rev, h->v, h->f[src], h->a[src],
                         h->f[dst], h->a[dst], h->target, err_slot);
  } else {
    if (check)
      hipLaunchKernelGGL(k_round_push<true>, dim3(h->ntiles), dim3(kBlock), 0, h->stream,
                         h->tiles, h->rowptr, h->rev, h->v, h->inbox[src], h->inbox[dst],
                         h->a[dst], h->target, err_slot);
    else
      hipLaunchKernelGGL(k_round_push<false>, dim3(h->ntiles), dim3(kBlock), 0, h->stream,
                         h->tiles, h->rowptr, h->rev, h->v, h->inbox[src], h->inbox[dst],
                         h->a[dst], h->target, err_slot);
  }
  HIP_TRY(hipGetLastError());
  h->cur = dst;
  h->rounds++;
  // refresh the packing plan from a_r (kernel 4 encodes with it from the next round on);
  // once the host has seen the narrowest width (8), every 8th time only: the plan and its
  // width copy stall the stream for ~20 us
  const int every = h->seen_width == 8 ? 8 * h->pack_every : h->pack_every;
  if (h->kernel >= 4 && h->pack && !h->dist && h->n_psample > 0 && h->rounds % every == 0) {
    hipLaunchKernelGGL(k_pack_plan, dim3(1), dim3(kBlock), 0, h->stream, cur_a(h), h->psample, h->pctl);
    HIP_TRY(hipGetLastError());
    if (!h->pw_pending) {  // the autotuner watches the width (poll_pack_width)
      HIP_TRY(hipMemcpyAsync(h->h_pw, &h->pctl[2].width, sizeof(int), hipMemcpyDeviceToHost, h->stream));
      HIP_TRY(hipEventRecord(h->ev_pw, h->stream));
      h->pw_pending = true;
    }
  }
  if (h->dist) {
    if (int rc = fu__dist_round_hook(h, 1)) return rc;
  }
  return FU_OK;
}

struct TuneCand {
  int kernel, nt, geo;
};
// kernel 7 (wave tiles) is not a candidate: slower than kernel 4 at 512x64 everywhere
// measured; it stays selectable as an option
// measured on ER-1M / R-MAT: 4+nt, 4 at 1024x256, 5 and 9 never win; they stay options
static std::vector<TuneCand> tune_cands(const fu_handle *h) {
  // fixed order (fu_get_info reports per index); kernels 6, 8, 10 are single-GPU only
  (void)h;
  return {{4, 0, 0}, {4, 0, 3}, {6, 0, 0}, {8, 0, 0}, {10, 0, 0}, {4, 0, 1}};
}
static int width_class(int w) { return w == 8 ? 1 : w == 16 ? 2 : w == 32 ? 3 : 0; }
static void use_cand(fu_handle *h, const TuneCand &c) {
  h->kernel = c.kernel;
  h->nt = c.nt;
  if (h->kernel == 7) h->wgeo = c.geo;
  else h->geo = c.geo;
}

int set_device(fu_handle *h) {
  HIP_TRY(hipSetDevice(h->device));
  return FU_OK;
}

}  // namespace

extern "C" {

int fu_device_count(int32_t *out) {
  if (!out) return fail(FU_ERR_ARG, "fu_device_count: NULL");
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
  *out = c;
  return FU_OK;
}

// Internal constructor shared by fu_create / fu_dist_create: uploads the local CSR.
int fu__create_common(int32_t n, int64_t e, const int64_t *rowptr, const int32_t *col,
                      const int32_t *rev, const double *value, int32_t device,
                      int64_t f_extra, int32_t a_extra, fu_handle **out) {
  FU_TRY_BEGIN
  // rev may be NULL only for the estimates-only multi-GPU halo (kernel 4 never reads rev)
  if (!out || n <= 0 || e < 0 || !rowptr || !value || (e > 0 && !col) || (e > 0 && !rev && f_extra != -1))
    return fail(FU_ERR_ARG, "fu_create: bad arguments");
  const bool no_rev = f_extra == -1;
  if (no_rev) f_extra = 0;
  if (e + f_extra >= (int64_t)INT32_MAX) return fail(FU_ERR_ARG, "fu_create: more than 2^31-1 edges");
  if (rowptr[0] != 0 || rowptr[n] != e) return fail(FU_ERR_ARG, "fu_create: rowptr[0] must be 0 and rowptr[n] == e");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(FU_ERR_HIP, "fu_create: no HIP device visible");
  if (device < 0 || device >= ndev) return fail(FU_ERR_ARG, "fu_create: device out of range");
  auto *h = new fu_handle();
  h->device = device;
  h->n = n;
  h->E = e;
  h->h_rowptr.assign(rowptr, rowptr + n + 1);
  if (e > 0) h->h_col.assign(col, col + e);
  std::vector<int32_t> rp32(n + 1);
  int32_t md = 0;
  for (int32_t i = 0; i <= n; ++i) {
    rp32[i] = (int32_t)rowptr[i];
    if (i < n) {
      if (rowptr[i + 1] < rowptr[i]) { delete h; return fail(FU_ERR_ARG, "fu_create: rowptr not monotone"); }
      md = std::max<int32_t>(md, (int32_t)(rowptr[i + 1] - rowptr[i]));
    }
  }
  h->max_deg = md;
  const int64_t fe = e + f_extra;
  const int32_t na = n + a_extra;
  h->na = na;
  for (int64_t k = 0; k < e; ++k) {
    if (col[k] < 0 || col[k] >= na || (!no_rev && (rev[k] < 0 || rev[k] >= fe))) {
      delete h;
      return fail(FU_ERR_ARG, "fu_create: col/rev index out of range at edge " + std::to_string(k));
    }
  }
  int rc = FU_OK;
  auto cleanup = [&](int code) { fu_destroy(h); return code; };
  if ((rc = set_device(h))) return cleanup(rc);
  {  // the side stream (kernel 4's heavy tiles: the long exact chains) gets the highest
     // priority, so its blocks are dispatched ahead of the light tiles when CU slots free up
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) lo = hi = 0;
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithPriority(&h->stream2, hipStreamNonBlocking, hi) != hipSuccess)
      return cleanup(fail(FU_ERR_HIP, "hipStreamCreate failed"));
  }
  {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0) h->n_cu = cus;
  }
  if (hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess ||
      hipEventCreate(&h->ev2) != hipSuccess || hipEventCreate(&h->ev3) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_pw, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming) != hipSuccess)
    return cleanup(fail(FU_ERR_HIP, "hipEventCreate failed"));
  if (hipHostMalloc(reinterpret_cast<void **>(&h->h_pw), sizeof(int), hipHostMallocDefault) != hipSuccess)
    return cleanup(fail(FU_ERR_ALLOC, "hipHostMalloc failed"));
  *h->h_pw = 0;
  if ((rc = dmalloc(&h->rowptr, n + 1)) || (rc = dmalloc(&h->col, e)) || (!no_rev && (rc = dmalloc(&h->rev, e))) ||
      (rc = dmalloc(&h->v, n)) || (rc = dmalloc(&h->f[0], (fe + 31) / 32 * 32)) ||
      (rc = dmalloc(&h->f[1], (fe + 31) / 32 * 32)) ||
      (rc = dmalloc(&h->a[0], na)) || (rc = dmalloc(&h->a[1], na)) || (rc = dmalloc(&h->target, n)) ||
      (rc = dmalloc(&h->err, 1)))
    return cleanup(rc);
  h->errcap = 1;
  if (hipMemcpy(h->rowptr, rp32.data(), sizeof(int) * (n + 1), hipMemcpyHostToDevice) != hipSuccess ||
      (e && hipMemcpy(h->col, col, sizeof(int) * e, hipMemcpyHostToDevice) != hipSuccess) ||
      (e && !no_rev && hipMemcpy(h->rev, rev, sizeof(int) * e, hipMemcpyHostToDevice) != hipSuccess) ||
      hipMemcpy(h->v, value, sizeof(double) * n, hipMemcpyHostToDevice) != hipSuccess)
    return cleanup(fail(FU_ERR_HIP, "fu_create: upload failed"));
  if ((e == 0 && hipMemset(h->col, 0, sizeof(int)) != hipSuccess) ||  // kernels 9/10 read col[0]
      hipMemset(h->f[0], 0, sizeof(double) * (fe ? fe : 1)) != hipSuccess ||
      hipMemset(h->f[1], 0, sizeof(double) * (fe ? fe : 1)) != hipSuccess ||
      hipMemset(h->a[0], 0, sizeof(double) * na) != hipSuccess ||
      hipMemset(h->a[1], 0, sizeof(double) * na) != hipSuccess)
    return cleanup(fail(FU_ERR_HIP, "fu_create: memset failed"));
  if ((rc = build_tiles(h))) return cleanup(rc);
  if ((rc = ensure_a2(h))) return cleanup(rc);
  if ((rc = dmalloc(&h->pctl, 3)) || (rc = dmalloc(&h->code[0], 4 * (size_t)na)) ||
      (rc = dmalloc(&h->code[1], 4 * (size_t)na)))
    return cleanup(rc);
  if (hipMemset(h->pctl, 0, sizeof(PackCtl) * 3) != hipSuccess) return cleanup(fail(FU_ERR_HIP, "fu_create: memset failed"));
  if (e > 0) {  // plan sample: the targets of 4096 pseudo-random edges (degree-weighted)
    const int ns = kPlanSamples;
    std::vector<int32_t> smp(ns);
    for (int q = 0; q < ns; ++q) smp[q] = col[splitmix_at(0x9ac4u, (uint64_t)q) % (uint64_t)e];
    if ((rc = dmalloc(&h->psample, ns))) return cleanup(rc);
    if (hipMemcpy(h->psample, smp.data(), sizeof(int32_t) * ns, hipMemcpyHostToDevice) != hipSuccess)
      return cleanup(fail(FU_ERR_HIP, "fu_create: upload failed"));
    h->n_psample = ns;
  }
  *out = h;
  return FU_OK;
  FU_TRY_END
}

int fu_create(int32_t n, int64_t e, const int64_t *rowptr, const int32_t *col,
              const int32_t *rev, const double *value, int32_t device, fu_handle **out) {
  FU_TRY_BEGIN
  if (!rowptr || n <= 0) return fail(FU_ERR_ARG, "fu_create: bad arguments");
  std::vector<int32_t> own_rev;
  if (!rev && e > 0) {
    fu_graph g;
    g.n = n;
    g.rowptr.assign(rowptr, rowptr + n + 1);
    if (!col) return fail(FU_ERR_ARG, "fu_create: col is NULL");
    g.col.assign(col, col + e);
    if (int rc = fu::build_rev(g)) return rc;
    own_rev.swap(g.rev);
    rev = own_rev.data();
  }
  return fu__create_common(n, e, rowptr, col, rev, value, device, 0, 0, out);
  FU_TRY_END
}

int fu_create_from_graph(const fu_graph *g, const double *value, int32_t device,
                         fu_handle **out) {
  if (!g) return fail(FU_ERR_ARG, "fu_create_from_graph: NULL graph");
  const int64_t E = g->rowptr[g->n];
  if ((int64_t)g->rev.size() != E) return fail(FU_ERR_GRAPH, "fu_create_from_graph: graph is not symmetric");
  return fu__create_common(g->n, E, g->rowptr.data(), g->col.data(), g->rev.data(), value, device, 0, 0, out);
}

int fu_create_from_graph_ex(const fu_graph *g, const double *value, int32_t device,
                            int32_t layout, fu_handle **out) {
  FU_TRY_BEGIN
  if (!g || !value || !out || layout < 0 || layout > 1) return fail(FU_ERR_ARG, "fu_create_from_graph_ex: bad arguments");
  if (layout == 0) return fu_create_from_graph(g, value, device, out);
  const int32_t n = g->n;
  std::vector<int32_t> nofo(n);
  fu_graph *rg = nullptr;
  if (int rc = fu_graph_relabel(g, 1, nofo.data(), &rg)) return rc;
  std::vector<double> v2(n);
  for (int32_t i = 0; i < n; ++i) v2[nofo[i]] = value[i];
  const int rc = fu_create_from_graph(rg, v2.data(), device, out);
  fu_graph_free(rg);
  if (rc) return rc;
  (*out)->h_new_of_old.swap(nofo);
  (*out)->h_orig_rowptr = g->rowptr;
  return FU_OK;
  FU_TRY_END
}

int fu_set_option(fu_handle *h, const char *key, int64_t value) {
  if (!h || !key) return fail(FU_ERR_ARG, "fu_set_option: NULL argument");
  if (int rc = set_device(h)) return rc;
  if (!std::strcmp(key, "kernel")) {
    if (value < 0 || value > 10) return fail(FU_ERR_ARG, "fu_set_option: kernel must be 0..10");
    if (h->dist && value != 0 && value != 2 && value != 4)  // 5, 6: single GPU only
      return fail(FU_ERR_ARG, "fu_set_option: multi-GPU supports kernels 2 (pull) and 4 (recon)");
    if (!h->rev && h->E > 0 && value >= 1 && value <= 3)
      return fail(FU_ERR_ARG, "fu_set_option: kernels 1-3 need the reverse-edge index (estimates-only halo)");
    if (h->rounds != 0) return fail(FU_ERR_STATE, "fu_set_option: kernel can only change before the first round (call fu_reset)");
    h->kernel = value == 0 ? 4 : (int)value;
    h->autotune = value == 0;
    h->tuned = false;
    h->nt = 0;
    if (h->kernel == 3) return ensure_inbox(h);
    if (h->kernel == 4 || h->kernel == 7) return ensure_a2(h);
    if (h->kernel == 9) {
      if (int rc = ensure_a2(h)) return rc;
      if (int rc = ensure_light(h)) {
        h->kernel = 4;
        return rc;
      }
    }
    if (h->kernel == 8 || h->kernel == 10) {
      if (int rc = ensure_a2(h)) return rc;
      if (int rc = ensure_stage(h)) {
        h->kernel = 4;
        return rc;
      }
    }
    if (h->kernel == 5 || h->kernel == 6) {
      if (int rc = ensure_a2(h)) return rc;
      if (int rc = ensure_split(h)) {
        h->kernel = 4;
        return rc;
      }
    }
    return FU_OK;
  }
  if (!std::strcmp(key, "stage_layout")) {  // kernel 8: -1 = by packing width, 0..3 forced
    if (value < -1 || value > 3) return fail(FU_ERR_ARG, "fu_set_option: stage_layout must be -1..3");
    h->st_force = (int)value;
    return FU_OK;
  }
  if (!std::strcmp(key, "pipe_bpc")) {  // kernels 9/10: persistent blocks per CU
    if (value < 1 || value > 64) return fail(FU_ERR_ARG, "fu_set_option: pipe_bpc must be in [1, 64]");
    h->pipe_bpc = (int)value;
    return FU_OK;
  }
  if (!std::strcmp(key, "diag")) {  // timing-only ablations (wrong results): tools builds only
#ifdef FU_DIAG
    h->diag = (int)value;
    return FU_OK;
#else
    (void)value;
    return fail(FU_ERR_ARG, "fu_set_option: 'diag' exists only in a -DFU_DIAG build (make DIAG=1)");
#endif
  }
  if (!std::strcmp(key, "nt")) {
    h->nt = value != 0;
    return FU_OK;
  }
  if (!std::strcmp(key, "pack")) {
    h->pack = value != 0;
    if (!h->pack) HIP_TRY(hipMemsetAsync(h->pctl + 2, 0, sizeof(PackCtl), h->stream));  // stop encoding
    return FU_OK;
  }
  if (!std::strcmp(key, "pack_every")) {
    if (value < 1 || value > (1 << 20)) return fail(FU_ERR_ARG, "fu_set_option: pack_every must be in [1, 2^20]");
    h->pack_every = (int)value;
    return FU_OK;
  }
  if (!std::strcmp(key, "bins")) {
    h->bins = value != 0;
    return build_tiles(h);
  }
  if (!std::strcmp(key, "wave_edges")) {  // kernel 7 wave tile: 256 (x32 nodes) or 512 (x64)
    if (value != 256 && value != 512) return fail(FU_ERR_ARG, "fu_set_option: wave_edges must be 256 or 512");
    h->wgeo = value == 512;
    return FU_OK;
  }
  if (!std::strcmp(key, "tile_edges")) {
    if (value != 2048 && value != 1024 && value != 512) return fail(FU_ERR_ARG, "fu_set_option: tile_edges must be 2048, 1024 or 512");
    h->tile_edges = (int)value;
    h->geo = h->tile_edges == 2048 ? 0 : h->tile_edges == 512 ? 3 : h->tile_nodes == 256 ? 2 : 1;
    return FU_OK;
  }
  if (!std::strcmp(key, "tile_nodes")) {
    if (value != 0 && value != 128 && value != 256) return fail(FU_ERR_ARG, "fu_set_option: tile_nodes must be 0, 128 or 256");
    h->tile_nodes = (int)value;
    h->geo = h->tile_edges == 2048 ? 0 : h->tile_edges == 512 ? 3 : h->tile_nodes == 256 ? 2 : 1;
    return FU_OK;
  }
  if (!std::strcmp(key, "stage_compact")) {  // kernel 8: u16 sidx with per-tile runs (1) or u32 (0)
    h->st_compact = value != 0;
    return FU_OK;
  }
  if (!std::strcmp(key, "fork_heavy")) {  // kernel 4: heavy tiles on a side stream (1) or in order (0)
    h->fork_heavy = value != 0;
    return FU_OK;
  }
  if (!std::strcmp(key, "hub_scan")) {  // mega hubs: parallel exact sums (1) or one chain (0)
    h->hub_scan = value != 0;
    return FU_OK;
  }
  if (!std::strcmp(key, "wave_heavy")) {  // kernel 4: heavy rows one per wave (1) or per block (0)
    h->wave_heavy = value != 0;
    return build_tiles(h);
  }
  if (!std::strcmp(key, "mega_hub")) {  // kernel 4: staged-chain rows (tests lower it)
    if (value < 1) return fail(FU_ERR_ARG, "fu_set_option: mega_hub must be >= 1");
    h->mega_hub = (int)std::min<int64_t>(value, INT32_MAX);
    return build_tiles(h);
  }
  if (!std::strcmp(key, "hub_threshold")) {
    if (value < 1) return fail(FU_ERR_ARG, "fu_set_option: hub_threshold must be >= 1");
    h->hub_threshold = (int)std::min<int64_t>(value, kTileEdges);
    return build_tiles(h);
  }
  return fail(FU_ERR_ARG, std::string("fu_set_option: unknown key '") + key + "'");
}

int fu_reset(fu_handle *h) {
  if (!h) return fail(FU_ERR_ARG, "fu_reset: NULL handle");
  if (int rc = set_device(h)) return rc;
  HIP_TRY(hipStreamSynchronize(h->stream));
  h->rounds = 0;
  h->cur = 0;
  h->pw_pending = false;  // the stream is idle: no plan copy in flight
  *h->h_pw = 0;           // round 0 clears the packing plan
  h->seen_width = 0;
  if (h->autotune && h->tuned && h->tune_cache[0] >= 0) {  // unpacked again: its winner
    use_cand(h, tune_cands(h)[h->tune_cache[0]]);
    h->tuned_width = 0;
  }
  return FU_OK;
}

int fu_set_targets(fu_handle *h, const double *target) {
  if (!h || !target) return fail(FU_ERR_ARG, "fu_set_targets: NULL argument");
  if (int rc = set_device(h)) return rc;
  std::vector<double> t2;
  if (!h->h_new_of_old.empty()) {  // caller numbering -> device numbering
    t2.resize(h->n);
    for (int32_t i = 0; i < h->n; ++i) t2[h->h_new_of_old[i]] = target[i];
    target = t2.data();
  }
  HIP_TRY(hipMemcpyAsync(h->target, target, sizeof(double) * h->n, hipMemcpyHostToDevice, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  h->has_target = true;
  return FU_OK;
}

int fu__err_slots(fu_handle *h, int count) {
  if (count <= h->errcap) return FU_OK;
  if (h->err) hipFree(h->err);
  h->err = nullptr;
  h->errcap = 0;
  if (int rc = dmalloc(&h->err, count)) return rc;
  h->errcap = count;
  return FU_OK;
}

// Kernels 4, 5 and 6 share the state layout (F[r & 1], A[r % 3]) and are all bitwise
// exact, so switching between them (or between kernel 4's tile geometries) mid-run changes
// nothing but speed. "auto" times each candidate on real rounds (1 warm + 4 timed each)
// once round 0 is done and keeps the fastest. The rounds count toward the caller's total,
// and the results are unchanged. The pass re-runs when the packing plan changes width (the
// packed gather shifts the balance between the candidates), at most kMaxTunes times.
constexpr int kMaxTunes = 4;

// width: the packing width the pass runs under (kernel 6 writes unpacked tables, so it is
// only a candidate while the table is unpacked)
static int autotune_kernel(fu_handle *h, int32_t *budget, int width) {
  const std::vector<TuneCand> cands = tune_cands(h);
  constexpr int kTimed = 8;
  auto active = [&](size_t c) {
    // multi-GPU: every rank must run the same rounds (each one is a halo exchange), so no
    // candidate is dropped and none stops early on rank-local timings
    return (h->dist || h->tune_out[c] < 2) && !(cands[c].kernel == 6 && width != 0) && !(h->dist && cands[c].kernel != 4);
  };
  int32_t need = 0;
  for (size_t c = 0; c < cands.size(); ++c) need += active(c) ? 1 + kTimed : 0;
  if (*budget < need) return FU_OK;  // not enough rounds in this call: try again later
  float best = 1e30f;
  int bi = -1;
  for (size_t c = 0; c < cands.size(); ++c) {
    // a candidate more than 1.3x slower than the winner in two passes sits out the later
    // ones (its last ns per round stays reported)
    if (!h->dist && h->tune_out[c] >= 2) continue;
    h->tune_ms[c] = 0.f;
    if (!active(c)) continue;
    if (cands[c].kernel == 9) {
      if (ensure_light(h) != FU_OK) {
        set_error("");
        continue;
      }
    } else if (cands[c].kernel == 8 || cands[c].kernel == 10) {
      if (ensure_stage(h) != FU_OK) {  // too many nodes for a slice layout
        set_error("");
        continue;
      }
    } else if (cands[c].kernel >= 5) {
      if (ensure_split(h) != FU_OK) {  // rows not sorted: column split not applicable
        set_error("");
        continue;
      }
    }
    h->kernel = cands[c].kernel;
    h->nt = cands[c].nt;
    if (h->kernel == 7) h->wgeo = cands[c].geo;
    else h->geo = cands[c].geo;
    // the warm round is timed too: a candidate more than twice the best per-round time so far
    // stops there (on R-MAT-24 the staged kernels take 3x kernel 4: 8 rounds of 30 ms each)
    HIP_TRY(hipEventRecord(h->ev0, h->stream));
    if (int rc = launch_round(h, nullptr)) return rc;
    HIP_TRY(hipEventRecord(h->ev1, h->stream));
    if (best < 1e30f && !h->dist) {
      HIP_TRY(hipEventSynchronize(h->ev1));
      float wms = 0.f;
      HIP_TRY(hipEventElapsedTime(&wms, h->ev0, h->ev1));
      if (wms > 2.f * best / kTimed) {
        h->tune_ms[c] = wms;
        *budget -= 1;
        continue;
      }
    }
    HIP_TRY(hipEventRecord(h->ev0, h->stream));
    for (int k = 0; k < kTimed; ++k)
      if (int rc = launch_round(h, nullptr)) return rc;
    HIP_TRY(hipEventRecord(h->ev1, h->stream));
    HIP_TRY(hipEventSynchronize(h->ev1));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, h->ev0, h->ev1));
    h->tune_ms[c] = ms / kTimed;
    *budget -= 1 + kTimed;
    if (ms < best) {
      best = ms;
      bi = (int)c;
    }
  }
  if (bi < 0) return fail(FU_ERR_STATE, "autotune: no candidate ran");
  for (size_t c = 0; c < cands.size(); ++c)
    if (h->tune_ms[c] > 1.3f * h->tune_ms[bi]) h->tune_out[c]++;
  use_cand(h, cands[bi]);
  h->tune_cache[width_class(width)] = bi;
  h->tuned = true;
  h->n_tunes++;
  return FU_OK;
}

// After each packing plan the host keeps an asynchronous copy of its width; a changed width
// re-arms the autotuner (checked without blocking).
static void poll_pack_width(fu_handle *h) {
  if (!h->pw_pending || hipEventQuery(h->ev_pw) != hipSuccess) return;
  h->pw_pending = false;
  h->seen_width = *h->h_pw;
  if (!h->autotune || !h->tuned || *h->h_pw == h->tuned_width) return;
  const int cached = h->tune_cache[width_class(*h->h_pw)];
  if (cached >= 0) {  // this width was tuned before (e.g. before fu_reset): reuse its winner
    use_cand(h, tune_cands(h)[cached]);
    h->tuned_width = *h->h_pw;
  } else if (h->n_tunes < kMaxTunes) {
    h->tuned = false;
  }
}

// The round loop shared by fu_run_collectall and fu_run_collectall_timed.
static int run_rounds(fu_handle *h, int32_t rounds, int32_t err_every, int nerr) {
  for (int32_t r = 0; r < rounds; ++r) {
    poll_pack_width(h);
    // tune between rounds when no error slot is pending in the rounds it would consume
    if (h->autotune && !h->tuned && h->kernel >= 4 && h->rounds >= 1 && nerr == 0) {
      int32_t budget = rounds - r;
      const int w = h->pw_pending ? h->tuned_width : *h->h_pw;
      if (int rc = autotune_kernel(h, &budget, w)) return rc;
      if (h->tuned) h->tuned_width = w;
      r = rounds - budget;
      if (r >= rounds) break;
    }
    unsigned long long *slot = nullptr;
    if (nerr > 0 && (r + 1) % err_every == 0) slot = h->err + ((r + 1) / err_every - 1);
    if (int rc = launch_round(h, slot)) return rc;
  }
  return FU_OK;
}

int fu_run_collectall(fu_handle *h, int32_t rounds, int32_t err_every, double *err_trace) {
  FU_TRY_BEGIN
  if (!h || rounds < 0) return fail(FU_ERR_ARG, "fu_run_collectall: bad arguments");
  if (err_every > 0 && !h->has_target) return fail(FU_ERR_STATE, "fu_run_collectall: err_every > 0 needs fu_set_targets");
  if (int rc = set_device(h)) return rc;
  const int nerr = err_every > 0 ? rounds / err_every : 0;
  if (nerr > 0) {
    if (int rc = fu__err_slots(h, nerr)) return rc;
    HIP_TRY(hipMemsetAsync(h->err, 0, sizeof(unsigned long long) * nerr, h->stream));
  }
  if (int rc = run_rounds(h, rounds, err_every, nerr)) return rc;
  if (nerr > 0) {
    if (h->dist) {
      if (int rc = fu__dist_round_hook(h, 100 + nerr)) return rc;  // all-reduce max, in place
    }
    std::vector<unsigned long long> bits(nerr);
    HIP_TRY(hipMemcpyAsync(bits.data(), h->err, sizeof(unsigned long long) * nerr, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    if (err_trace) std::memcpy(err_trace, bits.data(), sizeof(double) * nerr);
  }
  return FU_OK;
  FU_TRY_END
}

int fu_run_collectall_timed(fu_handle *h, int32_t rounds, float *ms) {
  FU_TRY_BEGIN
  if (!h || !ms || rounds < 0) return fail(FU_ERR_ARG, "fu_run_collectall_timed: bad arguments");
  if (int rc = set_device(h)) return rc;
  HIP_TRY(hipEventRecord(h->ev2, h->stream));
  if (int rc = run_rounds(h, rounds, 0, 0)) return rc;
  HIP_TRY(hipEventRecord(h->ev3, h->stream));
  HIP_TRY(hipEventSynchronize(h->ev3));
  HIP_TRY(hipEventElapsedTime(ms, h->ev2, h->ev3));
  return FU_OK;
  FU_TRY_END
}

int fu_tune(fu_handle *h) {
  FU_TRY_BEGIN
  if (!h) return fail(FU_ERR_ARG, "fu_tune: NULL handle");
  if (!h->autotune) return fail(FU_ERR_STATE, "fu_tune: the kernel is pinned (option kernel != 0)");
  if (int rc = set_device(h)) return rc;
  if (h->rounds == 0)
    if (int rc = launch_round(h, nullptr)) return rc;  // round 0 is not a tuning candidate
  HIP_TRY(hipStreamSynchronize(h->stream));
  poll_pack_width(h);
  const int w = h->pw_pending ? h->tuned_width : *h->h_pw;
  int32_t budget = INT32_MAX;
  if (int rc = autotune_kernel(h, &budget, w)) return rc;
  h->tuned_width = w;
  return FU_OK;
  FU_TRY_END
}

int fu_mark(fu_handle *h, int32_t slot) {
  if (!h || slot < 0 || slot >= 64) return fail(FU_ERR_ARG, "fu_mark: slot must be in [0, 64)");
  if (int rc = set_device(h)) return rc;
  if (!h->marks[slot]) HIP_TRY(hipEventCreate(&h->marks[slot]));
  HIP_TRY(hipEventRecord(h->marks[slot], h->stream));
  return FU_OK;
}

int fu_mark_elapsed(fu_handle *h, int32_t from, int32_t to, float *ms) {
  if (!h || !ms || from < 0 || from >= 64 || to < 0 || to >= 64 || !h->marks[from] || !h->marks[to])
    return fail(FU_ERR_ARG, "fu_mark_elapsed: unrecorded slot");
  if (int rc = set_device(h)) return rc;
  HIP_TRY(hipEventSynchronize(h->marks[to]));
  HIP_TRY(hipEventElapsedTime(ms, h->marks[from], h->marks[to]));
  return FU_OK;
}

int fu_max_err(fu_handle *h, double *out) {
  if (!h || !out) return fail(FU_ERR_ARG, "fu_max_err: NULL argument");
  if (!h->has_target) return fail(FU_ERR_STATE, "fu_max_err: call fu_set_targets first");
  if (int rc = set_device(h)) return rc;
  HIP_TRY(hipMemsetAsync(h->err, 0, sizeof(unsigned long long), h->stream));
  hipLaunchKernelGGL(k_max_err, dim3(std::min(1024u, grid_for(h->n))), dim3(kBlock), 0, h->stream,
                     h->n, cur_a(h), h->target, h->err);
  HIP_TRY(hipGetLastError());
  if (h->dist) {
    if (int rc = fu__dist_round_hook(h, 101)) return rc;  // all-reduce max of slot 0
  }
  unsigned long long bits = 0;
  HIP_TRY(hipMemcpyAsync(&bits, h->err, sizeof(bits), hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  std::memcpy(out, &bits, sizeof(double));
  return FU_OK;
}

int fu_get_estimates(fu_handle *h, double *a_out) {
  if (!h || !a_out) return fail(FU_ERR_ARG, "fu_get_estimates: NULL argument");
  if (int rc = set_device(h)) return rc;
  if (!h->h_new_of_old.empty()) {  // device numbering -> caller numbering
    std::vector<double> a2(h->n);
    HIP_TRY(hipMemcpyAsync(a2.data(), cur_a(h), sizeof(double) * h->n, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    for (int32_t i = 0; i < h->n; ++i) a_out[i] = a2[h->h_new_of_old[i]];
    return FU_OK;
  }
  HIP_TRY(hipMemcpyAsync(a_out, cur_a(h), sizeof(double) * h->n, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return FU_OK;
}

int fu_get_flows(fu_handle *h, double *f_out) {
  if (!h || (!f_out && h->E)) return fail(FU_ERR_ARG, "fu_get_flows: NULL argument");
  if (h->E == 0) return FU_OK;
  if (int rc = set_device(h)) return rc;
  const double *src = cur_f(h);
  if (h->kernel == 3 && h->rounds > 0) {
    if (!h->ftmp) {
      if (int rc = dmalloc(&h->ftmp, (size_t)h->E)) return rc;
    }
    hipLaunchKernelGGL(k_push_flows, dim3(grid_for(h->E)), dim3(kBlock), 0, h->stream, (long long)h->E,
                       h->rev, h->inbox[h->cur], h->ftmp);
    HIP_TRY(hipGetLastError());
    src = h->ftmp;
  } else if (h->kernel >= 4) {  // split words (st_f) -> doubles
    if (!h->ftmp) {
      if (int rc = dmalloc(&h->ftmp, (size_t)h->E)) return rc;
    }
    hipLaunchKernelGGL(k_unsplit, dim3(grid_for(h->E)), dim3(kBlock), 0, h->stream, (long long)h->E, src, h->ftmp);
    HIP_TRY(hipGetLastError());
    src = h->ftmp;
  }
  if (!h->h_new_of_old.empty()) {  // rows back to the caller's order (blocks, same order inside)
    std::vector<double> f2(h->E);
    HIP_TRY(hipMemcpyAsync(f2.data(), src, sizeof(double) * h->E, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    const auto &orp = h->h_orig_rowptr;
    for (int32_t i = 0; i < h->n; ++i) {
      const int64_t nb = h->h_rowptr[h->h_new_of_old[i]];
      std::memcpy(f_out + orp[i], f2.data() + nb, sizeof(double) * (orp[i + 1] - orp[i]));
    }
    return FU_OK;
  }
  HIP_TRY(hipMemcpyAsync(f_out, src, sizeof(double) * h->E, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  return FU_OK;
}

int fu_get_info(fu_handle *h, int64_t info[32]) {
  if (!h || !info) return fail(FU_ERR_ARG, "fu_get_info: NULL argument");
  info[0] = h->kernel;
  info[1] = h->nt;
  info[2] = h->autotune ? (h->tuned ? 2 : 1) : 0;
  info[3] = h->rounds;
  info[4] = kGeoEdges[h->geo];
  info[5] = kGeoNodes[h->geo];
  info[6] = h->n_tunes;
  info[7] = h->tuned_width;
  for (int k = 0; k < 12; ++k) info[8 + k] = (int64_t)(h->tune_ms[k] * 1e3f);  // ns per round
  {  // autotune winner per packing width 0, 8, 16, 32 (kernel * 10 + geometry; -1 = none)
    const std::vector<TuneCand> cands = tune_cands(h);
    for (int k = 0; k < 4; ++k)
      info[23 + k] = h->tune_cache[k] < 0 ? -1 : cands[h->tune_cache[k]].kernel * 10 + cands[h->tune_cache[k]].geo;
  }
  info[20] = h->n_hub;
  info[21] = h->n_piece;
  info[22] = 0;
  if (h->hub_redo) {
    if (int rc = set_device(h)) return rc;
    unsigned long long redo = 0;
    HIP_TRY(hipMemcpyAsync(&redo, h->hub_redo, sizeof(redo), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    info[22] = (int64_t)redo;
  }
  return FU_OK;
}

int fu_get_pack(fu_handle *h, int32_t width[3]) {
  if (!h || !width) return fail(FU_ERR_ARG, "fu_get_pack: NULL argument");
  if (int rc = set_device(h)) return rc;
  PackCtl p[3];
  HIP_TRY(hipMemcpyAsync(p, h->pctl, sizeof(p), hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  for (int k = 0; k < 3; ++k) width[k] = p[k].width;
  return FU_OK;
}

int fu_get_round(fu_handle *h, int64_t *rounds_done) {
  if (!h || !rounds_done) return fail(FU_ERR_ARG, "fu_get_round: NULL argument");
  *rounds_done = h->rounds;
  return FU_OK;
}

int fu_synchronize(fu_handle *h) {
  if (!h) return fail(FU_ERR_ARG, "fu_synchronize: NULL handle");
  if (int rc = set_device(h)) return rc;
  HIP_TRY(hipStreamSynchronize(h->stream));
  return FU_OK;
}

int fu_destroy(fu_handle *h) {
  if (!h) return FU_OK;
  hipSetDevice(h->device);
  if (h->stream) hipStreamSynchronize(h->stream);
  if (h->dist) fu__dist_free(h);
  void *ptrs[] = {h->rowptr, h->col, h->rev, h->v, h->f[0], h->f[1], h->a[0], h->a[1], h->a[2],
                  h->inbox[0], h->inbox[1], h->target, h->err, h->ftmp, h->tiles, h->tiles_geo[0],
                  h->tiles_geo[1], h->tiles_geo[2], h->tiles_geo[3], h->wtiles[0], h->wtiles[1],
                  h->wheavy[0], h->wheavy[1],
                  h->colpm, h->rowptr0, h->G, h->tiles_s, h->tiles_g, h->perm,
                  h->code[0], h->code[1], h->pctl, h->psample, h->st_tiles, h->st_gbase, h->st_heavy,
                  h->stG, h->st[0].aoff, h->st[0].aitem, h->st[0].colS, h->st[0].sidx, h->st[1].aoff,
                  h->st[1].aitem, h->st[1].colS, h->st[1].sidx, h->st[2].aoff, h->st[2].aitem,
                  h->st[2].colS, h->st[2].sidx, h->st[3].aoff, h->st[3].aitem, h->st[3].colS,
                  h->st[3].sidx, h->st[0].gbase, h->st[1].gbase, h->st[2].gbase, h->st[3].gbase,
                  h->hub_rows, h->hub_off, h->hubxy, h->hrows, h->hub_piece, h->hub_p0, h->psum,
                  h->hsum, h->hub_redo, h->st[0].sidx16, h->st[1].sidx16, h->st[2].sidx16,
                  h->st[3].sidx16, h->st[0].dtab, h->st[1].dtab, h->st[2].dtab, h->st[3].dtab};
  for (void *p : ptrs)
    if (p) hipFree(p);
  if (h->ev0) hipEventDestroy(h->ev0);
  if (h->ev1) hipEventDestroy(h->ev1);
  if (h->ev2) hipEventDestroy(h->ev2);
  if (h->ev3) hipEventDestroy(h->ev3);
  if (h->ev_pw) hipEventDestroy(h->ev_pw);
  for (hipEvent_t e : h->marks)
    if (e) hipEventDestroy(e);
  if (h->ev_fork) hipEventDestroy(h->ev_fork);
  if (h->ev_join) hipEventDestroy(h->ev_join);
  if (h->h_pw) hipHostFree(h->h_pw);
  if (h->stream) hipStreamDestroy(h->stream);
  if (h->stream2) hipStreamDestroy(h->stream2);
  delete h;
  return FU_OK;
}

// ======================================================================================
// replay
// ======================================================================================
struct fu_replay {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  int32_t n = 0, ticks = 0, cur_tick = 0;
  int64_t E = 0, n_msgs = 0;
  std::vector<int64_t> h_tto;
  long long *rowptr = nullptr;
  int *tasks = nullptr, *events = nullptr, *out_ids = nullptr;
  double *v = nullptr, *flow = nullptr, *est = nullptr, *last = nullptr;
  double2 *msg = nullptr;
  // persistent mode (built on first use)
  int persistent = 0;
  unsigned pers_blocks = 1;
  std::vector<int32_t> h_tasks, h_events, h_out_ids;
  long long *node_off = nullptr, *cursor = nullptr;
  int4 *node_ev = nullptr;
  int *node_tick = nullptr, *out_uid = nullptr, *scur = nullptr, *status = nullptr;
  unsigned long long *pay = nullptr;
  int64_t n_uid = 0;
  bool pers_ready = false;
};

static int replay_build_persistent(fu_replay *r) {
  if (r->pers_ready) return FU_OK;
  const int32_t n = r->n;
  const int64_t nt = (int64_t)r->h_tasks.size() / 3, ne = (int64_t)r->h_events.size() / 4;
  std::vector<int64_t> off(n + 1, 0);
  for (int64_t q = 0; q < nt; ++q) off[r->h_tasks[3 * q] + 1] += r->h_tasks[3 * q + 2] - r->h_tasks[3 * q + 1];
  for (int32_t i = 0; i < n; ++i) off[i + 1] += off[i];
  std::vector<int64_t> pos(off.begin(), off.end() - 1);
  std::vector<int4> nev(ne > 0 ? ne : 1);
  std::vector<int32_t> ntick(ne > 0 ? ne : 1);
  std::vector<int32_t> ouid(r->h_out_ids.size() > 0 ? r->h_out_ids.size() : 1);
  std::vector<int64_t> slot_uid(r->n_msgs > 0 ? r->n_msgs : 1, -1);
  int64_t U = 0;
  for (int32_t t = 0; t < r->ticks; ++t) {
    for (int64_t q = r->h_tto[t]; q < r->h_tto[t + 1]; ++q) {
      const int32_t node = r->h_tasks[3 * q];
      for (int32_t p = r->h_tasks[3 * q + 1]; p < r->h_tasks[3 * q + 2]; ++p) {
        const int32_t *e = &r->h_events[4 * (int64_t)p];
        int4 o = make_int4(e[0], e[1], e[2], e[3]);
        if (e[0] == FU_EV_RECV) {
          const int64_t u = slot_uid[e[2]];
          if (u < 0) return fail(FU_ERR_ARG, "replay: RECV of a message slot never written");
          o.z = (int)u;
        } else if (e[0] == FU_EV_FIRE_CA) {
          for (int32_t j = 0; j < e[1]; ++j) {
            slot_uid[r->h_out_ids[e[2] + j]] = U;
            ouid[e[2] + j] = (int32_t)U++;
          }
        } else {
          slot_uid[e[3]] = U;
          o.w = (int)U++;
        }
        if (U >= (int64_t)INT32_MAX) return fail(FU_ERR_ALLOC, "replay: more than 2^31 messages");
        nev[pos[node]] = o;
        ntick[pos[node]++] = t;
      }
    }
  }
  r->n_uid = U;
  if (int rc = dmalloc(&r->node_off, n + 1)) return rc;
  if (int rc = dmalloc(&r->node_ev, nev.size())) return rc;
  if (int rc = dmalloc(&r->node_tick, ntick.size())) return rc;
  if (int rc = dmalloc(&r->out_uid, ouid.size())) return rc;
  if (int rc = dmalloc(&r->pay, 2 * (size_t)std::max<int64_t>(U, 1))) return rc;
  if (int rc = dmalloc(&r->cursor, n)) return rc;
  if (int rc = dmalloc(&r->scur, n)) return rc;
  if (int rc = dmalloc(&r->status, 1)) return rc;
  HIP_TRY(hipMemcpy(r->node_off, off.data(), sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(r->node_ev, nev.data(), sizeof(int4) * nev.size(), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(r->node_tick, ntick.data(), sizeof(int32_t) * ntick.size(), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(r->out_uid, ouid.data(), sizeof(int32_t) * ouid.size(), hipMemcpyHostToDevice));
  std::vector<long long> cur(off.begin(), off.end() - 1);
  HIP_TRY(hipMemcpy(r->cursor, cur.data(), sizeof(long long) * n, hipMemcpyHostToDevice));
  HIP_TRY(hipMemset(r->scur, 0, sizeof(int) * n));
  double sentinel;
  std::memcpy(&sentinel, &kMsgSentinel, sizeof(double));
  hipLaunchKernelGGL(k_fill, dim3(grid_for(2 * std::max<int64_t>(U, 1))), dim3(kBlock), 0, r->stream,
                     (long long)(2 * std::max<int64_t>(U, 1)), sentinel, reinterpret_cast<double *>(r->pay));
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(r->stream));
  int per_cu = 0, ncu = 0;
  HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_replay_persist, kBlock, 0));
  HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, r->device));
  // stay below the occupancy bound (the API can over-report by one block per CU)
  const long long cap = std::max(1LL, (long long)std::max(1, per_cu - 1) * ncu);
  r->pers_blocks = (unsigned)std::min<long long>(cap, grid_for(r->n));
  r->pers_ready = true;
  return FU_OK;
}

int fu_replay_create(int32_t n, const int64_t *rowptr, const double *value, int32_t ticks,
                     const int64_t *tick_task_off, int64_t n_tasks, const int32_t *tasks,
                     int64_t n_events, const int32_t *events, int64_t n_out_ids,
                     const int32_t *out_ids, int64_t n_msgs, int32_t device,
                     fu_replay **out) {
  FU_TRY_BEGIN
  if (!out || n <= 0 || !rowptr || !value || ticks < 0 || !tick_task_off || n_tasks < 0 || n_events < 0 ||
      n_out_ids < 0 || n_msgs < 0)
    return fail(FU_ERR_ARG, "fu_replay_create: bad arguments");
  if (tick_task_off[0] != 0 || tick_task_off[ticks] != n_tasks) return fail(FU_ERR_ARG, "fu_replay_create: tick_task_off inconsistent");
  const int64_t E = rowptr[n];
  // validate the trace on the host: every index a kernel will dereference
  for (int64_t q = 0; q < n_tasks; ++q) {
    int32_t node = tasks[3 * q], b = tasks[3 * q + 1], e = tasks[3 * q + 2];
    if (node < 0 || node >= n || b < 0 || e < b || e > n_events) return fail(FU_ERR_ARG, "fu_replay_create: bad task " + std::to_string(q));
    const int64_t deg = rowptr[node + 1] - rowptr[node];
    for (int32_t p = b; p < e; ++p) {
      const int32_t *ev = events + 4 * (int64_t)p;
      bool ok;
      if (ev[0] == FU_EV_RECV) ok = ev[1] >= 0 && ev[1] < deg && ev[2] >= 0 && ev[2] < n_msgs;
      else if (ev[0] == FU_EV_FIRE_CA) ok = ev[1] >= 0 && ev[1] <= deg && ev[2] >= 0 && (int64_t)ev[2] + ev[1] <= n_out_ids;
      else if (ev[0] == FU_EV_FIRE_PW) ok = ev[1] >= 0 && ev[1] < deg && ev[2] > ev[1] && ev[2] <= deg && ev[3] >= 0 && ev[3] < n_msgs;
      else ok = false;
      if (!ok) return fail(FU_ERR_ARG, "fu_replay_create: bad event " + std::to_string(p));
    }
  }
  for (int64_t q = 0; q < n_out_ids; ++q)
    if (out_ids[q] < 0 || out_ids[q] >= n_msgs) return fail(FU_ERR_ARG, "fu_replay_create: bad out_id");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(FU_ERR_HIP, "fu_replay_create: no HIP device visible");
  if (device < 0 || device >= ndev) return fail(FU_ERR_ARG, "fu_replay_create: device out of range");
  auto *r = new fu_replay();
  auto cleanup = [&](int code) { fu_replay_destroy(r); return code; };
  r->device = device;
  r->n = n;
  r->ticks = ticks;
  r->E = E;
  r->n_msgs = n_msgs;
  r->h_tto.assign(tick_task_off, tick_task_off + ticks + 1);
  r->h_tasks.assign(tasks, tasks + 3 * n_tasks);
  r->h_events.assign(events, events + 4 * n_events);
  r->h_out_ids.assign(out_ids, out_ids + n_out_ids);
  if (hipSetDevice(device) != hipSuccess) return cleanup(fail(FU_ERR_HIP, "hipSetDevice failed"));
  if (hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) != hipSuccess) return cleanup(fail(FU_ERR_HIP, "hipStreamCreate failed"));
  if (hipEventCreate(&r->ev0) != hipSuccess || hipEventCreate(&r->ev1) != hipSuccess) return cleanup(fail(FU_ERR_HIP, "hipEventCreate failed"));
  int rc;
  if ((rc = dmalloc(&r->rowptr, n + 1)) || (rc = dmalloc(&r->tasks, 3 * n_tasks)) ||
      (rc = dmalloc(&r->events, 4 * n_events)) || (rc = dmalloc(&r->out_ids, n_out_ids)) ||
      (rc = dmalloc(&r->v, n)) || (rc = dmalloc(&r->flow, E)) || (rc = dmalloc(&r->est, E)) ||
      (rc = dmalloc(&r->last, n)) || (rc = dmalloc(&r->msg, n_msgs)))
    return cleanup(rc);
  static_assert(sizeof(long long) == sizeof(int64_t), "int64");
  if (hipMemcpy(r->rowptr, rowptr, sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice) != hipSuccess ||
      (n_tasks && hipMemcpy(r->tasks, tasks, sizeof(int32_t) * 3 * n_tasks, hipMemcpyHostToDevice) != hipSuccess) ||
      (n_events && hipMemcpy(r->events, events, sizeof(int32_t) * 4 * n_events, hipMemcpyHostToDevice) != hipSuccess) ||
      (n_out_ids && hipMemcpy(r->out_ids, out_ids, sizeof(int32_t) * n_out_ids, hipMemcpyHostToDevice) != hipSuccess) ||
      hipMemcpy(r->v, value, sizeof(double) * n, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(r->flow, 0, sizeof(double) * (E ? E : 1)) != hipSuccess ||
      hipMemset(r->est, 0, sizeof(double) * (E ? E : 1)) != hipSuccess ||
      hipMemset(r->last, 0, sizeof(double) * n) != hipSuccess ||
      hipMemset(r->msg, 0, sizeof(double2) * (n_msgs ? n_msgs : 1)) != hipSuccess)
    return cleanup(fail(FU_ERR_HIP, "fu_replay_create: upload failed"));
  *out = r;
  return FU_OK;
  FU_TRY_END
}

const fu_trace *fu__trace_view(const fu_trace *t, int32_t *n, int32_t *ticks,
                               const int64_t **urowptr, const int64_t **tto,
                               const int32_t **tasks, int64_t *n_tasks,
                               const int32_t **events, int64_t *n_events,
                               const int32_t **out_ids, int64_t *n_out, int64_t *n_msgs);

int fu_replay_create_from_trace(const fu_trace *t, const double *value, int32_t device,
                                fu_replay **out) {
  if (!t) return fail(FU_ERR_ARG, "fu_replay_create_from_trace: NULL trace");
  int32_t n, ticks;
  const int64_t *urp, *tto;
  const int32_t *tasks, *events, *oids;
  int64_t nt, ne, no, nm;
  fu__trace_view(t, &n, &ticks, &urp, &tto, &tasks, &nt, &events, &ne, &oids, &no, &nm);
  return fu_replay_create(n, urp, value, ticks, tto, nt, tasks, ne, events, no, oids, nm, device, out);
}

static int replay_ticks(fu_replay *r, int32_t tick_end, int32_t n_snap, const int32_t *snap_ticks,
                        double *snaps_dev) {
  if (r->persistent) {
    if (r->cur_tick > 0 && !r->pers_ready) return fail(FU_ERR_STATE, "replay: cannot switch to persistent mode mid-run");
    if (int rc = replay_build_persistent(r)) return rc;
    int32_t *d_st = nullptr;
    if (n_snap > 0) {
      if (int rc = dmalloc(&d_st, n_snap)) return rc;
      HIP_TRY(hipMemcpyAsync(d_st, snap_ticks, sizeof(int32_t) * n_snap, hipMemcpyHostToDevice, r->stream));
    }
    HIP_TRY(hipMemsetAsync(r->scur, 0, sizeof(int) * r->n, r->stream));
    HIP_TRY(hipMemsetAsync(r->status, 0, sizeof(int), r->stream));
    hipLaunchKernelGGL(k_replay_persist, dim3(r->pers_blocks), dim3(kBlock), 0, r->stream, r->n, tick_end,
                       r->node_off, r->node_ev, r->node_tick, r->out_uid, r->rowptr, r->v, r->flow,
                       r->est, r->last, r->pay, r->cursor, r->scur, n_snap, d_st, snaps_dev, r->status,
                       (long long)1 << 22);
    HIP_TRY(hipGetLastError());
    int st = 0;
    HIP_TRY(hipMemcpyAsync(&st, r->status, sizeof(int), hipMemcpyDeviceToHost, r->stream));
    HIP_TRY(hipStreamSynchronize(r->stream));
    if (d_st) hipFree(d_st);
    if (st) return fail(FU_ERR_STATE, "replay: persistent kernel hit its iteration bound");
    r->cur_tick = tick_end;
    return FU_OK;
  }
  int32_t si = 0;
  while (si < n_snap && snap_ticks[si] < r->cur_tick) ++si;
  for (int32_t t = r->cur_tick; t < tick_end; ++t) {
    const long long b = r->h_tto[t];
    const int cnt = (int)(r->h_tto[t + 1] - b);
    if (cnt > 0) {
      hipLaunchKernelGGL(k_replay_tick, dim3(grid_for(cnt)), dim3(kBlock), 0, r->stream, b, cnt,
                         r->tasks, r->rowptr, r->events, r->out_ids, r->v, r->flow, r->est,
                         r->last, r->msg);
      HIP_TRY(hipGetLastError());
    }
    while (si < n_snap && snap_ticks[si] == t) {
      HIP_TRY(hipMemcpyAsync(snaps_dev + (int64_t)si * r->n, r->last, sizeof(double) * r->n,
                             hipMemcpyDeviceToDevice, r->stream));
      ++si;
    }
  }
  r->cur_tick = tick_end;
  return FU_OK;
}

int fu_replay_run(fu_replay *r, int32_t tick_end, int32_t n_snap, const int32_t *snap_ticks,
                  double *snaps) {
  if (!r || tick_end < r->cur_tick || tick_end > r->ticks || n_snap < 0 || (n_snap > 0 && (!snap_ticks || !snaps)))
    return fail(FU_ERR_ARG, "fu_replay_run: bad arguments");
  for (int32_t k = 1; k < n_snap; ++k)
    if (snap_ticks[k] <= snap_ticks[k - 1]) return fail(FU_ERR_ARG, "fu_replay_run: snap_ticks must be ascending");
  HIP_TRY(hipSetDevice(r->device));
  double *d_snaps = nullptr;
  if (n_snap > 0) {
    if (int rc = dmalloc(&d_snaps, (size_t)n_snap * r->n)) return rc;
    hipMemsetAsync(d_snaps, 0, sizeof(double) * n_snap * r->n, r->stream);
  }
  int rc = replay_ticks(r, tick_end, n_snap, snap_ticks, d_snaps);
  if (rc == FU_OK && n_snap > 0) {
    if (hipMemcpyAsync(snaps, d_snaps, sizeof(double) * n_snap * r->n, hipMemcpyDeviceToHost, r->stream) != hipSuccess)
      rc = fail(FU_ERR_HIP, "fu_replay_run: snapshot copy failed");
  }
  if (hipStreamSynchronize(r->stream) != hipSuccess && rc == FU_OK) rc = fail(FU_ERR_HIP, "fu_replay_run: sync failed");
  if (d_snaps) hipFree(d_snaps);
  return rc;
}

int fu_replay_run_timed(fu_replay *r, int32_t tick_end, float *ms) {
  if (!r || !ms || tick_end < r->cur_tick || tick_end > r->ticks) return fail(FU_ERR_ARG, "fu_replay_run_timed: bad arguments");
  HIP_TRY(hipSetDevice(r->device));
  HIP_TRY(hipEventRecord(r->ev0, r->stream));
  if (int rc = replay_ticks(r, tick_end, 0, nullptr, nullptr)) return rc;
  HIP_TRY(hipEventRecord(r->ev1, r->stream));
  HIP_TRY(hipEventSynchronize(r->ev1));
  HIP_TRY(hipEventElapsedTime(ms, r->ev0, r->ev1));
  return FU_OK;
}

int fu_replay_get(fu_replay *r, double *last_avg, double *flows, double *est) {
  if (!r) return fail(FU_ERR_ARG, "fu_replay_get: NULL replay");
  HIP_TRY(hipSetDevice(r->device));
  if (last_avg) HIP_TRY(hipMemcpyAsync(last_avg, r->last, sizeof(double) * r->n, hipMemcpyDeviceToHost, r->stream));
  if (flows && r->E) HIP_TRY(hipMemcpyAsync(flows, r->flow, sizeof(double) * r->E, hipMemcpyDeviceToHost, r->stream));
  if (est && r->E) HIP_TRY(hipMemcpyAsync(est, r->est, sizeof(double) * r->E, hipMemcpyDeviceToHost, r->stream));
  HIP_TRY(hipStreamSynchronize(r->stream));
  return FU_OK;
}

int fu_replay_set_option(fu_replay *r, const char *key, int64_t value) {
  if (!r || !key) return fail(FU_ERR_ARG, "fu_replay_set_option: NULL argument");
  if (!std::strcmp(key, "persistent")) {
    if (r->cur_tick != 0) return fail(FU_ERR_STATE, "fu_replay_set_option: persistent must be set before the first tick");
    r->persistent = value != 0;
    if (!r->persistent) return FU_OK;
    // build the per-node event lists now, so that no host work lands inside a timed run
    HIP_TRY(hipSetDevice(r->device));
    return replay_build_persistent(r);
  }
  return fail(FU_ERR_ARG, std::string("fu_replay_set_option: unknown key '") + key + "'");
}

int fu_replay_destroy(fu_replay *r) {
  if (!r) return FU_OK;
  hipSetDevice(r->device);
  if (r->stream) hipStreamSynchronize(r->stream);
  void *ptrs[] = {r->rowptr, r->tasks, r->events, r->out_ids, r->v, r->flow, r->est, r->last, r->msg,
                  r->node_off, r->cursor, r->node_ev, r->node_tick, r->out_uid, r->scur, r->status, r->pay};
  for (void *p : ptrs)
    if (p) hipFree(p);
  if (r->ev0) hipEventDestroy(r->ev0);
  if (r->ev1) hipEventDestroy(r->ev1);
  if (r->stream) hipStreamDestroy(r->stream);
  delete r;
  return FU_OK;
}

}  // extern "C"

// Accessors for fu_dist.hip (fu_handle's layout stays private to this file).
extern "C" {
void *fu__handle_dist(fu_handle *h) { return h->dist; }
void fu__handle_set_dist(fu_handle *h, void *d) { h->dist = d; }
hipStream_t fu__handle_stream(fu_handle *h) { return h->stream; }
double *fu__handle_f(fu_handle *h, int which) { return h->f[which]; }
double *fu__handle_a(fu_handle *h, int which) { return h->a[which]; }
int fu__handle_cur(fu_handle *h) { return h->cur; }
unsigned long long *fu__handle_err(fu_handle *h) { return h->err; }
int fu__handle_device(fu_handle *h) { return h->device; }
double *fu__handle_cur_a(fu_handle *h) { return cur_a(h); }
double *fu__handle_cur_f(fu_handle *h) { return cur_f(h); }
int fu__handle_kernel(fu_handle *h) { return h->kernel; }
}
