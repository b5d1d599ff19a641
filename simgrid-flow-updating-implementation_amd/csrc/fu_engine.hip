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
#include <hip/hip_ext.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "fu_common.h"
#include "fu_plan.h"

using namespace fu;
namespace FP = fu::plan;

#define HIP_TRY(expr)                                                                     \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess)                                                                 \
      return fu::fail(FU_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));     \
  } while (0)

namespace {

// row-class and table constants shared with the host plans (fu_plan.h)
using FP::kGeoEdges;
using FP::kGeoNodes;
using FP::kHeavyRL;
using FP::kMidRL;
using FP::kMR;
using FP::kR0E;
using FP::kStageLds;
using FP::kStageRuns;
using FP::kStageTE;
using FP::kStageTN;
using FP::kTrBE;
using FP::kTrMaxP;

constexpr int kBlock = 256;      // threads per block (4 waves of 64)
static_assert(kBlock == FP::kHubBlk, "k_hub_stage / k_hub_flows blocks follow the plan's hub table");
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
// a_0 (the timeout fire on zero state) into A[0]; a_{-1} = 0.0 into A[2] (na slots, ghosts
// included); the three packing slots cleared (no codes yet)
__global__ __launch_bounds__(kBlock) void k_round0(int n, int na, const int *__restrict__ rowptr,
                                                   const double *__restrict__ v, double *__restrict__ a,
                                                   double *__restrict__ a_m1, unsigned long long *__restrict__ pctl) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i < 6) pctl[i] = 0ull;  // 3 x 16-byte PackCtl
  if (i < na) a_m1[i] = 0.0;
  if (i >= n) return;
  a[i] = ((v[i] - 0.0) + 0.0) / (double)(rowptr[i + 1] - rowptr[i] + 1);
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

// Round outputs (flows, estimates, codes) use plain write-back stores. Write-through (sc1)
// stores, so that no dirty lines wait for the launch boundary's L2 writeback, were measured
// in round 2 and removed: on ER-1M kernel 4 lost 4.5 us per round and kernel 8 gained nothing.

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
  if (pc.width == 8) *(reinterpret_cast<unsigned char *>(tab) + i) = (unsigned char)cd;
  else if (pc.width == 16) *(reinterpret_cast<unsigned short *>(tab) + i) = (unsigned short)cd;
  else *(reinterpret_cast<unsigned *>(tab) + i) = cd;
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

// NT threads (every lane in flight: kPlanSamples / NT sample loads, then as many gathers).
// pw_host (pinned host memory, or null) receives the width for the autotuner's poll, so no
// copy sits on the round's stream.
template <int NT>
__device__ __forceinline__ void plan_body(const double *__restrict__ a, const int *__restrict__ sample,
                                          PackCtl *ctl, int *pw_host) {
  constexpr int kPer = kPlanSamples / NT;
  __shared__ unsigned long long s_centre;
  __shared__ int s_cnt[3];
  const int t = threadIdx.x;
  if (t < 3) s_cnt[t] = 0;
  int idx[kPer];
  unsigned long long key[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) idx[k] = sample[t + k * NT];  // all loads in flight
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
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {  // wave sums, then one LDS add per wave
    n8 += __shfl_xor(n8, o, 64);
    n16 += __shfl_xor(n16, o, 64);
    n32 += __shfl_xor(n32, o, 64);
  }
  if ((t & 63) == 0) {
    atomicAdd(&s_cnt[0], n8);
    atomicAdd(&s_cnt[1], n16);
    atomicAdd(&s_cnt[2], n32);
  }
  __syncthreads();
  if (t == 0) {
    const int need = kPlanSamples - kPlanSamples / 200;
    const int w = s_cnt[0] >= need ? 8 : s_cnt[1] >= need ? 16 : s_cnt[2] >= need ? 32 : 0;
    PackCtl p;
    p.base = w ? c - (1ull << (w - 1)) : 0;
    p.width = w;
    p.pad = 0;
    ctl[2] = p;
    if (pw_host) *pw_host = w;
  }
}

__global__ __launch_bounds__(kBlock) void k_pack_plan(const double *__restrict__ a,
                                                      const int *__restrict__ sample,
                                                      PackCtl *__restrict__ ctl, int *pw_host) {
  plan_body<kBlock>(a, sample, ctl, pw_host);
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
// (non-temporal flow loads, stores or both measured slower again in round 5: ER-1M kernel 8
// +1.4 / +1.2 / +3.2 %, R-MAT-24 +1.2 / +8.9 / +11 %, profiles/r05/p)
__device__ __forceinline__ double ld_f(const double *F, int e) {
  const unsigned *w = reinterpret_cast<const unsigned *>(F);
  const long long i = fhi_idx(e);
  return __hiloint2double((int)w[i], (int)w[i + 32]);
}
__device__ __forceinline__ void st_fw(unsigned *p, unsigned v) { *p = v; }
// store f_r over f_old (the value the slot held)
__device__ __forceinline__ void st_f(double *F, int e, double v, double f_old) {
  unsigned *w = reinterpret_cast<unsigned *>(F);
  const long long i = fhi_idx(e);
  st_fw(w + i + 32, (unsigned)__double2loint(v));
  if (__double2hiint(v) != __double2hiint(f_old)) st_fw(w + i, (unsigned)__double2hiint(v));
}
__device__ __forceinline__ void st_f_full(double *F, int e, double v) {
  unsigned *w = reinterpret_cast<unsigned *>(F);
  const long long i = fhi_idx(e);
  st_fw(w + i + 32, (unsigned)__double2loint(v));
  st_fw(w + i, (unsigned)__double2hiint(v));
}

// Flow mode of a round launch (fm): round 0 writes no flows at all. f_{r-2} of round 1 is
// f_{-1} = -0.0 and f_{r-2} of round 2 is f_0 = (0.0 + a_0[i]) - 0.0 (CA:117 on zero state),
// a per-row constant of a_{r-2}[i] = own2, so rounds 1 and 2 compute the old flow instead of
// reading it (fm = 1, 2; fm = 0: read F) and store both words of the new one (the slot holds
// no earlier value). fu_get_flows after round 0 materialises f_0 (k_round0_flows).
__device__ __forceinline__ double old_flow(int fm, double own2) { return fm == 1 ? -0.0 : (0.0 + own2) - 0.0; }
__device__ __forceinline__ double ld_fo(const double *F, int e, int fm, double own2) {
  return fm == 0 ? ld_f(F, e) : old_flow(fm, own2);
}
__device__ __forceinline__ void st_fo(double *F, int e, double v, double f_old, int fm) {
  if (fm) st_f_full(F, e, v);
  else st_f(F, e, v, f_old);
}

// Round 0's flows, one thread per edge: f_0[e] = (0.0 + a_0[row]) - 0.0 into F[0]
// (CA:117 on zero state) and, if F1 is given, f_{-1} = -0.0 into F[1] (split words). The
// rounds never need them (fm above); fu_get_flows after round 0 does. A block owns kR0E consecutive edges: the host
// listed the row of every block's first edge (blk_row), the block's rows' pointers go to
// LDS, and each edge's row is a short binary search there (a hub's edges all land in one
// row; a block whose rows span more than kR0E, runs of isolated nodes, searches rowptr).
__global__ __launch_bounds__(kBlock) void k_round0_flows(long long E, const int *__restrict__ rowptr,
                                                         const int *__restrict__ blk_row,
                                                         const double *__restrict__ a, double *__restrict__ F0,
                                                         double *__restrict__ F1) {
  __shared__ int s_r[2];
  __shared__ int s_rp[kR0E + 1];
  const long long e0 = (long long)blockIdx.x * kR0E;
  const int t = threadIdx.x;
  if (t < 2) s_r[t] = blk_row[blockIdx.x + t];  // rows holding edges e0 and e0 + kR0E (host)
  __syncthreads();
  const int r0 = s_r[0], span = s_r[1] - s_r[0] + 1;
  const bool lds = span <= kR0E;
  if (lds)
    for (int q = t; q <= span; q += kBlock) s_rp[q] = rowptr[r0 + q];
  __syncthreads();
  // thread t: edges k0 .. k0 + 3, 4-aligned, so each split-word store is one 16-byte lane store
  const long long k0 = e0 + 4 * t;
  if (k0 >= E) return;
  auto rp = [&](int q) { return lds ? s_rp[q] : rowptr[r0 + q]; };
  int lo = 0, hi = span - 1;  // row of k0 relative to r0
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (rp(mid) <= k0) lo = mid; else hi = mid - 1;
  }
  unsigned hw[4], lw[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const long long k = k0 + u;
    while (lo + 1 < span && rp(lo + 1) <= k) ++lo;  // next rows (empty ones skipped)
    const double fv = k < E ? (0.0 + a[r0 + lo]) - 0.0 : 0.0;
    hw[u] = (unsigned)__double2hiint(fv);
    lw[u] = (unsigned)__double2loint(fv);
  }
  // split words: block k / 32 holds 32 high words, then 32 low words; E is padded to whole
  // 32-edge blocks in F, so the tail lanes write padding
  const long long j = ((k0 & ~31LL) << 1) | (k0 & 31);
  unsigned *w0 = reinterpret_cast<unsigned *>(F0), *w1 = reinterpret_cast<unsigned *>(F1);
  *reinterpret_cast<uint4 *>(w0 + j) = make_uint4(hw[0], hw[1], hw[2], hw[3]);
  *reinterpret_cast<uint4 *>(w0 + j + 32) = make_uint4(lw[0], lw[1], lw[2], lw[3]);
  if (!F1) return;
  const unsigned mh = (unsigned)__double2hiint(-0.0), ml = (unsigned)__double2loint(-0.0);
  *reinterpret_cast<uint4 *>(w1 + j) = make_uint4(mh, mh, mh, mh);
  *reinterpret_cast<uint4 *>(w1 + j + 32) = make_uint4(ml, ml, ml, ml);
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
// of one batch cover the LDS latency of the next), into two register batches used in turn
// (no register copies: those cost two more VALU instructions per element). The caller
// keeps xs and es in different LDS banks (es = xs + 8 TE + 8 bytes in the tiles), so the
// two addresses of one read do not conflict.
template <int B = kChainB>
__device__ __forceinline__ void chain_sum(const double *xs, const double *es, int cn, double &S, double &T) {
  const bool odd = threadIdx.x & 1;
  const double *src = odd ? es : xs;
  double acc = odd ? T : S;
  int q = 0;
  if (cn >= B) {
    double a[B], c[B];
#pragma unroll
    for (int k = 0; k < B; ++k) a[k] = src[k];
    q = B;
    for (;;) {
      if (q + B > cn) {
#pragma unroll
        for (int k = 0; k < B; ++k) acc = acc + a[k];
        break;
      }
#pragma unroll
      for (int k = 0; k < B; ++k) c[k] = src[q + k];
#pragma unroll
      for (int k = 0; k < B; ++k) acc = acc + a[k];
      q += B;
      if (q + B > cn) {
#pragma unroll
        for (int k = 0; k < B; ++k) acc = acc + c[k];
        break;
      }
#pragma unroll
      for (int k = 0; k < B; ++k) a[k] = src[q + k];
#pragma unroll
      for (int k = 0; k < B; ++k) acc = acc + c[k];
      q += B;
    }
  }
  for (; q < cn; ++q) acc = acc + src[q];
  S = __shfl(acc, 0);
  T = __shfl(acc, 1);
}


// Heavy rows (one per wave) up to 64 x max(kHeavyRL, chunk / 64) edges keep their operands
// in registers (measured on R-MAT-24: 8 or 16 per lane cost more in occupancy than the
// second pass they save).
// kernel 9's second heavy launch: rows of 64 x (kHeavyRL, kMidRL] edges keep their operands
// in registers (no second pass over the row for its flows), at a lower occupancy than the
// other heavy rows can afford (R-MAT-24: 19 % of the edges sit in rows of 641-1024)

// PRE (kernel 9): every edge's estimate a_{r-1}[col e] was pre-gathered into Gb[e] (edge
// order) by the two staging passes; the tile reads it coalesced instead of col + gather.
template <bool CHECK, int TE = kTileEdges, int TN = kTileNodes, int PART = 0,
          bool PRE = false, int HRL = kHeavyRL, bool RF = true>
__global__ __launch_bounds__(kBlock, (HRL > kHeavyRL ? 3 : 1)) void k_round_recon(
    const int4 *__restrict__ tiles, const int *__restrict__ rowptr,
    const int *__restrict__ col, const double *__restrict__ v, double *__restrict__ F,
    const double *__restrict__ a_prev, const double *__restrict__ a_prev2,
    double *__restrict__ a_new, const double *__restrict__ target,
    unsigned long long *__restrict__ err,
    const void *__restrict__ code_prev, void *__restrict__ code_new, PackCtl *__restrict__ ctl,
    int rslot, const double2 *__restrict__ hubxy, const int *__restrict__ hub_off,
    const int *__restrict__ hrows, int hub_sep, const double *__restrict__ Gb, int fm,
    const unsigned short *__restrict__ col16 = nullptr, const int *__restrict__ cbase = nullptr,
    const int *__restrict__ tnar = nullptr) {
  static_assert(TE % kBlock == 0 && TN <= kBlock && TN <= 256, "tile geometry");
  const PackCtl pp = ctl[rslot ^ 1];  // packing of a_{r-1} (the table gathered here)
  const PackCtl pc = ctl[2];          // packing of a_r (the table written here)
  if (blockIdx.x == 0 && threadIdx.x == 0) ctl[rslot] = pc;
  __shared__ double s_x[TE];   // f_{r-2} on load, fr after phase B
  __shared__ double s_er_buf[TE + 2];  // a_{r-1}[col e], one double off s_x's banks
  double *const s_er = s_er_buf + 1;
  __shared__ unsigned char s_own[TE];
  __shared__ int s_rp[TN + 1];
  __shared__ double s_a[TN];
  const int t = threadIdx.x;
  const int4 tl = tiles[blockIdx.x];
  unsigned long long eb = 0;


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
      constexpr int RL = HRL > PL ? HRL : PL;  // whole chunks (TE 2048: PL = 8)
      if (d <= 64 * RL) {
        // the whole row in registers (RL elements per lane, all loads in flight at
        // once): the chain runs chunk by chunk through the wave's LDS quarter and the flows
        // are written from the same registers, with no second pass over the row
        double fo[RL], er[RL];
        int cc[RL];
#pragma unroll
        for (int u = 0; u < RL; ++u) {
          const int k = lane + 64 * u;
          if constexpr (PRE) er[u] = k < d ? Gb[b + k] : 0.0;
          else cc[u] = k < d ? col[b + k] : 0;
          fo[u] = k < d ? ld_fo(F, b + k, fm, own2) : 0.0;
        }
        if constexpr (!PRE) {
#pragma unroll
          for (int u = 0; u < RL; ++u) er[u] = lane + 64 * u < d ? ld_est(pp, code_prev, a_prev, cc[u]) : 0.0;
        }
#pragma unroll
        for (int c = 0; c < RL / PL; ++c) {
          if (c * CH < d) {
            wave_sync();  // the previous chunk's chain is done with the buffer
#pragma unroll
            for (int j = 0; j < PL; ++j) {
              xs[lane + 64 * j] = recon_fr(fo[c * PL + j], er[c * PL + j], own2);
              es[lane + 64 * j] = er[c * PL + j];
            }
            wave_sync();
            // the register-resident mid launch: 8-element batches (its rows hold 64 VGPRs)
            chain_sum<(HRL > kHeavyRL ? 8 : kChainB)>(xs, es, min(CH, d - c * CH), S, T);
          }
        }
        const double a = ((v[i] - S) + T) / (double)(d + 1);
        if (lane == 0) {
          *(a_new + i) = a;
          if (pc.width) put_code(pc, code_new, i, a);
          if (CHECK) eb = err_bits(a, target[i]);
        }
#pragma unroll
        for (int u = 0; u < RL; ++u) {  // flows (CA:117-118)
          const int k = lane + 64 * u;
          if (k < d) st_fo(F, b + k, (recon_fr(fo[u], er[u], own2) + a) - er[u], fo[u], fm);
        }
      } else {
      // longer rows: chunk by chunk, the next chunk's loads in flight during this chunk's
      // chain; the flows in a second pass
      double fo[PL], er[PL], nf[PL], ng[PL];
      int nc[PL];
      auto fetch = [&](int c0) {
#pragma unroll
        for (int u = 0; u < PL; ++u) {
          const int k = c0 + lane + 64 * u;
          if constexpr (PRE) ng[u] = k < d ? Gb[b + k] : 0.0;
          else nc[u] = k < d ? col[b + k] : 0;
          nf[u] = k < d ? ld_fo(F, b + k, fm, own2) : 0.0;
        }
      };
      fetch(0);
      for (int c0 = 0; c0 < d; c0 += CH) {
#pragma unroll
        for (int u = 0; u < PL; ++u) {
          fo[u] = nf[u];
          if constexpr (PRE) er[u] = ng[u];
          else er[u] = c0 + lane + 64 * u < d ? ld_est(pp, code_prev, a_prev, nc[u]) : 0.0;
        }
        if (c0 + CH < d) fetch(c0 + CH);
        wave_sync();  // the previous chunk's chain is done with the buffer
#pragma unroll
        for (int u = 0; u < PL; ++u) {
          xs[lane + 64 * u] = recon_fr(fo[u], er[u], own2);
          es[lane + 64 * u] = er[u];
        }
        wave_sync();
        chain_sum(xs, es, min(CH, d - c0), S, T);
      }
      const double a = ((v[i] - S) + T) / (double)(d + 1);
      if (lane == 0) {
        *(a_new + i) = a;
        if (pc.width) put_code(pc, code_new, i, a);
        if (CHECK) eb = err_bits(a, target[i]);
      }
      for (int k0 = 0; k0 < d; k0 += 8 * 64) {  // flows (CA:117-118), 8 loads in flight per lane
        int cc[8];
        double fo[8], er[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int k = k0 + lane + 64 * u;
          if constexpr (PRE) er[u] = k < d ? Gb[b + k] : 0.0;
          else cc[u] = k < d ? col[b + k] : 0;
          fo[u] = k < d ? ld_fo(F, b + k, fm, own2) : 0.0;
        }
        if constexpr (!PRE) {
#pragma unroll
          for (int u = 0; u < 8; ++u)
            er[u] = k0 + lane + 64 * u < d ? ld_est(pp, code_prev, a_prev, cc[u]) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int k = k0 + lane + 64 * u;
          if (k < d) st_fo(F, b + k, (recon_fr(fo[u], er[u], own2) + a) - er[u], fo[u], fm);
        }
      }
      }  // rows longer than 64 x kHeavyRL
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
    const double2 *xy = PRE ? nullptr : hubxy + hub_off[blockIdx.x];
    const int d = e - b;
    double S = 0.0, T = 0.0;
    constexpr int CH = TE / 2, PL = CH / 64;  // pairs per chunk, per lane
    if (PRE && t < 64) {
      // kernel 9: the row's estimates are pre-gathered (Gb), so the chain wave streams Gb
      // and the old flows itself, coalesced, and rebuilds fr as k_hub_stage would
      const double own2 = a_prev2[i];
      double nf[PL], ng[PL];
#pragma unroll
      for (int u = 0; u < PL; ++u) {
        const int k = t + 64 * u;
        nf[u] = k < d ? ld_fo(F, b + k, fm, own2) : 0.0;
        ng[u] = k < d ? Gb[b + k] : 0.0;
      }
      for (int c0 = 0; c0 < d; c0 += CH) {
        double *xs = s_x + ((c0 / CH) & 1) * CH, *es = s_er + ((c0 / CH) & 1) * CH;
#pragma unroll
        for (int u = 0; u < PL; ++u) {
          xs[t + 64 * u] = recon_fr(nf[u], ng[u], own2);
          es[t + 64 * u] = ng[u];
        }
        const int c1 = c0 + CH;
#pragma unroll
        for (int u = 0; u < PL; ++u) {
          const int k = c1 + t + 64 * u;
          nf[u] = k < d ? ld_fo(F, b + k, fm, own2) : 0.0;
          ng[u] = k < d ? Gb[b + k] : 0.0;
        }
        wave_sync();
        chain_sum(xs, es, min(CH, d - c0), S, T);
        wave_sync();
      }
    } else if (!PRE && t < 64) {
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
        chain_sum(xs, es, min(CH, d - c0), S, T);
        wave_sync();
      }
    }
    if (t == 0) {
      const double a = ((v[i] - S) + T) / (double)(d + 1);
      s_a[0] = a;
      *(a_new + i) = a;
      if (pc.width) put_code(pc, code_new, i, a);
      if (CHECK) eb = err_bits(a, target[i]);
    }
    if (!PRE && !hub_sep) {  // else k_hub_flows writes the row's flows with many blocks
      __syncthreads();
      const double a = s_a[0];
      for (int k = t; k < d; k += kBlock) {
        const double2 p2 = xy[k];
        st_fo(F, b + k, (p2.x + a) - p2.y, fm ? 0.0 : ld_f(F, b + k), fm);
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
        const double er = PRE ? Gb[c0 + q] : ld_est(pp, code_prev, a_prev, col[c0 + q]);
        xs[q] = recon_fr(ld_fo(F, c0 + q, fm, own2), er, own2);
        es[q] = er;
      }
    };
    if (nch > 0) stage(0, t, kBlock);
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
      if (t >= 64) {
        if (c + 1 < nch) stage(c + 1, t - 64, kBlock - 64);
      } else {
        chain_sum(s_x + (c & 1) * CH, s_er + (c & 1) * CH, min(CH, e - (b + c * CH)), S, T);
      }
      __syncthreads();
    }
    if (t == 0) {
      const double a = ((v[i] - S) + T) / (double)(e - b + 1);
      s_a[0] = a;
      *(a_new + i) = a;
      if (pc.width) put_code(pc, code_new, i, a);
      if (CHECK) eb = err_bits(a, target[i]);
    }
    __syncthreads();
    const double a = s_a[0];
    for (int k = b + t; k < e; k += kBlock) {
      const double er = PRE ? Gb[k] : ld_est(pp, code_prev, a_prev, col[k]);
      const double fo = ld_fo(F, k, fm, own2);
      st_fo(F, k, (recon_fr(fo, er, own2) + a) - er, fo, fm);
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
  int rp, rp_last = 0;
  double vv, own2;
  if constexpr (PRE) {
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int q = t + k * kBlock;
      c[k] = 0;
      x[k] = 0.0;
      g[k] = 0.0;
      if (q < ne) {
        g[k] = Gb[e0 + q];
        x[k] = fm ? 0.0 : ld_f(F, e0 + q);
      }
    }
    rp = t <= nn ? rowptr[nb + t] : 0;
    if constexpr (TN == kBlock) rp_last = (t == 0 && nn == kBlock) ? rowptr[nb + kBlock] : 0;
    vv = t < nn ? v[nb + t] : 0.0;
    own2 = t < nn ? a_prev2[nb + t] : 0.0;
  } else {
    // the column indices first, then the flows (RF: round >= 3) and node words, every load
    // unconditional from a clamped index (col and F hold at least one element / 32-edge
    // block), so the gathers wait for the indices alone (in-order completion, vmcnt(N))
    // narrow tiles (tnar: every 1024-edge block of the tile has its columns within 32K ids of
    // the block's first row, cbase): a 2-byte offset per edge instead of the 4-byte column.
    // The column is formed after the flow and node loads are issued (below), so those stay
    // in flight while the gathers wait for the indices.
    const bool narrow = tnar && tnar[blockIdx.x];
    int cw[kPer], bs[kPer];
    if (narrow) {
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        const int q = t + k * kBlock;
        const int ci = q < ne ? e0 + q : (ne > 0 ? e0 : 0);
        cw[k] = col16[ci];
        bs[k] = cbase[ci >> 10];
      }
    } else {
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        const int q = t + k * kBlock;
        const int ci = q < ne ? e0 + q : (ne > 0 ? e0 : 0);
        cw[k] = col[ci];
        bs[k] = 32768;
      }
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) g[k] = 0.0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int q = t + k * kBlock;
      if constexpr (RF) {
        const double f = ld_f(F, q < ne ? e0 + q : 0);
        x[k] = q < ne ? f : 0.0;
      } else {
        x[k] = 0.0;
      }
    }
    const int tn = min(t, nn - 1);  // a light tile has at least one node
    const int rp0 = rowptr[nb + min(t, nn)];
    const double v0 = v[nb + tn], o0 = a_prev2[nb + tn];
    int rl0 = 0;
    if constexpr (TN == kBlock) rl0 = rowptr[nb + nn];  // the tile's end (256-node tiles)
    asm volatile("" ::: "memory");  // the loads above are issued before the first wait
    rp = t <= nn ? rp0 : 0;
    if constexpr (TN == kBlock) rp_last = (t == 0 && nn == kBlock) ? rl0 : 0;
    vv = t < nn ? v0 : 0.0;
    own2 = t < nn ? o0 : 0.0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) c[k] = t + k * kBlock < ne ? bs[k] + cw[k] - 32768 : 0;
  }
  if (PRE) {
  } else if (pp.width == 0) {
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int q = t + k * kBlock;
      g[k] = q < ne ? a_prev[c[k]] : 0.0;
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
    const double fo0 = fm ? old_flow(fm, own2) : 0.0;
    for (int q = qb; q < qe; ++q) {
      const double er = s_er[q];
      const double fr = recon_fr(fm ? fo0 : s_x[q], er, own2);
      s_x[q] = fr;
      s_own[q] = (unsigned char)t;
      S = S + fr;
      T = T + er;
    }
    const double a = ((vv - S) + T) / (double)(qe - qb + 1);
    s_a[t] = a;
    *(a_new + nb + t) = a;
    if (pc.width) put_code(pc, code_new, nb + t, a);
    if (CHECK) eb = err_bits(a, target[nb + t]);
  }
  __syncthreads();
  // phase C: new flows, coalesced, in place (CA:117-118)
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int q = t + k * kBlock;
    if (q < ne) {
      st_fo(F, e0 + q, (s_x[q] + s_a[s_own[q]]) - s_er[q], x[k], fm);
    }
  }
  if (CHECK) block_max_to(eb, err);
  }  // PART != 2
}

// ------------------------------------------------------------------------------------
// Kernel 8, "stage": LDS-staged slices. The a_{r-1}[col e] gather is the part of a round
// that does not stream: on ER every gather is a random L2 request (8 M per round), and the
// fp64 table (8 MB) does not fit an XCD's 4 MB L2. Kernel 8 splits a round into two launches:
//   * k_stage: the estimate table (codes, or doubles while unpacked) is cut into slices of
//     128 KB. A block copies slice s into LDS, then streams a contiguous range of the
//     slice's column offsets (u16) and writes the looked-up elements to G: coalesced reads,
//     16-byte lane-contiguous stores, random accesses only in LDS. G is slice-major: slice
//     s's region holds, tile by tile, the edges whose neighbour lies in slice s.
//   * k_round_staged: kernel 4's light tile (flow reconstruction, CA:98-99 + CA:105-128)
//     where each edge's estimate comes from G: the tile's edges of one slice are one
//     contiguous run of G, found through a u16 {position in the tile, run} per edge and
//     the tile's per-run offsets.
// One layout per table element width (1, 2, 4, 8 bytes; slice = 128 KB / width nodes). The
// device picks the layout from the table's actual packing width; a table wider than the
// layout is read from global memory by the stage launch, so correctness never depends on
// the host's view of the asynchronous packing plan. Rows above the tile limit run as
// kernel 4 heavy tiles in a launch of their own. Results are bitwise those of kernel 4.
// ------------------------------------------------------------------------------------
constexpr int kStageThreads = 1024;   // one block per CU (the slice takes 128 KB of its LDS)

struct StageArgs {
  int P[4], Q[4], SN[4], NB[4];        // slices, blocks per slice, nodes per slice, blocks
  const int4 *brange[4];               // per stage block: {begin, end} in G, slice, 0
  const unsigned short *colS[4];       // per G element: column offset in its slice (pads: 0)
  const unsigned short *sidx16[4];     // per light-tile edge, slice order: position | run << 10
  const int *dtab[4];                  // per light tile: kStageRuns x (G index - m) of each run
  int sel[4];                          // layout used for tables of width 8, 16, 32, 0
  int f64;                             // kernel 9: always stage the doubles (layout 3)
};
__device__ __forceinline__ int width_index(int width) {
  return width == 8 ? 0 : width == 16 ? 1 : width == 32 ? 2 : 3;
}

// EPL consecutive u16 column offsets (EPL = 16 / sizeof(T): one 16-byte G store per lane)
template <int EPL>
struct ColVec {
  uint4 w[EPL > 8 ? 2 : 1];
};
template <int EPL>
__device__ __forceinline__ void ld_cols(ColVec<EPL> &c, const unsigned short *p) {
  if constexpr (EPL == 2) c.w[0].x = *reinterpret_cast<const unsigned *>(p);
  else if constexpr (EPL == 4) {
    const uint2 v = *reinterpret_cast<const uint2 *>(p);
    c.w[0].x = v.x;
    c.w[0].y = v.y;
  } else if constexpr (EPL == 8) c.w[0] = *reinterpret_cast<const uint4 *>(p);
  else {
    c.w[0] = reinterpret_cast<const uint4 *>(p)[0];
    c.w[1] = reinterpret_cast<const uint4 *>(p)[1];
  }
}
template <int EPL>
__device__ __forceinline__ unsigned col_at(const ColVec<EPL> &c, int j) {
  const unsigned w = (&c.w[j >> 3].x)[(j >> 1) & 3];
  return (j & 1) ? w >> 16 : w & 0xFFFFu;
}

// Per lane per step: EPL = 16 / sizeof(T) elements, one lane-contiguous 16-byte G store.
// Steps per batch: enough that every lane keeps 64 B of column loads in flight whatever the
// element width (4 steps of 4-byte loads for doubles left 16 KB in flight per CU, ~2 TB/s at
// HBM latency).
template <typename T>
struct StageU {
  static constexpr int EPL = 16 / (int)sizeof(T);
  static constexpr int U = EPL >= 8 ? kStageU : kStageU * 8 / EPL;
};

// One batch: U steps of EPL elements per lane, all column loads first (caller), then the
// LDS (or global) lookups and one 16-byte store per step.
template <typename T, bool LDS>
__device__ __forceinline__ void stage_load(ColVec<StageU<T>::EPL> (&c)[StageU<T>::U], int g, int g1,
                                           const unsigned short *__restrict__ colS) {
  constexpr int EPL = StageU<T>::EPL, U = StageU<T>::U, STEP = kStageThreads * EPL;
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (g + u * STEP < g1) ld_cols<EPL>(c[u], colS + g + u * STEP);
}
template <typename T, bool LDS>
__device__ __forceinline__ void stage_put(const ColVec<StageU<T>::EPL> (&c)[StageU<T>::U], int g, int g1,
                                          const unsigned char *s_tab, const T *__restrict__ tab, int nb,
                                          T *__restrict__ G) {
  constexpr int EPL = StageU<T>::EPL, U = StageU<T>::U, STEP = kStageThreads * EPL;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int gg = g + u * STEP;
    if (gg < g1) {
      T val[EPL];
#pragma unroll
      for (int j = 0; j < EPL; ++j) {
        const unsigned off = col_at<EPL>(c[u], j);
        if constexpr (LDS) val[j] = reinterpret_cast<const T *>(s_tab)[off];
        else val[j] = tab[nb + (int)off];
      }
      // doubles non-temporal: G (64 MB on ER-1M, 4 GB of G_A on R-MAT-24) is streamed out
      // once and read back by the next launch (ER-1M kernel 8: 61.8 vs 62.7 us per round,
      // R-MAT-24 kernel 9: 6,728 vs 6,807 us; process-separated A/Bs, profiles/r05/n, o).
      // Packed codes (8-32 MB) stay write-back: they fit on chip until the tiles read them
      // (non-temporal there: 41.0 vs 38.8 us per 8-bit round, profiles/r05/q)
      typedef unsigned v4u __attribute__((ext_vector_type(4)));
      v4u w;
      __builtin_memcpy(&w, val, 16);
      if constexpr (sizeof(T) >= kStageNtMinBytes)
        __builtin_nontemporal_store(w, reinterpret_cast<v4u *>(G + gg));
      else
        *reinterpret_cast<v4u *>(G + gg) = w;
    }
  }
}

// Slice s of the table (element type T) -> LDS (LDS = false: the table is wider than the
// layout and is read from global memory), then the block's G range [g0, g1), software
// pipelined: the next batch's column loads are issued before the current batch is looked
// up and stored (two register sets, so no in-flight register is copied).
template <typename T, bool LDS>
__device__ __forceinline__ void stage_body(unsigned char *s_tab, int nb, int cnt, int g0, int g1,
                                           const unsigned short *__restrict__ colS,
                                           const T *__restrict__ tab, T *__restrict__ G) {
  constexpr int EPL = StageU<T>::EPL, U = StageU<T>::U, BSTEP = U * kStageThreads * EPL;
  constexpr int kW = kStageLds / 16 / kStageThreads;
  const int t = threadIdx.x;
  uint4 buf[kW];
  const int bytes = LDS ? cnt * (int)sizeof(T) : 0;
  const int w16 = bytes >> 4;
  if constexpr (LDS) {
    const uint4 *s16 = reinterpret_cast<const uint4 *>(tab + nb);
#pragma unroll
    for (int u = 0; u < kW; ++u) {
      const int k = t + u * kStageThreads;
      buf[u] = k < w16 ? s16[k] : make_uint4(0u, 0u, 0u, 0u);
    }
  }
  ColVec<EPL> ca[U], cb[U];
  int g = g0 + t * EPL;
  stage_load<T, LDS>(ca, g, g1, colS);
  if constexpr (LDS) {  // slice stores after the first batch's loads are in flight
#pragma unroll
    for (int u = 0; u < kW; ++u) {
      const int k = t + u * kStageThreads;
      if (k < w16) reinterpret_cast<uint4 *>(s_tab)[k] = buf[u];
    }
    const int tb = w16 << 4;
    if (t < bytes - tb) s_tab[tb + t] = reinterpret_cast<const unsigned char *>(tab + nb)[tb + t];
    __syncthreads();
  }
  for (;;) {
    if (g >= g1) break;
    stage_load<T, LDS>(cb, g + BSTEP, g1, colS);
    stage_put<T, LDS>(ca, g, g1, s_tab, tab, nb, G);
    g += BSTEP;
    if (g >= g1) break;
    stage_load<T, LDS>(ca, g + BSTEP, g1, colS);
    stage_put<T, LDS>(cb, g, g1, s_tab, tab, nb, G);
    g += BSTEP;
  }
}

__global__ __launch_bounds__(kStageThreads) void k_stage(StageArgs sa, int n,
                                                        const double *__restrict__ a_prev,
                                                        const void *__restrict__ code_prev,
                                                        PackCtl *ctl, int rslot,
                                                        void *__restrict__ G, const int *__restrict__ psample,
                                                        int *pw_host) {
  __shared__ __align__(16) unsigned char s_tab[kStageLds];
  // the packing plan from a_{r-1} (the table staged here; due after round r-1) rides on the
  // stage launch: k_round_staged, the plan's first reader, starts after this launch, so the
  // plan needs no launch (and stream slot) of its own. Its block is block 0, dispatched
  // first so its dependent loads overlap the staging; blocks 1-7 exit and the stage blocks
  // follow from block 8 on, on the XCDs (blockIdx % 8) they have without the plan.
  int bid = (int)blockIdx.x;
  if (psample) {
    if (bid == 0) plan_body<kStageThreads>(a_prev, psample, ctl, pw_host);
    if (bid < 8) return;
    bid -= 8;
  }
  const PackCtl pp = ctl[rslot ^ 1];
  // bytes per element of the table gathered (kernel 9 stages the doubles, always written)
  const int wb = (pp.width && !sa.f64) ? pp.width / 8 : 8;
  const int li = sa.f64 ? 3 : sa.sel[width_index(pp.width)];
  if (bid >= sa.NB[li]) return;
  const int4 rg = sa.brange[li][bid];
  if (rg.x >= rg.y) return;  // no slice here (grid rounded to whole XCD rows) or empty region
  const int LB = 1 << li;  // bytes per element the layout was built for
  const int SN = sa.SN[li];
  const int nb = rg.z * SN;
  const int cnt = min(SN, n - nb);
  const void *src = (pp.width && !sa.f64) ? code_prev : static_cast<const void *>(a_prev);
  const unsigned short *colS = sa.colS[li];
#define FU_BODY(T)                                                                                    \
  do {                                                                                                \
    if ((int)sizeof(T) <= LB)                                                                         \
      stage_body<T, true>(s_tab, nb, cnt, rg.x, rg.y, colS, reinterpret_cast<const T *>(src),         \
                          reinterpret_cast<T *>(G));                                                  \
    else                                                                                              \
      stage_body<T, false>(s_tab, nb, cnt, rg.x, rg.y, colS, reinterpret_cast<const T *>(src),        \
                           reinterpret_cast<T *>(G));                                                 \
  } while (0)
  if (wb == 1) FU_BODY(unsigned char);
  else if (wb == 2) FU_BODY(unsigned short);
  else if (wb == 4) FU_BODY(unsigned);
  else FU_BODY(unsigned long long);
#undef FU_BODY
}

// ------------------------------------------------------------------------------------
// Kernel 9, "pregather": propagation blocking for power-law graphs, where tiles touch far
// more slices than kernel 8's u16 index can address and most edges sit in heavy rows. Two
// passes turn every random gather a_{r-1}[col e] into streams:
//   * k_stage (doubles, 128 KB slices): G_A in slice-major order, within slice s the edges
//     whose neighbour lies in s, in edge order (so each bucket of kTrBE consecutive edges
//     has one contiguous run per slice);
//   * k_transpose: one block per bucket reads its runs (the run starts of every slice are
//     precomputed per bucket), scatters the values into LDS by their position in the bucket
//     and writes Gb[e] for the bucket's edges, coalesced.
// The round kernels (kernel 4's tiles, heavy rows and mega hubs, PRE = true) then read Gb[e]
// beside the flows. Bytes per edge: stage 2 + 8, transpose 8 + 2 + 8, round 8 (instead of
// col 4 + one random 8-byte gather).
// ------------------------------------------------------------------------------------
constexpr int kTrThreads = 1024;

// Persistent over its buckets: grid = 8 x (blocks per XCD); XCD x owns the contiguous
// bucket range [x per, (x + 1) per) and its blocks take every nj-th bucket of it. The next
// bucket's run starts (offT) are loaded while this bucket's G_A loads are in flight, and its
// G_B stores drain while the next bucket is scanned (with one block per bucket, each block
// paid the offT round trip first and held its slot until its stores were done).
template <bool NT>  // NT: the streamed G_B stores non-temporal
__global__ __launch_bounds__(kTrThreads, kTrWaves) void k_transpose(int b0, int nbk, int P, long long E,
                                                        const int *__restrict__ offT,
                                                        const double *__restrict__ GA,
                                                        const unsigned short *__restrict__ pos16,
                                                        double *__restrict__ GB) {
  __shared__ double s_v[kTrBE];
  __shared__ unsigned short s_m[kTrMaxP + 1];  // first element (bucket order) of each slice's run
  __shared__ int s_o[kTrMaxP];      // G_A index of each run
  __shared__ int s_c[kTrBE / 64 + 1];
  __shared__ int s_w[kTrThreads / 64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  // XCD-contiguous buckets (block b runs on XCD b % 8): a G_A line that ends one bucket's
  // run and starts the next bucket's is fetched into one L2, not two
  const int per = (nbk + 7) >> 3;
  const int nj = (int)(gridDim.x >> 3);
  int bk = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  const int bend = min((int)(blockIdx.x & 7) * per + per, nbk);
  if (bk >= bend) return;
  // runs: thread t owns slices 2t, 2t + 1
  int o[2], len[2];
  auto load_runs = [&](int bkk, int (&oo)[2], int (&ll)[2]) {
    const int bb = b0 + bkk;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int sl = 2 * t + j;
      oo[j] = sl < P ? offT[(long long)bb * P + sl] : 0;
      ll[j] = sl < P ? offT[(long long)(bb + 1) * P + sl] - oo[j] : 0;
    }
  };
  load_runs(bk, o, len);
  for (;;) {
  const int bb = b0 + bk;
  const long long e0 = (long long)bb * kTrBE;
  const int ne = (int)min((long long)kTrBE, E - e0);
  // exclusive scan of len0 + len1 over the block: wave shuffles, then the 16 wave totals
  int x = len[0] + len[1];
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) s_w[w] = x;
  __syncthreads();
  int base = 0;
  for (int k = 0; k < w; ++k) base += s_w[k];
  const int excl = base + x - (len[0] + len[1]);
  if (2 * t < P) {
    s_m[2 * t] = excl;
    s_o[2 * t] = o[0];
  }
  if (2 * t + 1 < P) {
    s_m[2 * t + 1] = excl + len[0];
    s_o[2 * t + 1] = o[1];
  }
  if (t == 0) {  // staged elements of the bucket (< ne when mega-hub edges are left out)
    int tot = 0;
    for (int k = 0; k < kTrThreads / 64; ++k) tot += s_w[k];
    s_m[P] = tot;
  }
  __syncthreads();
  const int nst = s_m[P];
  // coarse table: the run holding element 64 k (s_c), so each element's search spans only
  // the runs of its 64-element stretch
  if (t < kTrBE / 64) {
    const int m = t * 64;
    int lo = 1, hi = P;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (s_m[mid] > m) hi = mid; else lo = mid + 1;
    }
    s_c[t] = lo;
  }
  if (t == 0) s_c[kTrBE / 64] = P;
  __syncthreads();
  // element m (the bucket's G_A runs in slice order) -> G_A index; all searches first, then
  // every load of the thread in flight at once, then the LDS scatter by bucket position
  constexpr int kPerT = kTrBE / kTrThreads;
  int g[kPerT];
#pragma unroll
  for (int k = 0; k < kPerT; ++k) {
    const int m = t + k * kTrThreads;
    g[k] = -1;
    if (m < nst) {
      int lo = s_c[m >> 6], hi = s_c[(m >> 6) + 1];  // first boundary s_m[s] > m lies in [lo, hi]
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s_m[mid] > m) hi = mid; else lo = mid + 1;
      }
      const int run = lo - 1;  // s_m[run] <= m < s_m[run + 1]: a non-empty run
      g[k] = s_o[run] + (m - s_m[run]);
    }
  }
  double val[kPerT];
  unsigned short pos[kPerT];
#pragma unroll
  for (int k = 0; k < kPerT; ++k) {
    // plain loads (non-temporal G_A loads beside the non-temporal stores: 6,703 vs 6,612 us
    // per round on R-MAT-24, profiles/r05/u)
    val[k] = g[k] >= 0 ? GA[g[k]] : 0.0;
    pos[k] = g[k] >= 0 ? pos16[g[k]] : (unsigned short)0;
  }
  const int next = bk + nj;
  if (next < bend) load_runs(next, o, len);  // in flight beside this bucket's loads
#pragma unroll
  for (int k = 0; k < kPerT; ++k)
    if (g[k] >= 0) s_v[pos[k]] = val[k];
  __syncthreads();
  for (int q = t; q < ne; q += kTrThreads) {
    if constexpr (NT) __builtin_nontemporal_store(s_v[q], GB + e0 + q);
    else GB[e0 + q] = s_v[q];
  }
  if (next >= bend) break;
  __syncthreads();  // the shared tables and s_v are rewritten for the next bucket
  bk = next;
  }
}

// Kernel 9: the isolated rows at the end of the degree layout (the last light tiles have no
// edges): a_r = ((v - 0.0) + 0.0) / 1 (CA:106-113 with no neighbours), as a light tile
// computes it, one thread per row instead of a tile block per 128 rows.
__global__ __launch_bounds__(kBlock) void k_isolated(int i0, int n, const double *__restrict__ v,
                                                     double *__restrict__ a_new, const double *__restrict__ target,
                                                     unsigned long long *__restrict__ err, void *__restrict__ code_new,
                                                     PackCtl *__restrict__ ctl, int rslot, int check) {
  const PackCtl pc = ctl[2];
  if (blockIdx.x == 0 && threadIdx.x == 0) ctl[rslot] = pc;
  const int i = i0 + blockIdx.x * kBlock + threadIdx.x;
  unsigned long long eb = 0;
  if (i < n) {
    const double a = ((v[i] - 0.0) + 0.0) / (double)1;
    *(a_new + i) = a;
    if (pc.width) put_code(pc, code_new, i, a);
    if (check) eb = err_bits(a, target[i]);
  }
  if (check) block_max_to(eb, err);
}

template <bool CHECK, int TE, int TN, bool RF = true, bool LO = true>
__global__ __launch_bounds__(kBlock) void k_round_staged(
    const int4 *__restrict__ tiles, int t0, int ntl,
    const int *__restrict__ rowptr, const int *__restrict__ col,
    const StageArgs sa, const void *__restrict__ G, const double *__restrict__ v,
    double *__restrict__ F, const double *__restrict__ a_prev, const double *__restrict__ a_prev2,
    double *__restrict__ a_new, const double *__restrict__ target,
    unsigned long long *__restrict__ err, void *__restrict__ code_new, PackCtl *__restrict__ ctl,
    int rslot, int fm) {
  static_assert(TE % kBlock == 0 && TN <= kBlock, "tile geometry");
  static_assert(TE <= 1024, "the u16 staged index holds a 10-bit tile position");
  const PackCtl pp = ctl[rslot ^ 1];
  const int lsel = sa.sel[width_index(pp.width)];
  const PackCtl pc = ctl[2];
  if (blockIdx.x == 0 && threadIdx.x == 0) ctl[rslot] = pc;
  __shared__ double s_x[TE];
  __shared__ double s_er[TE];
  __shared__ unsigned char s_own[TE];
  __shared__ int s_rp[TN + 1];
  __shared__ double s_a[TN];
  const int t = threadIdx.x;
  unsigned long long eb = 0;
  // XCD-aware order: block b runs on XCD b % 8; consecutive tiles go to the same XCD, so
  // the G runs that neighbouring tiles share in every slice region meet in one L2
  const int xcd = blockIdx.x & 7, per = ntl >> 3, rem = ntl & 7;
  const int tile = t0 + xcd * per + min(xcd, rem) + (int)(blockIdx.x >> 3);
  const int4 tl = tiles[tile];
  const int nb = tl.x, nn = tl.y - tl.x;
  const int e0 = tl.z, ne = tl.w - tl.z;
  constexpr int kPer = TE / kBlock;
  const unsigned short *__restrict__ s16 = sa.sidx16[lsel];
  unsigned si[kPer];  // position in the tile
  double x[kPer], g[kPer];
  int gi[kPer];
  // Load order (LO): the run offsets and staged indices first, the flows and node words
  // after them, so the G loads (which need only the former) issue while the flows are in
  // flight (in-order completion: waiting for a load waits for every load issued before it).
  int rp;
  double vv, own2;
  if constexpr (LO) {
  {  // u16 position | run << 10; G index = m + D[run] (lane `run` holds D)
    const int dl = sa.dtab[lsel][(size_t)tile * kStageRuns + (t & 63)];
    unsigned short c16[kPer];
    // unconditional loads from clamped (always valid) indices, so the compiler can wait for
    // the staged indices alone (vmcnt(N)) instead of for every load (a skipped load would
    // change the count)
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int q = t + k * kBlock;
      const unsigned short c = s16[q < ne ? e0 + q : 0];
      c16[k] = q < ne ? c : (unsigned short)0;
    }
    if constexpr (RF) {
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        const int q = t + k * kBlock;
        const double f = ld_f(F, q < ne ? e0 + q : 0);
        x[k] = q < ne ? f : 0.0;
      }
    } else {
#pragma unroll
      for (int k = 0; k < kPer; ++k) x[k] = 0.0;
    }
    const int tn = min(t, nn - 1);  // a light tile has at least one node
    const int rp0 = rowptr[nb + min(t, nn)];
    const double v0 = v[nb + tn], o0 = a_prev2[nb + tn];
    asm volatile("" ::: "memory");  // every load above issued before the first wait (no sinking)
    rp = t <= nn ? rp0 : 0;
    vv = t < nn ? v0 : 0.0;
    own2 = t < nn ? o0 : 0.0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int q = t + k * kBlock;
      const int dd = __shfl(dl, (int)(c16[k] >> 10));
      si[k] = c16[k] & 1023u;
      gi[k] = q < ne ? q + dd : -1;
    }
  }
  } else {  // the round-1 order: indices and flows interleaved (measured against LO)
  {  // u16 position | run << 10; G index = m + D[run] (lane `run` holds D)
    const int dl = sa.dtab[lsel][(size_t)tile * kStageRuns + (t & 63)];
    unsigned short c16[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int q = t + k * kBlock;
      c16[k] = q < ne ? s16[e0 + q] : (unsigned short)0;
      x[k] = q < ne && RF ? ld_f(F, e0 + q) : 0.0;
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int q = t + k * kBlock;
      const int dd = __shfl(dl, (int)(c16[k] >> 10));
      si[k] = c16[k] & 1023u;
      gi[k] = q < ne ? q + dd : -1;
    }
  }
  rp = t <= nn ? rowptr[nb + t] : 0;
  vv = t < nn ? v[nb + t] : 0.0;
  own2 = t < nn ? a_prev2[nb + t] : 0.0;
  }
  // every G load of the tile first, then decode (escapes gather the double via col)
  if (pp.width == 0) {
#pragma unroll
    for (int k = 0; k < kPer; ++k)
      g[k] = gi[k] >= 0 ? reinterpret_cast<const double *>(G)[gi[k]] : 0.0;
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
    const double fo0 = fm ? old_flow(fm, own2) : 0.0;
    for (int q = qb; q < qe; ++q) {
      const double er = s_er[q];
      const double fr = recon_fr(fm ? fo0 : s_x[q], er, own2);
      s_x[q] = fr;
      s_own[q] = (unsigned char)t;
      S = S + fr;
      T = T + er;
    }
    const double a = ((vv - S) + T) / (double)(qe - qb + 1);
    s_a[t] = a;
    *(a_new + nb + t) = a;
    if (pc.width) put_code(pc, code_new, nb + t, a);
    if (CHECK) eb = err_bits(a, target[nb + t]);
  }
  __syncthreads();
  // phase C: new flows, coalesced, in place (CA:117-118)
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int q = t + k * kBlock;
    if (q < ne) {
      st_fo(F, e0 + q, (s_x[q] + s_a[s_own[q]]) - s_er[q], x[k], fm);
    }
  }
  if (CHECK) block_max_to(eb, err);
}


// ------------------------------------------------------------------------------------
// Kernel 9's heavy rows (degree > 64 x kHeavyRL, <= mega_hub), many rows per chain wave.
// A row's two sums are exact left-to-right chains (CA:106, CA:110), so each element costs
// one dependent fp64 add per sum. With one row per wave (k_round_recon's heavy tiles) a
// wave64 v_add_f64 advances two chains (even lanes S, odd lanes T), and on R-MAT-24 the
// chains of these rows kept the SIMDs busy for ~1.2 ms per round beside their memory
// traffic. Here a block takes kMR rows of similar length (the rows are sorted by degree),
// its four waves stage chunks of kMCH elements of every row, (fr, er) into LDS, and ONE
// wave runs all 2 kMR chains at once (lane 2r: S of row r, lane 2r + 1: T), with the loads
// of the next chunk in flight meanwhile. Then a flow pass re-reads the old flows and the
// pre-gathered estimates (CA:117-118). Same operations in the same order as every other
// path: the results are bitwise equal.
// ------------------------------------------------------------------------------------
//
// LAG (option "lag", kernel 9): no flow pass. Round r leaves f_r unwritten and instead
// materialises f_{r-2} while it stages the row: F holds f_{r-4} and f_{r-2} = (recon(f_{r-4}, er_{r-2}, a_{r-4}) +
// a_{r-2}) - er_{r-2} is exactly what round r - 2's flow pass would have written (CA:117-118,
// same operations, same operands: er_{r-2} from the G_B ring, a_{r-4} from the per-row
// history `hist`). So a lagged row costs 32 B per edge (f and G_B of two rounds, one flow
// store) instead of 40 (both re-read for the flow pass). LAGM = 1: F holds f_{r-2}
// already (fm = 1, 2: computed, and stored as the base of round r + 2); LAGM = 2: F holds
// f_{r-4} (the previous round of this parity was lagged). lag_finalize
// writes f_r when another kernel, fu_get_flows or a tile rebuild needs it.
constexpr int kMCH = 64;  // elements per row per chunk (one per lane)
template <bool CHECK, int LAGM = 0>  // LAGM: 0 = no lag, 1 = lagin 0, 2 = lagin 1
__global__ __launch_bounds__(kBlock) void k_heavy_multi(
    const int *__restrict__ hrows, int nrows, const int *__restrict__ rowptr, const double *__restrict__ v,
    double *__restrict__ F, const double *__restrict__ a_prev2, double *__restrict__ a_new,
    const double *__restrict__ target, unsigned long long *__restrict__ err, void *__restrict__ code_new,
    PackCtl *__restrict__ ctl, const double *__restrict__ Gb, int fm,
    const double *__restrict__ Gb_old = nullptr, double *__restrict__ hist = nullptr) {
  constexpr bool LAG = LAGM > 0;
  constexpr bool mat = LAGM == 2;
  // sh[buf][2 r + {0: fr, 1: er}][q]; a row stride of kMCH + 1 doubles puts the 32 chain lanes'
  // reads of one step on 32 different bank pairs
  __shared__ double sh[2][2 * kMR][kMCH + 1];
  __shared__ int s_b[kMR], s_d[kMR];
  __shared__ double s_o2[kMR], s_a[kMR], s_o4[kMR];
  const PackCtl pc = ctl[2];  // packing of a_r (the table written here)
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  const int r0 = blockIdx.x * kMR;
  if (t < kMR) {
    const bool ok = r0 + t < nrows;
    const int i = ok ? hrows[r0 + t] : 0;
    const int b = ok ? rowptr[i] : 0;
    s_b[t] = b;
    s_d[t] = ok ? rowptr[i + 1] - b : 0;
    const double o2 = ok ? a_prev2[i] : 0.0;
    s_o2[t] = o2;
    if (LAG) {  // a_{r-4} of the row (written by round r - 2), then a_{r-2} for round r + 2
      s_o4[t] = ok && mat ? hist[r0 + t] : 0.0;
      if (ok) hist[r0 + t] = o2;
    }
  }
  __syncthreads();
  // wave w stages rows 4 w .. 4 w + 3; element c kMCH + lane of each
  int rb[4], rd[4];
  double ro2[4], ro4[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    rb[j] = s_b[4 * w + j];
    rd[j] = s_d[4 * w + j];
    ro2[j] = s_o2[4 * w + j];
    ro4[j] = LAG ? s_o4[4 * w + j] : 0.0;
  }
  const int nch = (s_d[0] + kMCH - 1) / kMCH;  // rows sorted longest first
  // two register sets, each one chunk of the wave's 4 rows: the loads run two chunks ahead of
  // the chain. Loads are unconditional from clamped indices (the compiler then waits for a
  // set by count, vmcnt(N), not for everything)
  double fo0[4], er0[4], fo1[4], er1[4];
  double eo0[4], eo1[4];  // LAGM 2: er_{r-2} (G_B of round r - 2)
  auto load = [&](double (&fo)[4], double (&er)[4], double (&eo)[4], int c) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = min(c * kMCH + lane, max(rd[j] - 1, 0));
      er[j] = Gb[rb[j] + k];
      if constexpr (mat) eo[j] = Gb_old[rb[j] + k];
      if constexpr (mat) fo[j] = ld_f(F, rb[j] + k);
      else fo[j] = ld_fo(F, rb[j] + k, fm, ro2[j]);
    }
  };
  auto put = [&](const double (&fo)[4], const double (&er)[4], const double (&eo)[4], int c, int buf) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = 4 * w + j;
      const bool in = c * kMCH + lane < rd[j];
      double f2 = fo[j];  // f_{r-2}
      if (LAG && in) {
        const int e = rb[j] + c * kMCH + lane;
        if constexpr (mat) {  // round r - 2's flow (CA:117-118), from f_{r-4}
          f2 = (recon_fr(fo[j], eo[j], ro4[j]) + ro2[j]) - eo[j];
          st_f(F, e, f2, fo[j]);
        } else if (fm) {  // f_{-1} / f_0, the base round r + 2 materialises from
          st_f_full(F, e, f2);
        }
      }
      sh[buf][2 * r][lane] = in ? recon_fr(f2, er[j], ro2[j]) : 0.0;
      sh[buf][2 * r + 1][lane] = in ? er[j] : 0.0;
    }
  };
  // chain lanes: lane 2 r + h (wave 0, lanes < 2 kMR)
  const int cr = lane >> 1, ch = lane & 1;
  double acc = 0.0;
  auto chain = [&](int c, int buf) {
    if (w == 0 && lane < 2 * kMR) {
      const int len = min(kMCH, max(0, s_d[cr] - c * kMCH));
      const double *src = sh[buf][lane];
      int q = 0;
      if (len == kMCH) {  // a full chunk: the next 8 LDS reads in flight beside the 8 dependent adds
        double x[8], y[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = src[u];
#pragma unroll
        for (int b = 0; b < kMCH; b += 16) {
#pragma unroll
          for (int u = 0; u < 8; ++u) y[u] = src[b + 8 + u];
#pragma unroll
          for (int u = 0; u < 8; ++u) acc = acc + x[u];
          if (b + 16 < kMCH) {
#pragma unroll
            for (int u = 0; u < 8; ++u) x[u] = src[b + 16 + u];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) acc = acc + y[u];
        }
        q = len;
      }
      for (; q + 8 <= len; q += 8) {
        double x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = src[q + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc = acc + x[u];
      }
      for (; q < len; ++q) acc = acc + src[q];
    }
  };
  if (nch > 0) {
    load(fo0, er0, eo0, 0);
    load(fo1, er1, eo1, 1);
    put(fo0, er0, eo0, 0, 0);
  }
  __syncthreads();
  for (int c = 0; c < nch; c += 2) {
    // chunk c in buffer 0, chunk c + 1 in flight in set 1
    if (c + 2 < nch) load(fo0, er0, eo0, c + 2);
    chain(c, 0);
    __syncthreads();
    if (c + 1 >= nch) break;
    put(fo1, er1, eo1, c + 1, 1);
    __syncthreads();
    // chunk c + 1 in buffer 1, chunk c + 2 in flight in set 0
    if (c + 3 < nch) load(fo1, er1, eo1, c + 3);
    chain(c + 1, 1);
    __syncthreads();
    if (c + 2 >= nch) break;
    put(fo0, er0, eo0, c + 2, 0);
    __syncthreads();
  }
  unsigned long long eb = 0;
  if (w == 0) {
    const double T = __shfl(acc, (lane & ~1) + 1);  // row cr's T (lane 2 cr + 1)
    if (lane < 2 * kMR && ch == 0 && r0 + cr < nrows) {
      const int i = hrows[r0 + cr];
      const double a = ((v[i] - acc) + T) / (double)(s_d[cr] + 1);
      s_a[cr] = a;
      *(a_new + i) = a;
      if (pc.width) put_code(pc, code_new, i, a);
      if (CHECK) eb = err_bits(a, target[i]);
    }
  }
  if (LAG) {  // round r + 2 (or k_lag_final) writes the flows
    if (CHECK) block_max_to(eb, err);
    return;
  }
  __syncthreads();
  // flows (CA:117-118): wave w, its rows, 8 elements per lane in flight
#pragma unroll 1
  for (int j = 0; j < 4; ++j) {
    const int b = rb[j], d = rd[j];
    const double own2 = ro2[j], a = s_a[4 * w + j];
    for (int k0 = 0; k0 < d; k0 += 8 * 64) {
      double f8[8], e8[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + lane + 64 * u;
        e8[u] = k < d ? Gb[b + k] : 0.0;
        f8[u] = k < d ? ld_fo(F, b + k, fm, own2) : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + lane + 64 * u;
        if (k < d) st_fo(F, b + k, (recon_fr(f8[u], e8[u], own2) + a) - e8[u], f8[u], fm);
      }
    }
  }
  if (CHECK) block_max_to(eb, err);
}

// Lagged rows (k_heavy_multi<LAG>): write the flows f_{r'} their last round r' of this
// parity left unwritten: F holds f_{r'-2}, Gb = er_{r'} (G_B of round r'), hist = a_{r'-2},
// a = a_{r'} (CA:117-118, the flow pass k_heavy_multi would have run). One block per row.
__global__ __launch_bounds__(kBlock) void k_lag_final(const int *__restrict__ rows, const int *__restrict__ rowptr,
                                                      double *__restrict__ F, const double *__restrict__ Gb,
                                                      const double *__restrict__ hist,
                                                      const double *__restrict__ a) {
  const int i = rows[blockIdx.x];
  const int b = rowptr[i], d = rowptr[i + 1] - b;
  const double own2 = hist[blockIdx.x], an = a[i];
  for (int k0 = 0; k0 < d; k0 += 8 * kBlock) {
    double f8[8], e8[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = k0 + (int)threadIdx.x + kBlock * u;
      e8[u] = k < d ? Gb[b + k] : 0.0;
      f8[u] = k < d ? ld_f(F, b + k) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = k0 + (int)threadIdx.x + kBlock * u;
      if (k < d) st_f(F, b + k, (recon_fr(f8[u], e8[u], own2) + an) - e8[u], f8[u]);
    }
  }
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
                                                      double2 *__restrict__ hubxy, int fm,
                                                      const int *__restrict__ hub_blk) {
  const long long q = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (q >= total) return;
  // hubs[h] = {node, row begin, row end, offset}: the block's first edge's hub from the host
  // table (a hub of > mega_hub edges spans whole blocks), then at most a step or two on
  int lo = hub_blk[blockIdx.x];
  while (lo + 1 < nhub && hubs[lo + 1].w <= q) ++lo;
  const int4 hb = hubs[lo];
  const int k = hb.y + (int)(q - hb.w);
  const PackCtl pp = ctl[rslot ^ 1];
  const double er = ld_est(pp, code_prev, a_prev, col[k]);
  const double own2 = a_prev2[hb.x];
  hubxy[q] = make_double2(recon_fr(ld_fo(F, k, fm, own2), er, own2), er);
}


// Mega hubs: the flows of every hub edge (CA:117-118) once the hub blocks have written a_r,
// with many blocks (the hub block's own loop would hold one CU for d / 256 iterations on
// the round's critical path).
__global__ __launch_bounds__(kBlock) void k_hub_flows(int nhub, const int4 *__restrict__ hubs, long long total,
                                                      const double2 *__restrict__ hubxy,
                                                      const double *__restrict__ a_new, double *__restrict__ F,
                                                      const double *__restrict__ Gb,
                                                      const double *__restrict__ a_prev2, int fm,
                                                      const int *__restrict__ hub_blk) {
  const long long q = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (q >= total) return;
  // hubs[h] = {node, row begin, row end, offset}: the block's first edge's hub from the host
  // table (a hub of > mega_hub edges spans whole blocks), then at most a step or two on
  int lo = hub_blk[blockIdx.x];
  while (lo + 1 < nhub && hubs[lo + 1].w <= q) ++lo;
  const int4 hb = hubs[lo];
  const int k = hb.y + (int)(q - hb.w);
  const double a = a_new[hb.x];
  if (Gb) {  // kernel 9: (fr, er) rebuilt from the pre-gathered estimate and the old flow
    const double own2 = a_prev2[hb.x];
    const double er = Gb[k], fo = ld_fo(F, k, fm, own2);
    st_fo(F, k, (recon_fr(fo, er, own2) + a) - er, fo, fm);
    return;
  }
  const double2 p2 = hubxy[q];
  st_fo(F, k, (p2.x + a) - p2.y, fm ? 0.0 : ld_f(F, k), fm);
}

// split-word flows -> doubles (fu_get_flows of kernels >= 4)
__global__ void k_unsplit(long long cnt, const double *__restrict__ src, double *__restrict__ dst) {
  long long q = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (q < cnt) dst[q] = ld_f(src, (int)q);
}
// fu_copy_bandwidth: a plain float4 copy, grid-stride (the part's streaming rate)
__global__ __launch_bounds__(kBlock) void k_copy4(long long cnt, const float4 *__restrict__ src,
                                                  float4 *__restrict__ dst) {
  const long long stride = (long long)gridDim.x * kBlock;
  for (long long q = (long long)blockIdx.x * kBlock + threadIdx.x; q < cnt; q += stride) dst[q] = src[q];
}

__global__ void k_fill(long long cnt, double val, double *__restrict__ p) {
  long long q = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (q < cnt) p[q] = val;
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


// k_replay_persist with one node per thread and the node's state (its row of flows and
// estimate caches, cursor, snapshot cursor, last average) kept in registers for the whole
// run (degree <= MAXD): an event costs its own loads instead of also re-reading the node's
// state from memory on every pass. Same event semantics and order as k_replay_persist.
//
// The replay is bound by the time one lock-step iteration of a wave takes, not by the
// trace's dependence depth (RR-64K pairwise: ~6 message hops per 100 ticks; a node runs
// {receive, fire} every other tick), and an iteration ends waiting for its vector-memory
// operations, which retire in issue order: loads, and the write-through message stores.
// So an iteration issues as few of them as it can, in a fixed order:
//   * the lane's next events sit in a 16-entry LDS ring of packed 8-byte descriptors
//     (ev_dec), refilled 8 at a time (64 contiguous bytes); they land during one iteration
//     and are written to the ring at the head of the next;
//   * every iteration ends with exactly TWO 16-byte sc1 polls (the payloads of the lane's
//     next two receives, both tagged halves each) and then, on the pairwise path
//     (CA = false), exactly TWO 16-byte sc1 stores (the iteration's messages {flow, avg}),
//     each aimed at the node's scratch slot when there is none: the next iteration waits
//     for the polls and leaves the stores in flight (vmcnt(2)), instead of waiting for every
//     store's write-through;
//   * an iteration runs up to kRW events in program order, a receive only once its payload
//     has arrived in one of the two polls, at most two pairwise fires: RR-64K runs two
//     {receive, fire} pairs per iteration.
// The collect-all path (k messages per fire) stores its messages as it goes.
constexpr int kRW = 4;       // events per iteration at most
constexpr int kScan = 4;     // ring entries searched for the next two receives
constexpr int kRing = 16;    // LDS ring entries per lane
constexpr int kRefill = 8;   // events per refill (64 contiguous bytes)
// packed 8-byte event: x = type | slot << 2 | k << 7 | tick << 12 (deg <= 16, tick < 2^20),
// y = message slot (receive, pairwise fire) or out_ids offset (collect-all fire); decoded to
// the int4 {type, slot | k << 8 (pairwise) / slot (receive) / k (collect-all), y, tick}
__device__ __forceinline__ int4 ev_dec(int2 e) {
  const int ty = e.x & 3, sl = (e.x >> 2) & 31, k = (e.x >> 7) & 31, tk = (int)((unsigned)e.x >> 12);
  return make_int4(ty, ty == FU_EV_FIRE_PW ? (sl | k << 8) : ty == FU_EV_RECV ? sl : k, e.y, tk);
}
template <int MAXD, bool CA>
__global__ __launch_bounds__(kBlock) void k_replay_persist_reg(
    int n, int tick_end, const long long *__restrict__ node_off, const int2 *__restrict__ node_evt,
    const int *__restrict__ out_uid, int n_uid,
    const long long *__restrict__ rowptr, const double *__restrict__ v, double *__restrict__ flow,
    double *__restrict__ est, double *__restrict__ last, unsigned long long *__restrict__ pay,
    long long *__restrict__ cursor, int *__restrict__ scur, int n_snap,
    const int *__restrict__ snap_ticks, double *__restrict__ snaps, int *__restrict__ status,
    long long max_iters) {
  __shared__ int2 s_ring[kRing * kBlock];  // entry k of lane t at k * kBlock + t
  const int node = blockIdx.x * kBlock + threadIdx.x;
  if (node >= n) return;  // (no block barrier below)
  int2 *ring = s_ring + threadIdx.x;
  long long p = cursor[node];
  const long long pe = node_off[node + 1];
  int sc = scur[node];
  const long long rb = rowptr[node];
  const int deg = (int)(rowptr[node + 1] - rb);
  double fl[MAXD], es[MAXD];
#pragma unroll
  for (int j = 0; j < MAXD; ++j) {
    fl[j] = j < deg ? flow[rb + j] : 0.0;
    es[j] = j < deg ? est[rb + j] : 0.0;
  }
  const double val = v[node];
  double lst = last[node];
  // ring: events p .. p + rv - 1 at entries rh, rh + 1, ... (mod kRing); fill = next event to load
  int rh = 0, rv = 0;
  long long fill = p;
  int2 r0, r1, r2, r3, r4, r5, r6, r7;  // the refill in flight (named registers: no private array)
  bool pend = false;
  int pcnt = 0;
#define FU_RING_REFILL()                                                    \
  do {                                                                      \
    const long long lo = max(0ll, pe - 1);                                  \
    r0 = node_evt[max(0ll, min(fill, lo))];                                 \
    r1 = node_evt[max(0ll, min(fill + 1, lo))];                             \
    r2 = node_evt[max(0ll, min(fill + 2, lo))];                             \
    r3 = node_evt[max(0ll, min(fill + 3, lo))];                             \
    r4 = node_evt[max(0ll, min(fill + 4, lo))];                             \
    r5 = node_evt[max(0ll, min(fill + 5, lo))];                             \
    r6 = node_evt[max(0ll, min(fill + 6, lo))];                             \
    r7 = node_evt[max(0ll, min(fill + 7, lo))];                             \
    pcnt = (int)max(0ll, min((long long)kRefill, pe - fill));               \
    fill += kRefill;                                                        \
    pend = true;                                                            \
  } while (0)
#define FU_RING_COMMIT()                                                    \
  do {                                                                      \
    ring[((rh + rv) & (kRing - 1)) * kBlock] = r0;                          \
    ring[((rh + rv + 1) & (kRing - 1)) * kBlock] = r1;                      \
    ring[((rh + rv + 2) & (kRing - 1)) * kBlock] = r2;                      \
    ring[((rh + rv + 3) & (kRing - 1)) * kBlock] = r3;                      \
    ring[((rh + rv + 4) & (kRing - 1)) * kBlock] = r4;                      \
    ring[((rh + rv + 5) & (kRing - 1)) * kBlock] = r5;                      \
    ring[((rh + rv + 6) & (kRing - 1)) * kBlock] = r6;                      \
    ring[((rh + rv + 7) & (kRing - 1)) * kBlock] = r7;                      \
    rv += pcnt;                                                             \
    pend = false;                                                           \
  } while (0)
  static_assert(kRefill == 8, "eight refill registers");
  FU_RING_REFILL();
  FU_RING_COMMIT();
  FU_RING_REFILL();
  FU_RING_COMMIT();
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(pay, 0, 0x7FFFFFF0, 0x00020000);
  const int scratch = n_uid + node;  // this node's scratch slot (idle polls and stores)
  // two polls in flight: the payloads of the lane's next two receives (slots pa, pb)
  unsigned long long ax = kMsgSentinel, ay = kMsgSentinel, bx = kMsgSentinel, by = kMsgSentinel;
  int pa = -1, pb = -1;
  auto ld16 = [&](int msg, unsigned long long &x, unsigned long long &y) {  // 16-byte sc1 load
    const u4 w = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(prs, msg * 16, 0, 16));
    x = (unsigned long long)w.x | ((unsigned long long)w.y << 32);
    y = (unsigned long long)w.z | ((unsigned long long)w.w << 32);
  };
  // a message = one 16-byte sc1 store (write-through, aux 16) of {flow, avg}: one fabric write
  // instead of two 8-byte ones (narrow sc1 stores cost 2.7x per byte, MI355X_MICROARCH.md)
  auto send = [&](int msg, double f, double a) {
    const unsigned long long fb = (unsigned long long)__double_as_longlong(f);
    const unsigned long long ab = (unsigned long long)__double_as_longlong(a);
    const u4 w = {(unsigned)fb, (unsigned)(fb >> 32), (unsigned)ab, (unsigned)(ab >> 32)};
    __builtin_amdgcn_raw_buffer_store_b128(w, prs, msg * 16, 0, 16);
  };
  // the slots of the first two receives among the ring's next kScan events (scratch if fewer;
  // scratch is never a message slot)
#define FU_NEXT_RECVS(ida, idb)                                              \
  do {                                                                       \
    ida = idb = scratch;                                                     \
    _Pragma("unroll") for (int j = 0; j < kScan; ++j) {                      \
      const int4 e = ev_dec(ring[((rh + j) & (kRing - 1)) * kBlock]);        \
      if (j < rv && e.w < tick_end && e.x == FU_EV_RECV) {                   \
        if (ida == scratch) ida = e.z;                                       \
        else if (idb == scratch) idb = e.z;                                  \
      }                                                                      \
    }                                                                        \
  } while (0)
  {
    int ia, ib;
    FU_NEXT_RECVS(ia, ib);
    pa = ia;
    ld16(ia, ax, ay);
    pb = ib;
    ld16(ib, bx, by);
    if (!CA) {
      send(scratch, 0.0, 0.0);
      send(scratch, 0.0, 0.0);
    }
  }
  long long it = 0;
  bool done = false;
  for (;;) {
    if (pend) FU_RING_COMMIT();
    const int4 h0 = ev_dec(ring[rh * kBlock]);
    done = rv > 0 ? h0.w >= tick_end : !pend && fill >= pe;
    if (__all(done)) break;
    bool prog = false;
    int o1 = scratch, o2 = scratch;  // the iteration's (at most two) pairwise messages
    double f1 = 0.0, a1 = 0.0, f2 = 0.0, a2 = 0.0;
    if (!done && rv > 0) {
      int m = 0;   // events run this iteration
      int nfo = 0; // pairwise fires this iteration
#pragma unroll
      for (int k = 0; k < kRW; ++k) {
        if (k >= rv) break;
        const int4 ev = k == 0 ? h0 : ev_dec(ring[((rh + k) & (kRing - 1)) * kBlock]);
        const int tk = ev.w;
        if (tk >= tick_end) break;
        unsigned long long mx = 0, my = 0;
        if (ev.x == FU_EV_RECV) {  // its payload must be one of the two polls, arrived
          if (pa == ev.z && ax != kMsgSentinel && ay != kMsgSentinel) {
            mx = ax;
            my = ay;
            pa = -1;
          } else if (pb == ev.z && bx != kMsgSentinel && by != kMsgSentinel) {
            mx = bx;
            my = by;
            pb = -1;
          } else {
            break;  // not arrived (or not polled yet): polled again at the end
          }
        } else if (!CA && nfo == 2) {
          break;  // two pairwise messages per iteration
        }
        while (sc < n_snap && snap_ticks[sc] < tk) snaps[(long long)sc++ * n + node] = lst;
        if (ev.x == FU_EV_RECV) {  // CA:98-99 / PW:98-99
#pragma unroll
          for (int j = 0; j < MAXD; ++j)
            if (j == ev.y) {
              es[j] = __longlong_as_double((long long)my);
              fl[j] = -__longlong_as_double((long long)mx);
            }
        } else if (CA && ev.x == FU_EV_FIRE_CA) {  // CA:105-125
          const int kk = ev.y;
          double S = 0.0, T = 0.0;
#pragma unroll
          for (int j = 0; j < MAXD; ++j)
            if (j < kk) S = S + fl[j];
          const double estimate = val - S;
#pragma unroll
          for (int j = 0; j < MAXD; ++j)
            if (j < kk) T = T + es[j];
          const double avg = (estimate + T) / (double)(kk + 1);
          lst = avg;
#pragma unroll
          for (int j = 0; j < MAXD; ++j)
            if (j < kk) {
              const double nf = (fl[j] + avg) - es[j];
              fl[j] = nf;
              es[j] = avg;
              send(out_uid[ev.z + j], nf, avg);
            }
        } else {  // FIRE_PW, PW:102-117: y = slot | k << 8
          const int sl = ev.y & 0xFF, kk = ev.y >> 8;
          double S = 0.0, fs = 0.0, esl = 0.0;
#pragma unroll
          for (int j = 0; j < MAXD; ++j) {
            if (j < kk) S = S + fl[j];
            if (j == sl) {
              fs = fl[j];
              esl = es[j];
            }
          }
          const double estimate = val - S;
          const double avg = (esl + estimate) / 2.0;
          lst = avg;
          const double nf = (fs + avg) - esl;
#pragma unroll
          for (int j = 0; j < MAXD; ++j)
            if (j == sl) {
              fl[j] = nf;
              es[j] = avg;
            }
          if (CA) {
            send(ev.z, nf, avg);
          } else if (nfo == 0) {
            o1 = ev.z;
            f1 = nf;
            a1 = avg;
          } else {
            o2 = ev.z;
            f2 = nf;
            a2 = avg;
          }
          ++nfo;
        }
        ++m;
      }
      if (m) {
        p += m;
        rh = (rh + m) & (kRing - 1);
        rv -= m;
        prog = true;
      }
    }
    if (!pend && rv <= kRing - kRefill && fill < pe) FU_RING_REFILL();  // lands during the next pass
    {  // the youngest operations, in this order every iteration: two polls, then two stores
      int ia, ib;
      FU_NEXT_RECVS(ia, ib);
      pa = ia;
      ld16(ia, ax, ay);
      pb = ib;
      ld16(ib, bx, by);
      if (!CA) {
        send(o1, f1, a1);
        send(o2, f2, a2);
      }
    }
    if (!__any(prog)) __builtin_amdgcn_s_sleep(kReplaySleep);
    if (++it > max_iters) {  // bounded spin: a bug must end the kernel, not hang the GPU
      atomicExch(status, 1);
      break;
    }
  }
  if (done)
    while (sc < n_snap && snap_ticks[sc] < tick_end) snaps[(long long)sc++ * n + node] = lst;
#pragma unroll
  for (int j = 0; j < MAXD; ++j)
    if (j < deg) {
      flow[rb + j] = fl[j];
      est[rb + j] = es[j];
    }
  cursor[node] = p;
  scur[node] = sc;
  last[node] = lst;
}
#undef FU_RING_REFILL
#undef FU_RING_COMMIT
#undef FU_NEXT_RECVS


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

// One round's launch context (state of round r-1 -> round r).
struct RoundCtx {
  int64_t r;
  int fm;                     // flow mode: rounds 1, 2 compute the old flows instead of reading them
  double *F;                  // F[r & 1]: f_{r-2} in, f_r out
  const double *ap, *ap2;     // a_{r-1}, a_{r-2}
  double *an;                 // a_r
  unsigned long long *err;    // error slot (nullptr: no check)
  bool plan;                  // a packing plan from a_{r-1} is still to run
};

// ======================================================================================
// handle
// ======================================================================================
constexpr int kPreMarks = 12;  // fu_mark slots created with the handle (a window's marks)

struct fu_handle {
  int device = 0;
  // layout 1 (fu_create_from_graph_ex): device node p = caller node old_of_new[p]; the
  // caller's row pointer maps flows back (rows moved as blocks)
  std::vector<int32_t> h_new_of_old;
  std::vector<int64_t> h_orig_rowptr;
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;            // kernel 4's heavy tiles, concurrently (fork_heavy)
  hipEvent_t ev0 = nullptr, ev1 = nullptr;  // autotune timing
  hipEvent_t ev2 = nullptr, ev3 = nullptr;  // fu_run_collectall_timed
  hipEvent_t marks[64] = {};                // fu_mark slots (the first kPreMarks at creation, others on first use)
  hipEvent_t r0_start = nullptr;            // fu_run_collectall_marked: mark 0 = the start of k_round0,
  hipEvent_t r0_stop = nullptr;             //   mark 1 (when it follows round 0) = its end
  hipEvent_t ev_pw = nullptr, ev_fork = nullptr, ev_join = nullptr;
  int32_t n = 0;
  int64_t E = 0;
  int32_t na = 0;  // estimate slots: n local + ghost estimates (multi-GPU)
  int32_t max_deg = 0;
  int *rowptr = nullptr, *col = nullptr;
  int *blk_row = nullptr;  // round 0: row of edge b * kR0E for every block b, then of edge E - 1
  unsigned short *col16 = nullptr;  // kernel 4 narrow tiles: col - cbase[e >> 10] + 32768 (0 where wide)
  int *cbase = nullptr;             // per 1024-edge block: its first edge's row, or -1 (a column >= 32K ids away)
  std::vector<int32_t> h_cbase;
  double *v = nullptr;
  double *f[2] = {nullptr, nullptr};           // F[r & 1]: f_{r-2} in, f_r out (split words)
  double *a[3] = {nullptr, nullptr, nullptr};  // A[r % 3] = a_r
  double *target = nullptr;
  unsigned long long *err = nullptr;
  int errcap = 0;
  double *ftmp = nullptr;
  int64_t rounds = 0;
  int kernel = 4;        // 4 = recon (LDS tiles), 8 = stage (LDS-staged slices + recon tiles)
  int geo = 1;           // kernel 4 tile geometry (kGeoEdges x kGeoNodes)
  int hub_threshold = 128;  // rows above it run as heavy rows (R-MAT-24: 128 beat 64, 256, 512)
  int mega_hub = 8192;   // degree above which a row's (fr, er) pairs are staged by many blocks
  int wave_heavy = 1;    // kernel 4: heavy rows one per wave
  int mid_heavy = 1;     // kernel 9: heavy rows of <= 64 x kMidRL edges in a register-resident launch
  int tr_bpx = 32;       // kernel 9: k_transpose blocks per XCD (1 per CU), each looping over buckets; 0 = one per bucket
  int staged_lo = 1;     // kernel 8: staged indices loaded before the flows (LO)
  int c16 = 1;           // kernel 4: narrow light tiles read 2-byte column offsets
  int multi_mid = 1;     // kernel 9: k_heavy_multi also takes the register launch's rows (257-1024)
  int split_hubs = 1;     // kernel 4: mega-hub tiles alone on the side stream
  int fork_heavy = 1;    // kernel 4: heavy tiles on stream2, concurrently with the light tiles
  bool autotune = true;  // kernel "auto": candidates timed on real rounds, fastest kept
  bool tuned = false;
  bool tune_for_width = false;  // the pending pass was armed by a packing-width change (poll_pack_width)
  bool tuning = false;     // inside an autotune pass: packing plans wait until it ends
  float tune_ms[8] = {};  // per candidate (tune_cands order), ms per round of the last pass
  int tune_out[8] = {};   // passes in which the candidate was > 1.3x the best (2: dropped)
  int n_tunes = 0;        // autotune passes so far (re-run when the packing width changes)
  int tuned_width = 0;    // packing width the last pass ran under
  int tune_cache[4] = {-1, -1, -1, -1};  // winner per packing width (0, 8, 16, 32), kept across fu_reset
  int *h_pw = nullptr;    // pinned copy of the plan's width, refreshed after each plan
  void *h_xfer[2] = {nullptr, nullptr};           // pinned bounce buffers of copy_out (kXfer bytes each)
  hipEvent_t ev_xfer[2] = {nullptr, nullptr};
  bool pw_pending = false;
  int *pw_dev = nullptr;      // h_pw as the device sees it (the plan kernels write the width there)
  bool plan_pending = false;  // a packing plan is due before the next round (from its table)
  std::vector<int64_t> h_rowptr;
  std::vector<int32_t> h_col;
  // kernel 4 tiles per geometry (all four built up front so autotuning can switch between
  // rounds): mega hubs, heavy rows, then light tiles
  int4 *tiles_geo[4] = {nullptr, nullptr, nullptr, nullptr};
  int *tnar_geo[4] = {nullptr, nullptr, nullptr, nullptr};  // per tile: narrow (col16) or not (int: a scalar load)
  int ntiles_geo[4] = {0, 0, 0, 0};
  int nheavy_geo[4] = {0, 0, 0, 0};  // leading non-light tiles
  int nbound_geo[4] = {0, 0, 0, 0};  // multi-GPU: light tiles with ghost neighbours, right after the heavy ones
  int niso_geo[4] = {0, 0, 0, 0};    // kernel 9: trailing light tiles of isolated rows only (k_isolated runs them)
  int iso0_geo[4] = {0, 0, 0, 0};    // ... their first row (rows [iso0, n) are isolated)
  FP::Tiles tiles1;                  // host copy of geometry 1's plan (kernel 9's schedule)
  int mid_geo[4][2] = {};            // heavy tiles [mid_geo[0], mid_geo[1]) lead with a row of 64 x (kHeavyRL, kMidRL] edges
  int multi_geo[4][2] = {};          // hrows offset and count of this geometry's sorted heavy rows
  int multi_heavy = 1;               // kernel 9: rows > 64 x kHeavyRL as k_heavy_multi blocks
  double *halo_a = nullptr;          // multi-GPU: the estimate buffer the round being launched writes
  std::vector<int32_t> h_hrows;
  int *hrows = nullptr;  // heavy rows of the wave-per-row tiles, longest first (per geometry)
  int n_hub = 0;
  int64_t hub_total = 0;
  int4 *hub_rows = nullptr;  // {node, row begin, row end, offset in hubxy}
  int *hub_blk = nullptr;    // per 256-edge block of the hub edges: the hub of its first edge
  int iso_rows = 1;           // kernel 9: trailing isolated-row tiles as k_isolated (1) or as light tiles (0)
  int multi_short = 1;        // kernel 9: the rows of 129-256 edges in the multi-row blocks too (1)
  int tr_nt = 1;              // kernel 9: non-temporal G_B stores in k_transpose (1)
  int *hub_off = nullptr;    // per mega tile: offset in hubxy
  double2 *hubxy = nullptr;  // (fr, er) per hub edge, staged each round
  // packed estimate table (see PackCtl): code[r & 1] = codes of a_r
  unsigned char *code[2] = {nullptr, nullptr};
  PackCtl *pctl = nullptr;  // [0], [1]: per code table; [2]: current encoding plan
  int *psample = nullptr;   // gather targets sampled for the plan
  int n_psample = 0;
  int pack = 1;             // 0 = off
  int pack_every = 16;      // rounds between encoding plans
  int tile_edges = 1024;    // option shadow of geo
  int tile_nodes = 0;
  bool has_target = false;
  // kernel 8 (LDS-staged slices): light tiles of kStageTE x kStageTN, heavy rows as kernel 4
  // heavy tiles, one slice layout per table element width
  struct StageLayout {
    int P = 0, Q = 0, SN = 0, NB = 0;     // slices, blocks per slice, nodes per slice, blocks (P = 0: not built)
    int4 *brange = nullptr;               // per stage block: {begin, end} in G, slice, 0
    unsigned short *colS = nullptr;       // per G element: column offset in its slice
    unsigned short *sidx16 = nullptr;     // per light-tile edge (slice order): position | run << 10
    int *dtab = nullptr;                  // per light tile: kStageRuns run offsets (G index - m)
  };
  StageLayout st[4];                      // element bytes 1, 2, 4, 8
  bool st_ready = false;
  std::string st_why;                     // why no layout could be built (kernel 8 unavailable)
  int4 *st_tiles = nullptr;               // light tiles
  int st_ntiles = 0;
  int st_nbound = 0;                      // multi-GPU: leading light tiles with ghost neighbours
  int4 *st_heavy = nullptr;               // rows above the tile limit ({i, -1, b, e})
  int st_nheavy = 0;
  void *stG = nullptr;                    // staged estimates, 8 B per G element
  int seen_width = 0;                     // packing width the host last saw
  int st_force = -1;                      // tests: force layout 0..3 (element bytes 1, 2, 4, 8)
  std::vector<FP::I4> h_light;            // host copy (layout construction)
  // kernel 9 (pregather): slice-major G_A, per-bucket run starts, edge-order Gb
  struct TransLayout {
    int P = 0, Q = 0, NB = 0, B = 0;      // slices, blocks per slice, stage blocks, buckets
    int Bh = 0;                           // buckets [0, Bh) hold the mega-hub rows' edges
    int Bm = 0;                           // buckets [0, Bm) hold every edge of the k_heavy_multi rows
    int4 *brange = nullptr;               // stage blocks: {begin, end} in G_A, slice, 0
    unsigned short *colS = nullptr;       // per G_A element: column offset in its slice
    unsigned short *pos16 = nullptr;      // per G_A element: position in its bucket
    int *offT = nullptr;                  // (B + 1) x P: G_A index where bucket b's run of slice s starts
    double *GA = nullptr;
    double *GBr[3] = {nullptr, nullptr, nullptr};  // G_B of round r in GBr[r % 3] (one buffer without lag)
    double *hist[2] = {nullptr, nullptr};          // lag: per parity, a_{r-2} of every lagged row
  };
  TransLayout tr;
  bool tr_ready = false;
  // kernel 9 option "lag" (k_heavy_multi<LAG>): per parity p, lagf[p] = F[p] holds f_{r'-2}
  // (not f_{r'}) on the lagged rows, r' = lag_round[p] the last round of that parity; the
  // lagged rows: lag_nmulti[p] heavy rows
  int lag = 1;
  int lagf[2] = {0, 0};
  int64_t lag_round[2] = {0, 0};
  int lag_nmulti[2] = {0, 0};
  std::string tr_why;
  int n_cu = 256;
  void *dist = nullptr;  // multi-GPU (fu_dist.hip)
};

extern "C" int fu__dist_round_hook(fu_handle *h, int phase);
extern "C" void fu__dist_free(fu_handle *h);
extern "C" int fu__dist_agree(fu_handle *h, int ok_local, int *ok_all);

namespace {


// The handle's graph as the host plans see it (fu_plan.h).
FP::Graph plan_graph(const fu_handle *h) {
  FP::Graph g;
  g.n = h->n;
  g.na = h->na;
  g.E = h->E;
  g.rowptr = h->h_rowptr.data();
  g.col = h->h_col.data();
  g.cbase = h->h_cbase.data();
  return g;
}

// host vector -> fresh device array (at least one element)
template <typename D, typename S>
int upload(D **dst, const std::vector<S> &src) {
  static_assert(sizeof(D) == sizeof(S), "upload: element layouts differ");
  if (*dst) hipFree(*dst);
  *dst = nullptr;
  if (int rc = dmalloc(dst, std::max<size_t>(1, src.size()))) return rc;
  if (!src.empty()) HIP_TRY(hipMemcpy(*dst, src.data(), sizeof(S) * src.size(), hipMemcpyHostToDevice));
  return FU_OK;
}

// Kernel 4 tiles of geometry g (FP::build_tiles_geom: mega hubs, heavy rows, light tiles, the
// trailing degree-0 rows), uploaded; the heavy rows are appended to h_hrows.
int build_tiles_geom(fu_handle *h, int geo) {
  FP::TileOpts o;
  o.hub_threshold = h->hub_threshold;
  o.mega_hub = h->mega_hub;
  o.wave_heavy = h->wave_heavy;
  FP::Tiles t;
  std::string why;
  if (!FP::build_tiles_geom(plan_graph(h), kGeoEdges[geo], kGeoNodes[geo], o, h->h_hrows, t, &why))
    return fail(FU_ERR_STATE, why);
  if (int rc = upload(&h->tiles_geo[geo], t.all)) return rc;
  if (int rc = upload(&h->tnar_geo[geo], t.narrow)) return rc;
  h->ntiles_geo[geo] = (int)t.all.size();
  h->nheavy_geo[geo] = t.nheavy;
  h->nbound_geo[geo] = t.nbound;
  h->mid_geo[geo][0] = t.mid[0];
  h->mid_geo[geo][1] = t.mid[1];
  h->multi_geo[geo][0] = t.multi[0];
  h->multi_geo[geo][1] = t.multi[1];
  h->niso_geo[geo] = t.niso;
  h->iso0_geo[geo] = t.iso0;
  if (geo == 1) h->tiles1 = t;
  return FU_OK;
}

// Mega-hub side arrays (same rows, same order as the -3 tiles of build_tiles_geom).
int build_hubs(fu_handle *h) {
  for (void *p : {(void *)h->hub_rows, (void *)h->hub_off, (void *)h->hubxy, (void *)h->hub_blk})
    if (p) hipFree(p);
  h->hub_blk = nullptr;
  h->hub_rows = nullptr;
  h->hub_off = nullptr;
  h->hubxy = nullptr;
  FP::Hubs hb;
  FP::build_hubs(plan_graph(h), h->mega_hub, hb);
  h->n_hub = (int)hb.rows.size();
  h->hub_total = hb.total;
  if (hb.rows.empty()) return FU_OK;
  if (int rc = upload(&h->hub_rows, hb.rows)) return rc;
  if (int rc = upload(&h->hub_off, hb.off)) return rc;
  if (int rc = dmalloc(&h->hubxy, (size_t)hb.total)) return rc;
  return upload(&h->hub_blk, hb.blk);
}

void free_transpose(fu_handle *h);
int lag_finalize_all(fu_handle *h);

int build_tiles(fu_handle *h) {
  if (int rc = lag_finalize_all(h)) return rc;  // the lagged rows' flows, before their lists change
  free_transpose(h);  // its hub exclusion follows the tiles
  h->h_hrows.clear();
  for (int g = 0; g < 4; ++g)
    if (int rc = build_tiles_geom(h, g)) return rc;
  if (h->hrows) hipFree(h->hrows);
  h->hrows = nullptr;
  if (int rc = dmalloc(&h->hrows, std::max<size_t>(1, h->h_hrows.size()))) return rc;
  if (!h->h_hrows.empty())
    HIP_TRY(hipMemcpy(h->hrows, h->h_hrows.data(), sizeof(int32_t) * h->h_hrows.size(), hipMemcpyHostToDevice));
  return build_hubs(h);
}

// Current estimate / flow buffers (A[r % 3] and F[r & 1] of the last round r).
inline double *cur_a(fu_handle *h) { return h->a[(int)((h->rounds + 2) % 3)]; }
inline double *cur_f(fu_handle *h) { return h->f[(int)((h->rounds + 1) & 1)]; }

// ---- kernel 8 preparation -------------------------------------------------------------

// Light tiles (kStageTE x kStageTN) and the rows above the tile limit (kernel 8).
int ensure_light(fu_handle *h) {
  if (h->st_tiles) return FU_OK;
  FP::StageLight sl;
  FP::build_stage_light(plan_graph(h), h->hub_threshold, sl);
  h->st_nbound = sl.nbound;
  h->h_light = sl.light;
  if (int rc = upload(&h->st_tiles, sl.light)) return rc;
  if (int rc = upload(&h->st_heavy, sl.heavy)) return rc;
  h->st_ntiles = (int)sl.light.size();
  h->st_nheavy = (int)sl.heavy.size();
  return FU_OK;
}

// The staged-estimate buffer G and the four slice layouts (element bytes 1, 2, 4, 8; slice =
// kStageLds / bytes nodes; FP::build_stage_layouts). A tile's edges of one slice are one
// contiguous run of G: per edge the round kernel reads u16 {position, run} and per tile the
// run offsets D (G index = m + D[run], m = index in slice order).
int ensure_stage(fu_handle *h) {
  if (h->st_ready) return FU_OK;
  if (!h->st_why.empty()) return fail(FU_ERR_GRAPH, h->st_why);
  if (int rc = ensure_light(h)) return rc;
  FP::StageLayout L[4];
  std::string why;
  if (!FP::build_stage_layouts(plan_graph(h), h->h_light, h->n_cu, L, &why)) {
    h->st_why = why;
    return fail(FU_ERR_GRAPH, why);
  }
  int64_t gmax = 16;
  for (int li = 0; li < 4; ++li) {
    auto &D = h->st[li];
    for (void *p : {(void *)D.brange, (void *)D.colS, (void *)D.sidx16, (void *)D.dtab})
      if (p) hipFree(p);
    D = fu_handle::StageLayout{};
    if (!L[li].P) continue;
    if (int rc = upload(&D.brange, L[li].brange)) return rc;
    if (int rc = upload(&D.colS, L[li].colS)) return rc;
    if (int rc = upload(&D.sidx16, L[li].sidx16)) return rc;
    if (int rc = upload(&D.dtab, L[li].dtab)) return rc;
    D.P = L[li].P;
    D.Q = L[li].Q;
    D.SN = L[li].SN;
    D.NB = L[li].NB;
    gmax = std::max<int64_t>(gmax, L[li].total);
  }
  if (int rc = dmalloc(reinterpret_cast<unsigned long long **>(&h->stG), (size_t)gmax)) return rc;
  HIP_TRY(hipMemset(h->stG, 0, sizeof(unsigned long long) * (size_t)gmax));
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
    sa.SN[li] = L.SN;
    sa.NB[li] = L.NB;
    sa.brange[li] = L.brange;
    sa.colS[li] = L.colS;
    sa.sidx16[li] = L.sidx16;
    sa.dtab[li] = L.dtab;
    if (L.P) g = std::max<unsigned>(g, (unsigned)L.NB);
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

// Kernel 9 preparation (see k_transpose): slices of 16K nodes, buckets of kTrBE edges. G_A:
// slice-major, within a slice in edge order, each slice's region starting at a multiple of
// 16 (the stage launch stores 16 bytes per lane); offT[b * P + s] = where bucket b's run of
// slice s starts (offT[B * P + s]: the end of slice s's elements); stage blocks cut each
// slice's region into Q pieces.
void free_transpose(fu_handle *h) {
  auto &T = h->tr;
  for (void *p : {(void *)T.brange, (void *)T.colS, (void *)T.pos16, (void *)T.offT, (void *)T.GA,
                  (void *)T.GBr[0], (void *)T.hist[0], (void *)T.hist[1]})
    if (p) hipFree(p);
  if (T.GBr[1] != T.GBr[0]) hipFree(T.GBr[1]);
  if (T.GBr[2] != T.GBr[0]) hipFree(T.GBr[2]);
  T = fu_handle::TransLayout{};
  h->tr_ready = false;
}

int ensure_transpose(fu_handle *h) {
  if (h->tr_ready) return FU_OK;
  if (!h->tr_why.empty()) return fail(FU_ERR_GRAPH, h->tr_why);
  FP::TransPlan tp;
  std::string why;
  const int32_t *mrows = h->h_hrows.empty() ? nullptr : h->h_hrows.data() + h->multi_geo[1][0];
  if (!FP::build_transpose(plan_graph(h), h->mega_hub, h->n_cu, mrows, h->multi_geo[1][1], tp, &why)) {
    h->tr_why = why;
    return fail(FU_ERR_GRAPH, why);
  }
  auto &T = h->tr;
  if (int rc = upload(&T.brange, tp.brange)) return rc;
  if (int rc = upload(&T.colS, tp.colS)) return rc;
  if (int rc = upload(&T.pos16, tp.pos)) return rc;
  if (int rc = upload(&T.offT, tp.offT)) return rc;
  if (int rc = dmalloc(&T.GA, (size_t)tp.total)) return rc;
  // G_B: a ring of three with lag (round r reads G_B of round r - 2 for the lagged rows)
  for (int k = 0; k < 3; ++k) {
    if (k && !h->lag) {
      T.GBr[k] = T.GBr[0];
      continue;
    }
    if (int rc = dmalloc(&T.GBr[k], (size_t)h->E)) return rc;
  }
  for (int p = 0; p < 2; ++p)
    if (int rc = dmalloc(&T.hist[p], (size_t)(h->multi_geo[1][1] + 1))) return rc;
  T.P = tp.P;
  T.Q = tp.Q;
  T.NB = tp.NB;
  T.B = tp.B;
  T.Bh = tp.Bh;
  T.Bm = tp.Bm;
  h->tr_ready = true;
  return FU_OK;
}

inline unsigned grid_for(long long work) { return (unsigned)((work + kBlock - 1) / kBlock); }

// Kernel 9 "lag": write the flows parity p's last round r' left unwritten on its lagged rows
// (k_lag_final: F[p] holds f_{r'-2}; G_B of r' is GBr[r' % 3], a_{r'} is A[r' % 3]). Valid
// while r' is one of the last two rounds (the A ring holds a_{r'}; no kernel-9 round has
// reused r''s G_B slot), which holds at every call site: before a round of another kernel,
// fu_get_flows, a tile rebuild, the option's change.
int lag_finalize(fu_handle *h, int p) {
  if (!h->lagf[p]) return FU_OK;
  const int64_t rr = h->lag_round[p];
  if (h->rounds - rr < 1 || h->rounds - rr > 2)  // A[rr % 3] or G_B[rr % 3] already reused
    return fail(FU_ERR_STATE, "lag_finalize: lagged round " + std::to_string(rr) + " is not one of the last two (" +
                                  std::to_string(h->rounds) + " rounds done)");
  const double *Gb = h->tr.GBr[rr % 3];
  const double *a = h->a[rr % 3];
  if (h->lag_nmulti[p])
    hipLaunchKernelGGL(k_lag_final, dim3(h->lag_nmulti[p]), dim3(kBlock), 0, h->stream, h->hrows + h->multi_geo[1][0],
                       h->rowptr, h->f[p], Gb, h->tr.hist[p], a);
  HIP_TRY(hipGetLastError());
  h->lagf[p] = 0;
  return FU_OK;
}
int lag_finalize_all(fu_handle *h) {
  for (int p = 0; p < 2; ++p)
    if (int rc = lag_finalize(h, p)) return rc;
  return FU_OK;
}

// k_transpose grid for nbk buckets: 8 XCDs x min(buckets per XCD, tr_bpx blocks per XCD)
// (tr_bpx 0: one block per bucket)
inline unsigned tr_grid(fu_handle *h, int nbk) {
  const int per = (nbk + 7) / 8;
  return 8u * (unsigned)(h->tr_bpx > 0 ? std::min(per, h->tr_bpx) : per);
}


// the packing plan as a one-block launch ahead of the round (paths without a stage launch)
void plan_alone(fu_handle *h, RoundCtx &c) {
  if (!c.plan) return;
  hipLaunchKernelGGL(k_pack_plan, dim3(1), dim3(kBlock), 0, h->stream, c.ap, h->psample, h->pctl, h->pw_dev);
  c.plan = false;
}

// Round 0 = the timeout fire on zero state (CA:33-34, CA:87-91): a_0 and a_{-1} = 0.0; no
// flows are written (rounds 1 and 2 compute f_{-1} and f_0 themselves: fm).
int launch_round0(fu_handle *h, RoundCtx &c) {
  static_assert(sizeof(PackCtl) * 3 == 6 * sizeof(unsigned long long), "k_round0 clears 3 PackCtl");
  h->lagf[0] = h->lagf[1] = 0;  // zero state: no lagged flows
  if (h->r0_start) {  // a timed window's first mark: the kernel's own start (hipExtLaunchKernel)
    hipExtLaunchKernelGGL(k_round0, dim3(grid_for(std::max(h->na, 6))), dim3(kBlock), 0, h->stream, h->r0_start,
                          h->r0_stop, 0, h->n, h->na, (const int *)h->rowptr, (const double *)h->v, h->a[0], h->a[2],
                          reinterpret_cast<unsigned long long *>(h->pctl));
    h->r0_start = h->r0_stop = nullptr;
  } else {
    hipLaunchKernelGGL(k_round0, dim3(grid_for(std::max(h->na, 6))), dim3(kBlock), 0, h->stream, h->n, h->na,
                       h->rowptr, h->v, h->a[0], h->a[2], reinterpret_cast<unsigned long long *>(h->pctl));
  }
  if (c.err)
    hipLaunchKernelGGL(k_max_err, dim3(std::min(1024u, grid_for(h->n))), dim3(kBlock), 0, h->stream, h->n,
                       h->a[0], h->target, c.err);
  if (h->dist) {  // a_0 of the boundary nodes to the peers
    h->halo_a = h->a[0];
    if (int rc = fu__dist_round_hook(h, 2)) return rc;
  }
  return FU_OK;
}

// Kernel 8: k_stage (carrying the packing plan), heavy rows as kernel 4 tiles, then the light
// tiles reading the staged estimates.
int launch_k8(fu_handle *h, RoundCtx &c) {
  constexpr bool C0 = false;
  const int r1 = (int)(c.r & 1);
  unsigned sgrid = 1;
  const StageArgs sa = stage_args(h, &sgrid);
  const void *cp = h->code[(c.r - 1) & 1];
  if (h->st_ntiles) {
    hipLaunchKernelGGL(k_stage, dim3(sgrid + (c.plan ? 8 : 0)), dim3(kStageThreads), 0, h->stream, sa, h->na, c.ap, cp,
                       h->pctl, r1, h->stG, c.plan ? h->psample : nullptr, h->pw_dev);
    c.plan = false;
  }
  plan_alone(h, c);
  auto heavy = [&](auto chk) {
    hipLaunchKernelGGL((k_round_recon<decltype(chk)::value, kStageTE, kStageTN>), dim3(h->st_nheavy),
                       dim3(kBlock), 0, h->stream, h->st_heavy, h->rowptr, h->col, h->v, c.F, c.ap, c.ap2, c.an,
                       h->target, c.err, cp, h->code[r1], h->pctl, r1, nullptr, nullptr, nullptr, 0, nullptr, c.fm);
  };
  if (h->st_nheavy) {
    if (c.err) heavy(std::true_type{});
    else heavy(std::false_type{});
  }
  // light tiles: rounds 1 and 2 (fm) read no flows (RF = false); LO = staged indices first
  // multi-GPU: the boundary tiles [0, st_nbound), then the halo goes out on the comm stream
  // beside the interior tiles
  auto light = [&](auto chk, auto rf, auto lo) -> int {
    // multi-GPU: the boundary tiles [0, st_nbound), then the rest
    const int nb = h->dist ? h->st_nbound : 0;
    for (int part = 0; part < 2; ++part) {
      const int t0 = part ? nb : 0, cnt = part ? h->st_ntiles - nb : nb;
      if (cnt)
        hipLaunchKernelGGL((k_round_staged<decltype(chk)::value, kStageTE, kStageTN, decltype(rf)::value,
                                           decltype(lo)::value>),
                           dim3(cnt), dim3(kBlock), 0, h->stream, h->st_tiles, t0, cnt, h->rowptr, h->col, sa,
                           h->stG, h->v, c.F, c.ap, c.ap2, c.an, h->target, c.err, h->code[r1], h->pctl, r1, c.fm);
      if (!part && h->dist) {  // boundary rows (and the heavy rows) done
        h->halo_a = c.an;
        if (int rc = fu__dist_round_hook(h, 2)) return rc;
      }
    }
    return FU_OK;
  };
  auto light_lo = [&](auto chk, auto rf) {
    return h->staged_lo ? light(chk, rf, std::true_type{}) : light(chk, rf, std::false_type{});
  };
  auto light_rf = [&](auto chk) {
    return c.fm ? light_lo(chk, std::false_type{}) : light_lo(chk, std::true_type{});
  };
  if (h->st_ntiles || h->dist) {
    if (c.err) return light_rf(std::true_type{});
    return light_rf(std::integral_constant<bool, C0>{});
  }
  return FU_OK;
}

// Kernel 9: k_stage -> k_transpose (the mega-hub buckets first) -> kernel 4's tiles reading
// the pre-gathered estimates; the mega hubs' chains and k_hub_flows on the side stream beside
// the remaining buckets and tiles.
int launch_k9(fu_handle *h, RoundCtx &c) {
  if (int rc = ensure_transpose(h)) return rc;  // rebuilt after a tile option changed
  double *Gb = h->tr.GBr[c.r % 3];
  const double *Gb_old = h->tr.GBr[(c.r + 1) % 3];  // G_B of round r - 2 (lag)
  if (!Gb) return fail(FU_ERR_STATE, "kernel 9: no pre-gather buffer");
  const int r1 = (int)(c.r & 1);
  const void *cp = h->code[(c.r - 1) & 1];
  // which launch computes which rows (FP::k9_schedule; tools/plan_check.cpp replays it)
  FP::K9Opts ko;
  ko.mid_heavy = h->mid_heavy;
  ko.multi_mid = h->multi_mid;
  ko.multi_short = h->multi_short;
  ko.multi_heavy = h->multi_heavy;
  ko.wave_heavy = h->wave_heavy;
  ko.iso_rows = h->iso_rows;
  const FP::K9Sched ks = FP::k9_schedule(h->tiles1, h->n_hub, ko);
  const int nmega = ks.nmega, nh = ks.nh, niso = ks.niso, nl = ks.nl, m0 = ks.m0, m1 = ks.m1;
  const int4 *tl = h->tiles_geo[1];
  const bool hubs = nmega > 0;
  // lag: the rows this round leaves their flows to round r + 2 (k_heavy_multi<LAG>): the
  // multi-row heavy rows
  const int n_multi = ks.n_multi, m1s = ks.m1s;
  const bool multi = ks.multi;
  const bool lag_multi = h->lag && multi;
  const int p = r1;
  if (h->lagf[p] && h->lag_nmulti[p] != (lag_multi ? n_multi : 0)) {
    if (int rc = lag_finalize(h, p)) return rc;  // the lagged set changed: write its flows first
  }
  const int lagm = lag_multi ? (h->lagf[p] ? 2 : 1) : 0;
  StageArgs sa{};
  for (int li = 0; li < 4; ++li) sa.sel[li] = 3;
  sa.P[3] = h->tr.P;
  sa.Q[3] = h->tr.Q;
  sa.SN[3] = kStageLds / 8;
  sa.NB[3] = h->tr.NB;
  sa.brange[3] = h->tr.brange;
  sa.colS[3] = h->tr.colS;
  sa.f64 = 1;
  {
    hipLaunchKernelGGL(k_stage, dim3(h->tr.NB + (c.plan ? 8 : 0)), dim3(kStageThreads), 0, h->stream, sa, h->na, c.ap,
                       cp, h->pctl, r1, h->tr.GA, c.plan ? h->psample : nullptr, h->pw_dev);
    c.plan = false;
  }
  plan_alone(h, c);
  const int bh = hubs ? h->tr.Bh : 0;
  auto tr_launch = [&](int b0, int nb) {
    if (h->tr_nt)
      hipLaunchKernelGGL(k_transpose<true>, dim3(tr_grid(h, nb)), dim3(kTrThreads), 0, h->stream, b0, nb, h->tr.P,
                         (long long)h->E, h->tr.offT, h->tr.GA, h->tr.pos16, Gb);
    else
      hipLaunchKernelGGL(k_transpose<false>, dim3(tr_grid(h, nb)), dim3(kTrThreads), 0, h->stream, b0, nb, h->tr.P,
                         (long long)h->E, h->tr.offT, h->tr.GA, h->tr.pos16, Gb);
  };
  if (bh) tr_launch(0, bh);
  if (hubs) {
    HIP_TRY(hipEventRecord(h->ev_fork, h->stream));
    HIP_TRY(hipStreamWaitEvent(h->stream2, h->ev_fork, 0));
  }
  if (h->tr.B > bh) tr_launch(bh, h->tr.B - bh);
  const bool chk = c.err != nullptr;
  if (hubs) {
    auto chains = [&](auto C) {
      hipLaunchKernelGGL((k_round_recon<decltype(C)::value, 1024, 128, 2, true>), dim3(nmega), dim3(kBlock),
                         0, h->stream2, tl, h->rowptr, h->col, h->v, c.F, c.ap, c.ap2, c.an, h->target, c.err, cp,
                         h->code[r1], h->pctl, r1, nullptr, nullptr, h->hrows, 1, Gb, c.fm);
    };
    if (chk) chains(std::true_type{});
    else chains(std::false_type{});
    hipLaunchKernelGGL(k_hub_flows, dim3(grid_for(h->hub_total)), dim3(kBlock), 0, h->stream2, h->n_hub, h->hub_rows,
                       (long long)h->hub_total, nullptr, c.an, c.F, Gb, c.ap2, c.fm, h->hub_blk);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(h->ev_join, h->stream2));
  }
  // heavy tiles [t0, t1) with RL register elements per lane
  auto heavy = [&](auto C, auto RL, int t0, int t1) {
    if (t1 > t0)
      hipLaunchKernelGGL((k_round_recon<decltype(C)::value, 1024, 128, 2, true, decltype(RL)::value>),
                         dim3(t1 - t0), dim3(kBlock), 0, h->stream, tl + t0, h->rowptr, h->col, h->v, c.F, c.ap, c.ap2,
                         c.an, h->target, c.err, cp, h->code[r1], h->pctl, r1, h->hubxy, h->hub_off, h->hrows, 1, Gb,
                         c.fm);
  };
  // the rows of the heavy tiles [nmega, m1) (4 rows each, longest first: every row of more
  // than 64 x kHeavyRL edges, and the few shorter ones sharing the last tile) as
  // k_heavy_multi blocks, many rows per chain wave
  // (multi_mid = 0: only the rows of [nmega, m0), longer than the register launch's; the rows
  // of [m0, m1) then stay in registers, one pass)
  auto tiles = [&](auto C) {
    if (multi) {
      auto hm = [&](auto L) {
        hipLaunchKernelGGL((k_heavy_multi<decltype(C)::value, decltype(L)::value>), dim3((n_multi + kMR - 1) / kMR),
                           dim3(kBlock), 0, h->stream, h->hrows + h->multi_geo[1][0], n_multi,
                           h->rowptr, h->v, c.F, c.ap2, c.an, h->target, c.err, h->code[r1], h->pctl, Gb, c.fm, Gb_old,
                           h->tr.hist[p]);
      };
      if (!lag_multi) hm(std::integral_constant<int, 0>{});
      else if (lagm == 1) hm(std::integral_constant<int, 1>{});
      else hm(std::integral_constant<int, 2>{});
      if (!h->multi_mid) heavy(C, std::integral_constant<int, kMidRL>{}, m0, m1);
    } else {
      heavy(C, std::integral_constant<int, kHeavyRL>{}, nmega, m0);
      heavy(C, std::integral_constant<int, kMidRL>{}, m0, m1);
    }
    heavy(C, std::integral_constant<int, kHeavyRL>{}, m1s, nh);
    if (niso)
      hipLaunchKernelGGL(k_isolated, dim3(grid_for(h->n - h->iso0_geo[1])), dim3(kBlock), 0, h->stream,
                         h->iso0_geo[1], h->n, h->v, c.an, h->target, c.err, h->code[r1], h->pctl, r1,
                         decltype(C)::value ? 1 : 0);
    if (nl)
      hipLaunchKernelGGL((k_round_recon<decltype(C)::value, 1024, 128, 1, true>), dim3(nl), dim3(kBlock), 0,
                         h->stream, tl + nh, h->rowptr, h->col, h->v, c.F, c.ap, c.ap2, c.an, h->target, c.err, cp,
                         h->code[r1], h->pctl, r1, nullptr, nullptr, nullptr, 0, Gb, c.fm);
  };
  if (chk) tiles(std::true_type{});
  else tiles(std::false_type{});
  HIP_TRY(hipGetLastError());
  if (hubs) HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_join, 0));
  if (h->dist) {  // multi-GPU: boundary rows sit in every row class, so a_r goes out after the round
    h->halo_a = c.an;
    if (int rc = fu__dist_round_hook(h, 2)) return rc;
  }
  if (lagm) {  // F[p] now holds f_{r-2} on the lagged rows; round r + 2 (or lag_finalize) writes f_r
    h->lagf[p] = 1;
    h->lag_round[p] = c.r;
    h->lag_nmulti[p] = lag_multi ? n_multi : 0;
  }
  return FU_OK;
}

// Kernel 4: heavy tiles (mega hubs, heavy rows) lead the tile list; with fork_heavy they run
// on the side stream beside the light tiles' launch (which keeps kernel 4's light-path
// register budget). Multi-GPU: the heavy tiles stay on the main stream, then the boundary
// light tiles, then the halo goes out beside the interior light tiles.
template <int TE, int TN>
int launch_k4_geo(fu_handle *h, RoundCtx &c) {
  const int r1 = (int)(c.r & 1);
  const void *cp = h->code[(c.r - 1) & 1];
  const int nh = h->nheavy_geo[h->geo], nl = h->ntiles_geo[h->geo] - nh;
  const int hub_sep = h->n_hub ? 1 : 0;  // k_hub_flows writes the hubs' flows after the chains
  const int nb = h->nbound_geo[h->geo];  // boundary light tiles (multi-GPU), then the interior
  const bool fork = nh > 0 && h->fork_heavy && !h->dist;
  hipStream_t hs = fork ? h->stream2 : h->stream;
  // with mega hubs, only their tiles go to the side stream (k_hub_stage -> chains ->
  // k_hub_flows), so the other heavy tiles need not wait for k_hub_stage
  const int nmh = fork && h->n_hub && h->split_hubs ? h->n_hub : nh;
  const int4 *tiles = h->tiles_geo[h->geo];
  if (fork) {
    HIP_TRY(hipEventRecord(h->ev_fork, h->stream));
    HIP_TRY(hipStreamWaitEvent(h->stream2, h->ev_fork, 0));
  }
  if (h->n_hub)
    hipLaunchKernelGGL(k_hub_stage, dim3(grid_for(h->hub_total)), dim3(kBlock), 0, hs, h->n_hub, h->hub_rows,
                       (long long)h->hub_total, h->col, c.F, c.ap, c.ap2, cp, h->pctl, r1, h->hubxy, c.fm, h->hub_blk);
  auto heavy = [&](auto C, hipStream_t st, int t0, int cnt) {
    if (cnt)
      hipLaunchKernelGGL((k_round_recon<decltype(C)::value, TE, TN, 2>), dim3(cnt), dim3(kBlock), 0, st,
                         tiles + t0, h->rowptr, h->col, h->v, c.F, c.ap, c.ap2, c.an, h->target, c.err, cp, h->code[r1],
                         h->pctl, r1, h->hubxy, h->hub_off, h->hrows, hub_sep, nullptr, c.fm);
  };
  // light tiles: rounds 1 and 2 (fm) read no flows (RF = false)
  auto light = [&](auto C, auto RF, int t0, int cnt) {
    if (cnt)
      hipLaunchKernelGGL((k_round_recon<decltype(C)::value, TE, TN, 1, false, kHeavyRL,
                                        decltype(RF)::value>),
                         dim3(cnt), dim3(kBlock), 0, h->stream, tiles + t0, h->rowptr, h->col, h->v, c.F, c.ap, c.ap2,
                         c.an, h->target, c.err, cp, h->code[r1], h->pctl, r1, nullptr, nullptr, nullptr, 0, nullptr,
                         c.fm, h->col16, h->cbase, h->c16 ? h->tnar_geo[h->geo] + t0 : nullptr);
  };
  auto light_rf = [&](auto C, int t0, int cnt) {
    if (c.fm) light(C, std::false_type{}, t0, cnt);
    else light(C, std::true_type{}, t0, cnt);
  };
  auto body = [&](auto C) -> int {
    heavy(C, hs, 0, nmh);             // mega hubs (or every heavy tile) on the side stream
    heavy(C, h->stream, nmh, nh - nmh);  // the other heavy tiles ahead of the light ones
    light_rf(C, nh, nb);
    if (h->dist) {  // boundary rows done: their estimates go out beside the interior tiles
      h->halo_a = c.an;
      if (int rc = fu__dist_round_hook(h, 2)) return rc;
    }
    light_rf(C, nh + nb, nl - nb);
    return FU_OK;
  };
  int rc;
  if (c.err) rc = body(std::true_type{});
  else rc = body(std::false_type{});
  if (rc) return rc;
  if (hub_sep)
    hipLaunchKernelGGL(k_hub_flows, dim3(grid_for(h->hub_total)), dim3(kBlock), 0, hs, h->n_hub, h->hub_rows,
                       (long long)h->hub_total, h->hubxy, c.an, c.F, nullptr, nullptr, c.fm, h->hub_blk);
  if (fork) {
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(h->ev_join, h->stream2));
    HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_join, 0));
  }
  return FU_OK;
}

int launch_k4(fu_handle *h, RoundCtx &c) {
  plan_alone(h, c);
  if (h->geo == 0) return launch_k4_geo<2048, 256>(h, c);
  if (h->geo == 2) return launch_k4_geo<1024, 256>(h, c);
  if (h->geo == 1) return launch_k4_geo<1024, 128>(h, c);
  return launch_k4_geo<512, 64>(h, c);
}

// The round body of rounds >= 1 for the handle's kernel.
int launch_body(fu_handle *h, RoundCtx &c) {
  if (h->kernel == 8) return launch_k8(h, c);
  if (h->kernel == 9) return launch_k9(h, c);
  return launch_k4(h, c);
}

// One round: state of round r-1 -> round r. err_slot: nullptr = no check.
int launch_round(fu_handle *h, unsigned long long *err_slot) {
  if (h->dist) {
    if (int rc = fu__dist_round_hook(h, 0)) return rc;
  }
  const int64_t r = h->rounds;
  RoundCtx c;
  c.r = r;
  c.fm = r == 1 ? 1 : r == 2 ? 2 : 0;  // rounds 1, 2: the old flows are computed, not read
  c.F = h->f[r & 1];
  c.ap = r > 0 ? h->a[(r - 1) % 3] : nullptr;
  c.ap2 = h->a[(r + 1) % 3];
  c.an = h->a[r % 3];
  c.err = err_slot;
  // a packing plan due from a_{r-1}: the stage launch of kernels 8 and 9 carries it (one more
  // block); every other path runs it first as a launch of its own
  // (held back during an autotune pass, so every candidate runs at the pass's width; any plan
  // is lossless, so a late one changes nothing but the table's width)
  c.plan = h->plan_pending && r > 0 && !h->tuning;
  if (!h->tuning) h->plan_pending = false;
  const bool plan_done = c.plan;
  int rc;
  // kernel 9's lag: another kernel reads F[r & 1] as f_{r-2}, so the lagged rows' flows of
  // round r - 2 are written first
  if (r > 0 && h->kernel != 9 && h->lagf[r & 1]) {
    if (int rc2 = lag_finalize(h, (int)(r & 1))) return rc2;
  }
  if (r == 0) rc = launch_round0(h, c);
  else rc = launch_body(h, c);
  if (rc) return rc;
  HIP_TRY(hipGetLastError());
  if (plan_done && !h->pw_pending) {  // the autotuner watches the width (poll_pack_width)
    HIP_TRY(hipEventRecord(h->ev_pw, h->stream));
    h->pw_pending = true;
  }
  h->rounds++;
  // a packing plan from a_r is due: the next round runs it ahead of its round kernels (on
  // its stage launch where it has one) and encodes a_{r+1} with it; once the host has seen
  // the narrowest width (8), every 8th time only
  const int every = h->seen_width == 8 ? 8 * h->pack_every : h->pack_every;
  if (h->pack && !h->dist && h->n_psample > 0 && h->rounds % every == 0) h->plan_pending = true;
  return FU_OK;
}

// Autotune candidates, fixed order (fu_get_info reports per index). Kernel 8 is single-GPU.
using FP::kCands;
using FP::kNCands;
using FP::kTimed;
using FP::TuneCand;
static int width_class(int w) { return w == 8 ? 1 : w == 16 ? 2 : w == 32 ? 3 : 0; }
static void use_cand(fu_handle *h, const TuneCand &c) {
  h->kernel = c.kernel;
  h->geo = c.geo;
}
int ensure_transpose(fu_handle *h);

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

// Internal constructor shared by fu_create / fu_dist_create: uploads the local CSR. The
// kernels never read a reverse-edge index (flows are reconstructed, kernel 4 §4.1), so only
// rowptr, col and the values go to the device. a_extra: ghost estimate slots (multi-GPU).
int fu__create_common(int32_t n, int64_t e, const int64_t *rowptr, const int32_t *col,
                      const double *value, int32_t device, int32_t a_extra, fu_handle **out) {
  FU_TRY_BEGIN
  if (!out || n <= 0 || e < 0 || !rowptr || !value || (e > 0 && !col) || a_extra < 0)
    return fail(FU_ERR_ARG, "fu_create: bad arguments");
  if (e >= (int64_t)INT32_MAX - 64) return fail(FU_ERR_ARG, "fu_create: more than 2^31-1 edges");
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
  const int32_t na = n + a_extra;
  h->na = na;
  for (int64_t k = 0; k < e; ++k) {
    if (col[k] < 0 || col[k] >= na) {
      delete h;
      return fail(FU_ERR_ARG, "fu_create: col index out of range at edge " + std::to_string(k));
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
  // the marks a timed window uses (bench.py: up to 12) exist before any window starts: event
  // creation costs the host tens of microseconds, which a window must not contain
  for (int k = 0; k < kPreMarks; ++k)
    if (hipEventCreate(&h->marks[k]) != hipSuccess) return cleanup(fail(FU_ERR_HIP, "hipEventCreate failed"));
  if (hipHostMalloc(reinterpret_cast<void **>(&h->h_pw), sizeof(int), hipHostMallocDefault) != hipSuccess)
    return cleanup(fail(FU_ERR_ALLOC, "hipHostMalloc failed"));
  *h->h_pw = 0;
  if (hipHostGetDevicePointer(reinterpret_cast<void **>(&h->pw_dev), h->h_pw, 0) != hipSuccess)
    return cleanup(fail(FU_ERR_HIP, "hipHostGetDevicePointer failed"));
  const int64_t fe = std::max<int64_t>(32, (e + 31) / 32 * 32);  // split-word flows: whole 32-edge blocks (one at least: clamped loads read edge 0)
  if ((rc = dmalloc(&h->rowptr, n + 1)) || (rc = dmalloc(&h->col, e)) || (rc = dmalloc(&h->v, n)) ||
      (rc = dmalloc(&h->f[0], fe)) || (rc = dmalloc(&h->f[1], fe)) || (rc = dmalloc(&h->a[0], na)) ||
      (rc = dmalloc(&h->a[1], na)) || (rc = dmalloc(&h->a[2], na)) || (rc = dmalloc(&h->target, n)) ||
      (rc = dmalloc(&h->err, 1)))
    return cleanup(rc);
  h->errcap = 1;
  if (hipMemcpy(h->rowptr, rp32.data(), sizeof(int) * (n + 1), hipMemcpyHostToDevice) != hipSuccess ||
      (e && hipMemcpy(h->col, col, sizeof(int) * e, hipMemcpyHostToDevice) != hipSuccess) ||
      hipMemcpy(h->v, value, sizeof(double) * n, hipMemcpyHostToDevice) != hipSuccess)
    return cleanup(fail(FU_ERR_HIP, "fu_create: upload failed"));
  if ((e == 0 && hipMemset(h->col, 0, sizeof(int)) != hipSuccess) ||
      hipMemset(h->f[0], 0, sizeof(double) * std::max<int64_t>(fe, 1)) != hipSuccess ||
      hipMemset(h->f[1], 0, sizeof(double) * std::max<int64_t>(fe, 1)) != hipSuccess ||
      hipMemset(h->a[0], 0, sizeof(double) * na) != hipSuccess || hipMemset(h->a[1], 0, sizeof(double) * na) != hipSuccess ||
      hipMemset(h->a[2], 0, sizeof(double) * na) != hipSuccess)
    return cleanup(fail(FU_ERR_HIP, "fu_create: memset failed"));
  {  // round 0's per-block rows; kernel 4's 2-byte column offsets (FP::build_blocks)
    std::vector<int32_t> br;
    std::vector<uint16_t> c16;
    FP::build_blocks(n, e, rowptr, col, br, h->h_cbase, c16);
    if ((rc = upload(&h->blk_row, br)) || (rc = upload(&h->col16, c16)) || (rc = upload(&h->cbase, h->h_cbase)))
      return cleanup(rc);
  }
  if ((rc = build_tiles(h))) return cleanup(rc);
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

// The flow reconstruction needs every i -> j to have its j -> i: a caller's rev is checked to
// be that pairing; without one, fu::build_rev checks symmetry (the index itself is not kept).
int fu_create(int32_t n, int64_t e, const int64_t *rowptr, const int32_t *col,
              const int32_t *rev, const double *value, int32_t device, fu_handle **out) {
  FU_TRY_BEGIN
  if (!rowptr || n <= 0 || e < 0 || (e > 0 && !col)) return fail(FU_ERR_ARG, "fu_create: bad arguments");
  if (rowptr[0] != 0 || rowptr[n] != e) return fail(FU_ERR_ARG, "fu_create: rowptr[0] must be 0 and rowptr[n] == e");
  if (e > 0 && !rev) {
    fu_graph g;
    g.n = n;
    g.rowptr.assign(rowptr, rowptr + n + 1);
    g.col.assign(col, col + e);
    if (int rc = fu::build_rev(g)) return rc;
  } else if (e > 0) {
    for (int32_t i = 0; i < n; ++i)
      for (int64_t k = rowptr[i]; k < rowptr[i + 1]; ++k) {
        const int32_t j = col[k];
        const int64_t r = rev[k];
        if (j < 0 || j >= n || r < rowptr[j] || r >= rowptr[j + 1] || col[r] != i)
          return fail(FU_ERR_GRAPH, "fu_create: rev is not the reverse-edge pairing (the graph must be symmetric) at edge " +
                                        std::to_string(k));
      }
  }
  return fu__create_common(n, e, rowptr, col, value, device, 0, out);
  FU_TRY_END
}

int fu_create_from_graph(const fu_graph *g, const double *value, int32_t device,
                         fu_handle **out) {
  if (!g) return fail(FU_ERR_ARG, "fu_create_from_graph: NULL graph");
  const int64_t E = g->rowptr[g->n];
  if ((int64_t)g->rev.size() != E) return fail(FU_ERR_GRAPH, "fu_create_from_graph: graph is not symmetric");
  return fu__create_common(g->n, E, g->rowptr.data(), g->col.data(), value, device, 0, out);
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
  FU_TRY_BEGIN
  if (!h || !key) return fail(FU_ERR_ARG, "fu_set_option: NULL argument");
  if (int rc = set_device(h)) return rc;
  if (!std::strcmp(key, "kernel")) {
    if (value != 0 && value != 4 && value != 8 && value != 9)
      return fail(FU_ERR_ARG, "fu_set_option: kernel must be 0 (auto), 4 (recon), 8 (stage) or 9 (pregather)");
    if (h->rounds != 0) return fail(FU_ERR_STATE, "fu_set_option: kernel can only change before the first round (call fu_reset)");
    int rc = FU_OK;
    if (value == 8) rc = ensure_stage(h);
    if (value == 9) rc = ensure_transpose(h);  // the slice limit counts ghost slots: rank-dependent
    if (h->dist) {  // RCCL ranks: a kernel that fails on one rank fails on all (collective)
      const std::string why = rc ? fu_last_error() : "";
      int all_ok = 1;
      if (int rc2 = fu__dist_agree(h, rc == FU_OK, &all_ok)) return rc2;
      if (rc) return fail(rc, why);
      if (!all_ok) return fail(FU_ERR_STATE, "fu_set_option: kernel " + std::to_string(value) + " failed on another rank");
    }
    if (rc) return rc;
    if (value == 9) h->geo = 1;
    h->kernel = value == 0 ? 4 : (int)value;
    h->autotune = value == 0;
    h->tuned = false;
    h->tune_for_width = false;
    return FU_OK;
  }
  if (!std::strcmp(key, "stage_layout")) {  // kernel 8: -1 = by packing width, 0..3 forced
    if (value < -1 || value > 3) return fail(FU_ERR_ARG, "fu_set_option: stage_layout must be -1..3");
    h->st_force = (int)value;
    return FU_OK;
  }
  if (!std::strcmp(key, "pack")) {
    h->pack = value != 0;
    if (!h->pack) {  // stop encoding (and drop a plan still due)
      h->plan_pending = false;
      HIP_TRY(hipMemsetAsync(h->pctl + 2, 0, sizeof(PackCtl), h->stream));
    }
    return FU_OK;
  }
  if (!std::strcmp(key, "pack_every")) {
    if (value < 1 || value > (1 << 20)) return fail(FU_ERR_ARG, "fu_set_option: pack_every must be in [1, 2^20]");
    h->pack_every = (int)value;
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
  if (!std::strcmp(key, "fork_heavy")) {  // kernel 4: heavy tiles on a side stream (1) or in order (0)
    h->fork_heavy = value != 0;
    return FU_OK;
  }
  if (!std::strcmp(key, "split_hubs")) {  // kernel 4: mega-hub tiles alone on the side stream (1)
    h->split_hubs = value != 0;
    return FU_OK;
  }
  if (!std::strcmp(key, "staged_lo")) {  // kernel 8: staged indices before the flows (1) or interleaved (0)
    h->staged_lo = value != 0;
    return FU_OK;
  }
  if (!std::strcmp(key, "tr_bpx")) {  // kernel 9: transpose blocks per XCD (0 = one per bucket)
    if (value < 0 || value > 1 << 20) return fail(FU_ERR_ARG, "fu_set_option: tr_bpx must be in [0, 2^20]");
    h->tr_bpx = (int)value;
    return FU_OK;
  }
  if (!std::strcmp(key, "lag")) {  // kernel 9: the multi-row heavy rows write f_r in round r + 2
    const int lv = value != 0;
    if (lv != h->lag) {
      if (int rc = lag_finalize_all(h)) return rc;  // flows first, with the current G_B ring
      free_transpose(h);                            // the ring's size follows the option
      h->lag = lv;
    }
    return FU_OK;
  }
  if (!std::strcmp(key, "tr_nt")) {  // kernel 9: k_transpose stores G_B non-temporally (1)
    if (value != 0 && value != 1) return fail(FU_ERR_ARG, "fu_set_option: tr_nt must be 0 or 1");
    h->tr_nt = (int)value;
    return FU_OK;
  }
  if (!std::strcmp(key, "multi_short")) {  // kernel 9: rows of 129-256 edges as multi-row blocks (1)
    h->multi_short = value != 0;
    return FU_OK;
  }
  if (!std::strcmp(key, "iso_rows")) {  // kernel 9: trailing isolated rows one thread each (1) or as tiles (0)
    h->iso_rows = value != 0;
    return FU_OK;
  }
  if (!std::strcmp(key, "multi_heavy")) {  // kernel 9: rows > 256 edges with many rows per chain wave (1)
    h->multi_heavy = value != 0;
    return FU_OK;
  }
  if (!std::strcmp(key, "c16")) {  // kernel 4: 2-byte column offsets for narrow light tiles (1) or not (0)
    h->c16 = value != 0;
    return FU_OK;
  }
  if (!std::strcmp(key, "multi_mid")) {  // kernel 9: rows of 257-1024 edges in k_heavy_multi (1) or in registers (0)
    h->multi_mid = value != 0;
    return FU_OK;
  }
  if (!std::strcmp(key, "mid_heavy")) {  // kernel 9: register-resident launch for rows of 257-1024 edges
    h->mid_heavy = value != 0;
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
    if (h->st_tiles) return fail(FU_ERR_STATE, "fu_set_option: hub_threshold must be set before kernel 8 is prepared");
    h->hub_threshold = (int)std::min<int64_t>(value, 2048);
    return build_tiles(h);
  }
  return fail(FU_ERR_ARG, std::string("fu_set_option: unknown key '") + key + "'");
  FU_TRY_END
}

int fu_reset(fu_handle *h) {
  FU_TRY_BEGIN
  if (!h) return fail(FU_ERR_ARG, "fu_reset: NULL handle");
  if (int rc = set_device(h)) return rc;
  if (h->dist) {  // phase 1: wait for the last halo, drain the comm stream, forget its rounds
    if (int rc = fu__dist_round_hook(h, 1)) return rc;
  }
  HIP_TRY(hipStreamSynchronize(h->stream));
  h->rounds = 0;
  h->lagf[0] = h->lagf[1] = 0;  // zero state: nothing lagged
  h->pw_pending = false;  // the stream is idle: no plan in flight
  h->plan_pending = false;  // round 0 clears the plan
  *h->h_pw = 0;           // round 0 clears the packing plan
  h->seen_width = 0;
  // unpacked again: its winner. A pass still pending for a width the rounds before the reset
  // reached (seen in calls too short for a pass) no longer applies; one armed by the kernel
  // option still runs.
  if (h->autotune && (h->tuned || h->tune_for_width) && h->tune_cache[0] >= 0) {
    use_cand(h, kCands[h->tune_cache[0]]);
    h->tuned_width = 0;
    h->tuned = true;
    h->tune_for_width = false;
  }
  return FU_OK;
  FU_TRY_END
}

int fu_set_targets(fu_handle *h, const double *target) {
  FU_TRY_BEGIN
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
  FU_TRY_END
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

// Kernels 4 (every geometry) and 8 share the state layout (F[r & 1], A[r % 3]) and are
// bitwise identical, so switching between them mid-run changes nothing but speed. "auto"
// times each candidate on real rounds (1 warm + 8 timed each) and keeps the fastest. The
// rounds count toward the caller's total and the results are unchanged. The pass re-runs
// when the packing plan changes width (the packed gather shifts the balance between the
// candidates), at most kMaxTunes times; fu_tune runs one pass on demand.
constexpr int kMaxTunes = 4;

static int autotune_kernel(fu_handle *h, int32_t *budget, int width) {
  // which candidate runs (FP::tune_steps): multi-GPU, every rank must run the same rounds
  // (each one is a halo exchange), so no candidate is dropped and none stops early on
  // rank-local timings (tools/plan_check --tune checks the count is rank-independent)
  FP::TuneRank tr;
  tr.dist = h->dist != nullptr;
  tr.width = width;
  for (int c = 0; c < kNCands; ++c) tr.tune_out[c] = h->tune_out[c];
  if (FP::tune_need(tr) > *budget) return FU_OK;  // not enough rounds in this call: try again later
  // the pass runs at the table's current width: the host's copy of it is exact once the stream
  // is idle, and no plan runs until the pass ends (h->tuning)
  HIP_TRY(hipStreamSynchronize(h->stream));
  h->pw_pending = false;
  h->seen_width = width = *h->h_pw;
  tr.width = width;
  if (FP::tune_need(tr) > *budget) return FU_OK;
  int steps[kNCands];
  FP::tune_steps(tr, steps);
  if (steps[2] != FP::kTuneSkip && ensure_stage(h) != FU_OK) {  // no slice layout fits this graph
    set_error("");
    tr.k8_ok = false;
  }
  if (steps[4] != FP::kTuneSkip && ensure_transpose(h) != FU_OK) {  // too many nodes for the slices
    set_error("");
    tr.k9_ok = false;
  }
  FP::tune_steps(tr, steps);
  const int32_t budget0 = *budget;
  h->tuning = true;
  struct Untune {
    fu_handle *h;
    ~Untune() { h->tuning = false; }
  } untune{h};
  float best = 1e30f;
  int bi = -1;
  for (int c = 0; c < kNCands; ++c) {
    if (!h->dist && h->tune_out[c] >= 2) continue;  // its last ns per round stays reported
    h->tune_ms[c] = 0.f;
    if (steps[c] == FP::kTuneSkip) continue;
    if (steps[c] == FP::kTuneStandIn) {
      // multi-GPU: this rank still runs the candidate's rounds (kernel 4), so that every
      // rank runs the same rounds (each is a halo exchange); its time is never the best
      use_cand(h, kCands[0]);
      for (int k = 0; k < 1 + kTimed; ++k)
        if (int rc = launch_round(h, nullptr)) return rc;
      *budget -= 1 + kTimed;
      h->tune_ms[c] = 1e30f;
      continue;
    }
    use_cand(h, kCands[c]);
    // the warm round is timed too: a candidate more than twice the best per-round time so far
    // stops there (on R-MAT-24 the staged kernel would take 3x kernel 4 for 8 rounds). The
    // events are recorded on an idle stream, so the warm round's time also holds the host's
    // first launch of the candidate's kernels; a slow warm round is therefore confirmed by a
    // second one, launched behind it, before the candidate is dropped
    HIP_TRY(hipEventRecord(h->ev0, h->stream));
    if (int rc = launch_round(h, nullptr)) return rc;
    HIP_TRY(hipEventRecord(h->ev1, h->stream));
    if (best < 1e30f && !h->dist) {
      HIP_TRY(hipEventSynchronize(h->ev1));
      float wms = 0.f;
      HIP_TRY(hipEventElapsedTime(&wms, h->ev0, h->ev1));
      *budget -= 1;
      if (wms > 2.f * best / kTimed) {
        HIP_TRY(hipEventRecord(h->ev0, h->stream));
        if (int rc = launch_round(h, nullptr)) return rc;
        if (int rc = launch_round(h, nullptr)) return rc;
        HIP_TRY(hipEventRecord(h->ev1, h->stream));
        HIP_TRY(hipEventSynchronize(h->ev1));
        HIP_TRY(hipEventElapsedTime(&wms, h->ev0, h->ev1));
        *budget -= 2;
        if (wms > 2.f * 2.f * best / kTimed) {
          h->tune_ms[c] = wms / 2.f;
          continue;
        }
      }
      *budget += 1;  // counted below with the timed rounds
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
      bi = c;
    }
  }
  if (bi < 0) return fail(FU_ERR_STATE, "autotune: no candidate ran");
  if (h->dist && budget0 - *budget != FP::tune_rounds_fixed(tr))
    return fail(FU_ERR_STATE, "autotune: a multi-GPU pass ran " + std::to_string(budget0 - *budget) + " rounds, not " +
                                  std::to_string(FP::tune_rounds_fixed(tr)) + " (the ranks would diverge)");
  for (int c = 0; c < kNCands; ++c)
    if (h->tune_ms[c] > 1.3f * h->tune_ms[bi]) h->tune_out[c]++;
  use_cand(h, kCands[bi]);
  h->tune_cache[width_class(width)] = bi;
  h->tuned_width = width;
  h->tuned = true;
  h->tune_for_width = false;
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
    use_cand(h, kCands[cached]);
    h->tuned_width = *h->h_pw;
  } else if (h->n_tunes < kMaxTunes) {
    h->tuned = false;
    h->tune_for_width = true;
  }
}

// The round loop shared by fu_run_collectall and fu_run_collectall_timed.
static int run_rounds(fu_handle *h, int32_t rounds, int32_t err_every, int nerr) {
  for (int32_t r = 0; r < rounds; ++r) {
    poll_pack_width(h);
    // tune between rounds when no error slot is pending in the rounds it would consume
    if (h->autotune && !h->tuned && h->rounds >= 1 && nerr == 0) {
      int32_t budget = rounds - r;
      const int w = h->pw_pending ? h->tuned_width : *h->h_pw;
      if (int rc = autotune_kernel(h, &budget, w)) return rc;
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
  if (h->dist) {  // the last round's halo (comm stream) inside the timed window
    if (int rc = fu__dist_round_hook(h, 0)) return rc;
  }
  HIP_TRY(hipEventRecord(h->ev3, h->stream));
  HIP_TRY(hipEventSynchronize(h->ev3));
  HIP_TRY(hipEventElapsedTime(ms, h->ev2, h->ev3));
  return FU_OK;
  FU_TRY_END
}

// A timed window in one host call: mark k (HIP event slot k) is recorded once rounds_at[k]
// rounds of this call have been queued (rounds_at[0] = 0: before the first). A window that
// starts with round 0 (after fu_reset, single GPU) takes mark 0 from k_round0's own start and,
// when mark 1 follows round 0, mark 1 from its end (hipExtLaunchKernel's start / stop events):
// an event recorded on the idle stream ahead of the launch would time-stamp at once and hold
// the first dispatch's latency, and a marker behind it its own ~5 us, in round 0's time.
int fu_run_collectall_marked(fu_handle *h, int32_t n_marks, const int32_t *rounds_at) {
  FU_TRY_BEGIN
  if (!h || !rounds_at || n_marks < 1 || n_marks > 64 || rounds_at[0] < 0)
    return fail(FU_ERR_ARG, "fu_run_collectall_marked: bad arguments (1..64 marks, rounds_at[0] >= 0)");
  for (int k = 1; k < n_marks; ++k)
    if (rounds_at[k] < rounds_at[k - 1]) return fail(FU_ERR_ARG, "fu_run_collectall_marked: rounds_at must not decrease");
  if (int rc = set_device(h)) return rc;
  for (int k = 0; k < n_marks; ++k)
    if (!h->marks[k]) HIP_TRY(hipEventCreate(&h->marks[k]));
  int32_t done = 0;
  const bool r0 = rounds_at[0] == 0 && n_marks > 1 && rounds_at[1] > 0 && h->rounds == 0 && !h->dist;
  const bool r0_end = r0 && rounds_at[1] == 1;
  for (int k = 0; k < n_marks; ++k) {
    if (rounds_at[k] > done) {
      if (int rc = run_rounds(h, rounds_at[k] - done, 0, 0)) {
        h->r0_start = h->r0_stop = nullptr;  // a failed call leaves no event armed for a later round 0
        return rc;
      }
      done = rounds_at[k];
    }
    if (h->dist) {  // a mark after a round includes that round's halo (comm stream)
      if (int rc = fu__dist_round_hook(h, 0)) return rc;
    }
    if (k == 0 && r0) {  // recorded by round 0's own launch
      h->r0_start = h->marks[0];
      if (r0_end) h->r0_stop = h->marks[1];
    } else if (!(k == 1 && r0_end)) {
      HIP_TRY(hipEventRecord(h->marks[k], h->stream));
    }
  }
  if (h->r0_start) {  // round 0 did not launch through launch_round0: never the case
    h->r0_start = h->r0_stop = nullptr;
    return fail(FU_ERR_STATE, "fu_run_collectall_marked: round 0 was not launched");
  }
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
  return FU_OK;
  FU_TRY_END
}

int fu_mark(fu_handle *h, int32_t slot) {
  if (!h || slot < 0 || slot >= 64) return fail(FU_ERR_ARG, "fu_mark: slot must be in [0, 64)");
  if (int rc = set_device(h)) return rc;
  if (!h->marks[slot]) HIP_TRY(hipEventCreate(&h->marks[slot]));
  if (h->dist) {  // a mark after a round includes that round's halo (comm stream)
    if (int rc = fu__dist_round_hook(h, 0)) return rc;
  }
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
  FU_TRY_BEGIN
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
  FU_TRY_END
}

// Device memory -> the caller's (pageable) host memory through two pinned kXfer-byte
// buffers: the DMA of chunk k runs while the host copies chunk k-1 out. A pageable
// hipMemcpyAsync stages through the runtime's own buffers one at a time (ER-1M's 8 MB of
// estimates: 31 ms on the box, profiles/r05/g/).
constexpr size_t kXfer = (size_t)4 << 20;

static int copy_out(fu_handle *h, void *dst, const void *src, size_t bytes) {
  for (int k = 0; k < 2; ++k) {
    if (!h->h_xfer[k] && hipHostMalloc(&h->h_xfer[k], kXfer, hipHostMallocDefault) != hipSuccess)
      return fail(FU_ERR_ALLOC, "hipHostMalloc (copy-out buffer) failed");
    if (!h->ev_xfer[k] && hipEventCreateWithFlags(&h->ev_xfer[k], hipEventDisableTiming) != hipSuccess)
      return fail(FU_ERR_HIP, "hipEventCreate failed");
  }
  const size_t nk = (bytes + kXfer - 1) / kXfer;
  for (size_t k = 0; k <= nk; ++k) {
    if (k < nk) {  // chunk k into buffer k & 1 (its previous chunk, k - 2, was copied out at k - 1)
      const size_t len = std::min(kXfer, bytes - k * kXfer);
      HIP_TRY(hipMemcpyAsync(h->h_xfer[k & 1], static_cast<const char *>(src) + k * kXfer, len,
                             hipMemcpyDeviceToHost, h->stream));
      HIP_TRY(hipEventRecord(h->ev_xfer[k & 1], h->stream));
    }
    if (k > 0) {  // chunk k - 1 out while chunk k is in flight
      const size_t j = k - 1, len = std::min(kXfer, bytes - j * kXfer);
      HIP_TRY(hipEventSynchronize(h->ev_xfer[j & 1]));
      std::memcpy(static_cast<char *>(dst) + j * kXfer, h->h_xfer[j & 1], len);
    }
  }
  return FU_OK;
}

int fu_get_estimates(fu_handle *h, double *a_out) {
  FU_TRY_BEGIN
  if (!h || !a_out) return fail(FU_ERR_ARG, "fu_get_estimates: NULL argument");
  if (int rc = set_device(h)) return rc;
  if (!h->h_new_of_old.empty()) {  // device numbering -> caller numbering
    std::vector<double> a2(h->n);
    if (int rc = copy_out(h, a2.data(), cur_a(h), sizeof(double) * h->n)) return rc;
    for (int32_t i = 0; i < h->n; ++i) a_out[i] = a2[h->h_new_of_old[i]];
    return FU_OK;
  }
  return copy_out(h, a_out, cur_a(h), sizeof(double) * h->n);
  FU_TRY_END
}

int fu_get_flows(fu_handle *h, double *f_out) {
  FU_TRY_BEGIN
  if (!h || (!f_out && h->E)) return fail(FU_ERR_ARG, "fu_get_flows: NULL argument");
  if (h->E == 0) return FU_OK;
  if (h->rounds == 0) {  // no round yet: every flow is 0.0 (CA:33)
    std::memset(f_out, 0, sizeof(double) * (size_t)h->E);
    return FU_OK;
  }
  if (int rc = set_device(h)) return rc;
  if (!h->ftmp) {
    if (int rc = dmalloc(&h->ftmp, (size_t)h->E)) return rc;
  }
  if (h->rounds >= 2) {  // kernel 9's lag: the last round's flows of its lagged rows
    if (int rc = lag_finalize(h, (int)((h->rounds - 1) & 1))) return rc;
  }
  if (h->rounds == 1)  // round 0 writes no flows (fm): f_0 = (0.0 + a_0[i]) - 0.0 on demand
    hipLaunchKernelGGL(k_round0_flows, dim3((unsigned)((h->E + kR0E - 1) / kR0E)), dim3(kBlock), 0, h->stream,
                       (long long)h->E, h->rowptr, h->blk_row, h->a[0], h->f[0], nullptr);
  // split words -> doubles
  hipLaunchKernelGGL(k_unsplit, dim3(grid_for(h->E)), dim3(kBlock), 0, h->stream, (long long)h->E, cur_f(h), h->ftmp);
  HIP_TRY(hipGetLastError());
  const double *src = h->ftmp;
  if (!h->h_new_of_old.empty()) {  // rows back to the caller's order (blocks, same order inside)
    std::vector<double> f2(h->E);
    if (int rc = copy_out(h, f2.data(), src, sizeof(double) * h->E)) return rc;
    const auto &orp = h->h_orig_rowptr;
    for (int32_t i = 0; i < h->n; ++i) {
      const int64_t nb = h->h_rowptr[h->h_new_of_old[i]];
      std::memcpy(f_out + orp[i], f2.data() + nb, sizeof(double) * (orp[i + 1] - orp[i]));
    }
    return FU_OK;
  }
  return copy_out(h, f_out, src, sizeof(double) * h->E);
  FU_TRY_END
}

int fu_get_info(fu_handle *h, int64_t info[32]) {
  if (!h || !info) return fail(FU_ERR_ARG, "fu_get_info: NULL argument");
  for (int k = 0; k < 32; ++k) info[k] = 0;
  info[0] = h->kernel;
  info[1] = 0;  // (reserved: kernel 4's removed "nt" option)
  info[2] = h->autotune ? (h->tuned ? 2 : 1) : 0;
  info[3] = h->rounds;
  info[4] = kGeoEdges[h->geo];
  info[5] = kGeoNodes[h->geo];
  info[6] = h->n_tunes;
  info[7] = h->tuned_width;
  for (int k = 0; k < kNCands; ++k) info[8 + k] = (int64_t)((double)h->tune_ms[k] * 1e6);  // ns per round
  info[20] = h->n_hub;
  for (int k = 0; k < 4; ++k)  // autotune winner per packing width 0, 8, 16, 32 (kernel * 10 + geometry; -1 = none)
    info[23 + k] = h->tune_cache[k] < 0 ? -1 : kCands[h->tune_cache[k]].kernel * 10 + kCands[h->tune_cache[k]].geo;
  for (int li = 0; li < 4; ++li) info[27 + li] = h->st[li].P;  // kernel 8 slices per layout (0 = not built)
  return FU_OK;
}

int fu_get_pack(fu_handle *h, int32_t width[3]) {
  FU_TRY_BEGIN
  if (!h || !width) return fail(FU_ERR_ARG, "fu_get_pack: NULL argument");
  if (int rc = set_device(h)) return rc;
  if (h->plan_pending && h->rounds > 0) {  // the plan due after the last round, as the next round would run it
    hipLaunchKernelGGL(k_pack_plan, dim3(1), dim3(kBlock), 0, h->stream, cur_a(h), h->psample, h->pctl, h->pw_dev);
    HIP_TRY(hipGetLastError());
    h->plan_pending = false;
  }
  PackCtl p[3];
  HIP_TRY(hipMemcpyAsync(p, h->pctl, sizeof(p), hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(hipStreamSynchronize(h->stream));
  for (int k = 0; k < 3; ++k) width[k] = p[k].width;
  return FU_OK;
  FU_TRY_END
}

int fu_get_round(fu_handle *h, int64_t *rounds_done) {
  if (!h || !rounds_done) return fail(FU_ERR_ARG, "fu_get_round: NULL argument");
  *rounds_done = h->rounds;
  return FU_OK;
}

int fu_mem_info(int32_t device, int64_t *free_bytes, int64_t *total_bytes) {
  if (!free_bytes || !total_bytes) return fail(FU_ERR_ARG, "fu_mem_info: NULL argument");
  int nd = 0;
  if (hipGetDeviceCount(&nd) != hipSuccess || nd == 0) return fail(FU_ERR_HIP, "fu_mem_info: no HIP device visible");
  if (device < 0 || device >= nd) return fail(FU_ERR_ARG, "fu_mem_info: bad device");
  HIP_TRY(hipSetDevice(device));
  size_t fr = 0, tot = 0;
  HIP_TRY(hipMemGetInfo(&fr, &tot));
  *free_bytes = (int64_t)fr;
  *total_bytes = (int64_t)tot;
  return FU_OK;
}

int fu_copy_bandwidth(int32_t device, int64_t bytes, int32_t iters, double *gbs) {
  FU_TRY_BEGIN
  if (!gbs || bytes < 16 * 1024 || iters < 1) return fail(FU_ERR_ARG, "fu_copy_bandwidth: bad arguments");
  int nd = 0;
  if (hipGetDeviceCount(&nd) != hipSuccess || nd == 0) return fail(FU_ERR_HIP, "fu_copy_bandwidth: no HIP device visible");
  if (device < 0 || device >= nd) return fail(FU_ERR_ARG, "fu_copy_bandwidth: bad device");
  HIP_TRY(hipSetDevice(device));
  const long long cnt = bytes / 2 / 16;  // half read, half written
  float4 *a = nullptr, *b = nullptr;
  if (int rc = dmalloc(&a, (size_t)cnt)) return rc;
  if (int rc = dmalloc(&b, (size_t)cnt)) {
    hipFree(a);
    return rc;
  }
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int rc = FU_OK;
  float best = 1e30f;
  const unsigned grid = 8u * 256u * 8u;  // 8 blocks per CU, grid-stride
  if (hipMemset(a, 0, sizeof(float4) * cnt) != hipSuccess || hipEventCreate(&e0) != hipSuccess ||
      hipEventCreate(&e1) != hipSuccess)
    rc = fail(FU_ERR_HIP, "fu_copy_bandwidth: setup");
  for (int k = 0; rc == FU_OK && k <= iters; ++k) {  // the first copy warms up, untimed
    hipEventRecord(e0, nullptr);
    hipLaunchKernelGGL(k_copy4, dim3(grid), dim3(kBlock), 0, nullptr, cnt, a, b);
    hipEventRecord(e1, nullptr);
    float ms = 0.f;
    if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess)
      rc = fail(FU_ERR_HIP, "fu_copy_bandwidth: copy");
    else if (k > 0)
      best = std::min(best, ms);
  }
  if (e0) hipEventDestroy(e0);
  if (e1) hipEventDestroy(e1);
  hipFree(a);
  hipFree(b);
  if (rc) return rc;
  *gbs = 2.0 * 16.0 * (double)cnt / (best * 1e-3) / 1e9;
  return FU_OK;
  FU_TRY_END
}

int fu_synchronize(fu_handle *h) {
  if (!h) return fail(FU_ERR_ARG, "fu_synchronize: NULL handle");
  if (int rc = set_device(h)) return rc;
  if (h->dist) {
    if (int rc = fu__dist_round_hook(h, 0)) return rc;  // the stream waits for the last halo
  }
  HIP_TRY(hipStreamSynchronize(h->stream));
  return FU_OK;
}

int fu_destroy(fu_handle *h) {
  if (!h) return FU_OK;
  hipSetDevice(h->device);
  if (h->stream) hipStreamSynchronize(h->stream);
  if (h->stream2) hipStreamSynchronize(h->stream2);
  if (h->dist) fu__dist_free(h);
  std::vector<void *> ptrs = {h->rowptr, h->col, h->blk_row, h->v, h->f[0], h->f[1], h->a[0], h->a[1], h->a[2], h->target,
                              h->err, h->ftmp, h->tiles_geo[0], h->tiles_geo[1], h->tiles_geo[2], h->tiles_geo[3],
                              h->hrows, h->hub_rows, h->hub_off, h->hubxy, h->hub_blk, h->code[0], h->code[1], h->pctl,
                              h->psample, h->st_tiles, h->st_heavy, h->stG, h->col16, h->cbase,
                              h->tnar_geo[0], h->tnar_geo[1], h->tnar_geo[2], h->tnar_geo[3]};
  free_transpose(h);
  for (const auto &L : h->st) {
    ptrs.push_back(L.brange);
    ptrs.push_back(L.colS);
    ptrs.push_back(L.sidx16);
    ptrs.push_back(L.dtab);
  }
  for (void *p : ptrs)
    if (p) hipFree(p);
  for (hipEvent_t e : {h->ev0, h->ev1, h->ev2, h->ev3, h->ev_pw, h->ev_fork, h->ev_join, h->ev_xfer[0], h->ev_xfer[1]})
    if (e) hipEventDestroy(e);
  for (hipEvent_t e : h->marks)
    if (e) hipEventDestroy(e);
  if (h->h_pw) hipHostFree(h->h_pw);
  for (void *p : h->h_xfer)
    if (p) hipHostFree(p);
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
  int2 *node_evt = nullptr;  // register kernel: packed 8-byte events (ev_dec)
  int *node_tick = nullptr, *out_uid = nullptr, *scur = nullptr, *status = nullptr;
  unsigned long long *pay = nullptr;
  int64_t n_uid = 0;
  bool pers_ready = false;
  int64_t max_deg = 0;
  int pers_reg = 1;       // option "persistent_reg": one node per thread, state in registers
  bool reg_ok = false;    // degree <= kReplayRegDeg and every node's thread resident at once
  bool has_ca = false;    // the trace holds collect-all fires
};
constexpr int kReplayRegDeg = 16;

// The register variant for the trace: row registers for degree <= 8 or <= 16, the collect-all
// fire path only when the trace has one (both cost registers, and the variant must keep
// every node's thread resident).
using ReplayRegKernel = void (*)(int, int, const long long *, const int2 *, const int *, int,
                                 const long long *, const double *, double *, double *, double *,
                                 unsigned long long *, long long *, int *, int, const int *, double *, int *,
                                 long long);
static ReplayRegKernel replay_reg_kernel(const fu_replay *r) {
  if (r->max_deg <= 8) return r->has_ca ? k_replay_persist_reg<8, true> : k_replay_persist_reg<8, false>;
  return r->has_ca ? k_replay_persist_reg<16, true> : k_replay_persist_reg<16, false>;
}

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
  std::vector<int2> nevt(ne > 0 ? ne : 1);
  bool pack_ok = r->ticks < (1 << 20);  // the register kernel's 8-byte events: tick < 2^20, slot, k < 32
  std::vector<int32_t> ouid(r->h_out_ids.size() > 0 ? r->h_out_ids.size() : 1);
  std::vector<int64_t> slot_uid(r->n_msgs > 0 ? r->n_msgs : 1, -1);
  int64_t U = 0;
  for (int32_t t = 0; t < r->ticks; ++t) {
    for (int64_t q = r->h_tto[t]; q < r->h_tto[t + 1]; ++q) {
      const int32_t node = r->h_tasks[3 * q];
      for (int32_t p = r->h_tasks[3 * q + 1]; p < r->h_tasks[3 * q + 2]; ++p) {
        const int32_t *e = &r->h_events[4 * (int64_t)p];
        int4 o = make_int4(e[0], e[1], e[2], e[3]);
        r->has_ca |= e[0] == FU_EV_FIRE_CA;
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
        {
          const int sl = o.x == FU_EV_FIRE_CA ? 0 : o.y;
          const int kk = o.x == FU_EV_FIRE_CA ? o.y : o.x == FU_EV_FIRE_PW ? o.z : 0;
          pack_ok &= sl < 32 && kk < 32;
          nevt[pos[node]] = make_int2((int)((unsigned)o.x | (unsigned)(sl & 31) << 2 | (unsigned)(kk & 31) << 7 |
                                            (unsigned)t << 12),
                                      o.x == FU_EV_FIRE_PW ? o.w : o.z);
        }
        ntick[pos[node]++] = t;
      }
    }
  }
  r->n_uid = U;
  if (int rc = dmalloc(&r->node_off, n + 1)) return rc;
  if (int rc = dmalloc(&r->node_ev, nev.size())) return rc;
  if (int rc = dmalloc(&r->node_tick, ntick.size())) return rc;
  if (int rc = dmalloc(&r->node_evt, nevt.size())) return rc;
  if (int rc = dmalloc(&r->out_uid, ouid.size())) return rc;
  // slots [U, U + n): per-node scratch slots of the register kernel's idle polls and stores
  if (int rc = dmalloc(&r->pay, 2 * (size_t)(U + n))) return rc;
  if (int rc = dmalloc(&r->cursor, n)) return rc;
  if (int rc = dmalloc(&r->scur, n)) return rc;
  if (int rc = dmalloc(&r->status, 1)) return rc;
  HIP_TRY(hipMemcpy(r->node_off, off.data(), sizeof(int64_t) * (n + 1), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(r->node_ev, nev.data(), sizeof(int4) * nev.size(), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(r->node_tick, ntick.data(), sizeof(int32_t) * ntick.size(), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(r->node_evt, nevt.data(), sizeof(int2) * nevt.size(), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(r->out_uid, ouid.data(), sizeof(int32_t) * ouid.size(), hipMemcpyHostToDevice));
  std::vector<long long> cur(off.begin(), off.end() - 1);
  HIP_TRY(hipMemcpy(r->cursor, cur.data(), sizeof(long long) * n, hipMemcpyHostToDevice));
  HIP_TRY(hipMemset(r->scur, 0, sizeof(int) * n));
  double sentinel;
  std::memcpy(&sentinel, &kMsgSentinel, sizeof(double));
  hipLaunchKernelGGL(k_fill, dim3(grid_for(2 * (U + n))), dim3(kBlock), 0, r->stream,
                     (long long)(2 * (U + n)), sentinel, reinterpret_cast<double *>(r->pay));
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(r->stream));
  int per_cu = 0, ncu = 0;
  HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_replay_persist, kBlock, 0));
  HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, r->device));
  // stay below the occupancy bound (the API can over-report by one block per CU)
  const long long cap = std::max(1LL, (long long)std::max(1, per_cu - 1) * ncu);
  r->pers_blocks = (unsigned)std::min<long long>(cap, grid_for(r->n));
  // the register variant needs one resident thread per node (a node's blocked receive is
  // retried by its own thread only)
  int per_cu_reg = 0;
  HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_reg, replay_reg_kernel(r), kBlock, 0));
  const long long cap_reg = (long long)std::max(0, per_cu_reg - 1) * ncu;
  // (and 16-byte payload polls at 32-bit byte offsets: below 2^27 messages)
  r->reg_ok = r->max_deg <= kReplayRegDeg && (long long)grid_for(r->n) <= cap_reg && U + n < (1LL << 27) && pack_ok;
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
  for (int32_t i = 0; i < n; ++i) r->max_deg = std::max<int64_t>(r->max_deg, rowptr[i + 1] - rowptr[i]);
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
  FU_TRY_BEGIN
  if (!t) return fail(FU_ERR_ARG, "fu_replay_create_from_trace: NULL trace");
  int32_t n, ticks;
  const int64_t *urp, *tto;
  const int32_t *tasks, *events, *oids;
  int64_t nt, ne, no, nm;
  fu__trace_view(t, &n, &ticks, &urp, &tto, &tasks, &nt, &events, &ne, &oids, &no, &nm);
  return fu_replay_create(n, urp, value, ticks, tto, nt, tasks, ne, events, no, oids, nm, device, out);
  FU_TRY_END
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
    if (r->reg_ok && r->pers_reg)
      hipLaunchKernelGGL(replay_reg_kernel(r), dim3(grid_for(r->n)), dim3(kBlock), 0, r->stream,
                         r->n, tick_end, r->node_off, r->node_evt, r->out_uid, (int)r->n_uid, r->rowptr, r->v,
                         r->flow, r->est, r->last, r->pay, r->cursor, r->scur, n_snap, d_st, snaps_dev, r->status,
                         (long long)1 << 22);
    else
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
  FU_TRY_BEGIN
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
  FU_TRY_END
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
  FU_TRY_BEGIN
  if (!r) return fail(FU_ERR_ARG, "fu_replay_get: NULL replay");
  HIP_TRY(hipSetDevice(r->device));
  if (last_avg) HIP_TRY(hipMemcpyAsync(last_avg, r->last, sizeof(double) * r->n, hipMemcpyDeviceToHost, r->stream));
  if (flows && r->E) HIP_TRY(hipMemcpyAsync(flows, r->flow, sizeof(double) * r->E, hipMemcpyDeviceToHost, r->stream));
  if (est && r->E) HIP_TRY(hipMemcpyAsync(est, r->est, sizeof(double) * r->E, hipMemcpyDeviceToHost, r->stream));
  HIP_TRY(hipStreamSynchronize(r->stream));
  return FU_OK;
  FU_TRY_END
}

int fu_replay_set_option(fu_replay *r, const char *key, int64_t value) {
  FU_TRY_BEGIN
  if (!r || !key) return fail(FU_ERR_ARG, "fu_replay_set_option: NULL argument");
  if (!std::strcmp(key, "persistent")) {
    if (r->cur_tick != 0) return fail(FU_ERR_STATE, "fu_replay_set_option: persistent must be set before the first tick");
    r->persistent = value != 0;
    if (!r->persistent) return FU_OK;
    // build the per-node event lists now, so that no host work lands inside a timed run
    HIP_TRY(hipSetDevice(r->device));
    return replay_build_persistent(r);
  }
  if (!std::strcmp(key, "persistent_reg")) {  // persistent mode: node state in registers (1, default)
    r->pers_reg = value != 0;
    return FU_OK;
  }
  return fail(FU_ERR_ARG, std::string("fu_replay_set_option: unknown key '") + key + "'");
  FU_TRY_END
}

int fu_replay_destroy(fu_replay *r) {
  if (!r) return FU_OK;
  hipSetDevice(r->device);
  if (r->stream) hipStreamSynchronize(r->stream);
  void *ptrs[] = {r->rowptr, r->tasks, r->events, r->out_ids, r->v, r->flow, r->est, r->last, r->msg,
                  r->node_off, r->cursor, r->node_ev, r->node_evt, r->node_tick, r->out_uid, r->scur, r->status, r->pay};
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
unsigned long long *fu__handle_err(fu_handle *h) { return h->err; }
int fu__handle_device(fu_handle *h) { return h->device; }
double *fu__handle_cur_a(fu_handle *h) { return cur_a(h); }
double *fu__handle_halo_a(fu_handle *h) { return h->halo_a; }
int64_t fu__handle_rounds(fu_handle *h) { return h->rounds; }

}
