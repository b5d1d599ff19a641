// Multi-GPU collect-all: one process per GPU, the graph split into contiguous node ranges,
// one halo exchange per round over RCCL (xGMI peer-to-peer).
//
// Every simulated mailbox transfer of the reference (Mailbox.put_async CA:124 /
// get_async CA:74) between nodes that live on different GPUs becomes one slot of a packed
// halo buffer. After each round the rank packs the new flows f_new[i->j] of its cut edges
// (receiver j remote) and the new estimates a_new[i] of its boundary nodes, then sends
// them to the owner of j with ncclSend/ncclRecv inside one group. The receiver stores them
// straight into its ghost flow slots (read through rev[] as -f_ji, CA:99) and ghost
// estimate slots (read through col[] as e_ij, CA:98). The sender packs in the receiver's
// slot order, so no unpack pass is needed. The round kernels are the single-GPU ones: they
// index the extended arrays and do not know about ranks.
//
// With kernel 4 (flow reconstruction, the default) a node rebuilds its neighbours' flows
// from their estimates, so the halo carries only the boundary estimates (8 B per boundary
// node per neighbouring part) and the ghost flow slots are unused.
//
// The convergence check all-reduces the per-rank max |a - target| with ncclMax on the
// uint64 bit patterns (ordered like non-negative doubles).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>
#include <vector>

#include "fu_common.h"

using namespace fu;

struct fu_handle;
extern "C" int fu__create_common(int32_t n, int64_t e, const int64_t *rowptr, const int32_t *col,
                                 const int32_t *rev, const double *value, int32_t device,
                                 int64_t f_extra, int32_t a_extra, fu_handle **out);


namespace {

struct DistState {
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0;
  int32_t n_local = 0;
  int64_t e_local = 0;
  std::vector<int64_t> send_f_off, recv_f_off, send_a_off, recv_a_off;
  int *send_f_idx = nullptr, *send_a_idx = nullptr;
  double *sbuf_f = nullptr, *sbuf_a = nullptr;
  int64_t n_send_f = 0, n_send_a = 0;
};

__global__ void k_pack(long long cnt, const int *__restrict__ idx, const double *__restrict__ src,
                       double *__restrict__ dst) {
  long long q = (long long)blockIdx.x * 256 + threadIdx.x;
  if (q < cnt) dst[q] = src[idx[q]];
}

}  // namespace

// Accessors implemented in fu_engine.hip (keeps fu_handle's layout private to that file).
extern "C" void *fu__handle_dist(fu_handle *h);
extern "C" void fu__handle_set_dist(fu_handle *h, void *d);
extern "C" hipStream_t fu__handle_stream(fu_handle *h);
extern "C" double *fu__handle_f(fu_handle *h, int which);
extern "C" double *fu__handle_a(fu_handle *h, int which);
extern "C" int fu__handle_cur(fu_handle *h);
extern "C" unsigned long long *fu__handle_err(fu_handle *h);
extern "C" int fu__handle_device(fu_handle *h);
extern "C" double *fu__handle_cur_a(fu_handle *h);
extern "C" double *fu__handle_cur_f(fu_handle *h);
extern "C" int fu__handle_kernel(fu_handle *h);

#define NCCL_TRY(expr)                                                                     \
  do {                                                                                     \
    ncclResult_t _r = (expr);                                                              \
    if (_r != ncclSuccess)                                                                 \
      return fu::fail(FU_ERR_NCCL, std::string(#expr) + ": " + ncclGetErrorString(_r));    \
  } while (0)

extern "C" {

int fu_dist_unique_id(uint8_t *id_out) {
  if (!id_out) return fail(FU_ERR_ARG, "fu_dist_unique_id: NULL");
  static_assert(sizeof(ncclUniqueId) == FU_UNIQUE_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id));
  std::memcpy(id_out, &id, sizeof(id));
  return FU_OK;
}

// phase 0: before a round (nothing); phase 1: after a round -> halo exchange of the new
// state; phase 100 + k: all-reduce max of k error slots.
int fu__dist_round_hook(fu_handle *h, int phase) {
  auto *d = static_cast<DistState *>(fu__handle_dist(h));
  hipStream_t s = fu__handle_stream(h);
  if (phase == 0) return FU_OK;
  if (phase >= 100) {
    const int k = phase - 100;
    unsigned long long *err = fu__handle_err(h);
    NCCL_TRY(ncclAllReduce(err, err, (size_t)k, ncclUint64, ncclMax, d->comm, s));
    return FU_OK;
  }
  // kernel 4 (flow reconstruction) needs only the neighbours' estimates: no ghost flows
  const bool flows = fu__handle_kernel(h) != 4;
  double *f = fu__handle_cur_f(h);
  double *a = fu__handle_cur_a(h);
  if (flows && d->n_send_f > 0) {
    hipLaunchKernelGGL(k_pack, dim3((unsigned)((d->n_send_f + 255) / 256)), dim3(256), 0, s,
                       (long long)d->n_send_f, d->send_f_idx, f, d->sbuf_f);
  }
  if (d->n_send_a > 0) {
    hipLaunchKernelGGL(k_pack, dim3((unsigned)((d->n_send_a + 255) / 256)), dim3(256), 0, s,
                       (long long)d->n_send_a, d->send_a_idx, a, d->sbuf_a);
  }
  hipError_t he = hipGetLastError();
  if (he != hipSuccess) return fail(FU_ERR_HIP, std::string("halo pack: ") + hipGetErrorString(he));
  NCCL_TRY(ncclGroupStart());
  for (int p = 0; p < d->nranks; ++p) {
    if (p == d->rank) continue;
    const int64_t sf = flows ? d->send_f_off[p + 1] - d->send_f_off[p] : 0;
    const int64_t rf = flows ? d->recv_f_off[p + 1] - d->recv_f_off[p] : 0;
    const int64_t sa = d->send_a_off[p + 1] - d->send_a_off[p];
    const int64_t ra = d->recv_a_off[p + 1] - d->recv_a_off[p];
    if (sf) NCCL_TRY(ncclSend(d->sbuf_f + d->send_f_off[p], (size_t)sf, ncclDouble, p, d->comm, s));
    if (rf) NCCL_TRY(ncclRecv(f + d->e_local + d->recv_f_off[p], (size_t)rf, ncclDouble, p, d->comm, s));
    if (sa) NCCL_TRY(ncclSend(d->sbuf_a + d->send_a_off[p], (size_t)sa, ncclDouble, p, d->comm, s));
    if (ra) NCCL_TRY(ncclRecv(a + d->n_local + d->recv_a_off[p], (size_t)ra, ncclDouble, p, d->comm, s));
  }
  NCCL_TRY(ncclGroupEnd());
  return FU_OK;
}

void fu__dist_free(fu_handle *h) {
  auto *d = static_cast<DistState *>(fu__handle_dist(h));
  if (!d) return;
  if (d->comm) ncclCommDestroy(d->comm);
  void *ptrs[] = {d->send_f_idx, d->send_a_idx, d->sbuf_f, d->sbuf_a};
  for (void *p : ptrs)
    if (p) hipFree(p);
  delete d;
  fu__handle_set_dist(h, nullptr);
}

int fu_dist_create(int32_t n_local, int64_t e_local, const int64_t *rowptr, const int32_t *col,
                   const int32_t *rev, const double *value, int32_t n_ghost_a,
                   int64_t n_ghost_f, int32_t nranks, int32_t rank, const int64_t *send_f_off,
                   const int32_t *send_f_idx, const int64_t *recv_f_off,
                   const int64_t *send_a_off, const int32_t *send_a_idx,
                   const int64_t *recv_a_off, const uint8_t *unique_id, int32_t device,
                   fu_handle **out) {
  FU_TRY_BEGIN
  if (!out || nranks < 1 || rank < 0 || rank >= nranks || !send_f_off || !recv_f_off || !send_a_off ||
      !recv_a_off || !unique_id || n_ghost_a < 0 || n_ghost_f < 0)
    return fail(FU_ERR_ARG, "fu_dist_create: bad arguments");
  if (recv_f_off[0] != 0 || recv_f_off[nranks] != n_ghost_f || recv_a_off[0] != 0 || recv_a_off[nranks] != n_ghost_a ||
      send_f_off[0] != 0 || send_a_off[0] != 0)
    return fail(FU_ERR_ARG, "fu_dist_create: halo offsets inconsistent with ghost counts");
  // rev == NULL: estimates-only halo (kernel 4); no ghost flows, flows plan must be empty
  if (!rev && (n_ghost_f != 0 || send_f_off[nranks] != 0))
    return fail(FU_ERR_ARG, "fu_dist_create: rev == NULL requires an empty flow halo");
  const int64_t nsf = send_f_off[nranks], nsa = send_a_off[nranks];
  for (int64_t q = 0; q < nsf; ++q)
    if (send_f_idx[q] < 0 || send_f_idx[q] >= e_local) return fail(FU_ERR_ARG, "fu_dist_create: send_f_idx out of range");
  for (int64_t q = 0; q < nsa; ++q)
    if (send_a_idx[q] < 0 || send_a_idx[q] >= n_local) return fail(FU_ERR_ARG, "fu_dist_create: send_a_idx out of range");
  fu_handle *h = nullptr;
  if (int rc = fu__create_common(n_local, e_local, rowptr, col, rev, value, device, rev ? n_ghost_f : -1,
                                 n_ghost_a, &h))
    return rc;
  auto *d = new DistState();
  fu__handle_set_dist(h, d);
  d->nranks = nranks;
  d->rank = rank;
  d->n_local = n_local;
  d->e_local = e_local;
  d->send_f_off.assign(send_f_off, send_f_off + nranks + 1);
  d->recv_f_off.assign(recv_f_off, recv_f_off + nranks + 1);
  d->send_a_off.assign(send_a_off, send_a_off + nranks + 1);
  d->recv_a_off.assign(recv_a_off, recv_a_off + nranks + 1);
  d->n_send_f = nsf;
  d->n_send_a = nsa;
  auto bail = [&](int code) { fu_destroy(h); return code; };
  auto alloc = [&](void **p, size_t bytes) { return hipMalloc(p, bytes ? bytes : 8) == hipSuccess; };
  if (!alloc((void **)&d->send_f_idx, sizeof(int) * nsf) || !alloc((void **)&d->send_a_idx, sizeof(int) * nsa) ||
      !alloc((void **)&d->sbuf_f, sizeof(double) * nsf) || !alloc((void **)&d->sbuf_a, sizeof(double) * nsa))
    return bail(fail(FU_ERR_ALLOC, "fu_dist_create: halo buffers"));
  if ((nsf && hipMemcpy(d->send_f_idx, send_f_idx, sizeof(int) * nsf, hipMemcpyHostToDevice) != hipSuccess) ||
      (nsa && hipMemcpy(d->send_a_idx, send_a_idx, sizeof(int) * nsa, hipMemcpyHostToDevice) != hipSuccess))
    return bail(fail(FU_ERR_HIP, "fu_dist_create: upload halo plan"));
  ncclUniqueId id;
  std::memcpy(&id, unique_id, sizeof(id));
  ncclResult_t r = ncclCommInitRank(&d->comm, nranks, id, rank);
  if (r != ncclSuccess) {
    d->comm = nullptr;
    return bail(fail(FU_ERR_NCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r)));
  }
  // kernel 4, "auto": its tile geometries are timed on real rounds; the halo carries only the
  // boundary estimates
  if (int rc = fu_set_option(h, "kernel", 0)) return bail(rc);
  *out = h;
  return FU_OK;
  FU_TRY_END
}

}  // extern "C"
