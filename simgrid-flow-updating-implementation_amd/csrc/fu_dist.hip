// Multi-GPU collect-all: one process per GPU, the graph split into contiguous node ranges,
// one halo exchange per round over RCCL (xGMI peer-to-peer).
//
// Every simulated mailbox transfer of the reference (Mailbox.put_async CA:124 /
// get_async CA:74) between nodes that live on different GPUs becomes one slot of a packed
// halo buffer. The round kernels rebuild a neighbour's flow from its estimates (flow
// reconstruction, kernel 4), so only the boundary ESTIMATES move: after each round the rank
// packs a_new[i] of its boundary nodes per neighbouring part and sends them with
// ncclSend/ncclRecv inside one group, straight into the receiver's ghost estimate slots (read
// through col[] as e_ij, CA:98). The sender packs in the receiver's slot order, so there is
// no unpack pass. The round kernels are the single-GPU ones: they index the extended
// estimate arrays and do not know about ranks.
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
                                 const double *value, int32_t device, int32_t a_extra, fu_handle **out);


namespace {

struct DistState {
  ncclComm_t comm = nullptr;  // null: the in-process transport (fu_dist_create_local)
  int nranks = 0, rank = 0;
  int32_t n_local = 0;
  int64_t e_local = 0;
  std::vector<int64_t> send_a_off, recv_a_off;
  int *send_a_idx = nullptr;
  double *sbuf_a = nullptr;
  int64_t n_send_a = 0;
  // Both transports run the halo of round r on comm_stream beside round r's interior tiles:
  // behind ev_bnd (boundary tiles done) the rank packs a_r of its boundary nodes there. RCCL
  // then sends / receives in one group on that stream. The in-process transport records
  // ev_packed instead, and fu_dist_exchange_local copies every peer's packed slots into this
  // rank's ghost slots on this rank's comm_stream (after ev_packed of the peer). Either way
  // ev_halo marks the ghost slots of a_r as written, and the next round waits for it.
  hipStream_t comm_stream = nullptr;
  hipEvent_t ev_bnd = nullptr, ev_halo = nullptr, ev_packed = nullptr;
  // timing events on comm_stream: from the start of the pack (boundary tiles done) to the
  // ghost slots written (fu_dist_halo_time)
  hipEvent_t ev_h0 = nullptr, ev_h1 = nullptr;
  bool timed_once = false;
  bool halo_pending = false;
  bool any_halo = true;          // RCCL transport: this rank sends or receives estimates (else no comm-stream hop)
  int64_t packed_round = -1;     // in-process transport: round whose packed halo awaits the exchange
  int64_t exchanged_round = -1;  // in-process transport: last round whose halo was exchanged
  unsigned long long *agree = nullptr;  // RCCL transport: one word for fu__dist_agree
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
extern "C" unsigned long long *fu__handle_err(fu_handle *h);
extern "C" int fu__handle_device(fu_handle *h);
extern "C" double *fu__handle_cur_a(fu_handle *h);
extern "C" double *fu__handle_halo_a(fu_handle *h);
extern "C" int64_t fu__handle_rounds(fu_handle *h);

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

#define HIPD_TRY(expr)                                                                    \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess) return fu::fail(FU_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

// phase 0: before a round (or a host sync): the main stream waits for the last halo.
// phase 1: fu_reset: as phase 0, then the comm stream drains and the in-process transport's
//   round bookkeeping restarts (round 0 may be packed and exchanged again).
// phase 2: mid-round, once the boundary tiles (and heavy rows) of round r are queued: behind
//   ev_bnd, pack a_r[send_a_idx] on comm_stream, concurrently with round r's interior tiles
//   (they never read ghost slots; the receives write only ghost slots [n_local, na) of the
//   buffer, the interior tiles only own slots). RCCL: the ncclSend/ncclRecv group follows on
//   comm_stream and records ev_halo. In-process transport: the pack records ev_packed, and
//   fu_dist_exchange_local queues the copies into the peers' ghost slots and their ev_halo.
// phase 100 + k: all-reduce max of k error slots (on comm_stream, joined back).
int fu__dist_round_hook(fu_handle *h, int phase) {
  auto *d = static_cast<DistState *>(fu__handle_dist(h));
  hipStream_t s = fu__handle_stream(h);
  if (phase == 0 || phase == 1) {
    if (d->halo_pending) HIPD_TRY(hipStreamWaitEvent(s, d->ev_halo, 0));
    d->halo_pending = false;
    if (phase == 1) {
      HIPD_TRY(hipStreamSynchronize(d->comm_stream));
      d->packed_round = d->exchanged_round = -1;
      d->timed_once = false;
    }
    return FU_OK;
  }
  if (phase >= 100) {
    if (!d->comm) return FU_OK;  // local transport: the caller combines the per-rank maxima
    const int k = phase - 100;
    unsigned long long *err = fu__handle_err(h);
    HIPD_TRY(hipEventRecord(d->ev_bnd, s));
    HIPD_TRY(hipStreamWaitEvent(d->comm_stream, d->ev_bnd, 0));
    NCCL_TRY(ncclAllReduce(err, err, (size_t)k, ncclUint64, ncclMax, d->comm, d->comm_stream));
    HIPD_TRY(hipEventRecord(d->ev_halo, d->comm_stream));
    HIPD_TRY(hipStreamWaitEvent(s, d->ev_halo, 0));
    return FU_OK;
  }
  double *a = fu__handle_halo_a(h);
  hipStream_t cs = d->comm_stream;
  if (d->comm && !d->any_halo) {  // nothing to exchange (one rank): no hop through the comm stream
    d->timed_once = true;
    return FU_OK;
  }
  HIPD_TRY(hipEventRecord(d->ev_bnd, s));
  HIPD_TRY(hipStreamWaitEvent(cs, d->ev_bnd, 0));
  HIPD_TRY(hipEventRecord(d->ev_h0, cs));
  if (d->n_send_a > 0) {
    hipLaunchKernelGGL(k_pack, dim3((unsigned)((d->n_send_a + 255) / 256)), dim3(256), 0, cs,
                       (long long)d->n_send_a, d->send_a_idx, a, d->sbuf_a);
  }
  hipError_t he = hipGetLastError();
  if (he != hipSuccess) return fail(FU_ERR_HIP, std::string("halo pack: ") + hipGetErrorString(he));
  if (!d->comm) {  // in-process transport: fu_dist_exchange_local moves the packed estimates
    HIPD_TRY(hipEventRecord(d->ev_packed, cs));
    d->packed_round = fu__handle_rounds(h);  // the round being launched
    return FU_OK;
  }
  NCCL_TRY(ncclGroupStart());
  for (int p = 0; p < d->nranks; ++p) {
    if (p == d->rank) continue;
    const int64_t sa = d->send_a_off[p + 1] - d->send_a_off[p];
    const int64_t ra = d->recv_a_off[p + 1] - d->recv_a_off[p];
    if (sa) NCCL_TRY(ncclSend(d->sbuf_a + d->send_a_off[p], (size_t)sa, ncclDouble, p, d->comm, cs));
    if (ra) NCCL_TRY(ncclRecv(a + d->n_local + d->recv_a_off[p], (size_t)ra, ncclDouble, p, d->comm, cs));
  }
  NCCL_TRY(ncclGroupEnd());
  HIPD_TRY(hipEventRecord(d->ev_halo, cs));
  HIPD_TRY(hipEventRecord(d->ev_h1, cs));
  d->timed_once = true;
  d->halo_pending = true;
  return FU_OK;
}

// Collective agreement on a host-side result (RCCL transport): *ok_all = the minimum of
// ok_local over all ranks, so a call that failed on one rank fails on every rank instead of
// leaving its peers to block in the next halo exchange. Every rank must call it. The
// in-process transport has one caller for all ranks, which sees every rank's result itself.
int fu__dist_agree(fu_handle *h, int ok_local, int *ok_all) {
  auto *d = static_cast<DistState *>(fu__handle_dist(h));
  *ok_all = ok_local;
  if (!d || !d->comm) return FU_OK;
  if (!d->agree) HIPD_TRY(hipMalloc((void **)&d->agree, sizeof(unsigned long long)));
  unsigned long long v = ok_local ? 1ull : 0ull;
  HIPD_TRY(hipStreamSynchronize(d->comm_stream));
  HIPD_TRY(hipMemcpyAsync(d->agree, &v, sizeof(v), hipMemcpyHostToDevice, d->comm_stream));
  NCCL_TRY(ncclAllReduce(d->agree, d->agree, 1, ncclUint64, ncclMin, d->comm, d->comm_stream));
  HIPD_TRY(hipMemcpyAsync(&v, d->agree, sizeof(v), hipMemcpyDeviceToHost, d->comm_stream));
  HIPD_TRY(hipStreamSynchronize(d->comm_stream));
  *ok_all = v != 0;
  return FU_OK;
}

void fu__dist_free(fu_handle *h) {
  auto *d = static_cast<DistState *>(fu__handle_dist(h));
  if (!d) return;
  if (d->comm_stream) hipStreamSynchronize(d->comm_stream);
  if (d->comm) ncclCommDestroy(d->comm);
  if (d->ev_bnd) hipEventDestroy(d->ev_bnd);
  if (d->ev_halo) hipEventDestroy(d->ev_halo);
  if (d->ev_packed) hipEventDestroy(d->ev_packed);
  if (d->ev_h0) hipEventDestroy(d->ev_h0);
  if (d->ev_h1) hipEventDestroy(d->ev_h1);
  if (d->comm_stream) hipStreamDestroy(d->comm_stream);
  void *ptrs[] = {d->send_a_idx, d->sbuf_a, d->agree};
  for (void *p : ptrs)
    if (p) hipFree(p);
  delete d;
  fu__handle_set_dist(h, nullptr);
}

static int dist_create(int32_t n_local, int64_t e_local, const int64_t *rowptr, const int32_t *col,
                       const int32_t *rev, const double *value, int32_t n_ghost_a,
                       int64_t n_ghost_f, int32_t nranks, int32_t rank, const int64_t *send_f_off,
                       const int32_t *send_f_idx, const int64_t *recv_f_off,
                       const int64_t *send_a_off, const int32_t *send_a_idx,
                       const int64_t *recv_a_off, const uint8_t *unique_id, int32_t device,
                       fu_handle **out) {
  FU_TRY_BEGIN
  if (!out || nranks < 1 || rank < 0 || rank >= nranks || !send_f_off || !recv_f_off || !send_a_off ||
      !recv_a_off || n_ghost_a < 0 || n_ghost_f < 0)
    return fail(FU_ERR_ARG, "fu_dist_create: bad arguments");
  if (recv_f_off[0] != 0 || recv_f_off[nranks] != n_ghost_f || recv_a_off[0] != 0 || recv_a_off[nranks] != n_ghost_a ||
      send_f_off[0] != 0 || send_a_off[0] != 0)
    return fail(FU_ERR_ARG, "fu_dist_create: halo offsets inconsistent with ghost counts");
  // estimates-only halo: flows are reconstructed from estimates, so there are no ghost flows
  if (rev || n_ghost_f != 0 || send_f_off[nranks] != 0)
    return fail(FU_ERR_ARG, "fu_dist_create: the halo carries estimates only (rev must be NULL, no ghost flows)");
  (void)send_f_idx;
  const int64_t nsa = send_a_off[nranks];
  for (int64_t q = 0; q < nsa; ++q)
    if (send_a_idx[q] < 0 || send_a_idx[q] >= n_local) return fail(FU_ERR_ARG, "fu_dist_create: send_a_idx out of range");
  fu_handle *h = nullptr;
  if (int rc = fu__create_common(n_local, e_local, rowptr, col, value, device, n_ghost_a, &h)) return rc;
  auto *d = new DistState();
  fu__handle_set_dist(h, d);
  d->nranks = nranks;
  d->rank = rank;
  d->n_local = n_local;
  d->e_local = e_local;
  d->send_a_off.assign(send_a_off, send_a_off + nranks + 1);
  d->recv_a_off.assign(recv_a_off, recv_a_off + nranks + 1);
  d->n_send_a = nsa;
  d->any_halo = nsa > 0 || recv_a_off[nranks] > 0;
  auto bail = [&](int code) { fu_destroy(h); return code; };
  auto alloc = [&](void **p, size_t bytes) { return hipMalloc(p, bytes ? bytes : 8) == hipSuccess; };
  if (!alloc((void **)&d->send_a_idx, sizeof(int) * nsa) || !alloc((void **)&d->sbuf_a, sizeof(double) * nsa))
    return bail(fail(FU_ERR_ALLOC, "fu_dist_create: halo buffers"));
  if (nsa && hipMemcpy(d->send_a_idx, send_a_idx, sizeof(int) * nsa, hipMemcpyHostToDevice) != hipSuccess)
    return bail(fail(FU_ERR_HIP, "fu_dist_create: upload halo plan"));
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&d->comm_stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&d->ev_bnd, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&d->ev_halo, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&d->ev_packed, hipEventDisableTiming) != hipSuccess ||
      hipEventCreate(&d->ev_h0) != hipSuccess || hipEventCreate(&d->ev_h1) != hipSuccess)
    return bail(fail(FU_ERR_HIP, "fu_dist_create: communication stream"));
  if (!unique_id) {  // fu_dist_create_local: no communicator (in-process transport). Kernel 4
    // pinned: an autotune pass would run rounds with no exchange between them
    if (int rc = fu_set_option(h, "kernel", 4)) return bail(rc);
    *out = h;
    return FU_OK;
  }
  ncclUniqueId id;
  std::memcpy(&id, unique_id, sizeof(id));
  ncclResult_t r = ncclCommInitRank(&d->comm, nranks, id, rank);
  if (r != ncclSuccess) {
    d->comm = nullptr;
    return bail(fail(FU_ERR_NCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r)));
  }
  // kernel 4, "auto": its tile geometries are timed on real rounds
  if (int rc = fu_set_option(h, "kernel", 0)) return bail(rc);
  *out = h;
  return FU_OK;
  FU_TRY_END
}

int fu_dist_create(int32_t n_local, int64_t e_local, const int64_t *rowptr, const int32_t *col,
                   const int32_t *rev, const double *value, int32_t n_ghost_a,
                   int64_t n_ghost_f, int32_t nranks, int32_t rank, const int64_t *send_f_off,
                   const int32_t *send_f_idx, const int64_t *recv_f_off,
                   const int64_t *send_a_off, const int32_t *send_a_idx,
                   const int64_t *recv_a_off, const uint8_t *unique_id, int32_t device,
                   fu_handle **out) {
  if (!unique_id) return fail(FU_ERR_ARG, "fu_dist_create: NULL unique_id");
  return dist_create(n_local, e_local, rowptr, col, rev, value, n_ghost_a, n_ghost_f, nranks, rank, send_f_off,
                     send_f_idx, recv_f_off, send_a_off, send_a_idx, recv_a_off, unique_id, device, out);
}

int fu_dist_create_local(int32_t n_local, int64_t e_local, const int64_t *rowptr, const int32_t *col,
                         const double *value, int32_t n_ghost_a, int32_t nranks, int32_t rank,
                         const int64_t *send_a_off, const int32_t *send_a_idx, const int64_t *recv_a_off,
                         int32_t device, fu_handle **out) {
  std::vector<int64_t> z(std::max(1, nranks + 1), 0);
  return dist_create(n_local, e_local, rowptr, col, nullptr, value, n_ghost_a, 0, nranks, rank, z.data(), nullptr,
                     z.data(), send_a_off, send_a_idx, recv_a_off, nullptr, device, out);
}

// In-process transport: the ranks of one process (handles on any devices of this process)
// exchange the halo of the round every rank has just launched, asynchronously, through the
// same comm_stream / event chain as RCCL. For every receiver q, on q's comm_stream: wait for
// each sender's ev_packed, copy its packed slots into q's ghost slots (the slot order RCCL
// uses), record q's ev_halo (q's next round waits for it). Then every sender's comm_stream
// waits for the ev_halo of the receivers it feeds, so its next pack cannot overwrite sbuf_a
// before they have copied it. No host synchronisation: many rounds can be queued per call
// (fu_dist_run_local), and the copies run beside the interior tiles of the round.
int fu_dist_exchange_local(fu_handle **hs, int32_t nranks) {
  FU_TRY_BEGIN
  if (!hs || nranks < 1) return fail(FU_ERR_ARG, "fu_dist_exchange_local: bad arguments");
  std::vector<DistState *> ds(nranks);
  for (int p = 0; p < nranks; ++p) {
    ds[p] = hs[p] ? static_cast<DistState *>(fu__handle_dist(hs[p])) : nullptr;
    if (!ds[p] || ds[p]->comm || ds[p]->rank != p || ds[p]->nranks != nranks)
      return fail(FU_ERR_ARG, "fu_dist_exchange_local: handle " + std::to_string(p) + " is not local-transport rank " +
                                  std::to_string(p) + " of " + std::to_string(nranks));
  }
  // every rank must have launched the same round r >= 0 and not yet exchanged its halo
  const int64_t r = fu__handle_rounds(hs[0]) - 1;
  for (int p = 0; p < nranks; ++p) {
    if (fu__handle_rounds(hs[p]) - 1 != r || r < 0)
      return fail(FU_ERR_STATE, "fu_dist_exchange_local: ranks have run different numbers of rounds (or none)");
    if (ds[p]->packed_round != r || ds[p]->exchanged_round == r)
      return fail(FU_ERR_STATE, "fu_dist_exchange_local: round " + std::to_string(r) + " of rank " +
                                    std::to_string(p) + " has no packed halo pending");
  }
  for (int q = 0; q < nranks; ++q)
    for (int p = 0; p < nranks; ++p)
      if (p != q && ds[p]->send_a_off[q + 1] - ds[p]->send_a_off[q] != ds[q]->recv_a_off[p + 1] - ds[q]->recv_a_off[p])
        return fail(FU_ERR_ARG, "fu_dist_exchange_local: halo plans of ranks " + std::to_string(p) + " and " +
                                    std::to_string(q) + " disagree");
  for (int q = 0; q < nranks; ++q) {
    HIPD_TRY(hipSetDevice(fu__handle_device(hs[q])));
    hipStream_t cs = ds[q]->comm_stream;
    double *a = fu__handle_halo_a(hs[q]) + ds[q]->n_local;  // a_r of the round just launched
    for (int p = 0; p < nranks; ++p) {
      const int64_t cnt = p == q ? 0 : ds[q]->recv_a_off[p + 1] - ds[q]->recv_a_off[p];
      if (!cnt) continue;
      HIPD_TRY(hipStreamWaitEvent(cs, ds[p]->ev_packed, 0));
      HIPD_TRY(hipMemcpyAsync(a + ds[q]->recv_a_off[p], ds[p]->sbuf_a + ds[p]->send_a_off[q], sizeof(double) * cnt,
                              hipMemcpyDefault, cs));
    }
    HIPD_TRY(hipEventRecord(ds[q]->ev_halo, cs));
    HIPD_TRY(hipEventRecord(ds[q]->ev_h1, cs));
    ds[q]->timed_once = true;
    ds[q]->halo_pending = true;
    ds[q]->exchanged_round = r;
  }
  for (int p = 0; p < nranks; ++p) {  // sbuf_a of p is free again once its receivers copied it
    HIPD_TRY(hipSetDevice(fu__handle_device(hs[p])));
    for (int q = 0; q < nranks; ++q)
      if (q != p && ds[p]->send_a_off[q + 1] > ds[p]->send_a_off[q])
        HIPD_TRY(hipStreamWaitEvent(ds[p]->comm_stream, ds[q]->ev_halo, 0));
  }
  return FU_OK;
  FU_TRY_END
}

// Device time of the last round's halo on this rank's comm stream: from the start of its pack
// (behind the boundary tiles) to its ghost slots written (RCCL group or in-process copies).
// It overlaps the round's interior tiles. Waits for that halo.
int fu_dist_halo_time(fu_handle *h, float *ms) {
  if (!h || !ms) return fail(FU_ERR_ARG, "fu_dist_halo_time: NULL argument");
  auto *d = static_cast<DistState *>(fu__handle_dist(h));
  if (!d) return fail(FU_ERR_ARG, "fu_dist_halo_time: not a multi-GPU handle");
  if (!d->timed_once) return fail(FU_ERR_STATE, "fu_dist_halo_time: no halo exchanged yet");
  if (d->comm && !d->any_halo) {  // a rank with nothing to exchange
    *ms = 0.0f;
    return FU_OK;
  }
  // in-process transport: ev_h0 is re-recorded by every round's pack, ev_h1 only by the
  // exchange, so the pair is one halo only when the last packed round was exchanged
  if (!d->comm && d->packed_round != d->exchanged_round)
    return fail(FU_ERR_STATE, "fu_dist_halo_time: round " + std::to_string(d->packed_round) +
                                  "'s halo is packed but not exchanged yet");
  HIPD_TRY(hipSetDevice(fu__handle_device(h)));
  HIPD_TRY(hipEventSynchronize(d->ev_h1));
  HIPD_TRY(hipEventElapsedTime(ms, d->ev_h0, d->ev_h1));
  return FU_OK;
}

// `rounds` rounds of every rank of the in-process transport, each followed by its halo
// exchange, all queued without a host synchronisation.
int fu_dist_run_local(fu_handle **hs, int32_t nranks, int32_t rounds) {
  if (!hs || nranks < 1 || rounds < 0) return fail(FU_ERR_ARG, "fu_dist_run_local: bad arguments");
  for (int32_t k = 0; k < rounds; ++k) {
    for (int p = 0; p < nranks; ++p)
      if (int rc = fu_run_collectall(hs[p], 1, 0, nullptr)) return rc;
    if (int rc = fu_dist_exchange_local(hs, nranks)) return rc;
  }
  return FU_OK;
}

}  // extern "C"
