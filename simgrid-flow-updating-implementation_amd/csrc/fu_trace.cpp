// Tick-level trace generator: the value-independent schedule of the reference run.
//
// The reference runs each node as a SimGrid actor executing Peer.loop
// (flowupdating-collectall.py:70-85, flowupdating-pairwise.py:69-84):
//     if comm is None: comm = mailbox.get_async()          CA:73-74
//     if comm.test(): msg = ...; comm = None; on_receive()  CA:76-82
//     tick()                                                CA:84
//     sleep_for(1.0)                                        CA:85
// Mailboxes are rendez-vous points: a put_async matches a posted get_async or is queued
// FIFO. Every route of the reference platform transfers in (0, 1) simulated seconds
// (SURVEY.md App. B), so a message matched at tick t is consumed at tick t+1 at the
// earliest. Whether a node fires depends only on who has been heard (CA:100-103), on tick
// counters (CA:87-91) and on clocks (PW:86-91), never on fp values. So the whole schedule
// can be generated here once and replayed on the GPU as one batch per tick.
//
// The generator emits, per tick, one task per actor that did something: its events in
// program order.
//   RECV    {0, slot, msg, 0}       on_receive cache update        (CA:98-99, PW:98-99)
//   FIRE_CA {1, k, out_off, 0}      avg_and_send over k neighbours (CA:105-128)
//   FIRE_PW {2, slot, k, msg_out}   avg_and_send(neigh)            (PW:102-117)
// Neighbours unknown to a receiver are appended to its row (CA:94-96 / PW:94-96), so each
// row of the union CSR is in insertion order: declared first (ACT:4-27), then first arrival.
//
// Message slots are recycled. A slot consumed at tick t becomes free at the end of tick t,
// so no slot is both read and written in the same tick batch.
//
// Fault injection (not in the reference, which never loses a
// message). faults = "drop=P,delay=D:Q,seed=S": each put_async (CA:124 / PW:116) is lost
// with probability P, or is held back D ticks with probability Q. Draws come from a
// SplitMix64 stream in put order, so the faulty schedule is as deterministic as the clean
// one. Lost messages exercise the timeouts (CA:87-91, PW:86-91), i.e. Flow Updating's
// self-healing. The fault model lives entirely in the schedule, so the GPU replay is the
// same code.
#include <cmath>
#include <cstring>
#include <limits>
#include <unordered_map>

#include "fu_common.h"

struct fu_trace {
  int32_t n = 0, mode = 0, ticks = 0;
  int64_t dropped = 0, delayed = 0;
  std::vector<int64_t> urowptr;
  std::vector<int32_t> ucol;
  std::vector<int64_t> tick_task_off;
  std::vector<int32_t> tasks;
  std::vector<int32_t> events;
  std::vector<int32_t> out_ids;
  std::vector<int64_t> first_avg_seq;
  std::vector<int32_t> fires;
  int64_t n_msg_slots = 0, dyn_adds = 0, msgs_sent = 0;
};

namespace {

using namespace fu;

// Transfers with link sharing (parity-unpinned against SimGrid, which
// cannot run offline). A message matched at tick t (the rendez-vous, CA:74 / CA:124)
// starts its transfer at time t: a latency phase of lat_factor * sum(route latencies) with
// no bandwidth, then `bytes` at the rate max-min fair sharing gives it. A shared link l
// offers bw_factor * bw_l to the transfers in their data phase that cross it, split by
// weighted progressive filling: a transfer's share is proportional to 1 / its sharing
// penalty, LV08's route latency sum + weight_S / bw_k over its links (weight_S = 0: equal
// shares); a FATPIPE link caps each transfer at bw_factor * bw_l without sharing, and with
// tcp_gamma > 0 the TCP window caps it at tcp_gamma / (2 * route latency sum) (SimGrid's
// CM02 / LV08 bounds). With cross > 0 (SimGrid's network/crosstraffic, 0.05 there) a transfer
// also loads every shared link of its reverse route with cross x its rate (the TCP
// acknowledgements), and a FATPIPE link of the reverse route only caps it at
// bw_factor * bw / cross. Rates change only when a transfer enters or leaves its data phase. Alone, a
// transfer takes lat_factor * sum(lat) + bytes / (bw_factor * min bw), the fixed per-route
// time of fu_trace_build_routes. The message is consumed at the first tick > its end
// (CA:76: the actor tests the receive once per tick). oracle/oracle.py (LinkNet) mirrors
// every operation in the same order, so both produce the same doubles.
struct LinkNet {
  int32_t n = 0, n_links = 0;
  const double *bw = nullptr, *lat = nullptr;
  const int32_t *shared = nullptr;
  const int64_t *roff = nullptr;
  const int32_t *rl = nullptr;
  double bytes = 154.0, lat_factor = 13.01, bw_factor = 0.97;
  double weight_S = 0.0, tcp_gamma = 0.0;  // LV08: 20537 and 4194304 (fu/platform.py)
  double cross = 0.0;                      // network/crosstraffic (SimGrid: 0.05; 0 = off)
  struct Flow {
    int64_t r;         // route index src * n + dst
    double lat_end;    // end of the latency phase
    double rem;        // bytes left (data phase)
    double cap;        // FATPIPE / TCP-window cap (inf: none)
    double pen;        // sharing penalty (1 with weight_S = 0: equal shares)
    double rate;
    double end;        // completion time (inf while running)
    int phase;         // 0 latency, 1 data, 2 done
    // the shared links the transfer loads and its coefficient on each: 1 on its route (in
    // route order), then cross on its reverse route's (crosstraffic; a link on both routes
    // appears twice)
    std::vector<std::pair<int32_t, double>> lk;
  };
  std::vector<Flow> fl;           // one per message id
  std::vector<int32_t> active;    // message ids not done, in start order
  double now = 0.0;

  void start(int32_t id, int32_t src, int32_t dst, double t) {
    if ((int32_t)fl.size() <= id) fl.resize(id + 1);
    Flow &f = fl[id];
    f.r = (int64_t)src * n + dst;
    double l = 0.0, cap = std::numeric_limits<double>::infinity(), sw = 0.0;
    f.lk.clear();
    for (int64_t k = roff[f.r]; k < roff[f.r + 1]; ++k) {
      l = l + lat[rl[k]];
      sw = sw + weight_S / bw[rl[k]];
      if (!shared[rl[k]]) cap = std::min(cap, bw_factor * bw[rl[k]]);
      else f.lk.emplace_back(rl[k], 1.0);
    }
    if (cross > 0.0) {
      const int64_t rb = (int64_t)dst * n + src;
      for (int64_t k = roff[rb]; k < roff[rb + 1]; ++k) {
        const int32_t q = rl[k];
        if (shared[q]) {
          f.lk.emplace_back(q, cross);
        } else {
          bool fwd = false;  // a FATPIPE link of both routes: consumption max(1, cross) = 1
          for (int64_t j = roff[f.r]; j < roff[f.r + 1]; ++j) fwd = fwd || rl[j] == q;
          if (!fwd) cap = std::min(cap, bw_factor * bw[q] / cross);
        }
      }
    }
    if (tcp_gamma > 0.0 && l > 0.0) cap = std::min(cap, tcp_gamma / (2.0 * l));
    f.lat_end = t + lat_factor * l;
    f.rem = bytes;
    f.cap = cap;
    f.pen = weight_S > 0.0 ? l + sw : 1.0;
    f.rate = 0.0;
    f.end = std::numeric_limits<double>::infinity();
    f.phase = 0;
    if (roff[f.r] == roff[f.r + 1]) {  // same host: no transfer
      f.phase = 2;
      f.end = t;
      return;
    }
    active.push_back(id);
  }
  // weighted progressive filling over the data-phase transfers (SimGrid's LMM max-min):
  // a link's level is its remaining capacity / the sum of 1 / penalty of its unfixed
  // transfers; the lowest level (or a transfer's cap * penalty) fixes the transfers it
  // binds at level / penalty (or their cap). weight_S = 0 gives every penalty 1: plain
  // max-min, equal shares. Parity-unpinned against SimGrid (fu.h)
  void rates() {
    std::vector<double> crem(n_links, 0.0), use(n_links, 0.0);
    std::vector<int32_t> cnt(n_links, 0);
    std::vector<int32_t> un;
    for (int32_t id : active) {
      if (fl[id].phase != 1) continue;
      un.push_back(id);
      for (const auto &lc : fl[id].lk) {
        cnt[lc.first]++;
        use[lc.first] = use[lc.first] + lc.second / fl[id].pen;
      }
    }
    for (int32_t l = 0; l < n_links; ++l) crem[l] = bw_factor * bw[l];
    while (!un.empty()) {
      double best = std::numeric_limits<double>::infinity();
      for (int32_t l = 0; l < n_links; ++l)
        if (cnt[l] > 0) best = std::min(best, std::max(0.0, crem[l] / use[l]));
      for (int32_t id : un) best = std::min(best, fl[id].cap * fl[id].pen);
      std::vector<int32_t> keep, fix;
      for (int32_t id : un) {
        bool b = fl[id].cap * fl[id].pen == best;
        for (size_t q = 0; q < fl[id].lk.size() && !b; ++q) {
          const int32_t l = fl[id].lk[q].first;
          b = cnt[l] > 0 && std::max(0.0, crem[l] / use[l]) == best;
        }
        (b ? fix : keep).push_back(id);
      }
      for (int32_t id : fix) {
        Flow &f = fl[id];
        f.rate = f.cap * f.pen == best ? f.cap : best / f.pen;
        for (const auto &lc : f.lk) {
          crem[lc.first] = crem[lc.first] - lc.second * f.rate;
          use[lc.first] = use[lc.first] - lc.second / f.pen;
          cnt[lc.first]--;
        }
      }
      un.swap(keep);
    }
  }
  // run the fluid model up to time T (every event at a time <= T is processed)
  void advance_to(double T) {
    for (;;) {
      rates();
      double nx = T;
      for (int32_t id : active) {
        const Flow &f = fl[id];
        if (f.phase == 0) nx = std::min(nx, f.lat_end);
        else if (f.rate > 0.0) nx = std::min(nx, now + f.rem / f.rate);
      }
      const double dt = nx - now;
      bool ev = false;
      std::vector<int32_t> keep;
      for (int32_t id : active) {
        Flow &f = fl[id];
        if (f.phase == 1) {
          if (f.rate > 0.0 && now + f.rem / f.rate <= nx) {
            f.phase = 2;
            f.end = nx;
            ev = true;
            continue;
          }
          f.rem = f.rem - f.rate * dt;
        } else if (f.lat_end <= nx) {
          f.phase = 1;
          ev = true;
          if (!(f.rem > 0.0)) {
            f.phase = 2;
            f.end = nx;
            continue;
          }
        }
        keep.push_back(id);
      }
      active.swap(keep);
      now = nx;
      if (!ev) return;  // nx == T with nothing due
    }
  }
  bool done_before(int32_t id, double t) const { return fl[id].phase == 2 && fl[id].end < t; }
};

struct Builder {
  int32_t n;
  int32_t mode;
  fu_trace &tr;
  std::vector<std::vector<int32_t>> nbrs;
  std::unordered_map<uint64_t, int32_t> slot_of;
  // collect-all state
  std::vector<std::vector<uint8_t>> heard;
  std::vector<int32_t> heard_cnt, counter;
  // pairwise state (clock of last average per neighbour slot; defaultdict(float) -> 0.0)
  std::vector<std::vector<double>> last;
  // receive side: 0 none, 1 posted (unmatched), 2 matched
  std::vector<int8_t> cstate;
  std::vector<int32_t> cmsg, ctick;
  // FIFO queues as linked lists over message ids
  std::vector<int32_t> qhead, qtail, qnext;
  std::vector<int32_t> msg_sender;
  std::vector<int32_t> free_ids, pending_free;
  int64_t first_seq = 0;
  int32_t t = 0;
  // faults
  double p_drop = 0.0, p_delay = 0.0;
  int32_t delay_ticks = 0;
  uint64_t fstate = 0;
  std::vector<std::vector<std::pair<int32_t, int32_t>>> delayed;  // due tick -> (dst, id)
  // route transfer times (seconds, n x n, sender row), NULL = every route under one tick
  const double *route = nullptr;
  LinkNet *net = nullptr;  // link sharing (fu_trace_build_links), else per-route times

  // whole ticks a transfer on src -> dst takes beyond the first: a message matched at tick t
  // completes at t + T and is consumed from tick t + floor(T) + 1 (t + 1 when T < 1, CA:76)
  int32_t extra(int32_t src, int32_t dst) const {
    if (!route) return 0;
    const double T = route[(int64_t)src * n + dst];
    if (!(T >= 1.0)) return 0;  // < 1 s, negative or NaN
    return T >= 1e9 ? 1000000000 : (int32_t)std::floor(T);
  }

  Builder(int32_t n_, int32_t mode_, fu_trace &tr_) : n(n_), mode(mode_), tr(tr_) {}

  int32_t alloc_msg(int32_t sender) {
    int32_t id;
    if (!free_ids.empty()) {
      id = free_ids.back();
      free_ids.pop_back();
    } else {
      id = (int32_t)msg_sender.size();
      msg_sender.push_back(-1);
      qnext.push_back(-1);
    }
    msg_sender[id] = sender;
    qnext[id] = -1;
    tr.msgs_sent++;
    return id;
  }

  void deliver(int32_t dst, int32_t id) {
    if (p_drop > 0.0 || p_delay > 0.0) {
      const double u = u01(splitmix_next(fstate));
      if (u < p_drop) {  // lost: the slot is never consumed and frees at the end of the tick
        pending_free.push_back(id);
        tr.dropped++;
        return;
      }
      if (u < p_drop + p_delay) {
        const int32_t due = t + delay_ticks;
        if (due >= (int32_t)delayed.size()) delayed.resize(due + 1);
        delayed[due].emplace_back(dst, id);
        tr.delayed++;
        return;
      }
    }
    arrive(dst, id);
  }

  void arrive(int32_t dst, int32_t id) {
    if (cstate[dst] == 1) {  // posted receive: matched now, transfer in flight
      cstate[dst] = 2;
      cmsg[dst] = id;
      ctick[dst] = t;
      if (net) net->start(id, msg_sender[id], dst, (double)t);
    } else {
      if (qtail[dst] < 0) qhead[dst] = id;
      else qnext[qtail[dst]] = id;
      qtail[dst] = id;
    }
  }

  void note_fire(int32_t i) {
    if (tr.fires[i]++ == 0) tr.first_avg_seq[i] = first_seq++;
  }

  void push_event(int32_t a, int32_t b, int32_t c, int32_t d) {
    tr.events.push_back(a);
    tr.events.push_back(b);
    tr.events.push_back(c);
    tr.events.push_back(d);
  }

  void fire_ca(int32_t i) {  // CA:105-128
    const int32_t k = (int32_t)nbrs[i].size();
    push_event(FU_EV_FIRE_CA, k, (int32_t)tr.out_ids.size(), 0);
    note_fire(i);
    for (int32_t s = 0; s < k; ++s) {
      int32_t id = alloc_msg(i);
      tr.out_ids.push_back(id);
      deliver(nbrs[i][s], id);
    }
    std::fill(heard[i].begin(), heard[i].end(), 0);  // CA:127
    heard_cnt[i] = 0;
    counter[i] = 0;  // CA:128
  }

  void fire_pw(int32_t i, int32_t s) {  // PW:102-117
    const int32_t k = (int32_t)nbrs[i].size();
    int32_t id = alloc_msg(i);
    push_event(FU_EV_FIRE_PW, s, k, id);
    note_fire(i);
    last[i][s] = (double)t;  // PW:111
    deliver(nbrs[i][s], id);
  }

  int32_t slot_for(int32_t i, int32_t sender) {
    uint64_t key = ((uint64_t)(uint32_t)i << 32) | (uint32_t)sender;
    auto it = slot_of.find(key);
    if (it != slot_of.end()) return it->second;
    int32_t s = (int32_t)nbrs[i].size();  // CA:94-95: append unknown sender
    nbrs[i].push_back(sender);
    slot_of.emplace(key, s);
    if (mode == FU_MODE_COLLECTALL) heard[i].push_back(0);
    else last[i].push_back(0.0);
    tr.dyn_adds++;
    return s;
  }

  void step(int32_t i) {
    const int64_t ev0 = (int64_t)tr.events.size() / 4;
    if (cstate[i] == 0) {  // CA:73-74
      if (qhead[i] >= 0) {
        int32_t id = qhead[i];
        qhead[i] = qnext[id];
        if (qhead[i] < 0) qtail[i] = -1;
        cstate[i] = 2;
        cmsg[i] = id;
        ctick[i] = t;
        if (net) net->start(id, msg_sender[id], i, (double)t);
      } else {
        cstate[i] = 1;
      }
    }
    if (cstate[i] == 2 && (net ? net->done_before(cmsg[i], (double)t)
                               : ctick[i] + extra(msg_sender[cmsg[i]], i) < t)) {  // CA:76-82
      int32_t id = cmsg[i];
      cstate[i] = 0;
      int32_t s = slot_for(i, msg_sender[id]);
      push_event(FU_EV_RECV, s, id, 0);
      pending_free.push_back(id);
      if (mode == FU_MODE_COLLECTALL) {
        if (!heard[i][s]) {  // CA:100
          heard[i][s] = 1;
          heard_cnt[i]++;
        }
        if (heard_cnt[i] == (int32_t)nbrs[i].size()) fire_ca(i);  // CA:102-103
      } else {
        fire_pw(i, s);  // PW:100
      }
    }
    if (mode == FU_MODE_COLLECTALL) {  // CA:87-91
      if (++counter[i] >= 50) fire_ca(i);
    } else {  // PW:86-91
      const double thr = (double)t - 50.0;
      for (int32_t s = 0; s < (int32_t)nbrs[i].size(); ++s)
        if (last[i][s] < thr) fire_pw(i, s);
    }
    const int64_t ev1 = (int64_t)tr.events.size() / 4;
    if (ev1 > ev0) {
      tr.tasks.push_back(i);
      tr.tasks.push_back((int32_t)ev0);
      tr.tasks.push_back((int32_t)ev1);
    }
  }
};

bool parse_faults(const char *f, double &drop, double &delay, int32_t &dticks, uint64_t &seed) {
  drop = delay = 0.0;
  dticks = 0;
  seed = 0;
  if (!f || !*f) return true;
  std::string s(f);
  size_t pos = 0;
  while (pos < s.size()) {
    size_t end = s.find(',', pos);
    if (end == std::string::npos) end = s.size();
    std::string kv = s.substr(pos, end - pos);
    size_t eq = kv.find('=');
    if (eq == std::string::npos) return false;
    std::string k = kv.substr(0, eq), v = kv.substr(eq + 1);
    char *e = nullptr;
    if (k == "drop") {
      drop = std::strtod(v.c_str(), &e);
      if (*e || drop < 0 || drop > 1) return false;
    } else if (k == "delay") {
      size_t c = v.find(':');
      if (c == std::string::npos) return false;
      dticks = (int32_t)std::strtol(v.substr(0, c).c_str(), &e, 10);
      if (*e || dticks < 1) return false;
      delay = std::strtod(v.substr(c + 1).c_str(), &e);
      if (*e || delay < 0 || delay > 1) return false;
    } else if (k == "seed") {
      seed = std::strtoull(v.c_str(), &e, 10);
      if (*e) return false;
    } else {
      return false;
    }
    pos = end + 1;
  }
  return drop + delay <= 1.0;
}

bool parse_order(const char *order, int &kind, uint64_t &seed) {
  if (!order || !std::strcmp(order, "fwd")) { kind = 0; return true; }
  if (!std::strcmp(order, "rev")) { kind = 1; return true; }
  if (!std::strncmp(order, "rand:", 5)) {
    char *end = nullptr;
    seed = std::strtoull(order + 5, &end, 10);
    if (end == order + 5 || *end) return false;
    kind = 2;
    return true;
  }
  return false;
}

}  // namespace

extern "C" {

int fu_trace_build(int32_t n, const int64_t *decl_rowptr, const int32_t *decl_col,
                   int32_t mode, int32_t ticks, const char *order, fu_trace **out) {
  return fu_trace_build_ex(n, decl_rowptr, decl_col, mode, ticks, order, nullptr, out);
}

int fu_trace_build_ex(int32_t n, const int64_t *decl_rowptr, const int32_t *decl_col,
                      int32_t mode, int32_t ticks, const char *order, const char *faults,
                      fu_trace **out) {
  return fu_trace_build_routes(n, decl_rowptr, decl_col, mode, ticks, order, faults, nullptr, out);
}

static int build_trace(int32_t n, const int64_t *decl_rowptr, const int32_t *decl_col, int32_t mode,
                       int32_t ticks, const char *order, const char *faults, const double *route_s, LinkNet *net,
                       fu_trace **out);

int fu_trace_build_routes(int32_t n, const int64_t *decl_rowptr, const int32_t *decl_col,
                          int32_t mode, int32_t ticks, const char *order, const char *faults,
                          const double *route_s, fu_trace **out) {
  return build_trace(n, decl_rowptr, decl_col, mode, ticks, order, faults, route_s, nullptr, out);
}

int fu_trace_build_links(int32_t n, const int64_t *decl_rowptr, const int32_t *decl_col, int32_t mode,
                         int32_t ticks, const char *order, const char *faults, int32_t n_links,
                         const double *link_bw, const double *link_lat, const int32_t *link_shared,
                         const int64_t *route_off, const int32_t *route_links, double msg_bytes,
                         double lat_factor, double bw_factor, fu_trace **out) {
  return fu_trace_build_links_cross(n, decl_rowptr, decl_col, mode, ticks, order, faults, n_links, link_bw,
                                    link_lat, link_shared, route_off, route_links, msg_bytes, lat_factor, bw_factor,
                                    0.0, 0.0, 0.0, out);
}

int fu_trace_build_links_ex(int32_t n, const int64_t *decl_rowptr, const int32_t *decl_col, int32_t mode,
                            int32_t ticks, const char *order, const char *faults, int32_t n_links,
                            const double *link_bw, const double *link_lat, const int32_t *link_shared,
                            const int64_t *route_off, const int32_t *route_links, double msg_bytes,
                            double lat_factor, double bw_factor, double weight_S, double tcp_gamma,
                            fu_trace **out) {
  return fu_trace_build_links_cross(n, decl_rowptr, decl_col, mode, ticks, order, faults, n_links, link_bw,
                                    link_lat, link_shared, route_off, route_links, msg_bytes, lat_factor, bw_factor,
                                    weight_S, tcp_gamma, 0.0, out);
}

int fu_trace_build_links_cross(int32_t n, const int64_t *decl_rowptr, const int32_t *decl_col, int32_t mode,
                               int32_t ticks, const char *order, const char *faults, int32_t n_links,
                               const double *link_bw, const double *link_lat, const int32_t *link_shared,
                               const int64_t *route_off, const int32_t *route_links, double msg_bytes,
                               double lat_factor, double bw_factor, double weight_S, double tcp_gamma,
                               double crosstraffic, fu_trace **out) {
  FU_TRY_BEGIN
  if (n <= 0 || n_links < 0 || !route_off || (n_links > 0 && (!link_bw || !link_lat || !link_shared)) ||
      !(msg_bytes >= 0.0) || !(lat_factor >= 0.0) || !(bw_factor > 0.0) || !(weight_S >= 0.0) ||
      !(tcp_gamma >= 0.0) || !(crosstraffic >= 0.0) || !(crosstraffic <= 1.0))
    return fail(FU_ERR_ARG, "fu_trace_build_links: bad arguments");
  const int64_t nr = (int64_t)n * n;
  if (route_off[0] != 0) return fail(FU_ERR_ARG, "fu_trace_build_links: route_off[0] must be 0");
  for (int64_t r = 0; r < nr; ++r) {
    if (route_off[r + 1] < route_off[r]) return fail(FU_ERR_ARG, "fu_trace_build_links: route_off not ascending");
    for (int64_t k = route_off[r]; k < route_off[r + 1]; ++k)
      if (!route_links || route_links[k] < 0 || route_links[k] >= n_links)
        return fail(FU_ERR_ARG, "fu_trace_build_links: route link out of range");
  }
  for (int32_t l = 0; l < n_links; ++l)
    if (!(link_bw[l] > 0.0) || !(link_lat[l] >= 0.0))
      return fail(FU_ERR_ARG, "fu_trace_build_links: link bandwidths must be > 0, latencies >= 0");
  LinkNet net;
  net.n = n;
  net.n_links = n_links;
  net.bw = link_bw;
  net.lat = link_lat;
  net.shared = link_shared;
  net.roff = route_off;
  net.rl = route_links;
  net.bytes = msg_bytes;
  net.lat_factor = lat_factor;
  net.bw_factor = bw_factor;
  net.weight_S = weight_S;
  net.tcp_gamma = tcp_gamma;
  net.cross = crosstraffic;
  return build_trace(n, decl_rowptr, decl_col, mode, ticks, order, faults, nullptr, &net, out);
  FU_TRY_END
}

static int build_trace(int32_t n, const int64_t *decl_rowptr, const int32_t *decl_col, int32_t mode,
                       int32_t ticks, const char *order, const char *faults, const double *route_s, LinkNet *net,
                       fu_trace **out) {
  FU_TRY_BEGIN
  if (!out || n <= 0 || !decl_rowptr || ticks < 0 || (mode != FU_MODE_COLLECTALL && mode != FU_MODE_PAIRWISE))
    return fail(FU_ERR_ARG, "fu_trace_build: bad arguments");
  int okind = 0;
  uint64_t oseed = 0;
  if (!parse_order(order, okind, oseed)) return fail(FU_ERR_ARG, std::string("fu_trace_build: bad order '") + (order ? order : "") + "'");
  double p_drop, p_delay;
  int32_t dticks;
  uint64_t fseed;
  if (!parse_faults(faults, p_drop, p_delay, dticks, fseed))
    return fail(FU_ERR_ARG, std::string("fu_trace_build: bad faults '") + (faults ? faults : "") + "' (drop=P,delay=D:Q,seed=S)");
  auto *tr = new fu_trace();
  tr->n = n;
  tr->mode = mode;
  tr->ticks = ticks;
  tr->first_avg_seq.assign(n, -1);
  tr->fires.assign(n, 0);
  Builder B(n, mode, *tr);
  B.p_drop = p_drop;
  B.p_delay = p_delay;
  B.delay_ticks = dticks;
  B.fstate = fseed;
  B.route = route_s;
  B.net = net;
  B.nbrs.resize(n);
  for (int32_t i = 0; i < n; ++i) {
    for (int64_t k = decl_rowptr[i]; k < decl_rowptr[i + 1]; ++k) {
      int32_t j = decl_col[k];
      if (j < 0 || j >= n || j == i) { delete tr; return fail(FU_ERR_GRAPH, "fu_trace_build: bad neighbour id (out of range or self)"); }
      uint64_t key = ((uint64_t)(uint32_t)i << 32) | (uint32_t)j;
      if (B.slot_of.count(key)) { delete tr; return fail(FU_ERR_GRAPH, "fu_trace_build: duplicate neighbour"); }
      B.slot_of.emplace(key, (int32_t)B.nbrs[i].size());
      B.nbrs[i].push_back(j);
    }
  }
  if (mode == FU_MODE_COLLECTALL) {
    B.heard.resize(n);
    for (int32_t i = 0; i < n; ++i) B.heard[i].assign(B.nbrs[i].size(), 0);
    B.heard_cnt.assign(n, 0);
    B.counter.assign(n, 0);
  } else {
    B.last.resize(n);
    for (int32_t i = 0; i < n; ++i) B.last[i].assign(B.nbrs[i].size(), 0.0);
  }
  B.cstate.assign(n, 0);
  B.cmsg.assign(n, -1);
  B.ctick.assign(n, -1);
  B.qhead.assign(n, -1);
  B.qtail.assign(n, -1);
  std::vector<int32_t> perm(n);
  for (int32_t i = 0; i < n; ++i) perm[i] = okind == 1 ? n - 1 - i : i;
  uint64_t st = oseed;
  tr->tick_task_off.push_back(0);
  for (int32_t t = 0; t < ticks; ++t) {
    B.t = t;
    if (net) net->advance_to((double)t);  // transfers that end before tick t are consumable
    if (t < (int32_t)B.delayed.size()) {  // held-back messages reach their mailbox now
      for (auto &m : B.delayed[t]) B.arrive(m.first, m.second);
      B.delayed[t].clear();
    }
    if (okind == 2) {  // per-tick Fisher-Yates, j = r % (i+1) (same as oracle.tick_orders)
      for (int32_t i = 0; i < n; ++i) perm[i] = i;
      for (int32_t i = n - 1; i > 0; --i) {
        uint64_t j = splitmix_next(st) % (uint64_t)(i + 1);
        std::swap(perm[i], perm[j]);
      }
    }
    for (int32_t q = 0; q < n; ++q) B.step(perm[q]);
    for (int32_t id : B.pending_free) B.free_ids.push_back(id);
    B.pending_free.clear();
    tr->tick_task_off.push_back((int64_t)tr->tasks.size() / 3);
    if ((int64_t)tr->events.size() / 4 >= (int64_t)INT32_MAX || (int64_t)tr->out_ids.size() >= (int64_t)INT32_MAX) {
      delete tr;
      return fail(FU_ERR_ALLOC, "fu_trace_build: trace exceeds 2^31 events");
    }
  }
  tr->n_msg_slots = (int64_t)B.msg_sender.size();
  tr->urowptr.assign(n + 1, 0);
  for (int32_t i = 0; i < n; ++i) tr->urowptr[i + 1] = tr->urowptr[i] + (int64_t)B.nbrs[i].size();
  tr->ucol.reserve(tr->urowptr[n]);
  for (int32_t i = 0; i < n; ++i) tr->ucol.insert(tr->ucol.end(), B.nbrs[i].begin(), B.nbrs[i].end());
  *out = tr;
  return FU_OK;
  FU_TRY_END
}

int fu_trace_info(const fu_trace *t, int64_t info[8]) {
  if (!t || !info) return fail(FU_ERR_ARG, "fu_trace_info: NULL argument");
  info[0] = t->urowptr[t->n];
  info[1] = (int64_t)t->tasks.size() / 3;
  info[2] = (int64_t)t->events.size() / 4;
  info[3] = (int64_t)t->out_ids.size();
  info[4] = t->n_msg_slots;
  info[5] = t->ticks;
  info[6] = t->dyn_adds;
  info[7] = t->msgs_sent;
  return FU_OK;
}

int fu_trace_fault_stats(const fu_trace *t, int64_t *dropped, int64_t *delayed) {
  if (!t) return fail(FU_ERR_ARG, "fu_trace_fault_stats: NULL trace");
  if (dropped) *dropped = t->dropped;
  if (delayed) *delayed = t->delayed;
  return FU_OK;
}

int fu_trace_export(const fu_trace *t, int64_t *union_rowptr, int32_t *union_col,
                    int64_t *tick_task_off, int32_t *tasks, int32_t *events,
                    int32_t *out_ids, int64_t *first_avg_seq, int32_t *fires) {
  if (!t) return fail(FU_ERR_ARG, "fu_trace_export: NULL trace");
  auto cp = [](void *dst, const void *src, size_t bytes) {
    if (dst && bytes) std::memcpy(dst, src, bytes);
  };
  cp(union_rowptr, t->urowptr.data(), sizeof(int64_t) * t->urowptr.size());
  cp(union_col, t->ucol.data(), sizeof(int32_t) * t->ucol.size());
  cp(tick_task_off, t->tick_task_off.data(), sizeof(int64_t) * t->tick_task_off.size());
  cp(tasks, t->tasks.data(), sizeof(int32_t) * t->tasks.size());
  cp(events, t->events.data(), sizeof(int32_t) * t->events.size());
  cp(out_ids, t->out_ids.data(), sizeof(int32_t) * t->out_ids.size());
  cp(first_avg_seq, t->first_avg_seq.data(), sizeof(int64_t) * t->first_avg_seq.size());
  cp(fires, t->fires.data(), sizeof(int32_t) * t->fires.size());
  return FU_OK;
}

int fu_trace_free(fu_trace *t) {
  delete t;
  return FU_OK;
}

// Accessors used by the device side (fu_engine.hip) without exposing the struct layout.
const fu_trace *fu__trace_view(const fu_trace *t, int32_t *n, int32_t *ticks,
                               const int64_t **urowptr, const int64_t **tto,
                               const int32_t **tasks, int64_t *n_tasks,
                               const int32_t **events, int64_t *n_events,
                               const int32_t **out_ids, int64_t *n_out, int64_t *n_msgs) {
  *n = t->n;
  *ticks = t->ticks;
  *urowptr = t->urowptr.data();
  *tto = t->tick_task_off.data();
  *tasks = t->tasks.data();
  *n_tasks = (int64_t)t->tasks.size() / 3;
  *events = t->events.data();
  *n_events = (int64_t)t->events.size() / 4;
  *out_ids = t->out_ids.data();
  *n_out = (int64_t)t->out_ids.size();
  *n_msgs = t->n_msg_slots;
  return t;
}

}  // extern "C"
