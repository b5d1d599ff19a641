/* CPU oracle, C restatement. THIS IS TEST INFRASTRUCTURE (see oracle/oracle.py header).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only
 * as the checker or the timed CPU baseline. The product never links it.
 *
 * Parity is PINNED: tests/test_oracle_golden.py checks these functions against
 * tests/golden/ (fixtures generated from the reference's own Peer arithmetic).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp). No fast-math: results must
 * be bitwise equal to Python floats.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* One collect-all round from (f_old, a_old) to (f_new, a_new).
 * Follows flowupdating-collectall.py: on_receive CA:98-99 (f_ij <- -f_ji, e_ij <- a_j) for
 * every neighbour, then avg_and_send CA:105-119 with left-to-right sums in row order
 * (CA:106 sum() from int 0 == 0.0 + x0 + ...; CA:109-111), a = ((v - S) + T) / (deg + 1)
 * (CA:107, CA:113), f = (fr + a) - er (CA:117). */
static void round_ca(int32_t n, const int64_t *rowptr, const int32_t *col, const int32_t *rev,
                     const double *v, const double *f_old, const double *a_old,
                     double *f_new, double *a_new, int nthreads) {
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1024) num_threads(nthreads)
#endif
  for (int32_t i = 0; i < n; ++i) {
    int64_t b = rowptr[i], e = rowptr[i + 1];
    double S = 0.0, T = 0.0;
    for (int64_t k = b; k < e; ++k) {
      S = S + (-f_old[rev[k]]);
      T = T + a_old[col[k]];
    }
    double a = ((v[i] - S) + T) / (double)(e - b + 1);
    a_new[i] = a;
    for (int64_t k = b; k < e; ++k) f_new[k] = ((-f_old[rev[k]]) + a) - a_old[col[k]];
  }
  (void)nthreads;
}

/* The same round with a 64-bit reverse index (graphs of 2^31 or more directed edges, which
 * the engine runs as partitions; the arithmetic is round_ca's). */
static void round_ca64(int32_t n, const int64_t *rowptr, const int32_t *col, const int64_t *rev,
                       const double *v, const double *f_old, const double *a_old,
                       double *f_new, double *a_new, int nthreads) {
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1024) num_threads(nthreads)
#endif
  for (int32_t i = 0; i < n; ++i) {
    int64_t b = rowptr[i], e = rowptr[i + 1];
    double S = 0.0, T = 0.0;
    for (int64_t k = b; k < e; ++k) {
      S = S + (-f_old[rev[k]]);
      T = T + a_old[col[k]];
    }
    double a = ((v[i] - S) + T) / (double)(e - b + 1);
    a_new[i] = a;
    for (int64_t k = b; k < e; ++k) f_new[k] = ((-f_old[rev[k]]) + a) - a_old[col[k]];
  }
  (void)nthreads;
}

/* rev[k] = the position of edge (col[k] -> i) for edge k = (i -> col[k]), 64-bit; the first
 * match in row col[k] (simple graphs have one). Returns the number of edges without a reverse
 * edge (0 for a symmetric graph). */
int64_t fuo_rev64(int32_t n, const int64_t *rowptr, const int32_t *col, int64_t *rev, int nthreads) {
  int64_t bad = 0;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 4096) num_threads(nthreads) reduction(+ : bad)
#endif
  for (int32_t i = 0; i < n; ++i) {
    for (int64_t k = rowptr[i]; k < rowptr[i + 1]; ++k) {
      const int32_t j = col[k];
      int64_t q = rowptr[j], qe = rowptr[j + 1];
      while (q < qe && col[q] != i) ++q;
      if (q < qe) rev[k] = q;
      else { rev[k] = -1; ++bad; }
    }
  }
  (void)nthreads;
  return bad;
}

/* Round 0: timeout fire on zero state (CA:33-34, CA:87-91). */
static void round0_ca(int32_t n, const int64_t *rowptr, const double *v, double *f,
                      double *a, int nthreads) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(nthreads)
#endif
  for (int32_t i = 0; i < n; ++i) {
    int64_t b = rowptr[i], e = rowptr[i + 1];
    double ai = ((v[i] - 0.0) + 0.0) / (double)(e - b + 1);
    a[i] = ai;
    for (int64_t k = b; k < e; ++k) f[k] = (0.0 + ai) - 0.0;
  }
  (void)nthreads;
}

/* Run rounds [0, rounds) from zero state. a_out[n], f_out[E]. Returns 0. */
int fuo_ca_sync(int32_t n, const int64_t *rowptr, const int32_t *col, const int32_t *rev,
                const double *v, int32_t rounds, double *a_out, double *f_out,
                int nthreads) {
  int64_t E = rowptr[n];
  if (rounds <= 0) return -1;
  double *f2 = (double *)malloc(sizeof(double) * (size_t)(E > 0 ? E : 1));
  double *a2 = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
  if (!f2 || !a2) { free(f2); free(a2); return -2; }
  double *fa = f_out, *aa = a_out, *fb = f2, *ab = a2;
  round0_ca(n, rowptr, v, fa, aa, nthreads);
  for (int32_t r = 1; r < rounds; ++r) {
    round_ca(n, rowptr, col, rev, v, fa, aa, fb, ab, nthreads);
    double *t = fa; fa = fb; fb = t;
    t = aa; aa = ab; ab = t;
  }
  if (fa != f_out) memcpy(f_out, fa, sizeof(double) * (size_t)E);
  if (aa != a_out) memcpy(a_out, aa, sizeof(double) * (size_t)n);
  free(f2);
  free(a2);
  return 0;
}

/* fuo_ca_sync with a 64-bit reverse index (fuo_rev64). */
int fuo_ca_sync64(int32_t n, const int64_t *rowptr, const int32_t *col, const int64_t *rev,
                  const double *v, int32_t rounds, double *a_out, double *f_out, int nthreads) {
  int64_t E = rowptr[n];
  if (rounds <= 0) return -1;
  double *f2 = (double *)malloc(sizeof(double) * (size_t)(E > 0 ? E : 1));
  double *a2 = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
  if (!f2 || !a2) { free(f2); free(a2); return -2; }
  double *fa = f_out, *aa = a_out, *fb = f2, *ab = a2;
  round0_ca(n, rowptr, v, fa, aa, nthreads);
  for (int32_t r = 1; r < rounds; ++r) {
    round_ca64(n, rowptr, col, rev, v, fa, aa, fb, ab, nthreads);
    double *t = fa; fa = fb; fb = t;
    t = aa; aa = ab; ab = t;
  }
  if (fa != f_out) memcpy(f_out, fa, sizeof(double) * (size_t)E);
  if (aa != a_out) memcpy(a_out, aa, sizeof(double) * (size_t)n);
  free(f2);
  free(a2);
  return 0;
}

/* Continue from a given state for `rounds` more rounds (r >= 1 semantics), in place.
 * Used by the CPU baseline to time steady-state rounds. */
int fuo_ca_rounds(int32_t n, const int64_t *rowptr, const int32_t *col, const int32_t *rev,
                  const double *v, int32_t rounds, double *a, double *f, int nthreads) {
  int64_t E = rowptr[n];
  double *f2 = (double *)malloc(sizeof(double) * (size_t)(E > 0 ? E : 1));
  double *a2 = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
  if (!f2 || !a2) { free(f2); free(a2); return -2; }
  double *fa = f, *aa = a, *fb = f2, *ab = a2;
  for (int32_t r = 0; r < rounds; ++r) {
    round_ca(n, rowptr, col, rev, v, fa, aa, fb, ab, nthreads);
    double *t = fa; fa = fb; fb = t;
    t = aa; aa = ab; ab = t;
  }
  if (fa != f) memcpy(f, fa, sizeof(double) * (size_t)E);
  if (aa != a) memcpy(a, aa, sizeof(double) * (size_t)n);
  free(f2);
  free(a2);
  return 0;
}

/* Trace replay (event format of include/fu.h), sequential in event order.
 * RECV    (0, slot, msg, -):      CA:98-99 / PW:98-99
 * FIRE_CA (1, k, out_off, -):     CA:105-125 over slots [0, k)
 * FIRE_PW (2, slot, k, msg_out):  PW:102-117, flows summed over slots [0, k)
 * snap_ticks (sorted) / snaps[n_snap * n]: last_avg after the given ticks. */
int fuo_replay(int32_t n, const int64_t *rowptr, const double *v, int32_t n_ticks,
               const int64_t *tick_task_off, const int32_t *tasks, const int32_t *events,
               const int32_t *out_ids, int64_t n_msgs, int32_t n_snap,
               const int32_t *snap_ticks, double *snaps, double *last, double *flow,
               double *est) {
  int64_t E = rowptr[n];
  double *mf = (double *)malloc(sizeof(double) * (size_t)(n_msgs > 0 ? n_msgs : 1));
  double *ma = (double *)malloc(sizeof(double) * (size_t)(n_msgs > 0 ? n_msgs : 1));
  if (!mf || !ma) { free(mf); free(ma); return -2; }
  memset(flow, 0, sizeof(double) * (size_t)E);
  memset(est, 0, sizeof(double) * (size_t)E);
  memset(last, 0, sizeof(double) * (size_t)n);
  int32_t si = 0;
  for (int32_t t = 0; t < n_ticks; ++t) {
    for (int64_t ti = tick_task_off[t]; ti < tick_task_off[t + 1]; ++ti) {
      int32_t node = tasks[3 * ti], eb = tasks[3 * ti + 1], ee = tasks[3 * ti + 2];
      double *fl = flow + rowptr[node];
      double *es = est + rowptr[node];
      for (int32_t q = eb; q < ee; ++q) {
        const int32_t *ev = events + 4 * (int64_t)q;
        if (ev[0] == 0) {
          es[ev[1]] = ma[ev[2]];
          fl[ev[1]] = -mf[ev[2]];
        } else if (ev[0] == 1) {
          int32_t k = ev[1];
          double S = 0.0, T = 0.0;
          for (int32_t j = 0; j < k; ++j) S = S + fl[j];
          double estimate = v[node] - S;
          for (int32_t j = 0; j < k; ++j) T = T + es[j];
          double avg = (estimate + T) / (double)(k + 1);
          last[node] = avg;
          for (int32_t j = 0; j < k; ++j) {
            double nf = (fl[j] + avg) - es[j];
            fl[j] = nf;
            es[j] = avg;
            int32_t m = out_ids[ev[2] + j];
            mf[m] = nf;
            ma[m] = avg;
          }
        } else {
          int32_t s = ev[1], k = ev[2], m = ev[3];
          double S = 0.0;
          for (int32_t j = 0; j < k; ++j) S = S + fl[j];
          double estimate = v[node] - S;
          double avg = (es[s] + estimate) / 2.0;
          last[node] = avg;
          double nf = (fl[s] + avg) - es[s];
          fl[s] = nf;
          es[s] = avg;
          mf[m] = nf;
          ma[m] = avg;
        }
      }
    }
    while (si < n_snap && snap_ticks[si] == t) {
      memcpy(snaps + (int64_t)si * n, last, sizeof(double) * (size_t)n);
      ++si;
    }
  }
  free(mf);
  free(ma);
  return 0;
}

int fuo_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
