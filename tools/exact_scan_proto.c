// Host prototype of the parallel exact left-to-right fp64 sum used for hub rows.
//
// Python's sum(...) (flowupdating-collectall.py:106, 110) is the sequential chain
// s_{k+1} = fl(s_k + x_k), s_0 = 0. This program checks, against that chain, the
// decomposition the GPU kernel uses:
//   1. an approximate prefix p_k (any order) gives the speculative binade e_k of s_{k+1};
//   2. a step whose e_k differs from e_{k-1} is a boundary: it is done as one exact fp64 add
//      in a short serial pass over the boundaries;
//   3. inside a segment of constant e every s_k is a multiple of u = 2^(e-52), so
//      s_{k+1} = u * (m_k + t_k) with t_k = round(x_k / u) (ties: the even m). t_k depends on
//      m_k only through its parity: a step is a 2-state transducer (t0, t1, q0, q1), and
//      compositions of transducers are associative, so the segment sums are a segmented scan;
//   4. verification: every non-boundary result has 2^52 < |m| < 2^53 (its exact sum was in
//      binade e, so fl rounded at u), and every boundary result is a multiple of its u.
//      Any failure -> the caller runs the sequential chain (same bits, slower).
// Build: gcc -O2 -ffp-contract=off -o /tmp/esp tools/exact_scan_proto.c -lm && /tmp/esp
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  int64_t t[2];
  uint8_t q[2];
} Tr;  // input parity p -> add t[p], output parity q[p]

static Tr tr_id(void) {
  Tr r = {{0, 0}, {0, 1}};
  return r;
}
static Tr tr_cat(Tr a, Tr b) {  // a then b
  Tr r;
  for (int p = 0; p < 2; ++p) {
    r.t[p] = a.t[p] + b.t[a.q[p]];
    r.q[p] = b.q[a.q[p]];
  }
  return r;
}

static int binade(double x) {  // exponent of |x| (x normal, nonzero); 0 / subnormal -> -2000
  if (x == 0.0 || !isfinite(x) || fabs(x) < 0x1p-1022) return -2000;
  int e;
  frexp(x, &e);
  return e - 1;
}

// one step inside a segment of ulp exponent ue (u = 2^ue); *bad on overflow
static Tr tr_step(double x, int ue, int *bad) {
  const double y = ldexp(x, -ue);
  if (!(fabs(y) < 0x1p62)) {
    *bad = 1;
    return tr_id();
  }
  const double fl = floor(y), fr = y - fl;
  const int64_t f = (int64_t)fl;
  Tr r;
  for (int p = 0; p < 2; ++p) {
    int64_t t;
    if (fr < 0.5) t = f;
    else if (fr > 0.5) t = f + 1;
    else t = ((p + f) & 1) ? f + 1 : f;  // tie: the even result
    r.t[p] = t;
    r.q[p] = (uint8_t)((p + t) & 1);
  }
  return r;
}

static double seq_sum(const double *x, int n) {
  double s = 0.0;
  for (int k = 0; k < n; ++k) s = s + x[k];
  return s;
}

// Returns 1 and *out = the exact chain when verified, 0 when the caller must fall back.
static int par_sum(const double *x, int n, int nthr, double *out, int *nseg_out) {
  if (n == 0) {
    *out = 0.0;
    return 1;
  }
  // 1. approximate prefix (per-thread chunk sums + exclusive scan, like the block scan)
  const int c = (n + nthr - 1) / nthr;
  double *cs = calloc(nthr + 1, sizeof(double));
  for (int t = 0; t < nthr; ++t)
    for (int k = t * c; k < n && k < (t + 1) * c; ++k) cs[t + 1] += x[k];
  for (int t = 0; t < nthr; ++t) cs[t + 1] += cs[t];
  int *e = malloc(sizeof(int) * n);
  for (int t = 0; t < nthr; ++t) {
    double p = cs[t];
    for (int k = t * c; k < n && k < (t + 1) * c; ++k) {
      p += x[k];
      e[k] = binade(p);
    }
  }
  free(cs);
  // 2 + 3. segments, transducer per segment (sequential composition here; the kernel does a
  // segmented scan)
  int bad = 0, nseg = 0;
  double s = 0.0;
  int k = 0;
  while (k < n) {
    const int ek = e[k];
    if (ek == -2000) {  // zero / subnormal speculation: no segment, plain step
      s = s + x[k];
      ++k;
      ++nseg;
      continue;
    }
    const int ue = ek - 52;
    s = s + x[k];  // boundary step: exact fp64 add
    ++nseg;
    const double mm = ldexp(s, -ue);
    if (mm != floor(mm) || !(fabs(mm) < 0x1p53)) {
      bad = 1;
      break;
    }
    int64_t m = (int64_t)mm;
    int j = k + 1;
    while (j < n && e[j] == ek) {
      Tr st = tr_step(x[j], ue, &bad);
      m += st.t[m & 1];
      const int64_t am = m < 0 ? -m : m;
      if (!(am > (1LL << 52) && am < (1LL << 53))) bad = 1;  // 4. verification
      ++j;
    }
    if (bad) break;
    s = ldexp((double)m, ue);
    k = j;
  }
  free(e);
  *nseg_out = nseg;
  if (bad) return 0;
  *out = s;
  return 1;
}

static uint64_t rs = 88172645463325252ull;
static double urand(void) {
  rs ^= rs << 13;
  rs ^= rs >> 7;
  rs ^= rs << 17;
  return (double)(rs >> 11) * 0x1p-53;
}

int main(void) {
  const int sizes[] = {1, 2, 3, 7, 64, 100, 1000, 4097, 65536, 400000};
  long trials = 0, fallbacks = 0, wrong = 0, fb_mode[7] = {0};
  for (int mode = 0; mode < 7; ++mode) {
    for (int si = 0; si < 10; ++si) {
      const int n = sizes[si];
      const int reps = n > 10000 ? 20 : 400;
      double *x = malloc(sizeof(double) * n);
      for (int r = 0; r < reps; ++r) {
        for (int k = 0; k < n; ++k) {
          double v;
          switch (mode) {
            case 0: v = 100.0 * urand(); break;                    // estimates (T)
            case 1: v = 50.0 + 1e-9 * (urand() - 0.5); break;      // converged estimates
            case 2: v = 40.0 * (urand() - 0.5); break;             // flows (S): random walk
            case 3: v = ldexp(floor(urand() * 8) - 4, -3); break;  // dyadic: exact zeros, ties
            case 4: v = (urand() - 0.5) * ldexp(1.0, (int)(urand() * 60) - 30); break;  // wide range
            case 5: v = (k & 1) ? 1.0 : ldexp(1.0, 53); break;     // ties at 2^53
            default: v = (urand() < 0.5 ? -1 : 1) * (1.0 + ldexp(urand(), -40)); break;
          }
          x[k] = v;
        }
        const double ref = seq_sum(x, n);
        double got;
        int nseg;
        ++trials;
        if (!par_sum(x, n, 256, &got, &nseg)) {
          ++fallbacks;
          ++fb_mode[mode];
          continue;
        }
        if (memcmp(&got, &ref, 8) != 0) {
          ++wrong;
          if (wrong < 10) printf("WRONG mode %d n %d: %.17g vs %.17g\n", mode, n, got, ref);
        }
        if (r == 0 && n == 400000) printf("mode %d n %d segments %d\n", mode, n, nseg);
      }
      free(x);
    }
  }
  for (int m = 0; m < 7; ++m) printf("mode %d fallbacks %ld\n", m, fb_mode[m]);
  printf("trials %ld fallbacks %ld wrong %ld\n", trials, fallbacks, wrong);
  return wrong != 0;
}
