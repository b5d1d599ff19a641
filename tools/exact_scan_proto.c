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


// ---------------------------------------------------------------------------------------
// v2: the GPU decomposition. Pieces of XB = 2048 elements (one block, 8 per thread) are
// summarised independently (given the approximate sum of everything before the piece):
// the head run (elements before the piece's first boundary), then per boundary its element
// and the run that follows it. A run summary carries the transducer plus the min / max of
// its partial increments, so one serial pass over pieces and boundaries both applies and
// verifies every run in O(1).
#define XB 2048
#define XT 8
#define MAXB 64
#define SPECIAL (-100000)
typedef struct {
  int64_t t[2];
  uint8_t q[2];
  int64_t mn, mx;  // min / max partial increment over the run's results (both parities)
  int len;
} Run;
typedef struct {
  double x;
  int ue;
  Run run;
} Bnd;
typedef struct {
  int first_ue;  // ulp exponent the head run assumes
  Run head;
  int nb;        // boundaries (> MAXB: dense, the serial pass walks the elements)
  Bnd b[MAXB];
} Piece;

// speculation key of a value: ulp exponent and sign (a run keeps both); SPECIAL for 0,
// subnormals, inf, nan
static int ulp_key(double x) {
  uint64_t bits;
  memcpy(&bits, &x, 8);
  const int E = (int)((bits >> 52) & 0x7ff);
  if (E == 0 || E == 0x7ff) return SPECIAL;
  return ((E - 1075) << 1) | (int)(bits >> 63);
}
static int key_ue(int key) { return key >> 1; }
static Run run_id(void) {
  Run r = {{0, 0}, {0, 1}, INT64_MAX, INT64_MIN, 0};
  return r;
}
static Run run_push(Run a, Tr st) {  // a then one step
  Run r;
  for (int p = 0; p < 2; ++p) {
    r.t[p] = a.t[p] + st.t[a.q[p]];
    r.q[p] = st.q[a.q[p]];
  }
  r.mn = a.mn;
  r.mx = a.mx;
  for (int p = 0; p < 2; ++p) {
    if (r.t[p] < r.mn) r.mn = r.t[p];
    if (r.t[p] > r.mx) r.mx = r.t[p];
  }
  r.len = a.len + 1;
  return r;
}
// apply a run to M (units 2^ue, M != 0), verifying every result stays strictly inside the binade
static int run_apply(const Run *r, int64_t *M) {
  if (r->len == 0) return 1;
  const int64_t lo = 1LL << 52, hi = 1LL << 53, m = *M;
  if (m > 0) {
    if (!(m + r->mn > lo && m + r->mx < hi)) return 0;
  } else {
    if (!(m + r->mx < -lo && m + r->mn > -hi)) return 0;
  }
  *M = m + r->t[m & 1];
  return 1;
}

static void summarise(const double *x, int n, double pre, Piece *P) {
  // approximate prefix as the block does it: thread sums, exclusive scan, then in-thread
  double ts[XB / XT + 1];
  ts[0] = pre;
  for (int t = 0; t < XB / XT; ++t) {
    double s = 0;
    for (int i = 0; i < XT; ++i) {
      const int k = t * XT + i;
      if (k < n) s += x[k];
    }
    ts[t + 1] = ts[t] + s;
  }
  P->first_ue = ulp_key(pre);
  P->head = run_id();
  P->nb = 0;
  int prev = P->first_ue, in_head = 1, bad = 0;
  Run *cur = &P->head;
  for (int t = 0; t < XB / XT; ++t) {
    double p = ts[t];
    for (int i = 0; i < XT; ++i) {
      const int k = t * XT + i;
      if (k >= n) break;
      p += x[k];
      const int ue = ulp_key(p);
      if (ue == SPECIAL || ue != prev || prev == SPECIAL) {
        in_head = 0;
        if (P->nb < MAXB) {
          P->b[P->nb].x = x[k];
          P->b[P->nb].ue = ue;
          P->b[P->nb].run = run_id();
          cur = &P->b[P->nb].run;
        } else {
          cur = NULL;
        }
        P->nb++;
      } else if (cur) {
        Tr st = tr_step(x[k], key_ue(ue), &bad);
        *cur = run_push(*cur, st);
        if (bad) cur->mn = INT64_MIN;  // forces the verification to fail
      }
      prev = ue;
    }
  }
  (void)in_head;
}

// serial pass over the pieces of a row; returns 0 when verification fails (fallback)
static long why[8];
static int serial_pass(const double *x, int n, const Piece *Ps, int np, double *out) {
  double s = 0.0;
  int uec = SPECIAL;  // actual ulp exponent of s
  int64_t M = 0;
  for (int q = 0; q < np; ++q) {
    const Piece *P = &Ps[q];
    const int pb = q * XB, pn = n - pb < XB ? n - pb : XB;
    if (P->nb > MAXB) {  // dense piece: element by element
      for (int k = 0; k < pn; ++k) s = s + x[pb + k];
      uec = ulp_key(s);
      if (uec != SPECIAL) M = (int64_t)ldexp(s, -key_ue(uec));
      continue;
    }
    if (P->head.len) {
      if (uec == SPECIAL || uec != P->first_ue) { why[0]++; return 0; }
      if (!run_apply(&P->head, &M)) { why[1]++; return 0; }
      s = ldexp((double)M, key_ue(uec));
    }
    for (int j = 0; j < P->nb; ++j) {
      s = s + P->b[j].x;
      uec = ulp_key(s);
      if (P->b[j].run.len) {
        if (uec == SPECIAL || uec != P->b[j].ue) { why[2 + (uec == SPECIAL)]++; return 0; }
        M = (int64_t)ldexp(s, -key_ue(uec));
        if (!run_apply(&P->b[j].run, &M)) {
          if (why[4] < 3) printf("fail piece %d bnd %d/%d M %lld mn %lld mx %lld len %d t %lld %lld ue %d x %g\n", q, j, P->nb, (long long)M, (long long)P->b[j].run.mn, (long long)P->b[j].run.mx, P->b[j].run.len, (long long)P->b[j].run.t[0], (long long)P->b[j].run.t[1], uec, P->b[j].x);
          why[4]++; return 0; }
        s = ldexp((double)M, key_ue(uec));
      } else if (uec != SPECIAL) {
        M = (int64_t)ldexp(s, -key_ue(uec));
      }
    }
  }
  *out = s;
  return 1;
}

static int par_sum2(const double *x, int n, double *out, int *nbnd) {
  const int np = (n + XB - 1) / XB;
  Piece *Ps = malloc(sizeof(Piece) * (np ? np : 1));
  double pre = 0.0;
  *nbnd = 0;
  for (int q = 0; q < np; ++q) {  // piece sums are approximate: any order will do
    const int pb = q * XB, pn = n - pb < XB ? n - pb : XB;
    summarise(x + pb, pn, pre, &Ps[q]);
    *nbnd += Ps[q].nb;
    double ps = 0;
    for (int k = 0; k < pn; ++k) ps += x[pb + k];
    pre += ps;
  }
  const int ok = serial_pass(x, n, Ps, np, out);
  free(Ps);
  return ok;
}

static uint64_t rs = 88172645463325252ull;
static double urand(void) {
  rs ^= rs << 13;
  rs ^= rs >> 7;
  rs ^= rs << 17;
  return (double)(rs >> 11) * 0x1p-53;
}

static int from_file(const char *path) {  // raw doubles: chain sequences to test
  FILE *f = fopen(path, "rb");
  if (!f) return 2;
  fseek(f, 0, SEEK_END);
  const long n = ftell(f) / 8;
  fseek(f, 0, SEEK_SET);
  double *x = malloc(8 * n);
  if (fread(x, 8, n, f) != (size_t)n) return 2;
  fclose(f);
  double got, ref = seq_sum(x, (int)n);
  int nb;
  memset(why, 0, sizeof(why));
  const int ok = par_sum2(x, (int)n, &got, &nb);
  printf("n %ld boundaries %d ok %d same %d why %ld %ld %ld %ld %ld\n", n, nb, ok, ok && memcmp(&got, &ref, 8) == 0,
         why[0], why[1], why[2], why[3], why[4]);
  const int np = (int)((n + XB - 1) / XB);
  int dense = 0;
  double pre = 0.0;
  for (int q = 0; q < np; ++q) {
    Piece P;
    const int pn = n - q * XB < XB ? (int)(n - q * XB) : XB;
    summarise(x + q * XB, pn, pre, &P);
    if (P.nb > MAXB) ++dense;
    for (int k = 0; k < pn; ++k) pre += x[q * XB + k];
  }
  printf("pieces %d dense %d\n", np, dense);
  free(x);
  return 0;
}

int main(int argc, char **argv) {
  if (argc > 1) return from_file(argv[1]);
  const int sizes[] = {1, 2, 3, 7, 64, 100, 1000, 4097, 65536, 400000};
  long trials = 0, fallbacks = 0, wrong = 0, fb_mode[7] = {0}, fb2[7] = {0}, wrong2 = 0;
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
        {
          double g2;
          int nb2;
          if (!par_sum2(x, n, &g2, &nb2)) {
            ++fb2[mode];
          } else if (memcmp(&g2, &ref, 8) != 0) {
            ++wrong2;
            if (wrong2 < 10) printf("WRONG2 mode %d n %d: %.17g vs %.17g\n", mode, n, g2, ref);
          }
        }
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
  for (int m = 0; m < 7; ++m) printf("mode %d fallbacks %ld (v2 %ld)\n", m, fb_mode[m], fb2[m]);
  printf("v2 wrong %ld why %ld %ld %ld %ld %ld\n", wrong2, why[0], why[1], why[2], why[3], why[4]);
  printf("trials %ld fallbacks %ld wrong %ld\n", trials, fallbacks, wrong);
  return wrong != 0 || wrong2 != 0;
}
