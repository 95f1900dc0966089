/*
 * amr_hilbert.c -- CPU restatement of |scipy.signal.hilbert(x)| for a real
 * double x, as modem.fsk_demodulate computes it (modem.py:309, 315).
 *
 * TEST INFRASTRUCTURE ONLY (the oracle's FSK envelope stage; see
 * amr_oracle.c's header).  The product path never links or calls it.
 *
 * The arithmetic lives in third-party code the reference calls, restated
 * here from its published algorithm and pinned bit for bit against it in
 * this container (tests/test_oracle_golden.py::test_oracle_hilbert_is_scipys,
 * tools/pocketfft_probe.py): scipy 1.15.3 / numpy 2.2.6.
 *
 *   scipy.signal.hilbert (signal/_signaltools.py): Xf = scipy.fft.fft(x);
 *     h = [1, 2, ..., 2, 1 (n even), 0, ...] as complex; ifft(Xf * h).
 *   scipy.fft.fft of REAL input is pocketfft's real transform (rfftp, the
 *     FFTPACK-derived radf2/radf3/radf4/radf5 passes, factors 4 first, then
 *     one 2 moved to the front, then odd factors, applied last-factor-first)
 *     with the second half filled by conjugate symmetry (pypocketfft
 *     c2c_sym_internal).
 *   Xf * h: numpy's complex multiply, re = fma(xr, hr, -(xi*hi)),
 *     im = fma(xr, hi, xi*hr) on this AVX-512/FMA3 host.
 *   scipy.fft.ifft: pocketfft's complex transform (cfftp, passes 8 / 4 / 2 /
 *     3 / 5 with the same factor order, backward twiddles w, then x * 1/n,
 *     1/n = double(1 / long double n)).
 *   Twiddles: pocketfft's sincos_2pibyn -- two tables v1 (fine) and v2
 *     (coarse), entries from libm cos / sin of x * ang by octant, ang =
 *     double(0.25L * pi / n) in long double; entry k = v1[k & mask] *
 *     v2[k >> shift] (conjugated mirror above n / 2).
 *   np.abs of complex128 (numpy's AVX-512 kernel): hi * sqrt(fma(r, r, 1)),
 *     hi = max(|re|, |im|), r = min / hi (0 when hi is 0).
 * Only 5-smooth lengths are restated (radices 2, 3, 4, 5, 8: every length
 * the FSK four-step path plans); oracle_hilbert_env returns -1 for others
 * and oracle.py falls back to scipy itself.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fno-fast-math).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { double r, i; } cpx;

static inline cpx cadd(cpx a, cpx b) { cpx c = {a.r + b.r, a.i + b.i}; return c; }
static inline cpx csub(cpx a, cpx b) { cpx c = {a.r - b.r, a.i - b.i}; return c; }
/* special_mul<fwd>: v * conj(w) forward, v * w backward (backward only here) */
static inline cpx smul(cpx v, cpx w) { cpx c = {v.r * w.r - v.i * w.i, v.r * w.i + v.i * w.r}; return c; }
static inline cpx rot90(cpx a) { cpx c = {-a.i, a.r}; return c; }   /* ROTX90<false> */

/* ---- sincos_2pibyn -------------------------------------------------------- */
typedef struct { int64_t n, mask, shift; cpx *v1, *v2; } twid_t;

static cpx calc(int64_t x, int64_t n, double ang)
{
  cpx c;
  x <<= 3;
  if (x < 4 * n) {
    if (x < 2 * n) {
      if (x < n) { c.r = cos((double)x * ang); c.i = sin((double)x * ang); return c; }
      c.r = sin((double)(2 * n - x) * ang); c.i = cos((double)(2 * n - x) * ang); return c;
    }
    x -= 2 * n;
    if (x < n) { c.r = -sin((double)x * ang); c.i = cos((double)x * ang); return c; }
    c.r = -cos((double)(2 * n - x) * ang); c.i = sin((double)(2 * n - x) * ang); return c;
  }
  x = 8 * n - x;
  if (x < 2 * n) {
    if (x < n) { c.r = cos((double)x * ang); c.i = -sin((double)x * ang); return c; }
    c.r = sin((double)(2 * n - x) * ang); c.i = -cos((double)(2 * n - x) * ang); return c;
  }
  x -= 2 * n;
  if (x < n) { c.r = -sin((double)x * ang); c.i = -cos((double)x * ang); return c; }
  c.r = -cos((double)(2 * n - x) * ang); c.i = -sin((double)(2 * n - x) * ang); return c;
}

static int twid_init(twid_t *t, int64_t n)
{
  const double ang = (double)(0.25L * 3.141592653589793238462643383279502884197L / (long double)n);
  const int64_t nval = (n + 2) / 2;
  int64_t shift = 1;
  while ((((int64_t)1) << shift) * (((int64_t)1) << shift) < nval) ++shift;
  t->n = n;
  t->shift = shift;
  t->mask = (((int64_t)1) << shift) - 1;
  const int64_t n1 = t->mask + 1, n2 = (nval + t->mask) / (t->mask + 1);
  t->v1 = malloc(sizeof(cpx) * (size_t)n1);
  t->v2 = malloc(sizeof(cpx) * (size_t)n2);
  if (!t->v1 || !t->v2) return -1;
  t->v1[0].r = 1.0; t->v1[0].i = 0.0;
  for (int64_t i = 1; i < n1; ++i) t->v1[i] = calc(i, n, ang);
  t->v2[0].r = 1.0; t->v2[0].i = 0.0;
  for (int64_t i = 1; i < n2; ++i) t->v2[i] = calc(i * (t->mask + 1), n, ang);
  return 0;
}

static void twid_free(twid_t *t) { free(t->v1); free(t->v2); }

static cpx twid_get(const twid_t *t, int64_t idx)
{
  cpx c;
  if (2 * idx <= t->n) {
    const cpx x1 = t->v1[idx & t->mask], x2 = t->v2[idx >> t->shift];
    c.r = x1.r * x2.r - x1.i * x2.i;
    c.i = x1.r * x2.i + x1.i * x2.r;
    return c;
  }
  idx = t->n - idx;
  const cpx x1 = t->v1[idx & t->mask], x2 = t->v2[idx >> t->shift];
  c.r = x1.r * x2.r - x1.i * x2.i;
  c.i = -(x1.r * x2.i + x1.i * x2.r);
  return c;
}

/* ---- factorisations ------------------------------------------------------- */
static int factorize(int64_t n, int with8, int *f)
{
  int nf = 0;
  if (with8)
    while (n % 8 == 0) { f[nf++] = 8; n /= 8; }
  while (n % 4 == 0) { f[nf++] = 4; n /= 4; }
  if (n % 2 == 0) { n /= 2; f[nf++] = 2; int t = f[0]; f[0] = f[nf - 1]; f[nf - 1] = t; }
  for (int d = 3; (int64_t)d * d <= n; d += 2)
    while (n % d == 0) { f[nf++] = d; n /= d; }
  if (n > 1) { if (n > 5) return -1; f[nf++] = (int)n; }
  for (int k = 0; k < nf; ++k)
    if (f[k] > 5 && f[k] != 8) return -1;
  return nf;
}

/* ---- rfftp forward passes (radfN), real data ------------------------------ */
#define CC(a, b, c) cc[(a) + ido * ((b) + l1 * (c))]
#define WA(x, i) wa[(i) + (x) * (ido - 1)]

static void radf2(int64_t ido, int64_t l1, const double *cc, double *ch, const double *wa)
{
#define CH(a, b, c) ch[(a) + ido * ((b) + 2 * (c))]
  for (int64_t k = 0; k < l1; k++) {
    CH(0, 0, k) = CC(0, k, 0) + CC(0, k, 1);
    CH(ido - 1, 1, k) = CC(0, k, 0) - CC(0, k, 1);
  }
  if ((ido & 1) == 0)
    for (int64_t k = 0; k < l1; k++) {
      CH(0, 1, k) = -CC(ido - 1, k, 1);
      CH(ido - 1, 0, k) = CC(ido - 1, k, 0);
    }
  if (ido <= 2) return;
  for (int64_t k = 0; k < l1; k++)
    for (int64_t i = 2; i < ido; i += 2) {
      const int64_t ic = ido - i;
      const double tr2 = wa[i - 2] * CC(i - 1, k, 1) + wa[i - 1] * CC(i, k, 1);
      const double ti2 = wa[i - 2] * CC(i, k, 1) - wa[i - 1] * CC(i - 1, k, 1);
      CH(i - 1, 0, k) = CC(i - 1, k, 0) + tr2;
      CH(ic - 1, 1, k) = CC(i - 1, k, 0) - tr2;
      CH(i, 0, k) = ti2 + CC(i, k, 0);
      CH(ic, 1, k) = ti2 - CC(i, k, 0);
    }
#undef CH
}

static void radf3(int64_t ido, int64_t l1, const double *cc, double *ch, const double *wa)
{
  const double taur = -0.5, taui = 0.8660254037844386467637231707529362;
#define CH(a, b, c) ch[(a) + ido * ((b) + 3 * (c))]
  for (int64_t k = 0; k < l1; k++) {
    const double cr2 = CC(0, k, 1) + CC(0, k, 2);
    CH(0, 0, k) = CC(0, k, 0) + cr2;
    CH(0, 2, k) = taui * (CC(0, k, 2) - CC(0, k, 1));
    CH(ido - 1, 1, k) = CC(0, k, 0) + taur * cr2;
  }
  if (ido == 1) return;
  for (int64_t k = 0; k < l1; k++)
    for (int64_t i = 2; i < ido; i += 2) {
      const int64_t ic = ido - i;
      const double dr2 = WA(0, i - 2) * CC(i - 1, k, 1) + WA(0, i - 1) * CC(i, k, 1);
      const double di2 = WA(0, i - 2) * CC(i, k, 1) - WA(0, i - 1) * CC(i - 1, k, 1);
      const double dr3 = WA(1, i - 2) * CC(i - 1, k, 2) + WA(1, i - 1) * CC(i, k, 2);
      const double di3 = WA(1, i - 2) * CC(i, k, 2) - WA(1, i - 1) * CC(i - 1, k, 2);
      const double cr2 = dr2 + dr3, ci2 = di2 + di3;
      CH(i - 1, 0, k) = CC(i - 1, k, 0) + cr2;
      CH(i, 0, k) = CC(i, k, 0) + ci2;
      const double tr2 = CC(i - 1, k, 0) + taur * cr2, ti2 = CC(i, k, 0) + taur * ci2;
      const double tr3 = taui * (di2 - di3), ti3 = taui * (dr3 - dr2);
      CH(i - 1, 2, k) = tr2 + tr3;
      CH(ic - 1, 1, k) = tr2 - tr3;
      CH(i, 2, k) = ti2 + ti3;
      CH(ic, 1, k) = ti3 - ti2;
    }
#undef CH
}

static void radf4(int64_t ido, int64_t l1, const double *cc, double *ch, const double *wa)
{
  const double hsqt2 = 0.707106781186547524400844362104849;
#define CH(a, b, c) ch[(a) + ido * ((b) + 4 * (c))]
  for (int64_t k = 0; k < l1; k++) {
    const double tr1 = CC(0, k, 3) + CC(0, k, 1);
    CH(0, 2, k) = CC(0, k, 3) - CC(0, k, 1);
    const double tr2 = CC(0, k, 0) + CC(0, k, 2);
    CH(ido - 1, 1, k) = CC(0, k, 0) - CC(0, k, 2);
    CH(0, 0, k) = tr2 + tr1;
    CH(ido - 1, 3, k) = tr2 - tr1;
  }
  if ((ido & 1) == 0)
    for (int64_t k = 0; k < l1; k++) {
      const double ti1 = -hsqt2 * (CC(ido - 1, k, 1) + CC(ido - 1, k, 3));
      const double tr1 = hsqt2 * (CC(ido - 1, k, 1) - CC(ido - 1, k, 3));
      CH(ido - 1, 0, k) = CC(ido - 1, k, 0) + tr1;
      CH(ido - 1, 2, k) = CC(ido - 1, k, 0) - tr1;
      CH(0, 3, k) = ti1 + CC(ido - 1, k, 2);
      CH(0, 1, k) = ti1 - CC(ido - 1, k, 2);
    }
  if (ido <= 2) return;
  for (int64_t k = 0; k < l1; k++)
    for (int64_t i = 2; i < ido; i += 2) {
      const int64_t ic = ido - i;
      const double cr2 = WA(0, i - 2) * CC(i - 1, k, 1) + WA(0, i - 1) * CC(i, k, 1);
      const double ci2 = WA(0, i - 2) * CC(i, k, 1) - WA(0, i - 1) * CC(i - 1, k, 1);
      const double cr3 = WA(1, i - 2) * CC(i - 1, k, 2) + WA(1, i - 1) * CC(i, k, 2);
      const double ci3 = WA(1, i - 2) * CC(i, k, 2) - WA(1, i - 1) * CC(i - 1, k, 2);
      const double cr4 = WA(2, i - 2) * CC(i - 1, k, 3) + WA(2, i - 1) * CC(i, k, 3);
      const double ci4 = WA(2, i - 2) * CC(i, k, 3) - WA(2, i - 1) * CC(i - 1, k, 3);
      const double tr1 = cr4 + cr2, tr4 = cr4 - cr2;
      const double ti1 = ci2 + ci4, ti4 = ci2 - ci4;
      const double tr2 = CC(i - 1, k, 0) + cr3, tr3 = CC(i - 1, k, 0) - cr3;
      const double ti2 = CC(i, k, 0) + ci3, ti3 = CC(i, k, 0) - ci3;
      CH(i - 1, 0, k) = tr2 + tr1;
      CH(ic - 1, 3, k) = tr2 - tr1;
      CH(i, 0, k) = ti1 + ti2;
      CH(ic, 3, k) = ti1 - ti2;
      CH(i - 1, 2, k) = tr3 + ti4;
      CH(ic - 1, 1, k) = tr3 - ti4;
      CH(i, 2, k) = tr4 + ti3;
      CH(ic, 1, k) = tr4 - ti3;
    }
#undef CH
}

static void radf5(int64_t ido, int64_t l1, const double *cc, double *ch, const double *wa)
{
  const double tr11 = 0.3090169943749474241022934171828191, ti11 = 0.9510565162951535721164393333793821;
  const double tr12 = -0.8090169943749474241022934171828191, ti12 = 0.5877852522924731291687059546390728;
#define CH(a, b, c) ch[(a) + ido * ((b) + 5 * (c))]
  for (int64_t k = 0; k < l1; k++) {
    const double cr2 = CC(0, k, 4) + CC(0, k, 1), ci5 = CC(0, k, 4) - CC(0, k, 1);
    const double cr3 = CC(0, k, 3) + CC(0, k, 2), ci4 = CC(0, k, 3) - CC(0, k, 2);
    CH(0, 0, k) = CC(0, k, 0) + cr2 + cr3;
    CH(ido - 1, 1, k) = CC(0, k, 0) + tr11 * cr2 + tr12 * cr3;
    CH(0, 2, k) = ti11 * ci5 + ti12 * ci4;
    CH(ido - 1, 3, k) = CC(0, k, 0) + tr12 * cr2 + tr11 * cr3;
    CH(0, 4, k) = ti12 * ci5 - ti11 * ci4;
  }
  if (ido == 1) return;
  for (int64_t k = 0; k < l1; k++)
    for (int64_t i = 2; i < ido; i += 2) {
      const int64_t ic = ido - i;
      const double dr2 = WA(0, i - 2) * CC(i - 1, k, 1) + WA(0, i - 1) * CC(i, k, 1);
      const double di2 = WA(0, i - 2) * CC(i, k, 1) - WA(0, i - 1) * CC(i - 1, k, 1);
      const double dr3 = WA(1, i - 2) * CC(i - 1, k, 2) + WA(1, i - 1) * CC(i, k, 2);
      const double di3 = WA(1, i - 2) * CC(i, k, 2) - WA(1, i - 1) * CC(i - 1, k, 2);
      const double dr4 = WA(2, i - 2) * CC(i - 1, k, 3) + WA(2, i - 1) * CC(i, k, 3);
      const double di4 = WA(2, i - 2) * CC(i, k, 3) - WA(2, i - 1) * CC(i - 1, k, 3);
      const double dr5 = WA(3, i - 2) * CC(i - 1, k, 4) + WA(3, i - 1) * CC(i, k, 4);
      const double di5 = WA(3, i - 2) * CC(i, k, 4) - WA(3, i - 1) * CC(i - 1, k, 4);
      const double cr2 = dr5 + dr2, ci5 = dr5 - dr2;
      const double ci2 = di2 + di5, cr5 = di2 - di5;
      const double cr3 = dr4 + dr3, ci4 = dr4 - dr3;
      const double ci3 = di3 + di4, cr4 = di3 - di4;
      CH(i - 1, 0, k) = CC(i - 1, k, 0) + cr2 + cr3;
      CH(i, 0, k) = CC(i, k, 0) + ci2 + ci3;
      const double tr2 = CC(i - 1, k, 0) + tr11 * cr2 + tr12 * cr3;
      const double ti2 = CC(i, k, 0) + tr11 * ci2 + tr12 * ci3;
      const double tr3 = CC(i - 1, k, 0) + tr12 * cr2 + tr11 * cr3;
      const double ti3 = CC(i, k, 0) + tr12 * ci2 + tr11 * ci3;
      const double tr5 = cr5 * ti11 + cr4 * ti12, tr4 = cr5 * ti12 - cr4 * ti11;
      const double ti5 = ci5 * ti11 + ci4 * ti12, ti4 = ci5 * ti12 - ci4 * ti11;
      CH(i - 1, 2, k) = tr2 + tr5;
      CH(ic - 1, 1, k) = tr2 - tr5;
      CH(i, 2, k) = ti2 + ti5;
      CH(ic, 1, k) = ti5 - ti2;
      CH(i - 1, 4, k) = tr3 + tr4;
      CH(ic - 1, 3, k) = tr3 - tr4;
      CH(i, 4, k) = ti3 + ti4;
      CH(ic, 3, k) = ti4 - ti3;
    }
#undef CH
}
#undef CC
#undef WA

/* ---- cfftp backward passes, complex data ---------------------------------- */
#define CC(a, b, c) cc[(a) + ido * ((b) + IP * (c))]
#define CH(a, b, c) ch[(a) + ido * ((b) + l1 * (c))]
#define WA(x, i) wa[(i) - 1 + (x) * (ido - 1)]

static void pass2b(int64_t ido, int64_t l1, const cpx *cc, cpx *ch, const cpx *wa)
{
  enum { IP = 2 };
  for (int64_t k = 0; k < l1; ++k) {
    CH(0, k, 0) = cadd(CC(0, 0, k), CC(0, 1, k));
    CH(0, k, 1) = csub(CC(0, 0, k), CC(0, 1, k));
    for (int64_t i = 1; i < ido; ++i) {
      CH(i, k, 0) = cadd(CC(i, 0, k), CC(i, 1, k));
      CH(i, k, 1) = smul(csub(CC(i, 0, k), CC(i, 1, k)), WA(0, i));
    }
  }
}

static void pass3b(int64_t ido, int64_t l1, const cpx *cc, cpx *ch, const cpx *wa)
{
  enum { IP = 3 };
  const double tw1r = -0.5, tw1i = 0.8660254037844386467637231707529362;
  for (int64_t k = 0; k < l1; ++k)
    for (int64_t i = 0; i < ido; ++i) {
      const cpx t0 = CC(i, 0, k), t1 = cadd(CC(i, 1, k), CC(i, 2, k)), t2 = csub(CC(i, 1, k), CC(i, 2, k));
      CH(i, k, 0) = cadd(t0, t1);
      const cpx ca = {t0.r + t1.r * tw1r, t0.i + t1.i * tw1r};
      const cpx cb = {-(t2.i * tw1i), t2.r * tw1i};
      if (i == 0) {
        CH(0, k, 1) = cadd(ca, cb);
        CH(0, k, 2) = csub(ca, cb);
      } else {
        CH(i, k, 1) = smul(cadd(ca, cb), WA(0, i));
        CH(i, k, 2) = smul(csub(ca, cb), WA(1, i));
      }
    }
}

static void pass4b(int64_t ido, int64_t l1, const cpx *cc, cpx *ch, const cpx *wa)
{
  enum { IP = 4 };
  for (int64_t k = 0; k < l1; ++k)
    for (int64_t i = 0; i < ido; ++i) {
      const cpx t2 = cadd(CC(i, 0, k), CC(i, 2, k)), t1 = csub(CC(i, 0, k), CC(i, 2, k));
      const cpx t3 = cadd(CC(i, 1, k), CC(i, 3, k));
      const cpx t4 = rot90(csub(CC(i, 1, k), CC(i, 3, k)));
      if (i == 0) {
        CH(0, k, 0) = cadd(t2, t3);
        CH(0, k, 2) = csub(t2, t3);
        CH(0, k, 1) = cadd(t1, t4);
        CH(0, k, 3) = csub(t1, t4);
      } else {
        CH(i, k, 0) = cadd(t2, t3);
        CH(i, k, 1) = smul(cadd(t1, t4), WA(0, i));
        CH(i, k, 2) = smul(csub(t2, t3), WA(1, i));
        CH(i, k, 3) = smul(csub(t1, t4), WA(2, i));
      }
    }
}

static void pass5b(int64_t ido, int64_t l1, const cpx *cc, cpx *ch, const cpx *wa)
{
  enum { IP = 5 };
  const double tw1r = 0.3090169943749474241022934171828191, tw1i = 0.9510565162951535721164393333793821;
  const double tw2r = -0.8090169943749474241022934171828191, tw2i = 0.5877852522924731291687059546390728;
  for (int64_t k = 0; k < l1; ++k)
    for (int64_t i = 0; i < ido; ++i) {
      const cpx t0 = CC(i, 0, k);
      const cpx t1 = cadd(CC(i, 1, k), CC(i, 4, k)), t4 = csub(CC(i, 1, k), CC(i, 4, k));
      const cpx t2 = cadd(CC(i, 2, k), CC(i, 3, k)), t3 = csub(CC(i, 2, k), CC(i, 3, k));
      CH(i, k, 0).r = t0.r + t1.r + t2.r;
      CH(i, k, 0).i = t0.i + t1.i + t2.i;
      for (int s = 0; s < 2; ++s) {
        const int u1 = s ? 2 : 1, u2 = s ? 3 : 4;
        const double twar = s ? tw2r : tw1r, twbr = s ? tw1r : tw2r;
        const double twai = s ? tw2i : tw1i, twbi = s ? -tw1i : tw2i;
        const cpx ca = {t0.r + twar * t1.r + twbr * t2.r, t0.i + twar * t1.i + twbr * t2.i};
        const cpx cb = {-(twai * t4.i + twbi * t3.i), twai * t4.r + twbi * t3.r};
        if (i == 0) {
          CH(0, k, u1) = cadd(ca, cb);
          CH(0, k, u2) = csub(ca, cb);
        } else {
          CH(i, k, u1) = smul(cadd(ca, cb), WA(u1 - 1, i));
          CH(i, k, u2) = smul(csub(ca, cb), WA(u2 - 1, i));
        }
      }
    }
}

static inline cpx rot45b(cpx a)
{
  const double h = 0.707106781186547524400844362104849;
  cpx c = {h * (a.r - a.i), h * (a.i + a.r)};
  return c;
}
static inline cpx rot135b(cpx a)
{
  const double h = 0.707106781186547524400844362104849;
  cpx c = {h * (-a.r - a.i), h * (a.r - a.i)};
  return c;
}

static void pass8b(int64_t ido, int64_t l1, const cpx *cc, cpx *ch, const cpx *wa)
{
  enum { IP = 8 };
  for (int64_t k = 0; k < l1; ++k)
    for (int64_t i = 0; i < ido; ++i) {
      cpx a1 = cadd(CC(i, 1, k), CC(i, 5, k)), a5 = csub(CC(i, 1, k), CC(i, 5, k));
      cpx a3 = cadd(CC(i, 3, k), CC(i, 7, k)), a7 = csub(CC(i, 3, k), CC(i, 7, k));
      cpx t = a1;
      a1 = cadd(t, a3);
      a3 = rot90(csub(t, a3));
      a7 = rot90(a7);
      t = a5;
      a5 = rot45b(cadd(t, a7));
      a7 = rot135b(csub(t, a7));
      cpx a0 = cadd(CC(i, 0, k), CC(i, 4, k)), a4 = csub(CC(i, 0, k), CC(i, 4, k));
      cpx a2 = cadd(CC(i, 2, k), CC(i, 6, k)), a6 = csub(CC(i, 2, k), CC(i, 6, k));
      if (i == 0) {
        const cpx s02 = cadd(a0, a2), d02 = csub(a0, a2);
        CH(0, k, 0) = cadd(s02, a1);
        CH(0, k, 4) = csub(s02, a1);
        CH(0, k, 2) = cadd(d02, a3);
        CH(0, k, 6) = csub(d02, a3);
        a6 = rot90(a6);
        const cpx s46 = cadd(a4, a6), d46 = csub(a4, a6);
        CH(0, k, 1) = cadd(s46, a5);
        CH(0, k, 5) = csub(s46, a5);
        CH(0, k, 3) = cadd(d46, a7);
        CH(0, k, 7) = csub(d46, a7);
      } else {
        t = a0;
        a0 = cadd(t, a2);
        a2 = csub(t, a2);
        CH(i, k, 0) = cadd(a0, a1);
        CH(i, k, 4) = smul(csub(a0, a1), WA(3, i));
        CH(i, k, 2) = smul(cadd(a2, a3), WA(1, i));
        CH(i, k, 6) = smul(csub(a2, a3), WA(5, i));
        a6 = rot90(a6);
        t = a4;
        a4 = cadd(t, a6);
        a6 = csub(t, a6);
        CH(i, k, 1) = smul(cadd(a4, a5), WA(0, i));
        CH(i, k, 5) = smul(csub(a4, a5), WA(4, i));
        CH(i, k, 3) = smul(cadd(a6, a7), WA(2, i));
        CH(i, k, 7) = smul(csub(a6, a7), WA(6, i));
      }
    }
}
#undef CC
#undef CH
#undef WA

/* |hilbert(x)| (x real, length n), into env.  0, or -1 if n is not 5-smooth. */
int oracle_hilbert_env(const double *x, int64_t n, double *env)
{
  int fr[64], fc[64];
  const int nr = factorize(n, 0, fr), nc = factorize(n, 1, fc);
  if (n < 1 || nr < 0 || nc < 0) return -1;
  twid_t tw;
  double *r1 = malloc(sizeof(double) * (size_t)n), *r2 = malloc(sizeof(double) * (size_t)n);
  cpx *c1 = malloc(sizeof(cpx) * (size_t)n), *c2 = malloc(sizeof(cpx) * (size_t)n);
  double *rtw = malloc(sizeof(double) * (size_t)(2 * n + 8));
  cpx *ctw = malloc(sizeof(cpx) * (size_t)(8 * n + 8));
  int rc = (r1 && r2 && c1 && c2 && rtw && ctw) ? twid_init(&tw, n) : -1;
  if (rc == 0) {
    /* rfftp twiddles, per factor in factor order */
    const double *rt[64];
    int64_t off = 0, l1 = 1;
    for (int k = 0; k < nr; ++k) {
      const int64_t ip = fr[k], ido = n / (l1 * ip);
      rt[k] = rtw + off;
      if (k < nr - 1)
        for (int64_t j = 1; j < ip; ++j)
          for (int64_t i = 1; i <= (ido - 1) / 2; ++i) {
            const cpx w = twid_get(&tw, j * l1 * i);
            rtw[off + (j - 1) * (ido - 1) + 2 * i - 2] = w.r;
            rtw[off + (j - 1) * (ido - 1) + 2 * i - 1] = w.i;
          }
      off += (ip - 1) * (ido - 1);
      l1 *= ip;
    }
    /* forward real transform, last factor first */
    memcpy(r1, x, sizeof(double) * (size_t)n);
    double *p1 = r1, *p2 = r2;
    l1 = n;
    for (int k1 = 0; k1 < nr; ++k1) {
      const int k = nr - k1 - 1;
      const int64_t ip = fr[k], ido = n / l1;
      l1 /= ip;
      if (ip == 4) radf4(ido, l1, p1, p2, rt[k]);
      else if (ip == 2) radf2(ido, l1, p1, p2, rt[k]);
      else if (ip == 3) radf3(ido, l1, p1, p2, rt[k]);
      else radf5(ido, l1, p1, p2, rt[k]);
      double *t = p1; p1 = p2; p2 = t;
    }
    /* halfcomplex -> spectrum (pypocketfft c2c_sym: conjugate mirror), times h */
    cpx *X = c1;
    X[0].r = p1[0]; X[0].i = 0.0;
    for (int64_t i = 1; i <= (n - 1) / 2; ++i) {
      X[i].r = p1[2 * i - 1]; X[i].i = p1[2 * i];
      X[n - i].r = p1[2 * i - 1]; X[n - i].i = -p1[2 * i];
    }
    if (n % 2 == 0) { X[n / 2].r = p1[n - 1]; X[n / 2].i = 0.0; }
    for (int64_t i = 0; i < n; ++i) {
      /* scipy.signal.hilbert's h: 1 at 0 (and n/2), 2 below n/2, 0 above */
      const double hr = (i == 0 || 2 * i == n) ? 1.0 : (2 * i < n ? 2.0 : 0.0), hi = 0.0;
      const double xr = X[i].r, xi = X[i].i;
      X[i].r = fma(xr, hr, -(xi * hi));
      X[i].i = fma(xr, hi, xi * hr);
    }
    /* cfftp twiddles (complex), per factor */
    const cpx *ct[64];
    off = 0; l1 = 1;
    for (int k = 0; k < nc; ++k) {
      const int64_t ip = fc[k], ido = n / (l1 * ip);
      ct[k] = ctw + off;
      for (int64_t j = 1; j < ip; ++j)
        for (int64_t i = 1; i < ido; ++i) ctw[off + (j - 1) * (ido - 1) + i - 1] = twid_get(&tw, j * l1 * i);
      off += (ip - 1) * (ido - 1);
      l1 *= ip;
    }
    /* backward complex transform, first factor first */
    cpx *q1 = c1, *q2 = c2;
    l1 = 1;
    for (int k = 0; k < nc; ++k) {
      const int64_t ip = fc[k], ido = n / (l1 * ip);
      if (ip == 4) pass4b(ido, l1, q1, q2, ct[k]);
      else if (ip == 8) pass8b(ido, l1, q1, q2, ct[k]);
      else if (ip == 2) pass2b(ido, l1, q1, q2, ct[k]);
      else if (ip == 3) pass3b(ido, l1, q1, q2, ct[k]);
      else pass5b(ido, l1, q1, q2, ct[k]);
      cpx *t = q1; q1 = q2; q2 = t;
      l1 *= ip;
    }
    const double fct = (double)(1.0L / (long double)n);
    for (int64_t i = 0; i < n; ++i) {
      const double re = q1[i].r * fct, im = q1[i].i * fct;
      /* np.abs(complex128), numpy's AVX-512 kernel */
      const double ar = fabs(re), ai = fabs(im);
      const double hi = ar > ai ? ar : ai, lo = ar > ai ? ai : ar;
      env[i] = hi == 0.0 ? 0.0 : hi * sqrt(fma(lo / hi, lo / hi, 1.0));
    }
    twid_free(&tw);
  }
  free(r1); free(r2); free(c1); free(c2); free(rtw); free(ctw);
  return rc;
}
