/*
 * amr_pocketfft.c -- CPU restatement of the FFTs the reference's FSK and WAV
 * paths run through scipy.fft (pocketfft), and of the two reference steps
 * built on them:
 *   |scipy.signal.hilbert(x)|      modem.fsk_demodulate       (modem.py:309, 315)
 *   scipy.signal.resample(x, num)  decoder.decode_wav_file    (decoder.py:385-387)
 *
 * TEST INFRASTRUCTURE ONLY (the oracle; see amr_oracle.c's header).  The
 * product path never links or calls it.
 *
 * The arithmetic lives in third-party code the reference calls -- scipy 1.15.3
 * (scipy.fft's bundled pocketfft C++ header, pypocketfft) and numpy 2.2.6 --
 * restated here from pocketfft's published algorithm and pinned bit for bit
 * against scipy + numpy in this container on every length 1..2000 and the
 * FSK / WAV lengths (tests/test_oracle_golden.py::test_oracle_pocketfft_*,
 * ::test_oracle_hilbert_is_scipys, ::test_oracle_resample_is_scipys).
 *
 * pocketfft, as scipy.fft runs it on one float64 row:
 *   plan choice (pocketfft_c / pocketfft_r): lengths < 50 or whose largest
 *     prime factor p has p*p <= n run the FFTPACK-style plan; otherwise
 *     Bluestein when 1.5 * 2 * cost(good_size(2n-1)) < cost(n) (x 0.5 for the
 *     real plan), cost = n * sum over factors (2 per factor 2, p for 3 and 5,
 *     1.1 p above), good_size = the smallest 2^a 3^b 5^c 7^d 11^e >= n.
 *   complex plan (cfftp): factors 8s, 4s, one 2 moved to the front, odd
 *     factors ascending; passes 2/3/4/5/7/8/11 and a generic pass (p > 11)
 *     applied first factor first; twiddles w^(j l1 i) per factor; the result
 *     times fct (skipped when fct == 1).
 *   real plan (rfftp): factors 4s, one 2 to the front, odd factors; forward
 *     passes radf2/3/4/5/g last factor first, backward radb2/3/4/5/g first
 *     factor first; output in FFTPACK's halfcomplex order r0 r1 i1 r2 i2 ...
 *   Bluestein (fftblue): chirp b_m = w_2n^(m^2 mod 2n) from sincos_2pibyn(2n),
 *     a length-n2 cfftp convolution with the FFT of b/n2 precomputed.
 *   Twiddles: sincos_2pibyn -- two tables v1 (fine) and v2 (coarse), entries
 *     from glibc's sincos of x * ang by octant (gcc merges pocketfft's
 *     cos / sin pair; sincos differs from sin / cos in the last ulp for some
 *     arguments), ang = double(0.25L * pi / n) in long double; entry k =
 *     v1[k & mask] * v2[k >> shift] (conjugated mirror above n / 2).
 *   scipy.fft.fft of REAL input: the real plan forward, then the spectrum's
 *     second half filled by conjugate symmetry over bins 0..n/2 (pypocketfft
 *     c2c_sym_internal's rev_iter -- which also conjugates bins 0 and n/2,
 *     leaving -0.0 imaginary parts there).
 * numpy:
 *   Xf * h (complex128 multiply, this AVX-512/FMA3 host):
 *     re = fma(xr, hr, -(xi*hi)), im = fma(xr, hi, xi*hr)  
 *   np.abs(complex128): hi * sqrt(fma(r, r, 1)), hi = max(|re|, |im|),
 *     r = min / hi (0 when hi is 0).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fno-fast-math).
 *
 * Derived from pocketfft (the FFT library bundled with scipy 1.15.3 as
 * scipy.fft's pypocketfft), whose notice follows; the FFTPACK algorithms it
 * implements are by Paul N. Swarztrauber (public domain).
 *
 *   Copyright (C) 2010-2019 Max-Planck-Society
 *   All rights reserved.
 *
 *   Redistribution and use in source and binary forms, with or without
 *   modification, are permitted provided that the following conditions are met:
 *
 *   * Redistributions of source code must retain the above copyright notice,
 *     this list of conditions and the following disclaimer.
 *   * Redistributions in binary form must reproduce the above copyright notice,
 *     this list of conditions and the following disclaimer in the documentation
 *     and/or other materials provided with the distribution.
 *   * Neither the name of the copyright holder nor the names of its contributors
 *     may be used to endorse or promote products derived from this software
 *     without specific prior written permission.
 *
 *   THIS SOFTWARE IS PROVIDED BY THE COPYRIGHT HOLDERS AND CONTRIBUTORS "AS IS"
 *   AND ANY EXPRESS OR IMPLIED WARRANTIES, INCLUDING, BUT NOT LIMITED TO, THE
 *   IMPLIED WARRANTIES OF MERCHANTABILITY AND FITNESS FOR A PARTICULAR PURPOSE ARE
 *   DISCLAIMED. IN NO EVENT SHALL THE COPYRIGHT HOLDER OR CONTRIBUTORS BE LIABLE
 *   FOR ANY DIRECT, INDIRECT, INCIDENTAL, SPECIAL, EXEMPLARY, OR CONSEQUENTIAL
 *   DAMAGES (INCLUDING, BUT NOT LIMITED TO, PROCUREMENT OF SUBSTITUTE GOODS OR
 *   SERVICES; LOSS OF USE, DATA, OR PROFITS; OR BUSINESS INTERRUPTION) HOWEVER
 *   CAUSED AND ON ANY THEORY OF LIABILITY, WHETHER IN CONTRACT, STRICT LIABILITY,
 *   OR TORT (INCLUDING NEGLIGENCE OR OTHERWISE) ARISING IN ANY WAY OUT OF THE USE
 *   OF THIS SOFTWARE, EVEN IF ADVISED OF THE POSSIBILITY OF SUCH DAMAGE.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { double r, i; } cpx;

static inline cpx cadd(cpx a, cpx b) { cpx c = {a.r + b.r, a.i + b.i}; return c; }
static inline cpx csub(cpx a, cpx b) { cpx c = {a.r - b.r, a.i - b.i}; return c; }
static inline cpx cscale(cpx a, double f) { cpx c = {a.r * f, a.i * f}; return c; }
/* special_mul<fwd>: v * conj(w) forward, v * w backward */
static inline cpx smul(cpx v, cpx w, int fwd)
{
  cpx c;
  if (fwd) { c.r = v.r * w.r + v.i * w.i; c.i = v.i * w.r - v.r * w.i; }
  else { c.r = v.r * w.r - v.i * w.i; c.i = v.r * w.i + v.i * w.r; }
  return c;
}
/* ROTX90<fwd>: times -i forward, +i backward */
static inline cpx rot90(cpx a, int fwd) { cpx c; if (fwd) { c.r = a.i; c.i = -a.r; } else { c.r = -a.i; c.i = a.r; } return c; }

/* ---- sincos_2pibyn -------------------------------------------------------- */
typedef struct { int64_t n, mask, shift; cpx *v1, *v2; } twid_t;

/* cos and sin of one argument through glibc's sincos: scipy's pocketfft is
 * built by gcc, which merges the std::cos / std::sin pair of sincos_2pibyn's
 * calc into one sincos call -- and glibc's sincos differs from its sin / cos
 * in the last ulp for some arguments (e.g. sin(70 * pi / 372)), so the pair
 * must come from sincos to equal scipy's twiddles */
static void sc(double v, double *s, double *c) { sincos(v, s, c); }

static cpx calc(int64_t x, int64_t n, double ang)
{
  cpx c;
  double sv, cv;
  x <<= 3;
  if (x < 4 * n) {
    if (x < 2 * n) {
      if (x < n) { sc((double)x * ang, &sv, &cv); c.r = cv; c.i = sv; return c; }
      sc((double)(2 * n - x) * ang, &sv, &cv); c.r = sv; c.i = cv; return c;
    }
    x -= 2 * n;
    if (x < n) { sc((double)x * ang, &sv, &cv); c.r = -sv; c.i = cv; return c; }
    sc((double)(2 * n - x) * ang, &sv, &cv); c.r = -cv; c.i = sv; return c;
  }
  x = 8 * n - x;
  if (x < 2 * n) {
    if (x < n) { sc((double)x * ang, &sv, &cv); c.r = cv; c.i = -sv; return c; }
    sc((double)(2 * n - x) * ang, &sv, &cv); c.r = sv; c.i = -cv; return c;
  }
  x -= 2 * n;
  if (x < n) { sc((double)x * ang, &sv, &cv); c.r = -sv; c.i = -cv; return c; }
  sc((double)(2 * n - x) * ang, &sv, &cv); c.r = -cv; c.i = -sv; return c;
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
  if (!t->v1 || !t->v2) { free(t->v1); free(t->v2); t->v1 = t->v2 = NULL; return -1; }
  t->v1[0].r = 1.0; t->v1[0].i = 0.0;
  for (int64_t i = 1; i < n1; ++i) t->v1[i] = calc(i, n, ang);
  t->v2[0].r = 1.0; t->v2[0].i = 0.0;
  for (int64_t i = 1; i < n2; ++i) t->v2[i] = calc(i * (t->mask + 1), n, ang);
  return 0;
}

static void twid_free(twid_t *t) { free(t->v1); free(t->v2); t->v1 = t->v2 = NULL; }

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

/* ---- pocketfft's util ------------------------------------------------------ */
static int64_t largest_prime_factor(int64_t n)
{
  int64_t res = 1;
  while ((n & 1) == 0) { res = 2; n >>= 1; }
  for (int64_t x = 3; x * x <= n; x += 2)
    while (n % x == 0) { res = x; n /= x; }
  if (n > 1) res = n;
  return res;
}

static double cost_guess(int64_t n)
{
  const double lfp = 1.1;   /* penalty for non-hardcoded larger factors */
  const int64_t ni = n;
  double result = 0.;
  while ((n & 1) == 0) { result += 2; n >>= 1; }
  for (int64_t x = 3; x * x <= n; x += 2)
    while (n % x == 0) {
      result += (x <= 5) ? (double)x : lfp * (double)x;
      n /= x;
    }
  if (n > 1) result += (n <= 5) ? (double)n : lfp * (double)n;
  return result * (double)ni;
}

/* smallest 2^a 3^b 5^c 7^d 11^e >= n */
static int64_t good_size_cmplx(int64_t n)
{
  if (n <= 12) return n;
  int64_t best = 2 * n;
  for (int64_t f11 = 1; f11 < best; f11 *= 11)
    for (int64_t f117 = f11; f117 < best; f117 *= 7)
      for (int64_t f1175 = f117; f1175 < best; f1175 *= 5) {
        int64_t x = f1175;
        while (x < n) x *= 2;
        for (;;) {
          if (x < n) x *= 3;
          else if (x > n) {
            if (x < best) best = x;
            if (x & 1) break;
            x >>= 1;
          } else return n;
        }
      }
  return best;
}

/* 1 when pocketfft_{c,r}(n) picks Bluestein */
static int use_bluestein(int64_t n, int real)
{
  const int64_t tmp = (n < 50) ? 0 : largest_prime_factor(n);
  if (tmp * tmp <= n) return 0;
  const double comp1 = real ? 0.5 * cost_guess(n) : cost_guess(n);
  double comp2 = 2 * cost_guess(good_size_cmplx(2 * n - 1));
  comp2 *= 1.5;   /* pocketfft's fudge factor */
  return comp2 < comp1;
}

/* ---- factorisations ------------------------------------------------------- */
#define MAXF 64
static int factorize(int64_t n, int with8, int64_t *f)
{
  int nf = 0;
  if (with8)
    while ((n & 7) == 0) { f[nf++] = 8; n >>= 3; }
  while ((n & 3) == 0) { f[nf++] = 4; n >>= 2; }
  if ((n & 1) == 0) { n >>= 1; f[nf++] = 2; int64_t t = f[0]; f[0] = f[nf - 1]; f[nf - 1] = t; }
  for (int64_t d = 3; d * d <= n; d += 2)
    while (n % d == 0) { f[nf++] = d; n /= d; }
  if (n > 1) f[nf++] = n;
  return nf;
}

/* ======================= complex plan (cfftp) ============================== */
typedef struct {
  int64_t len;
  int nf;
  int64_t fct[MAXF];
  cpx *tw[MAXF], *tws[MAXF];
  cpx *mem;
} cfftp_t;

static int cfftp_init(cfftp_t *p, int64_t len)
{
  memset(p, 0, sizeof(*p));
  p->len = len;
  if (len == 1) return 0;
  p->nf = factorize(len, 1, p->fct);
  int64_t twsz = 0, l1 = 1;
  for (int k = 0; k < p->nf; ++k) {
    const int64_t ip = p->fct[k], ido = len / (l1 * ip);
    twsz += (ip - 1) * (ido - 1);
    if (ip > 11) twsz += ip;
    l1 *= ip;
  }
  p->mem = malloc(sizeof(cpx) * (size_t)(twsz + 1));
  twid_t comp;
  if (!p->mem || twid_init(&comp, len)) { free(p->mem); p->mem = NULL; return -1; }
  int64_t memofs = 0;
  l1 = 1;
  for (int k = 0; k < p->nf; ++k) {
    const int64_t ip = p->fct[k], ido = len / (l1 * ip);
    p->tw[k] = p->mem + memofs;
    memofs += (ip - 1) * (ido - 1);
    for (int64_t j = 1; j < ip; ++j)
      for (int64_t i = 1; i < ido; ++i) p->tw[k][(j - 1) * (ido - 1) + i - 1] = twid_get(&comp, j * l1 * i);
    if (ip > 11) {
      p->tws[k] = p->mem + memofs;
      memofs += ip;
      for (int64_t j = 0; j < ip; ++j) p->tws[k][j] = twid_get(&comp, j * l1 * ido);
    }
    l1 *= ip;
  }
  twid_free(&comp);
  return 0;
}

static void cfftp_free(cfftp_t *p) { free(p->mem); p->mem = NULL; }

#define CC(a, b, c) cc[(a) + ido * ((b) + IP * (c))]
#define CH(a, b, c) ch[(a) + ido * ((b) + l1 * (c))]
#define WA(x, i) wa[(i) - 1 + (x) * (ido - 1)]

static void pass2(int64_t ido, int64_t l1, const cpx *cc, cpx *ch, const cpx *wa, int fwd)
{
  enum { IP = 2 };
  for (int64_t k = 0; k < l1; ++k) {
    CH(0, k, 0) = cadd(CC(0, 0, k), CC(0, 1, k));
    CH(0, k, 1) = csub(CC(0, 0, k), CC(0, 1, k));
    for (int64_t i = 1; i < ido; ++i) {
      CH(i, k, 0) = cadd(CC(i, 0, k), CC(i, 1, k));
      CH(i, k, 1) = smul(csub(CC(i, 0, k), CC(i, 1, k)), WA(0, i), fwd);
    }
  }
}

static void pass3(int64_t ido, int64_t l1, const cpx *cc, cpx *ch, const cpx *wa, int fwd)
{
  enum { IP = 3 };
  const double tw1r = -0.5, tw1i = (fwd ? -1 : 1) * 0.8660254037844386467637231707529362;
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
        CH(i, k, 1) = smul(cadd(ca, cb), WA(0, i), fwd);
        CH(i, k, 2) = smul(csub(ca, cb), WA(1, i), fwd);
      }
    }
}

static void pass4(int64_t ido, int64_t l1, const cpx *cc, cpx *ch, const cpx *wa, int fwd)
{
  enum { IP = 4 };
  for (int64_t k = 0; k < l1; ++k)
    for (int64_t i = 0; i < ido; ++i) {
      const cpx t2 = cadd(CC(i, 0, k), CC(i, 2, k)), t1 = csub(CC(i, 0, k), CC(i, 2, k));
      const cpx t3 = cadd(CC(i, 1, k), CC(i, 3, k));
      const cpx t4 = rot90(csub(CC(i, 1, k), CC(i, 3, k)), fwd);
      if (i == 0) {
        CH(0, k, 0) = cadd(t2, t3);
        CH(0, k, 2) = csub(t2, t3);
        CH(0, k, 1) = cadd(t1, t4);
        CH(0, k, 3) = csub(t1, t4);
      } else {
        CH(i, k, 0) = cadd(t2, t3);
        CH(i, k, 1) = smul(cadd(t1, t4), WA(0, i), fwd);
        CH(i, k, 2) = smul(csub(t2, t3), WA(1, i), fwd);
        CH(i, k, 3) = smul(csub(t1, t4), WA(2, i), fwd);
      }
    }
}

/* passes 5, 7 and 11: t0 = CC(0); pairs t[j] = CC(j) + CC(ip-j), d[j] =
 * CC(j) - CC(ip-j) (j = 1..h, h = (ip-1)/2); output u = 1..h:
 *   ca = t0 + c(u,1) t[1] + ... + c(u,h) t[h]   (left to right)
 *   cb = (-(s(u,1) d[1].i + ...), s(u,1) d[1].r + ...)
 *   CH(u) = ca + cb, CH(ip-u) = ca - cb (then the twiddles for i > 0)
 * c(u,j) = cos(2 pi (u j mod ip) / ip) and s(u,j) the matching sin with the
 * sign of the reduction (pocketfft's PARTSTEP tables, generated here). */
static void passodd(int ip, int64_t ido, int64_t l1, const cpx *cc, cpx *ch, const cpx *wa, int fwd)
{
  static const double c5[3] = {1.0, 0.3090169943749474241022934171828191, -0.8090169943749474241022934171828191};
  static const double s5[3] = {0.0, 0.9510565162951535721164393333793821, 0.5877852522924731291687059546390728};
  static const double c7[4] = {1.0, 0.6234898018587335305250048840042398, -0.2225209339563144042889025644967948,
                               -0.9009688679024191262361023195074451};
  static const double s7[4] = {0.0, 0.7818314824680298087084445266740578, 0.9749279121818236070181316829939312,
                               0.433883739117558120475768332848359};
  static const double c11[6] = {1.0, 0.8412535328311811688618116489193677, 0.4154150130018864255292741492296232,
                                -0.1423148382732851404437926686163697, -0.6548607339452850640569250724662936,
                                -0.9594929736144973898903680570663277};
  static const double s11[6] = {0.0, 0.5406408174555975821076359543186917, 0.9096319953545183714117153830790285,
                                0.9898214418809327323760920377767188, 0.7557495743542582837740358439723444,
                                0.2817325568414296977114179153466169};
  const double *cs = ip == 5 ? c5 : ip == 7 ? c7 : c11, *sn = ip == 5 ? s5 : ip == 7 ? s7 : s11;
  const int h = (ip - 1) / 2;
  const int64_t IPv = ip;
#undef CC
#define CC(a, b, c) cc[(a) + ido * ((b) + IPv * (c))]
  for (int64_t k = 0; k < l1; ++k)
    for (int64_t i = 0; i < ido; ++i) {
      cpx t[6], d[6];
      const cpx t0 = CC(i, 0, k);
      for (int j = 1; j <= h; ++j) {
        t[j] = cadd(CC(i, j, k), CC(i, ip - j, k));
        d[j] = csub(CC(i, j, k), CC(i, ip - j, k));
      }
      cpx s0 = t0;
      for (int j = 1; j <= h; ++j) { s0.r = s0.r + t[j].r; }
      for (int j = 1; j <= h; ++j) { s0.i = s0.i + t[j].i; }
      CH(i, k, 0) = s0;
      for (int u = 1; u <= h; ++u) {
        cpx ca = t0, cb;
        double cbr = 0.0, cbi = 0.0;
        for (int j = 1; j <= h; ++j) {
          int r = (int)(((int64_t)u * j) % ip);
          double sg = 1.0;
          if (r > h) { r = ip - r; sg = -1.0; }
          const double cr = cs[r], si = (fwd ? -1.0 : 1.0) * sn[r];
          ca.r = ca.r + cr * t[j].r;
          ca.i = ca.i + cr * t[j].i;
          /* y1*d.r y2*d.r ...: the first term as is, later ones +- |y| * d */
          if (j == 1) { cbi = si * d[j].r; cbr = si * d[j].i; }
          else if (sg > 0) { cbi = cbi + si * d[j].r; cbr = cbr + si * d[j].i; }
          else { cbi = cbi - si * d[j].r; cbr = cbr - si * d[j].i; }
        }
        cb.r = -cbr;
        cb.i = cbi;
        if (i == 0) {
          CH(0, k, u) = cadd(ca, cb);
          CH(0, k, ip - u) = csub(ca, cb);
        } else {
          CH(i, k, u) = smul(cadd(ca, cb), WA(u - 1, i), fwd);
          CH(i, k, ip - u) = smul(csub(ca, cb), WA(ip - u - 1, i), fwd);
        }
      }
    }
#undef CC
#define CC(a, b, c) cc[(a) + ido * ((b) + IP * (c))]
}

static inline cpx rot45(cpx a, int fwd)
{
  const double h = 0.707106781186547524400844362104849;
  cpx c;
  if (fwd) { c.r = h * (a.r + a.i); c.i = h * (a.i - a.r); }
  else { c.r = h * (a.r - a.i); c.i = h * (a.i + a.r); }
  return c;
}
static inline cpx rot135(cpx a, int fwd)
{
  const double h = 0.707106781186547524400844362104849;
  cpx c;
  if (fwd) { c.r = h * (a.i - a.r); c.i = h * (-a.r - a.i); }
  else { c.r = h * (-a.r - a.i); c.i = h * (a.r - a.i); }
  return c;
}

static void pass8(int64_t ido, int64_t l1, const cpx *cc, cpx *ch, const cpx *wa, int fwd)
{
  enum { IP = 8 };
  for (int64_t k = 0; k < l1; ++k)
    for (int64_t i = 0; i < ido; ++i) {
      cpx a1 = cadd(CC(i, 1, k), CC(i, 5, k)), a5 = csub(CC(i, 1, k), CC(i, 5, k));
      cpx a3 = cadd(CC(i, 3, k), CC(i, 7, k)), a7 = csub(CC(i, 3, k), CC(i, 7, k));
      cpx t = a1;
      a1 = cadd(t, a3);
      a3 = rot90(csub(t, a3), fwd);
      a7 = rot90(a7, fwd);
      t = a5;
      a5 = rot45(cadd(t, a7), fwd);
      a7 = rot135(csub(t, a7), fwd);
      cpx a0 = cadd(CC(i, 0, k), CC(i, 4, k)), a4 = csub(CC(i, 0, k), CC(i, 4, k));
      cpx a2 = cadd(CC(i, 2, k), CC(i, 6, k)), a6 = csub(CC(i, 2, k), CC(i, 6, k));
      if (i == 0) {
        const cpx s02 = cadd(a0, a2), d02 = csub(a0, a2);
        CH(0, k, 0) = cadd(s02, a1);
        CH(0, k, 4) = csub(s02, a1);
        CH(0, k, 2) = cadd(d02, a3);
        CH(0, k, 6) = csub(d02, a3);
        a6 = rot90(a6, fwd);
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
        CH(i, k, 4) = smul(csub(a0, a1), WA(3, i), fwd);
        CH(i, k, 2) = smul(cadd(a2, a3), WA(1, i), fwd);
        CH(i, k, 6) = smul(csub(a2, a3), WA(5, i), fwd);
        a6 = rot90(a6, fwd);
        t = a4;
        a4 = cadd(t, a6);
        a6 = csub(t, a6);
        CH(i, k, 1) = smul(cadd(a4, a5), WA(0, i), fwd);
        CH(i, k, 5) = smul(csub(a4, a5), WA(4, i), fwd);
        CH(i, k, 3) = smul(cadd(a6, a7), WA(2, i), fwd);
        CH(i, k, 7) = smul(csub(a6, a7), WA(6, i), fwd);
      }
    }
}
#undef CC
#undef CH
#undef WA

/* generic pass (p > 11): the result lands in cc (CX), not ch */
static void passg(int64_t ido, int64_t ip, int64_t l1, cpx *cc, cpx *ch, const cpx *wa, const cpx *csarr, int fwd)
{
  const int64_t cdim = ip, ipph = (ip + 1) / 2, idl1 = ido * l1;
#define CH(a, b, c) ch[(a) + ido * ((b) + l1 * (c))]
#define CC(a, b, c) cc[(a) + ido * ((b) + cdim * (c))]
#define CX(a, b, c) cc[(a) + ido * ((b) + l1 * (c))]
#define CX2(a, b) cc[(a) + idl1 * (b)]
#define CH2(a, b) ch[(a) + idl1 * (b)]
  cpx *wal = malloc(sizeof(cpx) * (size_t)ip);
  wal[0].r = 1.0; wal[0].i = 0.0;
  for (int64_t i = 1; i < ip; ++i) { wal[i].r = csarr[i].r; wal[i].i = fwd ? -csarr[i].i : csarr[i].i; }

  for (int64_t k = 0; k < l1; ++k)
    for (int64_t i = 0; i < ido; ++i) CH(i, k, 0) = CC(i, 0, k);
  for (int64_t j = 1, jc = ip - 1; j < ipph; ++j, --jc)
    for (int64_t k = 0; k < l1; ++k)
      for (int64_t i = 0; i < ido; ++i) {
        CH(i, k, j) = cadd(CC(i, j, k), CC(i, jc, k));
        CH(i, k, jc) = csub(CC(i, j, k), CC(i, jc, k));
      }
  for (int64_t k = 0; k < l1; ++k)
    for (int64_t i = 0; i < ido; ++i) {
      cpx tmp = CH(i, k, 0);
      for (int64_t j = 1; j < ipph; ++j) tmp = cadd(tmp, CH(i, k, j));
      CX(i, k, 0) = tmp;
    }
  for (int64_t l = 1, lc = ip - 1; l < ipph; ++l, --lc) {
    for (int64_t ik = 0; ik < idl1; ++ik) {
      CX2(ik, l).r = CH2(ik, 0).r + wal[l].r * CH2(ik, 1).r + wal[2 * l].r * CH2(ik, 2).r;
      CX2(ik, l).i = CH2(ik, 0).i + wal[l].r * CH2(ik, 1).i + wal[2 * l].r * CH2(ik, 2).i;
      CX2(ik, lc).r = -(wal[l].i * CH2(ik, ip - 1).i + wal[2 * l].i * CH2(ik, ip - 2).i);
      CX2(ik, lc).i = wal[l].i * CH2(ik, ip - 1).r + wal[2 * l].i * CH2(ik, ip - 2).r;
    }
    int64_t iwal = 2 * l;
    int64_t j = 3, jc = ip - 3;
    for (; j < ipph - 1; j += 2, jc -= 2) {
      iwal += l; if (iwal > ip) iwal -= ip;
      const cpx xwal = wal[iwal];
      iwal += l; if (iwal > ip) iwal -= ip;
      const cpx xwal2 = wal[iwal];
      for (int64_t ik = 0; ik < idl1; ++ik) {
        CX2(ik, l).r += CH2(ik, j).r * xwal.r + CH2(ik, j + 1).r * xwal2.r;
        CX2(ik, l).i += CH2(ik, j).i * xwal.r + CH2(ik, j + 1).i * xwal2.r;
        CX2(ik, lc).r -= CH2(ik, jc).i * xwal.i + CH2(ik, jc - 1).i * xwal2.i;
        CX2(ik, lc).i += CH2(ik, jc).r * xwal.i + CH2(ik, jc - 1).r * xwal2.i;
      }
    }
    for (; j < ipph; ++j, --jc) {
      iwal += l; if (iwal > ip) iwal -= ip;
      const cpx xwal = wal[iwal];
      for (int64_t ik = 0; ik < idl1; ++ik) {
        CX2(ik, l).r += CH2(ik, j).r * xwal.r;
        CX2(ik, l).i += CH2(ik, j).i * xwal.r;
        CX2(ik, lc).r -= CH2(ik, jc).i * xwal.i;
        CX2(ik, lc).i += CH2(ik, jc).r * xwal.i;
      }
    }
  }
  free(wal);
  /* shuffling and twiddling */
  if (ido == 1)
    for (int64_t j = 1, jc = ip - 1; j < ipph; ++j, --jc)
      for (int64_t ik = 0; ik < idl1; ++ik) {
        const cpx t1 = CX2(ik, j), t2 = CX2(ik, jc);
        CX2(ik, j) = cadd(t1, t2);
        CX2(ik, jc) = csub(t1, t2);
      }
  else
    for (int64_t j = 1, jc = ip - 1; j < ipph; ++j, --jc)
      for (int64_t k = 0; k < l1; ++k) {
        const cpx t1 = CX(0, k, j), t2 = CX(0, k, jc);
        CX(0, k, j) = cadd(t1, t2);
        CX(0, k, jc) = csub(t1, t2);
        for (int64_t i = 1; i < ido; ++i) {
          const cpx x1 = cadd(CX(i, k, j), CX(i, k, jc)), x2 = csub(CX(i, k, j), CX(i, k, jc));
          CX(i, k, j) = smul(x1, wa[(j - 1) * (ido - 1) + i - 1], fwd);
          CX(i, k, jc) = smul(x2, wa[(jc - 1) * (ido - 1) + i - 1], fwd);
        }
      }
#undef CH
#undef CC
#undef CX
#undef CX2
#undef CH2
}

/* c (len) in place: the transform, times fct (fct == 1: no multiply) */
static int cfftp_exec(const cfftp_t *p, cpx *c, double fct, int fwd)
{
  const int64_t len = p->len;
  if (len == 1) { c[0] = cscale(c[0], fct); return 0; }
  cpx *ch = malloc(sizeof(cpx) * (size_t)len);
  if (!ch) return -1;
  cpx *p1 = c, *p2 = ch;
  int64_t l1 = 1;
  for (int k = 0; k < p->nf; ++k) {
    const int64_t ip = p->fct[k], l2 = ip * l1, ido = len / l2;
    switch (ip) {
      case 4: pass4(ido, l1, p1, p2, p->tw[k], fwd); break;
      case 8: pass8(ido, l1, p1, p2, p->tw[k], fwd); break;
      case 2: pass2(ido, l1, p1, p2, p->tw[k], fwd); break;
      case 3: pass3(ido, l1, p1, p2, p->tw[k], fwd); break;
      case 5: case 7: case 11: passodd((int)ip, ido, l1, p1, p2, p->tw[k], fwd); break;
      default: {
        passg(ido, ip, l1, p1, p2, p->tw[k], p->tws[k], fwd);
        cpx *t = p1; p1 = p2; p2 = t;
      }
    }
    cpx *t = p1; p1 = p2; p2 = t;
    l1 = l2;
  }
  if (p1 != c) {
    if (fct != 1.0)
      for (int64_t i = 0; i < len; ++i) c[i] = cscale(ch[i], fct);
    else
      memcpy(c, p1, sizeof(cpx) * (size_t)len);
  } else if (fct != 1.0) {
    for (int64_t i = 0; i < len; ++i) c[i] = cscale(c[i], fct);
  }
  free(ch);
  return 0;
}

/* ========================= real plan (rfftp) =============================== */
typedef struct {
  int64_t len;
  int nf;
  int64_t fct[MAXF];
  double *tw[MAXF], *tws[MAXF];
  double *mem;
} rfftp_t;

static int rfftp_init(rfftp_t *p, int64_t len)
{
  memset(p, 0, sizeof(*p));
  p->len = len;
  if (len == 1) return 0;
  p->nf = factorize(len, 0, p->fct);
  int64_t twsz = 0, l1 = 1;
  for (int k = 0; k < p->nf; ++k) {
    const int64_t ip = p->fct[k], ido = len / (l1 * ip);
    twsz += (ip - 1) * (ido - 1);
    if (ip > 5) twsz += 2 * ip;
    l1 *= ip;
  }
  p->mem = calloc((size_t)(twsz + 1), sizeof(double));
  twid_t twid;
  if (!p->mem || twid_init(&twid, len)) { free(p->mem); p->mem = NULL; return -1; }
  double *ptr = p->mem;
  l1 = 1;
  for (int k = 0; k < p->nf; ++k) {
    const int64_t ip = p->fct[k], ido = len / (l1 * ip);
    if (k < p->nf - 1) {   /* the last factor needs no twiddles */
      p->tw[k] = ptr;
      ptr += (ip - 1) * (ido - 1);
      for (int64_t j = 1; j < ip; ++j)
        for (int64_t i = 1; i <= (ido - 1) / 2; ++i) {
          const cpx w = twid_get(&twid, j * l1 * i);
          p->tw[k][(j - 1) * (ido - 1) + 2 * i - 2] = w.r;
          p->tw[k][(j - 1) * (ido - 1) + 2 * i - 1] = w.i;
        }
    }
    if (ip > 5) {   /* extra factors of the generic passes */
      p->tws[k] = ptr;
      ptr += 2 * ip;
      p->tws[k][0] = 1.;
      p->tws[k][1] = 0.;
      for (int64_t i = 2, ic = 2 * ip - 2; i <= ic; i += 2, ic -= 2) {
        const cpx w = twid_get(&twid, i / 2 * (len / ip));
        p->tws[k][i] = w.r;
        p->tws[k][i + 1] = w.i;
        p->tws[k][ic] = w.r;
        p->tws[k][ic + 1] = -w.i;
      }
    }
    l1 *= ip;
  }
  twid_free(&twid);
  return 0;
}

static void rfftp_free(rfftp_t *p) { free(p->mem); p->mem = NULL; }

/* ---- forward passes (radfN) ---- */
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

/* generic forward pass: the result lands in cc, not ch */
static void radfg(int64_t ido, int64_t ip, int64_t l1, double *cc, double *ch, const double *wa, const double *csarr)
{
  const int64_t cdim = ip, ipph = (ip + 1) / 2, idl1 = ido * l1;
#define CC(a, b, c) cc[(a) + ido * ((b) + cdim * (c))]
#define CH(a, b, c) ch[(a) + ido * ((b) + l1 * (c))]
#define C1(a, b, c) cc[(a) + ido * ((b) + l1 * (c))]
#define C2(a, b) cc[(a) + idl1 * (b)]
#define CH2(a, b) ch[(a) + idl1 * (b)]
  if (ido > 1) {
    for (int64_t j = 1, jc = ip - 1; j < ipph; ++j, --jc) {
      const int64_t is = (j - 1) * (ido - 1), is2 = (jc - 1) * (ido - 1);
      for (int64_t k = 0; k < l1; ++k) {
        int64_t idij = is, idij2 = is2;
        for (int64_t i = 1; i <= ido - 2; i += 2) {
          const double t1 = C1(i, k, j), t2 = C1(i + 1, k, j), t3 = C1(i, k, jc), t4 = C1(i + 1, k, jc);
          const double x1 = wa[idij] * t1 + wa[idij + 1] * t2, x2 = wa[idij] * t2 - wa[idij + 1] * t1,
                       x3 = wa[idij2] * t3 + wa[idij2 + 1] * t4, x4 = wa[idij2] * t4 - wa[idij2 + 1] * t3;
          C1(i, k, j) = x3 + x1;
          C1(i + 1, k, jc) = x3 - x1;
          C1(i + 1, k, j) = x2 + x4;
          C1(i, k, jc) = x2 - x4;
          idij += 2;
          idij2 += 2;
        }
      }
    }
  }
  for (int64_t j = 1, jc = ip - 1; j < ipph; ++j, --jc)
    for (int64_t k = 0; k < l1; ++k) {
      const double t1 = C1(0, k, j), t2 = C1(0, k, jc);
      C1(0, k, j) = t2 + t1;
      C1(0, k, jc) = t2 - t1;
    }
  for (int64_t l = 1, lc = ip - 1; l < ipph; ++l, --lc) {
    for (int64_t ik = 0; ik < idl1; ++ik) {
      CH2(ik, l) = C2(ik, 0) + csarr[2 * l] * C2(ik, 1) + csarr[4 * l] * C2(ik, 2);
      CH2(ik, lc) = csarr[2 * l + 1] * C2(ik, ip - 1) + csarr[4 * l + 1] * C2(ik, ip - 2);
    }
    int64_t iang = 2 * l;
    int64_t j = 3, jc = ip - 3;
    for (; j < ipph - 3; j += 4, jc -= 4) {
      iang += l; if (iang > ip) iang -= ip;
      const double ar1 = csarr[2 * iang], ai1 = csarr[2 * iang + 1];
      iang += l; if (iang > ip) iang -= ip;
      const double ar2 = csarr[2 * iang], ai2 = csarr[2 * iang + 1];
      iang += l; if (iang > ip) iang -= ip;
      const double ar3 = csarr[2 * iang], ai3 = csarr[2 * iang + 1];
      iang += l; if (iang > ip) iang -= ip;
      const double ar4 = csarr[2 * iang], ai4 = csarr[2 * iang + 1];
      for (int64_t ik = 0; ik < idl1; ++ik) {
        CH2(ik, l) += ar1 * C2(ik, j) + ar2 * C2(ik, j + 1) + ar3 * C2(ik, j + 2) + ar4 * C2(ik, j + 3);
        CH2(ik, lc) += ai1 * C2(ik, jc) + ai2 * C2(ik, jc - 1) + ai3 * C2(ik, jc - 2) + ai4 * C2(ik, jc - 3);
      }
    }
    for (; j < ipph - 1; j += 2, jc -= 2) {
      iang += l; if (iang > ip) iang -= ip;
      const double ar1 = csarr[2 * iang], ai1 = csarr[2 * iang + 1];
      iang += l; if (iang > ip) iang -= ip;
      const double ar2 = csarr[2 * iang], ai2 = csarr[2 * iang + 1];
      for (int64_t ik = 0; ik < idl1; ++ik) {
        CH2(ik, l) += ar1 * C2(ik, j) + ar2 * C2(ik, j + 1);
        CH2(ik, lc) += ai1 * C2(ik, jc) + ai2 * C2(ik, jc - 1);
      }
    }
    for (; j < ipph; ++j, --jc) {
      iang += l; if (iang > ip) iang -= ip;
      const double ar = csarr[2 * iang], ai = csarr[2 * iang + 1];
      for (int64_t ik = 0; ik < idl1; ++ik) {
        CH2(ik, l) += ar * C2(ik, j);
        CH2(ik, lc) += ai * C2(ik, jc);
      }
    }
  }
  for (int64_t ik = 0; ik < idl1; ++ik) CH2(ik, 0) = C2(ik, 0);
  for (int64_t j = 1; j < ipph; ++j)
    for (int64_t ik = 0; ik < idl1; ++ik) CH2(ik, 0) += C2(ik, j);
  for (int64_t k = 0; k < l1; ++k)
    for (int64_t i = 0; i < ido; ++i) CC(i, 0, k) = CH(i, k, 0);
  for (int64_t j = 1, jc = ip - 1; j < ipph; ++j, --jc) {
    const int64_t j2 = 2 * j - 1;
    for (int64_t k = 0; k < l1; ++k) {
      CC(ido - 1, j2, k) = CH(0, k, j);
      CC(0, j2 + 1, k) = CH(0, k, jc);
    }
  }
  if (ido == 1) return;
  for (int64_t j = 1, jc = ip - 1; j < ipph; ++j, --jc) {
    const int64_t j2 = 2 * j - 1;
    for (int64_t k = 0; k < l1; ++k)
      for (int64_t i = 1, ic = ido - i - 2; i <= ido - 2; i += 2, ic -= 2) {
        CC(i, j2 + 1, k) = CH(i, k, j) + CH(i, k, jc);
        CC(ic, j2, k) = CH(i, k, j) - CH(i, k, jc);
        CC(i + 1, j2 + 1, k) = CH(i + 1, k, j) + CH(i + 1, k, jc);
        CC(ic + 1, j2, k) = CH(i + 1, k, jc) - CH(i + 1, k, j);
      }
  }
#undef CC
#undef CH
#undef C1
#undef C2
#undef CH2
}

/* ---- backward passes (radbN) ---- */
#define CC(a, b, c) cc[(a) + ido * ((b) + IP * (c))]
#define CH(a, b, c) ch[(a) + ido * ((b) + l1 * (c))]
#define WA(x, i) wa[(i) + (x) * (ido - 1)]

static void radb2(int64_t ido, int64_t l1, const double *cc, double *ch, const double *wa)
{
  enum { IP = 2 };
  for (int64_t k = 0; k < l1; k++) {
    CH(0, k, 0) = CC(0, 0, k) + CC(ido - 1, 1, k);
    CH(0, k, 1) = CC(0, 0, k) - CC(ido - 1, 1, k);
  }
  if ((ido & 1) == 0)
    for (int64_t k = 0; k < l1; k++) {
      CH(ido - 1, k, 0) = 2 * CC(ido - 1, 0, k);
      CH(ido - 1, k, 1) = -2 * CC(0, 1, k);
    }
  if (ido <= 2) return;
  for (int64_t k = 0; k < l1; ++k)
    for (int64_t i = 2; i < ido; i += 2) {
      const int64_t ic = ido - i;
      CH(i - 1, k, 0) = CC(i - 1, 0, k) + CC(ic - 1, 1, k);
      const double tr2 = CC(i - 1, 0, k) - CC(ic - 1, 1, k);
      const double ti2 = CC(i, 0, k) + CC(ic, 1, k);
      CH(i, k, 0) = CC(i, 0, k) - CC(ic, 1, k);
      CH(i, k, 1) = WA(0, i - 2) * ti2 + WA(0, i - 1) * tr2;
      CH(i - 1, k, 1) = WA(0, i - 2) * tr2 - WA(0, i - 1) * ti2;
    }
}

static void radb3(int64_t ido, int64_t l1, const double *cc, double *ch, const double *wa)
{
  enum { IP = 3 };
  const double taur = -0.5, taui = 0.8660254037844386467637231707529362;
  for (int64_t k = 0; k < l1; k++) {
    const double tr2 = 2 * CC(ido - 1, 1, k);
    const double cr2 = CC(0, 0, k) + taur * tr2;
    CH(0, k, 0) = CC(0, 0, k) + tr2;
    const double ci3 = 2 * taui * CC(0, 2, k);
    CH(0, k, 2) = cr2 + ci3;
    CH(0, k, 1) = cr2 - ci3;
  }
  if (ido == 1) return;
  for (int64_t k = 0; k < l1; k++)
    for (int64_t i = 2, ic = ido - 2; i < ido; i += 2, ic -= 2) {
      const double tr2 = CC(i - 1, 2, k) + CC(ic - 1, 1, k);
      const double ti2 = CC(i, 2, k) - CC(ic, 1, k);
      const double cr2 = CC(i - 1, 0, k) + taur * tr2;
      const double ci2 = CC(i, 0, k) + taur * ti2;
      CH(i - 1, k, 0) = CC(i - 1, 0, k) + tr2;
      CH(i, k, 0) = CC(i, 0, k) + ti2;
      const double cr3 = taui * (CC(i - 1, 2, k) - CC(ic - 1, 1, k));
      const double ci3 = taui * (CC(i, 2, k) + CC(ic, 1, k));
      const double dr3 = cr2 + ci3, dr2 = cr2 - ci3;
      const double di2 = ci2 + cr3, di3 = ci2 - cr3;
      CH(i, k, 1) = WA(0, i - 2) * di2 + WA(0, i - 1) * dr2;
      CH(i - 1, k, 1) = WA(0, i - 2) * dr2 - WA(0, i - 1) * di2;
      CH(i, k, 2) = WA(1, i - 2) * di3 + WA(1, i - 1) * dr3;
      CH(i - 1, k, 2) = WA(1, i - 2) * dr3 - WA(1, i - 1) * di3;
    }
}

static void radb4(int64_t ido, int64_t l1, const double *cc, double *ch, const double *wa)
{
  enum { IP = 4 };
  const double sqrt2 = 1.414213562373095048801688724209698;
  for (int64_t k = 0; k < l1; k++) {
    const double tr2 = CC(0, 0, k) + CC(ido - 1, 3, k), tr1 = CC(0, 0, k) - CC(ido - 1, 3, k);
    const double tr3 = 2 * CC(ido - 1, 1, k);
    const double tr4 = 2 * CC(0, 2, k);
    CH(0, k, 0) = tr2 + tr3;
    CH(0, k, 2) = tr2 - tr3;
    CH(0, k, 3) = tr1 + tr4;
    CH(0, k, 1) = tr1 - tr4;
  }
  if ((ido & 1) == 0)
    for (int64_t k = 0; k < l1; k++) {
      const double ti1 = CC(0, 3, k) + CC(0, 1, k), ti2 = CC(0, 3, k) - CC(0, 1, k);
      const double tr2 = CC(ido - 1, 0, k) + CC(ido - 1, 2, k), tr1 = CC(ido - 1, 0, k) - CC(ido - 1, 2, k);
      CH(ido - 1, k, 0) = tr2 + tr2;
      CH(ido - 1, k, 1) = sqrt2 * (tr1 - ti1);
      CH(ido - 1, k, 2) = ti2 + ti2;
      CH(ido - 1, k, 3) = -sqrt2 * (tr1 + ti1);
    }
  if (ido <= 2) return;
  for (int64_t k = 0; k < l1; ++k)
    for (int64_t i = 2; i < ido; i += 2) {
      const int64_t ic = ido - i;
      const double tr2 = CC(i - 1, 0, k) + CC(ic - 1, 3, k), tr1 = CC(i - 1, 0, k) - CC(ic - 1, 3, k);
      const double ti1 = CC(i, 0, k) + CC(ic, 3, k), ti2 = CC(i, 0, k) - CC(ic, 3, k);
      const double tr4 = CC(i, 2, k) + CC(ic, 1, k), ti3 = CC(i, 2, k) - CC(ic, 1, k);
      const double tr3 = CC(i - 1, 2, k) + CC(ic - 1, 1, k), ti4 = CC(i - 1, 2, k) - CC(ic - 1, 1, k);
      CH(i - 1, k, 0) = tr2 + tr3;
      const double cr3 = tr2 - tr3;
      CH(i, k, 0) = ti2 + ti3;
      const double ci3 = ti2 - ti3;
      const double cr4 = tr1 + tr4, cr2 = tr1 - tr4;
      const double ci2 = ti1 + ti4, ci4 = ti1 - ti4;
      CH(i, k, 1) = WA(0, i - 2) * ci2 + WA(0, i - 1) * cr2;
      CH(i - 1, k, 1) = WA(0, i - 2) * cr2 - WA(0, i - 1) * ci2;
      CH(i, k, 2) = WA(1, i - 2) * ci3 + WA(1, i - 1) * cr3;
      CH(i - 1, k, 2) = WA(1, i - 2) * cr3 - WA(1, i - 1) * ci3;
      CH(i, k, 3) = WA(2, i - 2) * ci4 + WA(2, i - 1) * cr4;
      CH(i - 1, k, 3) = WA(2, i - 2) * cr4 - WA(2, i - 1) * ci4;
    }
}

static void radb5(int64_t ido, int64_t l1, const double *cc, double *ch, const double *wa)
{
  enum { IP = 5 };
  const double tr11 = 0.3090169943749474241022934171828191, ti11 = 0.9510565162951535721164393333793821;
  const double tr12 = -0.8090169943749474241022934171828191, ti12 = 0.5877852522924731291687059546390728;
  for (int64_t k = 0; k < l1; k++) {
    const double ti5 = CC(0, 2, k) + CC(0, 2, k);
    const double ti4 = CC(0, 4, k) + CC(0, 4, k);
    const double tr2 = CC(ido - 1, 1, k) + CC(ido - 1, 1, k);
    const double tr3 = CC(ido - 1, 3, k) + CC(ido - 1, 3, k);
    CH(0, k, 0) = CC(0, 0, k) + tr2 + tr3;
    const double cr2 = CC(0, 0, k) + tr11 * tr2 + tr12 * tr3;
    const double cr3 = CC(0, 0, k) + tr12 * tr2 + tr11 * tr3;
    const double ci5 = ti5 * ti11 + ti4 * ti12, ci4 = ti5 * ti12 - ti4 * ti11;
    CH(0, k, 4) = cr2 + ci5;
    CH(0, k, 1) = cr2 - ci5;
    CH(0, k, 3) = cr3 + ci4;
    CH(0, k, 2) = cr3 - ci4;
  }
  if (ido == 1) return;
  for (int64_t k = 0; k < l1; ++k)
    for (int64_t i = 2, ic = ido - 2; i < ido; i += 2, ic -= 2) {
      const double tr2 = CC(i - 1, 2, k) + CC(ic - 1, 1, k), tr5 = CC(i - 1, 2, k) - CC(ic - 1, 1, k);
      const double ti5 = CC(i, 2, k) + CC(ic, 1, k), ti2 = CC(i, 2, k) - CC(ic, 1, k);
      const double tr3 = CC(i - 1, 4, k) + CC(ic - 1, 3, k), tr4 = CC(i - 1, 4, k) - CC(ic - 1, 3, k);
      const double ti4 = CC(i, 4, k) + CC(ic, 3, k), ti3 = CC(i, 4, k) - CC(ic, 3, k);
      CH(i - 1, k, 0) = CC(i - 1, 0, k) + tr2 + tr3;
      CH(i, k, 0) = CC(i, 0, k) + ti2 + ti3;
      const double cr2 = CC(i - 1, 0, k) + tr11 * tr2 + tr12 * tr3;
      const double ci2 = CC(i, 0, k) + tr11 * ti2 + tr12 * ti3;
      const double cr3 = CC(i - 1, 0, k) + tr12 * tr2 + tr11 * tr3;
      const double ci3 = CC(i, 0, k) + tr12 * ti2 + tr11 * ti3;
      const double cr5 = tr5 * ti11 + tr4 * ti12, cr4 = tr5 * ti12 - tr4 * ti11;
      const double ci5 = ti5 * ti11 + ti4 * ti12, ci4 = ti5 * ti12 - ti4 * ti11;
      const double dr4 = cr3 + ci4, dr3 = cr3 - ci4;
      const double di3 = ci3 + cr4, di4 = ci3 - cr4;
      const double dr5 = cr2 + ci5, dr2 = cr2 - ci5;
      const double di2 = ci2 + cr5, di5 = ci2 - cr5;
      CH(i, k, 1) = WA(0, i - 2) * di2 + WA(0, i - 1) * dr2;
      CH(i - 1, k, 1) = WA(0, i - 2) * dr2 - WA(0, i - 1) * di2;
      CH(i, k, 2) = WA(1, i - 2) * di3 + WA(1, i - 1) * dr3;
      CH(i - 1, k, 2) = WA(1, i - 2) * dr3 - WA(1, i - 1) * di3;
      CH(i, k, 3) = WA(2, i - 2) * di4 + WA(2, i - 1) * dr4;
      CH(i - 1, k, 3) = WA(2, i - 2) * dr4 - WA(2, i - 1) * di4;
      CH(i, k, 4) = WA(3, i - 2) * di5 + WA(3, i - 1) * dr5;
      CH(i - 1, k, 4) = WA(3, i - 2) * dr5 - WA(3, i - 1) * di5;
    }
}
#undef CC
#undef CH
#undef WA

/* generic backward pass: the result lands in ch */
static void radbg(int64_t ido, int64_t ip, int64_t l1, double *cc, double *ch, const double *wa, const double *csarr)
{
  const int64_t cdim = ip, ipph = (ip + 1) / 2, idl1 = ido * l1;
#define CC(a, b, c) cc[(a) + ido * ((b) + cdim * (c))]
#define CH(a, b, c) ch[(a) + ido * ((b) + l1 * (c))]
#define C1(a, b, c) cc[(a) + ido * ((b) + l1 * (c))]
#define C2(a, b) cc[(a) + idl1 * (b)]
#define CH2(a, b) ch[(a) + idl1 * (b)]
  for (int64_t k = 0; k < l1; ++k)
    for (int64_t i = 0; i < ido; ++i) CH(i, k, 0) = CC(i, 0, k);
  for (int64_t j = 1, jc = ip - 1; j < ipph; ++j, --jc) {
    const int64_t j2 = 2 * j - 1;
    for (int64_t k = 0; k < l1; ++k) {
      CH(0, k, j) = 2 * CC(ido - 1, j2, k);
      CH(0, k, jc) = 2 * CC(0, j2 + 1, k);
    }
  }
  if (ido != 1) {
    for (int64_t j = 1, jc = ip - 1; j < ipph; ++j, --jc) {
      const int64_t j2 = 2 * j - 1;
      for (int64_t k = 0; k < l1; ++k)
        for (int64_t i = 1, ic = ido - i - 2; i <= ido - 2; i += 2, ic -= 2) {
          CH(i, k, j) = CC(i, j2 + 1, k) + CC(ic, j2, k);
          CH(i, k, jc) = CC(i, j2 + 1, k) - CC(ic, j2, k);
          CH(i + 1, k, j) = CC(i + 1, j2 + 1, k) - CC(ic + 1, j2, k);
          CH(i + 1, k, jc) = CC(i + 1, j2 + 1, k) + CC(ic + 1, j2, k);
        }
    }
  }
  for (int64_t l = 1, lc = ip - 1; l < ipph; ++l, --lc) {
    for (int64_t ik = 0; ik < idl1; ++ik) {
      C2(ik, l) = CH2(ik, 0) + csarr[2 * l] * CH2(ik, 1) + csarr[4 * l] * CH2(ik, 2);
      C2(ik, lc) = csarr[2 * l + 1] * CH2(ik, ip - 1) + csarr[4 * l + 1] * CH2(ik, ip - 2);
    }
    int64_t iang = 2 * l;
    int64_t j = 3, jc = ip - 3;
    for (; j < ipph - 3; j += 4, jc -= 4) {
      iang += l; if (iang > ip) iang -= ip;
      const double ar1 = csarr[2 * iang], ai1 = csarr[2 * iang + 1];
      iang += l; if (iang > ip) iang -= ip;
      const double ar2 = csarr[2 * iang], ai2 = csarr[2 * iang + 1];
      iang += l; if (iang > ip) iang -= ip;
      const double ar3 = csarr[2 * iang], ai3 = csarr[2 * iang + 1];
      iang += l; if (iang > ip) iang -= ip;
      const double ar4 = csarr[2 * iang], ai4 = csarr[2 * iang + 1];
      for (int64_t ik = 0; ik < idl1; ++ik) {
        C2(ik, l) += ar1 * CH2(ik, j) + ar2 * CH2(ik, j + 1) + ar3 * CH2(ik, j + 2) + ar4 * CH2(ik, j + 3);
        C2(ik, lc) += ai1 * CH2(ik, jc) + ai2 * CH2(ik, jc - 1) + ai3 * CH2(ik, jc - 2) + ai4 * CH2(ik, jc - 3);
      }
    }
    for (; j < ipph - 1; j += 2, jc -= 2) {
      iang += l; if (iang > ip) iang -= ip;
      const double ar1 = csarr[2 * iang], ai1 = csarr[2 * iang + 1];
      iang += l; if (iang > ip) iang -= ip;
      const double ar2 = csarr[2 * iang], ai2 = csarr[2 * iang + 1];
      for (int64_t ik = 0; ik < idl1; ++ik) {
        C2(ik, l) += ar1 * CH2(ik, j) + ar2 * CH2(ik, j + 1);
        C2(ik, lc) += ai1 * CH2(ik, jc) + ai2 * CH2(ik, jc - 1);
      }
    }
    for (; j < ipph; ++j, --jc) {
      iang += l; if (iang > ip) iang -= ip;
      const double war = csarr[2 * iang], wai = csarr[2 * iang + 1];
      for (int64_t ik = 0; ik < idl1; ++ik) {
        C2(ik, l) += war * CH2(ik, j);
        C2(ik, lc) += wai * CH2(ik, jc);
      }
    }
  }
  for (int64_t j = 1; j < ipph; ++j)
    for (int64_t ik = 0; ik < idl1; ++ik) CH2(ik, 0) += CH2(ik, j);
  for (int64_t j = 1, jc = ip - 1; j < ipph; ++j, --jc)
    for (int64_t k = 0; k < l1; ++k) {
      CH(0, k, jc) = C1(0, k, j) + C1(0, k, jc);
      CH(0, k, j) = C1(0, k, j) - C1(0, k, jc);
    }
  if (ido == 1) return;
  for (int64_t j = 1, jc = ip - 1; j < ipph; ++j, --jc)
    for (int64_t k = 0; k < l1; ++k)
      for (int64_t i = 1; i <= ido - 2; i += 2) {
        CH(i, k, j) = C1(i, k, j) - C1(i + 1, k, jc);
        CH(i, k, jc) = C1(i, k, j) + C1(i + 1, k, jc);
        CH(i + 1, k, j) = C1(i + 1, k, j) + C1(i, k, jc);
        CH(i + 1, k, jc) = C1(i + 1, k, j) - C1(i, k, jc);
      }
  for (int64_t j = 1; j < ip; ++j) {
    const int64_t is = (j - 1) * (ido - 1);
    for (int64_t k = 0; k < l1; ++k) {
      int64_t idij = is;
      for (int64_t i = 1; i <= ido - 2; i += 2) {
        const double t1 = CH(i, k, j), t2 = CH(i + 1, k, j);
        CH(i, k, j) = wa[idij] * t1 - wa[idij + 1] * t2;
        CH(i + 1, k, j) = wa[idij] * t2 + wa[idij + 1] * t1;
        idij += 2;
      }
    }
  }
#undef CC
#undef CH
#undef C1
#undef C2
#undef CH2
}

static void copy_and_norm(double *c, double *p1, int64_t n, double fct)
{
  if (p1 != c) {
    if (fct != 1.)
      for (int64_t i = 0; i < n; ++i) c[i] = fct * p1[i];
    else
      memcpy(c, p1, sizeof(double) * (size_t)n);
  } else if (fct != 1.) {
    for (int64_t i = 0; i < n; ++i) c[i] *= fct;
  }
}

/* c (len) in place; r2hc: forward (halfcomplex out), else backward (halfcomplex in) */
static int rfftp_exec(const rfftp_t *p, double *c, double fct, int r2hc)
{
  const int64_t n = p->len;
  if (n == 1) { c[0] *= fct; return 0; }
  double *ch = malloc(sizeof(double) * (size_t)n);
  if (!ch) return -1;
  double *p1 = c, *p2 = ch;
  if (r2hc) {
    int64_t l1 = n;
    for (int k1 = 0; k1 < p->nf; ++k1) {
      const int k = p->nf - k1 - 1;
      const int64_t ip = p->fct[k], ido = n / l1;
      l1 /= ip;
      switch (ip) {
        case 4: radf4(ido, l1, p1, p2, p->tw[k]); break;
        case 2: radf2(ido, l1, p1, p2, p->tw[k]); break;
        case 3: radf3(ido, l1, p1, p2, p->tw[k]); break;
        case 5: radf5(ido, l1, p1, p2, p->tw[k]); break;
        default: {
          radfg(ido, ip, l1, p1, p2, p->tw[k], p->tws[k]);
          double *t = p1; p1 = p2; p2 = t;
        }
      }
      double *t = p1; p1 = p2; p2 = t;
    }
  } else {
    int64_t l1 = 1;
    for (int k = 0; k < p->nf; ++k) {
      const int64_t ip = p->fct[k], ido = n / (ip * l1);
      switch (ip) {
        case 4: radb4(ido, l1, p1, p2, p->tw[k]); break;
        case 2: radb2(ido, l1, p1, p2, p->tw[k]); break;
        case 3: radb3(ido, l1, p1, p2, p->tw[k]); break;
        case 5: radb5(ido, l1, p1, p2, p->tw[k]); break;
        default: radbg(ido, ip, l1, p1, p2, p->tw[k], p->tws[k]); break;
      }
      double *t = p1; p1 = p2; p2 = t;
      l1 *= ip;
    }
  }
  copy_and_norm(c, p1, n, fct);
  free(ch);
  return 0;
}

/* ============================ Bluestein ==================================== */
typedef struct {
  int64_t n, n2;
  cfftp_t plan;
  cpx *bk, *bkf;   /* bk: n, bkf: n2 / 2 + 1 */
} blue_t;

static int blue_init(blue_t *b, int64_t n)
{
  memset(b, 0, sizeof(*b));
  b->n = n;
  b->n2 = good_size_cmplx(n * 2 - 1);
  if (cfftp_init(&b->plan, b->n2)) return -1;
  b->bk = malloc(sizeof(cpx) * (size_t)n);
  b->bkf = malloc(sizeof(cpx) * (size_t)(b->n2 / 2 + 1));
  cpx *tbkf = malloc(sizeof(cpx) * (size_t)b->n2);
  twid_t tmp;
  if (!b->bk || !b->bkf || !tbkf || twid_init(&tmp, 2 * n)) { free(tbkf); return -1; }
  /* b_k */
  b->bk[0].r = 1; b->bk[0].i = 0;
  int64_t coeff = 0;
  for (int64_t m = 1; m < n; ++m) {
    coeff += 2 * m - 1;
    if (coeff >= 2 * n) coeff -= 2 * n;
    b->bk[m] = twid_get(&tmp, coeff);
  }
  twid_free(&tmp);
  /* the zero-padded, Fourier transformed b_k, with normalisation */
  const double xn2 = 1.0 / (double)b->n2;
  tbkf[0] = cscale(b->bk[0], xn2);
  for (int64_t m = 1; m < n; ++m) tbkf[m] = tbkf[b->n2 - m] = cscale(b->bk[m], xn2);
  for (int64_t m = n; m <= b->n2 - n; ++m) { tbkf[m].r = 0.; tbkf[m].i = 0.; }
  if (cfftp_exec(&b->plan, tbkf, 1., 1)) { free(tbkf); return -1; }
  for (int64_t i = 0; i < b->n2 / 2 + 1; ++i) b->bkf[i] = tbkf[i];
  free(tbkf);
  return 0;
}

static void blue_free(blue_t *b) { cfftp_free(&b->plan); free(b->bk); free(b->bkf); b->bk = b->bkf = NULL; }

static int blue_fft(const blue_t *b, cpx *c, double fct, int fwd)
{
  const int64_t n = b->n, n2 = b->n2;
  cpx *akf = malloc(sizeof(cpx) * (size_t)n2);
  if (!akf) return -1;
  for (int64_t m = 0; m < n; ++m) akf[m] = smul(c[m], b->bk[m], fwd);
  const cpx zero = cscale(akf[0], 0.);
  for (int64_t m = n; m < n2; ++m) akf[m] = zero;
  if (cfftp_exec(&b->plan, akf, 1., 1)) { free(akf); return -1; }
  /* the convolution */
  akf[0] = smul(akf[0], b->bkf[0], !fwd);
  for (int64_t m = 1; m < (n2 + 1) / 2; ++m) {
    akf[m] = smul(akf[m], b->bkf[m], !fwd);
    akf[n2 - m] = smul(akf[n2 - m], b->bkf[m], !fwd);
  }
  if ((n2 & 1) == 0) akf[n2 / 2] = smul(akf[n2 / 2], b->bkf[n2 / 2], !fwd);
  if (cfftp_exec(&b->plan, akf, 1., 0)) { free(akf); return -1; }
  for (int64_t m = 0; m < n; ++m) c[m] = cscale(smul(akf[m], b->bk[m], fwd), fct);
  free(akf);
  return 0;
}

/* exec_r: real data through the complex Bluestein transform */
static int blue_exec_r(const blue_t *b, double *c, double fct, int fwd)
{
  const int64_t n = b->n;
  cpx *tmp = malloc(sizeof(cpx) * (size_t)n);
  if (!tmp) return -1;
  int rc;
  if (fwd) {
    const double zero = 0. * c[0];
    for (int64_t m = 0; m < n; ++m) { tmp[m].r = c[m]; tmp[m].i = zero; }
    rc = blue_fft(b, tmp, fct, 1);
    c[0] = tmp[0].r;
    for (int64_t m = 1; m < n; ++m) c[m] = (m & 1) ? tmp[(m + 1) / 2].r : tmp[m / 2].i;
  } else {
    tmp[0].r = c[0];
    tmp[0].i = c[0] * 0.;
    for (int64_t m = 1; m < n; ++m) {
      if (m & 1) tmp[(m + 1) / 2].r = c[m];
      else tmp[m / 2].i = c[m];
    }
    if ((n & 1) == 0) tmp[n / 2].i = 0. * c[0];
    for (int64_t m = 1; 2 * m < n; ++m) { tmp[n - m].r = tmp[m].r; tmp[n - m].i = -tmp[m].i; }
    rc = blue_fft(b, tmp, fct, 0);
    for (int64_t m = 0; m < n; ++m) c[m] = tmp[m].r;
  }
  free(tmp);
  return rc;
}

/* ====================== pocketfft_c / pocketfft_r =========================== */
typedef struct { int blue; cfftp_t pack; blue_t bl; } pfc_t;
typedef struct { int blue; rfftp_t pack; blue_t bl; } pfr_t;

static int pfc_init(pfc_t *p, int64_t n)
{
  p->blue = use_bluestein(n, 0);
  return p->blue ? blue_init(&p->bl, n) : cfftp_init(&p->pack, n);
}
static void pfc_free(pfc_t *p) { if (p->blue) blue_free(&p->bl); else cfftp_free(&p->pack); }
static int pfc_exec(const pfc_t *p, cpx *c, double fct, int fwd)
{
  return p->blue ? blue_fft(&p->bl, c, fct, fwd) : cfftp_exec(&p->pack, c, fct, fwd);
}
static int pfr_init(pfr_t *p, int64_t n)
{
  p->blue = use_bluestein(n, 1);
  return p->blue ? blue_init(&p->bl, n) : rfftp_init(&p->pack, n);
}
static void pfr_free(pfr_t *p) { if (p->blue) blue_free(&p->bl); else rfftp_free(&p->pack); }
static int pfr_exec(const pfr_t *p, double *c, double fct, int r2hc)
{
  return p->blue ? blue_exec_r(&p->bl, c, fct, r2hc) : rfftp_exec(&p->pack, c, fct, r2hc);
}

/* ============================ entry points ================================== */

/* plan kinds for the tests: 1 Bluestein, 0 FFTPACK-style */
int oracle_pf_uses_bluestein(int64_t n, int real) { return n >= 1 ? use_bluestein(n, real) : -1; }
int64_t oracle_pf_good_size(int64_t n) { return good_size_cmplx(n); }

/* scipy.fft.rfft(x): n reals -> n / 2 + 1 complex (interleaved) */
int oracle_pf_rfft(const double *x, int64_t n, double *out)
{
  if (n < 1) return -1;
  pfr_t p;
  double *t = malloc(sizeof(double) * (size_t)n);
  if (!t || pfr_init(&p, n)) { free(t); return -1; }
  memcpy(t, x, sizeof(double) * (size_t)n);
  int rc = pfr_exec(&p, t, 1., 1);
  out[0] = t[0]; out[1] = 0.;
  int64_t i = 1, ii = 1;
  for (; i < n - 1; i += 2, ++ii) { out[2 * ii] = t[i]; out[2 * ii + 1] = t[i + 1]; }
  if (i < n) { out[2 * ii] = t[i]; out[2 * ii + 1] = 0.; }
  pfr_free(&p);
  free(t);
  return rc;
}

/* scipy.fft.irfft(X, n): n / 2 + 1 complex (interleaved) -> n reals, times 1 / n */
int oracle_pf_irfft(const double *X, int64_t n, double *y)
{
  if (n < 1) return -1;
  pfr_t p;
  if (pfr_init(&p, n)) return -1;
  y[0] = X[0];
  int64_t i = 1, ii = 1;
  for (; i < n - 1; i += 2, ++ii) { y[i] = X[2 * ii]; y[i + 1] = X[2 * ii + 1]; }
  if (i < n) y[i] = X[2 * ii];
  const int rc = pfr_exec(&p, y, (double)(1.0L / (long double)n), 0);
  pfr_free(&p);
  return rc;
}

/* scipy.fft.fft / ifft of complex input (interleaved, in place); ifft scales by 1 / n */
int oracle_pf_cfft(double *c, int64_t n, int inverse)
{
  if (n < 1) return -1;
  pfc_t p;
  if (pfc_init(&p, n)) return -1;
  const int rc = pfc_exec(&p, (cpx *)c, inverse ? (double)(1.0L / (long double)n) : 1., !inverse);
  pfc_free(&p);
  return rc;
}

/* |scipy.signal.hilbert(x)| (x real, length n), into env */
int oracle_hilbert_env(const double *x, int64_t n, double *env)
{
  if (n < 1) return -1;
  cpx *X = malloc(sizeof(cpx) * (size_t)n);
  double *hc = malloc(sizeof(double) * (size_t)(2 * (n / 2 + 1)));
  if (!X || !hc) { free(X); free(hc); return -1; }
  int rc = oracle_pf_rfft(x, n, hc);
  if (rc == 0) {
    /* pypocketfft c2c_sym: bins 0..n/2 from r2c, each conjugated into n - i
       (bins 0 and n/2 onto themselves: their imaginary parts become -0.0) */
    for (int64_t i = 0; i <= n / 2; ++i) { X[i].r = hc[2 * i]; X[i].i = hc[2 * i + 1]; }
    for (int64_t i = 0; i <= n / 2; ++i) {
      const cpx v = X[i];
      X[(n - i) % n].r = v.r;
      X[(n - i) % n].i = -v.i;
    }
    for (int64_t i = 0; i < n; ++i) {
      /* scipy.signal.hilbert's h: 1 at 0 (and n/2), 2 below n/2, 0 above */
      const double hr = (i == 0 || 2 * i == n) ? 1.0 : (2 * i < n ? 2.0 : 0.0), hi = 0.0;
      const double xr = X[i].r, xi = X[i].i;
      X[i].r = fma(xr, hr, -(xi * hi));
      X[i].i = fma(xr, hi, xi * hr);
    }
    rc = oracle_pf_cfft((double *)X, n, 1);
  }
  if (rc == 0)
    for (int64_t i = 0; i < n; ++i) {
      /* np.abs(complex128), numpy's AVX-512 kernel */
      const double ar = fabs(X[i].r), ai = fabs(X[i].i);
      const double hi = ar > ai ? ar : ai, lo = ar > ai ? ai : ar;
      env[i] = hi == 0.0 ? 0.0 : hi * sqrt(fma(lo / hi, lo / hi, 1.0));
    }
  free(X);
  free(hc);
  return rc;
}

/* scipy.signal.resample(x, num) for a real 1-D x of length nx (no window,
 * time domain; decoder.py:385-387): rfft, spectrum copy with the Nyquist bin
 * doubled (down) or halved (up) for an even min(num, nx), irfft(., num),
 * times float(num) / float(nx) */
int oracle_resample(const double *x, int64_t nx, int64_t num, double *y)
{
  if (nx < 1 || num < 1) return -1;
  double *X = malloc(sizeof(double) * (size_t)(2 * (nx / 2 + 1)));
  double *Y = calloc((size_t)(2 * (num / 2 + 1)), sizeof(double));
  if (!X || !Y) { free(X); free(Y); return -1; }
  int rc = oracle_pf_rfft(x, nx, X);
  if (rc == 0) {
    const int64_t N = num < nx ? num : nx, nyq = N / 2 + 1;
    memcpy(Y, X, sizeof(double) * (size_t)(2 * nyq));
    if (N % 2 == 0) {
      /* numpy's complex multiply by (s + 0j): fma(r, s, -(i*0)), fma(r, 0, i*s) */
      double s = 0.0;
      if (num < nx) s = 2.0;
      else if (nx < num) s = 0.5;
      if (s != 0.0) {
        const double r = Y[2 * (N / 2)], im = Y[2 * (N / 2) + 1];
        Y[2 * (N / 2)] = fma(r, s, -(im * 0.0));
        Y[2 * (N / 2) + 1] = fma(r, 0.0, im * s);
      }
    }
    rc = oracle_pf_irfft(Y, num, y);
    if (rc == 0) {
      const double f = (double)num / (double)nx;
      for (int64_t i = 0; i < num; ++i) y[i] *= f;
    }
  }
  free(X);
  free(Y);
  return rc;
}

/* numpy's complex abs and multiply as modelled above, for the host probe
 * (oracle.numpy_complex_is_modelled): abs_out[i] = |z[i]|, mul_out[i] = z[i] * w[i] */
void oracle_np_complex_model(const double *z, const double *w, int64_t n, double *abs_out, double *mul_out)
{
  for (int64_t i = 0; i < n; ++i) {
    const double zr = z[2 * i], zi = z[2 * i + 1], wr = w[2 * i], wi = w[2 * i + 1];
    const double ar = fabs(zr), ai = fabs(zi);
    const double hi = ar > ai ? ar : ai, lo = ar > ai ? ai : ar;
    abs_out[i] = hi == 0.0 ? 0.0 : hi * sqrt(fma(lo / hi, lo / hi, 1.0));
    mul_out[2 * i] = fma(zr, wr, -(zi * wi));
    mul_out[2 * i + 1] = fma(zr, wi, zi * wr);
  }
}
