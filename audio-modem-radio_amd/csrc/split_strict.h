// split_strict.h -- host design of the PSK time-split layout's STRICT error
// bound (DESIGN.md §3.3 "Strict mode"; psk_split_kernels.hip KS0-KS5 with
// PskSplit::strict).
//
// The default split layout keeps a decision when it clears E = kappa * peak|x|,
// kappa = 64.25 u (g1_bp + g1_lp): a MEASURED premise (the worst error seen
// over the test signal classes is >= 54x below it).  The strict mode replaces
// E by a bound that holds for every input, per stream and per symbol, from
// quantities the kernels measure on the stream itself:
//
//   * every DF-II-T step of scipy's order (y = z0 + b0 x; z_j = (z_{j+1} +
//     x b_{j+1}) - y a_{j+1}) commits, per state, at most u(|p| + |q| + |r| +
//     |z'|) of rounding (each IEEE operation errs by <= u |result|); with
//     |q| <= (1+u)(|z| + |p|), |z'| <= (1+u)(|q| + |r|) and the output's
//     u(|b0 x| + |y|) fed into every state through a, the step's injected
//     error summed over states is at most
//        D = U (2 sum_{i>=1} |z_i| + kx |x| + ky |y|),  U = u (1+u)^4,
//        kx = 3 sum_{j>=1} |b_j| + |b0| sum_{j>=1} |a_j|,  ky = 3 sum_{j>=1} |a_j|
//     (evaluated per step on the pre-step states; the zero-tap and
//     palindromic forms only drop exact zeros);
//   * an error d injected into state j reaches the output m steps later as
//     g_j(m) d (the zero-input response), so a pass's output differs from the
//     exact-arithmetic pass on the same input by at most g1x * max D, g1x =
//     1 + sum_m max_j |g_j(m)| (the 1: the output's own rounding);
//   * both the split and the serial (reference) pass commit such rounding;
//     the serial's magnitudes differ from the split's by at most the bound
//     itself, which a cap (2^-10 of the pass's input peak, checked at the end;
//     a stream over it is flagged) makes a second-order term;
//   * a chunk's start state (KS0: sum_m K[m] v(o0 - 1 - m) by FMA chains and
//     a 64-lane butterfly) differs from the exact state by at most
//     gamma_{ceil(w/64) + 7} sum |K||v| (+ the tables' rounding, + the
//     truncated terms m >= w: tk * peak), reaching the chunk's outputs with at
//     most max_{m < L} max_j |g_j(m)|;
//   * the band-pass backward pass passes its input error with at most
//     ||h||_1 + max |tz| (tz: the zero-input output from scipy's zi, whose
//     start zi * y1[-1] carries the last input's error);
//   * the mixer, the low-pass odd extension (x3 at its samples) and the two
//     low-pass passes pass the band-pass error X per symbol with a per-plan
//     table lpc[k] (the exact sum over the low-pass's |h| and |tz| at that
//     symbol's position, edges included); the low-pass's own rounding, its
//     warm-up truncation and the extension's rounding are per-plan constants
//     times the low-pass input's peak.
//
// Everything here is host arithmetic in long double (responses to decay below
// 1e-40 of their peak; every table rounded up).
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "amr_internal.h"

namespace amr {

// block bound (KB, psk_split_kernels.hip): the per-step bounds D summed over
// blocks of kStrictBlk outputs, convolved at block resolution with window
// maxima of the responses (exact within the block: 1.3x of the per-sample
// convolution, against 5x for the stream's max D), the responses cut where
// their remaining mass is below kStrictCut of the total and that remainder
// charged at the stream's max D
constexpr double kStrictCut = 1e-4;   // (kStrictBlk: amr_internal.h)

struct StrictDesign {
  bool ok = false;
  // block kernels (band-pass): W [nw] output block J <- D block J - d (the pass's own rounding),
  // K12 [nk] forward block J <- pass-1 D block J + d - k12_off (pass-1 rounding through pass 2),
  // HS [nh] forward block J <- S1 block J + d (the start errors through pass 2),
  // GS [ng] a chunk's block q <- its start error, TZ [nz] pass-2 block q <- E1 at the last sample
  std::vector<double> W, K12, HS, GS, TZ;
  int k12_off = 0;
  double w_tail = 0, k12_tail = 0, hs_tail = 0, tz_tail = 0;   // the cut remainders (x max D, x max S, x E1 last)
  // low-pass window: symbol k's bound uses X over samples within lp_rad of it (plus the first and
  // last blocks, the extension's sources); the rest at most lp_tail x max X
  int64_t lp_rad = 0;
  double lp_tail = 0;
  // band-pass
  double g1x = 0, gmax = 0, hz = 0, tk = 0, zi_sum = 0, kx = 0, ky = 0, zb = 0, gam = 0;
  std::vector<double> gm_pmax;   // [m] max_{m' <= m} max_j |g_j(m')| (the chunk's start error reach)
  std::vector<double> kabs;      // [w1] sum_i |K_i[m]| of the KS0 tables as rounded
  std::vector<double> z0abs;     // [w1 + 1] sum_i |Z0_i[t]|
  // low-pass
  std::vector<double> lpc;       // [n_sym] the band-pass error's reach to symbol k
  double c3 = 0;                 // x the low-pass input peak P3: own rounding, warm-up truncation, extension rounding
  double lp_kx = 0, lp_ky = 0;
};

namespace strict_detail {
typedef long double LD;
constexpr LD kU = 1.0L / 9007199254740992.0L;   // 2^-53
inline LD up(LD v) { return v * (1.0L + 1e-12L); }

// zero-input responses of a DF-II-T (a[0] = 1): out[m] = max_j |g_j(m)| (the
// output m steps after a unit error in state j), tz[m] = the output from the
// start state zi; state magnitude sums for state errors and input
struct Responses {
  std::vector<LD> gm, tz, h;
  LD zb = 0;        // sum_i (sum_m |state_i after a unit input, m steps| + sup_t |state_i from zi|)
  bool ok = false;
};
inline Responses responses(const Iir& f, int64_t max_steps = 8000000) {
  Responses r;
  const int N = f.nt - 1;
  std::vector<LD> a(f.nt), b(f.nt);
  for (int i = 0; i < f.nt; ++i) { a[i] = f.a[i]; b[i] = f.b[i]; }
  // N unit-state responses + the zi response + the input response, together
  std::vector<LD> zs((size_t)(N + 2) * N, 0.0L);
  for (int i = 0; i < N; ++i) zs[(size_t)i * N + i] = 1.0L;
  for (int i = 0; i < N; ++i) zs[(size_t)N * N + i] = f.zi[i];
  std::vector<LD> ksum(N, 0.0L), zisup(N, 0.0L);
  LD peak = 1.0L;
  bool decayed = false;
  for (int64_t m = 0; m < max_steps && !decayed; ++m) {
    LD g = 0.0L, live = 0.0L;
    for (int v = 0; v < N + 2; ++v) {
      LD* z = &zs[(size_t)v * N];
      const LD x = (v == N + 1 && m == 0) ? 1.0L : 0.0L;   // the input response: a unit sample at m = 0
      const LD y = z[0] + b[0] * x;
      if (v < N) g = std::max(g, std::fabs(y));
      else if (v == N) r.tz.push_back(y);
      else r.h.push_back(y);
      for (int j = 0; j < N - 1; ++j) z[j] = z[j + 1] + b[j + 1] * x - a[j + 1] * y;
      z[N - 1] = b[N] * x - a[N] * y;
      for (int j = 0; j < N; ++j) {
        live = std::max(live, std::fabs(z[j]));
        if (v == N + 1) ksum[j] += std::fabs(z[j]);
        if (v == N) zisup[j] = std::max(zisup[j], std::fabs(z[j]));
      }
    }
    r.gm.push_back(g);
    peak = std::max(peak, live);
    decayed = m > 8 * N && live < 1e-40L * peak;
  }
  if (!decayed) return r;
  for (int j = 0; j < N; ++j) r.zb += ksum[j] + std::max(zisup[j], std::fabs((LD)f.zi[j]));
  r.ok = std::isfinite((double)r.zb);
  return r;
}
inline LD sum_abs(const std::vector<LD>& v) {
  LD s = 0.0L;
  for (LD x : v) s += std::fabs(x);
  return s;
}
inline LD max_abs(const std::vector<LD>& v) {
  LD s = 0.0L;
  for (LD x : v) s = std::max(s, std::fabs(x));
  return s;
}
}  // namespace strict_detail

// The band-pass half of the design (both filtfilt passes of one filter; the
// FSK split's strict mode uses it per tone): bp the filter, K [w1][N], Z0
// [w1 + 1][N] the convolution-start tables as the device holds them.  Fills
// the band-pass fields and block kernels of d; false when a response does not
// decay.
inline bool strict_design_bp(const Iir& bp, const double* K, const double* Z0, int64_t w1, StrictDesign& d,
                             const strict_detail::Responses& rb) {
  using namespace strict_detail;
  if (!rb.ok || w1 < 1) return false;
  const int N = bp.nt - 1;
  const LD U = kU * std::pow(1.0L + kU, 4);
  LD g1x = 1.0L, gmax = 0.0L;
  d.gm_pmax.resize(rb.gm.size());
  for (size_t m = 0; m < rb.gm.size(); ++m) {
    g1x += rb.gm[m];
    gmax = std::max(gmax, rb.gm[m]);
    d.gm_pmax[m] = (double)up(gmax);
  }
  d.g1x = (double)up(g1x * (1.0L + 1e-30L));
  d.gmax = (double)up(gmax);
  d.hz = (double)up(sum_abs(rb.h) + max_abs(rb.tz));
  LD ca = 0.0L, cb = 0.0L, zis = 0.0L;
  for (int j = 1; j <= N; ++j) { ca += std::fabs((LD)bp.a[j]); cb += std::fabs((LD)bp.b[j]); }
  for (int j = 0; j < N; ++j) zis += std::fabs((LD)bp.zi[j]);
  d.kx = (double)up(U * (3.0L * cb + std::fabs((LD)bp.b[0]) * ca));
  d.ky = (double)up(U * 3.0L * ca);
  d.zi_sum = (double)up(zis);
  d.zb = (double)up(rb.zb);
  // KS0's truncation: the state response to inputs m >= w1 back and the zi
  // start decayed past w1, per unit input peak (long double, to decay)
  {
    std::vector<LD> z(N), zz(N);
    for (int i = 0; i < N; ++i) { z[i] = (LD)bp.b[i + 1] - (LD)bp.a[i + 1] * (LD)bp.b[0]; zz[i] = bp.zi[i]; }
    LD tk = 0.0L, z0sup = 0.0L, live = 1.0L, pk = 1.0L;
    for (int64_t m = 0; m < 8000000 && (m <= w1 || live > 1e-40L * pk); ++m) {
      live = 0.0L;
      if (m >= w1)
        for (int i = 0; i < N; ++i) tk += std::fabs(z[i]);
      if (m > w1) {
        LD s = 0.0L;
        for (int i = 0; i < N; ++i) s += std::fabs(zz[i]);
        z0sup = std::max(z0sup, s);
      }
      for (auto* v : {&z, &zz}) {
        const LD y = (*v)[0];
        for (int i = 0; i < N - 1; ++i) (*v)[i] = (*v)[i + 1] - (LD)bp.a[i + 1] * y;
        (*v)[N - 1] = -(LD)bp.a[N] * y;
        for (int i = 0; i < N; ++i) {
          live = std::max(live, std::fabs((*v)[i]));
          pk = std::max(pk, std::fabs((*v)[i]));
        }
      }
    }
    d.tk = (double)up(tk + z0sup + 1e-30L);
  }
  // KS0's dot product: chains of ceil(w1 / 64) FMAs, a 6-level butterfly and
  // the Z0 FMA -> gamma_{n}; plus the tables' own rounding (once, from long
  // double: u |K|, and the long double recursion's, far below another u)
  {
    const LD nn = (LD)((w1 + 63) / 64 + 7);
    const LD gam = nn * kU / (1.0L - nn * kU);
    d.gam = (double)up(gam + 2.0L * kU);
  }
  d.kabs.resize((size_t)w1);
  d.z0abs.resize((size_t)w1 + 1);
  for (int64_t m = 0; m < w1; ++m) {
    LD s = 0.0L;
    for (int i = 0; i < N; ++i) s += std::fabs((LD)K[m * N + i]);
    d.kabs[(size_t)m] = (double)up(s);
  }
  for (int64_t t = 0; t <= w1; ++t) {
    LD s = 0.0L;
    for (int i = 0; i < N; ++i) s += std::fabs((LD)Z0[t * N + i]);
    d.z0abs[(size_t)t] = (double)up(s);
  }
  // ---- block kernels (long double, rounded up)
  {
    const int BS = kStrictBlk;
    // Gx(m) = Gm(m), Gx(-1) = 1; cut at Mg where sum_{m >= Mg} Gm < kStrictCut g1x
    LD gtot = 1.0L;
    for (LD g : rb.gm) gtot += g;
    int64_t Mg = (int64_t)rb.gm.size();
    {
      LD rem = 0.0L;
      for (int64_t m = (int64_t)rb.gm.size() - 1; m >= 0; --m) {
        if (rem + rb.gm[(size_t)m] > (LD)kStrictCut * gtot) break;
        rem += rb.gm[(size_t)m];
        Mg = m;
      }
      d.w_tail = (double)up(rem);
    }
    auto Gx = [&](int64_t m) -> LD { return m == -1 ? 1.0L : (m >= 0 && m < Mg ? rb.gm[(size_t)m] : 0.0L); };
    // W[dl]: output t in block J, input s in block J - dl: m = t - 1 - s in [16 dl - 16, 16 dl + 14]
    const int nw = (int)((Mg + 1 + BS - 1) / BS + 1);
    d.W.assign((size_t)nw, 0.0);
    for (int dl = 0; dl < nw; ++dl) {
      LD mx = 0.0L;
      for (int64_t m = (int64_t)BS * dl - BS; m <= (int64_t)BS * dl + BS - 2; ++m) mx = std::max(mx, Gx(m));
      d.W[(size_t)dl] = (double)up(mx);
    }
    // GS[q] = max_{r in [16q, 16q + 15]} Gm(r) (uncut: a chunk's start error, r < L <= 64 blocks)
    d.GS.assign(64, 0.0);
    for (int q = 0; q < 64; ++q) {
      LD mx = 0.0L;
      for (int64_t r = (int64_t)BS * q; r < (int64_t)BS * q + BS && (size_t)r < rb.gm.size(); ++r) mx = std::max(mx, rb.gm[(size_t)r]);
      d.GS[(size_t)q] = (double)up(mx);
    }
    // |h| cut at Mh
    LD htot = sum_abs(rb.h);
    int64_t Mh = (int64_t)rb.h.size();
    {
      LD rem = 0.0L;
      for (int64_t m = (int64_t)rb.h.size() - 1; m >= 0; --m) {
        if (rem + std::fabs(rb.h[(size_t)m]) > (LD)kStrictCut * htot) break;
        rem += std::fabs(rb.h[(size_t)m]);
        Mh = m;
      }
      d.hs_tail = (double)up(rem);
      // K12's cut remainder: sum_k sum_m |h(k)| Gx(m) over (k >= Mh or m >= Mg) <= htot w_tail + rem gtot
      d.k12_tail = (double)up(htot * (LD)d.w_tail + rem * gtot);
    }
    auto ha = [&](int64_t k) -> LD { return k >= 0 && k < Mh ? std::fabs(rb.h[(size_t)k]) : 0.0L; };
    // K12(dl) = sum_{k >= max(0, dl)} |h(k)| Gx(k - 1 - dl), dl = s - j in [-Mh, Mg]
    std::vector<LD> k12((size_t)(Mh + Mg + 2), 0.0L);
    for (int64_t dl = -Mh; dl <= Mg + 1; ++dl) {
      LD acc = 0.0L;
      for (int64_t k = std::max<int64_t>(0, dl); k < Mh; ++k) acc += ha(k) * Gx(k - 1 - dl);
      k12[(size_t)(dl + Mh)] = acc;
    }
    // K12 block window: forward block J (j = 16 J + t), D1 block b = J + db (s = 16 b + r): dl = s - j in
    // [16 db - 15, 16 db + 15]; db from -ceil((Mh+15)/16) to ceil((Mg+16)/16)
    const int dbn = (int)((Mh + BS) / BS + 1), dbp = (int)((Mg + 2 * BS) / BS + 1);
    d.k12_off = dbn;
    d.K12.assign((size_t)(dbn + dbp + 1), 0.0);
    for (int db = -dbn; db <= dbp; ++db) {
      LD mx = 0.0L;
      for (int64_t dl = (int64_t)BS * db - (BS - 1); dl <= (int64_t)BS * db + (BS - 1); ++dl)
        if (dl >= -Mh && dl <= Mg + 1) mx = std::max(mx, k12[(size_t)(dl + Mh)]);
      d.K12[(size_t)(db + dbn)] = (double)up(mx);
    }
    // HS[db]: sum_{j' >= j} |h(j' - j)| S(j') with S block-constant: j = 16 J + t, j' in block J + db
    const int nh = (int)((Mh + BS - 1) / BS + 2);
    d.HS.assign((size_t)nh, 0.0);
    for (int db = 0; db < nh; ++db) {
      LD mx = 0.0L;
      for (int t = 0; t < BS; ++t) {
        LD sum = 0.0L;
        for (int r = 0; r < BS; ++r) sum += ha((int64_t)BS * db + r - t);
        mx = std::max(mx, sum);
      }
      d.HS[(size_t)db] = (double)up(mx);
    }
    // TZ[q] = max |tz(k2)| over pass-2 block q, cut where the rest stays below kStrictCut max|tz|
    const LD tzm = max_abs(rb.tz);
    int64_t Mz = (int64_t)rb.tz.size();
    while (Mz > 0 && std::fabs(rb.tz[(size_t)Mz - 1]) < (LD)kStrictCut * tzm) --Mz;
    LD tzrest = 0.0L;
    for (size_t m = (size_t)Mz; m < rb.tz.size(); ++m) tzrest = std::max(tzrest, std::fabs(rb.tz[m]));
    d.tz_tail = (double)up(tzrest);
    d.TZ.assign((size_t)((Mz + BS - 1) / BS + 1), 0.0);
    for (size_t q = 0; q < d.TZ.size(); ++q) {
      LD mx = 0.0L;
      for (int64_t m = (int64_t)q * BS; m < (int64_t)q * BS + BS && m < Mz; ++m) mx = std::max(mx, std::fabs(rb.tz[(size_t)m]));
      d.TZ[q] = (double)up(mx);
    }
  }
  return std::isfinite(d.g1x) && std::isfinite(d.hz) && std::isfinite(d.tk);
}

// bp, lp: the plan's filters; K [w1][8], Z0 [w1 + 1][8]: KS0's tables as the
// device holds them; n, first, sps, n_sym: the plan's shape; w2: the low-pass
// warm-up.  ok = false when a response does not decay (no strict mode).
inline StrictDesign strict_design(const Iir& bp, const Iir& lp, const double* K, const double* Z0, int64_t w1,
                                  int64_t w2, int64_t n, int64_t first, int64_t sps, int64_t n_sym) {
  using namespace strict_detail;
  StrictDesign d;
  const Responses rb = responses(bp), rl = responses(lp);
  if (!rl.ok || n_sym < 2 || !strict_design_bp(bp, K, Z0, w1, d, rb)) return d;
  const int Nl = lp.nt - 1;
  const LD U = kU * std::pow(1.0L + kU, 4);
  // ---- low-pass: the band-pass error X per sample reaches symbol k's sample
  // t (ext index s = t + pad2) with at most lpc[k] X:
  //   input weight w(s) = 3 on the odd extension (2 x[0] - x[k]), 1 inside;
  //   A(s) = sum_{l <= s} |h(l)| w(s - l) + 3 |tz(s)|        (forward pass)
  //   B(s) = sum_k |h(k)| A(s + k) + |tz(m2 - 1 - s)| A(m2 - 1)   (backward)
  const int pad2 = 3 * lp.nt;
  const int64_t m2 = n + 2 * (int64_t)pad2;
  std::vector<LD> habs(rl.h.size());
  for (size_t i = 0; i < habs.size(); ++i) habs[i] = std::fabs(rl.h[i]);
  std::vector<LD> H(habs.size() + 1, 0.0L);   // H[i] = sum_{l < i} |h(l)|
  for (size_t i = 0; i < habs.size(); ++i) H[i + 1] = H[i] + habs[i];
  const LD h1 = H.back();
  auto Hc = [&](int64_t s) -> LD {            // sum_{l <= s} |h(l)|
    if (s < 0) return 0.0L;
    return (size_t)(s + 1) < H.size() ? H[(size_t)s + 1] : h1;
  };
  auto tzs = [&](int64_t s) -> LD { return s >= 0 && (size_t)s < rl.tz.size() ? std::fabs(rl.tz[(size_t)s]) : 0.0L; };
  auto A = [&](int64_t s) -> LD {
    return Hc(s) + 2.0L * (Hc(s) - Hc(s - pad2)) + 2.0L * Hc(s - pad2 - n) + 3.0L * tzs(s);
  };
  const LD tail = 1e-30L * h1 * (3.0L * h1 + 3.0L);   // past the decayed responses
  const LD Aend = A(m2 - 1);
  d.lpc.resize((size_t)n_sym);
  for (int64_t k = 0; k < n_sym; ++k) {
    const int64_t s = first + k * sps + pad2;
    LD B = 0.0L;
    const int64_t kmax = std::min<int64_t>((int64_t)habs.size(), m2 - s);
    for (int64_t q = 0; q < kmax; ++q) B += habs[(size_t)q] * A(s + q);
    B += tzs(m2 - 1 - s) * Aend + tail;
    d.lpc[(size_t)k] = (double)up(B);
  }
  // the low-pass's own rounding (split and serial, both passes), its warm-up
  // truncation and the extension's rounding, per unit low-pass input peak P3
  // (P3 = 3 (max|f| + X): the odd extension of f * lo)
  {
    LD cal = 0.0L, cbl = 0.0L;
    for (int j = 1; j <= Nl; ++j) { cal += std::fabs((LD)lp.a[j]); cbl += std::fabs((LD)lp.b[j]); }
    const LD kxl = 3.0L * cbl + std::fabs((LD)lp.b[0]) * cal, kyl = 3.0L * cal;
    LD g1l = 1.0L;
    for (LD g : rl.gm) g1l += g;
    const LD hzl = h1 + max_abs(rl.tz);
    // states <= zb P (incl. the zi start), outputs <= hzl P, for both paths:
    // the split / serial difference is within the 2^-10 caps of P
    const LD dstep = U * (2.0L * rl.zb + kxl + kyl * hzl) * (1.0L + 0x1p-8L);
    const LD own3 = 2.0L * g1l * dstep;                 // pass 3 (input P3)
    const LD own4 = 2.0L * g1l * dstep * hzl;           // pass 4 (input <= hzl P3)
    LD tailg = 0.0L;                                    // sup_{m >= w2} max_j |g_j(m)|
    for (size_t m = (size_t)std::max<int64_t>(w2, 0); m < rl.gm.size(); ++m) tailg = std::max(tailg, rl.gm[m]);
    const LD trunc = 2.0L * tailg * rl.zb * hzl;        // both passes' dropped start states
    const LD ext = 2.1L * kU * hzl * hzl;               // fl(2 x0 - x) of both paths, weight 1 (P3 already x3)
    d.c3 = (double)up(own3 * hzl + own4 + trunc + ext + 1e-30L);
    d.lp_kx = (double)kxl;
    d.lp_ky = (double)kyl;
  }
  {
    // low-pass radius: |h_lp| mass beyond R / 2 below kStrictCut h1 -> pairs (k, l) with |k - l| > R
    // carry at most 2 h1 rem (x 3: the extension's weight)
    LD rem = 0.0L;
    int64_t R2 = (int64_t)habs.size();
    for (int64_t m = (int64_t)habs.size() - 1; m >= 0; --m) {
      if (rem + habs[(size_t)m] > (LD)kStrictCut * h1) break;
      rem += habs[(size_t)m];
      R2 = m;
    }
    d.lp_rad = 2 * R2 + 2;
    d.lp_tail = (double)up(6.0L * h1 * rem + 1e-30L);
  }
  d.ok = std::isfinite(d.g1x) && std::isfinite(d.hz) && std::isfinite(d.tk) && std::isfinite(d.c3) &&
         d.g1x * (d.kx + 2.0 * d.ky) < 0.125;
  for (double v : d.lpc) d.ok = d.ok && std::isfinite(v);
  return d;
}

}  // namespace amr
