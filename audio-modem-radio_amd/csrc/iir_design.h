// iir_design.h -- host-side analysis of a DF-II-T recursion for the
// time-split layouts (PSK: api.cpp split_design; FSK:
// fsk_api.cpp fsk_split_design, §3d): how far a chunk's zero start and its
// rounding trajectory can move the outputs.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "amr_internal.h"

namespace amr {

// The DF-II-T's responses with zero input (scipy's recursion, a[0] = 1):
//   g_i  the output after a unit error in state i -- how one step's rounding
//        in state i reaches the output; g1 = sum_i sum_m |g_i(m)|, and
//        tail(m) = sup_{m' >= m} sum_i |g_i(m')| (what a state error left m
//        steps back still contributes);
//   h    the output and states after a unit input sample: h1 = ||h||_1 (the
//        L1 gain), zmax = max_i ||h_{x -> z_i}||_1 (a state per unit input peak).
struct IirGains {
  double g1 = 0.0, h1 = 0.0, zmax = 0.0;
  std::vector<double> tail;
  bool ok = false;
};
inline IirGains iir_gains(const Iir& f) {
  IirGains r;
  const int N = f.nt - 1;
  constexpr int64_t kMaxSteps = 4000000;
  std::vector<double> zs((size_t)N * N, 0.0);
  for (int i = 0; i < N; ++i) zs[(size_t)i * N + i] = 1.0;
  bool decayed = false;
  for (int64_t m = 0; m < kMaxSteps && !decayed; ++m) {
    double t = 0.0, live = 0.0;
    for (int i = 0; i < N; ++i) {
      double* z = &zs[(size_t)i * N];
      const double y = z[0];
      for (int j = 0; j < N - 1; ++j) z[j] = z[j + 1] - f.a[j + 1] * y;
      z[N - 1] = -f.a[N] * y;
      t += std::fabs(y);
      for (int j = 0; j < N; ++j) live = std::max(live, std::fabs(z[j]));
    }
    r.g1 += t;
    r.tail.push_back(t);
    decayed = live < 1e-40 && m > 4 * N;
  }
  if (!decayed || !std::isfinite(r.g1)) return r;
  for (int64_t m = (int64_t)r.tail.size() - 2; m >= 0; --m) r.tail[(size_t)m] = std::max(r.tail[(size_t)m], r.tail[(size_t)m + 1]);
  std::vector<double> z(N, 0.0), zsum(N, 0.0);
  double x = 1.0;
  decayed = false;
  for (int64_t m = 0; m < kMaxSteps && !decayed; ++m) {
    const double y = z[0] + f.b[0] * x;
    for (int j = 0; j < N - 1; ++j) z[j] = z[j + 1] + f.b[j + 1] * x - f.a[j + 1] * y;
    z[N - 1] = f.b[N] * x - f.a[N] * y;
    r.h1 += std::fabs(y);
    double live = 0.0;
    for (int j = 0; j < N; ++j) {
      zsum[j] += std::fabs(z[j]);
      live = std::max(live, std::fabs(z[j]));
    }
    x = 0.0;
    decayed = live < 1e-40 && m > 4 * N;
  }
  r.zmax = *std::max_element(zsum.begin(), zsum.end());
  r.ok = decayed && std::isfinite(r.h1) && std::isfinite(r.zmax);
  return r;
}
// ||y||_2 of the DF-II-T's output with zero input from scipy's zi state (the
// transient a filtfilt pass's zi * x0 start adds per unit x0), in long
// double; -1 if it has not decayed within the step limit
inline double zi_response_l2(const Iir& f) {
  const int N = f.nt - 1;
  long double z[8] = {0};
  for (int i = 0; i < N; ++i) z[i] = f.zi[i];
  long double s2 = 0.0L;
  for (int64_t m = 0; m < 4000000; ++m) {
    const long double y = z[0];
    for (int j = 0; j < N - 1; ++j) z[j] = z[j + 1] - (long double)f.a[j + 1] * y;
    z[N - 1] = -(long double)f.a[N] * y;
    s2 += y * y;
    long double live = 0.0L;
    for (int j = 0; j < N; ++j) live = std::max(live, std::fabs(z[j]));
    if (live < 1e-40L && m > 4 * N) return (double)std::sqrt(s2) * (1.0 + 0x1p-30);
  }
  return -1.0;
}
// the first m with tail(m) * scale <= tol (-1: none within the response)
inline int64_t warmup_for(const IirGains& g, double scale, double tol) {
  for (size_t m = 0; m < g.tail.size(); ++m)
    if (g.tail[m] * scale <= tol) return (int64_t)m;
  return -1;
}
// ||a||_1 of scipy.signal.hilbert's analytic-signal kernel a = ifft(h) at
// length n (h = 1, 2, ..., 2, [1 at n/2 for even n], 0, ...): a[0] = 1 and,
// for k > 0, a[k] = i (2/n) sum_{j=1..P} sin(2 pi j k / n), P = ceil(n/2) - 1
// -- the real part is the identity.  So a band-pass output off by at most e
// per sample moves each |analytic| sample by at most e * ||a||_1 (a circular
// convolution), ~ (2/pi) ln n (7.4 at n = 96000).  Summed in long double,
// symmetric halves once.
inline double hilbert_l1(int64_t n) {
  if (n < 2) return 1.0;
  const int64_t P = (n + 1) / 2 - 1;
  const long double pi = 3.141592653589793238462643383279502884L;
  long double sum = 0.0L;
  for (int64_t k = 1; k <= n / 2; ++k) {
    const long double th = 2.0L * pi * (long double)k / (long double)n;
    const long double sh = std::sin(0.5L * th);
    const long double v = std::fabs(2.0L * std::sin(0.5L * (long double)P * th) *
                                    std::sin(0.5L * (long double)(P + 1) * th) / (sh * (long double)n));
    sum += (2 * k == n) ? v : 2.0L * v;
  }
  return (double)(1.0L + sum);
}

// The time-split layouts' convolution start states (psk_split_kernels.hip
// KS0, fsk_kernels.hip FS0): tables for a filter f (nt - 1 states, DF-II-T, a[0] = 1) in long
// double, rounded once: K[m] = the state after a unit input and m zero inputs
// (m < w), Z0[t] = scipy's zi after t zero inputs (t <= w; Z0[0] = zi
// exactly).  The state before input t0 of a run that started at 0 from zi v0
// is Z0[t0] v0 + sum_{m < t0} K[m] v(t0 - 1 - m); a run's warm-up computes
// the same map truncated at m < w (rows of nt - 1 doubles)
inline void split_state_tables(const Iir& f, int64_t w, double* K, double* Z0) {
  const int ns = f.nt - 1;
  long double z[kMaxTaps], y;
  auto zero_step = [&]() {
    y = z[0];
    for (int i = 0; i < ns - 1; ++i) z[i] = z[i + 1] - (long double)f.a[i + 1] * y;
    z[ns - 1] = -(long double)f.a[ns] * y;
  };
  for (int i = 0; i < ns; ++i)
    z[i] = (long double)f.b[i + 1] - (long double)f.a[i + 1] * (long double)f.b[0];
  for (int64_t m = 0; m < w; ++m) {
    for (int i = 0; i < ns; ++i) K[m * ns + i] = (double)z[i];
    zero_step();
  }
  for (int i = 0; i < ns; ++i) { z[i] = f.zi[i]; Z0[i] = f.zi[i]; }
  for (int64_t t = 1; t <= w; ++t) {
    zero_step();
    for (int i = 0; i < ns; ++i) Z0[t * ns + i] = (double)z[i];
  }
}
}  // namespace amr
