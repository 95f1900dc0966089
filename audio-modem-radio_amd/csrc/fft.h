// fft.h -- the batched fp64 FFT (fft_kernels.hip): launch descriptors shared
// with the host, the launchers, and host-side planning.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>
#include <vector>

#include "amr_internal.h"

namespace amr {

constexpr int kFftTile = 8;       // rows (transforms) per workgroup: 8 x 16 B = one 128-B line per column step
constexpr int kFftThreads = 256;
constexpr int kFftMaxL = 640;     // longest in-LDS transform: 8 rows x 641 x 16 B = 82 KB of LDS
constexpr int kFftMaxVals = kFftTile * kFftMaxL / kFftThreads;   // complex values a thread holds per stage
constexpr int kFftMaxStages = 12;

// One radix-r Stockham stage over rows of length L (host-precomputed so the
// kernels never divide by a runtime value: q = int((i + 0.5f) * inv) is exact
// for the index ranges used, |i| < 2^20).
struct FftStage {
  int r;          // radix 2/3/4/5
  int ns;         // product of the previous radices
  int nb;         // L / r butterflies per row
  int tstep;      // L / (ns * r): W_(ns r)^(k q) = W_L^(k q tstep)
  float inv_nb, inv_ns;
};

struct FftLen {
  int L;
  int nst;
  float inv_L;
  FftStage st[kFftMaxStages];
  const double2* tw;              // W_L^t, t < L (forward sign)
};

// n = n1 * n2; input index j = j1 + n1*j2, output index k = k2 + n2*k1.
struct FftDesc {
  int64_t n;
  int n1, n2;
  FftLen a;                       // length n2: the column pass / the final row pass of a filter
  FftLen c;                       // length n1: the row pass / the middle pass of a filter
  const double2* twn;             // W_n^t, t < n
};

// What the last pass does with each output X[b][k] (k < n):
//   kStore     dst[b][k] = X
//   kHilbert   dst[b][k] = -i*sgn(k) * X     (sgn = +1 for 0 < 2k < n, -1 for
//              2k > n, 0 at k = 0 and k = n/2: scipy.signal.hilbert's h - 1)
//   kEnvelope  X = H[z] = H[f_mark] + i*H[f_space];  f = z[b][k]:
//              cmp[b][k] = hypot(f.x, X.x) > hypot(f.y, X.y)        (modem.py:309,315)
//   kEnvOut    the two envelopes themselves -> dst[b][k] = (|a_mark|, |a_space|)
//   kMulTab    dst[b][k] = X * tab[k]        (Bluestein: times FFT(chirp))
enum FftEpiMode : int { kStore = 0, kHilbert = 1, kEnvelope = 2, kEnvOut = 3, kMulTab = 4 };

struct FftEpi {
  int mode;
  int64_t n;               // logical length (row stride of z / cmp / dst)
  const double2* z;        // kEnvelope / kEnvOut
  uint8_t* cmp;            // kEnvelope
  const double2* tab;      // kMulTab
};

// X = FFT_n(in) or IFFT_n(in) (inverse: conj on load, conj and 1/n on store).
// Two kernels (column pass in -> tmp, row pass tmp -> out); out may alias in.
hipError_t launch_fft(const double2* in, double2* tmp, double2* out, const FftDesc& d, int64_t batch, bool inverse,
                      hipStream_t st);
// out = epi(IFFT_n(mid(FFT_n(in)))), mid = kHilbert (times -i*sgn(k)) or kMulTab
// (times tab[k]).  Three kernels: column pass in -> t1; middle pass (row FFT,
// mid, conj, second row FFT, twiddle) t1 -> t2; final row pass t2 -> epi.
// t2 may alias in and out may alias t1; t1 may not alias in.
hipError_t launch_fft_filter(const double2* in, double2* t1, double2* t2, double2* out, const FftDesc& d,
                             int64_t batch, int mid, const double2* tab, const FftEpi& epi, hipStream_t st);
hipError_t launch_bs_pre(const double2* x, double2* a, const double2* w, int64_t n, int64_t M, int64_t batch,
                         bool inverse, hipStream_t st);
hipError_t launch_bs_post(const double2* y, double2* out, const double2* w, int64_t n, int64_t M, int64_t batch,
                          bool inverse, const FftEpi& epi, hipStream_t st);
hipError_t fft_configure_smem();

// ---- host planning -------------------------------------------------------

inline bool smooth5(int64_t m) {
  for (int p : {2, 3, 5})
    while (m % p == 0) m /= p;
  return m == 1;
}

inline std::vector<int> radices_for(int L) {
  std::vector<int> r;
  int m = L;
  while (m % 4 == 0) { r.push_back(4); m /= 4; }
  while (m % 2 == 0) { r.push_back(2); m /= 2; }
  while (m % 3 == 0) { r.push_back(3); m /= 3; }
  while (m % 5 == 0) { r.push_back(5); m /= 5; }
  return r;
}

// n = n1 * n2 with both 5-smooth and <= kFftMaxL, n1 as close to sqrt(n) as possible.
inline bool fft_split(int64_t n, int& n1, int& n2) {
  int best = -1;
  double bestd = 1e300;
  for (int64_t a = 1; a <= kFftMaxL; ++a) {
    if (n % a) continue;
    const int64_t b = n / a;
    if (b > kFftMaxL || !smooth5(a) || !smooth5(b)) continue;
    const double dd = std::fabs(std::log((double)a) - std::log((double)b));
    if (dd < bestd) { bestd = dd; best = (int)a; }
  }
  if (best < 0) return false;
  n1 = best;
  n2 = (int)(n / best);
  return true;
}

// smallest 5-smooth m >= lo that splits (Bluestein length)
inline int64_t fft_good_size(int64_t lo) {
  for (int64_t m = lo;; ++m) {
    int a, b;
    if (smooth5(m) && fft_split(m, a, b)) return m;
  }
}

// Stage table of a length-L row transform (radices from radices_for).
inline bool fill_fft_len(FftLen& f, int L, const double2* tw) {
  const std::vector<int> r = radices_for(L);
  if ((int)r.size() > kFftMaxStages || L > kFftMaxL) return false;
  f.L = L;
  f.nst = (int)r.size();
  f.inv_L = 1.0f / (float)L;
  f.tw = tw;
  int ns = 1;
  for (int i = 0; i < f.nst; ++i) {
    FftStage& s = f.st[i];
    s.r = r[(size_t)i];
    s.ns = ns;
    s.nb = L / s.r;
    s.tstep = L / (ns * s.r);
    s.inv_nb = 1.0f / (float)s.nb;
    s.inv_ns = 1.0f / (float)s.ns;
    ns *= s.r;
  }
  return true;
}

inline std::vector<double> twiddles(int64_t L) {   // interleaved W_L^t = exp(-2 pi i t / L)
  std::vector<double> w((size_t)(2 * L));
  for (int64_t t = 0; t < L; ++t) {
    const double a = -2.0 * M_PI * (double)t / (double)L;
    w[2 * t] = std::cos(a);
    w[2 * t + 1] = std::sin(a);
  }
  return w;
}

}  // namespace amr
