// fft.h -- the four-step FFT (fft_kernels.hip): launch descriptors shared with
// the host, the launchers, and host-side planning.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>
#include <vector>

#include "amr_internal.h"

namespace amr {

constexpr int kFftTile = 8;       // transforms per workgroup
constexpr int kFftThreads = 256;
constexpr int kFftMaxL = 640;     // 2 LDS buffers * 8 rows * 640 * 16 B = 160 KiB
constexpr int kFftMaxStages = 12;

struct FftLen {
  int L;
  int nst;
  int r[kFftMaxStages];           // radices, applied in order
  const double2* tw;              // W_L^t, t < L (forward sign)
};

struct FftDesc {
  int64_t n;
  int n1, n2;
  FftLen a;                       // length n2 (pass A)
  FftLen c;                       // length n1 (pass C)
  const double2* twn;             // W_n^t, t < n
};

enum FftEpiMode : int { kStore = 0, kHilbert = 1, kEnvelope = 2, kEnvOut = 3, kMulTab = 4 };

struct FftEpi {
  int mode;
  int64_t n;               // logical length (row stride of z / cmp / dst)
  const double2* z;        // kEnvelope / kEnvOut
  uint8_t* cmp;            // kEnvelope
  const double2* tab;      // kMulTab
};

hipError_t launch_fft(const double2* in, double2* tmp, double2* out, const FftDesc& d, int64_t batch, bool inverse,
                      const FftEpi& epi, hipStream_t st);
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
