// fft.h -- the batched fp64 FFT (fft_kernels.hip): launch descriptors shared
// with the host, the launchers, and host-side planning.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "amr_internal.h"

namespace amr {

constexpr int kFftTile = 8;        // rows (transforms) per workgroup: 8 x 16 B = one 128-B line per column step
constexpr int kFftThreads = 256;   // four waves: every stage is one butterfly per thread (8 * 25 <= 256)
constexpr int kFftMaxR = 25;       // largest radix of one stage
constexpr int kFftMaxL = kFftMaxR * kFftMaxR;   // two stages per row transform

// Radices one stage can run as a register-resident DFT: a*b with a, b in 1..5.
inline bool fft_radix_ok(int r) {
  switch (r) {
    case 1: case 2: case 3: case 4: case 5: case 6: case 8: case 9: case 10: case 12: case 15: case 16:
    case 20: case 25: return true;
  }
  return false;
}

// LDS layout of one row's intermediate Y[j][m] (j < Q, m < P): position
// j + qp*m with qp = Q rounded up to odd, and the row stride S = 2 (mod 16)
// 16-B slots, so the 8 rows x 2 columns a 16-lane group touches fall in 16
// distinct bank slots.
__host__ __device__ constexpr int fft_block(int Q) { return Q | 1; }
__host__ __device__ constexpr int fft_row_stride(int P, int Q) {
  return P * fft_block(Q) + ((2 - P * fft_block(Q)) % 16 + 16) % 16;
}

// A row transform of length L = r1 * r2 (P = r1, Q = r2) in two register
// stages: radix P over stride Q, then twiddles W_L^(j m) and radix Q
// (fft_kernels.hip); r1 >= r2, r2 == 1 for a single stage.
struct FftLen {
  int L, r1, r2;
  int qp;                         // fft_block(r2)
  int S;                          // fft_row_stride(r1, r2)
  float inv_r2;                   // 1/r2 for the row-major thread mapping (exact division, fft_kernels.hip)
  const double2* tw;              // W_L^t, t < L (forward sign)
};

// n = n1 * n2; input index j = j1 + n1*j2, output index k = k2 + n2*k1.
struct FftDesc {
  int64_t n;
  int n1, n2;
  FftLen a;                       // length n2: the column pass / the final row pass of a filter
  FftLen c;                       // length n1: the row pass / the middle pass of a filter
  const double2* tw_lo;           // W_n^t, t < 256
  const double2* tw_hi;           // W_n^(256 t), t < ceil(n / 256)
};

// What the last pass does with each output X[b][k] (k < n):
//   kStore     dst[b][k] = X
//   kHilbert   dst[b][k] = -i*sgn(k) * X     (sgn = +1 for 0 < 2k < n, -1 for
//              2k > n, 0 at k = 0 and k = n/2: scipy.signal.hilbert's h - 1)
//   kEnvelope  X = H[z] = H[f_mark] + i*H[f_space];  f = z[b][k]:
//              bit k = hypot(f.x, X.x) > hypot(f.y, X.y)             (modem.py:309,315)
//              packed 8 per byte in the row-pass tile order (fft_bit_byte)
//   kEnvOut    the two envelopes themselves -> dst[b][k] = (|a_mark|, |a_space|)
//   kMulTab    dst[b][k] = X * tab[k]        (Bluestein: times FFT(chirp))
enum FftEpiMode : int { kStore = 0, kHilbert = 1, kEnvelope = 2, kEnvOut = 3, kMulTab = 4 };

struct FftEpi {
  int mode;
  int64_t n;               // logical length (row stride of z / cmp / dst)
  const double2* z;        // kEnvelope / kEnvOut
  uint8_t* bits;           // kEnvelope: [b][bits_stride] bytes
  int64_t bits_stride;
  const double2* tab;      // kMulTab
  const double* amb;       // kEnvelope, optional: [b] the stream's ambiguity scale (amr_internal.h
  uint32_t* xflags;        // amb_scale) -> bit b of xflags[b / 32] set on a compare inside the margin
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
// launch_fft_filter(kHilbert, kEnvelope) in the live-column layout
// (amr_internal.h LiveCols; fft_kernels.hip k_*_live): zb = [B][L | D], cb = [B][nl * n2]
hipError_t launch_fft_hilbert_live(double2* zb, double2* cb, double2* db, const FftDesc& d, int64_t batch,
                                   const LiveCols& lc, const FftEpi& epi, hipStream_t st);
hipError_t launch_bs_pre(const double2* x, double2* a, const double2* w, int64_t n, int64_t M, int64_t batch,
                         bool inverse, hipStream_t st);
hipError_t launch_bs_post(const double2* y, double2* out, const double2* w, int64_t n, int64_t M, int64_t batch,
                          bool inverse, const FftEpi& epi, hipStream_t st);
hipError_t fft_configure_smem();
// six-step transpose (+ twiddle W_M^(r c) from tw_lo/tw_hi, conjugated when inverse)
hipError_t launch_transpose(const double2* in, double2* out, int64_t R, int64_t C, int64_t batch,
                            const double2* tw_lo, const double2* tw_hi, bool inverse, hipStream_t st);

// Compare bits of a length-n filter output: sample k = r + rn1*kk (r < rn1,
// kk < rn2) is bit (r & 7) of byte (r >> 3)*rn2 + kk -- the order in which a
// final row pass (8 rows r per workgroup, all kk) produces them, so every
// workgroup writes one contiguous run of bytes.  rn1 = n1, rn2 = n2 for a
// four-step length; rn1 = n, rn2 = 1 (plain bit order) after Bluestein.
__host__ __device__ inline int64_t fft_bits_stride(int64_t rn1, int64_t rn2) { return ((rn1 + 7) >> 3) * rn2; }

// ---- host planning -------------------------------------------------------

// L = r1 * r2 with both radices runnable, r1 >= r2, r2 as large as possible.
inline bool fft_factor(int L, int& r1, int& r2) {
  for (int b = kFftMaxR; b >= 1; --b) {
    if (L % b || !fft_radix_ok(b)) continue;
    const int a = L / b;
    if (a >= b && fft_radix_ok(a)) {
      r1 = a;
      r2 = b;
      return true;
    }
  }
  return false;
}

// n = n1 * n2 with both factorable, n1 as close to sqrt(n) as possible.
inline bool fft_split(int64_t n, int& n1, int& n2) {
  int best = -1;
  double bestd = 1e300;
  for (int64_t a = 1; a <= kFftMaxL; ++a) {
    if (n % a) continue;
    const int64_t b = n / a;
    int x, y;
    if (b > kFftMaxL || !fft_factor((int)a, x, y) || !fft_factor((int)b, x, y)) continue;
    const double dd = std::fabs(std::log((double)a) - std::log((double)b));
    if (dd < bestd) { bestd = dd; best = (int)a; }
  }
  if (best < 0) return false;
  n1 = best;
  n2 = (int)(n / best);
  return true;
}

// M = L1 * L2 with both two-pass lengths (the six-step plan past the two-pass
// limit): L1 <= L2, L1 as large as possible.
inline bool fft_six_split(int64_t M, int64_t& L1, int64_t& L2) {
  const int64_t lim = (int64_t)kFftMaxL * kFftMaxL;
  for (int64_t a = (int64_t)std::sqrt((double)M) + 1; a >= 2; --a) {
    if (M % a) continue;
    const int64_t b = M / a;
    if (a > b || b > lim) continue;
    int x, y;
    if (fft_split(a, x, y) && fft_split(b, x, y)) {
      L1 = a;
      L2 = b;
      return true;
    }
  }
  return false;
}

inline bool fft_plannable(int64_t m) {
  int a, b;
  int64_t c, d;
  return fft_split(m, a, b) || fft_six_split(m, c, d);
}

// Bluestein length: the smallest two-pass length >= lo, else the smallest
// six-step one (only 5-smooth lengths run at all)
inline int64_t fft_good_size(int64_t lo) {
  const int64_t hi = (int64_t)kFftMaxL * kFftMaxL * kFftMaxL * kFftMaxL;
  std::vector<int64_t> cand;
  for (int64_t p2 = 1; p2 <= 2 * lo && p2 <= hi; p2 *= 2)
    for (int64_t p3 = p2; p3 <= 2 * lo && p3 <= hi; p3 *= 3)
      for (int64_t p5 = p3; p5 <= 2 * lo && p5 <= hi; p5 *= 5)
        if (p5 >= lo) cand.push_back(p5);
  std::sort(cand.begin(), cand.end());
  int a, b;
  for (int64_t m : cand)                       // a two-pass length when one exists (fewer passes)
    if (m <= (int64_t)kFftMaxL * kFftMaxL && fft_split(m, a, b)) return m;
  for (int64_t m : cand)
    if (fft_plannable(m)) return m;
  return -1;
}

inline bool fill_fft_len(FftLen& f, int L, const double2* tw) {
  if (!fft_factor(L, f.r1, f.r2)) return false;
  f.L = L;
  f.qp = fft_block(f.r2);
  f.S = fft_row_stride(f.r1, f.r2);
  f.inv_r2 = 1.0f / (float)f.r2;
  f.tw = tw;
  return true;
}

inline std::vector<double> twiddles(int64_t L, int64_t count, int64_t step = 1) {
  // interleaved W_L^(t*step) = exp(-2 pi i t step / L), t < count; the
  // exponent is reduced mod L in integers so the angle is exact before libm
  std::vector<double> w((size_t)(2 * count));
  for (int64_t t = 0; t < count; ++t) {
    const int64_t e = (t * step) % L;
    const double a = -2.0 * M_PI * (double)e / (double)L;
    w[2 * t] = std::cos(a);
    w[2 * t + 1] = std::sin(a);
  }
  return w;
}

}  // namespace amr
