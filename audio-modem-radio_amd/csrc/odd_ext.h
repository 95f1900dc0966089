// odd_ext.h -- the band-pass input as scipy's filtfilt sees it: the samples
// converted to float64 and the odd extension (scipy _arraytools.odd_ext,
// padtype='odd', padlen = 3 * ntaps) around them.  Shared by the PSK kernels
// (psk_common.h) and the FSK F1 kernels (fsk_kernels.hip).
//
// scipy forms the extension 2*x[0] - x[k] on the CALLER's array, so in the
// caller's dtype (reference modem.py:77, 198, 308 pass `samples` straight to
// filtfilt): float32 rounds it in float32, and an int16 capture with
// |x[0]| > 16383 WRAPS (2 * an int16 array stays int16 under NEP 50).  The
// kernels' storage types (float32, float64, and int16 read as PCM / 32768 for
// decode_wav_file) form it themselves (In<T>::ext); for every other caller
// dtype -- raw integers of any width, bool, float16 -- the host builds the
// 2 * pad extension samples per stream with numpy in that dtype and hands them
// over as a table (PskBuffers::edge / FskParams::edge, include/amr.h
// amr_psk_demod_host_edges), and the samples themselves go in as an exact
// float32 / float64 copy.  DESIGN.md §2 item 7.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace amr {

// input conversion + odd extension in the INPUT's precision
template <typename T> struct In;
template <> struct In<float> {
  static __device__ __forceinline__ double cvt(float v) { return (double)v; }
  static __device__ __forceinline__ double ext(float e, float v) { return (double)(2.0f * e - v); }
};
template <> struct In<double> {
  static __device__ __forceinline__ double cvt(double v) { return v; }
  static __device__ __forceinline__ double ext(double e, double v) { return 2.0 * e - v; }
};
template <> struct In<int16_t> {   // decode_wav_file: float64 = int16 / 32768 (exact)
  static __device__ __forceinline__ double cvt(int16_t v) { return (double)v / 32768.0; }
  static __device__ __forceinline__ double ext(int16_t e, int16_t v) { return 2.0 * cvt(e) - cvt(v); }
};

// The extension samples of one stream: left(j) is extended index j (j < pad:
// 2 x[0] - x[pad - j]), right(r) is extended index pad + n + r (r < pad:
// 2 x[n-1] - x[n-2-r]).  tab: the host's [2 * pad] row for this stream (the
// left pad, then the right), or null to form them from x.  The branch is
// uniform over a launch and sits outside the kernels' sample loops.
template <typename T> struct OddExt {
  const T* x;
  const double* tab;
  int64_t n;
  int pad;
  T x0, xl;
  __device__ __forceinline__ OddExt(const T* xs, const double* edge, int64_t row, int64_t n_, int pad_)
      : x(xs), tab(edge ? edge + row * 2 * (int64_t)pad_ : nullptr), n(n_), pad(pad_), x0(xs[0]), xl(xs[n_ - 1]) {}
  __device__ __forceinline__ double left(int64_t j) const { return tab ? tab[j] : In<T>::ext(x0, x[pad - j]); }
  __device__ __forceinline__ double right(int64_t r) const { return tab ? tab[pad + r] : In<T>::ext(xl, x[n - 2 - r]); }
  // the input peak pk (max |x|; NaN / inf dominate) raised to the largest
  // |table sample|: F2's margin must scale with what the filters saw
  // (fsk_kernels.hip AMB).  Without a table the extension is within 3 pk, the
  // case the margin was sized on; a wrapped table sample can exceed that
  // (uint8 x[0] = 0, x[k] = 1: 0 - 1 wraps to 255).  A NaN pk stays NaN.
  __device__ __forceinline__ double peak_with_tab(double pk) const {
    if (tab)
      for (int j = 0; j < 2 * pad; ++j) {
        const double v = fabs(tab[j]);
        pk = v > pk ? v : pk;
      }
    return pk;
  }
};

}  // namespace amr
