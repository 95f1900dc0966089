// fsk_kernels.hip -- batched FSK demodulation for gfx950.
//
// Replaces, for a batch of equal-length streams, the reference
//   modem.fsk_demodulate  (/root/reference/modem.py:298-341)
// (and its aliases fsk_high_speed_demodulate modem.py:355-356,
//  ft8_demodulate modem.py:391, decoder.py:426-432).
//
// Per stream:                                              reference
//   f_t   = filtfilt(butter(3, [(t-b)/nyq, (t+b)/nyq]), x)  modem.py:307-308
//   env_t = |hilbert(f_t)|                                  modem.py:309
//   bit_i = env_mark_i > env_space_i                        modem.py:315
//   decided bit per symbol = majority over bits[i-q, i+q)   modem.py:320-323
//   sync on "FB", pack MSB first from idx or 0              modem.py:326-341
//
// Kernels:
//   F1 k_fsk_bandpass  lane = (stream, tone): both band-pass filtfilts, exact
//                      scipy op order (same step as K1), output packed as the
//                      complex signal z = f_mark + i f_space, stream-major.
//   F2/F3              forward FFT of z (fft_kernels.hip), times -i*sgn(k)
//   F4/F5              inverse FFT  -> H[z] = H[f_mark] + i H[f_space]   (the
//                      Hilbert transform is real-linear, so one complex FFT
//                      pair serves both tones); the last pass forms both
//                      envelopes hypot(f, H f) and writes the compare bit.
//   F6 k_fsk_decide    thread = (stream, output word): window majority, bits
//                      MSB first -> words (then k_sync_pack, util_kernels.hip)
// Parity: the FFT cannot reproduce pocketfft's rounding; envelopes agree to
// ~1e-15 relative and decisions are compared bit for bit with the reference
// (tests/test_gpu_parity.py), with the envelope tolerance stated there.
#include "amr_internal.h"

namespace amr {

template <typename T> struct FIn;
template <> struct FIn<float> {
  static __device__ __forceinline__ double cvt(float v) { return (double)v; }
  static __device__ __forceinline__ double ext(float e, float v) { return (double)(2.0f * e - v); }
};
template <> struct FIn<double> {
  static __device__ __forceinline__ double cvt(double v) { return v; }
  static __device__ __forceinline__ double ext(double e, double v) { return 2.0 * e - v; }
};
template <> struct FIn<int16_t> {
  static __device__ __forceinline__ double cvt(int16_t v) { return (double)v / 32768.0; }
  static __device__ __forceinline__ double ext(int16_t e, int16_t v) { return 2.0 * cvt(e) - cvt(v); }
};

// scipy lfilter step (DF-II-T, exact order), 7 taps, per-lane coefficients
__device__ __forceinline__ double fsk_step(double (&z)[6], const double (&b)[7], const double (&a)[7], double x) {
  const double y = z[0] + b[0] * x;
#pragma unroll
  for (int i = 0; i < 5; ++i) z[i] = (z[i + 1] + x * b[i + 1]) - y * a[i + 1];
  z[5] = x * b[6] - y * a[6];
  return y;
}

// F1.  wave = 32 streams x 2 tones; s1 scratch time-major [wave][j][64].
template <typename T>
__global__ __launch_bounds__(64) void k_fsk_bandpass(const void* xv, int64_t x_stride, int64_t n_streams,
                                                     double* __restrict__ s1, double* __restrict__ z,
                                                     FskParams p, FskIir f) {
  const int lane = threadIdx.x;
  const int tone = lane & 1;
  const int64_t w = blockIdx.x;
  const int64_t s = w * 32 + (lane >> 1);
  const int64_t last = n_streams - 1;
  const T* __restrict__ x = reinterpret_cast<const T*>(xv) + (s < last ? s : last) * x_stride;
  const int64_t n = p.n;
  const int pad = p.pad;
  const int64_t m = n + 2 * (int64_t)pad;
  double b[7], a[7], zs[6];
#pragma unroll
  for (int i = 0; i < 7; ++i) { b[i] = f.b[tone][i]; a[i] = f.a[tone][i]; }
  double* __restrict__ sc = s1 + (size_t)w * m * 64 + lane;
  auto S = [&](int64_t j) -> double& { return sc[(size_t)j * 64]; };

  const T x0 = x[0], xl = x[n - 1];
  const double e0 = FIn<T>::ext(x0, x[pad]);
#pragma unroll
  for (int i = 0; i < 6; ++i) zs[i] = f.zi[tone][i] * e0;
  for (int j = 0; j < pad; ++j) S(j) = fsk_step(zs, b, a, FIn<T>::ext(x0, x[pad - j]));
  constexpr int CH = 16;
  const int64_t nm = (n / CH) * CH;
  T nxt[CH];
#pragma unroll
  for (int k = 0; k < CH; ++k) nxt[k] = nm > 0 ? x[k] : T(0);
  for (int64_t c = 0; c < nm; c += CH) {
    T cur[CH];
#pragma unroll
    for (int k = 0; k < CH; ++k) cur[k] = nxt[k];
    const int64_t cn = c + CH < nm ? c + CH : c;
#pragma unroll
    for (int k = 0; k < CH; ++k) nxt[k] = x[cn + k];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < CH; ++k) S(pad + c + k) = fsk_step(zs, b, a, FIn<T>::cvt(cur[k]));
    __builtin_amdgcn_sched_barrier(0);
  }
  for (int64_t i = nm; i < n; ++i) S(pad + i) = fsk_step(zs, b, a, FIn<T>::cvt(x[i]));
  double ylast = 0.0;
  for (int j = 0; j < pad; ++j) {
    ylast = fsk_step(zs, b, a, FIn<T>::ext(xl, x[n - 2 - j]));
    S(pad + n + j) = ylast;
  }
  __threadfence();
#pragma unroll
  for (int i = 0; i < 6; ++i) zs[i] = f.zi[tone][i] * ylast;
  for (int64_t j = m - 1; j >= pad + n; --j) (void)fsk_step(zs, b, a, S(j));
  // outputs i = n-1 .. 0 -> z[s][i].tone  (stream-major complex)
  double* __restrict__ zo = z + (size_t)(s < last ? s : last) * n * 2 + tone;
  for (int64_t i = n - 1; i >= 0; --i) {
    const double y = fsk_step(zs, b, a, S(pad + i));
    if (s < n_streams) zo[(size_t)i * 2] = y;
  }
}

// F6.  thread = (stream, word): bit b of the stream is 1 when more than half of
// cmp[i-q, min(i+q, n)) are 1, i = sps/2 + b*sps  (np.mean(chunk) > 0.5)
__global__ __launch_bounds__(64) void k_fsk_decide(const uint8_t* __restrict__ cmp, uint32_t* __restrict__ words,
                                                   int64_t n_streams, FskParams p) {
  const int64_t wi = blockIdx.x;
  const int64_t s = (int64_t)blockIdx.y * 64 + threadIdx.x;
  if (s >= n_streams) return;
  const uint8_t* __restrict__ c = cmp + (size_t)s * p.n;
  const int64_t q = p.sps / 4, half = p.sps / 2;
  uint32_t word = 0;
  for (int u = 0; u < 32; ++u) {
    const int64_t bi = wi * 32 + u;
    if (bi >= p.n_bits) break;
    const int64_t i = half + bi * p.sps;
    const int64_t lo = i - q, hi = (i + q < p.n) ? i + q : p.n;
    int64_t ones = 0;
    for (int64_t k = lo; k < hi; ++k) ones += c[k];
    word |= (2 * ones > hi - lo ? 1u : 0u) << (31 - u);
  }
  words[(size_t)s * p.n_words + wi] = word;
}

hipError_t launch_fsk_bandpass(int dtype, const void* x, int64_t x_stride, int64_t n_streams, double* s1, double* z,
                               const FskParams& p, const FskIir& f, hipStream_t st) {
  const unsigned grid = (unsigned)((n_streams + 31) / 32);
  switch (dtype) {
    case kF32: hipLaunchKernelGGL(k_fsk_bandpass<float>, dim3(grid), dim3(64), 0, st, x, x_stride, n_streams, s1, z, p, f); break;
    case kF64: hipLaunchKernelGGL(k_fsk_bandpass<double>, dim3(grid), dim3(64), 0, st, x, x_stride, n_streams, s1, z, p, f); break;
    case kI16: hipLaunchKernelGGL(k_fsk_bandpass<int16_t>, dim3(grid), dim3(64), 0, st, x, x_stride, n_streams, s1, z, p, f); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_fsk_decide(const uint8_t* cmp, uint32_t* words, int64_t n_streams, const FskParams& p,
                             hipStream_t st) {
  if (p.n_words < 1 || p.n_bits < 1) return hipSuccess;
  hipLaunchKernelGGL(k_fsk_decide, dim3((unsigned)p.n_words, (unsigned)((n_streams + 63) / 64)), dim3(64), 0, st,
                     cmp, words, n_streams, p);
  return hipGetLastError();
}

}  // namespace amr
