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
//   F1 k_fsk_bandpass  lane = (stream, tone): both band-pass filtfilts, output
//                      packed as the complex signal z = f_mark + i f_space,
//                      stream-major.
//   F2 (fft_kernels.hip) H[z] = IFFT(-i sgn(k) FFT(z)) = H[f_mark] + i H[f_space]
//                      (the Hilbert transform is real-linear, so one complex
//                      transform pair serves both tones); its last pass forms
//                      both envelopes hypot(f, H f) and packs the compare bits.
//   F3 k_fsk_decide    thread = (stream, bit): window majority, ballot-packed
//                      MSB first into words (then k_sync_pack, util_kernels.hip)
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

// lfilter step (DF-II-T), 7 taps, per-lane coefficients, contracted:
//   y = b0*x + z0 ; z[i] = z[i+1] + x*b[i+1] - y*a[i+1] ; z[5] = x*b6 - y*a6
// The FSK decision compares two envelopes that already pass through an FFT
// whose rounding differs from pocketfft's, so this stage is held to the
// envelope tolerance (1e-9 relative, tests/test_gpu_fsk.py), not op order;
// fused multiply-adds halve its FP64 instruction count.
__device__ __forceinline__ double fsk_step(double (&z)[6], const double (&b)[7], const double (&a)[7], double x) {
  const double y = __builtin_fma(b[0], x, z[0]);
#pragma unroll
  for (int i = 0; i < 5; ++i) z[i] = __builtin_fma(-y, a[i + 1], __builtin_fma(x, b[i + 1], z[i + 1]));
  z[5] = __builtin_fma(-y, a[6], x * b[6]);
  return y;
}

typedef unsigned v4u __attribute__((ext_vector_type(4)));   // native vector (HIP's uint4 is a struct)

constexpr int kFskTile = 64;          // samples per input tile
constexpr int kFskChunk = 32;         // samples per backward chunk (16 pairs)

// s1: [wave][q/2][64 lanes][2] doubles (q = j + (pad & 1), so the body starts on a pair)
__device__ __forceinline__ size_t fsk_pair_index(int64_t w, int64_t m_pairs, int64_t q, int lane) {
  return ((size_t)(w * m_pairs + (q >> 1)) * 64 + lane) * 2 + (q & 1);
}

// F1.  wave = 32 streams x 2 tones (lane = 2*stream + tone).  Input rows are
// loaded 16 B per lane (64 samples of 32 streams per tile) and transposed
// through LDS; the forward output goes to s1 as one 1 KiB row per sample pair;
// the backward output is staged in LDS and written as 512 B row segments of
// z (stream-major complex, f_mark + i f_space).
template <typename T>
__global__ __launch_bounds__(64) void k_fsk_bandpass(const void* xv, int64_t x_stride, int64_t n_streams,
                                                     double* __restrict__ s1, double2* __restrict__ z,
                                                     FskParams p, FskIir f) {
  constexpr int RB = kFskTile * (int)sizeof(T);     // bytes per stream row per tile
  constexpr int PITCH = RB + 16;
  constexpr int LPR = RB / 16;                      // lanes per row in a load
  constexpr int RPI = 64 / LPR;                     // rows per load instruction
  constexpr int NI = 32 / RPI;                      // load instructions per tile
  __shared__ __attribute__((aligned(16))) uint8_t tin[2][32][PITCH];
  __shared__ __attribute__((aligned(16))) double tout[32][kFskChunk * 2 + 2];   // [stream][i][tone], padded
  const int lane = threadIdx.x;
  const int tone = lane & 1, sl = lane >> 1;
  const int64_t w = blockIdx.x;
  const int64_t s = w * 32 + sl;
  const int64_t last = n_streams - 1;
  const T* __restrict__ xall = reinterpret_cast<const T*>(xv);
  const T* __restrict__ x = xall + (s < last ? s : last) * x_stride;
  const int64_t n = p.n;
  const int pad = p.pad;
  const int64_t m = n + 2 * (int64_t)pad;
  const int qs = pad & 1;
  const int64_t m_pairs = (m + qs + 1) >> 1;
  double b[7], a[7], zs[6];
#pragma unroll
  for (int i = 0; i < 7; ++i) { b[i] = f.b[tone][i]; a[i] = f.a[tone][i]; }

  // ---- forward pass -------------------------------------------------------
  const T x0 = x[0], xl = x[n - 1];
  const double e0 = FIn<T>::ext(x0, x[pad]);
#pragma unroll
  for (int i = 0; i < 6; ++i) zs[i] = f.zi[tone][i] * e0;
  for (int j = 0; j < pad; ++j)
    s1[fsk_pair_index(w, m_pairs, j + qs, lane)] = fsk_step(zs, b, a, FIn<T>::ext(x0, x[pad - j]));
  const int64_t n_tiles = n / kFskTile;
  const int64_t n_main = n_tiles * kFskTile;
  if (n_tiles > 0) {
    const int rsub = lane / LPR, cb = (lane % LPR) * 16;
    const uint8_t* rowp[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int64_t rs = w * 32 + RPI * i + rsub;
      rowp[i] = reinterpret_cast<const uint8_t*>(xall + (rs < last ? rs : last) * x_stride) + cb;
    }
    v4u r[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) r[i] = *reinterpret_cast<const v4u*>(rowp[i]);
#pragma unroll
    for (int i = 0; i < NI; ++i) *reinterpret_cast<v4u*>(&tin[0][RPI * i + rsub][cb]) = r[i];
    __syncthreads();
    for (int64_t t = 0; t < n_tiles; ++t) {
      const int cur = (int)(t & 1);
      const int64_t tn = (t + 1 < n_tiles) ? t + 1 : t;   // unconditional (clamped) prefetch
#pragma unroll
      for (int i = 0; i < NI; ++i) r[i] = *reinterpret_cast<const v4u*>(rowp[i] + tn * RB);
      __builtin_amdgcn_sched_barrier(0);
      const int64_t q0 = pad + qs + t * kFskTile;         // even
      double2* __restrict__ dst = reinterpret_cast<double2*>(s1) + (size_t)(w * m_pairs + (q0 >> 1)) * 64 + lane;
      constexpr int PER = 16 / (int)sizeof(T);
#pragma unroll
      for (int k = 0; k < kFskTile; k += PER) {
        const v4u v = *reinterpret_cast<const v4u*>(&tin[cur][sl][k * sizeof(T)]);
        T xs[PER];
        __builtin_memcpy(xs, &v, 16);
#pragma unroll
        for (int u = 0; u < PER; u += 2) {
          const double y0 = fsk_step(zs, b, a, FIn<T>::cvt(xs[u]));
          const double y1 = fsk_step(zs, b, a, FIn<T>::cvt(xs[u + 1]));
          dst[((k + u) >> 1) * 64] = make_double2(y0, y1);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < NI; ++i) *reinterpret_cast<v4u*>(&tin[cur ^ 1][RPI * i + rsub][cb]) = r[i];
      __syncthreads();
    }
  }
  for (int64_t i = n_main; i < n; ++i)
    s1[fsk_pair_index(w, m_pairs, pad + i + qs, lane)] = fsk_step(zs, b, a, FIn<T>::cvt(x[i]));
  double ylast = 0.0;
  for (int j = 0; j < pad; ++j) {
    ylast = fsk_step(zs, b, a, FIn<T>::ext(xl, x[n - 2 - j]));
    s1[fsk_pair_index(w, m_pairs, pad + n + j + qs, lane)] = ylast;
  }
  __threadfence();

  // ---- backward pass ------------------------------------------------------
#pragma unroll
  for (int i = 0; i < 6; ++i) zs[i] = f.zi[tone][i] * ylast;
  for (int64_t j = m - 1; j >= pad + n; --j) (void)fsk_step(zs, b, a, s1[fsk_pair_index(w, m_pairs, j + qs, lane)]);
  const int64_t nc = n / kFskChunk;                 // full chunks, processed top-down
  const int64_t n_lo = nc * kFskChunk;
  double* __restrict__ zd = reinterpret_cast<double*>(z);
  for (int64_t i = n - 1; i >= n_lo; --i) {         // top remainder, one sample at a time
    const double y = fsk_step(zs, b, a, s1[fsk_pair_index(w, m_pairs, pad + i + qs, lane)]);
    if (s < n_streams) zd[((size_t)s * n + i) * 2 + tone] = y;
  }
  if (nc > 0) {
    const double2* __restrict__ src = reinterpret_cast<const double2*>(s1) + (size_t)w * m_pairs * 64 + lane;
    constexpr int PP = kFskChunk / 2;
    double2 ra[PP], rb[PP];
    auto load = [&](double2 (&r)[PP], int64_t c0) {
      const int64_t c = c0 < 0 ? 0 : c0;
      const int64_t qp = (pad + qs + c * kFskChunk) >> 1;
#pragma unroll
      for (int k = 0; k < PP; ++k) r[k] = src[(size_t)(qp + k) * 64];
    };
    // chunk c -> z[s][32c .. 32c+32): 32 streams x 512 B, two rows per store instruction
    auto run = [&](const double2 (&r)[PP], int64_t c) {
#pragma unroll
      for (int k = PP - 1; k >= 0; --k) {
        const double y1 = fsk_step(zs, b, a, r[k].y);
        const double y0 = fsk_step(zs, b, a, r[k].x);
        tout[sl][(2 * k) * 2 + tone] = y0;
        tout[sl][(2 * k + 1) * 2 + tone] = y1;
      }
      __syncthreads();
      const int half = lane >> 5, col = lane & 31;
#pragma unroll 4
      for (int rr = 0; rr < 32; rr += 2) {
        const int row = rr + half;
        const int64_t so = w * 32 + row;
        if (so < n_streams)
          z[(size_t)so * n + c * kFskChunk + col] =
              make_double2(tout[row][2 * col], tout[row][2 * col + 1]);
      }
      __syncthreads();
    };
    load(ra, nc - 1);
    load(rb, nc - 2);
    int64_t c = nc - 1;
    for (; c >= 1; c -= 2) {
      run(ra, c);
      __builtin_amdgcn_sched_barrier(0);
      load(ra, c - 2);
      __builtin_amdgcn_sched_barrier(0);
      run(rb, c - 1);
      __builtin_amdgcn_sched_barrier(0);
      load(rb, c - 3);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (c == 0) run(ra, 0);
  }
}

// F3.  thread = (stream, bit): bit b of the stream is 1 when more than half of
// the compare bits of samples [i-q, min(i+q, n)) are 1, i = sps/2 + b*sps
// (np.mean(chunk) > 0.5, modem.py:320-323).  Compare bits are in the final
// row pass's tile order (fft.h fft_bits_stride).  A wave covers 64
// consecutive bits; a ballot packs them MSB first into two words.
__global__ __launch_bounds__(64) void k_fsk_decide(const uint8_t* __restrict__ bits, uint32_t* __restrict__ words,
                                                   int64_t n_streams, FskParams p) {
  const int64_t s = blockIdx.y;
  const int64_t bi = (int64_t)blockIdx.x * 64 + threadIdx.x;
  const uint8_t* __restrict__ c = bits + (size_t)s * p.bits_stride;
  const int64_t q = p.sps / 4, half = p.sps / 2;
  bool bit = false;
  if (bi < p.n_bits) {
    const int64_t i = half + bi * p.sps;
    const int64_t lo = i - q, hi = (i + q < p.n) ? i + q : p.n;
    // sample lo = r + rn1*kk
    int64_t kk = (int64_t)(((float)lo + 0.5f) * p.inv_rn1);
    int64_t r = lo - kk * p.rn1;
    int64_t ones = 0;
    for (int64_t k = lo; k < hi; ++k) {
      ones += (c[(r >> 3) * p.rn2 + kk] >> (r & 7)) & 1;
      if (++r == p.rn1) {
        r = 0;
        ++kk;
      }
    }
    bit = 2 * ones > hi - lo;
  }
  const uint64_t mask = __ballot(bit);
  const int64_t w0 = (int64_t)blockIdx.x * 2;
  if (threadIdx.x == 0 && w0 < p.n_words) words[(size_t)s * p.n_words + w0] = __brev((uint32_t)mask);
  if (threadIdx.x == 32 && w0 + 1 < p.n_words) words[(size_t)s * p.n_words + w0 + 1] = __brev((uint32_t)(mask >> 32));
}

hipError_t launch_fsk_bandpass(int dtype, const void* x, int64_t x_stride, int64_t n_streams, double* s1, double2* z,
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
  hipLaunchKernelGGL(k_fsk_decide, dim3((unsigned)((p.n_bits + 63) / 64), (unsigned)n_streams), dim3(64), 0, st,
                     cmp, words, n_streams, p);
  return hipGetLastError();
}

}  // namespace amr
