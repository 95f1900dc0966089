// psk_kernels.hip -- batched DQPSK / DBPSK demodulation for gfx950 (MI355X).
//
// Replaces, for a batch of B streams at once, the per-stream reference
//   modem.qpsk_demodulate  (/root/reference/modem.py:189-266)
//   modem.bpsk_demodulate  (/root/reference/modem.py:68-135)
// and every alias that dispatches to them (psk8_demodulate modem.py:348,
// ofdm_demodulate_simple modem.py:375-376, decoder.py:422-434).
//
// Bit-exactness contract: every floating-point operation below is the one
// numpy/scipy performs, in the same order, with no contraction (this file is
// compiled with -ffp-contract=off; every fma() is an fma numpy itself uses).
// The oracle (oracle/amr_oracle.c) states the same arithmetic on the CPU.
//
// Pipeline for one batch (one kernel per stage, all streams in flight):
//   K1 k_bandpass_mix  lane = stream: band-pass filtfilt (forward pass to
//                      s1, backward pass from s1) fused with the LO mixer -> s2
//   K2 k_lowpass_fwd   lane = (stream, re|im): low-pass forward pass -> s3
//   K3 k_lowpass_bwd   lane = (stream, re|im): low-pass backward pass fused
//                      with symbol pick, differential product, slicer and the
//                      bit writer -> words
//   K3x k_lowpass_exact lane = stream: the complex low-pass with scipy's full
//                      signed-zero semantics, only for streams K2/K3 flagged
//   (K4 sync + pack lives in util_kernels.hip)
#include <math.h>

#include "amr_internal.h"

namespace amr {

// ---------------------------------------------------------------------------
// input conversion + odd extension in the INPUT's precision
// (scipy _arraytools.odd_ext: 2*x[0] - x[k] on the caller's dtype)
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

// class masks for __builtin_amdgcn_class (v_cmp_class_f64)
// bit: 0 sNaN 1 qNaN 2 -inf 3 -norm 4 -denorm 5 -0 6 +0 7 +denorm 8 +norm 9 +inf
constexpr int kClsX = 0x2B7;   // low-pass INPUT not provably safe: NaN, inf, denormal, -0
constexpr int kClsY = 0x2F7;   // low-pass OUTPUT not provably safe: the above and +0

// ---------------------------------------------------------------------------
// One step of scipy's real lfilter (DF-II-T), exact op order:
//   y = z0 + b0*x ; z[i] = (z[i+1] + x*b[i+1]) - y*a[i+1] ; z[last] = x*b[last] - y*a[last]
// ZODD: b[1], b[3], ... are +0.0 (Butterworth band-pass); x*(+0.0) is then one
// product shared by those taps -- the same value scipy computes for each.
template <int NT, bool ZODD>
__device__ __forceinline__ double df2t_step(double (&z)[NT - 1], const double (&b)[NT],
                                            const double (&a)[NT], double x) {
  const double y = z[0] + b[0] * x;
  const double xz = x * b[1];
#pragma unroll
  for (int i = 0; i < NT - 2; ++i) {
    const double xb = (ZODD && ((i + 1) & 1)) ? xz : x * b[i + 1];
    z[i] = (z[i + 1] + xb) - y * a[i + 1];
  }
  z[NT - 2] = x * b[NT - 1] - y * a[NT - 1];
  return y;
}

__device__ __forceinline__ size_t pair_index(int64_t group, int64_t m_pairs, int64_t q, int lane) {
  // [group][q/2][64 lanes][2] doubles
  return ((size_t)(group * m_pairs + (q >> 1)) * kWave + lane) * 2 + (q & 1);
}

// ---------------------------------------------------------------------------
// K1: band-pass filtfilt + mixer.  One wave per group of 64 streams, lane = stream.
//   forward : ext[j] (j < m1)  -> s1      (scipy filtfilt forward lfilter)
//   backward: s1 reversed      -> y2, trimmed to [pad1, pad1+n)
//   mixer   : bb[n] = (y2 + 0j) * lo[n]   numpy complex multiply, exact:
//             re = fma(y2, lo_re, -(0*lo_im)),  im = fma(y2, lo_im, 0*lo_re)
// s1 is indexed by q = j + (pad1 & 1) so that the main body starts on a pair.
constexpr int kChunk = 16;

template <int NT, bool ZODD, typename T>
__global__ __launch_bounds__(64) void k_bandpass_mix(PskBuffers buf, PskParams p, Iir f) {
  const int lane = threadIdx.x;
  const int64_t g = blockIdx.x;
  const int64_t s = g * kWave + lane;
  const int64_t sc = s < buf.n_streams ? s : buf.n_streams - 1;   // idle lanes shadow a real stream
  const T* __restrict__ x = reinterpret_cast<const T*>(buf.x) + sc * buf.x_stride;
  const int64_t n = p.n;
  const int pad = p.pad1;
  const int64_t m1 = p.m1;
  const int qs = pad & 1;                       // q = j + qs
  const int64_t m1_pairs = (m1 + qs + 1) >> 1;
  double* __restrict__ s1 = buf.s1;

  double b[NT], a[NT], z[NT - 1];
#pragma unroll
  for (int i = 0; i < NT; ++i) { b[i] = f.b[i]; a[i] = f.a[i]; }

  // ---- forward pass -------------------------------------------------------
  const T x0 = x[0], xl = x[n - 1];
  {
    const double e0 = In<T>::ext(x0, x[pad]);
#pragma unroll
    for (int i = 0; i < NT - 1; ++i) z[i] = f.zi[i] * e0;
  }
  for (int j = 0; j < pad; ++j) {               // left odd extension
    const double y = df2t_step<NT, ZODD>(z, b, a, In<T>::ext(x0, x[pad - j]));
    s1[pair_index(g, m1_pairs, j + qs, lane)] = y;
  }
  // main body: chunks of kChunk samples, next chunk prefetched into registers
  const int64_t n_main = (n / kChunk) * kChunk;
  {
    T nxt[kChunk];
#pragma unroll
    for (int k = 0; k < kChunk; ++k) nxt[k] = (n_main > 0) ? x[k] : T(0);
    for (int64_t c = 0; c < n_main; c += kChunk) {
      T cur[kChunk];
#pragma unroll
      for (int k = 0; k < kChunk; ++k) cur[k] = nxt[k];
      if (c + kChunk < n_main) {
#pragma unroll
        for (int k = 0; k < kChunk; ++k) nxt[k] = x[c + kChunk + k];
      }
      const int64_t q0 = pad + qs + c;          // even
      double2* __restrict__ dst = reinterpret_cast<double2*>(s1) + (size_t)(g * m1_pairs + (q0 >> 1)) * kWave + lane;
#pragma unroll
      for (int k = 0; k < kChunk; k += 2) {
        const double y0 = df2t_step<NT, ZODD>(z, b, a, In<T>::cvt(cur[k]));
        const double y1 = df2t_step<NT, ZODD>(z, b, a, In<T>::cvt(cur[k + 1]));
        dst[(k >> 1) * kWave] = make_double2(y0, y1);
      }
    }
  }
  for (int64_t i = n_main; i < n; ++i) {        // main-body remainder
    const double y = df2t_step<NT, ZODD>(z, b, a, In<T>::cvt(x[i]));
    s1[pair_index(g, m1_pairs, pad + i + qs, lane)] = y;
  }
  double ylast = 0.0;
  for (int j = 0; j < pad; ++j) {               // right odd extension
    ylast = df2t_step<NT, ZODD>(z, b, a, In<T>::ext(xl, x[n - 2 - j]));
    s1[pair_index(g, m1_pairs, pad + n + j + qs, lane)] = ylast;
  }

  // own stores must be visible to own loads below
  __threadfence();

  // ---- backward pass + mixer ----------------------------------------------
#pragma unroll
  for (int i = 0; i < NT - 1; ++i) z[i] = f.zi[i] * ylast;
  // the right extension region: outputs discarded (trimmed)
  for (int64_t j = m1 - 1; j >= pad + n; --j)
    (void)df2t_step<NT, ZODD>(z, b, a, s1[pair_index(g, m1_pairs, j + qs, lane)]);

  const double4* __restrict__ lo = reinterpret_cast<const double4*>(buf.lo);
  double2* __restrict__ bb = reinterpret_cast<double2*>(buf.s2) + (size_t)g * n * kWave + lane;
  // top remainder of the main body, one sample at a time (n % kChunk samples)
  const int64_t n_top = n - n_main;
  for (int64_t i = n - 1; i >= n - n_top; --i) {
    const double y = df2t_step<NT, ZODD>(z, b, a, s1[pair_index(g, m1_pairs, pad + i + qs, lane)]);
    const double4 l = lo[i];
    bb[(size_t)i * kWave] = make_double2(__builtin_fma(y, l.x, l.z), __builtin_fma(y, l.y, l.w));
  }
  // main body backward in chunks; q of chunk start is even
  {
    const double2* __restrict__ src = reinterpret_cast<const double2*>(s1) + (size_t)g * m1_pairs * kWave + lane;
    double2 nxt[kChunk / 2];
    const int64_t cstart = n_main - kChunk;
    if (n_main > 0) {
#pragma unroll
      for (int k = 0; k < kChunk / 2; ++k) nxt[k] = src[(size_t)(((pad + qs + cstart) >> 1) + k) * kWave];
    }
    for (int64_t c = cstart; c >= 0; c -= kChunk) {
      double2 cur[kChunk / 2];
#pragma unroll
      for (int k = 0; k < kChunk / 2; ++k) cur[k] = nxt[k];
      if (c >= kChunk) {
        const int64_t qp = (pad + qs + c - kChunk) >> 1;
#pragma unroll
        for (int k = 0; k < kChunk / 2; ++k) nxt[k] = src[(size_t)(qp + k) * kWave];
      }
#pragma unroll
      for (int k = kChunk / 2 - 1; k >= 0; --k) {
        const int64_t i1 = c + 2 * k + 1, i0 = c + 2 * k;
        const double y1 = df2t_step<NT, ZODD>(z, b, a, cur[k].y);
        const double4 l1 = lo[i1];
        bb[(size_t)i1 * kWave] = make_double2(__builtin_fma(y1, l1.x, l1.z), __builtin_fma(y1, l1.y, l1.w));
        const double y0 = df2t_step<NT, ZODD>(z, b, a, cur[k].x);
        const double4 l0 = lo[i0];
        bb[(size_t)i0 * kWave] = make_double2(__builtin_fma(y0, l0.x, l0.z), __builtin_fma(y0, l0.y, l0.w));
      }
    }
  }
  // (the left extension region of the backward pass produces only trimmed
  //  outputs and no state anyone reads: scipy's final zf is discarded)
}

// ---------------------------------------------------------------------------
// Low-pass kernels: lane l of wave w handles stream 32*(w&1) + l/2 of group
// w/2, component l&1 (0 = re, 1 = im).  s2 row of a half-group is 64
// contiguous doubles, so lane l simply reads element l of that row.
//
// The complex lfilter with real coefficients is two real recurrences EXCEPT
// for the sign of zero results (scipy evaluates b*x as b*xr - (+0)*xi, ...).
// K2/K3 run the separable recurrences and flag a stream whenever an operand
// could make the two differ (kClsX/kClsY above; DESIGN.md §Numerics proves the
// rule); K3x then recomputes that stream with the full complex semantics.

template <int NT>
__device__ __forceinline__ double df2t_lp(double (&z)[NT - 1], const double (&b)[NT],
                                          const double (&a)[NT], double x) {
  const double y = z[0] + b[0] * x;
#pragma unroll
  for (int i = 0; i < NT - 2; ++i) z[i] = (z[i + 1] + x * b[i + 1]) - y * a[i + 1];
  z[NT - 2] = x * b[NT - 1] - y * a[NT - 1];
  return y;
}

template <int NT>
__global__ __launch_bounds__(64) void k_lowpass_fwd(PskBuffers buf, PskParams p, Iir f) {
  const int lane = threadIdx.x;
  const int64_t w = blockIdx.x;                 // wave index = 2*group + half
  const int64_t g = w >> 1, h = w & 1;
  const int64_t n = p.n;
  const int pad = p.pad2;
  const int qs = pad & 1;
  const int64_t m2_pairs = (p.m2 + qs + 1) >> 1;
  const double* __restrict__ in = buf.s2 + ((size_t)g * n * kWave + h * 32) * 2 + lane;   // + n*128
  double* __restrict__ s3 = buf.s3;

  double b[NT], a[NT], z[NT - 1];
#pragma unroll
  for (int i = 0; i < NT; ++i) { b[i] = f.b[i]; a[i] = f.a[i]; }
  bool bad = false;
  auto X = [&](int64_t i) { return in[(size_t)i * 2 * kWave]; };

  const double x0 = X(0), xl = X(n - 1);
  const double e0 = 2.0 * x0 - X(pad);
  bad |= __builtin_amdgcn_class(e0, kClsY);     // zi * ext[0] must not meet a zero
#pragma unroll
  for (int i = 0; i < NT - 1; ++i) z[i] = f.zi[i] * e0;
  for (int j = 0; j < pad; ++j) {
    const double e = 2.0 * x0 - X(pad - j);
    bad |= __builtin_amdgcn_class(e, kClsX);
    const double y = df2t_lp<NT>(z, b, a, e);
    bad |= __builtin_amdgcn_class(y, kClsY);
    s3[pair_index(w, m2_pairs, j + qs, lane)] = y;
  }
  const int64_t n_main = (n / kChunk) * kChunk;
  {
    double nxt[kChunk];
#pragma unroll
    for (int k = 0; k < kChunk; ++k) nxt[k] = (n_main > 0) ? X(k) : 0.0;
    for (int64_t c = 0; c < n_main; c += kChunk) {
      double cur[kChunk];
#pragma unroll
      for (int k = 0; k < kChunk; ++k) cur[k] = nxt[k];
      if (c + kChunk < n_main) {
#pragma unroll
        for (int k = 0; k < kChunk; ++k) nxt[k] = X(c + kChunk + k);
      }
      const int64_t q0 = pad + qs + c;
      double2* __restrict__ dst = reinterpret_cast<double2*>(s3) + (size_t)(w * m2_pairs + (q0 >> 1)) * kWave + lane;
#pragma unroll
      for (int k = 0; k < kChunk; k += 2) {
        bad |= __builtin_amdgcn_class(cur[k], kClsX);
        const double y0 = df2t_lp<NT>(z, b, a, cur[k]);
        bad |= __builtin_amdgcn_class(y0, kClsY);
        bad |= __builtin_amdgcn_class(cur[k + 1], kClsX);
        const double y1 = df2t_lp<NT>(z, b, a, cur[k + 1]);
        bad |= __builtin_amdgcn_class(y1, kClsY);
        dst[(k >> 1) * kWave] = make_double2(y0, y1);
      }
    }
  }
  for (int64_t i = n_main; i < n; ++i) {
    const double e = X(i);
    bad |= __builtin_amdgcn_class(e, kClsX);
    const double y = df2t_lp<NT>(z, b, a, e);
    bad |= __builtin_amdgcn_class(y, kClsY);
    s3[pair_index(w, m2_pairs, pad + i + qs, lane)] = y;
  }
  for (int j = 0; j < pad; ++j) {
    const double e = 2.0 * xl - X(n - 2 - j);
    bad |= __builtin_amdgcn_class(e, kClsX);
    const double y = df2t_lp<NT>(z, b, a, e);
    bad |= __builtin_amdgcn_class(y, kClsY);
    s3[pair_index(w, m2_pairs, pad + n + j + qs, lane)] = y;
  }
  // stream flag = re lane | im lane
  const int fl = bad ? 1 : 0;
  const int other = __shfl_xor(fl, 1);
  const int64_t s = g * kWave + h * 32 + (lane >> 1);
  if ((lane & 1) == 0 && s < buf.n_streams) buf.flags[s] = fl | other;
}

// Exact sector decision of modem.py:216-241 for diff = (dr, di).
// Far from a sector edge (|di| vs |dr| differ by more than 2^-30 relative)
// the sector is read off the signs; near an edge (or for zeros / NaN / inf)
// the reference's own steps are replayed: atan2, +2pi if negative, and the
// same four comparisons against the same double constants.
__device__ __forceinline__ uint32_t qpsk_dibit(double dr, double di) {
  const double adr = fabs(dr), adi = fabs(di);
  const double d = adi - adr;
  const double thr = (adr + adi) * 0x1p-30;
  if (d < -thr) return dr > 0 ? 0u : 3u;        // |angle| < pi/4 -> 00 ; near pi -> 11
  if (d > thr) return di > 0 ? 1u : 2u;         // near +pi/2 -> 01 ; near -pi/2 -> 10
  double ang = atan2(di, dr);
  if (ang < 0) ang += 2 * M_PI;
  if (ang < M_PI / 4 || ang > 7 * M_PI / 4) return 0u;
  if (M_PI / 4 <= ang && ang < 3 * M_PI / 4) return 1u;
  if (3 * M_PI / 4 <= ang && ang < 5 * M_PI / 4) return 3u;
  return 2u;
}

// diff = s_{k+1} * conj(s_k) with numpy's complex multiply (see oracle)
__device__ __forceinline__ void diff_np(double ar, double ai, double sr, double si, double& dr, double& di) {
  const double br = sr, bi = -si;
  dr = __builtin_fma(ar, br, -(ai * bi));
  di = __builtin_fma(ar, bi, ai * br);
}

template <int NT>
__global__ __launch_bounds__(64) void k_lowpass_bwd(PskBuffers buf, PskParams p, Iir f) {
  const int lane = threadIdx.x;
  const int64_t w = blockIdx.x;
  const int64_t g = w >> 1, h = w & 1;
  const int64_t n = p.n;
  const int pad = p.pad2;
  const int qs = pad & 1;
  const int64_t m2 = p.m2;
  const int64_t m2_pairs = (m2 + qs + 1) >> 1;
  const double* __restrict__ s3 = buf.s3;
  const int64_t s = g * kWave + h * 32 + (lane >> 1);
  const bool is_re = (lane & 1) == 0;
  const bool writer = is_re && s < buf.n_streams;
  uint32_t* __restrict__ words = buf.words + (size_t)(s < buf.n_streams ? s : 0) * p.n_words;

  double b[NT], a[NT], z[NT - 1];
#pragma unroll
  for (int i = 0; i < NT; ++i) { b[i] = f.b[i]; a[i] = f.a[i]; }
  bool bad = false;

  const double ylast = s3[pair_index(w, m2_pairs, m2 - 1 + qs, lane)];
#pragma unroll
  for (int i = 0; i < NT - 1; ++i) z[i] = f.zi[i] * ylast;
  for (int64_t j = m2 - 1; j >= pad + n; --j) {
    const double y = df2t_lp<NT>(z, b, a, s3[pair_index(w, m2_pairs, j + qs, lane)]);
    bad |= __builtin_amdgcn_class(y, kClsY);
  }

  // symbols k = S-1 .. 0 at baseband index first + k*sps
  int64_t k = p.n_sym - 1;
  int64_t next_n = p.first + k * p.sps;
  double pr = 0.0, pim = 0.0;
  uint32_t acc = 0;

  auto on_output = [&](int64_t i, double y) {
    bad |= __builtin_amdgcn_class(y, kClsY);
    if (i == next_n) {                          // uniform branch
      const double other = __shfl_xor(y, 1);
      const double cr = is_re ? y : other, ci = is_re ? other : y;
      if (k < p.n_sym - 1) {                    // diff index k: s_{k+1} * conj(s_k)
        double dr, di;
        diff_np(pr, pim, cr, ci, dr, di);
        int64_t pos;
        if (p.kind == kQpsk) {
          pos = 2 * k;
          acc |= qpsk_dibit(dr, di) << (30 - (pos & 31));
        } else {
          pos = k;
          acc |= (dr < 0 ? 1u : 0u) << (31 - (pos & 31));
        }
        if ((pos & 31) == 0) {
          if (writer) words[pos >> 5] = acc;
          acc = 0;
        }
      }
      pr = cr; pim = ci;
      --k;
      next_n -= p.sps;
    }
  };

  const int64_t n_main = (n / kChunk) * kChunk;
  const int64_t n_top = n - n_main;
  for (int64_t i = n - 1; i >= n - n_top; --i)
    on_output(i, df2t_lp<NT>(z, b, a, s3[pair_index(w, m2_pairs, pad + i + qs, lane)]));
  {
    const double2* __restrict__ src = reinterpret_cast<const double2*>(s3) + (size_t)w * m2_pairs * kWave + lane;
    double2 nxt[kChunk / 2];
    const int64_t cstart = n_main - kChunk;
    if (n_main > 0) {
#pragma unroll
      for (int kk = 0; kk < kChunk / 2; ++kk) nxt[kk] = src[(size_t)(((pad + qs + cstart) >> 1) + kk) * kWave];
    }
    for (int64_t c = cstart; c >= 0; c -= kChunk) {
      double2 cur[kChunk / 2];
#pragma unroll
      for (int kk = 0; kk < kChunk / 2; ++kk) cur[kk] = nxt[kk];
      if (c >= kChunk) {
        const int64_t qp = (pad + qs + c - kChunk) >> 1;
#pragma unroll
        for (int kk = 0; kk < kChunk / 2; ++kk) nxt[kk] = src[(size_t)(qp + kk) * kWave];
      }
#pragma unroll
      for (int kk = kChunk / 2 - 1; kk >= 0; --kk) {
        on_output(c + 2 * kk + 1, df2t_lp<NT>(z, b, a, cur[kk].y));
        on_output(c + 2 * kk, df2t_lp<NT>(z, b, a, cur[kk].x));
      }
    }
  }
  // left-extension outputs are trimmed but still pass through the detector
  for (int j = pad - 1; j >= 0; --j) {
    const double y = df2t_lp<NT>(z, b, a, s3[pair_index(w, m2_pairs, j + qs, lane)]);
    bad |= __builtin_amdgcn_class(y, kClsY);
  }
  const int fl = bad ? 1 : 0;
  const int other = __shfl_xor(fl, 1);
  if (writer) buf.flags[s] |= (fl | other);
}

// ---------------------------------------------------------------------------
// K3x: exact complex low-pass (scipy CDOUBLE_filt semantics) for flagged
// streams only.  lane = stream; scratch reuses s3 as [group][q][64] double2.
template <int NT>
__device__ __forceinline__ void df2t_cplx_step(double (&zr)[NT - 1], double (&zc)[NT - 1],
                                               const double (&b)[NT], const double (&a)[NT],
                                               double x0, double x1, double& y0, double& y1) {
  const double t0x = 0.0 * x1, t1x = 0.0 * x0;
  y0 = zr[0] + (b[0] * x0 - t0x);
  y1 = zc[0] + (t1x + b[0] * x1);
  const double t0y = 0.0 * y1, t1y = 0.0 * y0;
#pragma unroll
  for (int i = 0; i < NT - 2; ++i) {
    const double r = zr[i + 1] + (b[i + 1] * x0 - t0x);
    const double m = zc[i + 1] + (t1x + b[i + 1] * x1);
    zr[i] = r - (a[i + 1] * y0 - t0y);
    zc[i] = m - (t1y + a[i + 1] * y1);
  }
  zr[NT - 2] = (b[NT - 1] * x0 - t0x) - (a[NT - 1] * y0 - t0y);
  zc[NT - 2] = (t1x + b[NT - 1] * x1) - (t1y + a[NT - 1] * y1);
}

__device__ __forceinline__ void cmul_np(double ar, double ai, double br, double bi, double& re, double& im) {
  re = __builtin_fma(ar, br, -(ai * bi));
  im = __builtin_fma(ar, bi, ai * br);
}

template <int NT>
__global__ __launch_bounds__(64) void k_lowpass_exact(PskBuffers buf, PskParams p, Iir f) {
  const int lane = threadIdx.x;
  const int64_t g = blockIdx.x;
  const int64_t s = g * kWave + lane;
  const bool live = s < buf.n_streams && buf.flags[s] != 0;
  if (!__any(live)) return;                     // wave-uniform early exit (the common case)
  const int64_t n = p.n;
  const int pad = p.pad2;
  const int64_t m2 = p.m2;
  const double2* __restrict__ bb = reinterpret_cast<const double2*>(buf.s2) + (size_t)g * n * kWave + lane;
  double2* __restrict__ sc = reinterpret_cast<double2*>(buf.s3) + (size_t)g * m2 * kWave + lane;
  uint32_t* __restrict__ words = buf.words + (size_t)(s < buf.n_streams ? s : 0) * p.n_words;

  double b[NT], a[NT], zr[NT - 1], zc[NT - 1];
#pragma unroll
  for (int i = 0; i < NT; ++i) { b[i] = f.b[i]; a[i] = f.a[i]; }

  // odd extension with numpy complex ops: (2+0j)*x[0] - x[k]
  const double2 x0 = bb[0], xl = bb[(size_t)(n - 1) * kWave];
  double l2r, l2i, r2r, r2i;
  cmul_np(2.0, 0.0, x0.x, x0.y, l2r, l2i);
  cmul_np(2.0, 0.0, xl.x, xl.y, r2r, r2i);
  auto ext = [&](int64_t j) -> double2 {
    if (j < pad) { const double2 v = bb[(size_t)(pad - j) * kWave]; return make_double2(l2r - v.x, l2i - v.y); }
    if (j < pad + n) return bb[(size_t)(j - pad) * kWave];
    const double2 v = bb[(size_t)(n - 2 - (j - pad - n)) * kWave];
    return make_double2(r2r - v.x, r2i - v.y);
  };
  {
    const double2 e0 = ext(0);
#pragma unroll
    for (int i = 0; i < NT - 1; ++i) cmul_np(f.zi[i], 0.0, e0.x, e0.y, zr[i], zc[i]);
  }
  double y0 = 0, y1 = 0;
  for (int64_t j = 0; j < m2; ++j) {
    const double2 e = ext(j);
    df2t_cplx_step<NT>(zr, zc, b, a, e.x, e.y, y0, y1);
    sc[(size_t)j * kWave] = make_double2(y0, y1);
  }
  __threadfence();
#pragma unroll
  for (int i = 0; i < NT - 1; ++i) cmul_np(f.zi[i], 0.0, y0, y1, zr[i], zc[i]);

  int64_t k = p.n_sym - 1;
  int64_t next_n = p.first + k * p.sps;
  double pr = 0.0, pim = 0.0;
  uint32_t acc = 0;
  for (int64_t j = m2 - 1; j >= 0; --j) {
    const double2 e = sc[(size_t)j * kWave];
    double o0, o1;
    df2t_cplx_step<NT>(zr, zc, b, a, e.x, e.y, o0, o1);
    const int64_t i = j - pad;
    if (i == next_n && k >= 0) {
      if (k < p.n_sym - 1) {
        double dr, di;
        diff_np(pr, pim, o0, o1, dr, di);
        int64_t pos;
        if (p.kind == kQpsk) {
          pos = 2 * k;
          acc |= qpsk_dibit(dr, di) << (30 - (pos & 31));
        } else {
          pos = k;
          acc |= (dr < 0 ? 1u : 0u) << (31 - (pos & 31));
        }
        if ((pos & 31) == 0) {
          if (live) words[pos >> 5] = acc;
          acc = 0;
        }
      }
      pr = o0; pim = o1;
      --k;
      next_n -= p.sps;
    }
  }
}

// ---------------------------------------------------------------------------
// host-side launchers (called from api.cpp)
template <typename T>
static hipError_t launch_bp(int nt, bool zodd, const PskBuffers& b, const PskParams& p, const Iir& f,
                            hipStream_t st, int64_t groups) {
  dim3 grid((unsigned)groups), block(kWave);
  if (nt == 9 && zodd) { hipLaunchKernelGGL((k_bandpass_mix<9, true, T>), grid, block, 0, st, b, p, f); }
  else if (nt == 9) { hipLaunchKernelGGL((k_bandpass_mix<9, false, T>), grid, block, 0, st, b, p, f); }
  else if (nt == 7 && zodd) { hipLaunchKernelGGL((k_bandpass_mix<7, true, T>), grid, block, 0, st, b, p, f); }
  else if (nt == 7) { hipLaunchKernelGGL((k_bandpass_mix<7, false, T>), grid, block, 0, st, b, p, f); }
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_psk_bandpass(const PskBuffers& b, const PskParams& p, const Iir& f, hipStream_t st) {
  const int64_t groups = (b.n_streams + kWave - 1) / kWave;
  switch (b.dtype) {
    case kF32: return launch_bp<float>(f.nt, p.bp_zero_odd != 0, b, p, f, st, groups);
    case kF64: return launch_bp<double>(f.nt, p.bp_zero_odd != 0, b, p, f, st, groups);
    case kI16: return launch_bp<int16_t>(f.nt, p.bp_zero_odd != 0, b, p, f, st, groups);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_psk_lowpass_fwd(const PskBuffers& b, const PskParams& p, const Iir& f, hipStream_t st) {
  const int64_t groups = (b.n_streams + kWave - 1) / kWave;
  if (f.nt != 5) return hipErrorInvalidValue;
  hipLaunchKernelGGL((k_lowpass_fwd<5>), dim3((unsigned)(2 * groups)), dim3(kWave), 0, st, b, p, f);
  return hipGetLastError();
}

hipError_t launch_psk_lowpass_bwd(const PskBuffers& b, const PskParams& p, const Iir& f, hipStream_t st) {
  const int64_t groups = (b.n_streams + kWave - 1) / kWave;
  if (f.nt != 5) return hipErrorInvalidValue;
  hipLaunchKernelGGL((k_lowpass_bwd<5>), dim3((unsigned)(2 * groups)), dim3(kWave), 0, st, b, p, f);
  return hipGetLastError();
}

hipError_t launch_psk_lowpass_exact(const PskBuffers& b, const PskParams& p, const Iir& f, hipStream_t st) {
  const int64_t groups = (b.n_streams + kWave - 1) / kWave;
  if (f.nt != 5) return hipErrorInvalidValue;
  hipLaunchKernelGGL((k_lowpass_exact<5>), dim3((unsigned)groups), dim3(kWave), 0, st, b, p, f);
  return hipGetLastError();
}

}  // namespace amr
