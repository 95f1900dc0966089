// fsk_exact_kernels.hip -- the FSK path's exact fallback for streams with
// digital silence.
//
// Inside a stretch of exact zeros next to signal, both |hilbert| envelopes of
// fsk_demodulate (modem.py:307-315) are FFT rounding noise, so the reference's
// decisions there are whatever pocketfft's rounding makes them.  F1 flags a
// stream whose input holds such a stretch (fsk_kernels.hip, kExactRun); for a
// flagged stream this file recomputes the compare bits the reference's own
// way, bit for bit:
//   * filtfilt in scipy's operation order (DF-II-T without contraction, odd
//     extension in the input's precision -- oracle/amr_oracle.c
//     oracle_filtfilt), both tones;
//   * |scipy.signal.hilbert(f)| as pocketfft + numpy evaluate it: the real
//     forward transform (rfftp passes radf2/3/4/5, last factor first), the
//     conjugate-mirrored spectrum times scipy's h (numpy's FMA complex
//     multiply), the complex backward transform (cfftp passes 8/4/2/3/5),
//     x * 1/n, numpy's complex abs hi * sqrt(fma(r, r, 1)) -- the algorithm
//     oracle/amr_hilbert.c restates and pins against scipy; its twiddle
//     tables come from the host (fsk_api.cpp, the same generator);
//   * bit = env_mark > env_space, written in the final pass's byte layout
//     into a side buffer that F3 (k_fsk_decide) reads instead of the fast
//     path's bytes for a flagged stream.
// One workgroup per flagged stream (its slot of global scratch): every
// workgroup scans the launch's flag words (bit s of word s / 32) and takes
// the flagged streams k with k mod gridDim == blockIdx; the passes run
// across the workgroup with a barrier between passes.  With nothing flagged
// (every noisy capture) the launch reads 4 B per 32 streams.  Only 5-smooth four-step lengths
// (every length the benchmark and the live-column layout plan) take it.
#include "amr_internal.h"
#include "fsk_exact.h"

namespace amr {

template <typename T> struct XIn;
template <> struct XIn<float> {
  static __device__ double cvt(const float* x, int64_t i) { return (double)x[i]; }
  static __device__ double ext(const float* x, int64_t e, int64_t k) { return (double)(2.0f * x[e] - x[k]); }
};
template <> struct XIn<double> {
  static __device__ double cvt(const double* x, int64_t i) { return x[i]; }
  static __device__ double ext(const double* x, int64_t e, int64_t k) { return 2.0 * x[e] - x[k]; }
};
template <> struct XIn<int16_t> {
  static __device__ double cvt(const int16_t* x, int64_t i) { return (double)x[i] / 32768.0; }
  static __device__ double ext(const int16_t* x, int64_t e, int64_t k) { return 2.0 * cvt(x, e) - cvt(x, k); }
};

// ---- the serial filtfilt, scipy's order (one lane per tone) ----------------
// y (m samples, step +-1, in global scratch) is filtered in place.  Blocks of
// kDfBlock samples: the next block's loads are issued before this block's
// recursion, so the serial chain waits on FP64 latency, not on memory.
constexpr int kDfBlock = 16;
__device__ __forceinline__ double df2t_step(const double* b, const double* a, double* z, double xn) {
  const double yn = z[0] + b[0] * xn;
  for (int i = 0; i < 5; ++i) z[i] = z[i + 1] + xn * b[i + 1] - yn * a[i + 1];
  z[5] = xn * b[6] - yn * a[6];
  return yn;
}
__device__ void df2t_exact(const double* b, const double* a, double* z, double* y, int64_t m, int64_t step) {
  const int64_t nblk = m / kDfBlock;
  double cur[kDfBlock], nxt[kDfBlock];
  if (nblk > 0)
#pragma unroll
    for (int j = 0; j < kDfBlock; ++j) cur[j] = y[j * step];
  for (int64_t blk = 0; blk < nblk; ++blk) {
    const int64_t k0 = blk * kDfBlock;
    if (blk + 1 < nblk)
#pragma unroll
      for (int j = 0; j < kDfBlock; ++j) nxt[j] = y[(k0 + kDfBlock + j) * step];
#pragma unroll
    for (int j = 0; j < kDfBlock; ++j) cur[j] = df2t_step(b, a, z, cur[j]);
#pragma unroll
    for (int j = 0; j < kDfBlock; ++j) y[(k0 + j) * step] = cur[j];
#pragma unroll
    for (int j = 0; j < kDfBlock; ++j) cur[j] = nxt[j];
  }
  for (int64_t k = nblk * kDfBlock; k < m; ++k) y[k * step] = df2t_step(b, a, z, y[k * step]);
}

// ---- pocketfft passes over global scratch, spread across the workgroup ----
struct Cx { double r, i; };
__device__ __forceinline__ Cx cadd(Cx a, Cx b) { return {a.r + b.r, a.i + b.i}; }
__device__ __forceinline__ Cx csub(Cx a, Cx b) { return {a.r - b.r, a.i - b.i}; }
__device__ __forceinline__ Cx smulb(Cx v, Cx w) { return {v.r * w.r - v.i * w.i, v.r * w.i + v.i * w.r}; }
__device__ __forceinline__ Cx rot90b(Cx a) { return {-a.i, a.r}; }
__device__ __forceinline__ Cx rot45b(Cx a) {
  const double h = 0.707106781186547524400844362104849;
  return {h * (a.r - a.i), h * (a.i + a.r)};
}
__device__ __forceinline__ Cx rot135b(Cx a) {
  const double h = 0.707106781186547524400844362104849;
  return {h * (-a.r - a.i), h * (a.r - a.i)};
}

#define CC(a, b, c) cc[(a) + ido * ((b) + l1 * (c))]
#define WA(x, i) wa[(i) + (x) * (ido - 1)]

__device__ void radf2(int64_t ido, int64_t l1, const double* cc, double* ch, const double* wa) {
#define CH(a, b, c) ch[(a) + ido * ((b) + 2 * (c))]
  for (int64_t k = threadIdx.x; k < l1; k += blockDim.x) {
    CH(0, 0, k) = CC(0, k, 0) + CC(0, k, 1);
    CH(ido - 1, 1, k) = CC(0, k, 0) - CC(0, k, 1);
    if ((ido & 1) == 0) {
      CH(0, 1, k) = -CC(ido - 1, k, 1);
      CH(ido - 1, 0, k) = CC(ido - 1, k, 0);
    }
  }
  if (ido <= 2) return;
  const int64_t hi = (ido - 1) / 2;
  for (int64_t t = threadIdx.x; t < l1 * hi; t += blockDim.x) {
    const int64_t k = t / hi, i = 2 + 2 * (t - k * hi), ic = ido - i;
    const double tr2 = wa[i - 2] * CC(i - 1, k, 1) + wa[i - 1] * CC(i, k, 1);
    const double ti2 = wa[i - 2] * CC(i, k, 1) - wa[i - 1] * CC(i - 1, k, 1);
    CH(i - 1, 0, k) = CC(i - 1, k, 0) + tr2;
    CH(ic - 1, 1, k) = CC(i - 1, k, 0) - tr2;
    CH(i, 0, k) = ti2 + CC(i, k, 0);
    CH(ic, 1, k) = ti2 - CC(i, k, 0);
  }
#undef CH
}

__device__ void radf3(int64_t ido, int64_t l1, const double* cc, double* ch, const double* wa) {
  const double taur = -0.5, taui = 0.8660254037844386467637231707529362;
#define CH(a, b, c) ch[(a) + ido * ((b) + 3 * (c))]
  for (int64_t k = threadIdx.x; k < l1; k += blockDim.x) {
    const double cr2 = CC(0, k, 1) + CC(0, k, 2);
    CH(0, 0, k) = CC(0, k, 0) + cr2;
    CH(0, 2, k) = taui * (CC(0, k, 2) - CC(0, k, 1));
    CH(ido - 1, 1, k) = CC(0, k, 0) + taur * cr2;
  }
  if (ido == 1) return;
  const int64_t hi = (ido - 1) / 2;
  for (int64_t t = threadIdx.x; t < l1 * hi; t += blockDim.x) {
    const int64_t k = t / hi, i = 2 + 2 * (t - k * hi), ic = ido - i;
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

__device__ void radf4(int64_t ido, int64_t l1, const double* cc, double* ch, const double* wa) {
  const double hsqt2 = 0.707106781186547524400844362104849;
#define CH(a, b, c) ch[(a) + ido * ((b) + 4 * (c))]
  for (int64_t k = threadIdx.x; k < l1; k += blockDim.x) {
    const double tr1 = CC(0, k, 3) + CC(0, k, 1);
    CH(0, 2, k) = CC(0, k, 3) - CC(0, k, 1);
    const double tr2 = CC(0, k, 0) + CC(0, k, 2);
    CH(ido - 1, 1, k) = CC(0, k, 0) - CC(0, k, 2);
    CH(0, 0, k) = tr2 + tr1;
    CH(ido - 1, 3, k) = tr2 - tr1;
    if ((ido & 1) == 0) {
      const double ti1 = -hsqt2 * (CC(ido - 1, k, 1) + CC(ido - 1, k, 3));
      const double tr1b = hsqt2 * (CC(ido - 1, k, 1) - CC(ido - 1, k, 3));
      CH(ido - 1, 0, k) = CC(ido - 1, k, 0) + tr1b;
      CH(ido - 1, 2, k) = CC(ido - 1, k, 0) - tr1b;
      CH(0, 3, k) = ti1 + CC(ido - 1, k, 2);
      CH(0, 1, k) = ti1 - CC(ido - 1, k, 2);
    }
  }
  if (ido <= 2) return;
  const int64_t hi = (ido - 1) / 2;
  for (int64_t t = threadIdx.x; t < l1 * hi; t += blockDim.x) {
    const int64_t k = t / hi, i = 2 + 2 * (t - k * hi), ic = ido - i;
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

__device__ void radf5(int64_t ido, int64_t l1, const double* cc, double* ch, const double* wa) {
  const double tr11 = 0.3090169943749474241022934171828191, ti11 = 0.9510565162951535721164393333793821;
  const double tr12 = -0.8090169943749474241022934171828191, ti12 = 0.5877852522924731291687059546390728;
#define CH(a, b, c) ch[(a) + ido * ((b) + 5 * (c))]
  for (int64_t k = threadIdx.x; k < l1; k += blockDim.x) {
    const double cr2 = CC(0, k, 4) + CC(0, k, 1), ci5 = CC(0, k, 4) - CC(0, k, 1);
    const double cr3 = CC(0, k, 3) + CC(0, k, 2), ci4 = CC(0, k, 3) - CC(0, k, 2);
    CH(0, 0, k) = CC(0, k, 0) + cr2 + cr3;
    CH(ido - 1, 1, k) = CC(0, k, 0) + tr11 * cr2 + tr12 * cr3;
    CH(0, 2, k) = ti11 * ci5 + ti12 * ci4;
    CH(ido - 1, 3, k) = CC(0, k, 0) + tr12 * cr2 + tr11 * cr3;
    CH(0, 4, k) = ti12 * ci5 - ti11 * ci4;
  }
  if (ido == 1) return;
  const int64_t hi = (ido - 1) / 2;
  for (int64_t t = threadIdx.x; t < l1 * hi; t += blockDim.x) {
    const int64_t k = t / hi, i = 2 + 2 * (t - k * hi), ic = ido - i;
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

// complex backward passes: butterfly (k, i) per thread
#define CC(a, b, c) cc[(a) + ido * ((b) + IP * (c))]
#define CH(a, b, c) ch[(a) + ido * ((b) + l1 * (c))]
#define WA(x, i) wa[(i) - 1 + (x) * (ido - 1)]
template <int IP>
__device__ void cpass(int64_t ido, int64_t l1, const Cx* cc, Cx* ch, const Cx* wa) {
  for (int64_t t = threadIdx.x; t < l1 * ido; t += blockDim.x) {
    const int64_t k = t / ido, i = t - k * ido;
    if constexpr (IP == 2) {
      CH(i, k, 0) = cadd(CC(i, 0, k), CC(i, 1, k));
      const Cx d = csub(CC(i, 0, k), CC(i, 1, k));
      CH(i, k, 1) = i == 0 ? d : smulb(d, WA(0, i));
    } else if constexpr (IP == 3) {
      const double tw1r = -0.5, tw1i = 0.8660254037844386467637231707529362;
      const Cx t0 = CC(i, 0, k), t1 = cadd(CC(i, 1, k), CC(i, 2, k)), t2 = csub(CC(i, 1, k), CC(i, 2, k));
      CH(i, k, 0) = cadd(t0, t1);
      const Cx ca = {t0.r + t1.r * tw1r, t0.i + t1.i * tw1r};
      const Cx cb = {-(t2.i * tw1i), t2.r * tw1i};
      if (i == 0) {
        CH(0, k, 1) = cadd(ca, cb);
        CH(0, k, 2) = csub(ca, cb);
      } else {
        CH(i, k, 1) = smulb(cadd(ca, cb), WA(0, i));
        CH(i, k, 2) = smulb(csub(ca, cb), WA(1, i));
      }
    } else if constexpr (IP == 4) {
      const Cx t2 = cadd(CC(i, 0, k), CC(i, 2, k)), t1 = csub(CC(i, 0, k), CC(i, 2, k));
      const Cx t3 = cadd(CC(i, 1, k), CC(i, 3, k)), t4 = rot90b(csub(CC(i, 1, k), CC(i, 3, k)));
      if (i == 0) {
        CH(0, k, 0) = cadd(t2, t3);
        CH(0, k, 2) = csub(t2, t3);
        CH(0, k, 1) = cadd(t1, t4);
        CH(0, k, 3) = csub(t1, t4);
      } else {
        CH(i, k, 0) = cadd(t2, t3);
        CH(i, k, 1) = smulb(cadd(t1, t4), WA(0, i));
        CH(i, k, 2) = smulb(csub(t2, t3), WA(1, i));
        CH(i, k, 3) = smulb(csub(t1, t4), WA(2, i));
      }
    } else if constexpr (IP == 5) {
      const double tw1r = 0.3090169943749474241022934171828191, tw1i = 0.9510565162951535721164393333793821;
      const double tw2r = -0.8090169943749474241022934171828191, tw2i = 0.5877852522924731291687059546390728;
      const Cx t0 = CC(i, 0, k);
      const Cx t1 = cadd(CC(i, 1, k), CC(i, 4, k)), t4 = csub(CC(i, 1, k), CC(i, 4, k));
      const Cx t2 = cadd(CC(i, 2, k), CC(i, 3, k)), t3 = csub(CC(i, 2, k), CC(i, 3, k));
      CH(i, k, 0) = {t0.r + t1.r + t2.r, t0.i + t1.i + t2.i};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int u1 = s ? 2 : 1, u2 = s ? 3 : 4;
        const double twar = s ? tw2r : tw1r, twbr = s ? tw1r : tw2r;
        const double twai = s ? tw2i : tw1i, twbi = s ? -tw1i : tw2i;
        const Cx ca = {t0.r + twar * t1.r + twbr * t2.r, t0.i + twar * t1.i + twbr * t2.i};
        const Cx cb = {-(twai * t4.i + twbi * t3.i), twai * t4.r + twbi * t3.r};
        if (i == 0) {
          CH(0, k, u1) = cadd(ca, cb);
          CH(0, k, u2) = csub(ca, cb);
        } else {
          CH(i, k, u1) = smulb(cadd(ca, cb), WA(u1 - 1, i));
          CH(i, k, u2) = smulb(csub(ca, cb), WA(u2 - 1, i));
        }
      }
    } else {   // IP == 8
      Cx a1 = cadd(CC(i, 1, k), CC(i, 5, k)), a5 = csub(CC(i, 1, k), CC(i, 5, k));
      Cx a3 = cadd(CC(i, 3, k), CC(i, 7, k)), a7 = csub(CC(i, 3, k), CC(i, 7, k));
      Cx u = a1;
      a1 = cadd(u, a3);
      a3 = rot90b(csub(u, a3));
      a7 = rot90b(a7);
      u = a5;
      a5 = rot45b(cadd(u, a7));
      a7 = rot135b(csub(u, a7));
      Cx a0 = cadd(CC(i, 0, k), CC(i, 4, k)), a4 = csub(CC(i, 0, k), CC(i, 4, k));
      Cx a2 = cadd(CC(i, 2, k), CC(i, 6, k)), a6 = csub(CC(i, 2, k), CC(i, 6, k));
      if (i == 0) {
        const Cx s02 = cadd(a0, a2), d02 = csub(a0, a2);
        CH(0, k, 0) = cadd(s02, a1);
        CH(0, k, 4) = csub(s02, a1);
        CH(0, k, 2) = cadd(d02, a3);
        CH(0, k, 6) = csub(d02, a3);
        a6 = rot90b(a6);
        const Cx s46 = cadd(a4, a6), d46 = csub(a4, a6);
        CH(0, k, 1) = cadd(s46, a5);
        CH(0, k, 5) = csub(s46, a5);
        CH(0, k, 3) = cadd(d46, a7);
        CH(0, k, 7) = csub(d46, a7);
      } else {
        u = a0;
        a0 = cadd(u, a2);
        a2 = csub(u, a2);
        CH(i, k, 0) = cadd(a0, a1);
        CH(i, k, 4) = smulb(csub(a0, a1), WA(3, i));
        CH(i, k, 2) = smulb(cadd(a2, a3), WA(1, i));
        CH(i, k, 6) = smulb(csub(a2, a3), WA(5, i));
        a6 = rot90b(a6);
        u = a4;
        a4 = cadd(u, a6);
        a6 = csub(u, a6);
        CH(i, k, 1) = smulb(cadd(a4, a5), WA(0, i));
        CH(i, k, 5) = smulb(csub(a4, a5), WA(4, i));
        CH(i, k, 3) = smulb(cadd(a6, a7), WA(2, i));
        CH(i, k, 7) = smulb(csub(a6, a7), WA(6, i));
      }
    }
  }
}
#undef CC
#undef CH
#undef WA

// |hilbert(f)| of one real row f (n) into env; r1, r2: n doubles; c1, c2: n complex
__device__ void exact_env(const ExactFft& X, const double* f, double* r1, double* r2, Cx* c1, Cx* c2, double* env) {
  const int64_t n = X.n;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) r1[i] = f[i];
  __syncthreads();
  double *p1 = r1, *p2 = r2;
  int64_t l1 = n;
  for (int k1 = 0; k1 < X.nr; ++k1) {
    const int k = X.nr - k1 - 1;
    const int ip = X.fr[k];
    const int64_t ido = n / l1;
    l1 /= ip;
    const double* wa = X.rtw + X.rto[k];
    if (ip == 4) radf4(ido, l1, p1, p2, wa);
    else if (ip == 2) radf2(ido, l1, p1, p2, wa);
    else if (ip == 3) radf3(ido, l1, p1, p2, wa);
    else radf5(ido, l1, p1, p2, wa);
    __syncthreads();
    double* t = p1;
    p1 = p2;
    p2 = t;
  }
  // halfcomplex -> conjugate-mirrored spectrum, times h (numpy's FMA complex multiply)
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    double xr, xi;
    if (i == 0) { xr = p1[0]; xi = 0.0; }
    else if (2 * i == n) { xr = p1[n - 1]; xi = 0.0; }
    else if (2 * i < n) { xr = p1[2 * i - 1]; xi = p1[2 * i]; }
    else { xr = p1[2 * (n - i) - 1]; xi = -p1[2 * (n - i)]; }
    const double hr = (i == 0 || 2 * i == n) ? 1.0 : (2 * i < n ? 2.0 : 0.0), hi = 0.0;
    c1[i] = {__builtin_fma(xr, hr, -(xi * hi)), __builtin_fma(xr, hi, xi * hr)};
  }
  __syncthreads();
  Cx *q1 = c1, *q2 = c2;
  l1 = 1;
  for (int k = 0; k < X.nc; ++k) {
    const int ip = X.fc[k];
    const int64_t ido = n / (l1 * ip);
    const Cx* wa = reinterpret_cast<const Cx*>(X.ctw) + X.cto[k];
    switch (ip) {
      case 2: cpass<2>(ido, l1, q1, q2, wa); break;
      case 3: cpass<3>(ido, l1, q1, q2, wa); break;
      case 4: cpass<4>(ido, l1, q1, q2, wa); break;
      case 5: cpass<5>(ido, l1, q1, q2, wa); break;
      default: cpass<8>(ido, l1, q1, q2, wa); break;
    }
    __syncthreads();
    Cx* t = q1;
    q1 = q2;
    q2 = t;
    l1 *= ip;
  }
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const double re = q1[i].r * X.fct, im = q1[i].i * X.fct;
    const double ar = fabs(re), ai = fabs(im);
    const double h = ar > ai ? ar : ai, l = ar > ai ? ai : ar;
    env[i] = h == 0.0 ? 0.0 : h * __builtin_sqrt(__builtin_fma(l / h, l / h, 1.0));
  }
  __syncthreads();
}

constexpr int kExactThreads = 512;    // the envelope passes are latency-bound: 8 waves in flight

// The flagged streams of this launch's [s0, s0 + nb), in groups of G <= group
// per workgroup and round (G = the flagged count spread over the grid): the
// group's odd extensions, then its filtfilts one lane per (stream, tone) in
// wave 0 (the serial recursion is instruction-issue bound, so 64 lanes cost
// what 2 do), then per stream the exact envelopes with the whole workgroup
// and the compare bits in the final pass's byte layout -> xbits.
// Slot (blockIdx.x): r1, r2 (n), c1, c2 (n complex), e0, e1 (n), y[group][2][m].
template <typename T>
__global__ __launch_bounds__(kExactThreads) void k_fsk_exact(const void* xv, int64_t x_stride, int64_t s0, int64_t nb,
                                                   const uint32_t* __restrict__ flags, int group,
                                                   double* __restrict__ slots, int64_t slot_doubles,
                                                   uint8_t* __restrict__ xbits, FskParams p, FskIir f, ExactFft X) {
  const int64_t n = p.n;
  const int pad = p.pad;
  const int64_t m = n + 2 * (int64_t)pad;
  double* sl = slots + (size_t)blockIdx.x * slot_doubles;
  double* r1 = sl;
  double* r2 = r1 + n;
  Cx* c1 = reinterpret_cast<Cx*>(r2 + n);
  Cx* c2 = c1 + n;
  double* e0 = reinterpret_cast<double*>(c2 + n);
  double* e1 = e0 + n;
  double* yall = e1 + n;           // [group][2][m] extended signal / filter outputs
  __shared__ uint32_t words_sh[kExactThreads];
  __shared__ int32_t sel_sh[32];
  __shared__ int64_t total_sh;
  __shared__ int nsel_sh;
  const int64_t nw = (nb + 31) / 32;
  if (threadIdx.x == 0) total_sh = 0;
  __syncthreads();
  for (int64_t i = threadIdx.x; i < nw; i += blockDim.x) {
    const uint32_t wd = flags[i];
    if (wd) atomicAdd(reinterpret_cast<unsigned long long*>(&total_sh), (unsigned long long)__popc(wd));
  }
  __syncthreads();
  const int64_t total = total_sh;
  if (total == 0) return;
  const int64_t G = min((int64_t)group, (total + gridDim.x - 1) / gridDim.x);
  for (int64_t lo = (int64_t)blockIdx.x * G; lo < total; lo += (int64_t)gridDim.x * G) {
    const int64_t hi = min(lo + G, total);
    // the flagged streams of ordinals [lo, hi) -> sel_sh (thread 0 walks the words)
    int64_t seen = 0;
    if (threadIdx.x == 0) nsel_sh = 0;
    for (int64_t base = 0; base < nw; base += kExactThreads) {
      __syncthreads();
      words_sh[threadIdx.x] = base + threadIdx.x < nw ? flags[base + threadIdx.x] : 0u;
      __syncthreads();
      if (threadIdx.x == 0)
        for (int t = 0; t < kExactThreads && seen < hi; ++t) {
          uint32_t mm = words_sh[t];
          const int c = __popc(mm);
          if (seen + c <= lo) { seen += c; continue; }
          while (mm) {
            const int bit = __builtin_ctz(mm);
            mm &= mm - 1;
            if (seen >= lo && seen < hi) sel_sh[nsel_sh++] = (int32_t)((base + t) * 32 + bit);
            ++seen;
          }
        }
    }
    __syncthreads();
    const int gn = nsel_sh;
    // the odd extensions, in the input's precision (numpy's odd_ext)
    for (int g = 0; g < gn; ++g) {
      const T* x = reinterpret_cast<const T*>(xv) + (size_t)sel_sh[g] * x_stride;
      double* y0 = yall + (size_t)g * 2 * m;
      for (int64_t j = threadIdx.x; j < m; j += blockDim.x) {
        double v;
        if (j >= pad && j < pad + n) v = XIn<T>::cvt(x, j - pad);
        else if (j < pad) v = XIn<T>::ext(x, 0, pad - j);
        else v = XIn<T>::ext(x, n - 1, n - 2 - (j - pad - n));
        y0[j] = v;
        y0[m + j] = v;
      }
    }
    __syncthreads();
    if ((int)threadIdx.x < 2 * gn) {
      const int tone = threadIdx.x & 1;
      double* y = yall + (size_t)(threadIdx.x >> 1) * 2 * m + (size_t)tone * m;
      double b[7], a[7], z[6];
      for (int i = 0; i < 7; ++i) { b[i] = f.b[tone][i]; a[i] = f.a[tone][i]; }
      for (int i = 0; i < 6; ++i) z[i] = f.zi[tone][i] * y[0];
      df2t_exact(b, a, z, y, m, 1);
      for (int i = 0; i < 6; ++i) z[i] = f.zi[tone][i] * y[m - 1];
      df2t_exact(b, a, z, y + m - 1, m, -1);
    }
    __syncthreads();
    for (int g = 0; g < gn; ++g) {
      const double* y0 = yall + (size_t)g * 2 * m;
      exact_env(X, y0 + pad, r1, r2, c1, c2, e0);
      exact_env(X, y0 + m + pad, r1, r2, c1, c2, e1);
      // bits: byte (c0 / 8) * n2 + kk holds columns c0 .. c0 + 7 of row kk
      // (column c -> sample col(c) + n1 * kk; col = the live columns or all)
      const int ncol = p.lc.on ? p.lc.nl : (int)p.rn1;
      const int64_t n2 = p.rn2, n1 = p.lc.on ? p.lc.n1 : p.rn1;
      const int64_t nbytes = (int64_t)((ncol + 7) >> 3) * n2;
      uint8_t* ob = xbits + (size_t)(s0 + sel_sh[g]) * p.bits_stride;
      for (int64_t q = threadIdx.x; q < nbytes; q += blockDim.x) {
        const int64_t cb = q / n2, kk = q - cb * n2;
        unsigned byte = 0;
        for (int t = 0; t < 8; ++t) {
          const int c = (int)cb * 8 + t;
          if (c >= ncol) break;
          const int64_t col = p.lc.on ? lc_live_col(p.lc, c) : c;
          const int64_t i = col + n1 * kk;
          if (i < n && e0[i] > e1[i]) byte |= 1u << t;
        }
        ob[q] = (uint8_t)byte;
      }
      __syncthreads();
    }
  }
}

hipError_t launch_fsk_exact(int dtype, const void* x, int64_t x_stride, int64_t s0, int64_t nb, const uint32_t* flags,
                            int group, double* slots, int64_t slot_doubles, int n_slots, uint8_t* xbits,
                            const FskParams& p, const FskIir& f, const ExactFft& X, hipStream_t st) {
  switch (dtype) {
    case kF32: hipLaunchKernelGGL(k_fsk_exact<float>, dim3(n_slots), dim3(kExactThreads), 0, st, x, x_stride, s0, nb, flags, group, slots, slot_doubles, xbits, p, f, X); break;
    case kF64: hipLaunchKernelGGL(k_fsk_exact<double>, dim3(n_slots), dim3(kExactThreads), 0, st, x, x_stride, s0, nb, flags, group, slots, slot_doubles, xbits, p, f, X); break;
    case kI16: hipLaunchKernelGGL(k_fsk_exact<int16_t>, dim3(n_slots), dim3(kExactThreads), 0, st, x, x_stride, s0, nb, flags, group, slots, slot_doubles, xbits, p, f, X); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace amr
