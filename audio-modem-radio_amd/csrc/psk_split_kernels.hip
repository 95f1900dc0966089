// psk_split_kernels.hip -- the PSK time-split (chunk-parallel) layout, for
// one capture or a few: the latency path of the reference's own call pattern
// (filebeep_advanced_v2.py:324, 1112 decode one capture at a time).
//
// qpsk_demodulate / bpsk_demodulate (modem.py:189-266 / 68-135) are four
// serial recurrences per stream -- band-pass filtfilt forward and backward,
// low-pass filtfilt forward and backward (modem.py:194-204) -- so a lone
// stream's serial path is ~4 x 96 000 dependent steps (the row layout:
// 10.5 ms for one 1-s capture).  Here each pass is cut into
// chunks of L outputs, one lane per chunk, and every chunk starts its
// recursion W samples early from a zero state (or, the chunk that holds the
// pass's first sample, from scipy's exact initial state zi * x0).  The
// filters are stable, so after W samples the zero start has decayed below
// the rounding level (W per filter from its impulse responses,
// api.cpp split_design); what remains is a DIFFERENT ROUNDING TRAJECTORY:
// the chunked values differ from the serial ones by rounding noise amplified
// by the filter (a DF-II-T with poles at |z| = 0.989 amplifies its rounding
// by ~1e7).  So the symbols are NOT bit-exact, and the decisions are made
// exact by a margin instead:
//   * every symbol sample's error is below E = kappa * peak|x| (kappa per plan:
//     64 x the L1 noise gain u * sum_i ||g_i||_1 of both filters, which bounds
//     the measured worst error within 1.4x over tones, square waves, noise and
//     modulated signals at 10 parameter sets -- tests/test_gpu_split.py);
//   * a differential product whose decision could move by that much -- QPSK
//     ||di| - |dr|| or BPSK |dr| within sqrt2 E (|s0| + |s1| + E) -- flags its
//     stream (so does exact silence: every zero product is flagged);
//   * a flagged stream's batch is recomputed by the serial row-layout kernels
//     (psk_kernels.hip: bit-exact), launched behind these ones and gated on
//     the flag count on the device (they exit at once when it is zero).
// Unflagged decisions are therefore the reference's, bit for bit.
//
// Kernels (grid.y = stream, lanes = chunks; no LDS, no barriers):
//   KS0 k_split_bp_state_fwd / _bwd (default; AMR_PSK_SPLIT_CONV=0: off): a
//                        wave per chunk computes its band-pass start state by
//                        convolution -> zs [B][c1][8], KS1 / KS2 then run only
//                        their L outputs (no w1-step warm-up)
//   KS1 k_split_bp_fwd   ext(x) -> y1 [B][m1]   (+ the stream's peak |ext x|, the
//                        extension -- from the host's edge table for a raw
//                        integer capture (odd_ext.h) -- included)
//   KS2 k_split_bp_bwd   y1 reversed -> f [B][n]
//   KS3 k_split_lp_fwd   lane = (chunk, component): f * lo, odd ext -> y3 [B][2][m2]
//   KS4 k_split_lp_bwd   y3 reversed -> symbol samples sym [B][S][2]
//   KS5 k_split_slice    thread = (stream, word): numpy's fma differential
//                        product, the sector / sign decision, the margin
//                        check -> words, flag, count
// then k_sync_pack (util_kernels.hip) and the gated serial fallback (api.cpp).
// Each step is the lane kernels' arithmetic (psk_common.h df2t_step /
// bp_step_zo / lp_step), so a chunk's recursion is scipy's operation for
// operation from its start state (oracle/amr_oracle.c oracle_psk_split_symbols
// reproduces these symbols exactly).
#include <math.h>
#include <stdlib.h>

#include "amr_internal.h"
#include "psk_common.h"
#include "split_chain.h"

namespace amr {

template <bool ZO>
__device__ __forceinline__ double split_bp_step(double (&z)[8], const Iir& f, double x) {
  if constexpr (ZO) return bp_step_zo(z, f, x);
  else return df2t_step<8>(z, f, x);
}
template <bool ZO>
__device__ __forceinline__ void split_bp_warm(double (&z)[8], const Iir& f, double x) {
  if constexpr (ZO) (void)bp_warm_zo(z, f, x);
  else (void)bp_warm(z, f, x);
}
template <bool SYM>
__device__ __forceinline__ double split_lp_step(double (&z)[4], const Iir& f, double x) {
  if constexpr (SYM) return lp_step(z, f, x);
  else return df2t_step<4>(z, f, x);
}

// |v| as ordered bits (NaN above inf above every finite value)
__device__ __forceinline__ unsigned long long abs_bits(double v) {
  return (unsigned long long)__double_as_longlong(v) & 0x7fffffffffffffffULL;
}

// KS0 (sp.conv): a band-pass chunk's start state without a warm-up.  The
// state before output o0 of a pass that starts at 0 from zi v0 is
//   Z0[o0] v0 + sum_{m < o0} K[m] v(o0 - 1 - m)
// (K, Z0: the filter's state responses, api.cpp split_state_tables); the
// w1-step warm-up computes the same map truncated at m < w1 (the zero start),
// in w1 dependent steps of one lane.  Here it is a dot product over a whole
// wave: lane l takes m = l (mod 64) in ascending order (FMA), then a
// butterfly sum over the lanes (lane 0's order: ((p0 + p1) + (p2 + p3)) ...;
// oracle/amr_oracle.c conv_state restates it), the Z0 term while o0 <= w1.
// Chunk 0 keeps scipy's zi * v0.  One wave per chunk, four per workgroup
// (split_chain.h split_conv_state).
template <typename T>
__global__ __launch_bounds__(256) void k_split_bp_state_fwd(PskBuffers buf, PskParams p, PskSplit sp) {
  const int64_t s = blockIdx.y;
  const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= sp.c1) return;   // whole waves
  const T* __restrict__ x = reinterpret_cast<const T*>(buf.x) + s * buf.x_stride;
  const int64_t n = p.n;
  const int pad = p.pad1;
  const OddExt<T> ox(x, buf.edge, s, n, pad);
  split_conv_state<8>(
      sp.ktab, sp.z0tab, sp.w1, c * sp.L, ox.left(0),
      [&](int64_t j) -> double {
        if (j < pad) return ox.left(j);
        if (j < pad + n) return In<T>::cvt(x[j - pad]);
        return ox.right(j - pad - n);
      },
      sp.zs + (s * sp.c1 + c) * 8);
}

__global__ __launch_bounds__(256) void k_split_bp_state_bwd(PskBuffers buf, PskParams p, PskSplit sp) {
  const int64_t s = blockIdx.y;
  const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= sp.c1) return;
  const int64_t m1 = p.m1;
  const double* __restrict__ y1 = sp.y1 + s * m1;
  split_conv_state<8>(
      sp.ktab, sp.z0tab, sp.w1, c * sp.L, y1[m1 - 1], [&](int64_t k) { return y1[m1 - 1 - k]; },
      sp.zs + (s * sp.c1 + c) * 8);
}

// KS1: the band-pass's forward pass over ext(x) (odd extension in the input's
// precision, In<T>), outputs [o0, o1) of chunk c
template <typename T, bool ZO>
__global__ __launch_bounds__(64) void k_split_bp_fwd(PskBuffers buf, PskParams p, Iir f, PskSplit sp) {
  const int64_t s = blockIdx.y;
  const int64_t c = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (c >= sp.c1) return;
  const T* __restrict__ x = reinterpret_cast<const T*>(buf.x) + s * buf.x_stride;
  const int64_t n = p.n, m1 = p.m1;
  const int pad = p.pad1;
  const int64_t o0 = c * sp.L, o1 = o0 + sp.L < m1 ? o0 + sp.L : m1;
  const OddExt<T> ox(x, buf.edge, s, n, pad);
  double z[8];
  int64_t j = o0 - sp.w1;
  if (sp.conv) {   // KS0's start state
    j = o0;
    const double* zs = sp.zs + (s * sp.c1 + c) * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) z[i] = zs[i];
  } else if (j <= 0) {
    j = 0;
    const double e0 = ox.left(0);
#pragma unroll
    for (int i = 0; i < 8; ++i) z[i] = f.zi[i] * e0;
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) z[i] = 0.0;
  }
  double* __restrict__ y1 = sp.y1 + s * m1;
  unsigned long long pk = 0;
  auto body = [&](int64_t jj, double e) {
    if (jj < o0) {
      split_bp_warm<ZO>(z, f, e);
    } else {
      y1[jj] = split_bp_step<ZO>(z, f, e);
      const unsigned long long b = abs_bits(e);
      pk = b > pk ? b : pk;
    }
  };
  // head extension, the samples themselves, tail extension
  for (; j < o1 && j < pad; ++j) body(j, ox.left(j));
  const int64_t jm = o1 < pad + n ? o1 : pad + n;
  if (j < jm) {
    split_chain_2(
        j, o0, jm, fwd_blocks(x - pad, [](T v) { return In<T>::cvt(v); }),
        [&](int64_t jj) { return In<T>::cvt(x[jj - pad]); },
        [&](int64_t, double e) { split_bp_warm<ZO>(z, f, e); },
        [&](int64_t jj, double e) {
          y1[jj] = split_bp_step<ZO>(z, f, e);
          const unsigned long long b = abs_bits(e);
          pk = b > pk ? b : pk;
        });
    j = jm;
  }
  for (; j < o1; ++j) body(j, ox.right(j - pad - n));
  atomicMax(&sp.peak[s], pk);
}

// KS2: the band-pass's backward pass (scipy runs lfilter over y1 reversed,
// from zi * y1[-1]); chunk c covers reversed positions [o0, o1), i.e. f[i] for
// i = m1 - 1 - k - pad
template <bool ZO>
__global__ __launch_bounds__(64) void k_split_bp_bwd(PskBuffers buf, PskParams p, Iir f, PskSplit sp) {
  const int64_t s = blockIdx.y;
  const int64_t c = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (c >= sp.c1) return;
  const int64_t n = p.n, m1 = p.m1;
  const int pad = p.pad1;
  const double* __restrict__ y1 = sp.y1 + s * m1;
  double* __restrict__ fo = sp.f + s * n;
  const int64_t o0 = c * sp.L, o1 = o0 + sp.L < m1 ? o0 + sp.L : m1;
  double z[8];
  int64_t k = o0 - sp.w1;
  if (sp.conv) {   // KS0's start state
    k = o0;
    const double* zs = sp.zs + (s * sp.c1 + c) * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) z[i] = zs[i];
  } else if (k <= 0) {
    k = 0;
    const double yl = y1[m1 - 1];
#pragma unroll
    for (int i = 0; i < 8; ++i) z[i] = f.zi[i] * yl;
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) z[i] = 0.0;
  }
  split_chain_2(
      k, o0, o1, bwd_blocks(y1, m1 - 1), [&](int64_t kk) { return y1[m1 - 1 - kk]; },
      [&](int64_t, double v) { split_bp_warm<ZO>(z, f, v); },
      [&](int64_t kk, double v) {
        const double y = split_bp_step<ZO>(z, f, v);
        const int64_t i = m1 - 1 - kk - pad;
        if (i >= 0 && i < n) fo[i] = y;
      });
}

// KS3: the low-pass's forward pass of one component of the baseband
// (f + 0j) * lo (numpy's complex multiply: per component f * lo_c, except
// bb[0], whose addend -(0 * lo_im) / 0 * lo_re the plan's lo table carries --
// as k_lp_lane), odd extension 2 * x0 - x[k] per component
template <bool SYM>
__global__ __launch_bounds__(64) void k_split_lp_fwd(PskBuffers buf, PskParams p, Iir f, PskSplit sp) {
  const int64_t s = blockIdx.y;
  const int64_t q = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (q >= 2 * sp.c2) return;
  const int comp = (int)(q & 1);
  const int64_t c = q >> 1;
  const int64_t n = p.n, m2 = p.m2;
  const int pad = p.pad2;
  const double* __restrict__ fi = sp.f + s * n;
  const double* __restrict__ loc = buf.lo2 + (size_t)comp * n;
  const double* lo4 = buf.lo + 2 * comp;
  auto Xm = [&](int64_t i) { return fi[i] * loc[i]; };
  const double x0 = fi[0] * lo4[0] + lo4[1];
  const double xl = Xm(n - 1);
  const int64_t o0 = c * sp.L, o1 = o0 + sp.L < m2 ? o0 + sp.L : m2;
  double z[4];
  int64_t j = o0 - sp.w2;
  if (j <= 0) {
    j = 0;
    const double e0 = 2.0 * x0 - Xm(pad);
#pragma unroll
    for (int i = 0; i < 4; ++i) z[i] = f.zi[i] * e0;
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) z[i] = 0.0;
  }
  double* __restrict__ y3 = sp.y3 + ((size_t)s * 2 + comp) * m2;
  auto body = [&](int64_t jj, double e) {
    const double y = split_lp_step<SYM>(z, f, e);
    if (jj >= o0) y3[jj] = y;
  };
  for (; j < o1 && j <= pad; ++j) body(j, j < pad ? 2.0 * x0 - Xm(pad - j) : x0);
  const int64_t jm = o1 < pad + n ? o1 : pad + n;
  if (j < jm) {
    split_chain_2(
        j, o0, jm,
        [&](int64_t jj, double (&v)[kSplitRun]) {
          double a[kSplitRun], l[kSplitRun];
          run_load<kSplitRun>(fi + (jj - pad), a);
          run_load<kSplitRun>(loc + (jj - pad), l);
#pragma unroll
          for (int q = 0; q < kSplitRun; ++q) v[q] = a[q] * l[q];
        },
        [&](int64_t jj) { return Xm(jj - pad); },
        [&](int64_t, double e) { (void)split_lp_step<SYM>(z, f, e); },
        [&](int64_t jj, double e) { y3[jj] = split_lp_step<SYM>(z, f, e); });
    j = jm;
  }
  for (; j < o1; ++j) body(j, 2.0 * xl - Xm(n - 2 - (j - pad - n)));
}

// KS4: the low-pass's backward pass; the symbol samples baseband[first::sps]
// (modem.py:92, 209) go to sym [B][S][re, im]
template <bool SYM>
__global__ __launch_bounds__(64) void k_split_lp_bwd(PskBuffers buf, PskParams p, Iir f, PskSplit sp) {
  const int64_t s = blockIdx.y;
  const int64_t q = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (q >= 2 * sp.c2) return;
  const int comp = (int)(q & 1);
  const int64_t c = q >> 1;
  const int64_t n = p.n, m2 = p.m2, S = p.n_sym, first = p.first, sps = p.sps;
  const int pad = p.pad2;
  const double* __restrict__ y3 = sp.y3 + ((size_t)s * 2 + comp) * m2;
  double* __restrict__ so = sp.sym + (size_t)s * S * 2 + comp;
  const int64_t o0 = c * sp.L, o1 = o0 + sp.L < m2 ? o0 + sp.L : m2;
  double z[4];
  int64_t k = o0 - sp.w2;
  if (k <= 0) {
    k = 0;
    const double yl = y3[m2 - 1];
#pragma unroll
    for (int i = 0; i < 4; ++i) z[i] = f.zi[i] * yl;
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) z[i] = 0.0;
  }
  // over the outputs, sample i = m2 - 1 - k - pad falls by one per step:
  // r = (i - first) mod sps counts down to the next symbol sample
  const int64_t i0 = m2 - 1 - (k > o0 ? k : o0) - pad;
  int64_t r = ((i0 - first) % sps + sps) % sps;
  split_chain_2(
      k, o0, o1, bwd_blocks(y3, m2 - 1), [&](int64_t kk) { return y3[m2 - 1 - kk]; },
      [&](int64_t, double v) { (void)split_lp_step<SYM>(z, f, v); },
      [&](int64_t kk, double v) {
        const double y = split_lp_step<SYM>(z, f, v);
        const int64_t i = m2 - 1 - kk - pad;
        if (r == 0 && i >= first && i < n) so[(i - first) / sps * 2] = y;
        r = r == 0 ? sps - 1 : r - 1;
      });
}

// KS5: one thread per (stream, 32-bit word): the differential products of the
// word's symbols in numpy's fma form, the reference's decision (qpsk_dibit /
// real < 0, as K4a), and the margin: |s| <= |s|_1, a symbol's error <= E, so
// |d error|_1 <= sqrt2 E (|s0|_1 + |s1|_1 + E) (+ forming d's own rounding);
// a decision closer than that to its boundary -- QPSK's diagonals
// ||di| - |dr|| (K4a's 2^-29 sliver on top), BPSK's dr = 0 -- flags the stream
__global__ __launch_bounds__(64) void k_split_slice(PskBuffers buf, PskParams p, PskSplit sp) {
  const int64_t s = blockIdx.y;
  const int64_t w = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (w >= p.n_words) return;
  const bool qpsk = p.kind == kQpsk;
  const int per = qpsk ? 16 : 32;
  const int64_t S = p.n_sym;
  const int64_t k0 = w * per;
  const int64_t k1 = k0 + per < S - 1 ? k0 + per : S - 1;
  const double peak = __longlong_as_double((long long)sp.peak[s]);
  const double E = sp.kappa * peak;
  // tiny / huge / non-finite input: every decision goes the serial way
  bool flag = !(peak >= 0x1p-400 && peak <= 0x1p400);
  const double* __restrict__ sy = sp.sym + (size_t)s * S * 2;
  uint32_t word = 0;
  double br = sy[2 * k0], bi0 = sy[2 * k0 + 1];
  for (int64_t k = k0; k < k1; ++k) {
    const double pr = sy[2 * (k + 1)], pim = sy[2 * (k + 1) + 1];
    const double bi = -bi0;
    const double dr = __builtin_fma(pr, br, -(pim * bi));
    const double a0 = fabs(br) + fabs(bi), a1 = fabs(pr) + fabs(pim);
    const double md = 0x1.6a09e667f3bcdp+0 * E * (a0 + a1 + E) * (1.0 + 0x1p-40) + 0x1p-48 * (a0 * a1);
    if (qpsk) {
      const double di = __builtin_fma(pr, bi, pim * br);
      const double adr = fabs(dr), adi = fabs(di);
      if (!(fabs(adi - adr) > md + 0x1p-29 * (adr + adi))) flag = true;
      word |= qpsk_dibit(dr, di) << (30 - 2 * (int)(k & 15));
    } else {
      if (!(fabs(dr) > md)) flag = true;
      word |= (dr < 0 ? 1u : 0u) << (31 - (int)(k & 31));
    }
    br = pr;
    bi0 = pim;
  }
  buf.words[(size_t)s * p.n_words + w] = word;
  if (flag && atomicOr(&sp.flag[s], 1) == 0) atomicAdd(sp.count, 1);
}

// (KS0 +) KS1 + (KS0 +) KS2
hipError_t launch_psk_split_bp(const PskBuffers& b, const PskParams& p, const Iir& bp, const PskSplit& sp,
                               hipStream_t st) {
  const int64_t B = b.n_streams;
  if (B < 1) return hipSuccess;
  if (B > 65535 || bp.nt != 9) return hipErrorInvalidValue;
  const dim3 blk(64), g1((unsigned)((sp.c1 + 63) / 64), (unsigned)B);
  const dim3 blk0(256), g0((unsigned)((sp.c1 + 3) / 4), (unsigned)B);
  const bool zo = p.bp_zero_odd && p.bp_sym;
  if (sp.conv && (!sp.ktab || !sp.z0tab || !sp.zs)) return hipErrorInvalidValue;
  if (sp.conv) {
    switch (b.dtype) {
      case kF32: hipLaunchKernelGGL(k_split_bp_state_fwd<float>, g0, blk0, 0, st, b, p, sp); break;
      case kF64: hipLaunchKernelGGL(k_split_bp_state_fwd<double>, g0, blk0, 0, st, b, p, sp); break;
      case kI16: hipLaunchKernelGGL(k_split_bp_state_fwd<int16_t>, g0, blk0, 0, st, b, p, sp); break;
      default: return hipErrorInvalidValue;
    }
  }
  switch (b.dtype) {
    case kF32:
      if (zo) hipLaunchKernelGGL((k_split_bp_fwd<float, true>), g1, blk, 0, st, b, p, bp, sp);
      else hipLaunchKernelGGL((k_split_bp_fwd<float, false>), g1, blk, 0, st, b, p, bp, sp);
      break;
    case kF64:
      if (zo) hipLaunchKernelGGL((k_split_bp_fwd<double, true>), g1, blk, 0, st, b, p, bp, sp);
      else hipLaunchKernelGGL((k_split_bp_fwd<double, false>), g1, blk, 0, st, b, p, bp, sp);
      break;
    case kI16:
      if (zo) hipLaunchKernelGGL((k_split_bp_fwd<int16_t, true>), g1, blk, 0, st, b, p, bp, sp);
      else hipLaunchKernelGGL((k_split_bp_fwd<int16_t, false>), g1, blk, 0, st, b, p, bp, sp);
      break;
    default:
      return hipErrorInvalidValue;
  }
  if (sp.conv) hipLaunchKernelGGL(k_split_bp_state_bwd, g0, blk0, 0, st, b, p, sp);
  if (zo) hipLaunchKernelGGL((k_split_bp_bwd<true>), g1, blk, 0, st, b, p, bp, sp);
  else hipLaunchKernelGGL((k_split_bp_bwd<false>), g1, blk, 0, st, b, p, bp, sp);
  return hipGetLastError();
}

// KS3 + KS4
hipError_t launch_psk_split_lp(const PskBuffers& b, const PskParams& p, const Iir& lp, const PskSplit& sp,
                               hipStream_t st) {
  const int64_t B = b.n_streams;
  if (B < 1) return hipSuccess;
  if (B > 65535 || lp.nt != 5) return hipErrorInvalidValue;
  const dim3 blk(64), g2((unsigned)((2 * sp.c2 + 63) / 64), (unsigned)B);
  if (p.lp_sym) {
    hipLaunchKernelGGL((k_split_lp_fwd<true>), g2, blk, 0, st, b, p, lp, sp);
    hipLaunchKernelGGL((k_split_lp_bwd<true>), g2, blk, 0, st, b, p, lp, sp);
  } else {
    hipLaunchKernelGGL((k_split_lp_fwd<false>), g2, blk, 0, st, b, p, lp, sp);
    hipLaunchKernelGGL((k_split_lp_bwd<false>), g2, blk, 0, st, b, p, lp, sp);
  }
  return hipGetLastError();
}

// KS5
hipError_t launch_psk_split_slice(const PskBuffers& b, const PskParams& p, const PskSplit& sp, hipStream_t st) {
  const int64_t B = b.n_streams;
  if (B < 1 || p.n_words < 1 || p.n_bits < 1) return hipSuccess;
  if (B > 65535) return hipErrorInvalidValue;
  const dim3 blk(64), g5((unsigned)((p.n_words + 63) / 64), (unsigned)B);
  hipLaunchKernelGGL(k_split_slice, g5, blk, 0, st, b, p, sp);
  return hipGetLastError();
}

}  // namespace amr
