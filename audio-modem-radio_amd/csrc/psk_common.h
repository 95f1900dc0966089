// psk_common.h -- device helpers shared by the PSK kernel files
// (psk_kernels.hip: the state-per-lane kernels; psk_lane_kernels.hip: the
// lane-per-stream throughput kernels).  Both must evaluate the reference's
// arithmetic identically, so the conversions, layouts and the
// low-pass zero detector live here once.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "amr_internal.h"
#include "odd_ext.h"

namespace amr {

// input conversion + odd extension (In<T>, OddExt<T>): odd_ext.h

// class masks for __builtin_amdgcn_class (v_cmp_class_f64)
// bit: 0 sNaN 1 qNaN 2 -inf 3 -norm 4 -denorm 5 -0 6 +0 7 +denorm 8 +norm 9 +inf
constexpr int kClsX = 0x2B7;   // low-pass INPUT not provably safe: NaN, inf, denormal, -0
constexpr int kClsY = 0x2F7;   // low-pass OUTPUT not provably safe: the above and +0

// s2 (band-pass output f): [group][half][n2][32 streams][2 samples] doubles,
// so that a low-pass wave (one half-group) streams one 512 B row per 2 samples.
__device__ __forceinline__ size_t f_index(int64_t g, int64_t n2, int64_t i, int s_in_group) {
  const int h = s_in_group >> 5, sl = s_in_group & 31;
  return ((size_t)((g * 2 + h) * n2 + (i >> 1)) * 32 + sl) * 2 + (i & 1);
}

typedef unsigned v4u __attribute__((ext_vector_type(4)));   // native vector: SROA-friendly (HIP's uint4 is a struct)
typedef unsigned v2u __attribute__((ext_vector_type(2)));

// symbol buffer: [stream][symbol][re, im] doubles
// symbol samples [B/64][re, im][S][64]: a component's symbol k of 64
// streams is one 512-B line, written whole by the wave that computes it
// (the earlier [B/32][S][32][re, im] interleave left each store half a line
// and cost the lane low-pass ~15 % in flight); symbol k+1 is 64 doubles on.
__device__ __forceinline__ size_t sym_index(int64_t s, int64_t n_sym, int64_t k, int comp) {
  return ((size_t)((s >> 6) * 2 + comp) * (size_t)n_sym + (size_t)k) * 64 + (size_t)(s & 63);
}

typedef __attribute__((address_space(4))) const double CDouble;   // constant AS: uniform loads -> SMEM
constexpr float kTinyHi = 0x1p-126f;            // FLT_MIN

__device__ __forceinline__ float tiny_min3(float acc, double a, double b) {
  const float ha = __builtin_bit_cast(float, (unsigned)(__builtin_bit_cast(unsigned long long, a) >> 32));
  const float hb = __builtin_bit_cast(float, (unsigned)(__builtin_bit_cast(unsigned long long, b) >> 32));
  float r;
  asm("v_min3_f32 %0, %1, |%2|, |%3|" : "=v"(r) : "v"(acc), "v"(ha), "v"(hb));
  return r;
}


// ---- DF-II-T steps with all states of one stream in one lane (the lane
// kernels psk_lane_kernels.hip and the time-split kernels psk_split_kernels.hip)
// scipy lfilter's DF-II-T step with all states of one stream in one lane:
//   y = z0 + b0*x ;  z[j] = (z[j+1] + x*b[j+1]) - y*a[j+1] ;  z[last] = x*b[last] - y*a[last]
// (z[last] of the row kernels is (-0.0 + x*b) - y*a: -0.0 is the additive
// identity for every double, NaN included, so the forms agree bit for bit)
template <int NS>
__device__ __forceinline__ double df2t_step(double (&z)[NS], const Iir& f, double x) {
  const double y = z[0] + f.b[0] * x;
#pragma unroll
  for (int j = 0; j < NS - 1; ++j) z[j] = (z[j + 1] + x * f.b[j + 1]) - y * f.a[j + 1];
  z[NS - 1] = x * f.b[NS] - y * f.a[NS];
  return y;
}

// The band-pass's odd taps b1, b3, b5, b7 are exactly +0.0 (butter(4, band);
// the plan checks, PskParams::bp_zero_odd).  The step without them --
// z[i] = z[i+1] - y*a[i+1] for even i -- is scipy's bit for bit whenever
// z[i+1] + x*(+0.0) == z[i+1], i.e. unless z[i+1] is -0.0 (or x is inf / NaN,
// which makes the final states non-finite).  The detector keeps the minimum
// |hi word| (as float) of z1, z3, z5, z7 before every step: >= FLT_MIN means
// |z| >= 2^-1015, never a zero; a stream that fails, or ends non-finite, is
// flagged and its group re-run with every tap (k_bp_lane2's FIXUP form).
// 26 instead of 34 FP64 per step, + 2 v_min3_f32.
// The numerator is also palindromic (b8 == b0, b6 == b2 bit for bit,
// PskParams::bp_sym), so x*b8 IS x*b0 and x*b6 IS x*b2: 3 products, not 5.
// 23 FP64 per step instead of 34.
__device__ __forceinline__ double df2t_step_zo(double (&z)[8], const Iir& f, double x, float& acc) {
  acc = tiny_min3(acc, z[1], z[3]);
  acc = tiny_min3(acc, z[5], z[7]);
  const double p0 = f.b[0] * x, p2 = x * f.b[2], p4 = x * f.b[4];
  const double y = z[0] + p0;
  z[0] = z[1] - y * f.a[1];
  z[1] = (z[2] + p2) - y * f.a[2];
  z[2] = z[3] - y * f.a[3];
  z[3] = (z[4] + p4) - y * f.a[4];
  z[4] = z[5] - y * f.a[5];
  z[5] = (z[6] + p2) - y * f.a[6];
  z[6] = z[7] - y * f.a[7];
  z[7] = p0 - y * f.a[8];
  return y;
}

// The low-pass numerator k*[1,4,6,4,1] is palindromic (PskParams::lp_sym,
// required for the lane layout): x*b4 IS x*b0 and x*b3 IS x*b1.  15 FP64
// per step instead of 17, each result identical to df2t_step<4>.
__device__ __forceinline__ double lp_step(double (&z)[4], const Iir& f, double x) {
  const double p0 = f.b[0] * x, p1 = x * f.b[1], p2 = x * f.b[2];
  const double y = z[0] + p0;
  z[0] = (z[1] + p1) - y * f.a[1];
  z[1] = (z[2] + p2) - y * f.a[2];
  z[2] = (z[3] + p1) - y * f.a[3];
  z[3] = p0 - y * f.a[4];
  return y;
}

// df2t_step_zo without the zero-state detector: the time-split kernels
// (psk_split_kernels.hip) decide by margins, where the sign of an exact zero
// state -- all the skipped +0.0 taps can change -- moves no decision
// The time-split band-pass's WARM-UP steps (psk_split_kernels.hip: a chunk's
// recursion before its first output): not scipy's order -- only the state
// they leave matters, and it differs from the serial one by rounding either
// way -- so each tap is one FMA, 13 operations per step with
// the zero odd taps (bp_warm_zo) or 17 (bp_warm), against 23 / 33.
// oracle/amr_oracle.c chunked_pass restates it (its generic form, with
// fma(0, x, z) = z for the zero taps).
__device__ __forceinline__ double bp_warm_zo(double (&z)[8], const Iir& f, double x) {
  const double y = __builtin_fma(f.b[0], x, z[0]);
  z[0] = __builtin_fma(-f.a[1], y, z[1]);
  z[1] = __builtin_fma(-f.a[2], y, __builtin_fma(f.b[2], x, z[2]));
  z[2] = __builtin_fma(-f.a[3], y, z[3]);
  z[3] = __builtin_fma(-f.a[4], y, __builtin_fma(f.b[4], x, z[4]));
  z[4] = __builtin_fma(-f.a[5], y, z[5]);
  z[5] = __builtin_fma(-f.a[6], y, __builtin_fma(f.b[6], x, z[6]));
  z[6] = __builtin_fma(-f.a[7], y, z[7]);
  z[7] = __builtin_fma(-f.a[8], y, f.b[8] * x);
  return y;
}
__device__ __forceinline__ double bp_warm(double (&z)[8], const Iir& f, double x) {
  const double y = __builtin_fma(f.b[0], x, z[0]);
#pragma unroll
  for (int i = 0; i < 7; ++i) z[i] = __builtin_fma(-f.a[i + 1], y, __builtin_fma(f.b[i + 1], x, z[i + 1]));
  z[7] = __builtin_fma(-f.a[8], y, f.b[8] * x);
  return y;
}

__device__ __forceinline__ double bp_step_zo(double (&z)[8], const Iir& f, double x) {
  const double p0 = f.b[0] * x, p2 = x * f.b[2], p4 = x * f.b[4];
  const double y = z[0] + p0;
  z[0] = z[1] - y * f.a[1];
  z[1] = (z[2] + p2) - y * f.a[2];
  z[2] = z[3] - y * f.a[3];
  z[3] = (z[4] + p4) - y * f.a[4];
  z[4] = z[5] - y * f.a[5];
  z[5] = (z[6] + p2) - y * f.a[6];
  z[6] = z[7] - y * f.a[7];
  z[7] = p0 - y * f.a[8];
  return y;
}


// ---- the slicer decision (K4a, and the low-pass kernels that slice) ------
// Sector decision: far from a sector edge (|di| vs |dr| differ by more than
// 2^-30 relative) the sector is read off the signs; near an edge (or for
// zeros / NaN / inf) the reference's own steps are replayed: atan2, +2pi if
// negative, the same four comparisons against the same double constants.
// np.angle near a sector edge.  numpy evaluates arctan2 with its AVX-512
// (SVML) kernel on the hosts the reference ran on (the golden fixtures' host;
// numpy._core.__cpu_features__['AVX512_SKX']), which is not correctly rounded
// and differs from ocml's atan2 by an ulp on ~6 % of near-tie inputs -- the
// ones where an ulp decides the sector.  Within |t| < 2^-29 of the diagonal
// and for components of magnitude 2^-1015 .. 2^985 (~1e-306 .. 1e297), its
// result is, bit for bit (tests/test_gpu_slicer.py, tests/test_oracle_slicer.py):
//   t  = (|y| - |x|) / (|y| + |x|)
//   x > 0:  pi4 + (t + pi4_lo)                 x < 0:  pi - (pi4 - (pi_lo - (t + pi4_lo)))
// negated for y < 0, with pi4 split into double hi + lo (pi4_lo = pi/4 - pi4)
// and pi into hi + SVML's SHORT lo, 0x1.1a64p-53 (not pi - hi = 0x1.1a62633145c07p-53:
// bisecting numpy's rounding boundaries in the pi-side form located exactly
// this constant; with it 20 M near-tie angles agree bit for bit,
// tests/test_oracle_slicer.py).  Outside that domain (denormal or huge
// components, zeros, inf, NaN) ocml's atan2 is used.
__device__ __forceinline__ bool numpy_atan2_near_diag(double y, double x, double& ang) {
  const double ay = fabs(y), ax = fabs(x);
  if (!(ax >= 0x1p-1015 && ax <= 0x1p985 && ay >= 0x1p-1015 && ay <= 0x1p985)) return false;
  const double t = (ay - ax) / (ay + ax);
  if (!(fabs(t) < 0x1p-29)) return false;
  const double pi4 = 0x1.921fb54442d18p-1, pi4_lo = 0x1.1a62633145c07p-55;
  const double pi = 0x1.921fb54442d18p+1, pi_lo = 0x1.1a64p-53;   // SVML's short pi_lo
  const double a = x > 0 ? pi4 + (t + pi4_lo) : pi - (pi4 - (pi_lo - (t + pi4_lo)));
  ang = y < 0 ? -a : a;
  return true;
}

static __device__ __noinline__ uint32_t qpsk_dibit_slow(double dr, double di) {
  double ang;
  if (!numpy_atan2_near_diag(di, dr, ang)) ang = atan2(di, dr);
  if (ang < 0) ang += 2 * M_PI;
  if (ang < M_PI / 4 || ang > 7 * M_PI / 4) return 0u;
  if (M_PI / 4 <= ang && ang < 3 * M_PI / 4) return 1u;
  if (3 * M_PI / 4 <= ang && ang < 5 * M_PI / 4) return 3u;
  return 2u;
}

__device__ __forceinline__ uint32_t qpsk_dibit(double dr, double di) {
  const double adr = fabs(dr), adi = fabs(di);
  const double d = adi - adr;
  const double thr = (adr + adi) * 0x1p-30;
  if (d < -thr) return dr > 0 ? 0u : 3u;        // |angle| < pi/4 -> 00 ; near pi -> 11
  if (d > thr) return di > 0 ? 1u : 2u;         // near +pi/2 -> 01 ; near -pi/2 -> 10
  return qpsk_dibit_slow(dr, di);
}

}  // namespace amr
