// psk_common.h -- device helpers shared by the PSK kernel files
// (psk_kernels.hip: the state-per-lane kernels; psk_lane_kernels.hip: the
// lane-per-stream throughput kernels).  Both must evaluate the reference's
// arithmetic identically, so the conversions, layouts and the
// low-pass zero detector live here once.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

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


}  // namespace amr
