// split_chain.h -- the serial loop of a time-split chunk (psk_split_kernels.hip
// KS1-KS4, fsk_kernels.hip FS1-FS2): one lane runs one chunk's recursion over
// w + L consecutive samples, and the 64 lanes of a wave sit L samples apart,
// so a per-sample load is a 64-line gather.  Here each lane fetches its next
// kSplitRun samples as 16-byte vector loads (global_load_dwordx4 needs only
// 4-byte alignment on gfx950), one block ahead of the recursion: a lane then
// consumes whole cache lines in order and a wave issues 4-8 loads per 16
// steps instead of 16.
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>

namespace amr {

constexpr int kSplitRun = 16;   // samples per block, fetched one block ahead

// v[0..K) = p[0..K) for a 4-byte-aligned p (float, double); element loads for int16
template <int K, typename T>
__device__ __forceinline__ void run_load(const T* __restrict__ p, T (&v)[K]) {
  if constexpr (sizeof(T) == 4 || sizeof(T) == 8) {
    constexpr int W = 16 / (int)sizeof(T);
    typedef T V __attribute__((ext_vector_type(W), aligned(4)));
#pragma unroll
    for (int i = 0; i < K / W; ++i) {
      const V t = *reinterpret_cast<const V*>(p + i * W);
#pragma unroll
      for (int e = 0; e < W; ++e) v[i * W + e] = t[e];
    }
  } else {
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = p[k];
  }
}

// for j in [j0, j1): body(j, value j); blk(j, double (&)[kSplitRun]) loads the
// values of [j, j + kSplitRun), one(j) a single value (the ragged end)
template <typename Blk, typename One, typename Body>
__device__ __forceinline__ void split_chain_run(int64_t j0, int64_t j1, Blk blk, One one, Body body) {
  constexpr int K = kSplitRun;
  int64_t j = j0;
  if (j1 - j0 >= K) {
    double cur[K];
    blk(j, cur);
    for (; j + 2 * K <= j1; j += K) {
      double nxt[K];
      blk(j + K, nxt);
#pragma unroll
      for (int k = 0; k < K; ++k) body(j + k, cur[k]);
#pragma unroll
      for (int k = 0; k < K; ++k) cur[k] = nxt[k];
    }
#pragma unroll
    for (int k = 0; k < K; ++k) body(j + k, cur[k]);
    j += K;
  }
  for (; j < j1; ++j) body(j, one(j));
}

// A chunk's run in two phases: the warm-up [j0, o0) -- recursion only, no
// index math, stores or branches per step -- then the outputs [o0, j1).
template <typename Blk, typename One, typename Warm, typename Out>
__device__ __forceinline__ void split_chain_2(int64_t j0, int64_t o0, int64_t j1, Blk blk, One one, Warm warm,
                                              Out out) {
  const int64_t m = o0 < j1 ? o0 : j1;
  if (j0 < m) split_chain_run(j0, m, blk, one, warm);
  split_chain_run(j0 > o0 ? j0 : o0, j1, blk, one, out);
}

// blocks of a forward run over a[0..): values cvt(a[j]) for j in [j, j + K)
template <typename T, typename Cvt>
__device__ __forceinline__ auto fwd_blocks(const T* a, Cvt cvt) {
  return [=](int64_t j, double (&v)[kSplitRun]) {
    T raw[kSplitRun];
    run_load<kSplitRun>(a + j, raw);
#pragma unroll
    for (int k = 0; k < kSplitRun; ++k) v[k] = cvt(raw[k]);
  };
}

// blocks of a backward run over a double array: value k is a[top - k], for k
// in [k0, k0 + K) (one contiguous block a[top - k0 - K + 1 .. top - k0])
__device__ __forceinline__ auto bwd_blocks(const double* a, int64_t top) {
  return [=](int64_t k0, double (&v)[kSplitRun]) {
    double raw[kSplitRun];
    run_load<kSplitRun>(a + (top - k0 - kSplitRun + 1), raw);
#pragma unroll
    for (int k = 0; k < kSplitRun; ++k) v[k] = raw[kSplitRun - 1 - k];
  };
}

// The strict mode's bound on a start state's error (split_strict.h): the sum
// over states of |computed - exact| <= gam (sum_m kabs[m] |v(o0 - 1 - m)| +
// z0abs[o0] |v0|) -- the FMA chains, the butterfly and the tables' rounding;
// lane 0 stores it to *dst (0 for the chunk at the pass's start: scipy's own
// zi * v0).  Off when dst is null.
struct ConvBound {
  const double* kabs;
  const double* z0abs;
  double gam;
  double* dst;
};

// A chunk's start state by convolution (psk_split_kernels.hip KS0,
// fsk_kernels.hip FS0): NS states, K [w][NS] and Z0 [w + 1][NS]
// (iir_design.h split_state_tables), one wave per chunk; lane 0 writes zo.
template <int NS, bool ST = false, typename Val>
__device__ __forceinline__ void split_conv_state(const double* __restrict__ ktab, const double* __restrict__ z0tab,
                                                 int64_t w, int64_t o0, double v0, Val val, double* __restrict__ zo,
                                                 ConvBound cb = ConvBound{}) {
  static_assert(NS % 2 == 0, "pairs of states per 16-byte load");
  const int lane = (int)(threadIdx.x & 63);
  double acc[NS];
  [[maybe_unused]] double sa = 0.0;   // ST: sum kabs[m] |v|
#pragma unroll
  for (int i = 0; i < NS; ++i) acc[i] = 0.0;
  const int64_t M = o0 < w ? o0 : w;
  // four terms' loads in flight per lane, then their FMAs in ascending m
  typedef double V2 __attribute__((ext_vector_type(2)));
  constexpr int U = 4;
  for (int64_t m0 = lane; m0 < M; m0 += 64 * U) {
    double v[U];
    V2 k[U][NS / 2];
    [[maybe_unused]] double ka[U];      // ST: kabs, loaded with the rest (not behind the FMAs)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t m = m0 + 64 * u < M ? m0 + 64 * u : M - 1;   // clamped: loaded, not used
      v[u] = val(o0 - 1 - m);
      const V2* kp = reinterpret_cast<const V2*>(ktab + m * NS);
#pragma unroll
      for (int h = 0; h < NS / 2; ++h) k[u][h] = kp[h];
      if constexpr (ST) ka[u] = cb.kabs[m];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (m0 + 64 * u < M) {
#pragma unroll
        for (int h = 0; h < NS / 2; ++h) {
          acc[2 * h] = __builtin_fma(k[u][h][0], v[u], acc[2 * h]);
          acc[2 * h + 1] = __builtin_fma(k[u][h][1], v[u], acc[2 * h + 1]);
        }
        if constexpr (ST) sa = __builtin_fma(ka[u], fabs(v[u]), sa);
      }
    }
  }
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
#pragma unroll
    for (int i = 0; i < NS; ++i) acc[i] = acc[i] + __shfl_xor(acc[i], d, 64);
    if constexpr (ST) sa = sa + __shfl_xor(sa, d, 64);
  }
  if constexpr (ST) {
    if (lane == 0) {
      const double z0t = o0 <= w ? cb.z0abs[o0] * fabs(v0) : 0.0;
      *cb.dst = o0 > 0 ? cb.gam * (sa + z0t) : 0.0;
    }
  }
  if (lane == 0) {
    if (o0 == 0) {
#pragma unroll
      for (int i = 0; i < NS; ++i) zo[i] = z0tab[i] * v0;
    } else if (o0 <= w) {
#pragma unroll
      for (int i = 0; i < NS; ++i) zo[i] = __builtin_fma(z0tab[o0 * NS + i], v0, acc[i]);
    } else {
#pragma unroll
      for (int i = 0; i < NS; ++i) zo[i] = acc[i];
    }
  }
}

}  // namespace amr
