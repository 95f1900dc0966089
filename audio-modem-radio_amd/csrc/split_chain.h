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

}  // namespace amr
