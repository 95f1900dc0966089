// fft_kernels.hip -- batched double-precision complex FFT for gfx950, the
// transform under scipy.signal.hilbert in the FSK demodulator
// (modem.py:309; scipy.signal.hilbert = ifft(fft(x) * h)).
//
// Four-step decomposition n = n1 * n2 (both 5-smooth, <= kFftMaxL):
//   input index j = j1 + n1*j2, output index k = k2 + n2*k1
//   pass A: for each j1: length-n2 DFT over j2, times W_n^(j1*k2)  -> T[k2][j1]
//   pass C: for each k2: length-n1 DFT over j1                     -> X[k2 + n2*k1]
// Each pass is one kernel: a workgroup stages kFftTile transforms in LDS
// (tile rows loaded/stored as 128-B coalesced segments), runs a mixed-radix
// (2/3/4/5) Stockham autosort in ping-pong LDS buffers, and writes back.  The
// inverse transform is conj(FFT(conj(x))), done by conjugating on load/store.
// Twiddles come from host tables (W_L^t, t < L, fft_plan.h), one libm
// cos/sin per entry, so every factor is within an ulp of exact.
#include "fft.h"

namespace amr {

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
  return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 conj2(double2 a) { return make_double2(a.x, -a.y); }
// -i * a
__device__ __forceinline__ double2 mul_mi(double2 a) { return make_double2(a.y, -a.x); }

// forward radix-r DFTs (W = exp(-2 pi i / r))
__device__ __forceinline__ void dft2(double2* v) {
  const double2 a = v[0], b = v[1];
  v[0] = cadd(a, b);
  v[1] = csub(a, b);
}
__device__ __forceinline__ void dft3(double2* v) {
  const double c = -0.5, s = 0.86602540378443864676;   // cos, sin of 2pi/3
  const double2 t1 = cadd(v[1], v[2]), t2 = csub(v[1], v[2]);
  const double2 m = make_double2(v[0].x + c * t1.x, v[0].y + c * t1.y);
  const double2 u = make_double2(s * t2.y, -s * t2.x);   // -i*s*t2
  v[0] = cadd(v[0], t1);
  v[1] = cadd(m, u);
  v[2] = csub(m, u);
}
__device__ __forceinline__ void dft4(double2* v) {
  const double2 a0 = cadd(v[0], v[2]), a1 = csub(v[0], v[2]);
  const double2 b0 = cadd(v[1], v[3]), b1 = mul_mi(csub(v[1], v[3]));
  v[0] = cadd(a0, b0);
  v[2] = csub(a0, b0);
  v[1] = cadd(a1, b1);
  v[3] = csub(a1, b1);
}
__device__ __forceinline__ void dft5(double2* v) {
  const double c1 = 0.30901699437494742410, c2 = -0.80901699437494742410;   // cos(2pi/5), cos(4pi/5)
  const double s1 = 0.95105651629515357212, s2 = 0.58778525229247312917;    // sin(2pi/5), sin(4pi/5)
  const double2 t1 = cadd(v[1], v[4]), t2 = cadd(v[2], v[3]);
  const double2 t3 = csub(v[1], v[4]), t4 = csub(v[2], v[3]);
  const double2 m1 = make_double2(v[0].x + c1 * t1.x + c2 * t2.x, v[0].y + c1 * t1.y + c2 * t2.y);
  const double2 m2 = make_double2(v[0].x + c2 * t1.x + c1 * t2.x, v[0].y + c2 * t1.y + c1 * t2.y);
  // -i*(s1*t3 + s2*t4) and -i*(s2*t3 - s1*t4)
  const double2 n1 = mul_mi(make_double2(s1 * t3.x + s2 * t4.x, s1 * t3.y + s2 * t4.y));
  const double2 n2 = mul_mi(make_double2(s2 * t3.x - s1 * t4.x, s2 * t3.y - s1 * t4.y));
  v[0] = cadd(v[0], cadd(t1, t2));
  v[1] = cadd(m1, n1);
  v[4] = csub(m1, n1);
  v[2] = cadd(m2, n2);
  v[3] = csub(m2, n2);
}

// One Stockham stage (radix R) over kFftTile rows of length L: src -> dst.
template <int R>
__device__ __forceinline__ void stockham_stage(const double2* __restrict__ src, double2* __restrict__ dst, int L,
                                               int Ns, const double2* __restrict__ tw) {
  const int nb = L / R;
  const int tstep = L / (Ns * R);          // W_{Ns R}^{k q} = W_L^{k q tstep}
  for (int idx = threadIdx.x; idx < kFftTile * nb; idx += kFftThreads) {
    const int row = idx / nb, j = idx - row * nb;
    const double2* s = src + row * L;
    double2* d = dst + row * L;
    const int k = j % Ns;
    double2 v[R];
#pragma unroll
    for (int q = 0; q < R; ++q) v[q] = s[j + q * nb];
    if (Ns > 1) {
#pragma unroll
      for (int q = 1; q < R; ++q) v[q] = cmul(v[q], tw[k * q * tstep]);   // k*q*tstep < L
    }
    if constexpr (R == 2) dft2(v);
    if constexpr (R == 3) dft3(v);
    if constexpr (R == 4) dft4(v);
    if constexpr (R == 5) dft5(v);
    const int base = (j / Ns) * Ns * R + k;
#pragma unroll
    for (int q = 0; q < R; ++q) d[base + q * Ns] = v[q];
  }
}

// Runs all stages; returns the buffer holding the result (A or B).
__device__ double2* lds_fft(double2* A, double2* B, const FftLen& f) {
  int Ns = 1;
  double2* src = A;
  double2* dst = B;
  for (int s = 0; s < f.nst; ++s) {
    __syncthreads();
    switch (f.r[s]) {
      case 2: stockham_stage<2>(src, dst, f.L, Ns, f.tw); break;
      case 3: stockham_stage<3>(src, dst, f.L, Ns, f.tw); break;
      case 4: stockham_stage<4>(src, dst, f.L, Ns, f.tw); break;
      case 5: stockham_stage<5>(src, dst, f.L, Ns, f.tw); break;
    }
    Ns *= f.r[s];
    double2* t = src;
    src = dst;
    dst = t;
  }
  __syncthreads();
  return src;
}

// Pass A: in[b][j] (j = j1 + n1*j2) -> T[b][k2*n1 + j1] = W_n^(j1 k2) * DFT_n2(in[b][j1 + n1*:])[k2]
// inv: conjugate the input on load (inverse = conj(FFT(conj x))).
template <bool INV>
__global__ __launch_bounds__(kFftThreads) void k_fft_pass_a(const double2* __restrict__ in, double2* __restrict__ out,
                                                           FftDesc d, int64_t batch) {
  extern __shared__ __attribute__((aligned(16))) double2 smem[];
  const int tiles = (d.n1 + kFftTile - 1) / kFftTile;
  const int64_t b = blockIdx.x / tiles;
  const int j1_0 = (int)(blockIdx.x - b * tiles) * kFftTile;
  if (b >= batch) return;
  const int L = d.n2;
  double2* A = smem;
  double2* B = smem + kFftTile * L;
  const double2* src = in + (size_t)b * d.n;
  for (int idx = threadIdx.x; idx < kFftTile * L; idx += kFftThreads) {
    const int t = idx % kFftTile, j2 = idx / kFftTile;
    const int j1 = j1_0 + t;
    double2 v = j1 < d.n1 ? src[(size_t)j1 + (size_t)d.n1 * j2] : make_double2(0.0, 0.0);
    A[t * L + j2] = INV ? conj2(v) : v;
  }
  const double2* R = lds_fft(A, B, d.a);
  double2* dst = out + (size_t)b * d.n;
  for (int idx = threadIdx.x; idx < kFftTile * L; idx += kFftThreads) {
    const int t = idx % kFftTile, k2 = idx / kFftTile;
    const int j1 = j1_0 + t;
    if (j1 < d.n1) {
      const double2 w = d.twn[(int64_t)j1 * k2];   // j1*k2 < n1*n2 = n
      dst[(size_t)k2 * d.n1 + j1] = cmul(R[t * L + k2], w);
    }
  }
}

// What the last pass does with each output X[b][k] (k < e.n):
//   kStore     dst[b][k] = X
//   kHilbert   dst[b][k] = -i*sgn(k) * X     (sgn = +1 for 0 < 2k < n, -1 for
//              2k > n, 0 at k = 0 and k = n/2: scipy.signal.hilbert's h - 1)
//   kEnvelope  X = H[z] = H[f_mark] + i*H[f_space];  f = z[b][k]:
//              cmp[b][k] = hypot(f.x, X.x) > hypot(f.y, X.y)        (modem.py:309,315)
//   kEnvOut    the two envelopes themselves -> dst[b][k] = (|a_mark|, |a_space|)
//   kMulTab    dst[b][k] = X * tab[k]        (Bluestein: times FFT(chirp))
template <int MODE>
__device__ __forceinline__ void fft_epilogue(const FftEpi& e, double2* __restrict__ dst, int64_t b, int64_t k,
                                             double2 v) {
  const size_t o = (size_t)b * e.n + k;
  switch (MODE) {
    case kHilbert: {
      const int64_t k2 = 2 * k;
      v = (k == 0 || k2 == e.n) ? make_double2(0.0, 0.0) : (k2 < e.n ? mul_mi(v) : make_double2(-v.y, v.x));
      dst[o] = v;
      break;
    }
    case kEnvelope: {
      const double2 f = e.z[o];
      e.cmp[o] = hypot(f.x, v.x) > hypot(f.y, v.y) ? 1 : 0;
      break;
    }
    case kEnvOut: {
      const double2 f = e.z[o];
      dst[o] = make_double2(hypot(f.x, v.x), hypot(f.y, v.y));
      break;
    }
    case kMulTab: dst[o] = cmul(v, e.tab[k]); break;
    default: dst[o] = v; break;
  }
}

// Pass C: T[b][k2*n1 + j1] -> X[b][k2 + n2*k1] = DFT_n1(T[b][k2*n1 + :])[k1]
// inv: conjugate and scale by `scale`; then the epilogue.
template <bool INV, int MODE>
__global__ __launch_bounds__(kFftThreads) void k_fft_pass_c(const double2* __restrict__ in, double2* __restrict__ out,
                                                           FftDesc d, int64_t batch, double scale, FftEpi e) {
  extern __shared__ __attribute__((aligned(16))) double2 smem[];
  const int tiles = (d.n2 + kFftTile - 1) / kFftTile;
  const int64_t b = blockIdx.x / tiles;
  const int k2_0 = (int)(blockIdx.x - b * tiles) * kFftTile;
  if (b >= batch) return;
  const int L = d.n1;
  double2* A = smem;
  double2* B = smem + kFftTile * L;
  const double2* src = in + (size_t)b * d.n;
  for (int idx = threadIdx.x; idx < kFftTile * L; idx += kFftThreads) {
    const int t = idx / L, j1 = idx - t * L;
    const int k2 = k2_0 + t;
    A[t * L + j1] = k2 < d.n2 ? src[(size_t)k2 * d.n1 + j1] : make_double2(0.0, 0.0);
  }
  const double2* R = lds_fft(A, B, d.c);
  for (int idx = threadIdx.x; idx < kFftTile * L; idx += kFftThreads) {
    const int t = idx % kFftTile, k1 = idx / kFftTile;
    const int k2 = k2_0 + t;
    if (k2 < d.n2) {
      double2 v = R[t * L + k1];
      if (INV) v = make_double2(v.x * scale, -v.y * scale);
      fft_epilogue<MODE>(e, out, b, (int64_t)k2 + (int64_t)d.n2 * k1, v);
    }
  }
}

// Bluestein (n not 5-smooth): X_k = conj(w_k) * sum_j (x_j conj(w_j)) w_(k-j),
// w_j = exp(i pi j^2 / n), as a length-M circular convolution, M >= 2n-1.
//   pre:  a[b][j] = x[b][j] * conj(w_j) (j < n), 0 (n <= j < M); inv conjugates x
//   then  FFT_M(a) * FFT_M(bw) (kMulTab), IFFT_M
//   post: X_k = conj(w_k) * y[b][k]; inv conjugates and scales; then the epilogue
__global__ __launch_bounds__(256) void k_bs_pre(const double2* __restrict__ x, double2* __restrict__ a,
                                                const double2* __restrict__ w, int64_t n, int64_t M, int64_t batch,
                                                int inv) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= batch * M) return;
  const int64_t b = i / M, j = i - b * M;
  double2 v = make_double2(0.0, 0.0);
  if (j < n) {
    double2 xv = x[(size_t)b * n + j];
    if (inv) xv = conj2(xv);
    v = cmul(xv, conj2(w[j]));
  }
  a[i] = v;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_bs_post(const double2* __restrict__ y, double2* __restrict__ out,
                                                 const double2* __restrict__ w, int64_t n, int64_t M, int64_t batch,
                                                 int inv, double scale, FftEpi e) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= batch * n) return;
  const int64_t b = i / n, k = i - b * n;
  double2 v = cmul(y[(size_t)b * M + k], conj2(w[k]));
  if (inv) v = make_double2(v.x * scale, -v.y * scale);
  fft_epilogue<MODE>(e, out, b, k, v);
}

size_t fft_smem_bytes(const FftDesc& d, bool pass_a) {
  const int L = pass_a ? d.n2 : d.n1;
  return (size_t)2 * kFftTile * L * sizeof(double2);
}

// The (direction, epilogue) pairs the FSK path and the test entry points use;
// each is its own kernel so rocprof attributes time per stage.
#define AMR_FFT_VARIANTS(X) \
  X(false, kStore) X(true, kStore) X(false, kHilbert) X(true, kEnvelope) X(true, kEnvOut) X(false, kMulTab)

hipError_t launch_fft(const double2* in, double2* tmp, double2* out, const FftDesc& d, int64_t batch, bool inverse,
                      const FftEpi& epi, hipStream_t st) {
  const unsigned ga = (unsigned)(batch * ((d.n1 + kFftTile - 1) / kFftTile));
  const unsigned gc = (unsigned)(batch * ((d.n2 + kFftTile - 1) / kFftTile));
  const size_t sa = fft_smem_bytes(d, true), sc = fft_smem_bytes(d, false);
  if (inverse)
    hipLaunchKernelGGL(k_fft_pass_a<true>, dim3(ga), dim3(kFftThreads), sa, st, in, tmp, d, batch);
  else
    hipLaunchKernelGGL(k_fft_pass_a<false>, dim3(ga), dim3(kFftThreads), sa, st, in, tmp, d, batch);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const double scale = inverse ? 1.0 / (double)d.n : 1.0;
#define AMR_FFT_LAUNCH_C(I, M)                                                                          \
  if (inverse == I && epi.mode == M) {                                                                  \
    hipLaunchKernelGGL((k_fft_pass_c<I, M>), dim3(gc), dim3(kFftThreads), sc, st, tmp, out, d, batch, scale, epi); \
    return hipGetLastError();                                                                           \
  }
  AMR_FFT_VARIANTS(AMR_FFT_LAUNCH_C)
#undef AMR_FFT_LAUNCH_C
  return hipErrorInvalidValue;
}

hipError_t launch_bs_pre(const double2* x, double2* a, const double2* w, int64_t n, int64_t M, int64_t batch,
                         bool inverse, hipStream_t st) {
  const int64_t tot = batch * M;
  hipLaunchKernelGGL(k_bs_pre, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, x, a, w, n, M, batch,
                     inverse ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_bs_post(const double2* y, double2* out, const double2* w, int64_t n, int64_t M, int64_t batch,
                          bool inverse, const FftEpi& epi, hipStream_t st) {
  const int64_t tot = batch * n;
  const dim3 g((unsigned)((tot + 255) / 256));
  const int inv = inverse ? 1 : 0;
  const double scale = inverse ? 1.0 / (double)n : 1.0;
  switch (epi.mode) {
    case kStore: hipLaunchKernelGGL(k_bs_post<kStore>, g, dim3(256), 0, st, y, out, w, n, M, batch, inv, scale, epi); break;
    case kHilbert: hipLaunchKernelGGL(k_bs_post<kHilbert>, g, dim3(256), 0, st, y, out, w, n, M, batch, inv, scale, epi); break;
    case kEnvelope: hipLaunchKernelGGL(k_bs_post<kEnvelope>, g, dim3(256), 0, st, y, out, w, n, M, batch, inv, scale, epi); break;
    case kEnvOut: hipLaunchKernelGGL(k_bs_post<kEnvOut>, g, dim3(256), 0, st, y, out, w, n, M, batch, inv, scale, epi); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t fft_configure_smem() {
  const int bytes = 2 * kFftTile * kFftMaxL * (int)sizeof(double2);
  hipError_t e = hipFuncSetAttribute((const void*)k_fft_pass_a<false>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)k_fft_pass_a<true>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
#define AMR_FFT_ATTR_C(I, M)                                                                                 \
  if (e == hipSuccess)                                                                                       \
    e = hipFuncSetAttribute((const void*)k_fft_pass_c<I, M>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  AMR_FFT_VARIANTS(AMR_FFT_ATTR_C)
#undef AMR_FFT_ATTR_C
  return e;
}

}  // namespace amr
