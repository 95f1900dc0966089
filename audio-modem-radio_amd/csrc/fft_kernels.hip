// fft_kernels.hip -- batched double-precision complex FFT for gfx950, the
// transform under scipy.signal.hilbert in the FSK demodulator
// (modem.py:309; scipy.signal.hilbert = ifft(fft(x) * h)).
//
// Four-step decomposition n = n1 * n2 (both 5-smooth, <= kFftMaxL):
//   input index j = j1 + n1*j2, output index k = k2 + n2*k1
//   column pass: for each j1: length-n2 DFT over j2, times W_n^(j1*k2) -> T[k2*n1 + j1]
//   row pass:    for each k2: length-n1 DFT over j1                   -> X[k2 + n2*k1]
// The FSK path never materialises X: its forward row pass and the inverse's
// column pass are the same tiles (the inverse uses n = n2*n1 with the roles
// swapped: its input index k2 + n2*k1 is "j1' + n1'*j2'" with j1' = k2), so
// one middle kernel runs row-FFT -> multiply by -i*sgn(k) -> conj -> row-FFT ->
// twiddle, and the final row pass conjugates, scales and forms the envelopes.
// Three passes over HBM instead of four.
//
// Every pass: a workgroup owns kFftTile = 8 transforms (rows).  Global
// accesses move 8 consecutive complex values (one 128-B line) per column
// step; the transform itself is a mixed-radix (2/3/4/5) Stockham autosort in
// a single LDS buffer (rows padded by one element, so the 8 rows of a column
// fall in distinct banks), each stage staged through registers between two
// barriers.  The inverse transform is conj(FFT(conj(x))).
// Twiddles come from host tables (W_L^t, t < L, fft.h), one libm cos/sin per
// entry, so every factor is within an ulp of exact.
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

// exact floor(i / d) for 0 <= i < 2^20 given inv = 1/d rounded to float (fft.h)
__device__ __forceinline__ int fdiv(int i, float inv) { return (int)(((float)i + 0.5f) * inv); }

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

// One Stockham stage (radix R) over kFftTile rows of length L, in place in
// LDS: every thread reads its butterflies' inputs into registers, the block
// synchronises, then every thread writes its outputs.
template <int R>
__device__ __forceinline__ void stockham_stage(double2* buf, int S, const FftStage& sg,
                                               const double2* __restrict__ tw) {
  constexpr int MAXB = (kFftMaxVals + R - 1) / R;
  const int total = kFftTile * sg.nb;
  double2 v[MAXB][R];
  int dst[MAXB];
#pragma unroll
  for (int m = 0; m < MAXB; ++m) {
    const int idx = threadIdx.x + m * kFftThreads;
    if (idx < total) {
      const int row = fdiv(idx, sg.inv_nb);
      const int j = idx - row * sg.nb;
      const int g = fdiv(j, sg.inv_ns);
      const int k = j - g * sg.ns;
      const double2* s = buf + row * S + j;
#pragma unroll
      for (int q = 0; q < R; ++q) v[m][q] = s[q * sg.nb];
      if (sg.ns > 1) {
#pragma unroll
        for (int q = 1; q < R; ++q) v[m][q] = cmul(v[m][q], tw[k * q * sg.tstep]);   // k*q*tstep < L
      }
      if constexpr (R == 2) dft2(v[m]);
      if constexpr (R == 3) dft3(v[m]);
      if constexpr (R == 4) dft4(v[m]);
      if constexpr (R == 5) dft5(v[m]);
      dst[m] = row * S + g * sg.ns * R + k;
    }
  }
  __syncthreads();
#pragma unroll
  for (int m = 0; m < MAXB; ++m) {
    if ((int)threadIdx.x + m * kFftThreads < total) {
#pragma unroll
      for (int q = 0; q < R; ++q) buf[dst[m] + q * sg.ns] = v[m][q];
    }
  }
  __syncthreads();
}

// Transforms the kFftTile rows in buf (row stride S) in place.  Caller has
// synchronised after filling buf; returns synchronised.
__device__ void lds_fft(double2* buf, int S, const FftLen& f) {
  for (int s = 0; s < f.nst; ++s) {
    switch (f.st[s].r) {
      case 2: stockham_stage<2>(buf, S, f.st[s], f.tw); break;
      case 3: stockham_stage<3>(buf, S, f.st[s], f.tw); break;
      case 4: stockham_stage<4>(buf, S, f.st[s], f.tw); break;
      case 5: stockham_stage<5>(buf, S, f.st[s], f.tw); break;
    }
  }
}

// -i*sgn(k) * v for a length-n transform (scipy.signal.hilbert's h, minus the identity)
__device__ __forceinline__ double2 hilbert_mul(double2 v, int64_t k, int64_t n) {
  const int64_t k2 = 2 * k;
  return (k == 0 || k2 == n) ? make_double2(0.0, 0.0) : (k2 < n ? mul_mi(v) : make_double2(-v.y, v.x));
}

template <int MODE>
__device__ __forceinline__ void fft_epilogue(const FftEpi& e, double2* __restrict__ dst, int64_t b, int64_t k,
                                             double2 v) {
  const size_t o = (size_t)b * e.n + k;
  switch (MODE) {
    case kHilbert: dst[o] = hilbert_mul(v, k, e.n); break;
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

// Loads rows r0 .. r0+7 (each L contiguous values at src[r*L]) into buf.
__device__ __forceinline__ void load_rows(double2* buf, int S, const double2* __restrict__ src, int r0, int nrow,
                                          const FftLen& f, bool conj_in) {
  const int L = f.L;
  const int rows = min(kFftTile, nrow - r0);
  const double2* s = src + (size_t)r0 * L;
  for (int e = threadIdx.x; e < kFftTile * L; e += kFftThreads) {
    const int row = fdiv(e, f.inv_L);
    const int c = e - row * L;
    const double2 v = row < rows ? s[e] : make_double2(0.0, 0.0);
    buf[row * S + c] = conj_in ? conj2(v) : v;
  }
  __syncthreads();
}

// ---- column pass: in[b][j1 + n1*j2] -> T[b][k2*n1 + j1] = W_n^(j1 k2) * DFT_n2 ----
template <bool CONJ_IN>
__global__ __launch_bounds__(kFftThreads) void k_fft_cols(const double2* __restrict__ in, double2* __restrict__ out,
                                                         FftDesc d, int64_t batch) {
  extern __shared__ __attribute__((aligned(16))) double2 smem[];
  const int tiles = (d.n1 + kFftTile - 1) / kFftTile;
  const int64_t b = blockIdx.x / tiles;
  const int j1_0 = (int)(blockIdx.x - b * tiles) * kFftTile;
  if (b >= batch) return;
  const int L = d.n2, S = L + 1;
  const double2* src = in + (size_t)b * d.n;
  for (int idx = threadIdx.x; idx < kFftTile * L; idx += kFftThreads) {
    const int t = idx & (kFftTile - 1), j2 = idx / kFftTile;
    const int j1 = j1_0 + t;
    const double2 v = j1 < d.n1 ? src[(size_t)j1 + (size_t)d.n1 * j2] : make_double2(0.0, 0.0);
    smem[t * S + j2] = CONJ_IN ? conj2(v) : v;
  }
  __syncthreads();
  lds_fft(smem, S, d.a);
  double2* dst = out + (size_t)b * d.n;
  for (int idx = threadIdx.x; idx < kFftTile * L; idx += kFftThreads) {
    const int t = idx & (kFftTile - 1), k2 = idx / kFftTile;
    const int j1 = j1_0 + t;
    if (j1 < d.n1) dst[(size_t)k2 * d.n1 + j1] = cmul(smem[t * S + k2], d.twn[(int64_t)j1 * k2]);
  }
}

// ---- middle pass of a filter: rows k2 of T (length n1) -> X[k2 + n2*k1] ->
// Y = mid(X) -> conj -> DFT_n1 over k1 -> k2', times W_n^(k2 k2') ->
// T'[k2'*n2 + k2]  (the column pass of FFT(conj Y) with n = n2 * n1) --------
template <int MID>
__global__ __launch_bounds__(kFftThreads) void k_fft_mid(const double2* __restrict__ in, double2* __restrict__ out,
                                                        FftDesc d, int64_t batch, const double2* __restrict__ tab) {
  extern __shared__ __attribute__((aligned(16))) double2 smem[];
  const int tiles = (d.n2 + kFftTile - 1) / kFftTile;
  const int64_t b = blockIdx.x / tiles;
  const int r0 = (int)(blockIdx.x - b * tiles) * kFftTile;
  if (b >= batch) return;
  const int L = d.n1, S = L + 1;
  load_rows(smem, S, in + (size_t)b * d.n, r0, d.n2, d.c, false);
  lds_fft(smem, S, d.c);
  const int64_t n = d.n;
  for (int e = threadIdx.x; e < kFftTile * L; e += kFftThreads) {
    const int row = fdiv(e, d.c.inv_L);
    const int k1 = e - row * L;
    const int64_t k = (int64_t)(r0 + row) + (int64_t)d.n2 * k1;
    double2 v = smem[row * S + k1];
    if (MID == kHilbert)
      v = hilbert_mul(v, k, n);
    else
      v = r0 + row < d.n2 ? cmul(v, tab[k]) : make_double2(0.0, 0.0);
    smem[row * S + k1] = conj2(v);
  }
  __syncthreads();
  lds_fft(smem, S, d.c);
  double2* dst = out + (size_t)b * n;
  for (int idx = threadIdx.x; idx < kFftTile * L; idx += kFftThreads) {
    const int t = idx & (kFftTile - 1), k2p = idx / kFftTile;
    const int r = r0 + t;
    if (r < d.n2) dst[(size_t)k2p * d.n2 + r] = cmul(smem[t * S + k2p], d.twn[(int64_t)r * k2p]);
  }
}

// ---- row pass: rows r of in (length f.L, nrow rows) -> DFT -> out index
// r + nrow*k; CONJ_OUT conjugates and scales (inverse); then the epilogue --
template <bool CONJ_OUT, int MODE>
__global__ __launch_bounds__(kFftThreads) void k_fft_rows(const double2* __restrict__ in, double2* __restrict__ out,
                                                         FftLen f, int nrow, int64_t n, int64_t batch, double scale,
                                                         FftEpi e) {
  extern __shared__ __attribute__((aligned(16))) double2 smem[];
  const int tiles = (nrow + kFftTile - 1) / kFftTile;
  const int64_t b = blockIdx.x / tiles;
  const int r0 = (int)(blockIdx.x - b * tiles) * kFftTile;
  if (b >= batch) return;
  const int L = f.L, S = L + 1;
  load_rows(smem, S, in + (size_t)b * n, r0, nrow, f, false);
  lds_fft(smem, S, f);
  for (int idx = threadIdx.x; idx < kFftTile * L; idx += kFftThreads) {
    const int t = idx & (kFftTile - 1), k = idx / kFftTile;
    const int r = r0 + t;
    if (r < nrow) {
      double2 v = smem[t * S + k];
      if (CONJ_OUT) v = make_double2(v.x * scale, -v.y * scale);
      fft_epilogue<MODE>(e, out, b, (int64_t)r + (int64_t)nrow * k, v);
    }
  }
}

// Bluestein (n not 5-smooth): X_k = conj(w_k) * sum_j (x_j conj(w_j)) w_(k-j),
// w_j = exp(i pi j^2 / n), as a length-M circular convolution, M >= 2n-1.
//   pre:  a[b][j] = x[b][j] * conj(w_j) (j < n), 0 (n <= j < M); inv conjugates x
//   then  IFFT_M(FFT_M(a) * FFT_M(bw)): one launch_fft_filter (kMulTab)
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

static size_t fft_smem_bytes(int L) { return (size_t)kFftTile * (L + 1) * sizeof(double2); }

hipError_t launch_fft(const double2* in, double2* tmp, double2* out, const FftDesc& d, int64_t batch, bool inverse,
                      hipStream_t st) {
  const unsigned gcol = (unsigned)(batch * ((d.n1 + kFftTile - 1) / kFftTile));
  const unsigned grow = (unsigned)(batch * ((d.n2 + kFftTile - 1) / kFftTile));
  FftEpi e{};
  e.mode = kStore;
  e.n = d.n;
  if (inverse) {
    hipLaunchKernelGGL(k_fft_cols<true>, dim3(gcol), dim3(kFftThreads), fft_smem_bytes(d.n2), st, in, tmp, d, batch);
    hipLaunchKernelGGL((k_fft_rows<true, kStore>), dim3(grow), dim3(kFftThreads), fft_smem_bytes(d.n1), st,
                       tmp, out, d.c, d.n2, d.n, batch, 1.0 / (double)d.n, e);
  } else {
    hipLaunchKernelGGL(k_fft_cols<false>, dim3(gcol), dim3(kFftThreads), fft_smem_bytes(d.n2), st, in, tmp, d, batch);
    hipLaunchKernelGGL((k_fft_rows<false, kStore>), dim3(grow), dim3(kFftThreads), fft_smem_bytes(d.n1), st,
                       tmp, out, d.c, d.n2, d.n, batch, 1.0, e);
  }
  return hipGetLastError();
}

hipError_t launch_fft_filter(const double2* in, double2* t1, double2* t2, double2* out, const FftDesc& d,
                             int64_t batch, int mid, const double2* tab, const FftEpi& epi, hipStream_t st) {
  const unsigned gcol = (unsigned)(batch * ((d.n1 + kFftTile - 1) / kFftTile));
  const unsigned gmid = (unsigned)(batch * ((d.n2 + kFftTile - 1) / kFftTile));
  hipLaunchKernelGGL(k_fft_cols<false>, dim3(gcol), dim3(kFftThreads), fft_smem_bytes(d.n2), st, in, t1, d, batch);
  if (mid == kHilbert)
    hipLaunchKernelGGL(k_fft_mid<kHilbert>, dim3(gmid), dim3(kFftThreads), fft_smem_bytes(d.n1), st, t1, t2, d,
                       batch, tab);
  else if (mid == kMulTab)
    hipLaunchKernelGGL(k_fft_mid<kMulTab>, dim3(gmid), dim3(kFftThreads), fft_smem_bytes(d.n1), st, t1, t2, d,
                       batch, tab);
  else
    return hipErrorInvalidValue;
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) return err;
  // final row pass: the n1 rows k2' of T' (length n2) -> index k2' + n1*k1', conj, 1/n
  FftEpi e = epi;
  e.n = d.n;
  const unsigned gfin = (unsigned)(batch * ((d.n1 + kFftTile - 1) / kFftTile));
  const double scale = 1.0 / (double)d.n;
  const size_t sm = fft_smem_bytes(d.n2);
  switch (epi.mode) {
    case kStore:
      hipLaunchKernelGGL((k_fft_rows<true, kStore>), dim3(gfin), dim3(kFftThreads), sm, st, t2, out, d.a,
                         d.n1, d.n, batch, scale, e);
      break;
    case kEnvelope:
      hipLaunchKernelGGL((k_fft_rows<true, kEnvelope>), dim3(gfin), dim3(kFftThreads), sm, st, t2, out, d.a,
                         d.n1, d.n, batch, scale, e);
      break;
    case kEnvOut:
      hipLaunchKernelGGL((k_fft_rows<true, kEnvOut>), dim3(gfin), dim3(kFftThreads), sm, st, t2, out, d.a,
                         d.n1, d.n, batch, scale, e);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
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
  const int bytes = (int)fft_smem_bytes(kFftMaxL);
  const void* fns[] = {
      (const void*)k_fft_cols<false>, (const void*)k_fft_cols<true>, (const void*)k_fft_mid<kHilbert>,
      (const void*)k_fft_mid<kMulTab>, (const void*)k_fft_rows<false, kStore>,
      (const void*)k_fft_rows<true, kStore>, (const void*)k_fft_rows<true, kEnvelope>,
      (const void*)k_fft_rows<true, kEnvOut>};
  for (const void* f : fns) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace amr
