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
// Every pass: a workgroup of four waves owns kFftTile = 8 transforms (rows) of
// length L = P * Q <= 625, done as two register-resident stages:
//   stage 1: radix P (a composite a*b DFT in registers) straight from HBM,
//            outputs to LDS (one exchange per transform)
//   stage 2: radix Q from LDS, twiddle W_L^(j m), outputs straight to HBM
// Column accesses move 8 consecutive complex values (one 128-B line) per
// step; row accesses are contiguous.  The inverse transform is
// conj(FFT(conj(x))).  Twiddles come from host tables (fft.h), one libm
// cos/sin per entry with the exponent reduced in integers.
#include <algorithm>
#include <cstdlib>

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

// forward radix-p DFTs, p <= 5 (W = exp(-2 pi i / p))
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

template <int P>
__device__ __forceinline__ void dftp(double2* v) {
  if constexpr (P == 2) dft2(v);
  if constexpr (P == 3) dft3(v);
  if constexpr (P == 4) dft4(v);
  if constexpr (P == 5) dft5(v);
}

// R = A * B, A >= B, both <= 5
template <int R> struct RadixF;
template <> struct RadixF<1> { static constexpr int A = 1, B = 1; };
template <> struct RadixF<2> { static constexpr int A = 2, B = 1; };
template <> struct RadixF<3> { static constexpr int A = 3, B = 1; };
template <> struct RadixF<4> { static constexpr int A = 4, B = 1; };
template <> struct RadixF<5> { static constexpr int A = 5, B = 1; };
template <> struct RadixF<6> { static constexpr int A = 3, B = 2; };
template <> struct RadixF<8> { static constexpr int A = 4, B = 2; };
template <> struct RadixF<9> { static constexpr int A = 3, B = 3; };
template <> struct RadixF<10> { static constexpr int A = 5, B = 2; };
template <> struct RadixF<12> { static constexpr int A = 4, B = 3; };
template <> struct RadixF<15> { static constexpr int A = 5, B = 3; };
template <> struct RadixF<16> { static constexpr int A = 4, B = 4; };
template <> struct RadixF<20> { static constexpr int A = 5, B = 4; };
template <> struct RadixF<25> { static constexpr int A = 5, B = 5; };

// Length-R DFT in registers, R = A*B: q = B*q1 + q2, m = m1 + A*m2,
//   X[m1 + A m2] = sum_q2 W_B^(q2 m2) W_R^(q2 m1) sum_q1 v[B q1 + q2] W_A^(q1 m1)
// computed in place: on return v[B*m1 + m2] holds X[m1 + A*m2] (bfly_out<R>
// maps a register slot to its frequency).  W_R^t = tw[t * tstride] (the
// row's W_L table, tstride = L/R; wave-uniform loads).
template <int R>
__host__ __device__ constexpr int bfly_out(int slot) {
  return slot / RadixF<R>::B + RadixF<R>::A * (slot % RadixF<R>::B);
}

// inverse of bfly_out: the register slot holding frequency m
template <int R>
__host__ __device__ constexpr int bfly_slot(int m) {
  return RadixF<R>::B * (m % RadixF<R>::A) + m / RadixF<R>::A;
}

template <int R>
__device__ __forceinline__ void bfly(double2 (&v)[R], const double2* __restrict__ tw, int tstride) {
  constexpr int A = RadixF<R>::A, B = RadixF<R>::B;
  if constexpr (B == 1) {
    dftp<A>(v);
  } else {
#pragma unroll
    for (int q2 = 0; q2 < B; ++q2) {           // DFT_A down each column q2
      double2 a[A];
#pragma unroll
      for (int q1 = 0; q1 < A; ++q1) a[q1] = v[B * q1 + q2];
      dftp<A>(a);
#pragma unroll
      for (int m1 = 0; m1 < A; ++m1) v[B * m1 + q2] = q2 > 0 && m1 > 0 ? cmul(a[m1], tw[q2 * m1 * tstride]) : a[m1];
    }
#pragma unroll
    for (int m1 = 0; m1 < A; ++m1) {           // DFT_B along each row m1
      double2 c[B];
#pragma unroll
      for (int q2 = 0; q2 < B; ++q2) c[q2] = v[B * m1 + q2];
      dftp<B>(c);
#pragma unroll
      for (int m2 = 0; m2 < B; ++m2) v[B * m1 + m2] = c[m2];
    }
  }
}

#define AMR_FFT_RADICES(X) X(1) X(2) X(3) X(4) X(5) X(6) X(8) X(9) X(10) X(12) X(15) X(16) X(20) X(25)

// A row of length L = P*Q (fft.h FftLen: P = r1, Q = r2), element c = j + Q*q:
//   stage 1, per j < Q:  Y[j][m] = sum_q x[j + Q q] W_P^(q m)                  (m < P)
//   stage 2, per m < P:  X[m + P p] = sum_j W_Q^(j p) (W_L^(j m) Y[j][m])        (p < Q)
// Y lives in LDS at row t, position j + Qp*m (Qp = Q + pad, odd), so stage 1
// writes the positions it read (in place without hazards) and stage 2 reads
// contiguous blocks.  One butterfly per thread (8 * 25 <= kFftThreads).
//
// stage 1: ld(t, j, q) -> x[j + Q q];  st(t, j, m, v) stores Y[j][m].
// ROWFAST maps lanes along a row (contiguous sources), otherwise across the 8
// rows (column-strided sources, 8 consecutive columns = one 128-B line).
// twl: the row's W_L table in LDS.  fill_twl: copy it from f.tw after this
// stage's loads are issued, then a block barrier, so the two latencies overlap.
// QC: Q as a compile-time constant (0: runtime f.r2).
template <int P, int QC, bool ROWFAST, class Ld, class St>
__device__ __forceinline__ void fft_stage1(const FftLen& f, double2* twl, Ld ld, St st, bool fill_twl) {
  const int Q = QC ? QC : f.r2;
  const int idx = threadIdx.x;
  const bool on = idx < kFftTile * Q;
  int t, j;
  if (ROWFAST) {
    t = QC ? idx / QC : fdiv(idx, f.inv_r2);
    j = idx - t * Q;
  } else {
    t = idx & (kFftTile - 1);
    j = idx / kFftTile;
  }
  double2 v[P];
  if (on) {
#pragma unroll
    for (int q = 0; q < P; ++q) v[q] = ld(t, j, q);
  }
  if (fill_twl) {
    for (int i = threadIdx.x; i < f.L; i += blockDim.x) twl[i] = f.tw[i];
    __syncthreads();
  }
  if (on) {
    bfly<P>(v, twl, Q);
#pragma unroll
    for (int i = 0; i < P; ++i) st(t, j, bfly_out<P>(i), v[i]);
  }
}

// stage 2: ld(t, j, m) -> Y[j][m];  st(t, m, p, v) stores X[m + P p].
// Lanes run across the 8 rows so column-strided destinations coalesce.
// POSTTW: outputs are multiplied by base * step^p, (base, step) = tw(t, m)
// (the four-step twiddle W_n^(r (m + P p)), by recurrence: no per-output gathers).
// sync_between: a block barrier between the loads and the stores (stores to
// positions other threads read).
// PC: P as a compile-time constant (0: runtime f.r1).
// mperm (optional): the m a thread group serves, mperm[idx / kFftTile] for
// idx < kFftTile * nm -- an output-pruned stage computes only the nm values
// of m whose outputs are used, packed into the first waves.
template <int Q, int PC, bool POSTTW, class Ld, class Tw, class St>
__device__ __forceinline__ void fft_stage2(const FftLen& f, const double2* twl, Ld ld, Tw tw, St st,
                                           bool sync_between, const int* mperm = nullptr, int nm = 0) {
  const int P = PC ? PC : f.r1;
  const int idx = threadIdx.x;
  const bool on = idx < kFftTile * (mperm ? nm : P);
  const int t = idx & (kFftTile - 1);
  const int m = mperm ? (on ? mperm[idx / kFftTile] : 0) : idx / kFftTile;
  double2 v[Q];
  double2 base, step;
  if (on) {
    if constexpr (POSTTW) tw(t, m, base, step);
#pragma unroll
    for (int j = 0; j < Q; ++j) v[j] = ld(t, j, m);
#pragma unroll
    for (int j = 1; j < Q; ++j) v[j] = cmul(v[j], twl[j * m]);   // W_L^(j m), j*m < L
    bfly<Q>(v, twl, P);
  }
  if (sync_between) __syncthreads();
  if (on) {
    // frequencies in order p = 0..Q-1 (slot bfly_slot(p)); each value is
    // twiddled (POSTTW: base * step^p by recurrence) right before its store
#pragma unroll
    for (int p = 0; p < Q; ++p) {
      double2 x = v[bfly_slot<Q>(p)];
      if constexpr (POSTTW) {
        x = cmul(x, base);
        base = cmul(base, step);
      }
      st(t, m, p, x);
    }
  }
}

struct NoTw {
  __device__ void operator()(int, int, double2&, double2&) const {}
};

// (PC, QC) = (P, Q) of a specialised kernel, or (0, 0): radices from f at run time.
template <bool ROWFAST, int PC, int QC, class Ld, class St>
__device__ __forceinline__ void run_stage1(const FftLen& f, double2* twl, Ld ld, St st, bool fill_twl = false) {
  if constexpr (PC > 0) {
    fft_stage1<PC, QC, ROWFAST>(f, twl, ld, st, fill_twl);
  } else {
    switch (f.r1) {
#define AMR_S1(R) \
  case R: fft_stage1<R, 0, ROWFAST>(f, twl, ld, st, fill_twl); break;
      AMR_FFT_RADICES(AMR_S1)
#undef AMR_S1
    }
  }
}

template <bool POSTTW, int PC, int QC, class Ld, class St, class Tw = NoTw>
__device__ __forceinline__ void run_stage2(const FftLen& f, const double2* twl, Ld ld, St st,
                                           bool sync_between = false, Tw tw = Tw(), const int* mperm = nullptr,
                                           int nm = 0) {
  if constexpr (QC > 0) {
    fft_stage2<QC, PC, POSTTW>(f, twl, ld, tw, st, sync_between, mperm, nm);
  } else {
    switch (f.r2) {
#define AMR_S2(R) \
  case R: fft_stage2<R, 0, POSTTW>(f, twl, ld, tw, st, sync_between, mperm, nm); break;
      AMR_FFT_RADICES(AMR_S2)
#undef AMR_S2
    }
  }
}

// Logical block of a grid whose size is a multiple of 8: consecutive logical
// blocks (neighbouring tiles of one stream, whose column-strided 128-B
// segments share HBM lines) land on the same XCD and L2 (workgroups are
// dealt to the 8 XCDs round robin; a placement assumption for speed only).
__device__ __forceinline__ int64_t xcd_block() {
  return (int64_t)(blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
}
static inline unsigned grid8(int64_t blocks) { return (unsigned)((blocks + 7) & ~(int64_t)7); }

// LDS home of the row's W_L table (after the kFftTile rows)
__device__ __forceinline__ double2* twl_of(double2* smem, const FftLen& f) { return smem + kFftTile * f.S; }

// W_n^a = W_n^(256 hi) * W_n^lo  (a < n < 2^31)
__device__ __forceinline__ double2 twn(const FftDesc& d, unsigned a) {
  return cmul(d.tw_hi[a >> 8], d.tw_lo[a & 255]);
}

// -i*sgn(k) * v for a length-n transform (scipy.signal.hilbert's h, minus the identity)
__device__ __forceinline__ double2 hilbert_mul(double2 v, int64_t k, int64_t n) {   // k < n < 2^31
  const int64_t k2 = 2 * k;
  return (k == 0 || k2 == n) ? make_double2(0.0, 0.0) : (k2 < n ? mul_mi(v) : make_double2(-v.y, v.x));
}

// |a_mark| > |a_space| with a = f + i X (np.abs = hypot): compared as squares,
// exact up to the last ulp of the envelopes; hypot where squares could overflow
__device__ __forceinline__ bool env_gt(double2 f, double2 v) {
  const double big = fmax(fmax(fabs(f.x), fabs(v.x)), fmax(fabs(f.y), fabs(v.y)));
  if (big < 1e150) return __builtin_fma(f.x, f.x, v.x * v.x) > __builtin_fma(f.y, f.y, v.y * v.y);
  return hypot(f.x, v.x) > hypot(f.y, v.y);
}

// a compare the exact path must settle: |a_mark| and |a_space| closer than
// 2 delta (delta = tau peak|x|, c = 8 delta^2 = amb_scale) -- as squares,
// (m2 - s2)^2 <= c (m2 + s2) implies |.| - |.| <= 2 delta; c < 0: never,
// c = inf or NaN envelopes: always.  Envelopes past 1e150 only occur with
// c = inf (peak > 2^400), so the squares stay finite here.
__device__ __forceinline__ bool env_ambiguous(double2 f, double2 v, double c) {
  if (c < 0.0) return false;
  const double m2 = __builtin_fma(f.x, f.x, v.x * v.x), s2 = __builtin_fma(f.y, f.y, v.y * v.y);
  const double d = m2 - s2;
  return !(d * d > c * (m2 + s2));
}

// one wave's ambiguity votes for stream b -> its flag bit (one atomic per wave that found one)
__device__ __forceinline__ void flag_ambiguous(const FftEpi& e, int64_t b, bool amb) {
  if (__ballot(amb) != 0 && (threadIdx.x & 63) == 0)
    atomicOr(&e.xflags[b >> 5], 1u << (unsigned)(b & 31));
}

template <int MODE>
__device__ __forceinline__ void fft_epilogue(const FftEpi& e, double2* __restrict__ dst, int64_t b, int64_t k,
                                             double2 v) {
  const size_t o = (size_t)b * e.n + k;
  switch (MODE) {
    case kHilbert: dst[o] = hilbert_mul(v, k, e.n); break;
    case kEnvOut: {
      const double2 f = e.z[o];
      dst[o] = make_double2(hypot(f.x, v.x), hypot(f.y, v.y));
      break;
    }
    case kMulTab: dst[o] = cmul(v, e.tab[k]); break;
    default: dst[o] = v; break;
  }
}

// ---- column pass: in[b][j1 + n1*j2] -> T[b][k2*n1 + j1] = W_n^(j1 k2) * DFT_n2 ----
template <bool CONJ_IN, int PC, int QC>
__global__ __launch_bounds__(kFftThreads) void k_fft_cols(const double2* __restrict__ in, double2* __restrict__ out,
                                                         FftDesc d, int64_t batch) {
  extern __shared__ __attribute__((aligned(16))) double2 smem[];
  const int tiles = (d.n1 + kFftTile - 1) / kFftTile;
  const int64_t lb = xcd_block();
  const int64_t b = lb / tiles;
  const int j1_0 = (int)(lb - b * tiles) * kFftTile;
  if (b >= batch) return;
  const FftLen& f = d.a;
  const int P = PC ? PC : f.r1, Q = QC ? QC : f.r2;
  const int S = PC ? fft_row_stride(PC, QC) : f.S, Qp = fft_block(Q);
  const int n1 = d.n1;
  const double2* __restrict__ src = in + (size_t)b * d.n + j1_0;
  double2* __restrict__ dst = out + (size_t)b * d.n + j1_0;
  const int ncol = min(kFftTile, d.n1 - j1_0);
  double2* twl = twl_of(smem, f);
  run_stage1<false, PC, QC>(
      f, twl,
      [&](int t, int j, int q) {
        const double2 v = t < ncol ? src[(unsigned)(t + n1 * (j + Q * q))] : make_double2(0.0, 0.0);
        return CONJ_IN ? conj2(v) : v;
      },
      [&](int t, int j, int m, double2 v) { smem[t * S + j + Qp * m] = v; }, true);
  __syncthreads();
  run_stage2<true, PC, QC>(
      f, twl, [&](int t, int j, int m) { return smem[t * S + j + Qp * m]; },
      [&](int t, int m, int p, double2 v) {
        if (t < ncol) dst[(unsigned)(t + n1 * (m + P * p))] = v;
      },
      false,
      [&](int t, int m, double2& base, double2& step) {   // W_n^(j1 (m + P p))
        base = twn(d, (unsigned)((j1_0 + t) * m));
        step = twn(d, (unsigned)((j1_0 + t) * P));
      });
}

// ---- middle pass of a filter: rows k2 of T (length n1) -> X[k2 + n2*k1] ->
// Y = mid(X) -> conj -> DFT_n1 over k1 -> k2', times W_n^(k2 k2') ->
// T'[k2'*n2 + k2]  (the column pass of FFT(conj Y) with n = n2 * n1) --------
template <int MID, int PC, int QC>
__global__ __launch_bounds__(kFftThreads) void k_fft_mid(const double2* __restrict__ in, double2* __restrict__ out,
                                                        FftDesc d, int64_t batch, const double2* __restrict__ tab) {
  extern __shared__ __attribute__((aligned(16))) double2 smem[];
  const int tiles = (d.n2 + kFftTile - 1) / kFftTile;
  const int64_t lb = xcd_block();
  const int64_t b = lb / tiles;
  const int r0 = (int)(lb - b * tiles) * kFftTile;
  if (b >= batch) return;
  const FftLen& f = d.c;
  const int P = PC ? PC : f.r1, Q = QC ? QC : f.r2, L = P * Q;
  const int S = PC ? fft_row_stride(PC, QC) : f.S, Qp = fft_block(Q);
  const int64_t n = d.n;
  const int n2 = d.n2;
  const int nrow = min(kFftTile, d.n2 - r0);
  const double2* __restrict__ src = in + (size_t)b * n + (size_t)r0 * L;
  double2* __restrict__ dst = out + (size_t)b * n + r0;
  auto y_ld = [&](int t, int j, int m) { return smem[t * S + j + Qp * m]; };
  auto y_st = [&](int t, int j, int m, double2 v) { smem[t * S + j + Qp * m] = v; };
  double2* twl = twl_of(smem, f);
  // forward row DFT; its outputs X[k1], k1 = m + P p, stay in registers ...
  run_stage1<true, PC, QC>(
      f, twl,
      [&](int t, int j, int q) { return t < nrow ? src[(unsigned)(t * L + j + Q * q)] : make_double2(0.0, 0.0); },
      y_st, true);
  __syncthreads();
  // ... and go back to LDS in natural order (element c = k1 at j = c % Q,
  // q = c / Q) once every thread has read its stage-2 inputs
  run_stage2<false, PC, QC>(
      f, twl, y_ld,
      [&](int t, int m, int p, double2 v) {
        const int c = m + P * p;
        const unsigned k = (unsigned)(r0 + t + n2 * c);
        if (MID == kHilbert)
          v = hilbert_mul(v, k, n);
        else
          v = t < nrow ? cmul(v, tab[k]) : make_double2(0.0, 0.0);
        const int qq = QC ? c / QC : fdiv(c, f.inv_r2);
        smem[t * S + (c - Q * qq) + Qp * qq] = conj2(v);
      },
      true);
  __syncthreads();
  // forward row DFT of conj(Y) (stage 1 in place), then the twiddle to T'
  run_stage1<false, PC, QC>(f, twl, y_ld, y_st);
  __syncthreads();
  run_stage2<true, PC, QC>(
      f, twl, y_ld,
      [&](int t, int m, int p, double2 v) {
        if (t < nrow) dst[(unsigned)(t + n2 * (m + P * p))] = v;
      },
      false,
      [&](int t, int m, double2& base, double2& step) {   // W_n^(k2 (m + P p))
        base = twn(d, (unsigned)((r0 + t) * m));
        step = twn(d, (unsigned)((r0 + t) * P));
      });
}

// ---- row pass: rows r of in (length f.L, nrow rows) -> DFT -> out index
// r + nrow*k; CONJ_OUT conjugates and scales (inverse); then the epilogue --
template <bool CONJ_OUT, int MODE, int PC, int QC>
__global__ __launch_bounds__(kFftThreads) void k_fft_rows(const double2* __restrict__ in, double2* __restrict__ out,
                                                         FftLen f, int nrow_all, int64_t n, int64_t batch,
                                                         double scale, FftEpi e) {
  extern __shared__ __attribute__((aligned(16))) double2 smem[];
  const int tiles = (nrow_all + kFftTile - 1) / kFftTile;
  const int64_t lb = xcd_block();
  const int64_t b = lb / tiles;
  const int r0 = (int)(lb - b * tiles) * kFftTile;
  if (b >= batch) return;
  const int P = PC ? PC : f.r1, Q = QC ? QC : f.r2, L = P * Q;
  const int S = PC ? fft_row_stride(PC, QC) : f.S, Qp = fft_block(Q);
  const int nrow = min(kFftTile, nrow_all - r0);
  const double2* __restrict__ src = in + (size_t)b * n + (size_t)r0 * L;
  double2* twl = twl_of(smem, f);
  // kEnvelope with compile-time radices: the z values the epilogue compares
  // against are loaded first, so their latency overlaps the row loads'
  // instead of following the whole transform (thread (t, m) of stage 2
  // produces kk = m + P*p, p < Q)
  constexpr bool kPre = MODE == kEnvelope && QC > 0;
  double2 zp[kPre ? QC : 1];
  const double ambc = (MODE == kEnvelope && e.amb) ? e.amb[b] : -1.0;
  if constexpr (kPre) {
    const int t = threadIdx.x & (kFftTile - 1), m = threadIdx.x / kFftTile;
    if (threadIdx.x < kFftTile * PC && t < nrow) {
      const double2* __restrict__ zr = e.z + (size_t)b * n + (unsigned)(r0 + t);
#pragma unroll
      for (int p = 0; p < QC; ++p) zp[p] = zr[(unsigned)(nrow_all * (m + PC * p))];
    }
  }
  run_stage1<true, PC, QC>(
      f, twl,
      [&](int t, int j, int q) { return t < nrow ? src[(unsigned)(t * L + j + Q * q)] : make_double2(0.0, 0.0); },
      [&](int t, int j, int m, double2 v) { smem[t * S + j + Qp * m] = v; }, true);
  __syncthreads();
  run_stage2<false, PC, QC>(
      f, twl, [&](int t, int j, int m) { return smem[t * S + j + Qp * m]; },
      [&](int t, int m, int p, double2 v) {
        const int kk = m + P * p;
        if constexpr (MODE == kEnvelope) {
          // 8 lanes (t = 0..7) of one kk -> one byte of compare bits
          bool gt = false, amb = false;
          if (t < nrow) {
            v = make_double2(v.x * scale, -v.y * scale);
            const double2 f = kPre ? zp[p] : e.z[(size_t)b * n + (unsigned)(r0 + t + nrow_all * kk)];
            gt = env_gt(f, v);
            if (e.amb) amb = env_ambiguous(f, v, ambc);
          }
          if (e.amb) flag_ambiguous(e, b, amb);
          const uint64_t mask = __ballot(gt);
          if (t == 0) e.bits[(size_t)b * e.bits_stride + (size_t)(r0 >> 3) * L + kk] = (uint8_t)(mask >> (threadIdx.x & 56));
        } else if (t < nrow) {
          if (CONJ_OUT) v = make_double2(v.x * scale, -v.y * scale);
          fft_epilogue<MODE>(e, out, b, (unsigned)(r0 + t + nrow_all * kk), v);
        }
      });
}

// ---- the Hilbert filter in the live-column layout (amr_internal.h LiveCols) --
// Per stream: zb = [L | D] (the band-pass output z, live columns then dead
// columns, rows j2) and cb = C [nl * n2] (the live columns' transform).
//   column pass  live tiles  L -> C   (z's live columns stay intact: the
//                                      final pass reads them for |a|)
//                dead tiles  D -> D   (in place), or D -> db [nd * n2] when
//                                      the plan keeps all of z for the FSK
//                                      exact path (fsk_api.cpp keep_z)
//   middle pass  rows k2 of T from C (live c) and D (dead c); writes only
//                the live outputs k2' (no later pass reads the others), into
//                C row k2 at the live index of k2' -- the positions it read
//   final pass   live columns k2' of C (DFT_n2 down the column), conj, 1/n,
//                envelopes against z's live samples in L, compare bits
// so the middle pass writes 40 % and the final pass reads 2 x 40 % of a full
// pass at sps 10, and the plan holds 1.4 x n complex per
// stream instead of 3 x.
template <int PC, int QC>
__global__ __launch_bounds__(kFftThreads) void k_fft_cols_live(double2* zb, double2* cb, double2* db, FftDesc d,
                                                              int64_t batch, LiveCols lc) {
  extern __shared__ __attribute__((aligned(16))) double2 smem[];
  const int tl = (lc.nl + kFftTile - 1) / kFftTile, tiles = tl + (lc.nd + kFftTile - 1) / kFftTile;
  const int64_t lb = xcd_block();
  const int64_t b = lb / tiles;
  const int tile = (int)(lb - b * tiles);
  if (b >= batch) return;
  const FftLen& f = d.a;
  const int P = PC ? PC : f.r1, Q = QC ? QC : f.r2;
  const int S = PC ? fft_row_stride(PC, QC) : f.S, Qp = fft_block(Q);
  const bool live = tile < tl;
  const int c0 = (live ? tile : tile - tl) * kFftTile;
  const int rl = live ? lc.nl : lc.nd;                  // row length of this region
  const int64_t n2 = d.n2;
  // src and dst alias for the dead columns in place (db == nullptr): no __restrict__
  const double2* src = zb + (size_t)b * d.n + (live ? 0 : (size_t)lc.nl * n2) + c0;
  double2* dst = live ? cb + (size_t)b * lc.nl * n2 + c0
                      : (db ? db + (size_t)b * lc.nd * n2 : zb + (size_t)b * d.n + (size_t)lc.nl * n2) + c0;
  const int ncol = min(kFftTile, rl - c0);
  double2* twl = twl_of(smem, f);
  run_stage1<false, PC, QC>(
      f, twl,
      [&](int t, int j, int q) { return t < ncol ? src[(unsigned)(t + rl * (j + Q * q))] : make_double2(0.0, 0.0); },
      [&](int t, int j, int m, double2 v) { smem[t * S + j + Qp * m] = v; }, true);
  __syncthreads();
  run_stage2<true, PC, QC>(
      f, twl, [&](int t, int j, int m) { return smem[t * S + j + Qp * m]; },
      [&](int t, int m, int p, double2 v) {
        if (t < ncol) dst[(unsigned)(t + rl * (m + P * p))] = v;
      },
      false,
      [&](int t, int m, double2& base, double2& step) {   // W_n^(j1 (m + P p)), j1 = the column's index
        const int c = c0 + (t < ncol ? t : 0);
        const int j1 = live ? lc_live_col(lc, c) : lc_dead_col(lc, c);
        base = twn(d, (unsigned)(j1 * m));
        step = twn(d, (unsigned)(j1 * P));
      });
}

// TWG: the row's W_L table is read from global memory (L1 / scalar-cache
// resident: 4.8 KB shared by every workgroup) instead of LDS, and the position
// table is 16-bit, so four workgroups fit a CU's LDS instead of three.
// NT: threads per workgroup.  No stage runs more than 8 * 20 = 160 butterflies
// at the benchmark lengths, so NT = 192 (three waves) leaves one wave less idle
// per workgroup, and four workgroups per CU are then three waves per SIMD:
// 168 VGPRs, no spills (NT = 256 holds 128 and spills).
template <int PC, int QC, bool TWG, int NT = kFftThreads>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(TWG && PC > 0 ? (NT == kFftThreads ? 4 : 3) : 1))) void k_fft_mid_live(double2* zb, double2* cb, double2* db, FftDesc d, int64_t batch,
                                                             LiveCols lc) {
  extern __shared__ __attribute__((aligned(16))) double2 smem[];
  const int tiles = (d.n2 + kFftTile - 1) / kFftTile;
  const int64_t lb = xcd_block();
  const int64_t b = lb / tiles;
  const int r0 = (int)(lb - b * tiles) * kFftTile;
  if (b >= batch) return;
  const FftLen& f = d.c;
  const int P = PC ? PC : f.r1, Q = QC ? QC : f.r2;
  const int S = PC ? fft_row_stride(PC, QC) : f.S, Qp = fft_block(Q);
  const int64_t n = d.n;
  const int n2 = d.n2;
  const int nrow = min(kFftTile, d.n2 - r0);
  // rows k2 = r0 + t: live elements in C, dead ones in D (in place: no __restrict__)
  double2* crow = cb + (size_t)b * lc.nl * n2 + (size_t)r0 * lc.nl;
  const double2* drow = (db ? db + (size_t)b * lc.nd * n2 : zb + (size_t)b * n + (size_t)lc.nl * n2) +
                        (size_t)r0 * lc.nd;
  auto y_ld = [&](int t, int j, int m) { return smem[t * S + j + Qp * m]; };
  auto y_st = [&](int t, int j, int m, double2 v) { smem[t * S + j + Qp * m] = v; };
  // (TWG: never written -- the stage-1 fill is off)
  double2* twl = TWG ? const_cast<double2*>(f.tw) : twl_of(smem, f);
  // column c -> its live index l (>= 0) or ~(dead index d), once per workgroup
  // (the per-element form cost the pass more ALU than its FFT: 12.7 vs 10.9 ms)
  __shared__ int16_t cpos[kFftMaxL];
  for (int c = threadIdx.x; c < lc.n1; c += NT) {
    bool lv;
    const int pos = lc_col_pos(lc, c, lv);
    cpos[c] = lv ? pos : ~pos;
  }
  // the last stage's outputs m + P p: when sps divides P, column m + P p is
  // live exactly when m is, so only the live m are computed (packed into the
  // first waves; 8 of 20 at sps 10), the rest of that stage is skipped
  __shared__ int mlive[kFftMaxR];
  __shared__ int nmlive;
  if (threadIdx.x == 0) {
    const bool prune = lc.prune && P % lc.sps == 0;   // (cpos of m < P: m's own column)
    int k = 0;
    for (int m = 0; m < P; ++m)
      if (!prune || cpos[m] >= 0) mlive[k++] = m;
    nmlive = k;
  }
  __syncthreads();
  run_stage1<true, PC, QC>(
      f, twl,
      [&](int t, int j, int q) {
        if (t >= nrow) return make_double2(0.0, 0.0);
        const int pos = cpos[j + Q * q];
        return pos >= 0 ? crow[(unsigned)(t * lc.nl + pos)] : drow[(unsigned)(t * lc.nd + ~pos)];
      },
      y_st, !TWG);
  __syncthreads();
  run_stage2<false, PC, QC>(
      f, twl, y_ld,
      [&](int t, int m, int p, double2 v) {
        const int c = m + P * p;
        const unsigned k = (unsigned)(r0 + t + n2 * c);
        v = hilbert_mul(v, k, n);
        const int qq = QC ? c / QC : fdiv(c, f.inv_r2);
        smem[t * S + (c - Q * qq) + Qp * qq] = conj2(v);
      },
      true);
  __syncthreads();
  run_stage1<false, PC, QC>(f, twl, y_ld, y_st);
  __syncthreads();
  run_stage2<true, PC, QC>(
      f, twl, y_ld,
      [&](int t, int m, int p, double2 v) {
        const int pos = cpos[m + P * p];                    // output k2' = m + P p
        if (t < nrow && pos >= 0) crow[(unsigned)(t * lc.nl + pos)] = v;
      },
      false,
      [&](int t, int m, double2& base, double2& step) {   // W_n^(k2 (m + P p))
        base = twn(d, (unsigned)((r0 + t) * m));
        step = twn(d, (unsigned)((r0 + t) * P));
      },
      mlive, nmlive);
}

// final pass: live columns l0 .. l0+7 of C (length n2 each, stride nl) ->
// DFT, conj, 1/n -> compare against z's live samples (L) -> bits, byte
// (l0 / 8) * n2 + k1' (the decide kernel's live addressing)
template <int PC, int QC>
__global__ __launch_bounds__(kFftThreads) void k_fft_rows_live(const double2* __restrict__ zb,
                                                              const double2* __restrict__ cb, FftDesc d,
                                                              int64_t batch, double scale, FftEpi e, LiveCols lc) {
  extern __shared__ __attribute__((aligned(16))) double2 smem[];
  const int tiles = (lc.nl + kFftTile - 1) / kFftTile;
  const int64_t lb = xcd_block();
  const int64_t b = lb / tiles;
  const int l0 = (int)(lb - b * tiles) * kFftTile;
  if (b >= batch) return;
  const FftLen& f = d.a;
  const int P = PC ? PC : f.r1, Q = QC ? QC : f.r2, L = P * Q;
  const int S = PC ? fft_row_stride(PC, QC) : f.S, Qp = fft_block(Q);
  const int nl = lc.nl;
  const int ncol = min(kFftTile, nl - l0);
  const double2* __restrict__ src = cb + (size_t)b * nl * d.n2 + l0;
  const double2* __restrict__ zl = zb + (size_t)b * d.n + l0;     // L: [k1'][l]
  double2* twl = twl_of(smem, f);
  const double ambc = e.amb ? e.amb[b] : -1.0;
  constexpr bool kPre = QC > 0;
  double2 zp[kPre ? QC : 1];
  if constexpr (kPre) {
    const int t = threadIdx.x & (kFftTile - 1), m = threadIdx.x / kFftTile;
    if (threadIdx.x < kFftTile * PC && t < ncol) {
#pragma unroll
      for (int p = 0; p < QC; ++p) zp[p] = zl[(unsigned)(t + nl * (m + PC * p))];
    }
  }
  run_stage1<false, PC, QC>(
      f, twl,
      [&](int t, int j, int q) { return t < ncol ? src[(unsigned)(t + nl * (j + Q * q))] : make_double2(0.0, 0.0); },
      [&](int t, int j, int m, double2 v) { smem[t * S + j + Qp * m] = v; }, true);
  __syncthreads();
  run_stage2<false, PC, QC>(
      f, twl, [&](int t, int j, int m) { return smem[t * S + j + Qp * m]; },
      [&](int t, int m, int p, double2 v) {
        const int kk = m + P * p;
        bool gt = false, amb = false;
        if (t < ncol) {
          v = make_double2(v.x * scale, -v.y * scale);
          const double2 f = kPre ? zp[p] : zl[(unsigned)(t + nl * kk)];
          gt = env_gt(f, v);
          if (e.amb) amb = env_ambiguous(f, v, ambc);
        }
        if (e.amb) flag_ambiguous(e, b, amb);
        const uint64_t mask = __ballot(gt);
        if (t == 0) e.bits[(size_t)b * e.bits_stride + (size_t)(l0 >> 3) * L + kk] = (uint8_t)(mask >> (threadIdx.x & 56));
      });
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

// Bluestein post + envelope compare, plain bit order: thread = (stream, byte)
__global__ __launch_bounds__(256) void k_bs_post_env(const double2* __restrict__ y, const double2* __restrict__ w,
                                                     int64_t n, int64_t M, int64_t batch, double scale, FftEpi e) {
  const int64_t nbytes = (n + 7) >> 3;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= batch * nbytes) return;
  const int64_t b = i / nbytes, jb = i - b * nbytes;
  unsigned byte = 0;
  bool amb = false;
  const double ambc = e.amb ? e.amb[b] : -1.0;
  for (int u = 0; u < 8; ++u) {
    const int64_t k = jb * 8 + u;
    if (k >= n) break;
    double2 v = cmul(y[(size_t)b * M + k], conj2(w[k]));
    v = make_double2(v.x * scale, -v.y * scale);
    const double2 f = e.z[(size_t)b * n + k];
    byte |= (env_gt(f, v) ? 1u : 0u) << u;
    amb = amb || env_ambiguous(f, v, ambc);
  }
  e.bits[(size_t)b * e.bits_stride + jb] = (uint8_t)byte;
  if (amb) atomicOr(&e.xflags[b >> 5], 1u << (unsigned)(b & 31));   // rows vary across the wave
}

static size_t fft_smem_bytes(const FftLen& f) { return ((size_t)kFftTile * f.S + f.L) * sizeof(double2); }

// Specialised (P, Q) instantiations (compile-time radices: immediate LDS and
// HBM offsets, fewer live registers) for the lengths of the benchmark
// streams (96000 = 300 * 320, 300 = 20 * 15, 320 = 20 * 16); everything else
// runs the generic kernels (radices switched at run time).
#define AMR_FFT_PQ(f, CALL)                      \
  do {                                           \
    if ((f).r1 == 20 && (f).r2 == 16) {          \
      CALL(20, 16);                              \
    } else if ((f).r1 == 20 && (f).r2 == 15) {   \
      CALL(20, 15);                              \
    } else {                                     \
      CALL(0, 0);                                \
    }                                            \
  } while (0)

hipError_t launch_fft(const double2* in, double2* tmp, double2* out, const FftDesc& d, int64_t batch, bool inverse,
                      hipStream_t st) {
  const unsigned gcol = grid8(batch * ((d.n1 + kFftTile - 1) / kFftTile));
  const unsigned grow = grid8(batch * ((d.n2 + kFftTile - 1) / kFftTile));
  FftEpi e{};
  e.mode = kStore;
  e.n = d.n;
  const double scale = inverse ? 1.0 / (double)d.n : 1.0;
#define COLS(P, Q)                                                                                               \
  hipLaunchKernelGGL((k_fft_cols<true, P, Q>), dim3(gcol), dim3(kFftThreads), fft_smem_bytes(d.a), st, in, tmp, d, \
                     batch)
#define COLSF(P, Q)                                                                                               \
  hipLaunchKernelGGL((k_fft_cols<false, P, Q>), dim3(gcol), dim3(kFftThreads), fft_smem_bytes(d.a), st, in, tmp, d, \
                     batch)
#define ROWS(P, Q)                                                                                            \
  hipLaunchKernelGGL((k_fft_rows<true, kStore, P, Q>), dim3(grow), dim3(kFftThreads), fft_smem_bytes(d.c), st, \
                     tmp, out, d.c, d.n2, d.n, batch, scale, e)
#define ROWSF(P, Q)                                                                                            \
  hipLaunchKernelGGL((k_fft_rows<false, kStore, P, Q>), dim3(grow), dim3(kFftThreads), fft_smem_bytes(d.c), st, \
                     tmp, out, d.c, d.n2, d.n, batch, scale, e)
  if (inverse) {
    AMR_FFT_PQ(d.a, COLS);
    AMR_FFT_PQ(d.c, ROWS);
  } else {
    AMR_FFT_PQ(d.a, COLSF);
    AMR_FFT_PQ(d.c, ROWSF);
  }
#undef COLS
#undef COLSF
#undef ROWS
#undef ROWSF
  return hipGetLastError();
}

hipError_t launch_fft_filter(const double2* in, double2* t1, double2* t2, double2* out, const FftDesc& d,
                             int64_t batch, int mid, const double2* tab, const FftEpi& epi, hipStream_t st) {
  const unsigned gcol = grid8(batch * ((d.n1 + kFftTile - 1) / kFftTile));
  const unsigned gmid = grid8(batch * ((d.n2 + kFftTile - 1) / kFftTile));
  const unsigned gfin = grid8(batch * ((d.n1 + kFftTile - 1) / kFftTile));
  if (mid != kHilbert && mid != kMulTab) return hipErrorInvalidValue;
  if (epi.mode != kStore && epi.mode != kEnvelope && epi.mode != kEnvOut) return hipErrorInvalidValue;
#define COLSF(P, Q)                                                                                              \
  hipLaunchKernelGGL((k_fft_cols<false, P, Q>), dim3(gcol), dim3(kFftThreads), fft_smem_bytes(d.a), st, in, t1, d, \
                     batch)
  AMR_FFT_PQ(d.a, COLSF);
#undef COLSF
#define MIDK(P, Q)                                                                                                  \
  do {                                                                                                              \
    if (mid == kHilbert)                                                                                            \
      hipLaunchKernelGGL((k_fft_mid<kHilbert, P, Q>), dim3(gmid), dim3(kFftThreads), fft_smem_bytes(d.c), st, t1, \
                         t2, d, batch, tab);                                                                        \
    else                                                                                                            \
      hipLaunchKernelGGL((k_fft_mid<kMulTab, P, Q>), dim3(gmid), dim3(kFftThreads), fft_smem_bytes(d.c), st, t1,  \
                         t2, d, batch, tab);                                                                        \
  } while (0)
  AMR_FFT_PQ(d.c, MIDK);
#undef MIDK
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) return err;
  // final row pass: the n1 rows k2' of T' (length n2) -> index k2' + n1*k1', conj, 1/n
  FftEpi e = epi;
  e.n = d.n;
  const double scale = 1.0 / (double)d.n;
  const size_t sm = fft_smem_bytes(d.a);
#define FIN(P, Q)                                                                                                  \
  do {                                                                                                             \
    if (epi.mode == kStore)                                                                                        \
      hipLaunchKernelGGL((k_fft_rows<true, kStore, P, Q>), dim3(gfin), dim3(kFftThreads), sm, st, t2, out, d.a,  \
                         d.n1, d.n, batch, scale, e);                                                              \
    else if (epi.mode == kEnvelope)                                                                                \
      hipLaunchKernelGGL((k_fft_rows<true, kEnvelope, P, Q>), dim3(gfin), dim3(kFftThreads), sm, st, t2, out,    \
                         d.a, d.n1, d.n, batch, scale, e);                                                         \
    else                                                                                                           \
      hipLaunchKernelGGL((k_fft_rows<true, kEnvOut, P, Q>), dim3(gfin), dim3(kFftThreads), sm, st, t2, out, d.a, \
                         d.n1, d.n, batch, scale, e);                                                              \
  } while (0)
  AMR_FFT_PQ(d.a, FIN);
#undef FIN
  return hipGetLastError();
}

// The Hilbert filter + envelope compare of launch_fft_filter (kHilbert,
// kEnvelope) in the live-column layout: zb = [B][L | D] (z), cb = [B][nl * n2].
hipError_t launch_fft_hilbert_live(double2* zb, double2* cb, double2* db, const FftDesc& d, int64_t batch,
                                   const LiveCols& lc, const FftEpi& epi, hipStream_t st) {
  if (!lc.on || epi.mode != kEnvelope) return hipErrorInvalidValue;
  const int tl = (lc.nl + kFftTile - 1) / kFftTile, td = (lc.nd + kFftTile - 1) / kFftTile;
  const unsigned gcol = grid8(batch * (tl + td));
  const unsigned gmid = grid8(batch * ((d.n2 + kFftTile - 1) / kFftTile));
  const unsigned gfin = grid8(batch * tl);
  const double scale = 1.0 / (double)d.n;
  // (the column and final passes stay four-wave: three-wave workgroups
  // measured slower for them)
#define COLSL(P, Q) \
  hipLaunchKernelGGL((k_fft_cols_live<P, Q>), dim3(gcol), dim3(kFftThreads), fft_smem_bytes(d.a), st, zb, cb, db, d, batch, \
                     lc)
  AMR_FFT_PQ(d.a, COLSL);
#undef COLSL
  // AMR_FFT_MID_TWG=0: the W_L table in LDS (three workgroups per CU instead of four)
  static const bool twg = [] { const char* e = getenv("AMR_FFT_MID_TWG"); return !(e && e[0] == '0'); }();
  // three-wave workgroups (specialised lengths, TWG form; AMR_FFT_MID_NT=256:
  // four waves): solo Hilbert 23.6 -> 22.6 ms, fsk9600 step 33.2 -> 32.5 ms
  static const bool nt192 = [] { const char* e = getenv("AMR_FFT_MID_NT"); return !e || atoi(e) != 256; }();
  const size_t sm_mid = twg ? (size_t)kFftTile * d.c.S * sizeof(double2) : fft_smem_bytes(d.c);
#define MIDL(P, Q)                                                                                              \
  do {                                                                                                          \
    if (twg && nt192 && P > 0 && kFftTile * d.c.r1 <= 192 && kFftTile * d.c.r2 <= 192)                          \
      hipLaunchKernelGGL((k_fft_mid_live<P, Q, true, 192>), dim3(gmid), dim3(192), sm_mid, st, zb, cb, db, d,  \
                         batch, lc);                                                                            \
    else if (twg)                                                                                               \
      hipLaunchKernelGGL((k_fft_mid_live<P, Q, true>), dim3(gmid), dim3(kFftThreads), sm_mid, st, zb, cb, db, \
                         d, batch, lc);                                                                            \
    else                                                                                                        \
      hipLaunchKernelGGL((k_fft_mid_live<P, Q, false>), dim3(gmid), dim3(kFftThreads), sm_mid, st, zb, cb, db, \
                         d, batch, lc);                                                                            \
  } while (0)
  AMR_FFT_PQ(d.c, MIDL);
#undef MIDL
#define FINL(P, Q)                                                                                          \
  hipLaunchKernelGGL((k_fft_rows_live<P, Q>), dim3(gfin), dim3(kFftThreads), fft_smem_bytes(d.a), st, zb, cb, d, \
                     batch, scale, epi, lc)
  AMR_FFT_PQ(d.a, FINL);
#undef FINL
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
    case kEnvelope: {
      if (!inverse) return hipErrorInvalidValue;
      const int64_t tb = batch * ((n + 7) >> 3);
      hipLaunchKernelGGL(k_bs_post_env, dim3((unsigned)((tb + 255) / 256)), dim3(256), 0, st, y, w, n, M, batch,
                         scale, epi);
      break;
    }
    case kEnvOut: hipLaunchKernelGGL(k_bs_post<kEnvOut>, g, dim3(256), 0, st, y, out, w, n, M, batch, inv, scale, epi); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---- six-step pieces (lengths past the two-pass limit, fsk_api.cpp) ---------
// out[b][c][r] = in[b][r][c] (* W_M^(+-r c) when tw_lo), a 32 x 32 tile through
// LDS (odd pitch: column reads hit distinct banks).  r*c < M by construction.
__global__ __launch_bounds__(256) void k_transpose_tw(const double2* __restrict__ in, double2* __restrict__ out,
                                                      int64_t R, int64_t C, const double2* __restrict__ tw_lo,
                                                      const double2* __restrict__ tw_hi, int inv) {
  __shared__ double2 tile[32][33];
  const int64_t b = blockIdx.z;
  const int64_t r0 = (int64_t)blockIdx.y * 32, c0 = (int64_t)blockIdx.x * 32;
  const double2* __restrict__ src = in + (size_t)b * R * C;
  double2* __restrict__ dst = out + (size_t)b * R * C;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int64_t r = r0 + ty + k, c = c0 + tx;
    if (r < R && c < C) {
      double2 v = src[(size_t)r * C + c];
      if (tw_lo) {
        const uint64_t a = (uint64_t)r * (uint64_t)c;
        double2 w = cmul(tw_hi[a >> 8], tw_lo[a & 255]);
        if (inv) w = conj2(w);
        v = cmul(v, w);
      }
      tile[ty + k][tx] = v;
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int64_t c = c0 + ty + k, r = r0 + tx;
    if (r < R && c < C) dst[(size_t)c * R + r] = tile[tx][ty + k];
  }
}

hipError_t launch_transpose(const double2* in, double2* out, int64_t R, int64_t C, int64_t batch,
                            const double2* tw_lo, const double2* tw_hi, bool inverse, hipStream_t st) {
  if (batch <= 0 || R <= 0 || C <= 0) return hipSuccess;
  const dim3 g((unsigned)((C + 31) / 32), (unsigned)((R + 31) / 32), (unsigned)batch);
  hipLaunchKernelGGL(k_transpose_tw, g, dim3(256), 0, st, in, out, R, C, tw_lo, tw_hi, inverse ? 1 : 0);
  return hipGetLastError();
}


template <int P, int Q>
static hipError_t fft_set_smem(int bytes) {
  const void* fns[] = {
      (const void*)k_fft_cols<false, P, Q>, (const void*)k_fft_cols<true, P, Q>,
      (const void*)k_fft_mid<kHilbert, P, Q>, (const void*)k_fft_mid<kMulTab, P, Q>,
      (const void*)k_fft_rows<false, kStore, P, Q>, (const void*)k_fft_rows<true, kStore, P, Q>,
      (const void*)k_fft_rows<true, kEnvelope, P, Q>, (const void*)k_fft_rows<true, kEnvOut, P, Q>,
      (const void*)k_fft_cols_live<P, Q>, (const void*)k_fft_mid_live<P, Q, false>,
      (const void*)k_fft_mid_live<P, Q, true>, (const void*)k_fft_mid_live<P, Q, true, 192>,
      (const void*)k_fft_rows_live<P, Q>};
  for (const void* f : fns) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t fft_configure_smem() {
  const int bytes = (kFftTile * fft_row_stride(kFftMaxR, kFftMaxR) + kFftMaxL) * (int)sizeof(double2);
  hipError_t e = fft_set_smem<0, 0>(bytes);
  if (e == hipSuccess) e = fft_set_smem<20, 16>(bytes);
  if (e == hipSuccess) e = fft_set_smem<20, 15>(bytes);
  return e;
}

}  // namespace amr
