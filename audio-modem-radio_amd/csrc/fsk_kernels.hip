// fsk_kernels.hip -- batched FSK demodulation for gfx950.
//
// Replaces, for a batch of equal-length streams, the reference
//   modem.fsk_demodulate  (/root/reference/modem.py:298-341)
// (and its aliases fsk_high_speed_demodulate modem.py:355-356,
//  ft8_demodulate modem.py:391, decoder.py:426-432).
//
// Per stream:                                              reference
//   f_t   = filtfilt(butter(3, [(t-b)/nyq, (t+b)/nyq]), x)  modem.py:307-308
//   env_t = |hilbert(f_t)|                                  modem.py:309
//   bit_i = env_mark_i > env_space_i                        modem.py:315
//   decided bit per symbol = majority over bits[i-q, i+q)   modem.py:320-323
//   sync on "FB", pack MSB first from idx or 0              modem.py:326-341
//
// Kernels:
//   F1 k_fsk_bandpass  lane = (stream, tone): both band-pass filtfilts, output
//                      packed as the complex signal z = f_mark + i f_space,
//                      stream-major.
//   F2 (fft_kernels.hip) H[z] = IFFT(-i sgn(k) FFT(z)) = H[f_mark] + i H[f_space]
//                      (the Hilbert transform is real-linear, so one complex
//                      transform pair serves both tones); its last pass forms
//                      both envelopes hypot(f, H f) and packs the compare bits.
//   F3 k_fsk_decide    thread = (stream, bit): window majority, ballot-packed
//                      MSB first into words (then k_sync_pack, util_kernels.hip)
// Parity: the FFT cannot reproduce pocketfft's rounding; envelopes agree to
// ~1e-15 relative and decisions are compared bit for bit with the reference
// (tests/test_gpu_parity.py), with the envelope tolerance stated there.
#include <algorithm>
#include <cstdlib>

#include "amr_internal.h"
#include "odd_ext.h"
#include "split_chain.h"

namespace amr {

// the input's conversion and odd extension: In<T> / OddExt<T> (odd_ext.h)

// lfilter step (DF-II-T), 7 taps, per-lane coefficients, in scipy's own
// operation order (scipy.signal.lfilter's real DF-II-T loop, no contraction):
//   y = z0 + b0*x ; z[i] = (z[i+1] + x*b[i+1]) - y*a[i+1] ; z[5] = x*b6 - y*a6
// so the band-pass output f equals scipy's filtfilt bit for bit (the odd
// extension in the input's precision, zi * x0 and the checkpointed re-runs
// are exact too), and the envelopes differ from the reference's only by
// the FFTs' rounding -- the margin F2's exact-path flags are sized for.
// ZO (MODE 1): the plan's b1 = b3 = b5 = 0 exactly for both tones (always so
// for butter(3, band): b is k * poly([1,1,1,-1,-1,-1]) = k * [1,0,-3,0,3,0,-1]);
// then (z + x*0) == z for every z != 0 and those three products and sums are
// dropped (19 FP64 operations per step instead of 25; only the sign of an
// exact zero state can differ, which no envelope |.| sees).
// MODE 3: ZO and, as butter(3, band) always has (the plan checks), an
// antisymmetric numerator b6 = -b0, b4 = -b2 bit for bit: x*b6 IS -(x*b0),
// so z5 = x*b6 - y*a6 is (-(x*b0)) - y*a6 = -(x*b0) - y*a6 exactly, and
// z4 + x*b4 is z4 - x*b2: two products per step instead of four (17 FP64).
// MODE 2 (AMR_FSK_F1_FMA=1, a timing A/B only): the round-3 contracted form
// (10 FMAs per step), whose f is NOT scipy's -- its rounding grows with the
// band-pass filter's noise gain (~1e-10 of the peak at 1200 Bd), beyond the
// exact path's margin.
template <int MODE>
__device__ __forceinline__ double fsk_step(double (&z)[6], const double (&b)[7], const double (&a)[7], double x) {
  if constexpr (MODE == 2) {
    const double y = __builtin_fma(b[0], x, z[0]);
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const double zin = ((i & 1) == 0) ? z[i + 1] : __builtin_fma(x, b[i + 1], z[i + 1]);
      z[i] = __builtin_fma(-y, a[i + 1], zin);
    }
    z[5] = __builtin_fma(-y, a[6], x * b[6]);
    return y;
  } else if constexpr (MODE == 3) {
    const double xb0 = x * b[0], xb2 = x * b[2];
    const double y = z[0] + xb0;
    z[0] = z[1] - y * a[1];
    z[1] = (z[2] + xb2) - y * a[2];
    z[2] = z[3] - y * a[3];
    z[3] = (z[4] - xb2) - y * a[4];
    z[4] = z[5] - y * a[5];
    z[5] = -xb0 - y * a[6];
    return y;
  } else {
    const double y = z[0] + b[0] * x;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const double zin = (MODE == 1 && (i & 1) == 0) ? z[i + 1] : z[i + 1] + x * b[i + 1];
      z[i] = zin - y * a[i + 1];
    }
    z[5] = x * b[6] - y * a[6];
    return y;
  }
}

typedef unsigned v4u __attribute__((ext_vector_type(4)));   // native vector (HIP's uint4 is a struct)

// F1's input peak, for F2's ambiguity margin (amr_internal.h amb_scale,
// fsk_exact_kernels.hip): max |x| over the stream on the raw bits (integer
// work; NaN / inf dominate every finite value)
template <typename T> struct PeakT;
template <> struct PeakT<float> {
  static __device__ void acc(v4u v, uint32_t& hi, uint32_t&) {
    const uint32_t m = 0x7fffffffu;
    hi = max(hi, max(max(v.x & m, v.y & m), max(v.z & m, v.w & m)));
  }
  static __device__ void one(float x, uint32_t& hi, uint32_t&) { hi = max(hi, __float_as_uint(x) & 0x7fffffffu); }
  static __device__ double peak(uint32_t hi, uint32_t) { return (double)__uint_as_float(hi); }
};
template <> struct PeakT<double> {
  // hi: the largest |x| high word; lo: the low words OR-ed (denormals)
  static __device__ void acc(v4u v, uint32_t& hi, uint32_t& lo) {
    hi = max(hi, max(v.y & 0x7fffffffu, v.w & 0x7fffffffu));
    lo |= v.x | v.z;
  }
  static __device__ void one(double x, uint32_t& hi, uint32_t& lo) {
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    hi = max(hi, (uint32_t)(b >> 32) & 0x7fffffffu);
    lo |= (uint32_t)b;
  }
  // an upper bound (low word all ones); 0 only for a stream of exact zeros
  static __device__ double peak(uint32_t hi, uint32_t lo) {
    if (hi == 0 && lo == 0) return 0.0;
    return __hiloint2double((int)hi, (int)0xffffffffu);
  }
};
template <> struct PeakT<int16_t> {
  static __device__ uint32_t a2(uint32_t w) {
    const int l = (int)(int16_t)(w & 0xffffu), h = (int)w >> 16;
    return (uint32_t)max(abs(l), abs(h));
  }
  static __device__ void acc(v4u v, uint32_t& hi, uint32_t&) {
    hi = max(hi, max(max(a2(v.x), a2(v.y)), max(a2(v.z), a2(v.w))));
  }
  static __device__ void one(int16_t x, uint32_t& hi, uint32_t&) { hi = max(hi, (uint32_t)abs((int)x)); }
  static __device__ double peak(uint32_t hi, uint32_t) { return (double)hi / 32768.0; }
};


constexpr int kFskTile = 64;          // samples per input tile (and per checkpoint)

// F1 scratch, per wave: checkpoints ck[tile][6 states][64 lanes] doubles, then
// the forward outputs of the tail (the last n % 64 samples and the right
// extension) tl[j][64 lanes].
__host__ __device__ inline int64_t fsk_tail_len(int64_t n, int pad) { return n % kFskTile + pad; }
__host__ __device__ inline int64_t fsk_scratch_doubles_per_wave(int64_t n, int pad) {
  return ((n / kFskTile) * 6 + fsk_tail_len(n, pad)) * 64;
}

// F1.  wave = 32 streams x 2 tones (lane = 2*stream + tone), checkpointed
// filtfilt: the forward pass keeps only each 64-sample tile's starting state
// (and the short tail's outputs); the backward pass walks the tiles top-down,
// re-runs the forward recursion of a tile from its checkpoint (bit-identical
// outputs, kept in LDS), then runs the backward recursion over them.  HBM
// traffic per sample: x twice and z once, instead of also writing and
// re-reading the forward outputs.  Input tiles are loaded 16 B
// per lane and transposed through LDS; outputs are written back into the same
// LDS slots and stored as 1 KiB rows of z (stream-major f_mark + i f_space).
// LIVE: z in the live-column layout (amr_internal.h LiveCols), else [s][i].
template <bool LIVE>
__device__ __forceinline__ int64_t fsk_zoff(const FskParams& p, int64_t i) {
  if constexpr (LIVE) return lc_zoff(p.lc, (int)i);
  else return i;
}

template <typename T, int ZO, bool LIVE, bool AMB = false>
__global__ __launch_bounds__(64) void k_fsk_bandpass(const void* xv, int64_t x_stride, int64_t n_streams,
                                                     double* __restrict__ scratch, double2* __restrict__ z,
                                                     FskParams p, FskIir f) {
  constexpr int RB = kFskTile * (int)sizeof(T);     // bytes per stream row per tile
  constexpr int PITCH = RB + 16;
  constexpr int LPR = RB / 16;                      // lanes per row in a load
  constexpr int RPI = 64 / LPR;                     // rows per load instruction
  constexpr int NI = 32 / RPI;                      // load instructions per tile
  constexpr int YP = 66;                            // yb pitch (doubles): 16-B slot (33 l + row) % 16
  __shared__ __attribute__((aligned(16))) uint8_t tin[2][32][PITCH];
  __shared__ __attribute__((aligned(16))) double yb[kFskTile][YP];   // [sample][lane]
  const int lane = threadIdx.x;
  const int tone = lane & 1, sl = lane >> 1;
  const int64_t w = blockIdx.x;
  const int64_t s = w * 32 + sl;
  const int64_t last = n_streams - 1;
  const T* __restrict__ xall = reinterpret_cast<const T*>(xv);
  const T* __restrict__ x = xall + (s < last ? s : last) * x_stride;
  const int64_t n = p.n;
  const int pad = p.pad;
  const int64_t n_tiles = n / kFskTile;
  const int64_t n_main = n_tiles * kFskTile;
  double* __restrict__ ck = scratch + (size_t)w * fsk_scratch_doubles_per_wave(n, pad) + lane;
  double* __restrict__ tl = ck + (size_t)n_tiles * 6 * 64;
  double b[7], a[7], zs[6];
#pragma unroll
  for (int i = 0; i < 7; ++i) { b[i] = f.b[tone][i]; a[i] = f.a[tone][i]; }

  const int rsub = lane / LPR, cb = (lane % LPR) * 16;
  const uint8_t* rowp[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int64_t rs = w * 32 + RPI * i + rsub;
    rowp[i] = reinterpret_cast<const uint8_t*>(xall + (rs < last ? rs : last) * x_stride) + cb;
  }
  v4u r[NI];
  auto fetch = [&](int64_t t) {
#pragma unroll
    for (int i = 0; i < NI; ++i) r[i] = *reinterpret_cast<const v4u*>(rowp[i] + t * RB);
  };
  auto deposit = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NI; ++i) *reinterpret_cast<v4u*>(&tin[buf][RPI * i + rsub][cb]) = r[i];
  };
  uint32_t pk_hi = 0, pk_lo = 0;   // AMB: the input peak (PeakT)
  // forward steps over tile `buf`; emit(k, y)
  auto run_tile = [&](int buf, auto emit, bool det = false) {
    constexpr int PER = 16 / (int)sizeof(T);
#pragma unroll
    for (int k = 0; k < kFskTile; k += PER) {
      const v4u v = *reinterpret_cast<const v4u*>(&tin[buf][sl][k * sizeof(T)]);
      if (AMB && det) PeakT<T>::acc(v, pk_hi, pk_lo);
      T xs[PER];
      __builtin_memcpy(xs, &v, 16);
#pragma unroll
      for (int u = 0; u < PER; ++u) emit(k + u, fsk_step<ZO>(zs, b, a, In<T>::cvt(xs[u])));
    }
  };

  // ---- forward pass: checkpoints only ------------------------------------
  const OddExt<T> ox(x, p.edge, s < last ? s : last, n, pad);
  const double e0 = ox.left(0);
#pragma unroll
  for (int i = 0; i < 6; ++i) zs[i] = f.zi[tone][i] * e0;
  for (int j = 0; j < pad; ++j) (void)fsk_step<ZO>(zs, b, a, ox.left(j));   // trimmed later
  if (n_tiles > 0) {
    fetch(0);
    deposit(0);
    __syncthreads();
    for (int64_t t = 0; t < n_tiles; ++t) {
      const int cur = (int)(t & 1);
      fetch(t + 1 < n_tiles ? t + 1 : t);                 // unconditional (clamped) prefetch
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 6; ++i) ck[((size_t)t * 6 + i) * 64] = zs[i];
      run_tile(cur, [](int, double) {}, true);
      __builtin_amdgcn_sched_barrier(0);
      deposit(cur ^ 1);
      __syncthreads();
    }
  }
  for (int64_t i = n_main; i < n; ++i) {
    if constexpr (AMB) PeakT<T>::one(x[i], pk_hi, pk_lo);
    tl[(size_t)(i - n_main) * 64] = fsk_step<ZO>(zs, b, a, In<T>::cvt(x[i]));
  }
  if constexpr (AMB) {
    if (tone == 0 && s < n_streams)
      p.amb[s] = p.force_exact ? __builtin_inf() : amb_scale(ox.peak_with_tab(PeakT<T>::peak(pk_hi, pk_lo)), p.tau);
    if (lane == 0) p.xflags[w] = 0u;
  }
  double ylast = 0.0;
  for (int j = 0; j < pad; ++j) {
    ylast = fsk_step<ZO>(zs, b, a, ox.right(j));
    tl[(size_t)(n - n_main + j) * 64] = ylast;
  }
  __threadfence();

  // ---- backward pass --------------------------------------------------------
#pragma unroll
  for (int i = 0; i < 6; ++i) zs[i] = f.zi[tone][i] * ylast;
  for (int64_t j = n - n_main + pad - 1; j >= n - n_main; --j) (void)fsk_step<ZO>(zs, b, a, tl[(size_t)j * 64]);
  double* __restrict__ zd = reinterpret_cast<double*>(z);
  for (int64_t i = n - 1; i >= n_main; --i) {          // tail outputs, one sample at a time
    const double y = fsk_step<ZO>(zs, b, a, tl[(size_t)(i - n_main) * 64]);
    if (s < n_streams) zd[((size_t)s * n + fsk_zoff<LIVE>(p, i)) * 2 + tone] = y;
  }
  if (n_tiles > 0) {
    double zf[6], zb[6];
    fetch(n_tiles - 1);
#pragma unroll
    for (int i = 0; i < 6; ++i) zf[i] = ck[((size_t)(n_tiles - 1) * 6 + i) * 64];
    for (int64_t t = n_tiles - 1; t >= 0; --t) {
      deposit(0);
      __syncthreads();
      const int64_t tp = t > 0 ? t - 1 : 0;
      fetch(tp);                                            // next (lower) tile, and its checkpoint
#pragma unroll
      for (int i = 0; i < 6; ++i) zb[i] = ck[((size_t)tp * 6 + i) * 64];
      __builtin_amdgcn_sched_barrier(0);
      // forward recursion of tile t from its checkpoint -> yb
      double zsave[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) { zsave[i] = zs[i]; zs[i] = zf[i]; }
      run_tile(0, [&](int k, double y) { yb[k][lane] = y; });
#pragma unroll
      for (int i = 0; i < 6; ++i) { zs[i] = zsave[i]; zf[i] = zb[i]; }
      // backward recursion over it, outputs in place
#pragma unroll 8
      for (int k = kFskTile - 1; k >= 0; --k) yb[k][lane] = fsk_step<ZO>(zs, b, a, yb[k][lane]);
      __syncthreads();
      // 32 rows x 64 samples of z, one 1 KiB row per store instruction
      const int64_t zo = fsk_zoff<LIVE>(p, t * kFskTile + lane);
#pragma unroll 4
      for (int row = 0; row < 32; ++row) {
        const int64_t so = w * 32 + row;
        const double2 v = *reinterpret_cast<const double2*>(&yb[lane][2 * row]);
        if (so < n_streams) z[(size_t)so * n + zo] = v;
      }
      __syncthreads();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// F1, role-split form (the default).  Workgroup = two waves over the same 32
// streams x 2 tones: wave 0 runs every forward recursion, wave 1 every
// backward one, so the checkpointed filtfilt's second half overlaps:
//   phase 1  wave 0: forward pass keeping each 32-sample tile's starting
//            state (global scratch) and the tail's forward outputs (LDS)
//   phase 1b wave 1: backward recursion over the right extension and the
//            tail (outputs of the last n % 32 samples straight to z)
//   phase 2  iteration i: wave 0 stores tile T+1-i (1 KiB rows of z from
//            yb[i & 1], run backward by wave 1 in iteration i-1), then re-runs
//            tile T-1-i forward from its checkpoint into yb[i & 1], while wave 1
//            runs tile T-i backward in yb[(i-1) & 1]; one block barrier per
//            iteration
// 1024 waves fill the 1024 SIMDs at B = 16384 (the one-wave form: 512), and
// phase 2 costs one recursion per sample instead of two.  Arithmetic and
// order per recursion are those of k_fsk_bandpass (same outputs).
// AMR_FSK_TILE=64 (an A/B; default 32): samples per tile.  A tile of 64 held
// 77 KB of LDS per workgroup (two re-run buffers of 64 samples x 64 lanes),
// so two F1 workgroups filled a CU's LDS and no FFT-pass workgroup could sit
// beside them; 32 halves that at twice the checkpoints (3 B per sample):
// fsk9600 37.03-37.16 -> 34.68-34.79 ms/step, and 16 (four times the
// checkpoints) measured 35.75-35.77 against 32's 35.38-35.60 on another box
// (profiles/r05_fsk_f1_tile.txt); AMR_FSK_TILE=40 (f32 / f64; the generic
// load / store mapping below) measured 35.11-35.29 vs 34.55-34.61 ms/step
constexpr int kFsk2Tile = 32;
constexpr int kFsk2TileMin = 32;
__host__ __device__ inline int64_t fsk2_scratch_doubles_per_group(int64_t n, int tl = kFsk2Tile) {
  return (n / tl) * 6 * 64;
}

template <typename T, int ZO, bool LIVE, bool W1S, bool AMB = false, int TLT = kFsk2Tile>
__global__ __launch_bounds__(128) void k_fsk_bandpass2(const void* xv, int64_t x_stride, int64_t n_streams,
                                                       double* __restrict__ scratch, double2* __restrict__ z,
                                                       FskParams p, FskIir f) {
  constexpr int TL = TLT;
  constexpr int RB = TL * (int)sizeof(T);           // bytes per stream row per tile
  constexpr int PITCH = RB + 16;
  constexpr int LPR = RB / 16;                      // 16-B segments per stream row
  constexpr int SEG = 32 * LPR;                     // segments per tile (32 rows)
  constexpr int NI = (SEG + 63) / 64;               // load instructions per tile
  static_assert(RB % 16 == 0 && SEG % 64 == 0, "a tile's rows must split into whole 64-lane loads");
  constexpr int YP = 66;                            // yb pitch (doubles)
  __shared__ __attribute__((aligned(16))) uint8_t tin[1][32][PITCH];
  // two tile buffers, or the tail's forward outputs (n % TL + pad <= TL - 1 + 21 rows)
  constexpr int YR = 2 * TL > TL + 20 ? 2 * TL : TL + 20;
  __shared__ __attribute__((aligned(16))) double yb[YR][YP];
  __shared__ double ylast_sh[64];
  const int role = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int tone = lane & 1, sl = lane >> 1;
  const int64_t w = blockIdx.x;
  const int64_t s = w * 32 + sl;
  // list mode (p.xlist, the exact path): the streams F2 flagged, by ordinal
  // (row r of z is ordinal r's, x row p.xlist[r]); the count is read here
  int64_t ns = n_streams;
  if (p.xlist) {
    const int64_t c = *p.xcount;
    ns = c < n_streams ? c : n_streams;
    if (w * 32 >= ns) return;              // whole workgroup, before any barrier
  }
  const int64_t last = ns - 1;
  const T* __restrict__ xall = reinterpret_cast<const T*>(xv);
  auto xrow_index = [&](int64_t r) -> int64_t {   // the x row (and edge row) of z row r
    const int64_t rr = r < last ? r : last;
    return p.xlist ? (int64_t)p.xlist[rr] : rr;
  };
  auto xrow = [&](int64_t r) -> const T* { return xall + xrow_index(r) * x_stride; };
  const T* __restrict__ x = xrow(s);
  const int64_t n = p.n;
  const int pad = p.pad;
  const int64_t n_tiles = n / TL;
  const int64_t n_main = n_tiles * TL;
  const int64_t ntail = n - n_main + pad;            // <= TL - 1 + 21 <= YR
  double* __restrict__ ck = scratch + (size_t)w * fsk2_scratch_doubles_per_group(n, TL) + lane;
  double b[7], a[7], zs[6];
#pragma unroll
  for (int i = 0; i < 7; ++i) { b[i] = f.b[tone][i]; a[i] = f.a[tone][i]; }
  double* __restrict__ zd = reinterpret_cast<double*>(z);

  // wave 0's input path: 16 B per lane per row segment, two register sets so
  // every load has two tiles of work to land behind (tin is this wave's own)
  // instruction i, lane l: segment g = 64 i + l of the tile = row g / LPR,
  // bytes 16 (g % LPR) (for LPR | 64: rows 64 / LPR per instruction)
  const uint8_t* rowp[NI];
  int lrow[NI], lcb[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int g = 64 * i + lane;
    lrow[i] = g / LPR;
    lcb[i] = (g % LPR) * 16;
    rowp[i] = reinterpret_cast<const uint8_t*>(xrow(w * 32 + lrow[i])) + lcb[i];
  }
  v4u r0[NI], r1[NI];
  auto fetch = [&](v4u (&r)[NI], int64_t t) {
    t = t < 0 ? 0 : (t >= n_tiles ? n_tiles - 1 : t);   // clamped: unconditional loads
#pragma unroll
    for (int i = 0; i < NI; ++i) r[i] = *reinterpret_cast<const v4u*>(rowp[i] + t * RB);
  };
  auto deposit = [&](const v4u (&r)[NI]) {
#pragma unroll
    for (int i = 0; i < NI; ++i) *reinterpret_cast<v4u*>(&tin[0][lrow[i]][lcb[i]]) = r[i];
  };
  uint32_t pk_hi = 0, pk_lo = 0;   // AMB: the input peak (PeakT), first forward pass
  auto run_tile = [&](auto emit, bool det) {
    constexpr int PER = 16 / (int)sizeof(T);
#pragma unroll
    for (int k = 0; k < TL; k += PER) {
      const v4u v = *reinterpret_cast<const v4u*>(&tin[0][sl][k * sizeof(T)]);
      if (AMB && det) PeakT<T>::acc(v, pk_hi, pk_lo);
      T xs[PER];
      __builtin_memcpy(xs, &v, 16);
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const double xv = In<T>::cvt(xs[u]);
        emit(k + u, fsk_step<ZO>(zs, b, a, xv));
      }
    }
  };
  if (role == 0) {
    // ---- phase 1: forward pass, checkpoints only
    const OddExt<T> ox(x, p.edge, xrow_index(s), n, pad);
    const double e0 = ox.left(0);
#pragma unroll
    for (int i = 0; i < 6; ++i) zs[i] = f.zi[tone][i] * e0;
    for (int j = 0; j < pad; ++j) (void)fsk_step<ZO>(zs, b, a, ox.left(j));   // trimmed later
    if (n_tiles > 0) {
      fetch(r0, 0);
      fetch(r1, 1);
      auto fwd = [&](v4u (&r)[NI], int64_t t) {
        deposit(r);
        fetch(r, t + 2);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 6; ++i) ck[((size_t)t * 6 + i) * 64] = zs[i];
        run_tile([](int, double) {}, true);
        __builtin_amdgcn_sched_barrier(0);
      };
      int64_t t = 0;
      for (; t + 1 < n_tiles; t += 2) {
        fwd(r0, t);
        fwd(r1, t + 1);
      }
      if (t < n_tiles) fwd(r0, t);
    }
    // the tail's forward outputs -> yb rows 0..ntail-1 (flat), the last -> ylast
    for (int64_t i = n_main; i < n; ++i) {
      const T xi = x[i];
      if constexpr (AMB) PeakT<T>::one(xi, pk_hi, pk_lo);
      const double xv = In<T>::cvt(xi);
      (&yb[0][0])[(size_t)(i - n_main) * YP + lane] = fsk_step<ZO>(zs, b, a, xv);
    }
    if constexpr (AMB) {
      // this batch's margin scale, and the group's flag word cleared for F2
      if (tone == 0 && s < ns)
        p.amb[s] = p.force_exact ? __builtin_inf() : amb_scale(ox.peak_with_tab(PeakT<T>::peak(pk_hi, pk_lo)), p.tau);
      if (lane == 0) p.xflags[w] = 0u;
    }
    double yl = 0.0;
    for (int j = 0; j < pad; ++j) {
      yl = fsk_step<ZO>(zs, b, a, ox.right(j));
      (&yb[0][0])[(size_t)(n - n_main + j) * YP + lane] = yl;
    }
    ylast_sh[lane] = yl;
  }
  __syncthreads();                                     // phase 1 -> 1b
  if (role == 1) {
    // ---- phase 1b: backward over the right extension and the tail
    const double yl = ylast_sh[lane];
#pragma unroll
    for (int i = 0; i < 6; ++i) zs[i] = f.zi[tone][i] * yl;
    const double* tb = &yb[0][0];
    for (int64_t j = ntail - 1; j >= n - n_main; --j) (void)fsk_step<ZO>(zs, b, a, tb[(size_t)j * YP + lane]);
    for (int64_t i = n - 1; i >= n_main; --i) {
      const double y = fsk_step<ZO>(zs, b, a, tb[(size_t)(i - n_main) * YP + lane]);
      if (s < ns) zd[((size_t)s * n + fsk_zoff<LIVE>(p, i)) * 2 + tone] = y;
    }
  }
  __syncthreads();                                     // the tail rows of yb are free again
  // tile tz's 32 rows of z from yb buffer bb, after wave 1 has run it backward:
  // RPS rows per 1-KiB store instruction, lane -> (row, sample)
  auto store_tile = [&](int bb, int64_t tz) {
    const double (*buf)[YP] = &yb[bb * TL];
    if constexpr (64 % TL == 0) {
      constexpr int RPS = 64 / TL;
      const int sub = lane / TL, k = lane % TL;
      const int64_t zo = fsk_zoff<LIVE>(p, tz * TL + k);
#pragma unroll 4
      for (int row = 0; row < 32; row += RPS) {
        const int rr = row + sub;
        const int64_t so = w * 32 + rr;
        const double2 v = *reinterpret_cast<const double2*>(&buf[k][2 * rr]);
        if (so < ns) z[(size_t)so * n + zo] = v;
      }
    } else {
      // lanes k < TL, one row of TL samples per store instruction
      const int k = lane < TL ? lane : TL - 1;
      const int64_t zo = fsk_zoff<LIVE>(p, tz * TL + k);
#pragma unroll 4
      for (int row = 0; row < 32; ++row) {
        const int64_t so = w * 32 + row;
        const double2 v = *reinterpret_cast<const double2*>(&buf[k][2 * row]);
        if (lane < TL && so < ns) z[(size_t)so * n + zo] = v;
      }
    }
  };
  // ---- phase 2: wave 0 re-forwards tile T-1-i while wave 1 runs tile T-i backward
  // (W1S: and stores it right away -- the stores ride on the wave with less
  // arithmetic per tile; otherwise wave 0 stores it an iteration later)
  if (role == 0) {
    // tiles top-down; inputs and checkpoints two tiles ahead
    double c0[6], c1[6];
    auto ldck = [&](double (&c)[6], int64_t t) {
      t = t < 0 ? 0 : t;
#pragma unroll
      for (int i = 0; i < 6; ++i) c[i] = ck[((size_t)t * 6 + i) * 64];
    };
    if (n_tiles > 0) {
      fetch(r0, n_tiles - 1);
      ldck(c0, n_tiles - 1);
      fetch(r1, n_tiles - 2);
      ldck(c1, n_tiles - 2);
    }
    auto refwd = [&](v4u (&r)[NI], double (&c)[6], int64_t it) {
      const int64_t t = n_tiles - 1 - it;
      if (!W1S && it >= 2) store_tile((int)(it & 1), t + 2);   // done by wave 1 in iteration it-1
      if (t >= 0) {
        deposit(r);
#pragma unroll
        for (int i = 0; i < 6; ++i) zs[i] = c[i];
        fetch(r, t - 2);
        ldck(c, t - 2);
        __builtin_amdgcn_sched_barrier(0);
        double (*dst)[YP] = &yb[(it & 1) * TL];
        run_tile([&](int k, double y) { dst[k][lane] = y; }, false);
      }
      __syncthreads();
    };
    int64_t it = 0;
    for (; it + 1 <= n_tiles; it += 2) {
      refwd(r0, c0, it);
      refwd(r1, c1, it + 1);
    }
    if (it <= n_tiles) refwd(r0, c0, it);
    if (!W1S && n_tiles >= 1) store_tile((int)((n_tiles - 1) & 1), 0);   // wave 1's last tile
  } else {
    for (int64_t it = 0; it <= n_tiles; ++it) {
      if (it >= 1) {                                     // tile n_tiles - it, re-run forward by wave 0
        double (*buf)[YP] = &yb[((it - 1) & 1) * TL];
#pragma unroll 8
        for (int k = TL - 1; k >= 0; --k) buf[k][lane] = fsk_step<ZO>(zs, b, a, buf[k][lane]);
        if constexpr (W1S) store_tile((int)((it - 1) & 1), n_tiles - it);
      }
      __syncthreads();
    }
  }
}

// F3.  workgroup = stream: the stream's compare bits (in the final row pass's
// tile order, fft.h fft_bits_stride; 12 KB for a 1-s stream) are staged in
// LDS with coalesced loads, then thread = output word: bit b is 1 when more
// than half of the compare bits of samples [i-q, min(i+q, n)) are 1,
// i = sps/2 + b*sps (np.mean(chunk) > 0.5, modem.py:320-323); bits go MSB first.
// A stream whose bits exceed kDecideLdsMax (about 4.2 s at 96 kHz, or any
// longer capture) reads them straight from global memory (L1/L2-served:
// neighbouring words read neighbouring bytes) instead -- no LDS limit on n.
constexpr int kDecideThreads = 256;
constexpr int64_t kDecideLdsMax = 48 * 1024;

template <bool LDS>
__global__ __launch_bounds__(kDecideThreads) void k_fsk_decide(const uint8_t* __restrict__ bits,
                                                               uint32_t* __restrict__ words, int64_t n_streams,
                                                               FskParams p) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_bits[];
  const int64_t s = blockIdx.x;
  // a stream the exact fallback recomputed: its bits from there (fsk_exact_kernels.hip)
  const bool exact = p.xflags && ((p.xflags[s >> 5] >> (s & 31)) & 1u);
  const uint8_t* __restrict__ c = (exact ? p.xbits : bits) + (size_t)s * p.bits_stride;
  const uint8_t* __restrict__ sb = c;
  if constexpr (LDS) {
    const int nb = (int)p.bits_stride;
    // bits_stride need not be a multiple of 16 (nor rows 16-B aligned): bytes
    for (int i = threadIdx.x; i < nb; i += kDecideThreads) lds_bits[i] = c[i];
    __syncthreads();
    sb = lds_bits;
  }
  const int64_t q = p.sps / 4, half = p.sps / 2;
  for (int64_t w = threadIdx.x; w < p.n_words; w += kDecideThreads) {
    uint32_t word = 0;
    for (int u = 0; u < 32; ++u) {
      const int64_t bi = w * 32 + u;
      if (bi >= p.n_bits) break;
      const int64_t i = half + bi * p.sps;
      const int64_t lo = i - q, hi = (i + q < p.n) ? i + q : p.n;
      int64_t kk = (int64_t)(((float)lo + 0.5f) * p.inv_rn1);   // sample lo = r + rn1*kk
      int64_t r = lo - kk * p.rn1;
      int64_t ones = 0;
      if (p.lc.on) {
        // live-column bits: bit row = the column's live index; a window is
        // nw consecutive live columns of one sps block, so one row kk
        bool lv;
        const int l0 = lc_col_pos(p.lc, (int)r, lv);
        for (int64_t k = 0; k < hi - lo; ++k) {
          const int64_t l = l0 + k;
          ones += (sb[(l >> 3) * p.rn2 + kk] >> (l & 7)) & 1;
        }
      } else {
        for (int64_t k = lo; k < hi; ++k) {
          ones += (sb[(r >> 3) * p.rn2 + kk] >> (r & 7)) & 1;
          if (++r == p.rn1) {
            r = 0;
            ++kk;
          }
        }
      }
      word |= (2 * ones > hi - lo ? 1u : 0u) << (31 - u);
    }
    words[(size_t)s * p.n_words + w] = word;
  }
}

// ---- time-split F1 (one capture or a few: the reference's own call pattern,
// filebeep_advanced_v2.py:324 -> modem.fsk_demodulate, modem.py:307-308) ----
// The serial F1 is two dependent recursions of n + 2 pad steps per tone (9-10
// ms for a 1-s capture, whatever the batch).  Here each pass is cut into
// chunks of L outputs, lane = (chunk, tone), and a chunk starts w samples
// early from a zero state -- or, the chunk holding the pass's first sample,
// from scipy's zi * first-sample state.  The filters are stable, so the zero
// start has decayed below the rounding level after w samples (fsk_api.cpp
// fsk_split_design); what remains is a different rounding trajectory, within
// kappa * peak|ext x| of scipy's output (tests/test_split_margin.py measures
// it).  F2 then flags with the wider margin FskSplit::tau and the exact path
// re-runs the serial F1 for the flagged streams, so decisions stay the
// reference's.  Each step is F1's own (fsk_step<MODE>, scipy's order), so a
// chunk is scipy's lfilter operation for operation from its start state
// (oracle/amr_oracle.c oracle_fsk_split_bandpass restates it).
// a split chunk's warm-up step (before its first output): one FMA per tap
// (fsk_split_warm), as the PSK split's (psk_common.h bp_warm) -- only the
// state it leaves matters; oracle/amr_oracle.c chunked_pass_w restates it
__device__ __forceinline__ void fsk_split_warm(double (&z)[6], const double (&b)[7], const double (&a)[7], double x) {
  const double y = __builtin_fma(b[0], x, z[0]);
#pragma unroll
  for (int i = 0; i < 5; ++i) z[i] = __builtin_fma(-a[i + 1], y, __builtin_fma(b[i + 1], x, z[i + 1]));
  z[5] = __builtin_fma(-a[6], y, b[6] * x);
}

// FS0 (sp.conv): a chunk's start state by convolution instead of a w-step
// warm-up (split_chain.h split_conv_state; the PSK split's KS0): one wave
// per (chunk, tone), four per workgroup, -> zs; before FS1 over ext(x) and
// again before FS2 over y1 reversed
// STRICT (FskSplit::strict): the (stream, tone) scratch row and its bounds
__device__ __forceinline__ double* fsk_strict_row(const FskSplit& sp, int64_t s, int tone) {
  return sp.sc + ((size_t)s * 2 + tone) * sp.sstride;
}
__device__ __forceinline__ ConvBound fsk_conv_bound(const FskSplit& sp, int64_t s, int tone, int64_t off) {
  const StrictBp& d = sp.sb[tone];
  return ConvBound{d.kabs, d.z0abs, d.gam, fsk_strict_row(sp, s, tone) + off};
}
// the rounding one step of scipy's order commits, summed over states (split_strict.h):
// u2 sum_{i>=1} |z_i| + kx |x| + ky |y|, the pre-step |z1..z5| in this pairing
__device__ __forceinline__ double fsk_step_sz(const double (&z)[6]) {
  return ((fabs(z[1]) + fabs(z[2])) + (fabs(z[3]) + fabs(z[4]))) + fabs(z[5]);
}
__device__ __forceinline__ unsigned long long fsk_abs_bits(double v) {
  return (unsigned long long)__double_as_longlong(v) & 0x7fffffffffffffffULL;
}

template <typename T, bool ST>
__global__ __launch_bounds__(256) void k_fsk_split_state_fwd(const void* xv, int64_t x_stride, FskParams p,
                                                             FskSplit sp) {
  const int64_t s = blockIdx.y;
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= 2 * sp.c) return;   // whole waves
  const int tone = (int)(q & 1);
  const int64_t c = q >> 1;
  const T* __restrict__ x = reinterpret_cast<const T*>(xv) + s * x_stride;
  const int64_t n = p.n;
  const int pad = p.pad;
  const OddExt<T> ox(x, p.edge, s, n, pad);
  split_conv_state<6, ST>(
      sp.ktab + (size_t)tone * sp.w * 6, sp.z0tab + (size_t)tone * (sp.w + 1) * 6, sp.w, c * sp.L, ox.left(0),
      [&](int64_t j) -> double {
        if (j < pad) return ox.left(j);
        if (j < pad + n) return In<T>::cvt(x[j - pad]);
        return ox.right(j - pad - n);
      },
      sp.zs + (((size_t)s * 2 + tone) * sp.c + c) * 6,
      ST ? fsk_conv_bound(sp, s, tone, fsk_strict_off_ds1(sp) + c) : ConvBound{});
}
template <bool ST>
__global__ __launch_bounds__(256) void k_fsk_split_state_bwd(FskParams p, FskSplit sp) {
  const int64_t s = blockIdx.y;
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= 2 * sp.c) return;
  const int tone = (int)(q & 1);
  const int64_t c = q >> 1;
  const int64_t m1 = p.n + 2 * (int64_t)p.pad;
  const double* __restrict__ y1 = sp.y1 + ((size_t)s * 2 + tone) * m1;
  split_conv_state<6, ST>(
      sp.ktab + (size_t)tone * sp.w * 6, sp.z0tab + (size_t)tone * (sp.w + 1) * 6, sp.w, c * sp.L, y1[m1 - 1],
      [&](int64_t k) { return y1[m1 - 1 - k]; }, sp.zs + (((size_t)s * 2 + tone) * sp.c + c) * 6,
      ST ? fsk_conv_bound(sp, s, tone, fsk_strict_off_ds2(sp) + c) : ConvBound{});
}

// FS1: forward pass over ext(x) (odd extension in the input's precision, as
// F1), outputs [o0, o1) of chunk c for tone q & 1 -> y1; tone-0 lanes keep
// the stream's max |ext x|
template <typename T, int MODE, bool ST>
__global__ __launch_bounds__(64) void k_fsk_split_fwd(const void* xv, int64_t x_stride, FskParams p, FskIir f,
                                                      FskSplit sp) {
  const int64_t s = blockIdx.y;
  const int64_t q = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (q >= 2 * sp.c) return;
  const int tone = (int)(q & 1);
  const int64_t c = q >> 1;
  const T* __restrict__ x = reinterpret_cast<const T*>(xv) + s * x_stride;
  const int64_t n = p.n;
  const int pad = p.pad;
  const int64_t m1 = n + 2 * (int64_t)pad;
  const int64_t o0 = c * sp.L, o1 = o0 + sp.L < m1 ? o0 + sp.L : m1;
  double b[7], a[7], z[6];
#pragma unroll
  for (int i = 0; i < 7; ++i) { b[i] = f.b[tone][i]; a[i] = f.a[tone][i]; }
  const OddExt<T> ox(x, p.edge, s, n, pad);
  int64_t j = o0 - sp.w;
  if (sp.conv) {   // FS0's start state
    j = o0;
    const double* zs = sp.zs + (((size_t)s * 2 + tone) * sp.c + c) * 6;
#pragma unroll
    for (int i = 0; i < 6; ++i) z[i] = zs[i];
  } else if (j <= 0) {
    j = 0;
    const double e0 = ox.left(0);
#pragma unroll
    for (int i = 0; i < 6; ++i) z[i] = f.zi[tone][i] * e0;
  } else {
#pragma unroll
    for (int i = 0; i < 6; ++i) z[i] = 0.0;
  }
  double* __restrict__ y1 = sp.y1 + ((size_t)s * 2 + tone) * m1;
  unsigned long long pk = 0;
  // ST: this chunk's largest step bound and |y1|, and the step bounds summed
  // per block of kStrictBlk outputs (chunks start on block boundaries)
  [[maybe_unused]] double dmax = 0.0, ymax = 0.0, dsum = 0.0;
  [[maybe_unused]] int dcnt = 0;
  [[maybe_unused]] double* dblk = ST ? fsk_strict_row(sp, s, tone) : nullptr;
  [[maybe_unused]] const double kx = ST ? sp.sb[tone].kx : 0.0, ky = ST ? sp.sb[tone].ky : 0.0;
  auto out = [&](int64_t jj, double e) {
    if constexpr (ST) {
      const double sz = fsk_step_sz(z);
      const double y = fsk_step<MODE>(z, b, a, e);
      y1[jj] = y;
      const double dd = __builtin_fma(sp.u2, sz, __builtin_fma(kx, fabs(e), ky * fabs(y)));
      dmax = fmax(dmax, dd);
      dsum += dd;
      if (++dcnt == kStrictBlk) {
        dblk[jj / kStrictBlk] = dsum;
        dsum = 0.0;
        dcnt = 0;
      }
      ymax = fmax(ymax, fabs(y));                 // (NaN / inf input: the peak test flags the stream)
    } else {
      y1[jj] = fsk_step<MODE>(z, b, a, e);
    }
    const unsigned long long bits = fsk_abs_bits(e);
    pk = bits > pk ? bits : pk;
  };
  auto body = [&](int64_t jj, double e) {
    if (jj < o0) fsk_split_warm(z, b, a, e);
    else out(jj, e);
  };
  for (; j < o1 && j < pad; ++j) body(j, ox.left(j));
  const int64_t jm = o1 < pad + n ? o1 : pad + n;
  if (j < jm) {
    split_chain_2(
        j, o0, jm, fwd_blocks(x - pad, [](T v) { return In<T>::cvt(v); }),
        [&](int64_t jj) { return In<T>::cvt(x[jj - pad]); },
        [&](int64_t, double e) { fsk_split_warm(z, b, a, e); }, out);
    j = jm;
  }
  for (; j < o1; ++j) body(j, ox.right(j - pad - n));
  if (tone == 0) atomicMax(&sp.peak[s], pk);
  if constexpr (ST) {
    if (dcnt > 0) dblk[(o1 - 1) / kStrictBlk] = dsum;   // the pass's last, partial block
    atomicMax(sp.bnd + ((size_t)s * 2 + tone) * 8 + 0, fsk_abs_bits(dmax));
    atomicMax(sp.bnd + ((size_t)s * 2 + tone) * 8 + 2, fsk_abs_bits(ymax));
  }
}

// FS2: backward pass (scipy: lfilter over y1 reversed from zi * y1[-1]);
// chunk c covers reversed positions [o0, o1): f[i], i = m1 - 1 - k - pad, into
// z at F1's offsets (the live-column layout when the plan has it)
template <int MODE, bool LIVE, bool ST>
__global__ __launch_bounds__(64) void k_fsk_split_bwd(double* __restrict__ zd, FskParams p, FskIir f, FskSplit sp) {
  const int64_t s = blockIdx.y;
  const int64_t q = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (q >= 2 * sp.c) return;
  const int tone = (int)(q & 1);
  const int64_t c = q >> 1;
  const int64_t n = p.n;
  const int pad = p.pad;
  const int64_t m1 = n + 2 * (int64_t)pad;
  const int64_t o0 = c * sp.L, o1 = o0 + sp.L < m1 ? o0 + sp.L : m1;
  double b[7], a[7], z[6];
#pragma unroll
  for (int i = 0; i < 7; ++i) { b[i] = f.b[tone][i]; a[i] = f.a[tone][i]; }
  const double* __restrict__ y1 = sp.y1 + ((size_t)s * 2 + tone) * m1;
  int64_t k = o0 - sp.w;
  if (sp.conv) {   // FS0's start state
    k = o0;
    const double* zs = sp.zs + (((size_t)s * 2 + tone) * sp.c + c) * 6;
#pragma unroll
    for (int i = 0; i < 6; ++i) z[i] = zs[i];
  } else if (k <= 0) {
    k = 0;
    const double yl = y1[m1 - 1];
#pragma unroll
    for (int i = 0; i < 6; ++i) z[i] = f.zi[tone][i] * yl;
  } else {
#pragma unroll
    for (int i = 0; i < 6; ++i) z[i] = 0.0;
  }
  [[maybe_unused]] double dmax = 0.0, dsum = 0.0;   // ST: the largest step bound, block sums
  [[maybe_unused]] int dcnt = 0;
  [[maybe_unused]] double* dblk = ST ? fsk_strict_row(sp, s, tone) + fsk_strict_off_d2(sp) : nullptr;
  [[maybe_unused]] const double kx = ST ? sp.sb[tone].kx : 0.0, ky = ST ? sp.sb[tone].ky : 0.0;
  split_chain_2(
      k, o0, o1, bwd_blocks(y1, m1 - 1), [&](int64_t kk) { return y1[m1 - 1 - kk]; },
      [&](int64_t, double v) { fsk_split_warm(z, b, a, v); },
      [&](int64_t kk, double v) {
        [[maybe_unused]] double sz = 0.0;
        if constexpr (ST) sz = fsk_step_sz(z);
        const double y = fsk_step<MODE>(z, b, a, v);
        const int64_t i = m1 - 1 - kk - pad;
        if (i >= 0 && i < n) zd[((size_t)s * n + fsk_zoff<LIVE>(p, i)) * 2 + tone] = y;
        if constexpr (ST) {
          const double dd = __builtin_fma(sp.u2, sz, __builtin_fma(kx, fabs(v), ky * fabs(y)));
          dmax = fmax(dmax, dd);
          dsum += dd;
          if (++dcnt == kStrictBlk) {
            dblk[kk / kStrictBlk] = dsum;
            dsum = 0.0;
            dcnt = 0;
          }
        }
      });
  if constexpr (ST) {
    if (dcnt > 0) dblk[(o1 - 1) / kStrictBlk] = dsum;
    atomicMax(sp.bnd + ((size_t)s * 2 + tone) * 8 + 3, fsk_abs_bits(dmax));
  }
}

// KF1 / KF2 (STRICT; split_strict.h, as the PSK split's KB1 / KB2 per tone):
// thread = (forward block J, stream, tone) -- grid.y = 2 s + tone.
//   E1[J]  the forward pass's error at output block J: both paths' rounding
//          (block sums of D through W, the cut remainder at max D), the chunk
//          starts' errors (+ truncation tk * peak) through GS;
//   E2[J]  the backward pass's at forward block J: pass 1's rounding through
//          pass 2 (K12), the start errors through |h| (HS), the last input's
//          error through the zi start (TZ), its own rounding and starts.
// max E2 = F bounds |z_split - z_serial| on every sample of the tone while the
// a-posteriori caps hold (each pass's difference <= 2^-10 of its input peak).
constexpr int kKfThreads = 256;
constexpr double kKfTwo = 2.0 + 0x1p-20;
struct KfRow {
  double* row;
  unsigned long long* bw;
  double D1m, y1m, D2m, peak1, cap1, p2, cap2, c1;
};
__device__ __forceinline__ KfRow kf_row(const FskSplit& sp, int64_t s, int tone) {
  const StrictBp& d = sp.sb[tone];
  KfRow k;
  k.row = fsk_strict_row(sp, s, tone);
  k.bw = sp.bnd + ((size_t)s * 2 + tone) * 8;
  k.D1m = __longlong_as_double((long long)k.bw[0]);
  k.y1m = __longlong_as_double((long long)k.bw[2]);
  k.D2m = __longlong_as_double((long long)k.bw[3]);
  k.peak1 = __longlong_as_double((long long)sp.peak[s]);
  k.cap1 = 0x1p-10 * k.peak1;
  k.p2 = k.y1m + k.cap1;
  k.cap2 = 0x1p-10 * k.p2;
  const double sec1 = sp.u2 * d.zb * k.cap1 + d.ky * k.cap1;
  k.c1 = d.g1x * (sec1 + 2 * 0x1p-1060) + d.gmax * 0x1p-53 * d.zi_sum * k.peak1;
  return k;
}
__device__ __forceinline__ void kf_wave_max(unsigned long long* m, double v, bool live) {
  unsigned long long x = live ? fsk_abs_bits(v) : 0ull;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long y = __shfl_xor(x, o);
    x = y > x ? y : x;
  }
  if ((threadIdx.x & 63) == 0 && x != 0ull) atomicMax(m, x);
}
__global__ __launch_bounds__(kKfThreads) void k_fsk_strict_e1(FskSplit sp) {
  const int64_t s = blockIdx.y >> 1;
  const int tone = (int)(blockIdx.y & 1);
  const int64_t J = (int64_t)blockIdx.x * kKfThreads + threadIdx.x;
  const StrictBp& d = sp.sb[tone];
  const KfRow k = kf_row(sp, s, tone);
  const int64_t LB = sp.L / kStrictBlk;
  const double* d1 = k.row;
  const double* ds1 = k.row + fsk_strict_off_ds1(sp);
  double e = 0.0, st = 0.0;
  const bool live = J < sp.nb1;
  if (live) {
    double r = d.w_tail * k.D1m;
    const int64_t dn = J + 1 < d.nw ? J + 1 : d.nw;
#pragma unroll 8
    for (int64_t dl = 0; dl < dn; ++dl) r = __builtin_fma(d.W[dl], d1[J - dl], r);
    const int64_t c = J / LB;
    const int64_t q = J - c * LB;
    st = c > 0 ? (q < 64 ? d.GS[q] : d.gmax) * (ds1[c] + d.tk * k.peak1) : 0.0;
    e = kKfTwo * r + k.c1 + st;
    k.row[fsk_strict_off_s1(sp) + J] = st;
    k.row[fsk_strict_off_e1(sp) + J] = e;
  }
  kf_wave_max(k.bw + 1, e, live);
  kf_wave_max(k.bw + 4, st, live);
}
__global__ __launch_bounds__(kKfThreads) void k_fsk_strict_e2(FskParams p, FskSplit sp) {
  const int64_t s = blockIdx.y >> 1;
  const int tone = (int)(blockIdx.y & 1);
  const int64_t J = (int64_t)blockIdx.x * kKfThreads + threadIdx.x;
  const StrictBp& d = sp.sb[tone];
  const KfRow k = kf_row(sp, s, tone);
  const int64_t nb1 = sp.nb1, m1 = p.n + 2 * (int64_t)p.pad, LB = sp.L / kStrictBlk;
  const double* d1 = k.row;
  const double* d2 = k.row + fsk_strict_off_d2(sp);
  const double* ds2 = k.row + fsk_strict_off_ds2(sp);
  const double* e1 = k.row + fsk_strict_off_e1(sp);
  const double* s1 = k.row + fsk_strict_off_s1(sp);
  const double E1max = __longlong_as_double((long long)k.bw[1]), S1max = __longlong_as_double((long long)k.bw[4]);
  const double E1last = fmax(e1[nb1 - 1], nb1 > 1 ? e1[nb1 - 2] : 0.0);
  const double sec2 = sp.u2 * d.zb * k.cap2 + d.kx * E1max + d.ky * k.cap2;
  const double c2 = d.hz * k.c1 + d.g1x * (sec2 + 2 * 0x1p-1060) + 2.0 * d.gmax * 0x1p-53 * d.zi_sum * k.p2;
  auto own2 = [&](int64_t K) {
    if (K < 0 || K >= nb1) return 0.0;
    double r = d.w_tail * k.D2m;
    const int64_t dn = K + 1 < d.nw ? K + 1 : d.nw;
#pragma unroll 8
    for (int64_t dl = 0; dl < dn; ++dl) r = __builtin_fma(d.W[dl], d2[K - dl], r);
    const int64_t c = K / LB;
    const int64_t q = K - c * LB;
    const double st = c > 0 ? (q < 64 ? d.GS[q] : d.gmax) * (ds2[c] + d.tk * k.p2) : 0.0;
    return kKfTwo * r + st;
  };
  auto tzw = [&](int64_t q) { return q < d.nz ? d.TZ[q] : d.tz_tail; };
  double e = 0.0;
  const bool live = J < nb1;
  if (live) {
    double a = d.k12_tail * k.D1m;
    // the taps whose block lies inside the pass, in the same (ascending) order
    const int64_t klo = d.k12_off - J > 0 ? d.k12_off - J : 0;
    const int64_t khi = nb1 - J + d.k12_off < d.nk ? nb1 - J + d.k12_off : d.nk;
#pragma unroll 8
    for (int64_t kq = klo; kq < khi; ++kq) a = __builtin_fma(d.K12[kq], d1[J + kq - d.k12_off], a);
    double h = d.hs_tail * S1max;
    const int64_t hhi = nb1 - J < d.nh ? nb1 - J : d.nh;
#pragma unroll 8
    for (int64_t db = 0; db < hhi; ++db) h = __builtin_fma(d.HS[db], s1[J + db], h);
    const int64_t jhi = 16 * J + 15 < m1 - 1 ? 16 * J + 15 : m1 - 1;
    const int64_t k2lo = m1 - 1 - jhi, k2hi = m1 - 1 - 16 * J;
    const int64_t Ka = k2lo / kStrictBlk, Kb = k2hi / kStrictBlk;
    const double tz = fmax(tzw(Ka), tzw(Kb)) * E1last;
    const double o2 = fmax(own2(Ka), own2(Kb));
    e = kKfTwo * a + h + tz + o2 + c2;
    k.row[fsk_strict_off_e2(sp) + J] = e;
  }
  kf_wave_max(k.bw + 6, e, live);
}

// FS3: per stream, F2's margin scale from the input peak with the split's
// tau (exact mode 2: +inf, every stream exact), and its flag word cleared.
// STRICT: tau = the plan's + max over the tones of F * ||ifft(h)||_1 / peak
// (F from KF2), +inf when a tone's caps failed
__global__ __launch_bounds__(64) void k_fsk_split_amb(int64_t n_streams, FskParams p, FskSplit sp) {
  const int64_t s = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (s >= n_streams) return;
  const double peak = __longlong_as_double((long long)sp.peak[s]);
  double tau = sp.tau;
  bool ok = true;
  if (sp.strict && peak != 0.0) {   // (an all-zero stream: exact zeros on both paths, never flagged)
    double F = 0.0;
    for (int t = 0; t < 2; ++t) {
      const KfRow k = kf_row(sp, s, t);
      const double E1max = __longlong_as_double((long long)k.bw[1]), Fm = __longlong_as_double((long long)k.bw[6]);
      ok = ok && E1max <= k.cap1 && Fm <= k.cap2;   // false for NaN
      F = fmax(F, Fm);
    }
    tau = p.tau + F * sp.hl1 * (1.0 + 0x1p-40) / peak;
  }
  p.amb[s] = p.force_exact || !ok ? __builtin_inf() : amb_scale(peak, tau);
  if ((s & 31) == 0) p.xflags[s >> 5] = 0u;
}

template <int MODE, bool ST>
static hipError_t launch_fsk_split_t(int dtype, const void* x, int64_t x_stride, int64_t B, double2* z,
                                     const FskParams& p, const FskIir& f, const FskSplit& sp, hipStream_t st) {
  const dim3 blk(64), g((unsigned)((2 * sp.c + 63) / 64), (unsigned)B);
  const dim3 blk0(256), g0((unsigned)((2 * sp.c + 3) / 4), (unsigned)B);
  if (sp.conv && (!sp.ktab || !sp.z0tab || !sp.zs)) return hipErrorInvalidValue;
  if (sp.conv) {
    switch (dtype) {
      case kF32: hipLaunchKernelGGL((k_fsk_split_state_fwd<float, ST>), g0, blk0, 0, st, x, x_stride, p, sp); break;
      case kF64: hipLaunchKernelGGL((k_fsk_split_state_fwd<double, ST>), g0, blk0, 0, st, x, x_stride, p, sp); break;
      case kI16: hipLaunchKernelGGL((k_fsk_split_state_fwd<int16_t, ST>), g0, blk0, 0, st, x, x_stride, p, sp); break;
      default: return hipErrorInvalidValue;
    }
  }
  switch (dtype) {
    case kF32: hipLaunchKernelGGL((k_fsk_split_fwd<float, MODE, ST>), g, blk, 0, st, x, x_stride, p, f, sp); break;
    case kF64: hipLaunchKernelGGL((k_fsk_split_fwd<double, MODE, ST>), g, blk, 0, st, x, x_stride, p, f, sp); break;
    case kI16: hipLaunchKernelGGL((k_fsk_split_fwd<int16_t, MODE, ST>), g, blk, 0, st, x, x_stride, p, f, sp); break;
    default: return hipErrorInvalidValue;
  }
  double* zd = reinterpret_cast<double*>(z);
  if (sp.conv) hipLaunchKernelGGL((k_fsk_split_state_bwd<ST>), g0, blk0, 0, st, p, sp);
  if (p.lc.on) hipLaunchKernelGGL((k_fsk_split_bwd<MODE, true, ST>), g, blk, 0, st, zd, p, f, sp);
  else hipLaunchKernelGGL((k_fsk_split_bwd<MODE, false, ST>), g, blk, 0, st, zd, p, f, sp);
  if constexpr (ST) {
    const dim3 gk((unsigned)((sp.nb1 + kKfThreads - 1) / kKfThreads), (unsigned)(2 * B));
    hipLaunchKernelGGL(k_fsk_strict_e1, gk, dim3(kKfThreads), 0, st, sp);
    hipLaunchKernelGGL(k_fsk_strict_e2, gk, dim3(kKfThreads), 0, st, p, sp);
  }
  if (p.amb) hipLaunchKernelGGL(k_fsk_split_amb, dim3((unsigned)((B + 63) / 64)), blk, 0, st, B, p, sp);
  return hipGetLastError();
}

// F3 for a few streams (a one-capture call): one workgroup per stream leaves
// the decisions of a 1-s capture on 256 threads (~32 us); here thread = bit,
// the window's compare bits read straight from global memory (L2), and a
// wave's 64 bits packed by ballot into two MSB-first words -- the same
// majority as k_fsk_decide (np.mean(chunk) > 0.5, modem.py:320-323).
// grid = (ceil(n_bits / 256), streams)
__global__ __launch_bounds__(256) void k_fsk_decide_bits(const uint8_t* __restrict__ bits,
                                                         uint32_t* __restrict__ words, FskParams p) {
  const int64_t s = blockIdx.y;
  const int64_t bi = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool exact = p.xflags && ((p.xflags[s >> 5] >> (s & 31)) & 1u);
  const uint8_t* __restrict__ sb = (exact ? p.xbits : bits) + (size_t)s * p.bits_stride;
  bool one = false;
  if (bi < p.n_bits) {
    const int64_t q = p.sps / 4, half = p.sps / 2;
    const int64_t i = half + bi * p.sps;
    const int64_t lo = i - q, hi = (i + q < p.n) ? i + q : p.n;
    int64_t kk = (int64_t)(((float)lo + 0.5f) * p.inv_rn1);
    int64_t r = lo - kk * p.rn1;
    int64_t ones = 0;
    if (p.lc.on) {
      bool lv;
      const int l0 = lc_col_pos(p.lc, (int)r, lv);
      for (int64_t k = 0; k < hi - lo; ++k) {
        const int64_t l = l0 + k;
        ones += (sb[(l >> 3) * p.rn2 + kk] >> (l & 7)) & 1;
      }
    } else {
      for (int64_t k = lo; k < hi; ++k) {
        ones += (sb[(r >> 3) * p.rn2 + kk] >> (r & 7)) & 1;
        if (++r == p.rn1) {
          r = 0;
          ++kk;
        }
      }
    }
    one = 2 * ones > hi - lo;
  }
  const unsigned long long m = __ballot(one);
  const int lane = threadIdx.x & 63;
  if (lane == 0 || lane == 32) {
    const int64_t w = bi >> 5;
    const uint32_t half_mask = (uint32_t)(lane == 0 ? m : m >> 32);
    if (w < p.n_words) words[(size_t)s * p.n_words + w] = __brev(half_mask);
  }
}

int64_t fsk_bandpass_scratch_bytes(int64_t n_streams, int64_t n, int pad) {
  const int64_t per = std::max(fsk_scratch_doubles_per_wave(n, pad), fsk2_scratch_doubles_per_group(n, kFsk2TileMin));
  return ((n_streams + 31) / 32) * per * (int64_t)sizeof(double);
}

static bool fsk_one_wave() {
  static const bool v = [] { const char* e = getenv("AMR_FSK_BP1"); return e && e[0] == '1'; }();
  return v;
}

// fsk_step's MODE: 3 when the odd taps are zero and the numerator is
// antisymmetric (always, for butter(3, band)), 1 with zero odd taps only,
// else 0; AMR_FSK_ZO=0 forces 0; AMR_FSK_F1_FMA=1 the contracted form (2)
static int fsk_step_mode(const FskIir& f, bool allow_fma) {
  static const bool off = [] { const char* e = getenv("AMR_FSK_ZO"); return e && e[0] == '0'; }();
  static const bool fma = [] { const char* e = getenv("AMR_FSK_F1_FMA"); return e && e[0] == '1'; }();
  bool zo = !off, anti = true;
  for (int t = 0; t < 2; ++t) {
    if (f.b[t][1] != 0.0 || f.b[t][3] != 0.0 || f.b[t][5] != 0.0) zo = false;
    if (f.b[t][6] != -f.b[t][0] || f.b[t][4] != -f.b[t][2]) anti = false;
  }
  if (fma && allow_fma && zo) return 2;
  if (zo && anti) return 3;
  return zo ? 1 : 0;
}

template <int ZO, bool LIVE>
static hipError_t launch_fsk_bandpass_t(int dtype, const void* x, int64_t x_stride, int64_t n_streams, double* s1,
                                        double2* z, const FskParams& p, const FskIir& f, hipStream_t st) {
  const unsigned grid = (unsigned)((n_streams + 31) / 32);
  if (!fsk_one_wave() || p.xlist) {
    // AMR_FSK_W1S=0: wave 0 stores z (the round-2 schedule)
    static const bool w1s = [] { const char* e = getenv("AMR_FSK_W1S"); return !(e && e[0] == '0'); }();
    static const int tile_env = [] { const char* e = getenv("AMR_FSK_TILE"); return e ? atoi(e) : 0; }();
    const bool t64 = tile_env == 64, t40 = tile_env == 40 && dtype != kI16;
#define BP2(T, S, D)                                                                                                 \
  do {                                                                                                               \
    if (t64)                                                                                                         \
      hipLaunchKernelGGL((k_fsk_bandpass2<T, ZO, LIVE, S, D, 64>), dim3(grid), dim3(128), 0, st, x, x_stride,         \
                         n_streams, s1, z, p, f);                                                                    \
    else if (t40 && sizeof(T) != 2)                                                                                  \
      hipLaunchKernelGGL((k_fsk_bandpass2<T, ZO, LIVE, S, D, (sizeof(T) == 2 ? 32 : 40)>), dim3(grid), dim3(128), 0,  \
                         st, x, x_stride, n_streams, s1, z, p, f);                                                   \
    else                                                                                                             \
      hipLaunchKernelGGL((k_fsk_bandpass2<T, ZO, LIVE, S, D>), dim3(grid), dim3(128), 0, st, x, x_stride, n_streams,  \
                         s1, z, p, f);                                                                               \
  } while (0)
#define BP2D(T) do { if (p.amb) { if (w1s) BP2(T, true, true); else BP2(T, false, true); } else if (w1s) BP2(T, true, false); else BP2(T, false, false); } while (0)
    switch (dtype) {
      case kF32: BP2D(float); break;
      case kF64: BP2D(double); break;
      case kI16: BP2D(int16_t); break;
      default: return hipErrorInvalidValue;
    }
#undef BP2D
#undef BP2
    return hipGetLastError();
  }
#define BP1(T, A) hipLaunchKernelGGL((k_fsk_bandpass<T, ZO, LIVE, A>), dim3(grid), dim3(64), 0, st, x, x_stride, n_streams, s1, z, p, f)
#define BP1D(T) do { if (p.amb) BP1(T, true); else BP1(T, false); } while (0)
  switch (dtype) {
    case kF32: BP1D(float); break;
    case kF64: BP1D(double); break;
    case kI16: BP1D(int16_t); break;
    default: return hipErrorInvalidValue;
  }
#undef BP1D
#undef BP1
  return hipGetLastError();
}

// z: stream 0's block of this launch (callers staging a batch in chunks pass
// the chunk's first stream); p.lc.on selects the live-column layout
hipError_t launch_fsk_bandpass(int dtype, const void* x, int64_t x_stride, int64_t n_streams, double* s1, double2* z,
                               const FskParams& p, const FskIir& f, hipStream_t st) {
  const int mode = fsk_step_mode(f, !p.xlist);   // the exact path: scipy's order always
#define BPM(M) (p.lc.on ? launch_fsk_bandpass_t<M, true>(dtype, x, x_stride, n_streams, s1, z, p, f, st) \
                        : launch_fsk_bandpass_t<M, false>(dtype, x, x_stride, n_streams, s1, z, p, f, st))
  if (mode == 3) return BPM(3);
  if (mode == 2) return BPM(2);
  return mode == 1 ? BPM(1) : BPM(0);
#undef BPM
}

// FS1-FS3 over B streams of x (B <= 65535: grid.y); z in the plan's layout.
// sp.peak is cleared here; p.amb non-null: FS3 sets the margin scales.
hipError_t launch_fsk_split(int dtype, const void* x, int64_t x_stride, int64_t B, double2* z, const FskParams& p,
                            const FskIir& f, const FskSplit& sp, hipStream_t st) {
  if (B < 1) return hipSuccess;
  if (B > 65535 || p.nt != 7 || sp.L < 1 || sp.c < 1) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(sp.peak, 0, (size_t)B * sizeof(unsigned long long), st);
  if (e != hipSuccess) return e;
  if (sp.strict) {
    e = hipMemsetAsync(sp.bnd, 0, (size_t)B * 2 * 8 * sizeof(unsigned long long), st);
    if (e != hipSuccess) return e;
  }
  const int mode = fsk_step_mode(f, false);
  if (sp.strict) {
    // the strict bound covers the convolution starts and scipy's step order only
    if (!sp.conv || !sp.sc || !sp.bnd || sp.L % kStrictBlk != 0 || !sp.sb[0].kabs || !sp.sb[1].kabs)
      return hipErrorInvalidValue;
    if (mode == 3) return launch_fsk_split_t<3, true>(dtype, x, x_stride, B, z, p, f, sp, st);
    return mode == 1 ? launch_fsk_split_t<1, true>(dtype, x, x_stride, B, z, p, f, sp, st)
                     : launch_fsk_split_t<0, true>(dtype, x, x_stride, B, z, p, f, sp, st);
  }
  if (mode == 3) return launch_fsk_split_t<3, false>(dtype, x, x_stride, B, z, p, f, sp, st);
  return mode == 1 ? launch_fsk_split_t<1, false>(dtype, x, x_stride, B, z, p, f, sp, st)
                   : launch_fsk_split_t<0, false>(dtype, x, x_stride, B, z, p, f, sp, st);
}

hipError_t launch_fsk_decide(const uint8_t* cmp, uint32_t* words, int64_t n_streams, const FskParams& p,
                             hipStream_t st) {
  if (p.n_words < 1 || p.n_bits < 1) return hipSuccess;
  // AMR_FSK_DECIDE_GLOBAL=1: the global-memory form at every length (tests)
  static const bool force_global = [] { const char* e = getenv("AMR_FSK_DECIDE_GLOBAL"); return e && e[0] == '1'; }();
  // a few streams: thread per bit (k_fsk_decide_bits); AMR_FSK_DECIDE_BITS=0 keeps the per-stream form
  static const bool bits_off = [] { const char* e = getenv("AMR_FSK_DECIDE_BITS"); return e && e[0] == '0'; }();
  if (n_streams <= 64 && !bits_off && !force_global) {
    hipLaunchKernelGGL(k_fsk_decide_bits, dim3((unsigned)((p.n_bits + 255) / 256), (unsigned)n_streams), dim3(256), 0,
                       st, cmp, words, p);
    return hipGetLastError();
  }
  if (p.bits_stride <= kDecideLdsMax && !force_global)
    hipLaunchKernelGGL(k_fsk_decide<true>, dim3((unsigned)n_streams), dim3(kDecideThreads), (size_t)p.bits_stride,
                       st, cmp, words, n_streams, p);
  else
    hipLaunchKernelGGL(k_fsk_decide<false>, dim3((unsigned)n_streams), dim3(kDecideThreads), 0, st, cmp, words,
                       n_streams, p);
  return hipGetLastError();
}

}  // namespace amr
