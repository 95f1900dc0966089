// psk_lane_kernels.hip -- the PSK filtfilt passes with ONE STREAM PER LANE
// (the throughput layout), for gfx950.
//
// Same reference arithmetic as psk_kernels.hip (K1r/K1g band-pass, K2q/K3q
// low-pass; modem.py:194-204 -> scipy filtfilt/lfilter in DF-II-T order, no
// contraction), the same buffers downstream (f in s2 for the low-pass and
// K3x, symbols in s1 for K4a) and the same low-pass zero/denormal detector,
// so every stream's bytes are identical whichever layout ran.
//
// Why a second layout.  The state-per-lane kernels spread one stream over
// 4-16 lanes to keep ~1000 waves busy at B = 4096, but half of their
// instructions move states between lanes (DPP, selects), and their lanes do
// 8-16x the arithmetic one lane needs: measured register-only
// (tools/step_probe3.hip, one wave per SIMD) a lane-per-stream band-pass
// step issues 34 FP64 instructions for 64 streams and sustains 921
// stream-samples/ns against 303 for the 8-lane groups of K1g; the low-pass
// per component 1452 against 592 (quads).  The FP64 pipe is saturated at one
// wave per SIMD.  The price is parallelism: B = 4096 is only 64 band-pass
// waves, so this layout is picked when enough streams are in flight on the
// device (api.cpp) -- several batches at once, or big batches.
//
// Intermediates not written to HBM (checkpoint + recompute):
//   * band-pass (k_bp_lane): the forward pass keeps the filter state at the
//     start of every kBpT-sample tile (8 doubles); the backward pass re-runs
//     each tile forward from its checkpoint into registers and filters it
//     backward from there -- the forward output s1 (2 x 8 B/sample of HBM
//     traffic in the round-1 kernels) becomes 4 B/sample of re-read input
//     plus 4 B/sample of checkpoints.
//   * low-pass (k_lp_lane): the same over f with kLpT-sample tiles (4
//     doubles per component) -- the complex forward output s3 (2 x 16
//     B/sample) becomes a second read of f (8 B/sample, mostly L2: the re and
//     im waves of the same streams run on one XCD) plus 2 B/sample of
//     checkpoints.  Symbols are written straight from the backward pass.
// A re-run tile executes exactly the operations the forward pass executed,
// from exactly the same state, so it reproduces its outputs bit for bit.
#include <math.h>
#include <stdlib.h>

#include <type_traits>

#include "amr_internal.h"
#include "psk_common.h"

namespace amr {

constexpr int kBpT = 32;     // band-pass checkpoint tile (samples)
constexpr int kLpT = 40;     // low-pass checkpoint tile: a multiple of sps 5 / 10 / 20 (static symbol slots)
constexpr int kLpT2 = 20;    // the same for the role-split low-pass (LDS: 2 components x 2 buffers x tile)

// (the DF-II-T step functions df2t_step / df2t_step_zo / lp_step: psk_common.h)

template <bool ZO>
__device__ __forceinline__ double bp_step(double (&z)[8], const Iir& f, double x, float& acc) {
  if constexpr (ZO) return df2t_step_zo(z, f, x, acc);
  else return df2t_step<8>(z, f, x);
}

template <bool ZO>
__device__ __forceinline__ bool bp_bad(float acc, const double (&z)[8]) {
  if constexpr (!ZO) return false;
  bool bad = !(acc >= kTinyHi);
#pragma unroll
  for (int j = 0; j < 8; ++j) bad |= !__builtin_isfinite(z[j]);
  return bad;
}

// checkpoint + edge scratch inside the plan's s1 (band-pass) / s3 (low-pass)
__host__ __device__ inline int64_t bp_lane_edge_cap(int pad) { return kBpT + pad; }
__host__ __device__ inline int64_t lp_lane_edge_cap(int pad) { return 2 * (kLpT + pad); }
int64_t psk_lane_bp_scratch_doubles(int64_t n_streams, int64_t n, int pad) {
  const int64_t g = (n_streams + 63) / 64;
  return g * ((n / kBpT) * 8 + bp_lane_edge_cap(pad)) * 64;
}
int64_t psk_lane_lp_scratch_doubles(int64_t n_streams, int64_t n, int pad) {
  const int64_t g = (n_streams + 63) / 64;
  return 2 * g * ((n / kLpT2) * 4 + 2 * (kLpT + pad)) * 64;   // the smaller tile's checkpoints, the larger edges
}

// ---------------------------------------------------------------------------
// band-pass: lane = stream, wave = 64 streams.  Coefficients are wave-uniform
// (kernel arguments in SGPRs).  s1 = [G][nt][8][64] checkpoints, then
// [G][edge][64] tail outputs.
template <typename T, int WPB>
__global__ __launch_bounds__(64 * WPB) void k_bp_lane(PskBuffers buf, PskParams p, Iir f) {
  constexpr int TB = kBpT;
  constexpr int PER = 16 / (int)sizeof(T);      // samples per 16-B load
  constexpr int NL = TB / PER;                  // 16-B loads per tile
  static_assert(TB % PER == 0 && TB % 2 == 0, "tile = whole loads and whole pairs");
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * WPB + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (w * 64 >= buf.n_streams) return;          // wave-uniform
  const int64_t last = buf.n_streams - 1;
  const int64_t s = w * 64 + lane;
  const T* __restrict__ x = reinterpret_cast<const T*>(buf.x) + (s < last ? s : last) * buf.x_stride;
  const uint8_t* __restrict__ xb = reinterpret_cast<const uint8_t*>(x);
  const int64_t n = p.n, n2 = (n + 1) >> 1;
  const int pad = p.pad1;
  const int64_t nt = n / TB;
  const int64_t G = (buf.n_streams + 63) / 64;
  const int64_t ecap = bp_lane_edge_cap(pad);
  double* __restrict__ ck = buf.s1 + (size_t)w * nt * 8 * 64 + lane;
  double* __restrict__ eb = buf.s1 + (size_t)G * nt * 8 * 64 + (size_t)w * ecap * 64 + lane;
  // f = s2 in f_index layout: this lane's pair m at fo + m*64
  double* __restrict__ fo = buf.s2 + (size_t)(w * 2 + (lane >> 5)) * n2 * 64 + (lane & 31) * 2;

  auto load_tile = [&](int64_t t, v4u (&r)[NL]) {
#pragma unroll
    for (int k = 0; k < NL; ++k) r[k] = *reinterpret_cast<const v4u*>(xb + (size_t)t * TB * sizeof(T) + k * 16);
  };
  auto tile_x = [&](const v4u (&r)[NL], int k) -> double {
    T v[PER];
    __builtin_memcpy(v, &r[k / PER], 16);
    return In<T>::cvt(v[k % PER]);
  };

  // ---- forward pass: pads + tiles (checkpoints only) + tail (edge) --------
  double z[8];
  const OddExt<T> ox(x, buf.edge, s < last ? s : last, n, pad);
  {
    const double e0 = ox.left(0);
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = f.zi[j] * e0;
  }
  for (int jj = 0; jj < pad; ++jj) (void)df2t_step<8>(z, f, ox.left(jj));
  v4u xr[NL];
  if (nt > 0) load_tile(0, xr);
  for (int64_t t = 0; t < nt; ++t) {
#pragma unroll
    for (int j = 0; j < 8; ++j) ck[(t * 8 + j) * 64] = z[j];
    v4u cur[NL];
#pragma unroll
    for (int k = 0; k < NL; ++k) cur[k] = xr[k];
    load_tile(t + 1 < nt ? t + 1 : t, xr);      // next tile in flight during this one
#pragma unroll
    for (int k = 0; k < TB; ++k) (void)df2t_step<8>(z, f, tile_x(cur, k));
  }
  const int64_t i_tail = nt * TB;
  int ne = 0;
  for (int64_t i = i_tail; i < n; ++i) eb[(ne++) * 64] = df2t_step<8>(z, f, In<T>::cvt(x[i]));
  double ylast = 0.0;
  for (int jj = 0; jj < pad; ++jj) {
    ylast = df2t_step<8>(z, f, ox.right(jj));
    eb[(ne++) * 64] = ylast;
  }
  __threadfence();                              // checkpoints / edge re-read below

  // ---- backward pass ------------------------------------------------------
  double zb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) zb[j] = f.zi[j] * ylast;
  for (int e = ne - 1; e >= 0; --e) {
    const double y = df2t_step<8>(zb, f, eb[e * 64]);
    const int64_t i = i_tail + e;
    if (i < n) fo[(i >> 1) * 64 + (i & 1)] = y;
  }
  if (nt > 0) {
    load_tile(nt - 1, xr);
    double cn[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) cn[j] = ck[((nt - 1) * 8 + j) * 64];
    for (int64_t t = nt - 1; t >= 0; --t) {
      double zf[8];
      v4u cur[NL];
#pragma unroll
      for (int j = 0; j < 8; ++j) zf[j] = cn[j];
#pragma unroll
      for (int k = 0; k < NL; ++k) cur[k] = xr[k];
      const int64_t tp = t > 0 ? t - 1 : 0;     // the next (lower) tile's input and checkpoint in flight
      load_tile(tp, xr);
#pragma unroll
      for (int j = 0; j < 8; ++j) cn[j] = ck[(tp * 8 + j) * 64];
      double yt[TB];
#pragma unroll
      for (int k = 0; k < TB; ++k) yt[k] = df2t_step<8>(zf, f, tile_x(cur, k));
      double* const fp = fo + (size_t)(t * (TB / 2)) * 64;
#pragma unroll
      for (int k = TB - 1; k >= 1; k -= 2) {
        const double y1 = df2t_step<8>(zb, f, yt[k]);
        const double y0 = df2t_step<8>(zb, f, yt[k - 1]);
        *reinterpret_cast<double2*>(fp + (k >> 1) * 64) = make_double2(y0, y1);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// The band-pass forward pass of one group (lane = stream): pads + tiles
// (checkpoint at the start of every tile, no output) + tail (edge outputs);
// the zero-tap detector flags a stream it cannot vouch for.  Used by
// k_bp_lane2's forward role and, on its own, by k_bp_fwd.
template <typename T, bool ZO>
__device__ __forceinline__ void bp_forward_pass(const PskBuffers& buf, const PskParams& p, const Iir& f, int64_t w,
                                                int lane) {
  constexpr int TB = kBpT;
  constexpr int PER = 16 / (int)sizeof(T);
  constexpr int NL = TB / PER;
  const int64_t last = buf.n_streams - 1;
  const int64_t s = w * 64 + lane;
  const T* __restrict__ x = reinterpret_cast<const T*>(buf.x) + (s < last ? s : last) * buf.x_stride;
  const uint8_t* __restrict__ xb = reinterpret_cast<const uint8_t*>(x);
  const int64_t n = p.n;
  const int pad = p.pad1;
  const int64_t nt = n / TB;
  const int64_t G = (buf.n_streams + 63) / 64;
  const int64_t ecap = bp_lane_edge_cap(pad);
  const int64_t i_tail = nt * TB;
  double* __restrict__ ck = buf.s1 + (size_t)w * nt * 8 * 64 + lane;
  double* __restrict__ eb = buf.s1 + (size_t)G * nt * 8 * 64 + (size_t)w * ecap * 64 + lane;
  auto load_tile = [&](int64_t t, v4u (&r)[NL]) {
#pragma unroll
    for (int k = 0; k < NL; ++k) r[k] = *reinterpret_cast<const v4u*>(xb + (size_t)t * TB * sizeof(T) + k * 16);
  };
  auto tile_x = [&](const v4u (&r)[NL], int k) -> double {
    T v[PER];
    __builtin_memcpy(v, &r[k / PER], 16);
    return In<T>::cvt(v[k % PER]);
  };
  double z[8];
  float acc = __builtin_inff();
  const OddExt<T> ox(x, buf.edge, s < last ? s : last, n, pad);
  {
    const double e0 = ox.left(0);
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = f.zi[j] * e0;
  }
  for (int jj = 0; jj < pad; ++jj) (void)bp_step<ZO>(z, f, ox.left(jj), acc);
  v4u xr[NL];
  if (nt > 0) load_tile(0, xr);
  for (int64_t t = 0; t < nt; ++t) {
#pragma unroll
    for (int j = 0; j < 8; ++j) ck[(t * 8 + j) * 64] = z[j];
    v4u cur[NL];
#pragma unroll
    for (int k = 0; k < NL; ++k) cur[k] = xr[k];
    load_tile(t + 1 < nt ? t + 1 : t, xr);
#pragma unroll
    for (int k = 0; k < TB; ++k) (void)bp_step<ZO>(z, f, tile_x(cur, k), acc);
  }
  int e = 0;
  for (int64_t i = i_tail; i < n; ++i) eb[(e++) * 64] = bp_step<ZO>(z, f, In<T>::cvt(x[i]), acc);
  for (int jj = 0; jj < pad; ++jj) eb[(e++) * 64] = bp_step<ZO>(z, f, ox.right(jj), acc);
  if (bp_bad<ZO>(acc, z) && s <= last) atomicOr(&buf.bp_flags[s], 1);
}

// band-pass forward pass alone, wave = group (AMR_BP_PREFWD): k_bp_lane2<...,
// PRE> then runs only the re-run / backward roles.  The forward pass no
// longer holds an idle backward wave and its LDS for half the band-pass's
// life.
template <typename T, bool ZO>
__global__ __launch_bounds__(256) void k_bp_fwd(PskBuffers buf, PskParams p, Iir f) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (w * 64 >= buf.n_streams) return;          // wave-uniform
  bp_forward_pass<T, ZO>(buf, p, f, w, lane);
}

// ---------------------------------------------------------------------------
// band-pass, role-split: two waves per group of 64 streams (GPB groups per
// workgroup).  Wave 0 runs the forward pass (checkpoints + tail edge) while
// wave 1 waits; then, tile by tile from the end, wave 0 re-runs tile t-1
// forward from its checkpoint into one LDS buffer while wave 1 filters tile t
// backward out of the other buffer and stores f -- the backward pass and the
// re-run overlap, so the kernel takes two passes of latency instead of three
// and a batch has twice the waves.  One workgroup barrier per tile.
// FIXUP (with ZO false): the full-tap re-run of the groups the zero-tap
// launch flagged; a workgroup whose group has no flagged stream returns
// before its first barrier (2-wave, 108-VGPR workgroups: they find room
// beside the resident band-pass / low-pass waves, where the one-wave kernel's
// 168-VGPR four-wave workgroups waited up to 15 ms at 8192 streams).
// CK = 2 (AMR_BP_CK=2): a checkpoint every 2 tiles (64 samples: half the
// checkpoint bytes) while the LDS hand-off stays at one 32-sample tile, so
// the workgroup keeps its 64 KiB and two fit a CU.  The re-run role then
// reaches the second tile of a pair by first re-running the pair's first
// tile without outputs (1.5x its steps), holding the pair's inputs in
// registers (one more tile of them) -- bit for bit the same outputs.
// F32F (PskBuffers::f32f): f is stored rounded to float32 into the first half
// of the group's s2 slot (the f64 layout's element order, float elements),
// and each stream's max |f| (bits: NaN / inf dominate) into buf.fpeak.
template <typename T, int GPB, bool ZO, bool FIXUP = false, bool PRE = false, int CK = 1, bool F32F = false>
__global__ __launch_bounds__(128 * GPB) void k_bp_lane2(PskBuffers buf, PskParams p, Iir f) {
  static_assert(!(FIXUP && PRE), "the fix-up pass runs its own forward pass");
  static_assert(!(F32F && FIXUP), "the fix-up pass writes float64 f");
  static_assert(CK == 1 || (CK == 2 && !PRE), "64-sample checkpoints: the kernel's own forward pass");
  constexpr int TB = kBpT;
  constexpr int PER = 16 / (int)sizeof(T);
  constexpr int NL = TB / PER;
  static_assert(TB % PER == 0 && TB % 2 == 0, "tile = whole loads and whole pairs");
  __shared__ __attribute__((aligned(16))) double2 yb[GPB][2][TB / 2][64];   // forward outputs of a tile, by pairs
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int gi = wv >> 1, role = wv & 1;
  const int64_t w = (int64_t)blockIdx.x * GPB + gi;
  const bool active = w * 64 < buf.n_streams;   // inactive groups still meet every barrier
  const int64_t last = buf.n_streams - 1;
  const int64_t s = w * 64 + lane;
  if constexpr (FIXUP) {
    static_assert(GPB == 1 && !ZO, "the fix-up pass: one group per workgroup, every tap");
    if (!active) return;                        // workgroup-uniform (one group)
    if (!__syncthreads_or(s <= last && buf.bp_flags[s] != 0)) return;   // nothing flagged in this group
  }
  const T* __restrict__ x = reinterpret_cast<const T*>(buf.x) + (s < last ? s : last) * buf.x_stride;
  const uint8_t* __restrict__ xb = reinterpret_cast<const uint8_t*>(x);
  const int64_t n = p.n, n2 = (n + 1) >> 1;
  const int pad = p.pad1;
  const int64_t nt = n / TB;
  const int64_t G = (buf.n_streams + 63) / 64;
  const int64_t ecap = bp_lane_edge_cap(pad);
  const int64_t i_tail = nt * TB;
  const int ne = (int)(n - i_tail) + pad;
  double* __restrict__ ck = buf.s1 + (size_t)w * nt * 8 * 64 + lane;
  double* __restrict__ eb = buf.s1 + (size_t)G * nt * 8 * 64 + (size_t)w * ecap * 64 + lane;
  double* __restrict__ fo = buf.s2 + (size_t)(w * 2 + (lane >> 5)) * n2 * 64 + (lane & 31) * 2;
  [[maybe_unused]] float* __restrict__ fo32 =
      reinterpret_cast<float*>(buf.s2 + (size_t)w * 2 * n2 * 64) + (size_t)(lane >> 5) * n2 * 64 + (lane & 31) * 2;

  auto load_tile = [&](int64_t t, v4u (&r)[NL]) {
#pragma unroll
    for (int k = 0; k < NL; ++k) r[k] = *reinterpret_cast<const v4u*>(xb + (size_t)t * TB * sizeof(T) + k * 16);
  };
  auto tile_x = [&](const v4u (&r)[NL], int k) -> double {
    T v[PER];
    __builtin_memcpy(v, &r[k / PER], 16);
    return In<T>::cvt(v[k % PER]);
  };

  if (!PRE && role == 0 && active) {
    // ---- forward pass: pads + tiles (checkpoints only) + tail (edge) ------
    // (the same steps as bp_forward_pass, written out: through the device
    // function the compiler kept 238 VGPRs live here against 113)
    double z[8];
    float acc = __builtin_inff();
    const OddExt<T> ox(x, buf.edge, s < last ? s : last, n, pad);
    {
      const double e0 = ox.left(0);
#pragma unroll
      for (int j = 0; j < 8; ++j) z[j] = f.zi[j] * e0;
    }
    for (int jj = 0; jj < pad; ++jj) (void)bp_step<ZO>(z, f, ox.left(jj), acc);
    v4u xr[NL];
    if (nt > 0) load_tile(0, xr);
    for (int64_t t = 0; t < nt; ++t) {
      if (t % CK == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) ck[((t / CK) * 8 + j) * 64] = z[j];
      }
      v4u cur[NL];
#pragma unroll
      for (int k = 0; k < NL; ++k) cur[k] = xr[k];
      load_tile(t + 1 < nt ? t + 1 : t, xr);
#pragma unroll
      for (int k = 0; k < TB; ++k) (void)bp_step<ZO>(z, f, tile_x(cur, k), acc);
    }
    int e = 0;
    for (int64_t i = i_tail; i < n; ++i) eb[(e++) * 64] = bp_step<ZO>(z, f, In<T>::cvt(x[i]), acc);
    for (int jj = 0; jj < pad; ++jj) eb[(e++) * 64] = bp_step<ZO>(z, f, ox.right(jj), acc);
    if (bp_bad<ZO>(acc, z) && s <= last) atomicOr(&buf.bp_flags[s], 1);
    __threadfence();                            // checkpoints + edge: read by this wave and the backward wave
  }
  __syncthreads();

  if (role == 0 && CK == 2) {
    // ---- re-run tiles nt-1 ... 0 into LDS, checkpoints every 2 tiles -------
    // pair c = tiles (2c, 2c+1) from checkpoint c; tile 2c+1 re-runs tile 2c
    // first (no outputs).  Registers: the pair's inputs (xa, xb), the next
    // pair's arriving one tile ahead (xbn at the odd tile, xan at the even).
    v4u xa[NL], xb[NL], xan[NL], xbn[NL];
    double cc[8], ccn[8];
    if (active && nt > 0) {
      const int64_t c = (nt - 1) >> 1;
      load_tile(2 * c, xa);
      if (2 * c + 1 < nt) load_tile(2 * c + 1, xb);
#pragma unroll
      for (int j = 0; j < 8; ++j) cc[j] = ck[(c * 8 + j) * 64];
    }
    for (int64_t it = 0; it <= nt; ++it) {
      const int64_t t = nt - 1 - it;
      if (active && t >= 0) {
        const int64_t c = t >> 1, cp = c > 0 ? c - 1 : 0;
        double zf[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) zf[j] = cc[j];
        double2 (*ybuf)[64] = yb[gi][it & 1];
        float dummy = 0.0f;                     // the re-run repeats checked steps: no detector
        if (t & 1) {
          load_tile(2 * cp + 1, xbn);           // the next pair's second tile and checkpoint
#pragma unroll
          for (int j = 0; j < 8; ++j) ccn[j] = ck[(cp * 8 + j) * 64];
#pragma unroll
          for (int k = 0; k < TB; ++k) (void)bp_step<ZO>(zf, f, tile_x(xa, k), dummy);
#pragma unroll
          for (int k = 0; k < TB; k += 2) {
            const double y0 = bp_step<ZO>(zf, f, tile_x(xb, k), dummy);
            const double y1 = bp_step<ZO>(zf, f, tile_x(xb, k + 1), dummy);
            ybuf[k >> 1][lane] = make_double2(y0, y1);
          }
        } else {
          if (2 * c + 1 >= nt) {                // a top pair of one tile: nothing was prefetched for the next
            load_tile(2 * cp + 1, xbn);
#pragma unroll
            for (int j = 0; j < 8; ++j) ccn[j] = ck[(cp * 8 + j) * 64];
          }
          load_tile(2 * cp, xan);
#pragma unroll
          for (int k = 0; k < TB; k += 2) {
            const double y0 = bp_step<ZO>(zf, f, tile_x(xa, k), dummy);
            const double y1 = bp_step<ZO>(zf, f, tile_x(xa, k + 1), dummy);
            ybuf[k >> 1][lane] = make_double2(y0, y1);
          }
#pragma unroll
          for (int k = 0; k < NL; ++k) { xa[k] = xan[k]; xb[k] = xbn[k]; }
#pragma unroll
          for (int j = 0; j < 8; ++j) cc[j] = ccn[j];
        }
      }
      __syncthreads();
    }
  } else if (role == 0) {
    // ---- re-run tiles nt-1, nt-2, ... 0 forward into LDS --------------------
    v4u xr[NL];
    double cn[8];
    if (active && nt > 0) {
      load_tile(nt - 1, xr);
#pragma unroll
      for (int j = 0; j < 8; ++j) cn[j] = ck[((nt - 1) * 8 + j) * 64];
    }
    for (int64_t it = 0; it <= nt; ++it) {
      const int64_t t = nt - 1 - it;
      if (active && t >= 0) {
        double zf[8];
        v4u cur[NL];
#pragma unroll
        for (int j = 0; j < 8; ++j) zf[j] = cn[j];
#pragma unroll
        for (int k = 0; k < NL; ++k) cur[k] = xr[k];
        const int64_t tp = t > 0 ? t - 1 : 0;
        load_tile(tp, xr);
#pragma unroll
        for (int j = 0; j < 8; ++j) cn[j] = ck[(tp * 8 + j) * 64];
        double2 (*ybuf)[64] = yb[gi][it & 1];
        float dummy = 0.0f;                     // the re-run repeats checked steps: no detector
#pragma unroll
        for (int k = 0; k < TB; k += 2) {
          const double y0 = bp_step<ZO>(zf, f, tile_x(cur, k), dummy);
          const double y1 = bp_step<ZO>(zf, f, tile_x(cur, k + 1), dummy);
          ybuf[k >> 1][lane] = make_double2(y0, y1);
        }
      }
      __syncthreads();
    }
  } else {
    // ---- backward pass: the tail edge, then the tiles out of LDS -------------
    double zb[8];
    float acc = __builtin_inff();
    unsigned long long pk = 0;                  // F32F: max |f| as bits
    auto pk_acc = [&](double y) {
      if constexpr (F32F) {
        const unsigned long long b = (unsigned long long)__double_as_longlong(y) & 0x7fffffffffffffffULL;
        pk = b > pk ? b : pk;
      }
    };
    if (active) {
      const double ylast = eb[(ne - 1) * 64];
#pragma unroll
      for (int j = 0; j < 8; ++j) zb[j] = f.zi[j] * ylast;
      for (int e = ne - 1; e >= 0; --e) {
        const double y = bp_step<ZO>(zb, f, eb[e * 64], acc);
        const int64_t i = i_tail + e;
        if (i < n) {
          if constexpr (F32F) {
            fo32[(i >> 1) * 64 + (i & 1)] = (float)y;
            pk_acc(y);
          } else {
            fo[(i >> 1) * 64 + (i & 1)] = y;
          }
        }
      }
    }
    __syncthreads();                            // tile nt-1 is in buffer 0
    for (int64_t it = 1; it <= nt; ++it) {
      const int64_t t = nt - it;
      if (active) {
        const double2 (*ybuf)[64] = yb[gi][(it - 1) & 1];
        double* const fp = fo + (size_t)(t * (TB / 2)) * 64;
        float* const fp32 = fo32 + (size_t)(t * (TB / 2)) * 64;
#pragma unroll
        for (int k = TB / 2 - 1; k >= 0; --k) {
          const double2 yy = ybuf[k][lane];
          const double y1 = bp_step<ZO>(zb, f, yy.y, acc);
          const double y0 = bp_step<ZO>(zb, f, yy.x, acc);
          if constexpr (F32F) {
            *reinterpret_cast<float2*>(fp32 + k * 64) = make_float2((float)y0, (float)y1);
            pk_acc(y0);
            pk_acc(y1);
          } else {
            *reinterpret_cast<double2*>(fp + k * 64) = make_double2(y0, y1);
          }
        }
      }
      __syncthreads();
    }
    if (active && bp_bad<ZO>(acc, zb) && s <= last) atomicOr(&buf.bp_flags[s], 1);
    if constexpr (F32F) {
      if (active && s <= last) buf.fpeak[s] = __longlong_as_double((long long)pk);
    }
  }
}

// ---------------------------------------------------------------------------
// low-pass: lane = stream, wave = 64 streams x ONE component (so the LO
// multiplier is wave-uniform).  WPB == 1: blocks b and b+8 are the re and im
// waves of the same streams and land on the same XCD (blocks are dealt to the
// 8 XCDs round-robin); WPB >= 2: waves (2i, 2i+1) of a block are the re and
// im waves of one stream group, on one CU -- either way the second read of f
// is a cache hit (PMC: f is read from HBM once per pass).
// Mixer and detector exactly as K2q/K3q (psk_kernels.hip): bb[0] in numpy's
// full complex-multiply form, every other sample f*lo_c (equal whenever it
// is not a zero, and a zero is flagged); min over |hi words| of every input
// and output (forward) and every output (backward), final states finite.
// s3 = [2G][nt][4][64] checkpoints, then [2G][edge][64]: the head (pre-pad
// + tile 0) and tail (last partial tile + post-pad) forward outputs.
// SPS > 0: symbols at tile offsets FM + k*SPS (kLpT % SPS == 0, first % SPS
// == FM); SPS == 0: any sps (run-time symbol test per sample).
// Memory: f streams through a ring of NCH chunk slots (the next tile's chunk
// c is loaded as soon as this tile's chunk c is consumed: a tile of compute
// to arrive); the tile's LO multipliers arrive by one 8-B load per lane a tile
// ahead and are parked in a per-wave LDS double buffer, read back by
// broadcast ds_read_b128.
// (Tried: 3 waves per SIMD through a half-tile ring (CH 4), and a 20-sample
// tile at 4 waves per SIMD: both slower in flight and alone -- the loads
// need the whole tile of lead.)
#ifndef AMR_LP_WAVES
#define AMR_LP_WAVES 1
#endif
#ifndef AMR_LP_CH
#define AMR_LP_CH 8
#endif
#ifndef AMR_LP_REGION_SYMS
#define AMR_LP_REGION_SYMS 8     // fused slicer: symbols per slicing region at most (a power of two >= TL / sps)
#endif
// FUSE (static symbol slots, WPB >= 2): the slicer runs inside the backward
// pass.  Both component waves of a group park their symbol samples in an LDS
// ring (16 slots: a region -- the tail, RT tiles, the head -- holds at most 8
// symbols, and two consecutive regions never share a slot), meet at one
// workgroup barrier per region (RT = 2 tiles at sps 10: half the barriers of
// one per tile, a lone batch's low-pass 14.5 -> 13.7 ms; 16-symbol regions
// in a 32-slot ring measured slower), and the re wave forms s[k+1] * conj(s[k]),
// the sector decision (qpsk_dibit, as K4a) and the MSB-first words, storing
// each word as it completes.  No symbol leaves the chip (0.63 GB written and
// read back per 4096-stream batch before); streams the detector flags get
// their symbols from K3x and their words from K4a afterwards.
// F32F (with FUSE; PskBuffers::f32f): f arrives rounded to float32 (k_bp_lane2
// F32F), so the symbols differ from the reference's by at most
// E = p.f32_margin * fpeak[s] + 2^-120 (the rounding through the low-pass's L1
// gain, api.cpp f32_design); the re wave flags every decision within E of its
// boundary -- QPSK ||di| - |dr||, BPSK |dr| against sqrt2 E (|s0|_1 + |s1|_1 +
// E) -- into flags and bp_flags, and the fix-up band-pass, K3x and K4a redo
// those streams exactly.
template <int SPS, int FM, int WPB, bool FUSE = false, bool F32F = false>
__global__ __launch_bounds__(64 * WPB, SPS > 0 ? AMR_LP_WAVES : 1) void k_lp_lane(PskBuffers buf, PskParams p, Iir f) {
  static_assert(!FUSE || (SPS > 0 && WPB >= 2), "fused slicing: static slots, both components in one workgroup");
  static_assert(!F32F || FUSE, "the float32 hand-off's margin check runs in the fused slicer");
  using FV = typename std::conditional<F32F, float2, double2>::type;
  constexpr int TL = kLpT;
  constexpr int CH = AMR_LP_CH;                 // samples per f chunk (CH / 2 x 16 B per lane)
  constexpr int NCH = TL / CH, HC = CH / 2;
  constexpr int R = NCH % 2 == 0 ? NCH / 2 : NCH;   // ring slots: chunk q lands R chunks ahead of its use
  static_assert(TL % CH == 0 && TL <= 64, "tile = whole chunks; one LO value per lane");
  static_assert(SPS == 0 || (TL % SPS == 0 && FM < SPS), "static symbol slots");
  __shared__ __attribute__((aligned(16))) double lo_lds[WPB][2][TL];
  // FUSE: tiles per slicing region (one barrier each) -- as many as keep a
  // region within MS symbols -- and a ring of 2 MS symbol slots per wave (two
  // consecutive regions never share a slot)
  constexpr int SPR = TL / (SPS > 0 ? SPS : TL);                 // symbols per tile (static slots)
  constexpr int MS = AMR_LP_REGION_SYMS;
  constexpr int RT = MS / SPR > 1 ? MS / SPR : 1;
  constexpr int NSL = FUSE ? 2 * MS : 1;
  static_assert(!FUSE || (RT * SPR <= MS && (MS & (MS - 1)) == 0), "a region holds at most MS symbols");
  __shared__ double sring[FUSE ? WPB : 1][NSL][64];   // FUSE: symbol samples k at slot k & (NSL - 1)
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int64_t w;
  int comp;
  if constexpr (WPB == 1) {
    const int64_t bx = blockIdx.x, kx = bx >> 3;
    w = (kx >> 1) * 8 + (bx & 7);
    comp = (int)(kx & 1);
  } else {
    w = (int64_t)blockIdx.x * (WPB / 2) + (wv >> 1);
    comp = wv & 1;
  }
  const int64_t n = p.n, n2 = (n + 1) >> 1;
  const int pad = p.pad2;
  const int64_t nt = n / TL;
  if (w * 64 >= buf.n_streams) {                // wave-uniform
    if constexpr (FUSE) {                       // an idle group still meets the backward pass's barriers
      for (int64_t b = 0; b < (nt > 1 ? (nt - 1 + RT - 1) / RT : 0) + 2; ++b) __syncthreads();
    }
    return;
  }
  const int64_t s = w * 64 + lane;
  const int64_t G = (buf.n_streams + 63) / 64;
  const int64_t wc = w * 2 + comp;
  const int64_t ecap = lp_lane_edge_cap(pad);
  double* __restrict__ ck = buf.s3 + (size_t)wc * nt * 4 * 64 + lane;
  double* __restrict__ eh = buf.s3 + (size_t)2 * G * nt * 4 * 64 + (size_t)wc * ecap * 64 + lane;
  double* __restrict__ et = eh + (size_t)(pad + TL) * 64;
  const double* __restrict__ fl = buf.s2 + (size_t)(w * 2 + (lane >> 5)) * n2 * 64 + (lane & 31) * 2;
  const float* __restrict__ fl32 =
      reinterpret_cast<const float*>(buf.s2 + (size_t)w * 2 * n2 * 64) + (size_t)(lane >> 5) * n2 * 64 + (lane & 31) * 2;
  const double* __restrict__ lov = buf.lo2 + (size_t)comp * n;                   // lo_c[i], vector loads
  CDouble* const loc = (CDouble*)(buf.lo2 + (size_t)comp * n);                   // the same, scalar loads
  CDouble* const lo4 = (CDouble*)(buf.lo) + 2 * comp;                            // (mult, addend) at [4i]
  auto F = [&](int64_t i) -> double {
    if constexpr (F32F) return (double)fl32[(i >> 1) * 64 + (i & 1)];
    else return fl[(i >> 1) * 64 + (i & 1)];
  };
  auto Xm = [&](int64_t i) { return F(i) * loc[i]; };
  // f pairs of tile t, chunk c: this lane's 16 B (F32F: 8 B) at pair t*TL/2 + c*HC + k
  auto load_chunk = [&](int64_t t, int c, FV (&r)[HC]) {
    if constexpr (F32F) {
      const float2* fp = reinterpret_cast<const float2*>(fl32 + (size_t)(t * (TL / 2) + c * HC) * 64);
#pragma unroll
      for (int k = 0; k < HC; ++k) r[k] = fp[k * 32];
    } else {
      const double2* fp = reinterpret_cast<const double2*>(fl + (size_t)(t * (TL / 2) + c * HC) * 64);
#pragma unroll
      for (int k = 0; k < HC; ++k) r[k] = fp[k * 32];
    }
  };
  auto load_lo = [&](int64_t t) -> double { return lov[t * TL + (lane < TL ? lane : 0)]; };
  auto put_lo = [&](int64_t t, double v) {
    if (lane < TL) lo_lds[wv][t & 1][lane] = v;
  };
  // mixer inputs of chunk c from the chunk's f pairs and the tile's LDS multipliers
  auto chunk_e = [&](int64_t t, int c, const FV (&fv)[HC], double (&e)[CH]) {
    const double2* lp = reinterpret_cast<const double2*>(&lo_lds[wv][t & 1][c * CH]);
#pragma unroll
    for (int k = 0; k < HC; ++k) {
      const double2 l = lp[k];
      e[2 * k] = (double)fv[k].x * l.x;
      e[2 * k + 1] = (double)fv[k].y * l.y;
    }
  };

  // ---- forward pass ---------------------------------------------------------
  double z[4];
  float acc = __builtin_inff();
  bool bad = false;
  const double x0 = F(0) * lo4[0] + lo4[1];      // bb[0]: numpy's (f + 0j) * lo, +0 allowed (class-checked)
  const double xl = Xm(n - 1);
  bad |= __builtin_amdgcn_class(x0, kClsX);
  const double e0 = 2.0 * x0 - Xm(pad);
  bad |= __builtin_amdgcn_class(e0, kClsY);
#pragma unroll
  for (int j = 0; j < 4; ++j) z[j] = f.zi[j] * e0;
  for (int jj = 0; jj < pad; ++jj) {
    const double e = 2.0 * x0 - Xm(pad - jj);
    const double y = lp_step(z, f, e);
    acc = tiny_min3(acc, e, y);
    eh[jj * 64] = y;
  }
  const int64_t nh = n < TL ? n : TL;           // tile 0 (holds bb[0]): edge buffer, not recomputed
  for (int64_t i = 0; i < nh; ++i) {
    const double e = i == 0 ? x0 : Xm(i);
    const double y = lp_step(z, f, e);
    acc = tiny_min3(acc, i == 0 ? y : e, y);
    eh[(pad + i) * 64] = y;
  }
  FV ring[R][HC];
  if (nt > 1) {
#pragma unroll
    for (int c = 0; c < R; ++c) load_chunk(1, c, ring[c]);
    put_lo(1, load_lo(1));
  }
  for (int64_t t = 1; t < nt; ++t) {
    const int64_t tn = t + 1 < nt ? t + 1 : t;
    const double lon = load_lo(tn);
#pragma unroll
    for (int j = 0; j < 4; ++j) ck[(t * 4 + j) * 64] = z[j];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      FV fv[HC];
#pragma unroll
      for (int k = 0; k < HC; ++k) fv[k] = ring[c % R][k];
      if (c + R < NCH) load_chunk(t, c + R, ring[c % R]);
      else load_chunk(tn, c + R - NCH, ring[c % R]);
      double e[CH];
      chunk_e(t, c, fv, e);
#pragma unroll
      for (int k = 0; k < CH; k += 2) {
        const double y0 = lp_step(z, f, e[k]);
        const double y1 = lp_step(z, f, e[k + 1]);
        acc = tiny_min3(acc, e[k], e[k + 1]);
        acc = tiny_min3(acc, y0, y1);
      }
    }
    put_lo(tn, lon);
  }
  const int64_t i_tail = nt >= 1 ? nt * TL : nh;
  int ne = 0;
  for (int64_t i = i_tail; i < n; ++i) {
    const double e = Xm(i);
    const double y = lp_step(z, f, e);
    acc = tiny_min3(acc, e, y);
    et[(ne++) * 64] = y;
  }
  double ylast = 0.0;
  for (int jj = 0; jj < pad; ++jj) {
    const double e = 2.0 * xl - Xm(n - 2 - jj);
    ylast = lp_step(z, f, e);
    acc = tiny_min3(acc, e, ylast);
    et[(ne++) * 64] = ylast;
  }
  bad |= !(acc >= kTinyHi);
#pragma unroll
  for (int j = 0; j < 4; ++j) bad |= !__builtin_isfinite(z[j]);
  __threadfence();                              // checkpoints / edges re-read below

  // ---- backward pass ----------------------------------------------------------
  const int64_t S = p.n_sym, first = p.first, sps = p.sps;
  double* __restrict__ symp = buf.s1 + sym_index(s, S, 0, comp);   // symbol k at symp[k*64]
  auto put_sym = [&](int64_t k, double y) {
    if constexpr (FUSE) sring[wv][k & (NSL - 1)][lane] = y;
    else symp[k * 64] = y;
  };
  auto sym_out = [&](int64_t i, double y) {     // generic: a symbol sample at i?
    if (i >= first && (i - first) % sps == 0) put_sym((i - first) / sps, y);
  };
  // FUSE: the re wave slices the symbols of samples [i_lo, i_hi) once both
  // components are in the ring (diff_k = s[k+1] * conj(s[k]) in numpy's fma
  // form, exactly as K4a); words complete as k descends through 16j (32j)
  double pr = 0.0, pim = 0.0;                   // s[k+1]
  uint32_t wacc = 0;
  const bool qpsk = p.kind == kQpsk;
  // F32F: this stream's symbol error bound, and whether a decision fell inside it
  const double Em = F32F && s < buf.n_streams ? p.f32_margin * buf.fpeak[s] + 0x1p-120 : 0.0;
  bool mflag = false;
  auto region_done = [&](int64_t i_lo, int64_t i_hi) {
    if constexpr (FUSE) {
      __syncthreads();
      if (comp == 0) {
        const int64_t k_lo = i_lo <= first ? 0 : (i_lo - first + sps - 1) / sps;
        int64_t k_hi = i_hi - 1 < first ? -1 : (i_hi - 1 - first) / sps;
        if (k_hi > S - 1) k_hi = S - 1;
        for (int64_t k = k_hi; k >= k_lo; --k) {
          const double sr = sring[wv][k & (NSL - 1)][lane], si = sring[wv + 1][k & (NSL - 1)][lane];
          if (k <= S - 2) {
            const double br = sr, bi = -si;
            const double dr = __builtin_fma(pr, br, -(pim * bi));
            double md = 0.0;                    // F32F: the decision's margin (d's error bound)
            if constexpr (F32F) {
              const double a0 = fabs(br) + fabs(bi), a1 = fabs(pr) + fabs(pim);
              md = 0x1.6a09e667f3bcdp+0 * Em * (a0 + a1 + Em) * (1.0 + 0x1p-40) + 0x1p-48 * (a0 * a1);
              if (!qpsk && !(fabs(dr) > md)) mflag = true;
            }
            if (qpsk) {
              const double di = __builtin_fma(pr, bi, pim * br);
              if constexpr (F32F) {
                const double adr = fabs(dr), adi = fabs(di);
                if (!(fabs(adi - adr) > md + 0x1p-29 * (adr + adi))) mflag = true;
              }
              wacc |= qpsk_dibit(dr, di) << (30 - 2 * (int)(k & 15));
              if ((k & 15) == 0) {
                if (s < buf.n_streams) buf.words[(size_t)s * p.n_words + (k >> 4)] = wacc;
                wacc = 0;
              }
            } else {
              wacc |= (dr < 0 ? 1u : 0u) << (31 - (int)(k & 31));
              if ((k & 31) == 0) {
                if (s < buf.n_streams) buf.words[(size_t)s * p.n_words + (k >> 5)] = wacc;
                wacc = 0;
              }
            }
          }
          pr = sr;
          pim = si;
        }
      }
    }
  };
  float accb = __builtin_inff();
  double zb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) zb[j] = f.zi[j] * ylast;
  for (int e = ne - 1; e >= 0; --e) {
    const double y = lp_step(zb, f, et[e * 64]);
    accb = tiny_min3(accb, y, y);
    const int64_t i = i_tail + e;
    if (i < n) sym_out(i, y);
  }
  region_done(i_tail, n);
  if (nt > 1) {
    const int64_t q0 = SPS > 0 ? first / SPS : 0;
    double cn[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) cn[j] = ck[((nt - 1) * 4 + j) * 64];
#pragma unroll
    for (int c = 0; c < R; ++c) load_chunk(nt - 1, c, ring[c]);
    put_lo(nt - 1, load_lo(nt - 1));
    int64_t r_hi = nt * TL;                     // FUSE: upper bound of the region not yet sliced
    for (int64_t t = nt - 1; t >= 1; --t) {
      double zf[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) zf[j] = cn[j];
      const int64_t tp = t > 1 ? t - 1 : 1;     // the next (lower) tile's input and checkpoint in flight
#pragma unroll
      for (int j = 0; j < 4; ++j) cn[j] = ck[(tp * 4 + j) * 64];
      const double lop = load_lo(tp);
      double yt[TL];
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        FV fv[HC];
#pragma unroll
        for (int k = 0; k < HC; ++k) fv[k] = ring[c % R][k];
        if (c + R < NCH) load_chunk(t, c + R, ring[c % R]);
        else load_chunk(tp, c + R - NCH, ring[c % R]);
        double e[CH];
        chunk_e(t, c, fv, e);
#pragma unroll
        for (int k = 0; k < CH; ++k) yt[c * CH + k] = lp_step(zf, f, e[k]);
      }
#pragma unroll
      for (int k = TL - 1; k >= 1; k -= 2) {
        const double y1 = lp_step(zb, f, yt[k]);
        const double y0 = lp_step(zb, f, yt[k - 1]);
        accb = tiny_min3(accb, y1, y0);
        if constexpr (SPS > 0) {
          if (k % SPS == FM) put_sym(t * (TL / SPS) + (k - FM) / SPS - q0, y1);
          if ((k - 1) % SPS == FM) put_sym(t * (TL / SPS) + (k - 1 - FM) / SPS - q0, y0);
        } else {
          sym_out(t * TL + k, y1);
          sym_out(t * TL + k - 1, y0);
        }
      }
      put_lo(tp, lop);
      if ((nt - 1 - t) % RT == RT - 1 || t == 1) {
        region_done(t * TL, r_hi);
        r_hi = t * TL;
      }
    }
  }
  for (int e = pad + (int)nh - 1; e >= 0; --e) {
    const double y = lp_step(zb, f, eh[e * 64]);
    accb = tiny_min3(accb, y, y);
    const int64_t i = e - pad;
    if (i >= 0) sym_out(i, y);
  }
  region_done(0, nh);
  bad |= !(accb >= kTinyHi);
#pragma unroll
  for (int j = 0; j < 4; ++j) bad |= !__builtin_isfinite(zb[j]);
  if constexpr (F32F) bad |= mflag;
  if (bad && s < buf.n_streams) {
    atomicOr(&buf.flags[s], 1);
    if constexpr (F32F) atomicOr(&buf.bp_flags[s], 1);   // float64 f for K3x: the fix-up re-runs the group
  }
}

// ---------------------------------------------------------------------------
// low-pass, role-split: four waves per group of 64 streams -- (re, im) x
// (forward / re-run, backward).  The forward waves run the forward pass
// (checkpoints every TL2 samples, head / tail edges, the input/output zero
// detector) while the backward waves wait; then tile by tile from the end the
// forward waves re-run tile t-1 into an LDS buffer while the backward waves
// filter tile t out of the other one and write the symbol samples.  Two
// passes of latency instead of three.  Same arithmetic and detector as
// k_lp_lane; TL2 = 20 keeps the LDS of a group at 40 KB.
template <int SPS, int FM, int TL2>
__global__ __launch_bounds__(256) void k_lp_lane2(PskBuffers buf, PskParams p, Iir f) {
  constexpr int TL = TL2;
  constexpr int CH = TL % 8 == 0 ? 8 : 4;       // samples per f chunk
  constexpr int NCH = TL / CH, HC = CH / 2;
  static_assert(TL % CH == 0 && TL <= 64, "tile = whole chunks; one LO value per lane");
  static_assert(SPS == 0 || (TL % SPS == 0 && FM < SPS), "static symbol slots");
  __shared__ __attribute__((aligned(16))) double lo_lds[2][2][TL];              // [comp][buf]
  __shared__ __attribute__((aligned(16))) double2 yb[2][2][TL / 2][64];        // [comp][buf][pair][lane]
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int comp = wv & 1, role = wv >> 1;
  const int64_t w = blockIdx.x;
  if (w * 64 >= buf.n_streams) return;          // block-uniform: no barrier is skipped by part of a block
  const int64_t s = w * 64 + lane;
  const int64_t n = p.n, n2 = (n + 1) >> 1;
  const int pad = p.pad2;
  const int64_t nt = n / TL;
  const int64_t G = (buf.n_streams + 63) / 64;
  const int64_t wc = w * 2 + comp;
  const int64_t ecap = 2 * (TL + pad);
  double* __restrict__ ck = buf.s3 + (size_t)wc * nt * 4 * 64 + lane;
  double* __restrict__ eh = buf.s3 + (size_t)2 * G * nt * 4 * 64 + (size_t)wc * ecap * 64 + lane;
  double* __restrict__ et = eh + (size_t)(pad + TL) * 64;
  const double* __restrict__ fl = buf.s2 + (size_t)(w * 2 + (lane >> 5)) * n2 * 64 + (lane & 31) * 2;
  const double* __restrict__ lov = buf.lo2 + (size_t)comp * n;
  CDouble* const loc = (CDouble*)(buf.lo2 + (size_t)comp * n);
  CDouble* const lo4 = (CDouble*)(buf.lo) + 2 * comp;
  auto F = [&](int64_t i) { return fl[(i >> 1) * 64 + (i & 1)]; };
  auto Xm = [&](int64_t i) { return F(i) * loc[i]; };
  auto load_chunk = [&](int64_t t, int c, double2 (&r)[HC]) {
    const double2* fp = reinterpret_cast<const double2*>(fl + (size_t)(t * (TL / 2) + c * HC) * 64);
#pragma unroll
    for (int k = 0; k < HC; ++k) r[k] = fp[k * 32];
  };
  auto load_lo = [&](int64_t t) -> double { return lov[t * TL + (lane < TL ? lane : 0)]; };
  auto put_lo = [&](int64_t t, double v) {
    if (lane < TL) lo_lds[comp][t & 1][lane] = v;
  };
  auto chunk_e = [&](int64_t t, int c, const double2 (&fv)[HC], double (&e)[CH]) {
    const double2* lp = reinterpret_cast<const double2*>(&lo_lds[comp][t & 1][c * CH]);
#pragma unroll
    for (int k = 0; k < HC; ++k) {
      const double2 l = lp[k];
      e[2 * k] = fv[k].x * l.x;
      e[2 * k + 1] = fv[k].y * l.y;
    }
  };
  const int64_t nh = n < TL ? n : TL;
  const int64_t i_tail = nt >= 1 ? nt * TL : nh;
  const int ne = (int)(n - i_tail) + pad;

  if (role == 0) {
    // ---- forward pass (as k_lp_lane) ----------------------------------------
    double z[4];
    float acc = __builtin_inff();
    bool bad = false;
    const double x0 = F(0) * lo4[0] + lo4[1];
    const double xl = Xm(n - 1);
    bad |= __builtin_amdgcn_class(x0, kClsX);
    const double e0 = 2.0 * x0 - Xm(pad);
    bad |= __builtin_amdgcn_class(e0, kClsY);
#pragma unroll
    for (int j = 0; j < 4; ++j) z[j] = f.zi[j] * e0;
    for (int jj = 0; jj < pad; ++jj) {
      const double e = 2.0 * x0 - Xm(pad - jj);
      const double y = lp_step(z, f, e);
      acc = tiny_min3(acc, e, y);
      eh[jj * 64] = y;
    }
    for (int64_t i = 0; i < nh; ++i) {
      const double e = i == 0 ? x0 : Xm(i);
      const double y = lp_step(z, f, e);
      acc = tiny_min3(acc, i == 0 ? y : e, y);
      eh[(pad + i) * 64] = y;
    }
    double2 ring[NCH][HC];
    if (nt > 1) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) load_chunk(1, c, ring[c]);
      put_lo(1, load_lo(1));
    }
    for (int64_t t = 1; t < nt; ++t) {
      const int64_t tn = t + 1 < nt ? t + 1 : t;
      const double lon = load_lo(tn);
#pragma unroll
      for (int j = 0; j < 4; ++j) ck[(t * 4 + j) * 64] = z[j];
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        double2 fv[HC];
#pragma unroll
        for (int k = 0; k < HC; ++k) fv[k] = ring[c][k];
        load_chunk(tn, c, ring[c]);
        double e[CH];
        chunk_e(t, c, fv, e);
#pragma unroll
        for (int k = 0; k < CH; k += 2) {
          const double y0 = lp_step(z, f, e[k]);
          const double y1 = lp_step(z, f, e[k + 1]);
          acc = tiny_min3(acc, e[k], e[k + 1]);
          acc = tiny_min3(acc, y0, y1);
        }
      }
      put_lo(tn, lon);
    }
    int ee = 0;
    for (int64_t i = i_tail; i < n; ++i) {
      const double e = Xm(i);
      const double y = lp_step(z, f, e);
      acc = tiny_min3(acc, e, y);
      et[(ee++) * 64] = y;
    }
    for (int jj = 0; jj < pad; ++jj) {
      const double e = 2.0 * xl - Xm(n - 2 - jj);
      const double y = lp_step(z, f, e);
      acc = tiny_min3(acc, e, y);
      et[(ee++) * 64] = y;
    }
    bad |= !(acc >= kTinyHi);
#pragma unroll
    for (int j = 0; j < 4; ++j) bad |= !__builtin_isfinite(z[j]);
    if (bad && s < buf.n_streams) atomicOr(&buf.flags[s], 1);
    __threadfence();                            // checkpoints + edges: read by both roles
    __syncthreads();

    // ---- re-run tiles nt-1 .. 1 forward into LDS -----------------------------
    double cn[4];
    if (nt > 1) {
#pragma unroll
      for (int j = 0; j < 4; ++j) cn[j] = ck[((nt - 1) * 4 + j) * 64];
#pragma unroll
      for (int c = 0; c < NCH; ++c) load_chunk(nt - 1, c, ring[c]);
      put_lo(nt - 1, load_lo(nt - 1));
    }
    for (int64_t it = 0; it < nt; ++it) {       // it = nt-1 is the backward waves' last tile: barrier only
      const int64_t t = nt - 1 - it;
      if (t >= 1) {
        double zf[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) zf[j] = cn[j];
        const int64_t tp = t > 1 ? t - 1 : 1;
#pragma unroll
        for (int j = 0; j < 4; ++j) cn[j] = ck[(tp * 4 + j) * 64];
        const double lop = load_lo(tp);
        double2 (*ybuf)[64] = yb[comp][it & 1];
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
          double2 fv[HC];
#pragma unroll
          for (int k = 0; k < HC; ++k) fv[k] = ring[c][k];
          load_chunk(tp, c, ring[c]);
          double e[CH];
          chunk_e(t, c, fv, e);
#pragma unroll
          for (int k = 0; k < CH; k += 2) {
            const double y0 = lp_step(zf, f, e[k]);
            const double y1 = lp_step(zf, f, e[k + 1]);
            ybuf[(c * CH + k) >> 1][lane] = make_double2(y0, y1);
          }
        }
        put_lo(tp, lop);
      }
      __syncthreads();
    }
  } else {
    __syncthreads();                            // the forward pass is done
    const int64_t S = p.n_sym, first = p.first, sps = p.sps;
    double* __restrict__ symp = buf.s1 + sym_index(s, S, 0, comp);
    auto sym_out = [&](int64_t i, double y) {
      if (i >= first && (i - first) % sps == 0) symp[((i - first) / sps) * 64] = y;
    };
    float accb = __builtin_inff();
    double zb[4];
    const double ylast = et[(ne - 1) * 64];
#pragma unroll
    for (int j = 0; j < 4; ++j) zb[j] = f.zi[j] * ylast;
    for (int e = ne - 1; e >= 0; --e) {
      const double y = lp_step(zb, f, et[e * 64]);
      accb = tiny_min3(accb, y, y);
      const int64_t i = i_tail + e;
      if (i < n) sym_out(i, y);
    }
    // the forward waves meet nt barriers in their re-run loop: tile nt-1 is in
    // buffer 0 after the first (none at all when nt == 0)
    if (nt >= 1) __syncthreads();
    const int64_t q0 = SPS > 0 ? first / SPS : 0;
    for (int64_t it = 1; it < nt; ++it) {
      const int64_t t = nt - it;
      const double2 (*ybuf)[64] = yb[comp][(it - 1) & 1];
#pragma unroll
      for (int k = TL - 1; k >= 1; k -= 2) {
        const double2 yy = ybuf[k >> 1][lane];
        const double y1 = lp_step(zb, f, yy.y);
        const double y0 = lp_step(zb, f, yy.x);
        accb = tiny_min3(accb, y1, y0);
        if constexpr (SPS > 0) {
          if (k % SPS == FM) symp[(t * (TL / SPS) + (k - FM) / SPS - q0) * 64] = y1;
          if ((k - 1) % SPS == FM) symp[(t * (TL / SPS) + (k - 1 - FM) / SPS - q0) * 64] = y0;
        } else {
          sym_out(t * TL + k, y1);
          sym_out(t * TL + k - 1, y0);
        }
      }
      __syncthreads();
    }
    for (int e = pad + (int)nh - 1; e >= 0; --e) {
      const double y = lp_step(zb, f, eh[e * 64]);
      accb = tiny_min3(accb, y, y);
      const int64_t i = e - pad;
      if (i >= 0) sym_out(i, y);
    }
    bool bad = !(accb >= kTinyHi);
#pragma unroll
    for (int j = 0; j < 4; ++j) bad |= !__builtin_isfinite(zb[j]);
    if (bad && s < buf.n_streams) atomicOr(&buf.flags[s], 1);
  }
}

// ---------------------------------------------------------------------------
// host-side launchers (api.cpp)
static int lane_wpb() {
  // waves per workgroup of the lane kernels: AMR_LANE_WPB=1/2/4 (default 4:
  // with 16 batches in flight, 4-wave workgroups ran 4.85 ms/step against
  // 5.82 for one-wave workgroups -- the dispatcher spreads them better)
  static const int v = [] {
    const char* e = getenv("AMR_LANE_WPB");
    const int k = e ? atoi(e) : 4;
    return k == 1 || k == 2 ? k : 4;
  }();
  return v;
}

static int bp_split() {
  // role-split band-pass (k_bp_lane2): AMR_BP_SPLIT=0 turns it off
  static const int v = [] { const char* e = getenv("AMR_BP_SPLIT"); return e && e[0] == '0' ? 0 : 1; }();
  return v;
}

static int bp_prefwd() {
  // the band-pass forward pass as its own launch (k_bp_fwd) before the
  // role-split re-run / backward kernel: AMR_BP_PREFWD=1 / 0
  static const int v = [] { const char* e = getenv("AMR_BP_PREFWD"); return e && e[0] == '1' ? 1 : 0; }();
  return v;
}

static int bp_ck() {
  // band-pass checkpoint every AMR_BP_CK tiles (1 or 2; the LDS hand-off stays one tile)
  static const int v = [] { const char* e = getenv("AMR_BP_CK"); return e && e[0] == '2' ? 2 : 1; }();
  return v;
}

static int bp_zero_taps(const PskParams& p) {
  // skip the band-pass's +0.0 odd taps (detector + exact re-run of flagged
  // groups): AMR_BP_ZO=0 computes every tap instead
  static const int v = [] { const char* e = getenv("AMR_BP_ZO"); return e && e[0] == '0' ? 0 : 1; }();
  return v && p.bp_zero_odd && p.bp_sym;
}

template <typename T>
static hipError_t launch_bp(const PskBuffers& b, const PskParams& p, const Iir& f, hipStream_t st) {
  const int64_t g = (b.n_streams + 63) / 64;
  if (b.f32f) {
    // the float32 hand-off (the default throughput configuration only: split
    // roles, 4-wave workgroups, 32-sample checkpoints); its fix-up launch
    // comes after the low-pass, which flags streams too
    // (launch_psk_bandpass_fixup)
    if (!(bp_split() && lane_wpb() >= 2 && !bp_prefwd() && bp_ck() == 1)) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(b.bp_flags, 0, (size_t)b.n_streams * 4, st);
    if (e != hipSuccess) return e;
    const dim3 grid((unsigned)((g + 1) / 2)), block(256);
    if (bp_zero_taps(p)) hipLaunchKernelGGL((k_bp_lane2<T, 2, true, false, false, 1, true>), grid, block, 0, st, b, p, f);
    else hipLaunchKernelGGL((k_bp_lane2<T, 2, false, false, false, 1, true>), grid, block, 0, st, b, p, f);
    return hipGetLastError();
  }
  if (bp_split()) {
    const bool zo = bp_zero_taps(p);
    if (zo) {
      hipError_t e = hipMemsetAsync(b.bp_flags, 0, (size_t)b.n_streams * 4, st);
      if (e != hipSuccess) return e;
    }
    const dim3 grid((unsigned)(lane_wpb() >= 2 ? (g + 1) / 2 : g)), block(lane_wpb() >= 2 ? 256 : 128);
    if (lane_wpb() >= 2 && bp_prefwd()) {
      const dim3 fgrid((unsigned)((g + 3) / 4));
      if (zo) {
        hipLaunchKernelGGL((k_bp_fwd<T, true>), fgrid, dim3(256), 0, st, b, p, f);
        hipLaunchKernelGGL((k_bp_lane2<T, 2, true, false, true>), grid, block, 0, st, b, p, f);
      } else {
        hipLaunchKernelGGL((k_bp_fwd<T, false>), fgrid, dim3(256), 0, st, b, p, f);
        hipLaunchKernelGGL((k_bp_lane2<T, 2, false, false, true>), grid, block, 0, st, b, p, f);
      }
    } else if (lane_wpb() >= 2 && bp_ck() == 2) {
      if (zo) hipLaunchKernelGGL((k_bp_lane2<T, 2, true, false, false, 2>), grid, block, 0, st, b, p, f);
      else hipLaunchKernelGGL((k_bp_lane2<T, 2, false, false, false, 2>), grid, block, 0, st, b, p, f);
    } else if (lane_wpb() >= 2) {
      if (zo) hipLaunchKernelGGL((k_bp_lane2<T, 2, true>), grid, block, 0, st, b, p, f);
      else hipLaunchKernelGGL((k_bp_lane2<T, 2, false>), grid, block, 0, st, b, p, f);
    } else {
      if (zo) hipLaunchKernelGGL((k_bp_lane2<T, 1, true>), grid, block, 0, st, b, p, f);
      else hipLaunchKernelGGL((k_bp_lane2<T, 1, false>), grid, block, 0, st, b, p, f);
    }
    if (zo)   // every tap for the groups holding a flagged stream (the others exit at once)
      hipLaunchKernelGGL((k_bp_lane2<T, 1, false, true>), dim3((unsigned)g), dim3(128), 0, st, b, p, f);
    return hipGetLastError();
  }
  switch (lane_wpb()) {
    case 4: hipLaunchKernelGGL((k_bp_lane<T, 4>), dim3((unsigned)((g + 3) / 4)), dim3(256), 0, st, b, p, f); break;
    case 2: hipLaunchKernelGGL((k_bp_lane<T, 2>), dim3((unsigned)((g + 1) / 2)), dim3(128), 0, st, b, p, f); break;
    default: hipLaunchKernelGGL((k_bp_lane<T, 1>), dim3((unsigned)g), dim3(64), 0, st, b, p, f);
  }
  return hipGetLastError();
}

hipError_t launch_psk_bandpass_lane(const PskBuffers& b, const PskParams& p, const Iir& f, hipStream_t st) {
  if (f.nt != 9) return hipErrorInvalidValue;
  switch (b.dtype) {
    case kF32: return launch_bp<float>(b, p, f, st);
    case kF64: return launch_bp<double>(b, p, f, st);
    case kI16: return launch_bp<int16_t>(b, p, f, st);
    default: return hipErrorInvalidValue;
  }
}

// the float32 hand-off's fix-up: every tap, float64 f, for the groups holding
// a stream the band-pass detector or the low-pass margin flagged (bp_flags)
hipError_t launch_psk_bandpass_fixup(const PskBuffers& b, const PskParams& p, const Iir& f, hipStream_t st) {
  if (f.nt != 9) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((b.n_streams + 63) / 64)), block(128);
  switch (b.dtype) {
    case kF32: hipLaunchKernelGGL((k_bp_lane2<float, 1, false, true>), grid, block, 0, st, b, p, f); break;
    case kF64: hipLaunchKernelGGL((k_bp_lane2<double, 1, false, true>), grid, block, 0, st, b, p, f); break;
    case kI16: hipLaunchKernelGGL((k_bp_lane2<int16_t, 1, false, true>), grid, block, 0, st, b, p, f); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

static int lp_split() {
  // role-split low-pass (k_lp_lane2): AMR_LP_SPLIT=1 turns it on (off by
  // default: its 20-sample tiles double the checkpoint traffic and leave its
  // loads less time; 4.54 vs 4.29 ms/step at 16 in flight, same solo time)
  static const int v = [] { const char* e = getenv("AMR_LP_SPLIT"); return e && e[0] == '1' ? 1 : 0; }();
  return v;
}

template <int S_, int F_>
static bool launch_lp(const PskBuffers& b, const PskParams& p, const Iir& f, hipStream_t st) {
  const int64_t g = (b.n_streams + 63) / 64;
  if (lp_split()) {
    hipLaunchKernelGGL((k_lp_lane2<S_, F_, kLpT2>), dim3((unsigned)g), dim3(256), 0, st, b, p, f);
    return false;
  }
  // the slicer inside the low-pass (static slots, both components in one
  // workgroup) once at least 32768 streams are live: it saves the symbols'
  // HBM round trip (+4-5 % per step at 16 x 4096 in flight) but lengthens a
  // lone batch's low-pass (11.0 -> 13.7 ms: the re wave slices between
  // barriers), which is what a small live set (a 1024-stream shard) waits
  // on.  AMR_FUSED_SLICE=1 / 0 forces it on / off.
  static const int fuse_env = [] {
    const char* e = getenv("AMR_FUSED_SLICE");
    return e ? (e[0] == '1' ? 1 : 0) : -1;
  }();
  const int64_t live = b.n_streams * (b.inflight > 1 ? b.inflight : 1);
  const bool fuse = S_ > 0 && lane_wpb() >= 2 && (fuse_env >= 0 ? fuse_env == 1 : live >= 32768);
  if (b.f32f) {
    // the float32 hand-off needs the fused slicer (api.cpp asks psk_lane_fused first)
    if (!(fuse && S_ != 0 && lane_wpb() == 4)) return false;
    hipLaunchKernelGGL((k_lp_lane<S_, F_, 4, S_ != 0, S_ != 0>), dim3((unsigned)((g + 1) / 2)), dim3(256), 0, st, b, p, f);
    return true;
  }
  switch (lane_wpb()) {
    case 4:
      if (fuse) hipLaunchKernelGGL((k_lp_lane<S_, F_, 4, S_ != 0>), dim3((unsigned)((g + 1) / 2)), dim3(256), 0, st, b, p, f);
      else hipLaunchKernelGGL((k_lp_lane<S_, F_, 4>), dim3((unsigned)((g + 1) / 2)), dim3(256), 0, st, b, p, f);
      break;
    case 2:
      if (fuse) hipLaunchKernelGGL((k_lp_lane<S_, F_, 2, S_ != 0>), dim3((unsigned)g), dim3(128), 0, st, b, p, f);
      else hipLaunchKernelGGL((k_lp_lane<S_, F_, 2>), dim3((unsigned)g), dim3(128), 0, st, b, p, f);
      break;
    default:
      // a multiple of 16 blocks: the re/im XCD pairing is a bijection
      hipLaunchKernelGGL((k_lp_lane<S_, F_, 1>), dim3((unsigned)((2 * g + 15) / 16 * 16)), dim3(64), 0, st, b, p, f);
  }
  return fuse;
}

// whether launch_psk_lowpass_lane will run the fused slicer for this batch
// (the float32 hand-off's precondition, api.cpp)
bool psk_lane_fused(const PskBuffers& b, const PskParams& p) {
  const int fm = (int)(p.first % (p.sps > 0 ? p.sps : 1));
  const bool stat = p.first <= kLpT2 && ((p.sps == 10 && (fm == 5 || fm == 0)) || (p.sps == 5 && (fm == 2 || fm == 0)) ||
                                         (p.sps == 20 && (fm == 10 || fm == 0)));
  static const int fuse_env = [] {
    const char* e = getenv("AMR_FUSED_SLICE");
    return e ? (e[0] == '1' ? 1 : 0) : -1;
  }();
  const int64_t live = b.n_streams * (b.inflight > 1 ? b.inflight : 1);
  return stat && !lp_split() && lane_wpb() == 4 && (fuse_env >= 0 ? fuse_env == 1 : live >= 32768);
}

hipError_t launch_psk_lowpass_lane(const PskBuffers& b, const PskParams& p, const Iir& f, hipStream_t st,
                                   bool* sliced) {
  if (f.nt != 5) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(b.flags, 0, (size_t)b.n_streams * 4, st);
  if (e != hipSuccess) return e;
  const int fm = (int)(p.first % (p.sps > 0 ? p.sps : 1));
  bool fused = false;
  // the static symbol slots number tile t's symbols from t * (TL / SPS) - first / SPS:
  // valid (>= 0 from the first whole tile on) while first <= the tile length;
  // a later first (the C ABI allows any) takes the generic path
  if (p.first > kLpT2) fused = launch_lp<0, 0>(b, p, f, st);
  else if (p.sps == 10 && fm == 5) fused = launch_lp<10, 5>(b, p, f, st);
  else if (p.sps == 5 && fm == 2) fused = launch_lp<5, 2>(b, p, f, st);
  else if (p.sps == 20 && fm == 10) fused = launch_lp<20, 10>(b, p, f, st);
  else if (p.sps == 10 && fm == 0) fused = launch_lp<10, 0>(b, p, f, st);
  else if (p.sps == 5 && fm == 0) fused = launch_lp<5, 0>(b, p, f, st);
  else if (p.sps == 20 && fm == 0) fused = launch_lp<20, 0>(b, p, f, st);
  else fused = launch_lp<0, 0>(b, p, f, st);
  if (sliced) *sliced = fused;
  return hipGetLastError();
}

}  // namespace amr
