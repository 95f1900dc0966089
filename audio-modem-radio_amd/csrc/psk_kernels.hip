// psk_kernels.hip -- batched DQPSK / DBPSK demodulation for gfx950 (MI355X).
//
// Replaces, for a batch of B streams at once, the per-stream reference
//   modem.qpsk_demodulate  (/root/reference/modem.py:189-266)
//   modem.bpsk_demodulate  (/root/reference/modem.py:68-135)
// and every alias that dispatches to them (psk8_demodulate modem.py:348,
// ofdm_demodulate_simple modem.py:375-376, decoder.py:422-434).
//
// Bit-exactness contract: every floating-point operation below is the one
// numpy/scipy performs, in the same order, with no contraction (this file is
// compiled with -ffp-contract=off; every fma() is an fma numpy itself uses).
// The oracle (oracle/amr_oracle.c) states the same arithmetic on the CPU.
//
// Pipeline for one batch (one kernel per stage, all streams in flight):
//   K1r k_bandpass_row   16-lane DPP row = stream (lane 8+j owns state j):
//                        band-pass filtfilt.  Forward pass reads the caller's
//                        stream-major samples through an LDS tile and writes
//                        s1 through an LDS staging image; the backward pass
//                        streams s1 back through an LDS-DMA ring and writes
//                        the real filtered signal f to s2 the same way.
//   K2q k_lowpass_fwd_q  lane quad = one component of one stream (lane j owns
//                        state j), wave = 16 streams x (re|im): LO mixer
//                        (numpy's complex multiply) fused into the low-pass
//                        forward pass -> s3
//   K3q k_lowpass_bwd_q  same lanes: low-pass backward pass; the baseband at
//                        each symbol centre goes to the symbol buffer
//   K4a k_slice          workgroup = 64 streams x 32 words, lane = stream: differential product,
//                        QPSK/BPSK slicer, bit packing -> words (fully parallel)
//   K3x k_lowpass_exact  lane = stream: the complex low-pass with scipy's full
//                        signed-zero semantics, only for streams K2q/K3q flagged
//   (K4b sync + pack lives in util_kernels.hip)
// (The layouts they replaced -- lane per stream, K1q quads, K2/K3 lane pairs
// -- are in DESIGN.md §4's progression and the git history.)
//
// At the benchmark batch (4096 streams) every wave runs alone on its SIMD, so
// each kernel is bound by its per-sample instruction stream;
// the memory side is arranged so that no load is waited on before it has had
// many chunks of compute to land and every memory instruction carries as much
// distinct data as the layout allows.
#include <math.h>
#include <stdlib.h>

#include <type_traits>

#include "amr_internal.h"
#include "psk_common.h"

namespace amr {

constexpr int kTileBytes = 256;                 // bytes of one stream per input tile
constexpr int kTilePitch = kTileBytes + 16;     // LDS row pitch: conflict-free ds_read_b128 per lane
constexpr int kBwdChunk = 32;                   // samples per backward prefetch chunk (16 pairs)

// ---------------------------------------------------------------------------
// 64-bit DPP move within quads (two 32-bit moves; every quad_perm source lane
// is valid, so no "old" value is needed)
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long u = __builtin_bit_cast(long long, v);
  // every source lane of a quad_perm is valid, so no "old" value is needed
  const int lo = __builtin_amdgcn_mov_dpp((int)(u & 0xffffffff), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(u >> 32), CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
constexpr int kQuadBcast0 = 0x00;   // quad_perm [0,0,0,0]

// ---------------------------------------------------------------------------
// K1r: the 9-tap band-pass with ONE STATE PER LANE of a 16-lane DPP row.
// A lone wave issues one FP64 instruction every ~4.7 cycles, so what bounds a
// stream is the length of its per-sample instruction stream.  K1q needed 16
// (10 FP64 + 6 moves); here lane 8+j of row r owns z[j] of stream 4w+r and a
// sample costs 9:
//   t     = z + b0*x                   (lane 8: t IS y)
//   y     = v_mov_b64 row_newbcast:8   (one 64-bit DPP move)
//   zC    = row_shl:1 (z)              (z[j+1] from lane 9+j: two 32-bit moves)
//   z     = (zC + x*b[j+1]) - y*a[j+1]
// Lane 15 (z[7]) reads beyond its row: its lo word comes back 0 (bound_ctrl)
// and its hi word is never written, so it keeps 0x80000000 -- zC is exactly
// -0.0 there and (-0.0 + x*b8) - y*a8 == x*b8 - y*a8 bit for bit.  Lanes 0-7
// run the same instructions on garbage nobody reads.  At the benchmark batch
// (4096 streams) the kernel is 1024 waves = one per SIMD
// (tools/step_probe2.hip: 51.5 vs 76.3 cycles/sample for K1q).
constexpr int kRowStreams = 4;                  // streams (DPP rows) per wave
constexpr int kBpRing = 8;                      // K1r backward LDS-DMA ring depth (32-sample chunks)

// s_waitcnt vmcnt(N) alone (gfx9 encoding: vmcnt[3:0] + vmcnt[5:4] at [15:14],
// expcnt[6:4] = 7 and lgkmcnt[11:8] = 15 mean "don't wait")
// -- as inline asm: the compiler's waitcnt pass does not know what the DMA
// feeds and would drop a __builtin_amdgcn_s_waitcnt it considers redundant.
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(%0)" : : "i"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// LDS-DMA (global_load_lds_dwordx4: each lane's 16 B to lds_dst + lane*16)
// issued as inline asm, so that the compiler does not know a DMA is in
// flight: it would make every LDS access it cannot prove disjoint from the
// target wait vmcnt(0) (and always does at loop headers), draining the ring.
// The caller waits for the data itself (vm_wait, counting every vector-memory
// instruction issued after the DMA).  M0 is written and restored inside the
// statement (recipe of cdna_hip_programming.md); "memory" keeps the compiler's
// LDS accesses on their side of it.
// f(integral_constant<int, 0>), ..., f(integral_constant<int, N-1>)
template <int N, int I = 0, typename F>
__device__ __forceinline__ void static_for_up(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for_up<N, I + 1>(f);
  }
}
// f(integral_constant<int, N-1>), ..., f(integral_constant<int, 0>)
template <int N, typename F>
__device__ __forceinline__ void static_for_down(F&& f) {
  if constexpr (N > 0) {
    f(std::integral_constant<int, N - 1>{});
    static_for_down<N - 1>(f);
  }
}

__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ void dma16(const void* gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}

// per-wave LDS of K1r's backward pass (the DMA ring is a separate __shared__
// object so that the compiler's LDS-DMA tracking can tell the staging
// accesses do not alias it)
struct BwdStage {
  uint8_t stage[1024];                          // output image of one chunk
  uint8_t junk[2048];                           // writes of the non-writer lanes
};

__device__ __forceinline__ double row_bcast8(double v) {
  const long u = __builtin_bit_cast(long, v);
  const long r = __builtin_amdgcn_update_dpp(0L, u, 0x158, 0xF, 0xF, true);   // row_newbcast:8
  return __builtin_bit_cast(double, r);
}
// z[j+1] from the next lane of the row; hk is the hi word's DPP destination,
// carried across steps so that the out-of-row lane keeps 0x80000000
__device__ __forceinline__ double row_next(double v, int& hk) {
  const long long u = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(u & 0xffffffff), 0x101, 0xF, 0xF, true);   // row_shl:1
  hk = __builtin_amdgcn_update_dpp(hk, (int)(u >> 32), 0x101, 0xF, 0xF, false);
  return __builtin_bit_cast(double, ((long long)hk << 32) | (unsigned)lo);
}

struct RowIir {
  double b0, cb, ca;
};


__device__ __forceinline__ double row_step(const RowIir& c, double& z, int& hk, double x) {
  const double t = z + c.b0 * x;
  const double y = row_bcast8(t);
  const double zC = row_next(z, hk);
  z = (zC + x * c.cb) - y * c.ca;
  return y;
}

// s1 for K1r: [w][q/2][4 streams][2] doubles
__device__ __forceinline__ size_t row_pair_index(int64_t w, int64_t m_pairs, int64_t q, int r) {
  return ((size_t)(w * m_pairs + (q >> 1)) * kRowStreams + r) * 2 + (q & 1);
}

template <typename T, int WPB>
__global__ __launch_bounds__(256) void k_bandpass_row(PskBuffers buf, PskParams p, Iir f) {
  if (buf.gate && *buf.gate == 0) return;   // a gated launch (PskBuffers::gate): whole grid
  __shared__ __attribute__((aligned(16))) uint8_t tiles[WPB][2][kRowStreams][kTilePitch];
  __shared__ __attribute__((aligned(16))) uint8_t bwd_ring[WPB][kBpRing][1024];   // s1 chunks (LDS-DMA)
  __shared__ __attribute__((aligned(16))) BwdStage bwd_st[WPB];
  constexpr int TS = kTileBytes / (int)sizeof(T);
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform (buffer rsrc, LDS bases)
  const int lane = threadIdx.x & 63;
  const int r = lane >> 4, l = lane & 15;
  const int j = l & 7;                          // state owned (lanes 8-15; 0-7 mirror them)
  const int64_t w = (int64_t)blockIdx.x * WPB + wv;
  const int64_t s = w * kRowStreams + r;
  const int64_t last = buf.n_streams - 1;
  if (w * kRowStreams > last) return;           // whole wave past the batch (wave-uniform)
  auto& tile = tiles[wv];
  const T* __restrict__ xall = reinterpret_cast<const T*>(buf.x);
  const T* __restrict__ x = xall + (s < last ? s : last) * buf.x_stride;
  const int64_t n = p.n;
  const int pad = p.pad1;
  const int64_t m1 = p.m1;
  const int qs = pad & 1;
  const int64_t m1_pairs = (m1 + qs + 1) >> 1;
  double* __restrict__ s1 = buf.s1;

  RowIir c;
  c.b0 = f.b[0];
  c.cb = f.b[j + 1];
  c.ca = f.a[j + 1];
  const double zi = f.zi[j];
  double z;
  int hk = (int)0x80000000;

  // ---- forward pass -------------------------------------------------------
  const OddExt<T> ox(x, buf.edge, s < last ? s : last, n, pad);
  z = zi * ox.left(0);
  for (int jj = 0; jj < pad; ++jj) {
    const double y = row_step(c, z, hk, ox.left(jj));
    s1[row_pair_index(w, m1_pairs, jj + qs, r)] = y;
  }
  const int64_t n_tiles = n / TS;
  const int64_t n_main = n_tiles * TS;
  // main-body stores as in the backward pass: each pair's (y0, y1) into the
  // wave's LDS staging image from lane 8 of its row (conflict-free junk slots
  // for the others), read back every 16 pairs and stored as one 1-KiB
  // instruction 16 pairs later
  uint8_t* const stage = bwd_st[wv].stage;
  uint8_t* const wr_base = l == 8 ? stage + r * 16 : bwd_st[wv].junk + (lane + r) * 16;
  if (n_tiles > 0) {
    // one tile = 4 stream rows x 256 B: one 16-B load per lane
    const int cb = l * 16;
    const uint8_t* rowp = reinterpret_cast<const uint8_t*>(x) + cb;
    v4u rv = *reinterpret_cast<const v4u*>(rowp);
    *reinterpret_cast<v4u*>(&tile[0][r][cb]) = rv;
    // this lane's 16 B of each image: s1 pair (image base + lane/4), row lane&3
    uint8_t* sdst = reinterpret_cast<uint8_t*>(s1) + (((size_t)w * m1_pairs + ((pad + qs) >> 1)) * kRowStreams + lane) * 16;
    v4u img;
    auto tile_body = [&](int64_t t, auto firstc) {
      constexpr bool FIRST = decltype(firstc)::value;
      const int cur = (int)(t & 1);
      const int64_t tn = (t + 1 < n_tiles) ? t + 1 : t;
      rv = *reinterpret_cast<const v4u*>(rowp + tn * kTileBytes);
      __builtin_amdgcn_sched_barrier(0);
      constexpr int PER = 16 / (int)sizeof(T);
      // the row's whole tile into registers at once: one LDS round trip per
      // tile instead of one per 16 B (the reads are broadcasts, 4 addresses)
      v4u xv[TS / PER];
#pragma unroll
      for (int k = 0; k < TS / PER; ++k) xv[k] = *reinterpret_cast<const v4u*>(&tile[cur][r][k * 16]);
      static_for_up<TS / 2>([&](auto jc) {
        constexpr int jp = decltype(jc)::value;             // pair of the tile
        T xs[PER];
        __builtin_memcpy(xs, &xv[(2 * jp) / PER], 16);
        const double y0 = row_step(c, z, hk, In<T>::cvt(xs[(2 * jp) % PER]));
        const double y1 = row_step(c, z, hk, In<T>::cvt(xs[(2 * jp) % PER + 1]));
        *reinterpret_cast<v4u*>(wr_base + (jp % 16) * 64) = __builtin_bit_cast(v4u, make_double2(y0, y1));
        if constexpr (jp % 16 == 15) {
          if constexpr (!(FIRST && jp == 15)) {
            *reinterpret_cast<v4u*>(sdst) = img;
            sdst += 1024;
          }
          img = *reinterpret_cast<const v4u*>(stage + lane * 16);
        }
      });
      __builtin_amdgcn_sched_barrier(0);
      *reinterpret_cast<v4u*>(&tile[cur ^ 1][r][cb]) = rv;
    };
    static_assert(TS / 2 % 16 == 0, "a tile holds whole staging images");
    tile_body(0, std::true_type{});
    for (int64_t t = 1; t < n_tiles; ++t) tile_body(t, std::false_type{});
    *reinterpret_cast<v4u*>(sdst) = img;        // the last image
  }
  for (int64_t i = n_main; i < n; ++i) {
    const double y = row_step(c, z, hk, In<T>::cvt(x[i]));
    s1[row_pair_index(w, m1_pairs, pad + i + qs, r)] = y;
  }
  double ylast = 0.0;
  for (int jj = 0; jj < pad; ++jj) {
    ylast = row_step(c, z, hk, ox.right(jj));
    s1[row_pair_index(w, m1_pairs, pad + n + jj + qs, r)] = ylast;
  }
  __threadfence();

  // ---- backward pass ------------------------------------------------------
  z = zi * ylast;
  hk = (int)0x80000000;
  for (int64_t jj = m1 - 1; jj >= pad + n; --jj)
    (void)row_step(c, z, hk, s1[row_pair_index(w, m1_pairs, jj + qs, r)]);

  const int64_t n2 = (n + 1) >> 1;
  double* __restrict__ fo = buf.s2;
  const int64_t sgrp = s >> 6;
  const int sig = (int)(s & 63);
  const int64_t nb = n / kBwdChunk;
  const int64_t n_lo = nb * kBwdChunk;
  for (int64_t i = n - 1; i >= n_lo; --i) {
    const double y = row_step(c, z, hk, s1[row_pair_index(w, m1_pairs, pad + i + qs, r)]);
    fo[f_index(sgrp, n2, i, sig)] = y;
  }
  if (nb > 0) {
    // Main body, chunks of 32 samples walked downwards.  Every memory
    // instruction moves 1 KiB of distinct data: the TA spends the same cycles
    // on a wave instruction whatever its lanes hold, and with one load + one
    // store per sample pair from all 64 lanes it was busy 93 % of the kernel.
    //   in : one LDS-DMA (global_load_lds_dwordx4) per chunk = 16 pairs x 4
    //        rows of s1, into a ring of kBpRing chunks; each pair is then a
    //        broadcast ds_read_b128 (4 addresses per wave)
    //   out: each pair's (y0, y1) goes to an LDS staging image from lane 8 of
    //        its row (the other lanes write a junk area: no exec masking);
    //        per chunk one ds_read_b128 + one global store of the image
    // LDS-DMA completion is tracked by vmcnt only, and the compiler adds no
    // wait between the DMA and the ds_reads of its data: vm_wait() below.
    constexpr int PP = kBwdChunk / 2;
    static_assert(PP * kRowStreams * 16 == 1024, "one DMA wave-instruction per chunk");
    constexpr int R = kBpRing;
    uint8_t* const ring = bwd_ring[wv][0];
    uint8_t* const stage = bwd_st[wv].stage;
    // junk slots chosen so that the 8 lanes of each LDS cycle group write 8
    // different 16-B bank groups: lane l of row r -> bank group (l + r) mod 8,
    // the writer (l = 8) included
    uint8_t* const wr_base = l == 8 ? stage + r * 16 : bwd_st[wv].junk + (lane + r) * 16;
    // this lane's 16 B of each chunk: s1 pair (chunk base + lane/4), row lane&3
    const uint8_t* gsrc = reinterpret_cast<const uint8_t*>(s1) +
                          (((size_t)w * m1_pairs + ((pad + qs + (nb - 1) * kBwdChunk) >> 1)) * kRowStreams + lane) * 16;
    // ... and of each chunk's output image: f pair (chunk base + lane/4), stream lane&3
    const int64_t hgrp = (w * kRowStreams) >> 5;
    uint8_t* fdst = reinterpret_cast<uint8_t*>(fo) +
                    (((size_t)(hgrp * n2) + (size_t)((nb - 1) * PP) + (lane >> 2)) * 32 +
                     (size_t)(((w * kRowStreams) & 31) + (lane & 3))) * 16;
    auto dma = [&](int slot) {
      dma16(gsrc, lds_addr(ring + slot * 1024));
      gsrc -= 1024;
    };
    auto run = [&](int slot) {
      const uint8_t* rs = ring + slot * 1024 + r * 16;
      v4u xv[PP];                               // the whole chunk up front: one LDS round trip
#pragma unroll
      for (int k = 0; k < PP; ++k) xv[k] = *reinterpret_cast<const v4u*>(rs + k * 64);
      static_for_down<PP>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        const double2 xx = __builtin_bit_cast(double2, xv[k]);
        const double y1 = row_step(c, z, hk, xx.y);
        const double y0 = row_step(c, z, hk, xx.x);
        *reinterpret_cast<v4u*>(wr_base + k * 64) = __builtin_bit_cast(v4u, make_double2(y0, y1));
      });
    };
    // the image is read back right after its chunk and stored one chunk later,
    // when the read has long returned (LDS keeps the read ahead of the next
    // chunk's writes)
    v4u img;
    auto flush = [&](auto storec) {
      if constexpr (decltype(storec)::value) {
        *reinterpret_cast<v4u*>(fdst) = img;
        fdst -= (size_t)PP * 32 * 16;
      }
      img = *reinterpret_cast<const v4u*>(stage + lane * 16);
    };
#pragma unroll
    for (int u = 0; u < R; ++u) dma(u);
    int64_t cc = nb - 1;
    // first R chunks: fewer ops are younger than their DMA (no stores yet);
    // the very first chunk has no image to store yet
    static_for_up<R>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      if (cc - u < 0) return;
      vm_wait<R - 1>();
      run(u);
      dma(u);
      flush(std::integral_constant<bool, (u > 0)>{});
    });
    cc -= R;
    // steady state: each DMA has 2R-1 younger vector-memory ops when its
    // chunk comes up (R-1 DMAs + R stores)
    for (; cc >= 0; cc -= R) {
#pragma unroll
      for (int u = 0; u < R; ++u) {
        if (cc - u < 0) break;
        vm_wait<2 * R - 1>();
        run(u);
        dma(u);
        flush(std::true_type{});
      }
    }
    *reinterpret_cast<v4u*>(fdst) = img;        // the last chunk's image
    vm_wait<0>();                               // no DMA may land after the wave ends
  }
}

// ---------------------------------------------------------------------------
// K1g: the 9-tap band-pass with one state per lane of an 8-lane GROUP, 8
// streams per wave (K1r keeps 4: its row's lanes 0-7 only mirror lanes 8-15).
// Half the waves for the same streams: at B = 4096 the band-pass is 512 waves
// and leaves half the SIMDs to the other batch in flight (bench.py), at
// ~1.75x K1r's streams per issue slot (tools/step_probe2.hip "group8").
//   t  = z + b0*x                            (lane j = 0: t IS y)
//   y  = v_mov_b64 row_newbcast:0 (banks 0-1) then row_newbcast:8 (banks 2-3)
//   zC = row_shl:1 (z), and exactly -0.0 on the group's top lane j = 7
//        (two v_cndmask: lane 7 would read the next group's z0)
//   z  = (zC + x*b[j+1]) - y*a[j+1]
// Memory as K1r: forward input tiles of 8 streams x 128 B (one 16-B load per
// lane) through LDS; outputs through a 1-KiB LDS staging image (8 pairs x 8
// streams) stored with one instruction; backward input by LDS-DMA, 1 KiB =
// 8 pairs x 8 streams of s1 per chunk.
constexpr int kG8Streams = 8;                   // streams (8-lane groups) per wave
constexpr int kG8TileBytes = 128;               // bytes of one stream per forward input tile
constexpr int kG8Pitch = kG8TileBytes + 16;
constexpr int kG8Chunk = 16;                    // samples per backward DMA chunk (8 pairs)
constexpr int kG8Ring = 8;                      // backward DMA ring depth (chunks)

struct G8Stage {
  uint8_t stage[1024];                          // output image: [pair k][stream g] 16 B
  uint8_t junk[256];                            // writes of the non-writer lanes
};

// s1 for K1g: [w][q/2][8 streams][2] doubles
__device__ __forceinline__ size_t g8_pair_index(int64_t w, int64_t m_pairs, int64_t q, int g) {
  return ((size_t)(w * m_pairs + (q >> 1)) * kG8Streams + g) * 2 + (q & 1);
}

__device__ __forceinline__ double g8_step(const RowIir& c, double& z, bool top, double x) {
  const double t = z + c.b0 * x;
  const long u = __builtin_bit_cast(long, t);
  const long r1 = __builtin_amdgcn_update_dpp(0L, u, 0x150, 0xF, 0x3, false);    // row_newbcast:0 -> lanes 0-7
  const long r2 = __builtin_amdgcn_update_dpp(r1, u, 0x158, 0xF, 0xC, false);    // row_newbcast:8 -> lanes 8-15
  const double y = __builtin_bit_cast(double, r2);
  const long long zu = __builtin_bit_cast(long long, z);
  int lo = __builtin_amdgcn_update_dpp(0, (int)(zu & 0xffffffff), 0x101, 0xF, 0xF, true);   // row_shl:1
  int hi = __builtin_amdgcn_update_dpp(0, (int)(zu >> 32), 0x101, 0xF, 0xF, true);
  lo = top ? 0 : lo;
  hi = top ? (int)0x80000000 : hi;
  const double zC = __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
  z = (zC + x * c.cb) - y * c.ca;
  return y;
}

template <typename T, int WPB>
__global__ __launch_bounds__(256) void k_bandpass_g8(PskBuffers buf, PskParams p, Iir f) {
  if (buf.gate && *buf.gate == 0) return;   // a gated launch (PskBuffers::gate): whole grid
  __shared__ __attribute__((aligned(16))) uint8_t tiles[WPB][2][kG8Streams][kG8Pitch];
  __shared__ __attribute__((aligned(1024))) uint8_t ring[WPB][kG8Ring][1024];   // s1 chunks (LDS-DMA)
  __shared__ __attribute__((aligned(1024))) G8Stage st8[WPB];
  constexpr int TS = kG8TileBytes / (int)sizeof(T);    // samples per input tile
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int g = lane >> 3, j = lane & 7;
  const bool top = j == 7;
  const int64_t w = (int64_t)blockIdx.x * WPB + wv;
  const int64_t s = w * kG8Streams + g;
  const int64_t last = buf.n_streams - 1;
  if (w * kG8Streams > last) return;            // whole wave past the batch (wave-uniform)
  auto& tile = tiles[wv];
  const T* __restrict__ xall = reinterpret_cast<const T*>(buf.x);
  const T* __restrict__ x = xall + (s < last ? s : last) * buf.x_stride;
  const int64_t n = p.n;
  const int pad = p.pad1;
  const int64_t m1 = p.m1;
  const int qs = pad & 1;
  const int64_t m1_pairs = (m1 + qs + 1) >> 1;
  double* __restrict__ s1 = buf.s1;

  RowIir c;
  c.b0 = f.b[0];
  c.cb = f.b[j + 1];
  c.ca = f.a[j + 1];
  const double zi = f.zi[j];
  double z;

  // writer lane j = 0 of group g -> image slot (k, g); the 7 others -> junk
  // slots whose 16-B bank groups avoid the writer's ((8k + g) mod 16) and each
  // other within the 8-lane LDS cycle group (= this group)
  uint8_t* const stage = st8[wv].stage;
  uint8_t* const jb0 = st8[wv].junk + ((g + j) & 15) * 16;          // k even
  uint8_t* const jb1 = st8[wv].junk + ((g + j + 8) & 15) * 16;      // k odd
  auto wr_addr = [&](int k) -> uint8_t* {
    return j == 0 ? stage + (k * kG8Streams + g) * 16 : ((k & 1) ? jb1 : jb0);
  };

  // ---- forward pass -------------------------------------------------------
  const OddExt<T> ox(x, buf.edge, s < last ? s : last, n, pad);
  z = zi * ox.left(0);
  for (int jj = 0; jj < pad; ++jj) {
    const double y = g8_step(c, z, top, ox.left(jj));
    s1[g8_pair_index(w, m1_pairs, jj + qs, g)] = y;
  }
  const int64_t n_tiles = n / TS;
  const int64_t n_main = n_tiles * TS;
  if (n_tiles > 0) {
    // one tile = 8 stream rows x 128 B: one 16-B load per lane
    const int tr = lane >> 3, cb = (lane & 7) * 16;
    const T* __restrict__ xr = xall + ((w * kG8Streams + tr) < last ? (w * kG8Streams + tr) : last) * buf.x_stride;
    const uint8_t* rowp = reinterpret_cast<const uint8_t*>(xr) + cb;
    v4u rv = *reinterpret_cast<const v4u*>(rowp);
    *reinterpret_cast<v4u*>(&tile[0][tr][cb]) = rv;
    uint8_t* sdst = reinterpret_cast<uint8_t*>(s1) +
                    (((size_t)w * m1_pairs + ((pad + qs) >> 1)) * kG8Streams) * 16 + lane * 16;
    v4u img;
    auto tile_body = [&](int64_t t, auto firstc) {
      constexpr bool FIRST = decltype(firstc)::value;
      const int cur = (int)(t & 1);
      const int64_t tn = (t + 1 < n_tiles) ? t + 1 : t;
      rv = *reinterpret_cast<const v4u*>(rowp + tn * kG8TileBytes);
      __builtin_amdgcn_sched_barrier(0);
      constexpr int PER = 16 / (int)sizeof(T);
      v4u xv[TS / PER];
#pragma unroll
      for (int k = 0; k < TS / PER; ++k) xv[k] = *reinterpret_cast<const v4u*>(&tile[cur][g][k * 16]);
      static_for_up<TS / 2>([&](auto jc) {
        constexpr int jp = decltype(jc)::value;             // pair of the tile
        T xs[PER];
        __builtin_memcpy(xs, &xv[(2 * jp) / PER], 16);
        const double y0 = g8_step(c, z, top, In<T>::cvt(xs[(2 * jp) % PER]));
        const double y1 = g8_step(c, z, top, In<T>::cvt(xs[(2 * jp) % PER + 1]));
        *reinterpret_cast<v4u*>(wr_addr(jp % 8)) = __builtin_bit_cast(v4u, make_double2(y0, y1));
        if constexpr (jp % 8 == 7) {
          if constexpr (!(FIRST && jp == 7)) {
            *reinterpret_cast<v4u*>(sdst) = img;
            sdst += 1024;
          }
          img = *reinterpret_cast<const v4u*>(stage + lane * 16);
        }
      });
      __builtin_amdgcn_sched_barrier(0);
      *reinterpret_cast<v4u*>(&tile[cur ^ 1][tr][cb]) = rv;
    };
    static_assert(TS / 2 % 8 == 0, "a tile holds whole staging images");
    tile_body(0, std::true_type{});
    for (int64_t t = 1; t < n_tiles; ++t) tile_body(t, std::false_type{});
    *reinterpret_cast<v4u*>(sdst) = img;        // the last image
  }
  for (int64_t i = n_main; i < n; ++i) {
    const double y = g8_step(c, z, top, In<T>::cvt(x[i]));
    s1[g8_pair_index(w, m1_pairs, pad + i + qs, g)] = y;
  }
  double ylast = 0.0;
  for (int jj = 0; jj < pad; ++jj) {
    ylast = g8_step(c, z, top, ox.right(jj));
    s1[g8_pair_index(w, m1_pairs, pad + n + jj + qs, g)] = ylast;
  }
  __threadfence();

  // ---- backward pass ------------------------------------------------------
  z = zi * ylast;
  for (int64_t jj = m1 - 1; jj >= pad + n; --jj)
    (void)g8_step(c, z, top, s1[g8_pair_index(w, m1_pairs, jj + qs, g)]);

  const int64_t n2 = (n + 1) >> 1;
  double* __restrict__ fo = buf.s2;
  const int64_t sgrp = s >> 6;
  const int sig = (int)(s & 63);
  const int64_t nb = n / kG8Chunk;
  const int64_t n_lo = nb * kG8Chunk;
  for (int64_t i = n - 1; i >= n_lo; --i) {
    const double y = g8_step(c, z, top, s1[g8_pair_index(w, m1_pairs, pad + i + qs, g)]);
    fo[f_index(sgrp, n2, i, sig)] = y;
  }
  if (nb > 0) {
    constexpr int PP = kG8Chunk / 2;
    static_assert(PP * kG8Streams * 16 == 1024, "one DMA wave-instruction per chunk");
    constexpr int R = kG8Ring;
    uint8_t* const rg = ring[wv][0];
    // this lane's 16 B of each chunk: s1 pair (chunk base + lane/8), stream lane&7
    const uint8_t* gsrc = reinterpret_cast<const uint8_t*>(s1) +
                          (((size_t)w * m1_pairs + ((pad + qs + (nb - 1) * kG8Chunk) >> 1)) * kG8Streams + lane) * 16;
    // ... and of each chunk's output image: f pair (chunk base + lane/8), stream lane&7
    const int64_t s0 = w * kG8Streams;
    uint8_t* fdst = reinterpret_cast<uint8_t*>(fo) +
                    ((((size_t)((s0 >> 6) * 2 + ((s0 >> 5) & 1)) * n2) + (size_t)((nb - 1) * PP) + (lane >> 3)) * 32 +
                     (size_t)((s0 & 31) + (lane & 7))) * 16;
    auto dma = [&](int slot) {
      dma16(gsrc, lds_addr(rg + slot * 1024));
      gsrc -= 1024;
    };
    auto run = [&](int slot) {
      const uint8_t* rs = rg + slot * 1024 + g * 16;
      v4u xv[PP];                               // the whole chunk up front: one LDS round trip
#pragma unroll
      for (int k = 0; k < PP; ++k) xv[k] = *reinterpret_cast<const v4u*>(rs + k * 128);
      static_for_down<PP>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        const double2 xx = __builtin_bit_cast(double2, xv[k]);
        const double y1 = g8_step(c, z, top, xx.y);
        const double y0 = g8_step(c, z, top, xx.x);
        *reinterpret_cast<v4u*>(wr_addr(k)) = __builtin_bit_cast(v4u, make_double2(y0, y1));
      });
    };
    v4u img;
    auto flush = [&](auto storec) {
      if constexpr (decltype(storec)::value) {
        *reinterpret_cast<v4u*>(fdst) = img;
        fdst -= (size_t)PP * 32 * 16;
      }
      img = *reinterpret_cast<const v4u*>(stage + lane * 16);
    };
#pragma unroll
    for (int u = 0; u < R; ++u) dma(u);
    int64_t cc = nb - 1;
    static_for_up<R>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      if (cc - u < 0) return;
      vm_wait<R - 1>();
      run(u);
      dma(u);
      flush(std::integral_constant<bool, (u > 0)>{});
    });
    cc -= R;
    for (; cc >= 0; cc -= R) {
#pragma unroll
      for (int u = 0; u < R; ++u) {
        if (cc - u < 0) break;
        vm_wait<2 * R - 1>();
        run(u);
        dma(u);
        flush(std::true_type{});
      }
    }
    *reinterpret_cast<v4u*>(fdst) = img;        // the last chunk's image
    vm_wait<0>();                               // no DMA may land after the wave ends
  }
}

// ---------------------------------------------------------------------------
// Low-pass: the mixer (modem.py:200-201) is numpy's complex multiply
// (f + 0j) * lo:  re = fma(f, lo_re, -(0*lo_im)),  im = fma(f, lo_im, 0*lo_re);
// the plan stores, per sample and component, (lo_c, addend_c).
//
// The complex lfilter with real coefficients is two real recurrences EXCEPT
// for the sign of zero results (scipy evaluates b*x as b*xr - (+0)*xi, ...).
// The separable recurrences are exact whenever every tap product is a
// non-zero finite number, which holds when every input
// and output magnitude is >= 2^-1022 and nothing is inf/NaN.  K2q/K3q track
// that (the detector below) and flag a stream that fails it; K3x recomputes
// it with the full complex semantics.  The single sample that is +0 by
// construction (bb_im[0]: lo_im[0] == -0) is judged by its class instead: +0
// there is provably harmless.
constexpr int kLpChunk = 16;                    // samples per low-pass prefetch chunk

// ---------------------------------------------------------------------------
// K2q / K3q: the low-pass with ONE STATE PER LANE of a quad (lane j owns z[j]
// of the 5-tap recurrence); a wave serves 16 streams x one component, so the
// LO stays wave-uniform.  Per sample 11 VALU instead of the pair split's 16:
//   t  = z + b0*x ; y = quad_perm[0,0,0,0](t)
//   zC = quad_perm[1,2,3,3](z) * m      (m = 1, and 0 on the top lane j = 3)
//   z  = (zC + x*b[j+1]) - y*a[j+1]
// On the top lane zC*0 is a signed zero, and (+-0 + x*b4) == x*b4 whenever
// x*b4 != 0, i.e. whenever x != 0 (b4 >= 2^-50, checked at plan time): every
// input the detector lets through.  So the recurrence is scipy's bit for bit
// on every stream that is not flagged, and flagged streams are recomputed by
// K3x as before.
//
// Detector (one VALU per sample in K2q, half in K3q): the minimum over
// |hi word read as float32| of the values that must be >= 2^-1022.  That hi
// word is >= FLT_MIN exactly when the double's exponent field is >= 8, i.e.
// |v| >= 2^-1015, so zeros and denormals are always caught (values in
// [2^-1022, 2^-1015) are flagged too -- conservative, they take the exact
// path).  Infinities and NaN are sticky and caught by the final-state test.
// v_min3_f32 runs in inline asm so the compiler adds no NaN canonicalisation.
constexpr int kQuadShift = 0xF9;                // quad_perm [1,2,3,3]
constexpr int kLpQChunk = 8;                    // K2q main-body chunk (samples)
constexpr int kLpQRing = 8;                     // K2q f prefetch ring depth (8-sample chunks)
constexpr int kLpBRing = 5;                     // K3q prefetch ring depth (chunks of 20/16 samples)
struct Quad5 {
  double b0, cb, ca, cm;
};

__device__ __forceinline__ Quad5 quad5_coef(const Iir& f, int j, double& zi) {
  Quad5 c;
  c.b0 = f.b[0];
  c.cb = f.b[j + 1];
  c.ca = f.a[j + 1];
  c.cm = j == 3 ? 0.0 : 1.0;
  zi = f.zi[j];
  return c;
}

__device__ __forceinline__ double quad5_step(const Quad5& c, double& z, double x) {
  const double t = z + c.b0 * x;
  const double y = dpp_f64<kQuadBcast0>(t);
  const double zC = dpp_f64<kQuadShift>(z) * c.cm;
  z = (zC + x * c.cb) - y * c.ca;
  return y;
}

// s3 for K2q/K3q: [w16][comp][q/2][16 streams][2] doubles
__device__ __forceinline__ size_t s3q_index(int64_t w, int comp, int64_t m_pairs, int64_t q, int sq) {
  return ((((size_t)((w * 2 + comp) * m_pairs + (q >> 1))) * 16 + sq) * 2) + (q & 1);
}

__device__ __forceinline__ void quad_flag(PskBuffers& buf, int64_t s, int j, bool bad) {
  int fl = bad ? 1 : 0;
  fl |= __shfl_xor(fl, 1);
  fl |= __shfl_xor(fl, 2);
  if (j == 0 && s < buf.n_streams && fl) atomicOr(&buf.flags[s], 1);
}

__global__ __launch_bounds__(64) void k_lowpass_fwd_q(PskBuffers buf, PskParams p, Iir f) {
  if (buf.gate && *buf.gate == 0) return;   // a gated launch (PskBuffers::gate): whole grid
  const int lane = threadIdx.x;
  const int j = lane & 3, sq = lane >> 2;
  // blocks b and b+8 land on the same XCD (blocks are dealt to the 8 XCDs
  // round-robin) and run the re and im waves of the same 16 streams, so the
  // second read of their f rows is an L2 hit instead of a second HBM read
  const int64_t bx = blockIdx.x, kx = bx >> 3;
  const int64_t w = (kx >> 1) * 8 + (bx & 7);
  const int comp = (int)(kx & 1);
  const int64_t s = w * 16 + sq;
  if (w * 16 >= buf.n_streams) return;          // wave-uniform
  const int64_t n = p.n;
  const int64_t n2 = (n + 1) >> 1;
  const int pad = p.pad2;
  const int qs = pad & 1;
  const int64_t m2_pairs = (p.m2 + qs + 1) >> 1;
  const int64_t g = s >> 6;
  const double2* __restrict__ fsrc =
      reinterpret_cast<const double2*>(buf.s2) + (size_t)((g * 2 + ((s >> 5) & 1)) * n2) * 32 + (s & 31);
  const double2* __restrict__ lo = reinterpret_cast<const double2*>(buf.lo) + comp;   // (lo_c, addend) at lo[2i]
  const double* __restrict__ loc = buf.lo2 + comp * n;                               // lo_c alone
  double* __restrict__ s3 = buf.s3;

  double zi;
  const Quad5 c = quad5_coef(f, j, zi);
  bool bad = false;
  float acc = __builtin_inff();
  // numpy's (f + 0j) * lo: f*lo_c + addend (addend a signed zero)
  auto X = [&](int64_t i) {
    const double2 fp = fsrc[(size_t)(i >> 1) * 32];
    const double2 l = lo[2 * i];
    return ((i & 1) ? fp.y : fp.x) * l.x + l.y;
  };

  const double x0 = X(0), xl = X(n - 1);
  bad |= __builtin_amdgcn_class(x0, kClsX);     // bb[0]: +0 allowed (judged by class)
  const double e0 = 2.0 * x0 - X(pad);
  bad |= __builtin_amdgcn_class(e0, kClsY);
  double z = zi * e0;
  for (int jj = 0; jj < pad; ++jj) {
    const double e = 2.0 * x0 - X(pad - jj);
    const double y = quad5_step(c, z, e);
    acc = tiny_min3(acc, e, y);
    s3[s3q_index(w, comp, m2_pairs, jj + qs, sq)] = y;
  }
  const int64_t nc = n / kLpQChunk;
  const int64_t n_main = nc * kLpQChunk;
  // the first kLpChunk samples hold bb[0] (full complex-multiply form, class-checked above)
  const int64_t n_gen = n >= kLpChunk ? kLpChunk : n;
  for (int64_t i = 0; i < n_gen; ++i) {
    const double e = i == 0 ? x0 : X(i);
    const double y = quad5_step(c, z, e);
    acc = tiny_min3(acc, i == 0 ? y : e, y);
    s3[s3q_index(w, comp, m2_pairs, pad + i + qs, sq)] = y;
  }
  constexpr int64_t kC0 = kLpChunk / kLpQChunk;   // chunks covered by the generic loop
  if (nc > kC0) {
    // main body: bb = f * lo_c (equal to f*lo_c + addend whenever it is not a
    // zero, and a zero is flagged).  At 2+ waves per CU this kernel is bound
    // by the texture addresser (TA), which spends the same cycles on a 64-lane
    // memory instruction whatever it holds: the f loads move
    // 256 B of distinct data each (a quad shares its stream's 16 B), and the
    // old wave-uniform LO loads and quad-shared stores 16 B and 256 B.  So:
    //   * LO: one 16-B load per lane brings 128 samples (1 KiB) into an LDS
    //     ring of 4 blocks, two blocks ahead; the register ring then reads
    //     it by broadcast ds_read_b128 (no TA);
    //   * stores: each pair goes into an LDS staging image (every lane writes
    //     its own 16 B: contiguous, conflict-free), read back once per chunk
    //     as this lane's 16 B of the chunk's 1 KiB of s3 and stored one chunk
    //     later -- one store instruction per 8 samples instead of four.
    // f keeps its register ring (R chunks deep).  Loads run up to R chunks
    // (LO: 3 blocks) past the stream's end into the plan's slack (api.cpp)
    // instead of clamping: every instruction here costs a wave issue slot.
    constexpr int CH = kLpQChunk, PP = CH / 2, R = kLpQRing, RL = 2;
    constexpr int LB = 128;                     // LO samples per LDS block (16 B per lane)
    constexpr int CPB = LB / CH;                // chunks per LO block = one loop iteration
    static_assert(CPB == 2 * R && R % RL == 0, "loop iteration = one LO block = two f rings");
    __shared__ __attribute__((aligned(16))) double2 lo_ring[4][LB / 2];
    __shared__ __attribute__((aligned(16))) double2 stage[2][PP][16][4];   // [buf][pair][stream][quad lane]
    double2 fr[R][PP];
    double2 lr[RL][PP];                         // LO multipliers (wave-uniform, a pair per ds_read_b128)
    const double2* __restrict__ fnext = fsrc + (size_t)kC0 * PP * 32;   // next f chunk to load
    const double2* __restrict__ lblk = reinterpret_cast<const double2*>(loc + kC0 * CH) + lane;
    double2* __restrict__ dstc = reinterpret_cast<double2*>(s3) + (s3q_index(w, comp, m2_pairs, pad + qs + kC0 * CH, 0) >> 1) + lane;
    // the first chunk has no predecessor: its "previous image" goes to the
    // plan's front slack below s3 (api.cpp kFrontSlack), never read as data
    double2* __restrict__ pdst = reinterpret_cast<double2*>(s3) - 64 + lane;
    double2 img = make_double2(0.0, 0.0);
    double2* const swr = &stage[0][0][0][0] + lane;                       // this lane's slot of pair 0
    const double2* const srd = &stage[0][lane >> 4][lane & 15][((lane & 15) >> 1) & 3];
    auto loadf = [&](double2 (&d)[PP]) {
#pragma unroll
      for (int k = 0; k < PP; ++k) d[k] = fnext[k * 32];
      fnext += PP * 32;
    };
    auto loadl = [&](double2 (&d)[PP], const double2* src) {
#pragma unroll
      for (int k = 0; k < PP; ++k) d[k] = src[k];
    };
    auto run = [&](const double2 (&fv)[PP], const double2 (&lv)[PP], int sb) {
#pragma unroll
      for (int k = 0; k < PP; ++k) {
        const double e0v = fv[k].x * lv[k].x;
        const double e1v = fv[k].y * lv[k].y;
        const double y0 = quad5_step(c, z, e0v);
        const double y1 = quad5_step(c, z, e1v);
        acc = tiny_min3(acc, e0v, e1v);
        acc = tiny_min3(acc, y0, y1);
        swr[(sb * PP + k) * 64] = make_double2(y0, y1);
      }
      *pdst = img;                              // the previous chunk's 16 B (read back a chunk ago)
      img = srd[sb * PP * 64];                  // this chunk's (LDS keeps a wave's accesses in order)
      pdst = dstc;
      dstc += PP * 16;
    };
    // prologue: LO blocks 0 and 1, then the rings
    lo_ring[0][lane] = lblk[0];
    lo_ring[1][lane] = lblk[LB / 2];
    lblk += LB;
#pragma unroll
    for (int u = 0; u < R; ++u) {
      loadf(fr[u]);
      if (u < RL) loadl(lr[u], &lo_ring[0][u * PP]);
      __builtin_amdgcn_sched_barrier(0);
    }
    // iteration ib covers LO block ib (chunks kC0 + 16 ib ...): it loads
    // block ib+2 at its start and writes it to the ring half way, where slot
    // (ib+2)&3 last held block ib-2, long consumed
    int64_t cc = kC0;
    int ib = 0;
    for (; cc + CPB <= nc; cc += CPB, ++ib) {
      const double2* const l0 = &lo_ring[ib & 3][0];
      const double2* const l1 = &lo_ring[(ib + 1) & 3][0];
      double2* const lw = &lo_ring[(ib + 2) & 3][lane];
      double2 lpend;
#pragma unroll
      for (int u = 0; u < CPB; ++u) {
        if (u == 0) { lpend = *lblk; lblk += LB / 2; }
        if (u == R) *lw = lpend;
        run(fr[u % R], lr[u % RL], u & 1);
        __builtin_amdgcn_sched_barrier(0);
        loadf(fr[u % R]);
        loadl(lr[u % RL], u + RL < CPB ? l0 + (u + RL) * PP : l1 + (u + RL - CPB) * PP);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    {
      // tail (< 16 chunks of block ib, written one iteration ago)
      const double2* const l0 = &lo_ring[ib & 3][0];
#pragma unroll
      for (int u = 0; u < CPB; ++u) {
        if (cc + u < nc) {
          run(fr[u % R], lr[u % RL], u & 1);
          if (u < R) loadf(fr[u]);
          if (u + RL < CPB) loadl(lr[u % RL], l0 + (u + RL) * PP);
        }
      }
    }
    *pdst = img;
  }
  for (int64_t i = n_main > n_gen ? n_main : n_gen; i < n; ++i) {
    const double e = X(i);
    const double y = quad5_step(c, z, e);
    acc = tiny_min3(acc, e, y);
    s3[s3q_index(w, comp, m2_pairs, pad + i + qs, sq)] = y;
  }
  for (int jj = 0; jj < pad; ++jj) {
    const double e = 2.0 * xl - X(n - 2 - jj);
    const double y = quad5_step(c, z, e);
    acc = tiny_min3(acc, e, y);
    s3[s3q_index(w, comp, m2_pairs, pad + n + jj + qs, sq)] = y;
  }
  bad |= !(acc >= kTinyHi) || !__builtin_isfinite(z);
  quad_flag(buf, s, j, bad);
}

// K3q: SPS > 0 as K3 (static symbol offsets inside CH-sample chunks)
template <int SPS>
__global__ __launch_bounds__(64) void k_lowpass_bwd_q(PskBuffers buf, PskParams p, Iir f) {
  if (buf.gate && *buf.gate == 0) return;   // a gated launch (PskBuffers::gate): whole grid
  constexpr int CH = SPS > 0 ? 20 : kLpChunk;
  static_assert(SPS == 0 || CH % SPS == 0, "chunk must be a multiple of SPS");
  const int lane = threadIdx.x;
  const int j = lane & 3, sq = lane >> 2;
  const int64_t w = blockIdx.x >> 1;
  const int comp = blockIdx.x & 1;
  const int64_t s = w * 16 + sq;
  if (w * 16 >= buf.n_streams) return;
  const int64_t n = p.n;
  const int pad = p.pad2;
  const int qs = pad & 1;
  const int64_t m2 = p.m2;
  const int64_t m2_pairs = (m2 + qs + 1) >> 1;
  const double* __restrict__ s3 = buf.s3;
  double* __restrict__ sym = buf.s1;
  const int64_t S = p.n_sym;

  double zi;
  const Quad5 c = quad5_coef(f, j, zi);
  float acc = __builtin_inff();
  const double ylast = s3[s3q_index(w, comp, m2_pairs, m2 - 1 + qs, sq)];
  double z = zi * ylast;
  for (int64_t jj = m2 - 1; jj >= pad + n; --jj) {
    const double y = quad5_step(c, z, s3[s3q_index(w, comp, m2_pairs, jj + qs, sq)]);
    acc = tiny_min3(acc, y, y);
  }

  int64_t k = S - 1;
  int64_t next_n = p.first + k * p.sps;
  const size_t sym_base = sym_index(s, S, 0, comp);
  auto on_output = [&](int64_t i, double y) {
    if (i == next_n) {
      sym[sym_base + (size_t)k * 64] = y;
      --k;
      next_n = k >= 0 ? next_n - p.sps : -1;
    }
  };
  const int64_t nc = n / CH;
  const int64_t n_lo = nc * CH;
  for (int64_t i = n - 1; i >= n_lo; --i) {
    const double y = quad5_step(c, z, s3[s3q_index(w, comp, m2_pairs, pad + i + qs, sq)]);
    acc = tiny_min3(acc, y, y);
    on_output(i, y);
  }
  if (nc > 0) {
    // pointers walk down one chunk per run/load; loads run up to R chunks
    // below the block into the plan's front slack (api.cpp) instead of
    // clamping -- every instruction costs this wave an issue slot
    constexpr int PP = CH / 2;
    const double2* __restrict__ rnext = reinterpret_cast<const double2*>(s3) +
                                        ((size_t)(w * 2 + comp) * m2_pairs + ((pad + qs + (nc - 1) * CH) >> 1)) * 16 + sq;
    double* __restrict__ symp = sym + sym_base + (size_t)((nc - 1) * (SPS > 0 ? CH / SPS : 0)) * 64;
    constexpr int R = kLpBRing;
    double2 rr_[R][PP];
    auto load = [&](double2 (&r)[PP]) {
#pragma unroll
      for (int kk = 0; kk < PP; ++kk) r[kk] = rnext[kk * 16];
      rnext -= PP * 16;
    };
    auto run = [&](const double2 (&r)[PP], int64_t cc) {
      if constexpr (SPS > 0) {
#pragma unroll
        for (int kk = PP - 1; kk >= 0; --kk) {
          const double y1 = quad5_step(c, z, r[kk].y);
          const double y0 = quad5_step(c, z, r[kk].x);
          acc = tiny_min3(acc, y0, y1);
          if ((2 * kk + 1) % SPS == SPS / 2) symp[((2 * kk + 1) / SPS) * 64] = y1;
          if ((2 * kk) % SPS == SPS / 2) symp[((2 * kk) / SPS) * 64] = y0;
        }
        symp -= (CH / SPS) * 64;
      } else {
#pragma unroll
        for (int kk = PP - 1; kk >= 0; --kk) {
          const double y1 = quad5_step(c, z, r[kk].y);
          on_output(cc * CH + 2 * kk + 1, y1);
          const double y0 = quad5_step(c, z, r[kk].x);
          on_output(cc * CH + 2 * kk, y0);
          acc = tiny_min3(acc, y0, y1);
        }
      }
    };
#pragma unroll
    for (int u = 0; u < R; ++u) {
      load(rr_[u]);
      __builtin_amdgcn_sched_barrier(0);
    }
    int64_t cc = nc - 1;
    for (; cc >= R - 1; cc -= R) {
#pragma unroll
      for (int u = 0; u < R; ++u) {
        run(rr_[u], cc - u);
        __builtin_amdgcn_sched_barrier(0);
        load(rr_[u]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int u = 0; u < R; ++u)
      if (cc - u >= 0) run(rr_[u], cc - u);
  }
  for (int jj = pad - 1; jj >= 0; --jj) {
    const double y = quad5_step(c, z, s3[s3q_index(w, comp, m2_pairs, jj + qs, sq)]);
    acc = tiny_min3(acc, y, y);
  }
  quad_flag(buf, s, j, !(acc >= kTinyHi) || !__builtin_isfinite(z));
}

// ---------------------------------------------------------------------------
// K3x: exact complex low-pass (scipy CDOUBLE_filt semantics) for flagged
// streams only.  lane = stream; scratch reuses s3 as [group][j][64] double2;
// writes its symbols into the same sym buffer K3 fills.
template <int NT>
__device__ __forceinline__ void df2t_cplx_step(double (&zr)[NT - 1], double (&zc)[NT - 1],
                                               const double (&b)[NT], const double (&a)[NT],
                                               double x0, double x1, double& y0, double& y1) {
  const double t0x = 0.0 * x1, t1x = 0.0 * x0;
  y0 = zr[0] + (b[0] * x0 - t0x);
  y1 = zc[0] + (t1x + b[0] * x1);
  const double t0y = 0.0 * y1, t1y = 0.0 * y0;
#pragma unroll
  for (int i = 0; i < NT - 2; ++i) {
    const double r = zr[i + 1] + (b[i + 1] * x0 - t0x);
    const double m = zc[i + 1] + (t1x + b[i + 1] * x1);
    zr[i] = r - (a[i + 1] * y0 - t0y);
    zc[i] = m - (t1y + a[i + 1] * y1);
  }
  zr[NT - 2] = (b[NT - 1] * x0 - t0x) - (a[NT - 1] * y0 - t0y);
  zc[NT - 2] = (t1x + b[NT - 1] * x1) - (t1y + a[NT - 1] * y1);
}

__device__ __forceinline__ void cmul_np(double ar, double ai, double br, double bi, double& re, double& im) {
  re = __builtin_fma(ar, br, -(ai * bi));
  im = __builtin_fma(ar, bi, ai * br);
}

// K3x scratch: one slot per workgroup, up to kExactSlots of them, each walking
// the groups g = slot, slot + slots, ...  A slot keeps only the forward
// pass's state (8 doubles per lane) at the start of every kExactTile
// samples; the backward pass re-runs each tile forward from its checkpoint
// into LDS and filters it backward from there (the lane kernels' scheme,
// psk_lane_kernels.hip).  A slot is then m2/32 x 4 KiB (12 MB at n = 96 000)
// instead of the m2 x 1 KiB (98 MB) a stored forward pass takes, so a batch
// whose every stream is flagged (digital silence, gated captures,
// AMR_FORCE_EXACT_LOWPASS) runs one workgroup per group up to 8192 streams.
constexpr int kExactSlots = 128;
constexpr int kExactTile = 32;
int64_t psk_exact_slots(int64_t n_streams) {
  const int64_t g = (n_streams + kWave - 1) / kWave;
  return g < kExactSlots ? g : kExactSlots;
}
int64_t psk_exact_scratch_bytes(int64_t n_streams, int64_t m2) {
  const int64_t tiles = (m2 + kExactTile - 1) / kExactTile;
  return psk_exact_slots(n_streams) * tiles * 8 * kWave * 8;
}

template <int NT>
__global__ __launch_bounds__(64) void k_lowpass_exact(PskBuffers buf, PskParams p, Iir f) {
  if (buf.gate && *buf.gate == 0) return;   // a gated launch (PskBuffers::gate): whole grid
  static_assert(NT == 5, "checkpoint layout holds 2 x 4 states");
  const int lane = threadIdx.x;
  const int64_t n_groups = (buf.n_streams + kWave - 1) / kWave;
  const int64_t n = p.n;
  const int64_t n2 = (n + 1) >> 1;
  const int pad = p.pad2;
  const int64_t m2 = p.m2;
  const int64_t S = p.n_sym;
  const int64_t tiles = (m2 + kExactTile - 1) / kExactTile;
  const double4* __restrict__ lo = reinterpret_cast<const double4*>(buf.lo);   // [n]: (lr, c1, li, c2)
  // checkpoints [slot][tile][8][64] doubles
  double* __restrict__ ck = buf.s3 + (size_t)blockIdx.x * tiles * 8 * kWave + lane;
  double* __restrict__ sym = buf.s1;
  __shared__ double2 tile_out[kExactTile][kWave];
  for (int64_t g = blockIdx.x; g < n_groups; g += gridDim.x) {
    const int64_t s = g * kWave + lane;
    const bool live = s < buf.n_streams && buf.flags[s] != 0;
    if (!__any(live)) continue;                 // wave-uniform skip (the common case)

    double b[NT], a[NT], zr[NT - 1], zc[NT - 1];
#pragma unroll
    for (int i = 0; i < NT; ++i) { b[i] = f.b[i]; a[i] = f.a[i]; }

    auto bb = [&](int64_t i) -> double2 {       // (f + 0j) * lo[i], numpy's complex multiply
      const double fv = buf.s2[f_index(g, n2, i, lane)];
      const double4 l = lo[i];
      return make_double2(__builtin_fma(fv, l.x, l.y), __builtin_fma(fv, l.z, l.w));
    };
    // odd extension with numpy complex ops: (2+0j)*x[0] - x[k]
    const double2 x0 = bb(0), xl = bb(n - 1);
    double l2r, l2i, r2r, r2i;
    cmul_np(2.0, 0.0, x0.x, x0.y, l2r, l2i);
    cmul_np(2.0, 0.0, xl.x, xl.y, r2r, r2i);
    auto ext = [&](int64_t j) -> double2 {
      if (j < pad) { const double2 v = bb(pad - j); return make_double2(l2r - v.x, l2i - v.y); }
      if (j < pad + n) return bb(j - pad);
      const double2 v = bb(n - 2 - (j - pad - n));
      return make_double2(r2r - v.x, r2i - v.y);
    };
    {
      const double2 e0 = ext(0);
#pragma unroll
      for (int i = 0; i < NT - 1; ++i) cmul_np(f.zi[i], 0.0, e0.x, e0.y, zr[i], zc[i]);
    }
    // forward pass: keep the state at the start of every tile
    double y0 = 0, y1 = 0;
    for (int64_t t = 0; t < tiles; ++t) {
      double* c = ck + (size_t)t * 8 * kWave;
#pragma unroll
      for (int i = 0; i < NT - 1; ++i) { c[i * kWave] = zr[i]; c[(NT - 1 + i) * kWave] = zc[i]; }
      const int64_t j1 = (t + 1) * kExactTile < m2 ? (t + 1) * kExactTile : m2;
      for (int64_t j = t * kExactTile; j < j1; ++j) {
        const double2 e = ext(j);
        df2t_cplx_step<NT>(zr, zc, b, a, e.x, e.y, y0, y1);
      }
    }
    double wr[NT - 1], wc[NT - 1];              // backward state: zi * y[-1]
#pragma unroll
    for (int i = 0; i < NT - 1; ++i) cmul_np(f.zi[i], 0.0, y0, y1, wr[i], wc[i]);

    int64_t k = S - 1;
    int64_t next_n = p.first + k * p.sps;
    for (int64_t t = tiles - 1; t >= 0; --t) {
      // re-run tile t forward from its checkpoint (each lane reads back its own
      // stores: program order, no barrier needed), outputs into LDS
      const double* c = ck + (size_t)t * 8 * kWave;
#pragma unroll
      for (int i = 0; i < NT - 1; ++i) { zr[i] = c[i * kWave]; zc[i] = c[(NT - 1 + i) * kWave]; }
      const int64_t j0 = t * kExactTile;
      const int64_t j1 = j0 + kExactTile < m2 ? j0 + kExactTile : m2;
      for (int64_t j = j0; j < j1; ++j) {
        const double2 e = ext(j);
        double o0, o1;
        df2t_cplx_step<NT>(zr, zc, b, a, e.x, e.y, o0, o1);
        tile_out[j - j0][lane] = make_double2(o0, o1);
      }
      for (int64_t j = j1 - 1; j >= j0; --j) {
        const double2 e = tile_out[j - j0][lane];
        double o0, o1;
        df2t_cplx_step<NT>(wr, wc, b, a, e.x, e.y, o0, o1);
        if (j - pad == next_n && k >= 0) {
          if (live) {
            sym[sym_index(s, S, k, 0)] = o0;
            sym[sym_index(s, S, k, 1)] = o1;
          }
          --k;
          next_n -= p.sps;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// K4a: differential product + slicer + bit packing, fully parallel.
// One thread per (stream, 32-bit output word): word j holds the bits of diff
// indices [16j, 16j+16) (QPSK, 2 bits each) or [32j, 32j+32) (BPSK).
//   diff = s[k+1] * conj(s[k])   numpy complex multiply   modem.py:100, 214
//   QPSK sectors                                          modem.py:216-241
//   BPSK real(diff) < 0 -> 1                              modem.py:103-105
// Sector decision: qpsk_dibit (psk_common.h).
// Workgroup = 64 streams x kSliceWords consecutive words: wave w slices words
// w*8 .. w*8+7 of its 64 streams (lane = stream; symbol loads are whole
// 512-B lines, the running symbol carried from word to word), the words go
// through LDS and leave as 128-B row segments -- two streams per store
// instruction instead of 64 scattered 4-B words (which the L2 wrote back as
// partial lines: 84 MB of HBM writes for 9.8 MB of words per 4096 streams).
constexpr int kSliceWords = 32;
// only_flagged: the low-pass already sliced every stream it computed exactly
// (k_lp_lane FUSE); only the streams K3x recomputed get their words here.
template <int WV>
__global__ __launch_bounds__(64 * WV) void k_slice(PskBuffers buf, PskParams p, int only_flagged) {
  if (buf.gate && *buf.gate == 0) return;   // a gated launch (PskBuffers::gate): whole grid
  constexpr int WPW = kSliceWords / WV;         // words per wave
  __shared__ uint32_t wl[kWave][kSliceWords + 1];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int64_t s = (int64_t)blockIdx.y * kWave + lane;
  const bool live = s < buf.n_streams && (!only_flagged || buf.flags[s] != 0);
  const int64_t S = p.n_sym;
  const bool qpsk = p.kind == kQpsk;
  const int per = qpsk ? 16 : 32;
  const int64_t nd = S - 1;                     // number of diffs
  const int64_t jw = (int64_t)blockIdx.x * kSliceWords + wv * WPW;   // this wave's first word
  const double* __restrict__ sym = buf.s1;
  auto SYM = [&](int64_t k) { return make_double2(sym[sym_index(s, S, k, 0)], sym[sym_index(s, S, k, 1)]); };
  double2 prev = make_double2(0.0, 0.0);
  if (live) {
    const int64_t k0 = jw * per;
    prev = SYM(k0 < S ? k0 : S - 1);
  }
  for (int q = 0; q < WPW; ++q) {
    const int64_t j = jw + q;
    uint32_t word = 0;
    if (live && j < p.n_words) {
      const int64_t k0 = j * per;
      for (int u = 0; u < per; ++u) {
        const int64_t k = k0 + u;
        if (k >= nd) break;
        const double2 nx = SYM(k + 1);
        // diff_k = s_{k+1} * conj(s_k): numpy fma form (see oracle)
        const double br = prev.x, bi = -prev.y;
        const double dr = __builtin_fma(nx.x, br, -(nx.y * bi));
        if (qpsk) {
          const double di = __builtin_fma(nx.x, bi, nx.y * br);
          word |= qpsk_dibit(dr, di) << (30 - 2 * u);
        } else {
          word |= (dr < 0 ? 1u : 0u) << (31 - u);
        }
        prev = nx;
      }
    }
    wl[lane][wv * WPW + q] = word;
  }
  __syncthreads();
  const int jj = threadIdx.x & (kSliceWords - 1);
  const int64_t j = (int64_t)blockIdx.x * kSliceWords + jj;
#pragma unroll
  for (int i = 0; i < kWave / (2 * WV); ++i) {
    const int sl = i * 2 * WV + (threadIdx.x >> 5);   // 2 WV streams per pass, 32 words each
    const int64_t ss = (int64_t)blockIdx.y * kWave + sl;
    if (ss < buf.n_streams && j < p.n_words && (!only_flagged || buf.flags[ss] != 0))
      buf.words[(size_t)ss * p.n_words + j] = wl[sl][jj];
  }
}

// ---------------------------------------------------------------------------
// host-side launchers (called from api.cpp)
template <typename T>
static hipError_t launch_bp_row(const PskBuffers& b, const PskParams& p, const Iir& f, hipStream_t st) {
  // K1g once K1r would need more than one wave per SIMD (B > 4 x SIMDs: 4096
  // on an MI355X); K1r below (fewer instructions per wave, solo-faster).
  // AMR_BP_G8=0/1 forces either.
  static const int force = [] { const char* e = getenv("AMR_BP_G8"); return e ? (e[0] == '1' ? 1 : 0) : -1; }();
  static int simds[64] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev >= 0 && dev < 64 && simds[dev] == 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    simds[dev] = 4 * cus;
  }
  const int64_t nsimd = (dev >= 0 && dev < 64) ? simds[dev] : 1024;
  // streams in flight on the device: this batch times the caller's hint
  // (amr_psk_plan_set_inflight) -- K1g once they exceed 4 per SIMD
  const int64_t live = b.n_streams * (b.inflight > 1 ? b.inflight : 1);
  const bool g8 = force >= 0 ? force == 1 : live > (int64_t)kRowStreams * nsimd;
  // One wave per workgroup (the waves share nothing): with batches in
  // flight the dispatcher then places band-pass and low-pass waves SIMD by
  // SIMD instead of a band-pass CU at a time (measured 9.0 -> 8.9 ms, K1r,
  // two batches; 4-wave workgroups stay instantiable for A/B runs).
  if (g8) {
    const int64_t waves = (b.n_streams + kG8Streams - 1) / kG8Streams;
    hipLaunchKernelGGL((k_bandpass_g8<T, 1>), dim3((unsigned)waves), dim3(64), 0, st, b, p, f);
    return hipGetLastError();
  }
  const int64_t waves = (b.n_streams + kRowStreams - 1) / kRowStreams;
  hipLaunchKernelGGL((k_bandpass_row<T, 1>), dim3((unsigned)waves), dim3(64), 0, st, b, p, f);
  return hipGetLastError();
}

hipError_t launch_psk_bandpass(const PskBuffers& b, const PskParams& p, const Iir& f, hipStream_t st) {
  if (f.nt != 9) return hipErrorInvalidValue;   // butter(4, band): the plan checks
  switch (b.dtype) {
    case kF32: return launch_bp_row<float>(b, p, f, st);
    case kF64: return launch_bp_row<double>(b, p, f, st);
    case kI16: return launch_bp_row<int16_t>(b, p, f, st);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_psk_lowpass_fwd(const PskBuffers& b, const PskParams& p, const Iir& f, hipStream_t st) {
  if (f.nt != 5) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(b.flags, 0, (size_t)b.n_streams * 4, st);
  if (e != hipSuccess) return e;
  // a multiple of 16 blocks: the XCD pairing in k_lowpass_fwd_q is a bijection
  const dim3 gq((unsigned)((2 * ((b.n_streams + 15) / 16) + 15) / 16 * 16)), bq(kWave);
  hipLaunchKernelGGL(k_lowpass_fwd_q, gq, bq, 0, st, b, p, f);
  return hipGetLastError();
}

hipError_t launch_psk_lowpass_bwd(const PskBuffers& b, const PskParams& p, const Iir& f, hipStream_t st) {
  if (f.nt != 5) return hipErrorInvalidValue;
  const dim3 gq((unsigned)(2 * ((b.n_streams + 15) / 16))), bq(kWave);
  if (p.sps == 10 && p.first == 5) hipLaunchKernelGGL((k_lowpass_bwd_q<10>), gq, bq, 0, st, b, p, f);
  else if (p.sps == 5 && p.first == 2) hipLaunchKernelGGL((k_lowpass_bwd_q<5>), gq, bq, 0, st, b, p, f);
  else if (p.sps == 20 && p.first == 10) hipLaunchKernelGGL((k_lowpass_bwd_q<20>), gq, bq, 0, st, b, p, f);
  else hipLaunchKernelGGL((k_lowpass_bwd_q<0>), gq, bq, 0, st, b, p, f);
  return hipGetLastError();
}

hipError_t launch_psk_slice(const PskBuffers& b, const PskParams& p, hipStream_t st, bool only_flagged) {
  const int64_t groups = (b.n_streams + kWave - 1) / kWave;
  if (p.n_words < 1 || p.n_bits < 1) return hipSuccess;
  // 4 waves (8 words each) per workgroup: a 256-thread workgroup finds room
  // beside the resident band-pass / low-pass waves (a 1024-thread one waited
  // 10-13 ms per launch at 8192 streams); AMR_SLICE_WAVES=8/16 for A/B runs
  static const int waves = [] { const char* w = getenv("AMR_SLICE_WAVES"); return w ? atoi(w) : 4; }();
  const dim3 grid((unsigned)((p.n_words + kSliceWords - 1) / kSliceWords), (unsigned)groups);
  if (waves == 16)
    hipLaunchKernelGGL(k_slice<16>, grid, dim3(1024), 0, st, b, p, only_flagged ? 1 : 0);
  else if (waves == 8)
    hipLaunchKernelGGL(k_slice<8>, grid, dim3(512), 0, st, b, p, only_flagged ? 1 : 0);
  else
    hipLaunchKernelGGL(k_slice<4>, grid, dim3(256), 0, st, b, p, only_flagged ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_psk_lowpass_exact(const PskBuffers& b, const PskParams& p, const Iir& f, hipStream_t st) {
  if (f.nt != 5) return hipErrorInvalidValue;
  const int64_t slots = psk_exact_slots(b.n_streams);
  hipLaunchKernelGGL((k_lowpass_exact<5>), dim3((unsigned)slots), dim3(kWave), 0, st, b, p, f);
  return hipGetLastError();
}

}  // namespace amr
