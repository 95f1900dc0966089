// api.cpp -- the C ABI of libamr.so (include/amr.h): plans, HBM scratch,
// launches, timing and the RCCL gather.  Host code; compiled by hipcc.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "amr_internal.h"
#include "api_common.h"
#include "iir_design.h"
#include "split_strict.h"

namespace amr {
hipError_t launch_psk_bandpass(const PskBuffers&, const PskParams&, const Iir&, hipStream_t);
hipError_t launch_psk_lowpass_fwd(const PskBuffers&, const PskParams&, const Iir&, hipStream_t);
hipError_t launch_psk_lowpass_bwd(const PskBuffers&, const PskParams&, const Iir&, hipStream_t);
hipError_t launch_psk_lowpass_exact(const PskBuffers&, const PskParams&, const Iir&, hipStream_t);
hipError_t launch_psk_slice(const PskBuffers&, const PskParams&, hipStream_t, bool only_flagged = false);
hipError_t launch_psk_bandpass_lane(const PskBuffers&, const PskParams&, const Iir&, hipStream_t);
hipError_t launch_psk_bandpass_fixup(const PskBuffers&, const PskParams&, const Iir&, hipStream_t);
bool psk_lane_fused(const PskBuffers&, const PskParams&);
hipError_t launch_psk_lowpass_lane(const PskBuffers&, const PskParams&, const Iir&, hipStream_t, bool* sliced);
int64_t psk_lane_bp_scratch_doubles(int64_t n_streams, int64_t n, int pad);
int64_t psk_lane_lp_scratch_doubles(int64_t n_streams, int64_t n, int pad);
int64_t psk_exact_scratch_bytes(int64_t n_streams, int64_t m2);
hipError_t launch_synth_tile_noise(const float*, int64_t, int64_t, float*, int64_t, int64_t, float, uint64_t,
                                   hipStream_t);
hipError_t launch_sync_pack(const uint32_t*, int64_t, int64_t, int64_t, uint8_t*, int64_t, int64_t*, int64_t*,
                            hipStream_t);
hipError_t launch_sync_pack_gated(const uint32_t*, int64_t, int64_t, int64_t, uint8_t*, int64_t, int64_t*, int64_t*,
                                  const int32_t*, hipStream_t);
hipError_t launch_psk_split_bp(const PskBuffers&, const PskParams&, const Iir&, const PskSplit&, hipStream_t);
hipError_t launch_psk_split_lp(const PskBuffers&, const PskParams&, const Iir&, const PskSplit&, hipStream_t);
hipError_t launch_psk_split_slice(const PskBuffers&, const PskParams&, const PskSplit&, hipStream_t);
hipError_t launch_fec_decode(const uint8_t*, int64_t, const int64_t*, int64_t, uint8_t*, int64_t, int64_t*,
                             int32_t*, const uint32_t*, const uint32_t*, hipStream_t);
hipError_t launch_frame_parse(const uint8_t*, int64_t, const int64_t*, int64_t, int64_t, int32_t*, amr_frame_rec*,
                              const uint32_t*, const uint32_t*, hipStream_t);
}  // namespace amr

using namespace amr;

namespace {
thread_local std::string g_err;
}  // namespace

int amr::fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

hipError_t amr::memcpy_rows(void* dst, int64_t dst_pitch, const void* src, int64_t src_pitch, int64_t row_bytes,
                            int64_t B, hipMemcpyKind kind) {
  if (B <= 0 || row_bytes <= 0) return hipSuccess;
  const size_t span_src = (size_t)(src_pitch * (B - 1) + row_bytes);
  const size_t span_dst = (size_t)(dst_pitch * (B - 1) + row_bytes);
  // equal pitches: one copy (a D2H one only when the rows are dense, so the
  // caller's bytes between rows are never overwritten)
  if (dst_pitch == src_pitch && (row_bytes == dst_pitch || kind == hipMemcpyHostToDevice))
    return hipMemcpy(dst, src, span_src, kind);
  if (kind == hipMemcpyHostToDevice && dst_pitch == row_bytes) {   // pack on the host, one copy
    std::vector<uint8_t> h(span_dst);
    for (int64_t r = 0; r < B; ++r)
      std::memcpy(h.data() + r * dst_pitch, static_cast<const uint8_t*>(src) + r * src_pitch, (size_t)row_bytes);
    return hipMemcpy(dst, h.data(), span_dst, kind);
  }
  if (kind == hipMemcpyDeviceToHost) {                              // one copy, scatter on the host
    std::vector<uint8_t> h(span_src);
    hipError_t e = hipMemcpy(h.data(), src, span_src, kind);
    if (e != hipSuccess) return e;
    for (int64_t r = 0; r < B; ++r)
      std::memcpy(static_cast<uint8_t*>(dst) + r * dst_pitch, h.data() + r * src_pitch, (size_t)row_bytes);
    return hipSuccess;
  }
  return hipMemcpy2D(dst, (size_t)dst_pitch, src, (size_t)src_pitch, (size_t)row_bytes, (size_t)B, kind);
}

int amr::copy_batch_h2d(void* dst, const void* src, int64_t row_bytes, int64_t src_pitch, int64_t B,
                        hipStream_t st) {
  HIP_TRY(hipStreamSynchronize(st));
  HIP_TRY(memcpy_rows(dst, row_bytes, src, src_pitch, row_bytes, B, hipMemcpyHostToDevice));
  return AMR_OK;
}

int amr::copy_batch_d2h(void* dst, int64_t dst_pitch, const void* src, int64_t src_pitch, int64_t row_bytes,
                        int64_t B, hipStream_t st) {
  HIP_TRY(hipStreamSynchronize(st));
  HIP_TRY(memcpy_rows(dst, dst_pitch, src, src_pitch, row_bytes, B, hipMemcpyDeviceToHost));
  return AMR_OK;
}

int64_t amr::dtype_size(int dtype) {
  switch (dtype) {
    case AMR_DTYPE_F32: return 4;
    case AMR_DTYPE_F64: return 8;
    case AMR_DTYPE_I16: return 2;
  }
  return 0;
}

namespace {

// CRC32 tables for the FEC kernel (uploaded once per device)
struct CrcTables {
  uint32_t table[256];
  uint32_t x2n[32];
  CrcTables() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
      table[i] = c;
    }
    auto mul = [](uint32_t a, uint32_t b) {
      uint32_t m = 1u << 31, p = 0;
      for (int i = 0; i < 32; ++i) {
        if (a & m) p ^= b;
        m >>= 1;
        b = (b & 1) ? (b >> 1) ^ 0xEDB88320u : b >> 1;
      }
      return p;
    };
    uint32_t p = 1u << 30;  // x^1
    x2n[0] = p;
    for (int n = 1; n < 32; ++n) x2n[n] = p = mul(p, p);
  }
};

struct DeviceCrc {
  uint32_t* d = nullptr;  // [256 table][32 x2n]
};
std::mutex g_crc_mu;
DeviceCrc g_crc[64];

int device_crc(int dev, const uint32_t** table, const uint32_t** x2n) {
  std::lock_guard<std::mutex> lk(g_crc_mu);
  if (dev < 0 || dev >= 64) return fail(AMR_E_INVALID, "device ordinal out of range");
  if (!g_crc[dev].d) {
    static const CrcTables t;
    uint32_t* p = nullptr;
    HIP_TRY(hipMalloc(&p, sizeof(uint32_t) * 288));
    HIP_TRY(hipMemcpy(p, t.table, sizeof(t.table), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(p + 256, t.x2n, sizeof(t.x2n), hipMemcpyHostToDevice));
    g_crc[dev].d = p;
  }
  *table = g_crc[dev].d;
  *x2n = g_crc[dev].d + 256;
  return AMR_OK;
}

bool is_pos_zero(double v) { return v == 0.0 && !std::signbit(v); }
static bool same_bits(double a, double b) {
  uint64_t u, v;
  std::memcpy(&u, &a, 8);
  std::memcpy(&v, &b, 8);
  return u == v;
}

// Per-device staging of the synchronous host entries that take no plan
// (amr_fec_decode_host, amr_frame_parse_host): grow-only buffers kept for the
// process instead of hipMalloc/hipFree on every call; one call per device at a
// time (the lock is held for the whole call).
struct HostStaging {
  std::mutex mu;
  void* buf[6] = {};
  int64_t bytes[6] = {};
};
HostStaging g_staging[64];

hipError_t staging_get(HostStaging& hs, int slot, int64_t need, void** out) {
  if (hs.bytes[slot] < need || !hs.buf[slot]) {
    if (hs.buf[slot]) {
      hipError_t e = hipFree(hs.buf[slot]);
      if (e != hipSuccess) return e;
    }
    hs.buf[slot] = nullptr;
    hs.bytes[slot] = 0;
    const int64_t grow = std::max<int64_t>(need, hs.bytes[slot] * 2);
    hipError_t e = hipMalloc(&hs.buf[slot], (size_t)std::max<int64_t>(grow, 256));
    if (e != hipSuccess) return e;
    hs.bytes[slot] = std::max<int64_t>(grow, 256);
  }
  *out = hs.buf[slot];
  return hipSuccess;
}

}  // namespace

// doubles of slack below s1/s3: the backward passes prefetch up to a few
// chunks past the start of their block instead of clamping the index
constexpr int64_t kFrontSlack = 8192;
// streams in flight (batch x amr_psk_plan_set_inflight) from which the
// lane-per-stream layout runs
constexpr int64_t kLaneMinLiveStreams = 16384;
// time-split layout: picked for at most this many streams in
// flight (a flagged stream re-runs its batch serially, so the batch stays
// small enough that most batches have none); its error bound is kSplitSafety
// times the filters' L1 noise gain (split_design); chunks are at least
// kSplitMinL outputs, and longer once a batch would exceed kSplitLanes lanes
constexpr int64_t kSplitMaxLiveStreams = 64;
constexpr double kSplitSafety = 64.0;
constexpr int64_t kSplitMinL = 64;
constexpr int64_t kSplitLanes = 65536;
// with KS0's convolution start states: chunks of kSplitConvMinL..MaxL outputs,
// about kSplitConvChunks per call (the wall-time optimum at 1-64 captures of
// 96000 samples, tools/split_batch_probe.py)
constexpr int64_t kSplitConvMinL = 128;
constexpr int64_t kSplitConvMaxL = 1024;
constexpr int64_t kSplitConvChunks = 3072;

struct amr_psk_plan {
  std::mutex mu;
  int device = 0;
  hipStream_t stream = nullptr;
  PskParams p{};
  Iir bp{}, lp{};
  bool lp_exact_only = false;   // low-pass coefficients outside the separable proof
  int64_t max_streams = 0, groups = 0;
  int64_t m1_pairs = 0, m2_pairs = 0;
  int64_t out_cap = 0;
  // HBM scratch
  double* lo = nullptr;
  double* lo2 = nullptr;
  double* s1 = nullptr;   // = s1_base + kFrontSlack (backward prefetch may read below)
  double* s2 = nullptr;
  double* s3 = nullptr;   // = s3_base + kFrontSlack
  double* s1_base = nullptr;
  double* s3_base = nullptr;
  int64_t s1_bytes = 0, s3_bytes = 0;   // allocated (the row layout grows them on first use)
  uint32_t* words = nullptr;
  int32_t* flags = nullptr;
  int64_t scratch_bytes = 0;
  // staging for the host API (lazily sized)
  void* d_x = nullptr;
  int64_t d_x_bytes = 0;
  uint8_t* d_out = nullptr;
  int64_t* d_len = nullptr;
  int64_t* d_sync = nullptr;
  double* d_edge = nullptr;   // amr_psk_demod_host_edges' table [max_streams][2 pad1]
  int64_t d_edge_bytes = 0;
  uint8_t* d_fec = nullptr;   // FEC host API staging
  int64_t* d_fec_len = nullptr;
  int32_t* d_crc = nullptr;
  // timing
  bool timing = false;
  int inflight = 1;             // amr_psk_plan_set_inflight hint
  int last_layout = 0;          // AMR_LAYOUT_* of the last call
  hipEvent_t ev[AMR_T_COUNT + 1][2]{};
  bool ev_used[AMR_T_COUNT]{};
  int64_t last_exact = 0;
  GatherGate gate;              // an all-gather still reading this plan's outputs
  // time-split layout (psk_split_kernels.hip): designed on first use
  int forced_layout = -1;       // amr_psk_plan_set_layout (-1: by streams in flight)
  bool split_designed = false, split_ok = false;
  int64_t split_w1 = 0, split_w2 = 0, split_L = 0;
  double split_kappa = 0.0;
  unsigned long long* split_peak = nullptr;   // [max_streams], then flags [max_streams] and the count
  int32_t* split_flag = nullptr;
  int32_t* split_count = nullptr;
  double* split_tab = nullptr;    // [w1][8] K, then [w1 + 1][8] Z0 (split_state_tables), with the design
  double* split_zs = nullptr;     // [B][c1][8] chunk start states (grown per launch)
  int64_t split_zs_bytes = 0;
  // the split layout's STRICT bound (split_strict.h): -1 = the process default
  // (AMR_PSK_SPLIT_STRICT=1), else amr_psk_plan_set_split_strict; designed on
  // the first strict call (the device tables kabs | z0abs | lpc in strict_tab,
  // the per-stream maxima in strict_bnd)
  int strict_mode = -1;
  bool strict_designed = false;
  StrictDesign sdes;
  double* strict_tab = nullptr;
  unsigned long long* strict_bnd = nullptr;
  double* strict_sc = nullptr;    // the per-stream scratch of the block bound (PskSplit::sc), grown per call
  int64_t strict_sc_bytes = 0;
  bool last_f32f = false;       // the last lane-layout call handed f over in float32
  bool last_strict = false;     // the last split call decided with the strict bound
};

struct amr_comm {
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;
  int device = 0;
  int nranks = 1, rank = 0;
  std::mutex mu;                // every RCCL call on comm (amr_allgather*, the host collectives) and the staging buffer
  void* stage = nullptr;        // device staging of amr_comm_allgather_host / allreduce_max
  int64_t stage_bytes = 0;
};

namespace {
// bytes of s1 / s3 each layout needs (psk_kernels.hip / psk_lane_kernels.hip)
int64_t lane_s1_bytes(const amr_psk_plan* pl) {
  const int64_t g = pl->groups;
  return std::max(2 * g * std::max<int64_t>(pl->p.n_sym, 1) * kWave * 8,
                  psk_lane_bp_scratch_doubles(pl->max_streams, pl->p.n, pl->p.pad1) * 8);
}
int64_t lane_s3_bytes(const amr_psk_plan* pl) {
  return std::max(psk_lane_lp_scratch_doubles(pl->max_streams, pl->p.n, pl->p.pad2) * 8,
                  psk_exact_scratch_bytes(pl->max_streams, pl->p.m2));
}
int64_t row_s1_bytes(const amr_psk_plan* pl) {
  return std::max(pl->groups * pl->m1_pairs * kWave * 16, lane_s1_bytes(pl));
}
int64_t row_s3_bytes(const amr_psk_plan* pl) {
  return std::max(2 * pl->groups * pl->m2_pairs * kWave * 16, lane_s3_bytes(pl));
}
// The plan's geometry from its shape alone (no device work): PskParams'
// sizes, groups, DF-II-T pair counts and the output capacity.  Shared by
// amr_psk_plan_create and amr_psk_plan_bytes_estimate.
void psk_geometry(amr_psk_plan* pl, int kind, int64_t n, int64_t sps, int64_t first, int bp_nt, int lp_nt,
                  int64_t max_streams) {
  PskParams& p = pl->p;
  p.n = n;
  p.pad1 = 3 * bp_nt;
  p.pad2 = 3 * lp_nt;
  p.m1 = n + 2 * p.pad1;
  p.m2 = n + 2 * p.pad2;
  p.sps = sps;
  p.first = first;
  p.kind = kind;
  p.n_sym = n > first ? (n - first + sps - 1) / sps : 0;
  const int bps = kind == AMR_PSK_QPSK ? 2 : 1;
  p.n_bits = p.n_sym >= 2 ? (p.n_sym - 1) * bps : 0;
  p.n_words = p.n_bits > 0 ? (p.n_bits + 31) / 32 : 1;
  pl->max_streams = max_streams;
  pl->groups = (max_streams + kWave - 1) / kWave;
  const int qs1 = p.pad1 & 1, qs2 = p.pad2 & 1;
  pl->m1_pairs = (p.m1 + qs1 + 1) >> 1;
  pl->m2_pairs = (p.m2 + qs2 + 1) >> 1;
  pl->out_cap = p.n_bits / 8 + 1;
}

// the device buffers amr_psk_plan_create allocates, in order (lane-layout sizes of s1 / s3)
struct PskAlloc { int which; int64_t bytes; };
std::vector<PskAlloc> psk_allocs(const amr_psk_plan* pl) {
  const int64_t n = pl->p.n, g = pl->groups;
  return {{0, n * 4 * (int64_t)sizeof(double)},
          // + slack: K2q's prefetch runs up to a few chunks past the end (psk_kernels.hip)
          {1, (n * 2 + 1024) * (int64_t)sizeof(double)},
          // s1 doubles as the symbol buffer [2G][S][64] after the band-pass (psk_common.h sym_index)
          {2, kFrontSlack * 8 + lane_s1_bytes(pl)},
          {3, g * 2 * ((n + 1) / 2) * 32 * 16 + (1 << 16)},
          {4, kFrontSlack * 8 + lane_s3_bytes(pl)},
          {5, g * kWave * pl->p.n_words * 4},
          {6, 2 * g * kWave * 4},      // low-pass flags, then band-pass flags
          {7, pl->max_streams * 12 + 64}};   // time-split: input peaks, flags, the flagged count
}

// the most the plan can hold: `allocated` with s1 / s3 grown to the row
// layout's size (on its first call) + the host-API staging (allocated on
// the first amr_psk_demod_host)
int64_t psk_max_bytes(const amr_psk_plan* pl, int64_t allocated) {
  const int64_t have1 = pl->s1_bytes ? pl->s1_bytes : kFrontSlack * 8 + lane_s1_bytes(pl);
  const int64_t have3 = pl->s3_bytes ? pl->s3_bytes : kFrontSlack * 8 + lane_s3_bytes(pl);
  const int64_t grow = std::max<int64_t>(0, kFrontSlack * 8 + row_s1_bytes(pl) - have1) +
                       std::max<int64_t>(0, kFrontSlack * 8 + row_s3_bytes(pl) - have3);
  // + the host entries' staging: x (8 B per sample), outputs, the edge table
  return allocated + grow + pl->max_streams * pl->p.n * 8 + pl->max_streams * (pl->out_cap + 16) +
         pl->max_streams * 2 * pl->p.pad1 * 8;
}

// Grow one scratch buffer to `want` bytes.  The new block is allocated before
// the old one is released, so a failed grow leaves the plan exactly as it was
// (its pointers still valid for the layout that fits); only when that fails
// is the old block freed first (tight memory), and if even then the new size
// does not fit the old size is restored, or the buffer is left empty (NULL,
// 0 bytes) -- run_psk re-checks the sizes before every launch and refuses a
// plan whose buffers are too small instead of handing the kernels freed memory.
int grow_scratch(amr_psk_plan* pl, double** base, int64_t* have, int64_t want) {
  if (*have >= want && *base) return AMR_OK;
  static const bool fail_grow = [] {             // test hook: make every grow fail
    const char* e = std::getenv("AMR_TEST_FAIL_SCRATCH_GROW");
    return e && e[0] == '1';
  }();
  HIP_TRY(hipStreamSynchronize(pl->stream));     // queued work may still use the old block
  double* nb = nullptr;
  hipError_t e = fail_grow ? hipErrorOutOfMemory : hipMalloc(&nb, (size_t)want);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    const int64_t old = *have;
    HIP_TRY(hipFree(*base));
    *base = nullptr;
    *have = 0;
    pl->scratch_bytes -= old;
    e = fail_grow ? hipErrorOutOfMemory : hipMalloc(&nb, (size_t)want);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      if (old > 0 && hipMalloc(base, (size_t)old) == hipSuccess) {
        *have = old;
        pl->scratch_bytes += old;
      } else {
        (void)hipGetLastError();
        *base = nullptr;
      }
      return fail(AMR_E_NOMEM, "hipMalloc(" + std::to_string(want) + " B) for plan scratch: " + hipGetErrorString(e));
    }
  } else {
    HIP_TRY(hipFree(*base));
    pl->scratch_bytes -= *have;
  }
  *base = nb;
  pl->scratch_bytes += want;
  *have = want;
  return AMR_OK;
}

// s1 / s3 at least b1 / b3 bytes (incl. the front slack); the kernel pointers
// follow the (possibly new) blocks
int ensure_scratch(amr_psk_plan* pl, int64_t b1, int64_t b3) {
  int rc = grow_scratch(pl, &pl->s1_base, &pl->s1_bytes, b1);
  if (rc == AMR_OK) rc = grow_scratch(pl, &pl->s3_base, &pl->s3_bytes, b3);
  pl->s1 = pl->s1_base ? pl->s1_base + kFrontSlack : nullptr;
  pl->s3 = pl->s3_base ? pl->s3_base + kFrontSlack : nullptr;
  return rc;
}
}  // namespace

namespace amr {
int plan_stream(amr_psk_plan* plan, int* dev, hipStream_t* st) {
  *st = nullptr;
  if (plan) {
    *dev = plan->device;
    *st = plan->stream;
    HIP_TRY(hipSetDevice(*dev));
  } else {
    HIP_TRY(hipGetDevice(dev));
  }
  return AMR_OK;
}
}  // namespace amr

namespace {
void split_design(amr_psk_plan* pl);   // below, with run_psk
bool split_conv_on(const amr_psk_plan* pl);
bool split_strict_on(const amr_psk_plan* pl);
int strict_prepare(amr_psk_plan* pl);
bool split_design_core(const Iir& bp, const Iir& lp, int64_t n, int64_t n_sym, int64_t* w1, int64_t* w2,
                       double* kappa);
double f32_design(const Iir& lp);
int run_psk_split_front(amr_psk_plan* pl, const void* d_x, int dtype, int64_t B, int64_t x_stride, int64_t L,
                        double* ebound = nullptr);
int ensure(void** p, int64_t* have, int64_t need);
int psk_demod_host(amr_psk_plan* plan, const void* x, int dtype, int64_t B, int64_t x_stride, const double* edges,
                   uint8_t* out, int64_t out_stride, int64_t* out_len, int64_t* sync_idx);
}  // namespace

extern "C" {

int amr_abi_version(void) { return AMR_ABI_VERSION; }
#ifndef AMR_BUILD_ID
#define AMR_BUILD_ID "unknown"
#endif
const char* amr_build_id(void) { return AMR_BUILD_ID; }
const char* amr_last_error(void) { return g_err.c_str(); }

int amr_device_count(int* count) {
  if (!count) return fail(AMR_E_INVALID, "count is NULL");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *count = 0;
    return fail(AMR_E_NODEVICE, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
  }
  *count = n;
  return AMR_OK;
}

int amr_set_device(int device) {
  HIP_TRY(hipSetDevice(device));
  return AMR_OK;
}
int amr_malloc(void** dptr, int64_t bytes) {
  if (!dptr || bytes < 0) return fail(AMR_E_INVALID, "amr_malloc: bad argument");
  HIP_TRY(hipMalloc(dptr, (size_t)(bytes > 0 ? bytes : 1)));
  return AMR_OK;
}
int amr_free(void* dptr) {
  HIP_TRY(hipFree(dptr));
  return AMR_OK;
}
int amr_memcpy_h2d(void* dst, const void* src, int64_t bytes) {
  HIP_TRY(hipMemcpy(dst, src, (size_t)bytes, hipMemcpyHostToDevice));
  return AMR_OK;
}
int amr_memcpy_d2h(void* dst, const void* src, int64_t bytes) {
  HIP_TRY(hipMemcpy(dst, src, (size_t)bytes, hipMemcpyDeviceToHost));
  return AMR_OK;
}
int amr_memcpy_d2d(void* dst, const void* src, int64_t bytes) {
  HIP_TRY(hipMemcpy(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice));
  return AMR_OK;
}
int amr_device_synchronize(void) {
  HIP_TRY(hipDeviceSynchronize());
  return AMR_OK;
}

static void plan_free(amr_psk_plan* pl) {
  if (!pl) return;
  (void)hipSetDevice(pl->device);
  if (pl->stream) (void)hipStreamSynchronize(pl->stream);
  gate_free(pl->gate);
  for (auto* p : {(void*)pl->lo, (void*)pl->lo2, (void*)pl->s1_base, (void*)pl->s2, (void*)pl->s3_base, (void*)pl->words, (void*)pl->flags,
                  (void*)pl->split_peak, (void*)pl->split_tab, (void*)pl->split_zs, (void*)pl->strict_tab,
                  (void*)pl->strict_bnd, (void*)pl->strict_sc,
                  pl->d_x, (void*)pl->d_out, (void*)pl->d_len, (void*)pl->d_sync, (void*)pl->d_edge, (void*)pl->d_fec,
                  (void*)pl->d_fec_len, (void*)pl->d_crc})
    if (p) (void)hipFree(p);
  for (auto& e : pl->ev)
    for (auto& h : e)
      if (h) (void)hipEventDestroy(h);
  if (pl->stream) (void)hipStreamDestroy(pl->stream);
  delete pl;
}

int amr_psk_plan_create(amr_psk_plan** out, int device, int kind, int64_t n, int64_t sps, int64_t first,
                        const double* bp_b, const double* bp_a, const double* bp_zi, int bp_nt,
                        const double* lp_b, const double* lp_a, const double* lp_zi, int lp_nt,
                        const double* lo4, int64_t max_streams) {
  if (!out || !bp_b || !bp_a || !bp_zi || !lp_b || !lp_a || !lp_zi || !lo4)
    return fail(AMR_E_INVALID, "amr_psk_plan_create: NULL argument");
  *out = nullptr;
  if (kind != AMR_PSK_QPSK && kind != AMR_PSK_BPSK) return fail(AMR_E_INVALID, "unknown PSK kind");
  if (sps < 1 || first < 0 || max_streams < 1) return fail(AMR_E_INVALID, "bad sps/first/max_streams");
  if (bp_nt != 9 && bp_nt != 7) return fail(AMR_E_INVALID, "band-pass must have 7 or 9 taps");
  if (lp_nt != 5) return fail(AMR_E_INVALID, "low-pass must have 5 taps");
  if (bp_a[0] != 1.0 || lp_a[0] != 1.0) return fail(AMR_E_INVALID, "a[0] must be 1 (scipy butter form)");
  if (n <= 3 * bp_nt || n <= 3 * lp_nt)
    return fail(AMR_E_PADLEN, "The length of the input vector x must be greater than padlen, which is " +
                                  std::to_string(3 * (n <= 3 * bp_nt ? bp_nt : lp_nt)) + ".");
  auto* pl = new amr_psk_plan();
  pl->device = device;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    delete pl;
    return fail(AMR_E_NODEVICE, std::string("hipSetDevice: ") + hipGetErrorString(e));
  }
  psk_geometry(pl, kind, n, sps, first, bp_nt, lp_nt, max_streams);
  PskParams& p = pl->p;
  bool zodd = true;
  for (int i = 1; i < bp_nt; i += 2) zodd = zodd && is_pos_zero(bp_b[i]);
  p.bp_zero_odd = zodd ? 1 : 0;
  // butter()'s numerators are k * poly(zeros at +-1): palindromic, and the
  // kernels then form each distinct product x * b[i] once (psk_lane_kernels.hip)
  p.bp_sym = bp_nt == 9 && same_bits(bp_b[8], bp_b[0]) && same_bits(bp_b[6], bp_b[2]) ? 1 : 0;
  p.lp_sym = lp_nt == 5 && same_bits(lp_b[4], lp_b[0]) && same_bits(lp_b[3], lp_b[1]) ? 1 : 0;
  pl->bp.nt = bp_nt;
  pl->lp.nt = lp_nt;
  for (int i = 0; i < bp_nt; ++i) { pl->bp.b[i] = bp_b[i]; pl->bp.a[i] = bp_a[i]; }
  for (int i = 0; i < bp_nt - 1; ++i) pl->bp.zi[i] = bp_zi[i];
  for (int i = 0; i < lp_nt; ++i) { pl->lp.b[i] = lp_b[i]; pl->lp.a[i] = lp_a[i]; }
  for (int i = 0; i < lp_nt - 1; ++i) pl->lp.zi[i] = lp_zi[i];
  // separable low-pass proof needs b > 0 normal and zi, a normal non-zero
  for (int i = 0; i < lp_nt; ++i) {
    if (!(lp_b[i] > 0.0 && std::isnormal(lp_b[i]) && lp_b[i] >= 0x1p-50)) pl->lp_exact_only = true;
    if (i > 0 && !std::isnormal(lp_a[i])) pl->lp_exact_only = true;
  }
  for (int i = 0; i < lp_nt - 1; ++i)
    if (!std::isnormal(lp_zi[i])) pl->lp_exact_only = true;
  // test hook: route every stream through the exact complex low-pass kernel
  if (const char* f = std::getenv("AMR_FORCE_EXACT_LOWPASS"))
    if (f[0] == '1') pl->lp_exact_only = true;
  p.f32_margin = bp_nt == 9 && p.lp_sym ? f32_design(pl->lp) : 0.0;

  void** ptrs[] = {(void**)&pl->lo, (void**)&pl->lo2, (void**)&pl->s1_base, (void**)&pl->s2, (void**)&pl->s3_base,
                   (void**)&pl->words, (void**)&pl->flags, (void**)&pl->split_peak};
  struct A { void** ptr; int64_t bytes; };
  std::vector<A> allocs;
  for (const PskAlloc& a : psk_allocs(pl)) allocs.push_back({ptrs[a.which], a.bytes});
  for (const A& a : allocs) {
    e = hipMalloc(a.ptr, (size_t)a.bytes);
    if (e != hipSuccess) {
      plan_free(pl);
      return fail(AMR_E_NOMEM, "hipMalloc(" + std::to_string(a.bytes) + " B): " + hipGetErrorString(e));
    }
    pl->scratch_bytes += a.bytes;
  }
  pl->s1 = pl->s1_base + kFrontSlack;
  pl->s3 = pl->s3_base + kFrontSlack;
  pl->split_flag = reinterpret_cast<int32_t*>(pl->split_peak + max_streams);
  pl->split_count = pl->split_flag + max_streams;
  pl->s1_bytes = kFrontSlack * 8 + lane_s1_bytes(pl);
  pl->s3_bytes = kFrontSlack * 8 + lane_s3_bytes(pl);
  {
    // device LO layout [n][4] = (lo_re, -(0*lo_im), lo_im, 0*lo_re): per sample and
    // component the (multiplier, addend) pair of numpy's complex multiply
    std::vector<double> lo_dev((size_t)n * 4);
    for (int64_t i = 0; i < n; ++i) {
      lo_dev[4 * i + 0] = lo4[4 * i + 0];
      lo_dev[4 * i + 1] = lo4[4 * i + 2];
      lo_dev[4 * i + 2] = lo4[4 * i + 1];
      lo_dev[4 * i + 3] = lo4[4 * i + 3];
    }
    e = hipMemcpy(pl->lo, lo_dev.data(), (size_t)(n * 4 * sizeof(double)), hipMemcpyHostToDevice);
    // [2][n]: the multipliers alone (K2q's main-body mixer, psk_kernels.hip)
    for (int64_t i = 0; i < n; ++i) {
      lo_dev[(size_t)i] = lo4[4 * i + 0];
      lo_dev[(size_t)(n + i)] = lo4[4 * i + 1];
    }
    if (e == hipSuccess) e = hipMemcpy(pl->lo2, lo_dev.data(), (size_t)(n * 2 * sizeof(double)), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&pl->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    plan_free(pl);
    return fail(AMR_E_HIP, std::string("plan setup: ") + hipGetErrorString(e));
  }
  *out = pl;
  return AMR_OK;
}

int amr_psk_plan_destroy(amr_psk_plan* plan) {
  plan_free(plan);
  return AMR_OK;
}
int64_t amr_psk_plan_out_capacity(const amr_psk_plan* plan) { return plan ? plan->out_cap : -1; }
int64_t amr_psk_plan_scratch_bytes(const amr_psk_plan* plan) {
  if (!plan) return -1;
  return psk_max_bytes(plan, plan->scratch_bytes);
}

int64_t amr_psk_plan_bytes_estimate(int kind, int64_t n, int64_t sps, int64_t first, int bp_nt, int lp_nt,
                                    int64_t max_streams) {
  if ((kind != AMR_PSK_QPSK && kind != AMR_PSK_BPSK) || n < 1 || sps < 1 || first < 0 || max_streams < 1 ||
      bp_nt < 1 || lp_nt < 1)
    return fail(AMR_E_INVALID, "amr_psk_plan_bytes_estimate: bad argument");
  amr_psk_plan pl;
  psk_geometry(&pl, kind, n, sps, first, bp_nt, lp_nt, max_streams);
  int64_t total = 0;
  for (const PskAlloc& a : psk_allocs(&pl)) total += a.bytes;
  return psk_max_bytes(&pl, total);
}

int amr_psk_plan_synchronize(amr_psk_plan* plan) {
  if (!plan) return fail(AMR_E_INVALID, "plan is NULL");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  HIP_TRY(hipStreamSynchronize(plan->stream));
  HIP_TRY(gate_sync(plan->gate));
  return AMR_OK;
}

int amr_psk_plan_enable_timing(amr_psk_plan* plan, int on) {
  if (!plan) return fail(AMR_E_INVALID, "plan is NULL");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  if (on && !plan->ev[0][0]) {
    for (auto& e : plan->ev)
      for (auto& h : e) HIP_TRY(hipEventCreate(&h));
  }
  plan->timing = on != 0;
  return AMR_OK;
}

int amr_psk_plan_set_inflight(amr_psk_plan* plan, int batches) {
  if (!plan) return fail(AMR_E_INVALID, "plan is NULL");
  if (batches < 1) return fail(AMR_E_INVALID, "batches in flight must be >= 1");
  std::lock_guard<std::mutex> lk(plan->mu);
  plan->inflight = batches;
  return AMR_OK;
}

int amr_psk_plan_timings(amr_psk_plan* plan, float* ms, int count) {
  if (!plan || !ms) return fail(AMR_E_INVALID, "NULL argument");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  HIP_TRY(hipStreamSynchronize(plan->stream));
  for (int i = 0; i < count && i < AMR_T_COUNT; ++i) {
    ms[i] = -1.0f;
    if (!plan->timing || !plan->ev_used[i]) continue;
    HIP_TRY(hipEventSynchronize(plan->ev[i][1]));   // the launch slot may end on a comm stream (a gather)
    HIP_TRY(hipEventElapsedTime(&ms[i], plan->ev[i][0], plan->ev[i][1]));
  }
  return AMR_OK;
}

int amr_psk_plan_last_layout(const amr_psk_plan* plan) { return plan ? plan->last_layout : -1; }

int amr_psk_plan_set_layout(amr_psk_plan* plan, int layout) {
  if (!plan) return fail(AMR_E_INVALID, "plan is NULL");
  if (layout != -1 && layout != AMR_LAYOUT_ROW && layout != AMR_LAYOUT_LANE && layout != AMR_LAYOUT_SPLIT)
    return fail(AMR_E_INVALID, "unknown layout");
  std::lock_guard<std::mutex> lk(plan->mu);
  plan->forced_layout = layout;
  return AMR_OK;
}

int amr_psk_split_design(const double* bp_b, const double* bp_a, int bp_nt, const double* lp_b, const double* lp_a,
                         int lp_nt, int64_t n, int64_t n_sym, int64_t* warmup_bp, int64_t* warmup_lp, double* kappa) {
  if (!bp_b || !bp_a || !lp_b || !lp_a || !warmup_bp || !warmup_lp || !kappa || bp_nt < 2 || bp_nt > kMaxTaps ||
      lp_nt < 2 || lp_nt > kMaxTaps || n < 1 || n_sym < 0)
    return fail(AMR_E_INVALID, "amr_psk_split_design: bad argument");
  Iir bp{}, lp{};
  bp.nt = bp_nt;
  lp.nt = lp_nt;
  for (int i = 0; i < bp_nt; ++i) { bp.b[i] = bp_b[i]; bp.a[i] = bp_a[i]; }
  for (int i = 0; i < lp_nt; ++i) { lp.b[i] = lp_b[i]; lp.a[i] = lp_a[i]; }
  *warmup_bp = *warmup_lp = -1;
  *kappa = -1.0;
  if (!split_design_core(bp, lp, n, n_sym, warmup_bp, warmup_lp, kappa)) {
    *warmup_bp = *warmup_lp = -1;
    *kappa = -1.0;
    return fail(AMR_E_INVALID, "these filters do not allow the time-split layout");
  }
  return AMR_OK;
}

double amr_psk_f32_margin(const double* lp_b, const double* lp_a, int lp_nt) {
  if (!lp_b || !lp_a || lp_nt != 5) return 0.0;
  Iir lp{};
  lp.nt = lp_nt;
  for (int i = 0; i < lp_nt; ++i) { lp.b[i] = lp_b[i]; lp.a[i] = lp_a[i]; }
  return f32_design(lp);
}

int amr_psk_split_symbols_host(amr_psk_plan* plan, const void* x, int dtype, int64_t B, int64_t x_stride,
                               int64_t chunk, double* sym) {
  if (!plan || !x || !sym || B < 1) return fail(AMR_E_INVALID, "amr_psk_split_symbols_host: bad argument");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  if (B > plan->max_streams) return fail(AMR_E_CAPACITY, "batch exceeds plan max_streams");
  if (dtype_size(dtype) == 0 || x_stride < plan->p.n) return fail(AMR_E_INVALID, "bad dtype / x_stride");
  if (!plan->split_designed) split_design(plan);
  if (!plan->split_ok || plan->p.n_sym < 2) return fail(AMR_E_INVALID, "no time-split layout for this plan");
  // KS0's start states are B x ceil(m1 / L) x 64 B (and as many waves): a
  // chunk below the layout's own minimum is refused rather than allocated
  if (chunk < 0 || (chunk > 0 && chunk < kSplitConvMinL && split_conv_on(plan)))
    return fail(AMR_E_INVALID, "amr_psk_split_symbols_host: chunk must be 0 (the plan's) or >= 128 with the convolution starts");
  const int64_t n = plan->p.n, es = dtype_size(dtype);
  int64_t have = plan->d_x_bytes;
  HIP_TRY(hipStreamSynchronize(plan->stream));
  if (int rc = ensure(&plan->d_x, &have, B * n * es)) return rc;
  plan->d_x_bytes = have;
  if (int rc = copy_batch_h2d(plan->d_x, x, n * es, x_stride * es, B, plan->stream)) return rc;
  if (int rc = run_psk_split_front(plan, plan->d_x, dtype, B, n, chunk)) return rc;
  HIP_TRY(hipStreamSynchronize(plan->stream));
  HIP_TRY(hipMemcpy(sym, plan->s1, (size_t)(B * plan->p.n_sym * 2 * 8), hipMemcpyDeviceToHost));
  return AMR_OK;
}

int amr_psk_split_bounds_host(amr_psk_plan* plan, const void* x, int dtype, int64_t B, int64_t x_stride,
                              double* sym, double* ebound, double* scalars) {
  if (!plan || !x || !sym || !ebound || !scalars || B < 1)
    return fail(AMR_E_INVALID, "amr_psk_split_bounds_host: bad argument");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  if (B > plan->max_streams) return fail(AMR_E_CAPACITY, "batch exceeds plan max_streams");
  if (dtype_size(dtype) == 0 || x_stride < plan->p.n) return fail(AMR_E_INVALID, "bad dtype / x_stride");
  if (!plan->split_designed) split_design(plan);
  if (!plan->split_ok || plan->p.n_sym < 2) return fail(AMR_E_INVALID, "no time-split layout for this plan");
  const int64_t n = plan->p.n, es = dtype_size(dtype), S = plan->p.n_sym;
  int64_t have = plan->d_x_bytes;
  HIP_TRY(hipStreamSynchronize(plan->stream));
  if (int rc = ensure(&plan->d_x, &have, B * n * es)) return rc;
  plan->d_x_bytes = have;
  double* stage = nullptr;
  HIP_TRY(hipMalloc((void**)&stage, (size_t)(B * (S + 4) * 8)));
  int rc = copy_batch_h2d(plan->d_x, x, n * es, x_stride * es, B, plan->stream);
  if (!rc) rc = run_psk_split_front(plan, plan->d_x, dtype, B, n, 0, stage);
  if (!rc) {
    std::vector<double> h((size_t)(B * (S + 4)));
    if (hipStreamSynchronize(plan->stream) != hipSuccess ||
        hipMemcpy(sym, plan->s1, (size_t)(B * S * 2 * 8), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(h.data(), stage, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) {
      rc = fail(AMR_E_HIP, "amr_psk_split_bounds_host: copy failed");
    } else {
      for (int64_t i = 0; i < B; ++i) {
        std::memcpy(ebound + i * S, h.data() + i * (S + 4), (size_t)S * 8);
        std::memcpy(scalars + i * 4, h.data() + i * (S + 4) + S, 32);
      }
    }
  }
  (void)hipFree(stage);
  return rc;
}

int amr_psk_plan_set_split_strict(amr_psk_plan* plan, int mode) {
  if (!plan || mode < -1 || mode > 1) return fail(AMR_E_INVALID, "amr_psk_plan_set_split_strict: bad argument");
  std::lock_guard<std::mutex> lk(plan->mu);
  plan->strict_mode = mode;
  return AMR_OK;
}

int amr_psk_plan_split_strict(amr_psk_plan* plan) {
  if (!plan) return -1;
  std::lock_guard<std::mutex> lk(plan->mu);
  return split_strict_on(plan) ? 1 : 0;
}

int amr_psk_plan_last_strict(const amr_psk_plan* plan) { return plan ? (plan->last_strict ? 1 : 0) : -1; }

int amr_psk_split_strict_design(const double* bp_b, const double* bp_a, const double* bp_zi, int bp_nt,
                                const double* lp_b, const double* lp_a, const double* lp_zi, int lp_nt, int64_t n,
                                int64_t first, int64_t sps, double* consts, double* tabs) {
  if (!bp_b || !bp_a || !bp_zi || !lp_b || !lp_a || !lp_zi || !consts || bp_nt != 9 || lp_nt != 5 || n < 1 ||
      sps < 1 || first < 0)
    return fail(AMR_E_INVALID, "amr_psk_split_strict_design: bad argument");
  Iir bp{}, lp{};
  bp.nt = bp_nt;
  lp.nt = lp_nt;
  for (int i = 0; i < bp_nt; ++i) { bp.b[i] = bp_b[i]; bp.a[i] = bp_a[i]; }
  for (int i = 0; i < bp_nt - 1; ++i) bp.zi[i] = bp_zi[i];
  for (int i = 0; i < lp_nt; ++i) { lp.b[i] = lp_b[i]; lp.a[i] = lp_a[i]; }
  for (int i = 0; i < lp_nt - 1; ++i) lp.zi[i] = lp_zi[i];
  const int64_t n_sym = n > first ? (n - first + sps - 1) / sps : 0;
  int64_t w1 = 0, w2 = 0;
  double kappa = 0.0;
  for (int i = 0; i < 32; ++i) consts[i] = 0.0;
  if (!split_design_core(bp, lp, n, n_sym, &w1, &w2, &kappa)) return fail(AMR_E_INVALID, "no time-split layout");
  std::vector<double> tab((size_t)(2 * w1 + 1) * 8);
  split_state_tables(bp, w1, tab.data(), tab.data() + (size_t)w1 * 8);
  const StrictDesign d = strict_design(bp, lp, tab.data(), tab.data() + (size_t)w1 * 8, w1, w2, n, first, sps, n_sym);
  // the device table's layout: kabs | z0abs | lpc | W | K12 | HS | GS | TZ
  const double v[32] = {d.g1x, d.gmax, d.hz, d.tk, d.zi_sum, d.zb, d.kx, d.ky, 2.0 * 0x1p-53 * (1.0 + 0x1p-50),
                        d.gam, d.c3, (double)w1, (double)w2, (double)n_sym, (double)d.W.size(), (double)d.K12.size(),
                        (double)d.HS.size(), (double)d.GS.size(), (double)d.TZ.size(), (double)d.k12_off, d.w_tail,
                        d.k12_tail, d.hs_tail, d.tz_tail, d.lp_tail, (double)d.lp_rad, d.ok ? 1.0 : 0.0, kappa};
  for (int i = 0; i < 32; ++i) consts[i] = v[i];
  if (!d.ok) return fail(AMR_E_INVALID, "no strict bound for these filters");
  if (tabs) {
    double* o = tabs;
    for (const std::vector<double>* t : {&d.kabs, &d.z0abs, &d.lpc, &d.W, &d.K12, &d.HS, &d.GS, &d.TZ}) {
      std::memcpy(o, t->data(), t->size() * 8);
      o += t->size();
    }
  }
  return AMR_OK;
}

int amr_psk_plan_last_f32f(const amr_psk_plan* plan) { return plan ? (plan->last_f32f ? 1 : 0) : -1; }

int amr_split_state_tables(const double* b, const double* a, const double* zi, int nt, int64_t w, double* K,
                           double* Z0) {
  if (!b || !a || !zi || !K || !Z0 || nt < 2 || nt > kMaxTaps || w < 0)
    return fail(AMR_E_INVALID, "amr_split_state_tables: bad argument");
  Iir f{};
  f.nt = nt;
  for (int i = 0; i < nt; ++i) { f.b[i] = b[i]; f.a[i] = a[i]; }
  for (int i = 0; i < nt - 1; ++i) f.zi[i] = zi[i];
  split_state_tables(f, w, K, Z0);
  return AMR_OK;
}

int amr_psk_plan_split_conv(amr_psk_plan* plan) {
  if (!plan) return -1;
  std::lock_guard<std::mutex> lk(plan->mu);
  if (!plan->split_designed) {
    if (hipSetDevice(plan->device) != hipSuccess) return 0;
    split_design(plan);
  }
  return split_conv_on(plan) ? 1 : 0;
}

int amr_psk_plan_split_info(amr_psk_plan* plan, int64_t* flagged, int64_t* warmup_bp, int64_t* warmup_lp,
                            int64_t* chunk, double* kappa) {
  if (!plan) return fail(AMR_E_INVALID, "plan is NULL");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  if (!plan->split_designed) split_design(plan);
  if (flagged) {
    *flagged = -1;
    if (plan->last_layout == AMR_LAYOUT_SPLIT) {
      int32_t c = 0;
      HIP_TRY(hipStreamSynchronize(plan->stream));
      HIP_TRY(hipMemcpy(&c, plan->split_count, 4, hipMemcpyDeviceToHost));
      *flagged = c;
    }
  }
  if (warmup_bp) *warmup_bp = plan->split_ok ? plan->split_w1 : -1;
  if (warmup_lp) *warmup_lp = plan->split_ok ? plan->split_w2 : -1;
  if (chunk) *chunk = plan->split_L;
  if (kappa) *kappa = plan->split_ok ? plan->split_kappa : -1.0;
  return AMR_OK;
}

int amr_psk_plan_exact_streams(amr_psk_plan* plan, int64_t* count) {
  if (!plan || !count) return fail(AMR_E_INVALID, "NULL argument");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  HIP_TRY(hipStreamSynchronize(plan->stream));
  if (plan->last_layout == AMR_LAYOUT_SPLIT) {
    // the flag memsets behind the gate run whatever the count; the row
    // fallback (and its exact low-pass) ran only when a stream was flagged
    int32_t sc = 0;
    HIP_TRY(hipMemcpy(&sc, plan->split_count, 4, hipMemcpyDeviceToHost));
    if (sc == 0) {
      *count = 0;
      return AMR_OK;
    }
  }
  std::vector<int32_t> fl((size_t)plan->groups * kWave);
  HIP_TRY(hipMemcpy(fl.data(), plan->flags, fl.size() * 4, hipMemcpyDeviceToHost));
  int64_t c = 0;
  for (int64_t i = 0; i < plan->last_exact; ++i) c += fl[(size_t)i] != 0;
  *count = c;
  return AMR_OK;
}

}  // extern "C"

namespace {

// ---- time-split layout design (the filters' responses: iir_design.h)
// A chunked pass differs from the serial one by (1) the zero start state,
// decayed after w samples to at most tail(w) * zmax * (the pass's input peak)
// at the pass's output, then amplified by the later passes' L1 gains -- w is
// chosen to bring that below 1/16 of u * G, G = g1(band-pass) + g1(low-pass);
// and (2) a different rounding trajectory: measured <= 1.4 u G over tones,
// square waves, noise and modulated inputs at 10 filter sets
// (tests/test_gpu_split.py), so |symbol error| <= kappa * peak|x| with kappa =
// 64 u G plus the transients.  Input peaks per unit peak|x|: the band-pass
// forward pass 3 (odd extension), backward 3 h1_bp; the low-pass (f * lo,
// odd extension) 9 h1_bp^2, backward 9 h1_bp^2 h1_lp.
bool split_design_core(const Iir& bp, const Iir& lp, int64_t n, int64_t n_sym, int64_t* w1o, int64_t* w2o,
                       double* kappa) {
  if (bp.nt != 9 || lp.nt != 5 || 2 * n_sym > n + 6 * bp.nt) return false;
  const IirGains gb = iir_gains(bp), gl = iir_gains(lp);
  if (!gb.ok || !gl.ok) return false;
  const double u = 0x1p-53;
  const double G = gb.g1 + gl.g1;
  const double tol = 0x1p-4 * u * G;
  const int64_t w1 = warmup_for(gb, gb.zmax * 3.0 * gb.h1 * gl.h1 * gl.h1, tol);
  const int64_t w2 = warmup_for(gl, gl.zmax * 9.0 * gb.h1 * gb.h1 * gl.h1, tol);
  if (w1 < 0 || w2 < 0 || w1 > n / 4 || w2 > n / 4) return false;
  *w1o = w1;
  *w2o = w2;
  *kappa = (kSplitSafety + 0.25) * u * G;
  return std::isfinite(*kappa) && *kappa > 0.0;
}
// the launch's chunking: L (0: the plan's rule -- at least kSplitMinL
// outputs, and long enough to keep a batch within kSplitLanes lanes)
// AMR_PSK_SPLIT_CONV=0: the w1-step warm-ups instead of KS0's convolution
bool split_conv_on(const amr_psk_plan* pl) {
  static const bool conv_env = [] { const char* e = std::getenv("AMR_PSK_SPLIT_CONV"); return !(e && e[0] == '0'); }();
  return conv_env && pl->split_tab && pl->bp.nt == 9;
}
// the strict bound for this plan's split calls: amr_psk_plan_set_split_strict,
// else AMR_PSK_SPLIT_STRICT=1 (off by default: DESIGN.md §3.3)
bool split_strict_on(const amr_psk_plan* pl) {
  static const bool env = [] { const char* e = std::getenv("AMR_PSK_SPLIT_STRICT"); return e && e[0] == '1'; }();
  return pl->strict_mode >= 0 ? pl->strict_mode == 1 : env;
}
PskSplit split_params(amr_psk_plan* pl, int64_t B, int64_t L) {
  PskSplit sp{};
  // AMR_PSK_SPLIT_MINL: a fixed minimum chunk length instead of the rules (an A/B knob)
  static const int64_t min_l = [] {
    const char* e = std::getenv("AMR_PSK_SPLIT_MINL");
    const long v = e ? std::atol(e) : 0;
    return v >= 8 && v <= 65536 ? (int64_t)v : 0;
  }();
  sp.conv = split_conv_on(pl) ? 1 : 0;
  const int64_t lanes = (B * pl->p.m1 + kSplitLanes - 1) / kSplitLanes;
  if (L > 0) sp.L = L;
  else if (min_l > 0) sp.L = std::max<int64_t>(min_l, lanes);
  else if (sp.conv)   // KS0's work grows with the chunk count, KS1-KS4's serial steps with L
    sp.L = std::max<int64_t>(lanes, std::min<int64_t>(kSplitConvMaxL, std::max<int64_t>(
                                        kSplitConvMinL, (B * pl->p.m1 + kSplitConvChunks - 1) / kSplitConvChunks)));
  else sp.L = std::max<int64_t>(kSplitMinL, lanes);
  sp.w1 = pl->split_w1;
  sp.w2 = pl->split_w2;
  sp.c1 = (pl->p.m1 + sp.L - 1) / sp.L;
  sp.c2 = (pl->p.m2 + sp.L - 1) / sp.L;
  sp.kappa = pl->split_kappa;
  sp.y1 = pl->s1;
  sp.f = pl->s2;
  sp.y3 = pl->s3;
  sp.sym = pl->s1;
  sp.peak = pl->split_peak;
  sp.flag = pl->split_flag;
  sp.count = pl->split_count;
  sp.ktab = pl->split_tab;
  sp.z0tab = pl->split_tab ? pl->split_tab + (size_t)sp.w1 * 8 : nullptr;
  sp.zs = pl->split_zs;
  pl->split_L = sp.L;
  if (pl->strict_designed && pl->sdes.ok && split_strict_on(pl) && sp.conv) {
    const StrictDesign& d = pl->sdes;
    // chunks on block boundaries (the per-block step bounds stay within a lane)
    sp.L = (sp.L + kStrictBlk - 1) / kStrictBlk * kStrictBlk;
    sp.c1 = (pl->p.m1 + sp.L - 1) / sp.L;
    sp.c2 = (pl->p.m2 + sp.L - 1) / sp.L;
    pl->split_L = sp.L;
    sp.strict = 1;
    sp.bnd = pl->strict_bnd;
    const double* t = pl->strict_tab;
    sp.kabs = t;
    sp.z0abs = t + sp.w1;
    sp.lpc = t + 2 * sp.w1 + 1;
    const double* k = sp.lpc + pl->p.n_sym;
    sp.kW = k;
    sp.kK12 = sp.kW + d.W.size();
    sp.kHS = sp.kK12 + d.K12.size();
    sp.kGS = sp.kHS + d.HS.size();
    sp.kTZ = sp.kGS + d.GS.size();
    sp.nw = (int)d.W.size();
    sp.nk = (int)d.K12.size();
    sp.k12_off = d.k12_off;
    sp.nh = (int)d.HS.size();
    sp.nz = (int)d.TZ.size();
    sp.w_tail = d.w_tail;
    sp.k12_tail = d.k12_tail;
    sp.hs_tail = d.hs_tail;
    sp.tz_tail = d.tz_tail;
    sp.lp_tail = d.lp_tail;
    sp.lp_rad = d.lp_rad;
    sp.gam = d.gam;
    sp.u2 = 2.0 * 0x1p-53 * (1.0 + 0x1p-50);
    sp.kx = d.kx;
    sp.ky = d.ky;
    sp.g1x = d.g1x;
    sp.gmax = d.gmax;
    sp.hz = d.hz;
    sp.tk = d.tk;
    sp.zi_sum = d.zi_sum;
    sp.zb = d.zb;
    sp.c3 = d.c3;
    sp.nb1 = (pl->p.m1 + kStrictBlk - 1) / kStrictBlk;
    sp.nbs = (pl->p.n + kStrictBlk - 1) / kStrictBlk;
    sp.sstride = 5 * sp.nb1 + 2 * sp.c1 + sp.nbs + pl->p.n_sym + 4;
  }
  return sp;
}
// the strict scratch for B streams of this call's geometry
int ensure_strict_sc(amr_psk_plan* pl, PskSplit& sp, int64_t B) {
  if (!sp.strict) return AMR_OK;
  const int64_t need = B * sp.sstride * 8;
  if (pl->strict_sc_bytes < need || !pl->strict_sc) {
    HIP_TRY(hipStreamSynchronize(pl->stream));
    if (pl->strict_sc) HIP_TRY(hipFree(pl->strict_sc));
    pl->strict_sc = nullptr;
    pl->strict_sc_bytes = 0;
    HIP_TRY(hipMalloc((void**)&pl->strict_sc, (size_t)need));
    pl->strict_sc_bytes = need;
  }
  sp.sc = pl->strict_sc;
  return AMR_OK;
}
// the strict mode's design and device tables, on the first strict call
int strict_prepare(amr_psk_plan* pl) {
  if (pl->strict_designed) return AMR_OK;
  pl->strict_designed = true;
  if (!pl->split_ok || !pl->split_tab) return AMR_OK;
  const int64_t w = pl->split_w1;
  std::vector<double> tab((size_t)(2 * w + 1) * 8);
  split_state_tables(pl->bp, w, tab.data(), tab.data() + (size_t)w * 8);
  pl->sdes = strict_design(pl->bp, pl->lp, tab.data(), tab.data() + (size_t)w * 8, w, pl->split_w2, pl->p.n,
                           pl->p.first, pl->p.sps, pl->p.n_sym);
  if (!pl->sdes.ok) return AMR_OK;
  std::vector<double> dev(pl->sdes.kabs);
  for (const std::vector<double>* v : {&pl->sdes.z0abs, &pl->sdes.lpc, &pl->sdes.W, &pl->sdes.K12, &pl->sdes.HS,
                                       &pl->sdes.GS, &pl->sdes.TZ})
    dev.insert(dev.end(), v->begin(), v->end());
  HIP_TRY(hipMalloc((void**)&pl->strict_tab, dev.size() * 8));
  HIP_TRY(hipMemcpy(pl->strict_tab, dev.data(), dev.size() * 8, hipMemcpyHostToDevice));
  HIP_TRY(hipMalloc((void**)&pl->strict_bnd, (size_t)pl->max_streams * 64));
  return AMR_OK;
}
// The lane layout's float32 hand-off: the band-pass output f
// is exact (scipy's filtfilt) and rounded to float32 for the low-pass, so
// |f32 - f| <= 2^-24 |f| (+ 2^-149 below FLT_MIN, covered by the 2^-120 floor
// the kernel adds).  The odd extension's 2 g0 - g_k at most triples that, and
// the low-pass filtfilt (linear) passes it with at most its L1 gain squared;
// on top, the low-pass's own rounding on the changed input, bounded like the
// time-split layout's trajectories (64x the L1 noise gain, x3 for the
// extension).  Per component, so x sqrt2 for the complex symbol:
//   |symbol error| <= sqrt2 (3 h1^2 2^-24 (1 + 2^-20) + 192 u g1) max|f|
// 0 when the low-pass's responses do not decay (no hand-off then).
double f32_design(const Iir& lp) {
  const IirGains gl = iir_gains(lp);
  if (!gl.ok) return 0.0;
  const double m = 0x1.6a09e667f3bcdp+0 * (3.0 * gl.h1 * gl.h1 * 0x1p-24 * (1.0 + 0x1p-20) + 192.0 * 0x1p-53 * gl.g1);
  return std::isfinite(m) ? m : 0.0;
}
void split_design(amr_psk_plan* pl) {
  pl->split_designed = true;
  pl->split_ok = split_design_core(pl->bp, pl->lp, pl->p.n, pl->p.n_sym, &pl->split_w1, &pl->split_w2,
                                   &pl->split_kappa);
  if (!pl->split_ok) return;
  // the band-pass's convolution tables (KS0); without them the plan keeps the warm-ups
  const int64_t w = pl->split_w1;
  std::vector<double> tab((size_t)(2 * w + 1) * 8);
  split_state_tables(pl->bp, w, tab.data(), tab.data() + (size_t)w * 8);
  if (hipMalloc((void**)&pl->split_tab, tab.size() * 8) != hipSuccess ||
      hipMemcpy(pl->split_tab, tab.data(), tab.size() * 8, hipMemcpyHostToDevice) != hipSuccess) {
    if (pl->split_tab) (void)hipFree(pl->split_tab);
    pl->split_tab = nullptr;
    (void)hipGetLastError();
  }
}
int ensure_split_zs(amr_psk_plan* pl, const PskSplit& sp, int64_t B) {
  if (!sp.conv) return AMR_OK;
  const int64_t need = B * sp.c1 * 8 * 8;
  if (pl->split_zs_bytes >= need && pl->split_zs) return AMR_OK;
  HIP_TRY(hipStreamSynchronize(pl->stream));
  if (pl->split_zs) HIP_TRY(hipFree(pl->split_zs));
  pl->split_zs = nullptr;
  pl->split_zs_bytes = 0;
  HIP_TRY(hipMalloc((void**)&pl->split_zs, (size_t)need));
  pl->split_zs_bytes = need;
  return AMR_OK;
}

// Launch the whole PSK pipeline on plan->stream.  Caller holds plan->mu.
// d_edge: the band-pass's odd-extension table [B][2 pad1] of a raw-integer
// capture (odd_ext.h), or null
int run_psk(amr_psk_plan* pl, const void* d_x, int dtype, int64_t B, int64_t x_stride, uint8_t* d_out,
            int64_t out_stride, int64_t* d_len, int64_t* d_sync, uint8_t* d_fec, int64_t fec_stride,
            int64_t* d_fec_len, int32_t* d_crc, const double* d_edge = nullptr) {
  if (B < 0 || B > pl->max_streams) return fail(AMR_E_CAPACITY, "batch exceeds plan max_streams");
  if (dtype_size(dtype) == 0) return fail(AMR_E_INVALID, "unknown dtype");
  if (x_stride < pl->p.n) return fail(AMR_E_INVALID, "x_stride < n_samples");
  if (out_stride < pl->out_cap - 1 || out_stride < 1) return fail(AMR_E_INVALID, "out_stride too small");
  for (bool& u : pl->ev_used) u = false;
  pl->last_exact = B;
  if (B == 0) return AMR_OK;
  hipStream_t st = pl->stream;
  if (pl->timing) {
    pl->ev_used[AMR_T_LAUNCH] = true;
    HIP_TRY(hipEventRecord(pl->ev[AMR_T_LAUNCH][0], st));
  }
  // Layout: one stream per lane (psk_lane_kernels.hip) once
  // enough streams are in flight on the device to give it waves -- it does
  // a third of the arithmetic per stream -- else the state-per-lane kernels
  // (more waves per stream, lower latency).  AMR_PSK_LANE=0/1 forces either.
  // The time-split layout (psk_split_kernels.hip, §3.3) for one capture or a
  // few: chunk-parallel passes, margin-checked decisions, the serial row
  // kernels behind them for a flagged batch.  AMR_PSK_SPLIT=0/1 (and
  // amr_psk_plan_set_layout, which overrides every switch) force it off / on.
  static const int lane_force = [] {
    const char* e = std::getenv("AMR_PSK_LANE");
    return e ? (e[0] == '1' ? 1 : 0) : -1;
  }();
  static const int split_force = [] {
    const char* e = std::getenv("AMR_PSK_SPLIT");
    return e ? (e[0] == '1' ? 1 : 0) : -1;
  }();
  const int64_t live = B * (pl->inflight > 1 ? pl->inflight : 1);
  // the lane kernels are written for butter(4) band-pass / low-pass
  // coefficient shapes: 9 taps and a palindromic 5-tap low-pass
  const bool lane_ok = pl->bp.nt == 9 && pl->p.lp_sym;
  int layout;
  if (pl->forced_layout >= 0) layout = pl->forced_layout;
  else if (lane_force >= 0) layout = lane_force == 1 ? AMR_LAYOUT_LANE : AMR_LAYOUT_ROW;
  else if (split_force == 1) layout = AMR_LAYOUT_SPLIT;
  else if (live >= kLaneMinLiveStreams) layout = AMR_LAYOUT_LANE;
  else layout = split_force != 0 && live <= kSplitMaxLiveStreams ? AMR_LAYOUT_SPLIT : AMR_LAYOUT_ROW;
  if (layout == AMR_LAYOUT_LANE && !lane_ok) layout = AMR_LAYOUT_ROW;
  if (layout == AMR_LAYOUT_SPLIT) {
    if (!pl->split_designed) split_design(pl);
    if (!pl->split_ok || B > 65535 || pl->p.n_sym < 2) layout = AMR_LAYOUT_ROW;
  }
  const bool lane = layout == AMR_LAYOUT_LANE;
  pl->last_layout = layout;
  if (pl->p.n_sym >= 2) {
    // the sizes this layout's kernels assume (the row layout's full-length
    // intermediates are allocated on its first call; the time-split layout
    // keeps its passes' outputs in the same buffers and runs the row kernels
    // behind them); a plan whose earlier grow failed re-tries here and fails
    // cleanly if it still cannot
    const int64_t b1 = kFrontSlack * 8 + (lane ? lane_s1_bytes(pl) : row_s1_bytes(pl));
    const int64_t b3 = kFrontSlack * 8 + (lane ? lane_s3_bytes(pl) : row_s3_bytes(pl));
    if (int rc = ensure_scratch(pl, b1, b3)) return rc;
  }
  PskBuffers b{};
  b.x = d_x;
  b.x_stride = x_stride;
  b.dtype = dtype;
  b.n_streams = B;
  b.inflight = pl->inflight;
  b.lo = pl->lo;
  b.lo2 = pl->lo2;
  b.s1 = pl->s1;
  b.s2 = pl->s2;
  b.s3 = pl->s3;
  b.words = pl->words;
  b.flags = pl->flags;
  b.bp_flags = pl->flags + pl->groups * kWave;
  b.out = d_out;
  b.out_stride = out_stride;
  b.out_len = d_len;
  b.sync_idx = d_sync;
  b.edge = d_edge;
  // AMR_SYNC_EACH_KERNEL=1: synchronise after every launch so a fault names its kernel
  static const bool sync_each = [] {
    const char* e = std::getenv("AMR_SYNC_EACH_KERNEL");
    return e && e[0] == '1';
  }();
  auto mark = [&](int slot, int which) -> hipError_t {
    if (sync_each && which == 1) {
      hipError_t e = hipStreamSynchronize(st);
      if (e != hipSuccess) {
        static const char* names[] = {"bandpass", "lowpass_fwd", "lowpass_bwd", "lowpass_exact", "slice+sync_pack", "fec"};
        std::fprintf(stderr, "[amr] kernel slot %s failed: %s\n", names[slot], hipGetErrorString(e));
        return e;
      }
    }
    if (!pl->timing) return hipSuccess;
    pl->ev_used[slot] = true;
    return hipEventRecord(pl->ev[slot][which], st);
  };
  if (pl->p.n_sym < 2) {
    // modem.py:95-96, 211: fewer than two symbols -> b''
    HIP_TRY(gate_wait(pl->gate, st));
    HIP_TRY(hipMemsetAsync(d_len, 0, (size_t)B * 8, st));
    HIP_TRY(hipMemsetAsync(d_sync, 0xFF, (size_t)B * 8, st));
  } else if (layout == AMR_LAYOUT_SPLIT) {
    if (split_strict_on(pl))
      if (int rc = strict_prepare(pl)) return rc;
    PskSplit sp = split_params(pl, B, 0);
    if (int rc = ensure_split_zs(pl, sp, B)) return rc;
    if (int rc = ensure_strict_sc(pl, sp, B)) return rc;
    sp.zs = pl->split_zs;
    HIP_TRY(hipMemsetAsync(pl->split_peak, 0, (size_t)pl->max_streams * 12 + 4, st));   // peaks, flags, count
    if (sp.strict) HIP_TRY(hipMemsetAsync(sp.bnd, 0, (size_t)B * 64, st));
    pl->last_strict = sp.strict != 0;
    HIP_TRY(mark(AMR_T_BANDPASS, 0));
    HIP_TRY(launch_psk_split_bp(b, pl->p, pl->bp, sp, st));
    HIP_TRY(mark(AMR_T_BANDPASS, 1));
    HIP_TRY(mark(AMR_T_LOWPASS_FWD, 0));
    HIP_TRY(launch_psk_split_lp(b, pl->p, pl->lp, sp, st));
    HIP_TRY(mark(AMR_T_LOWPASS_FWD, 1));
    HIP_TRY(mark(AMR_T_SYNC_PACK, 0));
    HIP_TRY(launch_psk_split_slice(b, pl->p, sp, st));
    HIP_TRY(gate_wait(pl->gate, st));                  // the outputs: after any gather still reading them
    HIP_TRY(launch_sync_pack(pl->words, pl->p.n_words, pl->p.n_bits, B, d_out, out_stride, d_len, d_sync, st));
    HIP_TRY(mark(AMR_T_SYNC_PACK, 1));
    // the serial row kernels over the whole batch, each exiting at once while
    // no stream was flagged (the count on the device; no host round trip)
    PskBuffers g = b;
    g.gate = pl->split_count;
    HIP_TRY(mark(AMR_T_LOWPASS_EXACT, 0));
    HIP_TRY(launch_psk_bandpass(g, pl->p, pl->bp, st));
    if (pl->lp_exact_only) {
      HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)pl->flags, 1, (size_t)B, st));
    } else {
      HIP_TRY(launch_psk_lowpass_fwd(g, pl->p, pl->lp, st));
      HIP_TRY(launch_psk_lowpass_bwd(g, pl->p, pl->lp, st));
    }
    HIP_TRY(launch_psk_lowpass_exact(g, pl->p, pl->lp, st));
    HIP_TRY(launch_psk_slice(g, pl->p, st));
    HIP_TRY(launch_sync_pack_gated(pl->words, pl->p.n_words, pl->p.n_bits, B, d_out, out_stride, d_len, d_sync,
                                   pl->split_count, st));
    HIP_TRY(mark(AMR_T_LOWPASS_EXACT, 1));
  } else if (lane) {
    // AMR_PSK_F32F=1 (an A/B, off by default): the float32 hand-off of f
    // between the band-pass and the low-pass (PskBuffers::f32f, DESIGN.md
    // §3.1) when the low-pass slices fused.  Bit-exact (margin + fix-up), and
    // the two kernels ran 8-12 % faster in flight, but its rigorous margin
    // flags 3.6 % of the benchmark's streams, whose groups the fix-up and K3x
    // then redo: 13.9 vs 3.72-3.79 ms/step (profiles/r05_psk_f32f_ab.txt)
    static const bool f32f_env = [] { const char* e = std::getenv("AMR_PSK_F32F"); return e && e[0] == '1'; }();
    b.fpeak = reinterpret_cast<double*>(pl->split_peak);
    b.f32f = f32f_env && pl->p.f32_margin > 0.0 && !pl->lp_exact_only && psk_lane_fused(b, pl->p) ? 1 : 0;
    pl->last_f32f = b.f32f != 0;
    HIP_TRY(mark(AMR_T_BANDPASS, 0));
    HIP_TRY(launch_psk_bandpass_lane(b, pl->p, pl->bp, st));
    HIP_TRY(mark(AMR_T_BANDPASS, 1));
    bool sliced = false;                        // the low-pass wrote the words itself (k_lp_lane FUSE)
    if (pl->lp_exact_only) {
      HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)pl->flags, 1, (size_t)B, st));
    } else {
      // forward + backward low-pass in one kernel: timed in the lowpass_fwd slot
      HIP_TRY(mark(AMR_T_LOWPASS_FWD, 0));
      HIP_TRY(launch_psk_lowpass_lane(b, pl->p, pl->lp, st, &sliced));
      HIP_TRY(mark(AMR_T_LOWPASS_FWD, 1));
    }
    HIP_TRY(mark(AMR_T_LOWPASS_EXACT, 0));
    // AMR_PSK_F32F_NOFIX=1: a timing-only diagnostic (flagged streams' bytes then wrong): no fix-up
    static const bool nofix = [] { const char* e = std::getenv("AMR_PSK_F32F_NOFIX"); return e && e[0] == '1'; }();
    if (b.f32f && !nofix) HIP_TRY(launch_psk_bandpass_fixup(b, pl->p, pl->bp, st));   // float64 f of the flagged groups
    HIP_TRY(launch_psk_lowpass_exact(b, pl->p, pl->lp, st));
    HIP_TRY(mark(AMR_T_LOWPASS_EXACT, 1));
    HIP_TRY(mark(AMR_T_SYNC_PACK, 0));
    HIP_TRY(launch_psk_slice(b, pl->p, st, sliced));   // then only the K3x streams
    HIP_TRY(gate_wait(pl->gate, st));                  // the outputs: after any gather still reading them
    HIP_TRY(launch_sync_pack(pl->words, pl->p.n_words, pl->p.n_bits, B, d_out, out_stride, d_len, d_sync, st));
    HIP_TRY(mark(AMR_T_SYNC_PACK, 1));
  } else {
    HIP_TRY(mark(AMR_T_BANDPASS, 0));
    HIP_TRY(launch_psk_bandpass(b, pl->p, pl->bp, st));
    HIP_TRY(mark(AMR_T_BANDPASS, 1));
    if (pl->lp_exact_only) {
      // every stream takes the exact complex path
      HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)pl->flags, 1, (size_t)B, st));
    } else {
      HIP_TRY(mark(AMR_T_LOWPASS_FWD, 0));
      HIP_TRY(launch_psk_lowpass_fwd(b, pl->p, pl->lp, st));
      HIP_TRY(mark(AMR_T_LOWPASS_FWD, 1));
      HIP_TRY(mark(AMR_T_LOWPASS_BWD, 0));
      HIP_TRY(launch_psk_lowpass_bwd(b, pl->p, pl->lp, st));
      HIP_TRY(mark(AMR_T_LOWPASS_BWD, 1));
    }
    HIP_TRY(mark(AMR_T_LOWPASS_EXACT, 0));
    HIP_TRY(launch_psk_lowpass_exact(b, pl->p, pl->lp, st));
    HIP_TRY(mark(AMR_T_LOWPASS_EXACT, 1));
    HIP_TRY(mark(AMR_T_SYNC_PACK, 0));
    HIP_TRY(launch_psk_slice(b, pl->p, st));
    HIP_TRY(gate_wait(pl->gate, st));
    HIP_TRY(launch_sync_pack(pl->words, pl->p.n_words, pl->p.n_bits, B, d_out, out_stride, d_len, d_sync, st));
    HIP_TRY(mark(AMR_T_SYNC_PACK, 1));
  }
  if (d_fec) {
    const uint32_t *tab = nullptr, *x2n = nullptr;
    int rc = device_crc(pl->device, &tab, &x2n);
    if (rc) return rc;
    HIP_TRY(mark(AMR_T_FEC, 0));
    HIP_TRY(launch_fec_decode(d_out, out_stride, d_len, B, d_fec, fec_stride, d_fec_len, d_crc, tab, x2n, st));
    HIP_TRY(mark(AMR_T_FEC, 1));
  }
  if (pl->timing) HIP_TRY(hipEventRecord(pl->ev[AMR_T_LAUNCH][1], st));
  return AMR_OK;
}

// the time-split passes alone (KS1-KS4) with chunk length L: the symbol
// samples in s1 [B][S][2] (amr_psk_split_symbols_host); with ebound (device,
// [B][S] + [B][4]) the strict bound too, KS5 writing it there
// (amr_psk_split_bounds_host).  Caller holds mu.
int run_psk_split_front(amr_psk_plan* pl, const void* d_x, int dtype, int64_t B, int64_t x_stride, int64_t L,
                        double* ebound) {
  if (int rc = ensure_scratch(pl, kFrontSlack * 8 + row_s1_bytes(pl), kFrontSlack * 8 + row_s3_bytes(pl))) return rc;
  PskBuffers b{};
  b.x = d_x;
  b.x_stride = x_stride;
  b.dtype = dtype;
  b.n_streams = B;
  b.lo = pl->lo;
  b.lo2 = pl->lo2;
  const int saved = pl->strict_mode;
  if (ebound) {
    pl->strict_mode = 1;
    if (int rc = strict_prepare(pl)) { pl->strict_mode = saved; return rc; }
  }
  PskSplit sp = split_params(pl, B, L);
  pl->strict_mode = saved;
  if (ebound && !sp.strict) return fail(AMR_E_INVALID, "no strict bound for this plan (no convolution starts or design)");
  if (int rc = ensure_split_zs(pl, sp, B)) return rc;
  if (int rc = ensure_strict_sc(pl, sp, B)) return rc;
  sp.zs = pl->split_zs;
  HIP_TRY(hipMemsetAsync(pl->split_peak, 0, (size_t)pl->max_streams * 12 + 4, pl->stream));
  if (sp.strict) HIP_TRY(hipMemsetAsync(sp.bnd, 0, (size_t)B * 64, pl->stream));
  HIP_TRY(launch_psk_split_bp(b, pl->p, pl->bp, sp, pl->stream));
  HIP_TRY(launch_psk_split_lp(b, pl->p, pl->lp, sp, pl->stream));
  if (ebound) {
    b.words = pl->words;
    HIP_TRY(launch_psk_split_slice(b, pl->p, sp, pl->stream));
    // e(k) and the scalars of every stream, packed [B][S + 4]
    const int64_t S = pl->p.n_sym;
    HIP_TRY(hipMemcpy2DAsync(ebound, (size_t)(S + 4) * 8, sp.sc + strict_off_e(sp), (size_t)sp.sstride * 8,
                             (size_t)(S + 4) * 8, (size_t)B, hipMemcpyDeviceToDevice, pl->stream));
  }
  return AMR_OK;
}

int ensure(void** p, int64_t* have, int64_t need) {
  if (*have >= need && *p) return AMR_OK;
  if (*p) HIP_TRY(hipFree(*p));
  *p = nullptr;
  HIP_TRY(hipMalloc(p, (size_t)need));
  *have = need;
  return AMR_OK;
}

}  // namespace

extern "C" {

int amr_psk_demod_device(amr_psk_plan* plan, const void* d_x, int dtype, int64_t n_streams, int64_t x_stride,
                         uint8_t* d_out, int64_t out_stride, int64_t* d_out_len, int64_t* d_sync_idx) {
  if (!plan || (!d_x && n_streams) || (!d_out && n_streams) || (!d_out_len && n_streams) ||
      (!d_sync_idx && n_streams))
    return fail(AMR_E_INVALID, "amr_psk_demod_device: NULL argument");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  return run_psk(plan, d_x, dtype, n_streams, x_stride, d_out, out_stride, d_out_len, d_sync_idx, nullptr, 0,
                 nullptr, nullptr);
}

int amr_psk_demod_fec_device(amr_psk_plan* plan, const void* d_x, int dtype, int64_t n_streams,
                             int64_t x_stride, uint8_t* d_out, int64_t out_stride, int64_t* d_out_len,
                             int64_t* d_sync_idx, uint8_t* d_fec, int64_t fec_stride, int64_t* d_fec_len,
                             int32_t* d_crc_ok) {
  if (!plan || !d_fec || !d_fec_len || !d_crc_ok) return fail(AMR_E_INVALID, "NULL argument");
  if (fec_stride < out_stride) return fail(AMR_E_INVALID, "fec_stride < out_stride");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  return run_psk(plan, d_x, dtype, n_streams, x_stride, d_out, out_stride, d_out_len, d_sync_idx, d_fec,
                 fec_stride, d_fec_len, d_crc_ok);
}

int amr_psk_demod_device_edges(amr_psk_plan* plan, const void* d_x, int dtype, int64_t n_streams, int64_t x_stride,
                               const double* d_edges, uint8_t* d_out, int64_t out_stride, int64_t* d_out_len,
                               int64_t* d_sync_idx) {
  if (!plan || (n_streams && (!d_x || !d_edges || !d_out || !d_out_len || !d_sync_idx)))
    return fail(AMR_E_INVALID, "amr_psk_demod_device_edges: NULL argument");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  return run_psk(plan, d_x, dtype, n_streams, x_stride, d_out, out_stride, d_out_len, d_sync_idx, nullptr, 0,
                 nullptr, nullptr, d_edges);
}

int amr_psk_demod_host(amr_psk_plan* plan, const void* x, int dtype, int64_t B, int64_t x_stride,
                       uint8_t* out, int64_t out_stride, int64_t* out_len, int64_t* sync_idx) {
  return psk_demod_host(plan, x, dtype, B, x_stride, nullptr, out, out_stride, out_len, sync_idx);
}

int amr_psk_demod_host_edges(amr_psk_plan* plan, const void* x, int dtype, int64_t B, int64_t x_stride,
                             const double* edges, uint8_t* out, int64_t out_stride, int64_t* out_len,
                             int64_t* sync_idx) {
  if (B && !edges) return fail(AMR_E_INVALID, "amr_psk_demod_host_edges: NULL edges");
  return psk_demod_host(plan, x, dtype, B, x_stride, edges, out, out_stride, out_len, sync_idx);
}

}  // extern "C"

namespace {
int psk_demod_host(amr_psk_plan* plan, const void* x, int dtype, int64_t B, int64_t x_stride, const double* edges,
                   uint8_t* out, int64_t out_stride, int64_t* out_len, int64_t* sync_idx) {
  if (!plan || (B && (!x || !out || !out_len || !sync_idx)))
    return fail(AMR_E_INVALID, "amr_psk_demod_host: NULL argument");
  const int64_t es = dtype_size(dtype);
  if (!es) return fail(AMR_E_INVALID, "unknown dtype");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  if (B > plan->max_streams) return fail(AMR_E_CAPACITY, "batch exceeds plan max_streams");
  // the same argument contract as the device entry point (run_psk), checked
  // before any copy: a short out_stride would cut rows while out_len still
  // reports their full length
  if (x_stride < plan->p.n) return fail(AMR_E_INVALID, "x_stride < n_samples");
  if (out_stride < plan->out_cap - 1 || out_stride < 1) return fail(AMR_E_INVALID, "out_stride too small");
  if (B == 0) return AMR_OK;
  const int64_t n = plan->p.n;
  const int64_t cap = plan->out_cap;
  int rc = ensure(&plan->d_x, &plan->d_x_bytes, plan->max_streams * n * 8);
  if (rc) return rc;
  if (!plan->d_out) {
    HIP_TRY(hipMalloc(&plan->d_out, (size_t)(plan->max_streams * cap)));
    HIP_TRY(hipMalloc(&plan->d_len, (size_t)plan->max_streams * 8));
    HIP_TRY(hipMalloc(&plan->d_sync, (size_t)plan->max_streams * 8));
  }
  rc = copy_batch_h2d(plan->d_x, x, n * es, x_stride * es, B, plan->stream);
  if (rc) return rc;
  const double* d_edge = nullptr;
  if (edges) {
    const int64_t eb = B * 2 * plan->p.pad1 * 8;
    if ((rc = ensure((void**)&plan->d_edge, &plan->d_edge_bytes, plan->max_streams * 2 * plan->p.pad1 * 8))) return rc;
    HIP_TRY(hipMemcpyAsync(plan->d_edge, edges, (size_t)eb, hipMemcpyHostToDevice, plan->stream));
    d_edge = plan->d_edge;
  }
  rc = run_psk(plan, plan->d_x, dtype, B, n, plan->d_out, cap, plan->d_len, plan->d_sync, nullptr, 0, nullptr,
               nullptr, d_edge);
  if (rc) return rc;
  rc = copy_batch_d2h(out, out_stride, plan->d_out, cap, out_stride < cap ? out_stride : cap, B, plan->stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(out_len, plan->d_len, (size_t)B * 8, hipMemcpyDeviceToHost, plan->stream));
  HIP_TRY(hipMemcpyAsync(sync_idx, plan->d_sync, (size_t)B * 8, hipMemcpyDeviceToHost, plan->stream));
  HIP_TRY(hipStreamSynchronize(plan->stream));
  return AMR_OK;
}
}  // namespace

extern "C" {

// Queued host entry: upload, demod and download on the plan's stream, no
// wait.  With two or more plans used in turn, batch k+1's upload (PCIe) runs
// while batch k demodulates -- the PCIe-inclusive rate of a stream of
// batches is then the link's, not link + demod.  Host buffers
// must stay untouched until amr_psk_plan_synchronize; page-locked buffers
// (amr_host_register) make the copies truly asynchronous.
int amr_psk_demod_host_async(amr_psk_plan* plan, const void* x, int dtype, int64_t B, int64_t x_stride,
                             uint8_t* out, int64_t out_stride, int64_t* out_len, int64_t* sync_idx) {
  if (!plan || (B && (!x || !out || !out_len || !sync_idx)))
    return fail(AMR_E_INVALID, "amr_psk_demod_host_async: NULL argument");
  const int64_t es = dtype_size(dtype);
  if (!es) return fail(AMR_E_INVALID, "unknown dtype");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  if (B > plan->max_streams) return fail(AMR_E_CAPACITY, "batch exceeds plan max_streams");
  if (x_stride < plan->p.n) return fail(AMR_E_INVALID, "x_stride < n_samples");
  if (out_stride < plan->out_cap - 1 || out_stride < 1) return fail(AMR_E_INVALID, "out_stride too small");
  if (B == 0) return AMR_OK;
  const int64_t n = plan->p.n;
  const int64_t cap = plan->out_cap;
  if (!plan->d_x || plan->d_x_bytes < plan->max_streams * n * 8) {
    HIP_TRY(hipStreamSynchronize(plan->stream));          // a previous staging buffer may still be read
    if (int rc = ensure(&plan->d_x, &plan->d_x_bytes, plan->max_streams * n * 8)) return rc;
  }
  if (!plan->d_out) {
    HIP_TRY(hipMalloc(&plan->d_out, (size_t)(plan->max_streams * cap)));
    HIP_TRY(hipMalloc(&plan->d_len, (size_t)plan->max_streams * 8));
    HIP_TRY(hipMalloc(&plan->d_sync, (size_t)plan->max_streams * 8));
  }
  hipStream_t st = plan->stream;
  if (x_stride == n)
    HIP_TRY(hipMemcpyAsync(plan->d_x, x, (size_t)(B * n * es), hipMemcpyHostToDevice, st));
  else
    HIP_TRY(hipMemcpy2DAsync(plan->d_x, (size_t)(n * es), x, (size_t)(x_stride * es), (size_t)(n * es), (size_t)B,
                             hipMemcpyHostToDevice, st));
  if (int rc = run_psk(plan, plan->d_x, dtype, B, n, plan->d_out, cap, plan->d_len, plan->d_sync, nullptr, 0,
                       nullptr, nullptr))
    return rc;
  if (out_stride == cap)
    HIP_TRY(hipMemcpyAsync(out, plan->d_out, (size_t)(B * cap), hipMemcpyDeviceToHost, st));
  else
    HIP_TRY(hipMemcpy2DAsync(out, (size_t)out_stride, plan->d_out, (size_t)cap, (size_t)std::min(out_stride, cap),
                             (size_t)B, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(out_len, plan->d_len, (size_t)B * 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(sync_idx, plan->d_sync, (size_t)B * 8, hipMemcpyDeviceToHost, st));
  return AMR_OK;
}

int amr_host_alloc(void** p, int64_t bytes) {
  if (!p || bytes <= 0) return fail(AMR_E_INVALID, "amr_host_alloc: bad argument");
  HIP_TRY(hipHostMalloc(p, (size_t)bytes, hipHostMallocDefault));
  return AMR_OK;
}

int amr_host_free(void* p) {
  if (p) HIP_TRY(hipHostFree(p));
  return AMR_OK;
}

int amr_host_register(void* p, int64_t bytes) {
  if (!p || bytes <= 0) return fail(AMR_E_INVALID, "amr_host_register: bad argument");
  HIP_TRY(hipHostRegister(p, (size_t)bytes, hipHostRegisterDefault));
  return AMR_OK;
}

int amr_host_unregister(void* p) {
  if (!p) return fail(AMR_E_INVALID, "amr_host_unregister: NULL");
  HIP_TRY(hipHostUnregister(p));
  return AMR_OK;
}

int amr_fec_decode_host(const uint8_t* in, int64_t in_stride, const int64_t* in_len, int64_t n, uint8_t* out,
                        int64_t out_stride, int64_t* out_len, int32_t* crc_ok) {
  if (n < 0 || (n && (!in || !in_len || !out || !out_len || !crc_ok)))
    return fail(AMR_E_INVALID, "amr_fec_decode_host: NULL argument");
  if (n == 0) return AMR_OK;
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  const uint32_t *tab = nullptr, *x2n = nullptr;
  int rc = device_crc(dev, &tab, &x2n);
  if (rc) return rc;
  int64_t maxlen = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (in_len[i] < 0 || in_len[i] > in_stride || in_len[i] > out_stride)
      return fail(AMR_E_INVALID, "in_len out of range");
    maxlen = in_len[i] > maxlen ? in_len[i] : maxlen;
  }
  if (dev < 0 || dev >= 64) return fail(AMR_E_INVALID, "device ordinal out of range");
  HostStaging& hs = g_staging[dev];
  std::lock_guard<std::mutex> lk(hs.mu);
  uint8_t *d_in = nullptr, *d_out = nullptr;
  int64_t *d_in_len = nullptr, *d_out_len = nullptr;
  int32_t* d_crc = nullptr;
  const int64_t stride = maxlen > 0 ? maxlen : 1;
  hipError_t e = staging_get(hs, 0, n * stride, (void**)&d_in);
  if (e == hipSuccess) e = staging_get(hs, 1, n * stride, (void**)&d_out);
  if (e == hipSuccess) e = staging_get(hs, 2, n * 8, (void**)&d_in_len);
  if (e == hipSuccess) e = staging_get(hs, 3, n * 8, (void**)&d_out_len);
  if (e == hipSuccess) e = staging_get(hs, 4, n * 4, (void**)&d_crc);
  if (e == hipSuccess && maxlen > 0)
    e = memcpy_rows(d_in, stride, in, in_stride, maxlen, n, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_in_len, in_len, (size_t)n * 8, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = launch_fec_decode(d_in, stride, d_in_len, n, d_out, stride, d_out_len, d_crc, tab, x2n, 0);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess && maxlen > 0)
    e = memcpy_rows(out, out_stride, d_out, stride, maxlen, n, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(out_len, d_out_len, (size_t)n * 8, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(crc_ok, d_crc, (size_t)n * 4, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return fail(AMR_E_HIP, std::string("amr_fec_decode_host: ") + hipGetErrorString(e));
  return AMR_OK;
}

// ---- benchmark / test input generator --------------------------------------
int amr_synth_tile_noise(const float* d_base, int64_t n_base, int64_t n_samples, float* d_out, int64_t n_streams,
                         int64_t row_offset, float sigma, uint64_t seed) {
  if (n_streams < 0 || n_samples < 0 || (n_streams && (!d_base || !d_out || n_base < 1)))
    return fail(AMR_E_INVALID, "amr_synth_tile_noise: bad argument");
  HIP_TRY(launch_synth_tile_noise(d_base, n_base, n_samples, d_out, n_streams, row_offset < 0 ? 0 : row_offset, sigma,
                                  seed, nullptr));
  HIP_TRY(hipDeviceSynchronize());
  return AMR_OK;
}

// ---- the slicer stage alone (modem.py:214-241 / 100-105) ---------------------
int amr_psk_slice_host(int kind, const double* sym, int64_t n_streams, int64_t n_sym, uint32_t* words) {
  if (kind != AMR_PSK_QPSK && kind != AMR_PSK_BPSK) return fail(AMR_E_INVALID, "unknown PSK kind");
  if (n_streams < 0 || n_sym < 0 || (n_streams && n_sym && (!sym || !words)))
    return fail(AMR_E_INVALID, "amr_psk_slice_host: bad argument");
  PskParams p{};
  p.kind = kind;
  p.n_sym = n_sym;
  p.n_bits = n_sym >= 2 ? (n_sym - 1) * (kind == AMR_PSK_QPSK ? 2 : 1) : 0;
  p.n_words = p.n_bits > 0 ? (p.n_bits + 31) / 32 : 1;
  if (n_streams == 0 || p.n_bits == 0) return AMR_OK;
  // the symbol buffer layout the low-pass kernels write: [B/64][re, im][S][64] (psk_common.h sym_index)
  const int64_t g64 = (n_streams + 63) / 64;
  std::vector<double> h((size_t)(g64 * 2 * n_sym * 64), 0.0);
  for (int64_t s = 0; s < n_streams; ++s)
    for (int64_t k = 0; k < n_sym; ++k)
      for (int c = 0; c < 2; ++c)
        h[(size_t)(((s >> 6) * 2 + c) * n_sym + k) * 64 + (s & 63)] = sym[(s * n_sym + k) * 2 + c];
  double* d_sym = nullptr;
  uint32_t* d_words = nullptr;
  hipError_t e = hipMalloc(&d_sym, h.size() * 8);
  if (e == hipSuccess) e = hipMalloc(&d_words, (size_t)(n_streams * p.n_words) * 4);
  if (e == hipSuccess) e = hipMemcpy(d_sym, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    PskBuffers b{};
    b.n_streams = n_streams;
    b.s1 = d_sym;
    b.words = d_words;
    e = launch_psk_slice(b, p, nullptr);
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(words, d_words, (size_t)(n_streams * p.n_words) * 4, hipMemcpyDeviceToHost);
  if (d_sym) (void)hipFree(d_sym);
  if (d_words) (void)hipFree(d_words);
  if (e != hipSuccess) return fail(AMR_E_HIP, std::string("amr_psk_slice_host: ") + hipGetErrorString(e));
  return AMR_OK;
}

// ---- FBP frame parse (decoder.py:142-208) ------------------------------------
int amr_frame_parse_device(amr_psk_plan* plan, const uint8_t* d_in, int64_t in_stride, const int64_t* d_in_len,
                           int64_t n, int64_t max_cands, int32_t* d_n_cands, amr_frame_rec* d_recs) {
  if (n < 0 || max_cands < 1 || in_stride < 0 || (n && (!d_in || !d_in_len || !d_n_cands || !d_recs)))
    return fail(AMR_E_INVALID, "amr_frame_parse_device: bad argument");
  if (max_cands > AMR_FRAME_MAX_CANDS)
    return fail(AMR_E_INVALID, "max_cands > AMR_FRAME_MAX_CANDS (the kernel keeps at most that many records)");
  if (n == 0) return AMR_OK;
  int dev = 0;
  hipStream_t st = nullptr;
  if (plan) {
    dev = plan->device;
    st = plan->stream;
    HIP_TRY(hipSetDevice(dev));
  } else {
    HIP_TRY(hipGetDevice(&dev));
  }
  const uint32_t *tab = nullptr, *x2n = nullptr;
  int rc = device_crc(dev, &tab, &x2n);
  if (rc) return rc;
  HIP_TRY(launch_frame_parse(d_in, in_stride, d_in_len, n, max_cands, d_n_cands, d_recs, tab, x2n, st));
  return AMR_OK;
}

int amr_frame_parse_host(const uint8_t* in, int64_t in_stride, const int64_t* in_len, int64_t n, int64_t max_cands,
                         int32_t* n_cands, amr_frame_rec* recs) {
  if (n < 0 || max_cands < 1 || (n && (!in || !in_len || !n_cands || !recs)))
    return fail(AMR_E_INVALID, "amr_frame_parse_host: bad argument");
  if (max_cands > AMR_FRAME_MAX_CANDS)
    return fail(AMR_E_INVALID, "max_cands > AMR_FRAME_MAX_CANDS (the kernel keeps at most that many records)");
  if (n == 0) return AMR_OK;
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  const uint32_t *tab = nullptr, *x2n = nullptr;
  int rc = device_crc(dev, &tab, &x2n);
  if (rc) return rc;
  int64_t maxlen = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (in_len[i] < 0 || in_len[i] > in_stride) return fail(AMR_E_INVALID, "in_len out of range");
    maxlen = in_len[i] > maxlen ? in_len[i] : maxlen;
  }
  if (dev < 0 || dev >= 64) return fail(AMR_E_INVALID, "device ordinal out of range");
  HostStaging& hs = g_staging[dev];
  std::lock_guard<std::mutex> lk(hs.mu);
  uint8_t* d_in = nullptr;
  int64_t* d_in_len = nullptr;
  int32_t* d_cnt = nullptr;
  amr_frame_rec* d_recs = nullptr;
  const int64_t stride = maxlen > 0 ? maxlen : 1;
  hipError_t e = staging_get(hs, 0, n * stride, (void**)&d_in);
  if (e == hipSuccess) e = staging_get(hs, 2, n * 8, (void**)&d_in_len);
  if (e == hipSuccess) e = staging_get(hs, 4, n * 4, (void**)&d_cnt);
  if (e == hipSuccess) e = staging_get(hs, 5, n * max_cands * (int64_t)sizeof(amr_frame_rec), (void**)&d_recs);
  if (e == hipSuccess && maxlen > 0)
    e = memcpy_rows(d_in, stride, in, in_stride, maxlen, n, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_in_len, in_len, (size_t)n * 8, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = launch_frame_parse(d_in, stride, d_in_len, n, max_cands, d_cnt, d_recs, tab, x2n, 0);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(n_cands, d_cnt, (size_t)n * 4, hipMemcpyDeviceToHost);
  if (e == hipSuccess)
    e = hipMemcpy(recs, d_recs, (size_t)(n * max_cands) * sizeof(amr_frame_rec), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return fail(AMR_E_HIP, std::string("amr_frame_parse_host: ") + hipGetErrorString(e));
  return AMR_OK;
}

}  // extern "C"

namespace amr {
hipError_t gate_wait(GatherGate& g, hipStream_t st) {
  if (!g.pending) return hipSuccess;
  g.pending = false;                                // one wait covers every earlier gather
  return hipStreamWaitEvent(st, g.ev, 0);
}

hipError_t gate_sync(GatherGate& g) {
  if (!g.pending) return hipSuccess;
  g.pending = false;
  return hipEventSynchronize(g.ev);
}

void gate_free(GatherGate& g) {
  if (!g.ev) return;
  (void)hipEventSynchronize(g.ev);
  (void)hipEventDestroy(g.ev);
  g.ev = nullptr;
  g.pending = false;
}

// The gather on the communicator's own stream, in call order (so several
// plans -- batches in flight on several streams -- can share one
// communicator without two ranks ever entering its collectives in different
// orders).  With a gate (the producer plan's), the gather waits for the work
// already queued on the producer stream (event), and the producer's later
// work waits for the gather where it writes its outputs (gate_wait): its
// filters overlap the gather, and no plan's next batch queues behind another
// plan's gather.
int allgather_after(amr_comm* comm, const void* d_send, void* d_recv, int64_t bytes_per_rank, hipStream_t producer,
                    GatherGate* gate, hipEvent_t done) {
  if (!comm || !d_send || !d_recv || bytes_per_rank < 0) return fail(AMR_E_INVALID, "bad allgather args");
  // one RCCL call on the communicator at a time, whichever host thread makes
  // it (the host collectives take the same lock; lock order: plan, then comm)
  std::lock_guard<std::mutex> lk(comm->mu);
  HIP_TRY(hipSetDevice(comm->device));
  hipEvent_t before = nullptr;
  if (gate) {
    if (!gate->ev) HIP_TRY(hipEventCreateWithFlags(&gate->ev, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&before, hipEventDisableTiming));
    hipError_t e = hipEventRecord(before, producer);
    if (e == hipSuccess) e = hipStreamWaitEvent(comm->stream, before, 0);
    (void)hipEventDestroy(before);                 // released once the wait is done
    if (e != hipSuccess) return fail(AMR_E_HIP, std::string("amr_allgather: ") + hipGetErrorString(e));
  }
  ncclResult_t r = ncclAllGather(d_send, d_recv, (size_t)bytes_per_rank, ncclUint8, comm->comm, comm->stream);
  if (r != ncclSuccess) return fail(AMR_E_RCCL, std::string("ncclAllGather: ") + ncclGetErrorString(r));
  if (gate) {
    HIP_TRY(hipEventRecord(gate->ev, comm->stream));
    gate->pending = true;
  }
  if (done) HIP_TRY(hipEventRecord(done, comm->stream));
  return AMR_OK;
}
}  // namespace amr

extern "C" {

// ---- RCCL -------------------------------------------------------------------
int amr_comm_unique_id(uint8_t* id) {
  if (!id) return fail(AMR_E_INVALID, "id is NULL");
  static_assert(sizeof(ncclUniqueId) == AMR_UNIQUE_ID_BYTES, "unique id size");
  ncclUniqueId u;
  ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) return fail(AMR_E_RCCL, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  std::memcpy(id, &u, sizeof(u));
  return AMR_OK;
}

int amr_comm_create(amr_comm** comm, const uint8_t* id, int nranks, int rank, int device) {
  if (!comm || !id || nranks < 1 || rank < 0 || rank >= nranks) return fail(AMR_E_INVALID, "bad comm args");
  HIP_TRY(hipSetDevice(device));
  auto* c = new amr_comm();
  c->device = device;
  c->nranks = nranks;
  c->rank = rank;
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
  if (r != ncclSuccess) {
    delete c;
    return fail(AMR_E_RCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  }
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    ncclCommDestroy(c->comm);
    delete c;
    return fail(AMR_E_HIP, "hipStreamCreate failed");
  }
  *comm = c;
  return AMR_OK;
}

int amr_comm_destroy(amr_comm* comm) {
  if (!comm) return AMR_OK;
  (void)hipSetDevice(comm->device);
  if (comm->stream) (void)hipStreamSynchronize(comm->stream);
  if (comm->stage) (void)hipFree(comm->stage);
  if (comm->comm) ncclCommDestroy(comm->comm);
  if (comm->stream) (void)hipStreamDestroy(comm->stream);
  delete comm;
  return AMR_OK;
}

// Every collective of a communicator runs on the communicator's own stream, in
// call order, so that several plans (batches in flight on several streams)
// can share one communicator without two ranks ever entering its collectives
// in different orders.  With a plan, the gather waits for the work already on
// the plan's stream (event), and the plan's later work waits for the gather
// before it writes any output (the gather reads them); amr_psk_plan_synchronize
// also waits for it.
int amr_allgather(amr_comm* comm, const void* d_send, void* d_recv, int64_t bytes_per_rank, amr_psk_plan* plan) {
  if (!plan) return allgather_after(comm, d_send, d_recv, bytes_per_rank, nullptr, nullptr);
  std::lock_guard<std::mutex> lk(plan->mu);
  // the launch's timing slot ends when its outputs are gathered (AMR_T_LAUNCH)
  return allgather_after(comm, d_send, d_recv, bytes_per_rank, plan->stream, &plan->gate,
                         plan->timing && plan->ev_used[AMR_T_LAUNCH] ? plan->ev[AMR_T_LAUNCH][1] : nullptr);
}

int amr_comm_synchronize(amr_comm* comm) {
  if (!comm) return fail(AMR_E_INVALID, "comm is NULL");
  HIP_TRY(hipSetDevice(comm->device));
  HIP_TRY(hipStreamSynchronize(comm->stream));
  return AMR_OK;
}

int amr_comm_world(const amr_comm* comm, int* nranks, int* rank) {
  if (!comm || !nranks || !rank) return fail(AMR_E_INVALID, "amr_comm_world: NULL argument");
  *nranks = comm->nranks;
  *rank = comm->rank;
  return AMR_OK;
}

namespace {
// the comm's device staging buffer, at least `bytes` (caller holds comm->mu)
int comm_stage(amr_comm* c, int64_t bytes) {
  if (c->stage_bytes >= bytes && c->stage) return AMR_OK;
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (c->stage) HIP_TRY(hipFree(c->stage));
  c->stage = nullptr;
  c->stage_bytes = 0;
  HIP_TRY(hipMalloc(&c->stage, (size_t)bytes));
  c->stage_bytes = bytes;
  return AMR_OK;
}
}  // namespace

int amr_comm_allgather_host(amr_comm* comm, const void* send, void* recv, int64_t bytes_per_rank) {
  if (!comm || bytes_per_rank < 0 || (bytes_per_rank && (!send || !recv)))
    return fail(AMR_E_INVALID, "amr_comm_allgather_host: bad argument");
  if (bytes_per_rank == 0) return AMR_OK;
  std::lock_guard<std::mutex> lk(comm->mu);
  HIP_TRY(hipSetDevice(comm->device));
  const int64_t total = bytes_per_rank * (1 + comm->nranks);     // [send | recv (world slots)]
  if (int rc = comm_stage(comm, total)) return rc;
  uint8_t* d_send = static_cast<uint8_t*>(comm->stage);
  uint8_t* d_recv = d_send + bytes_per_rank;
  HIP_TRY(hipMemcpyAsync(d_send, send, (size_t)bytes_per_rank, hipMemcpyHostToDevice, comm->stream));
  ncclResult_t r = ncclAllGather(d_send, d_recv, (size_t)bytes_per_rank, ncclUint8, comm->comm, comm->stream);
  if (r != ncclSuccess) return fail(AMR_E_RCCL, std::string("ncclAllGather: ") + ncclGetErrorString(r));
  HIP_TRY(hipMemcpyAsync(recv, d_recv, (size_t)(bytes_per_rank * comm->nranks), hipMemcpyDeviceToHost, comm->stream));
  HIP_TRY(hipStreamSynchronize(comm->stream));
  return AMR_OK;
}

int amr_comm_allreduce_max(amr_comm* comm, double* values, int64_t count) {
  if (!comm || count < 0 || (count && !values)) return fail(AMR_E_INVALID, "amr_comm_allreduce_max: bad argument");
  if (count == 0) return AMR_OK;
  std::lock_guard<std::mutex> lk(comm->mu);
  HIP_TRY(hipSetDevice(comm->device));
  if (int rc = comm_stage(comm, count * 8)) return rc;
  double* d = static_cast<double*>(comm->stage);
  HIP_TRY(hipMemcpyAsync(d, values, (size_t)(count * 8), hipMemcpyHostToDevice, comm->stream));
  ncclResult_t r = ncclAllReduce(d, d, (size_t)count, ncclFloat64, ncclMax, comm->comm, comm->stream);
  if (r != ncclSuccess) return fail(AMR_E_RCCL, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
  HIP_TRY(hipMemcpyAsync(values, d, (size_t)(count * 8), hipMemcpyDeviceToHost, comm->stream));
  HIP_TRY(hipStreamSynchronize(comm->stream));
  return AMR_OK;
}

}  // extern "C"
