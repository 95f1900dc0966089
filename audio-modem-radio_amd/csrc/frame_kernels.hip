// frame_kernels.hip -- batched FBP frame parse for gfx950: the receive step
// after the demodulator.
//
// Replaces, for a batch of decoded byte streams at once, the per-stream
//   decoder.parse_fbp_stream_enhanced  (/root/reference/decoder.py:142-208)
// i.e. every b'FBPC' occurrence (raw.find in a loop, :152-159), in order, run
// through the reference's checks (:163-186) and the CRC32 of its payload
// (binascii.crc32, :189).  The kernel reports, per candidate, which check
// stopped it (or the CRC verdict) plus the header fields; the host turns the
// records into the reference's list of dicts and its log lines (decoder.py).
//
// One wave per stream.  Integer work: byte compares, wave ballots, the
// per-lane table CRC + crc32_combine tree shared with the FEC decode.
#include "amr_internal.h"
#include "amr.h"

namespace amr {

constexpr int kMaxLdsCands = 256;   // candidates a wave keeps in LDS for the CRC phase

__device__ __forceinline__ uint32_t crc_multmodp(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (int i = 0; i < 32; ++i) {
    if (a & m) p ^= b;
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ 0xEDB88320u : b >> 1;
  }
  return p;
}

__device__ __forceinline__ uint32_t crc_x8nmodp(int64_t len, const uint32_t* __restrict__ x2n) {
  uint32_t p = 1u << 31;
  int k = 3;
  while (len) {
    if (len & 1) p = crc_multmodp(x2n[k & 31], p);
    len >>= 1;
    ++k;
  }
  return p;
}

__device__ __forceinline__ uint32_t le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

__global__ __launch_bounds__(64) void k_frame_parse(const uint8_t* __restrict__ in, int64_t in_stride,
                                                    const int64_t* __restrict__ in_len, int64_t n_streams,
                                                    int64_t max_cands, int32_t* __restrict__ n_cands,
                                                    amr_frame_rec* __restrict__ recs,
                                                    const uint32_t* __restrict__ crc_table,
                                                    const uint32_t* __restrict__ x2n) {
  __shared__ uint32_t tab[256];
  __shared__ uint32_t xp[32];
  __shared__ int64_t c_ps[kMaxLdsCands];
  __shared__ uint32_t c_dlen[kMaxLdsCands];
  __shared__ int32_t c_pending[kMaxLdsCands];
  __shared__ uint32_t c_pcrc[kMaxLdsCands];
  const int lane = threadIdx.x;
  for (int i = lane; i < 256; i += kWave) tab[i] = crc_table[i];
  if (lane < 32) xp[lane] = x2n[lane];
  __syncthreads();
  const int64_t s = blockIdx.x;
  if (s >= n_streams) return;
  const uint8_t* __restrict__ raw = in + (size_t)s * in_stride;
  const int64_t L = in_len[s];
  amr_frame_rec* __restrict__ rec = recs + (size_t)s * max_cands;
  const int64_t keep = max_cands < kMaxLdsCands ? max_cands : kMaxLdsCands;

  // ---- 1. every magic position, in increasing order (decoder.py:152-159)
  int64_t cnt = 0;
  for (int64_t base = 0; base + 4 <= L; base += kWave) {
    const int64_t p = base + lane;
    const bool hit = p + 4 <= L && raw[p] == 'F' && raw[p + 1] == 'B' && raw[p + 2] == 'P' && raw[p + 3] == 'C';
    const uint64_t m = __ballot(hit);
    if (hit) {
      const int64_t k = cnt + __popcll(m & ((1ull << lane) - 1));
      if (k < keep) {
        // ---- 2. the reference's checks (decoder.py:163-186), in its order
        amr_frame_rec r{};
        r.start = p;
        r.status = AMR_FRAME_PENDING_CRC;
        int32_t pending = 0;
        if (p + 30 > L) {
          r.status = AMR_FRAME_SHORT;
        } else {
          const int32_t nl = raw[p + 4];
          r.name_len = nl;
          r.name_start = p + 5;
          const int64_t meta = p + 5 + nl;
          if (nl == 0) {
            r.status = AMR_FRAME_NONAME;
          } else if (meta + 24 > L) {
            r.status = AMR_FRAME_NOMETA;
          } else {
            r.part = le32(raw + meta);
            r.total = le32(raw + meta + 4);
            r.fsize = le32(raw + meta + 8);
            r.fcrc = le32(raw + meta + 12);
            r.dlen = le32(raw + meta + 16);
            r.pcrc = le32(raw + meta + 20);
            r.payload_start = meta + 24;
            if (r.dlen > 50000000u || r.dlen == 0) r.status = AMR_FRAME_BADLEN;
            else if (r.payload_start + (int64_t)r.dlen > L) r.status = AMR_FRAME_INCOMPLETE;
            else pending = 1;
          }
        }
        rec[k] = r;
        c_ps[k] = r.payload_start;
        c_dlen[k] = r.dlen;
        c_pending[k] = pending;
        c_pcrc[k] = r.pcrc;
      }
    }
    cnt += __popcll(m);
  }
  if (lane == 0) n_cands[s] = (int32_t)(cnt < 0x7fffffff ? cnt : 0x7fffffff);
  __syncthreads();

  // ---- 3. CRC32 of each pending payload, the whole wave per payload
  const int64_t nk = cnt < keep ? cnt : keep;
  for (int64_t k = 0; k < nk; ++k) {
    if (!c_pending[k]) continue;                // wave-uniform (LDS broadcast)
    const uint8_t* __restrict__ pay = raw + c_ps[k];
    const int64_t n = c_dlen[k];
    const int64_t c = (n + kWave - 1) / kWave;
    const int64_t lo = (int64_t)lane * c;
    const int64_t hi = lo + c < n ? lo + c : n;
    uint32_t crc = 0xFFFFFFFFu;
    for (int64_t i = lo; i < hi; ++i) crc = tab[(crc ^ pay[i]) & 0xFF] ^ (crc >> 8);
    crc ^= 0xFFFFFFFFu;
    int64_t len = hi > lo ? hi - lo : 0;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      const uint32_t rc = __shfl_down(crc, d);
      const int64_t rl = __shfl_down(len, d);
      if ((lane & (2 * d - 1)) == 0) {
        crc = crc_multmodp(crc_x8nmodp(rl, xp), crc) ^ rc;
        len += rl;
      }
    }
    if (lane == 0) {
      rec[k].calc_crc = crc;
      rec[k].status = (crc == c_pcrc[k]) ? AMR_FRAME_OK : AMR_FRAME_CRC_BAD;
    }
  }
}

hipError_t launch_frame_parse(const uint8_t* in, int64_t in_stride, const int64_t* in_len, int64_t n_streams,
                              int64_t max_cands, int32_t* n_cands, amr_frame_rec* recs, const uint32_t* crc_table,
                              const uint32_t* x2n, hipStream_t st) {
  if (n_streams <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_frame_parse, dim3((unsigned)n_streams), dim3(kWave), 0, st, in, in_stride, in_len, n_streams,
                     max_cands, n_cands, recs, crc_table, x2n);
  return hipGetLastError();
}

}  // namespace amr
