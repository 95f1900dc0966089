// api_common.h -- error plumbing shared by the C-ABI translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/amr.h"

namespace amr {
int fail(int code, const std::string& msg);   // sets amr_last_error(), returns code
int64_t dtype_size(int dtype);                // bytes per sample, 0 = unknown
// device + stream a *_device call on `plan` runs on (plan NULL: current device, null stream)
int plan_stream(amr_psk_plan* plan, int* dev, hipStream_t* st);
// B rows of `row_bytes` between pitched buffers without one DMA per row:
// equal pitches -> one copy; otherwise packed / scattered on the host around
// one copy (hipMemcpy2D only for a pitched device destination).
hipError_t memcpy_rows(void* dst, int64_t dst_pitch, const void* src, int64_t src_pitch, int64_t row_bytes,
                       int64_t B, hipMemcpyKind kind);
// Copy a host batch [B rows of `row_bytes`, `src_pitch` apart] into dense
// device rows, for the *_host entry points.  Waits for `st` first (its earlier
// work may still read dst), then copies synchronously: a dense source as one
// 1-D copy (pageable 1-D copies ran at 56 GB/s on the MI355X box where the
// pitched async copy of the same 6.3 GB ran at ~24, tools/host_path_probe.py).
int copy_batch_h2d(void* dst, const void* src, int64_t row_bytes, int64_t src_pitch, int64_t B, hipStream_t st);
// The output side: B rows of `row_bytes` from device rows `src_pitch` apart to
// host rows `dst_pitch` apart, after the work queued on `st`.  One 1-D copy
// (then a host-side scatter when the pitches differ): a pitched D2H copy into
// pageable memory ran as one transfer per row -- 16384 rows took 215 ms.
int copy_batch_d2h(void* dst, int64_t dst_pitch, const void* src, int64_t src_pitch, int64_t row_bytes, int64_t B,
                   hipStream_t st);
// A plan's hold on its outputs while an all-gather reads them
// (amr_allgather / amr_fsk_allgather with a plan): the gather waits for the
// plan's queued work, and the plan's later work waits for the gather only
// where it writes an output (gate_wait before its output kernels), so the
// next batch's filters run while the gather is in flight.  One event: the
// communicator's stream runs gathers in call order, so its latest record
// covers every earlier gather of the plan.
struct GatherGate {
  hipEvent_t ev = nullptr;
  bool pending = false;
};
hipError_t gate_wait(GatherGate& g, hipStream_t st);   // `st` waits for the pending gather
hipError_t gate_sync(GatherGate& g);                   // the host waits for it
void gate_free(GatherGate& g);
// the RCCL all-gather of amr_allgather / amr_fsk_allgather (api.cpp); gate
// NULL: no ordering against the producer stream; `done` (optional) is
// recorded on the comm's stream after the gather (the producer's launch timing)
int allgather_after(amr_comm* comm, const void* d_send, void* d_recv, int64_t bytes_per_rank, hipStream_t producer,
                    GatherGate* gate, hipEvent_t done = nullptr);
}  // namespace amr

#define HIP_TRY(expr)                                                                              \
  do {                                                                                             \
    hipError_t e_ = (expr);                                                                        \
    if (e_ != hipSuccess)                                                                          \
      return ::amr::fail(e_ == hipErrorOutOfMemory ? AMR_E_NOMEM : AMR_E_HIP,                      \
                         std::string(#expr) + ": " + hipGetErrorString(e_));                      \
  } while (0)
