// hbm_mix_probe.hip -- what HBM bandwidth a streaming kernel reaches on this
// MI355X at the read/write mixes of the demod passes:
//   mode 0  read only            (sum of a, one dword per wave written)
//   mode 1  copy, 1 read : 1 write
//   mode 2  2 reads : 1 write    (c = a + b; the PSK step is ~70 % reads)
//   mode 3  3 reads : 1 write
// 16-B vector loads and stores, grid-stride over 4 GiB per array, 8192
// workgroups of 256 threads (one access per lane and iteration) or 2048 with
// 4 / 8 independent accesses per lane in flight; the median of 10 launches after 2 warm-ups,
// timed with HIP events.  No result depends on the values.
// hipcc --offload-arch=gfx950 -O3 tools/hbm_mix_probe.hip -o tools/hbm_mix_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                      \
      return 1;                                                                \
    }                                                                          \
  } while (0)

// the same with U independent 16-B accesses in flight per lane and iteration
// (block-strided so every load instruction stays coalesced)
template <int MODE, int U>
__global__ __launch_bounds__(256) void k_mix_u(const double2* __restrict__ a, const double2* __restrict__ b,
                                               const double2* __restrict__ d, double2* __restrict__ c, size_t n) {
  double2 acc = make_double2(0.0, 0.0);
  const size_t stride = (size_t)gridDim.x * blockDim.x * U;
  for (size_t i0 = (size_t)blockIdx.x * blockDim.x * U + threadIdx.x; i0 < n; i0 += stride) {
    double2 va[U], vb[U], vd[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = i0 + (size_t)u * blockDim.x;
      va[u] = a[i];
      if constexpr (MODE >= 2) vb[u] = b[i];
      if constexpr (MODE >= 3) vd[u] = d[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = i0 + (size_t)u * blockDim.x;
      if constexpr (MODE == 0) {
        acc.x += va[u].x;
        acc.y += va[u].y;
      } else if constexpr (MODE == 1) {
        c[i] = va[u];
      } else if constexpr (MODE == 2) {
        c[i] = make_double2(va[u].x + vb[u].x, va[u].y + vb[u].y);
      } else {
        c[i] = make_double2(va[u].x + vb[u].x + vd[u].x, va[u].y + vb[u].y + vd[u].y);
      }
    }
  }
  if constexpr (MODE == 0)
    if (acc.x == 12345.678) c[threadIdx.x] = acc;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_mix(const double2* __restrict__ a, const double2* __restrict__ b,
                                             const double2* __restrict__ d, double2* __restrict__ c, size_t n) {
  double2 acc = make_double2(0.0, 0.0);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const double2 va = a[i];
    if constexpr (MODE == 0) {
      acc.x += va.x;
      acc.y += va.y;
    } else if constexpr (MODE == 1) {
      c[i] = va;
    } else if constexpr (MODE == 2) {
      const double2 vb = b[i];
      c[i] = make_double2(va.x + vb.x, va.y + vb.y);
    } else {
      const double2 vb = b[i], vd = d[i];
      c[i] = make_double2(va.x + vb.x + vd.x, va.y + vb.y + vd.y);
    }
  }
  if constexpr (MODE == 0)
    if (acc.x == 12345.678) c[threadIdx.x] = acc;   // keeps the loads; never true for zeroed inputs
}

template <int MODE, int U = 1>
int run(const double2* a, const double2* b, const double2* d, double2* c, size_t n) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> ms;
  for (int it = 0; it < 12; ++it) {
    CK(hipEventRecord(e0));
    if constexpr (U == 1) hipLaunchKernelGGL(k_mix<MODE>, dim3(8192), dim3(256), 0, 0, a, b, d, c, n);
    else hipLaunchKernelGGL((k_mix_u<MODE, U>), dim3(2048), dim3(256), 0, 0, a, b, d, c, n);
    CK(hipGetLastError());
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float t = 0;
    CK(hipEventElapsedTime(&t, e0, e1));
    if (it >= 2) ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  const double t = ms[ms.size() / 2] * 1e-3;
  const int reads = MODE == 0 ? 1 : MODE == 1 ? 1 : MODE == 2 ? 2 : 3;
  const int writes = MODE == 0 ? 0 : 1;
  const double bytes = (double)n * 16 * (reads + writes);
  std::printf("mode %d unroll %d  %d read : %d write  %.3f ms  %.0f GB/s\n", MODE, U, reads, writes, t * 1e3,
              bytes / t / 1e9);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return 0;
}

int main() {
  const size_t bytes = (size_t)4 << 30;
  const size_t n = bytes / 16;
  double2 *a, *b, *c, *d;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&c, bytes));
  CK(hipMalloc(&d, bytes));
  CK(hipMemset(a, 0, bytes));
  CK(hipMemset(b, 0, bytes));
  CK(hipMemset(d, 0, bytes));
  if (run<0>(a, b, d, c, n) || run<1>(a, b, d, c, n) || run<2>(a, b, d, c, n) || run<3>(a, b, d, c, n)) return 1;
  if (run<0, 4>(a, b, d, c, n) || run<1, 4>(a, b, d, c, n) || run<2, 4>(a, b, d, c, n) || run<3, 4>(a, b, d, c, n))
    return 1;
  if (run<0, 8>(a, b, d, c, n) || run<1, 8>(a, b, d, c, n) || run<2, 8>(a, b, d, c, n)) return 1;
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(c));
  CK(hipFree(d));
  return 0;
}
