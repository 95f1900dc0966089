// step_probe4.hip -- the serial fallback's per-step latency floor (VERDICT r5
// item 4): ONE stream, one wave, the 9-tap band-pass DF-II-T in scipy's order
// over N samples from registers/LDS-free inputs, checked bit for bit against
// the same recurrence on the host (-ffp-contract=off), timed with HIP events.
//   0  row16 (K1r today): lane 8+j owns z[j]; t = z + b0 x, y = bcast8(t),
//      zC = shl1(z), z = (zC + x b[j+1]) - y a[j+1]          (9 instructions)
//   1  row16, z0 replicated (every lane carries y's chain: add -> mul -> sub,
//      the two DPP moves off it)                               (13)
//   2  row16 "p form": lane 8+j owns p[j] = z[j] + b[j] x (the add scipy
//      forms first), so y = p[0] needs no extra add: inc = shl1(p) (the top
//      lane's out-of-row read returns its own b8 x), y = bcast8(p),
//      z = inc - a y, p = z + b x'                             (8)
//   3  p form, y's chain replicated in every lane: y' = (bcast(p1) - a1 y) + b0 x'
//   4  one lane owns every state (no DPP; 34 FP64 per sample)
//   5  the chain alone: y' = (c - a y) + b x (3 dependent FP64, the floor of
//      any exact form)
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/step_probe4.hip -o tools/step_probe4.bin
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

__device__ __forceinline__ double bcast16(double v, int lane_sel) {
  const long u = __builtin_bit_cast(long, v);
  long r;
  if (lane_sel == 8) r = __builtin_amdgcn_update_dpp(0L, u, 0x158, 0xF, 0xF, true);
  else r = __builtin_amdgcn_update_dpp(0L, u, 0x159, 0xF, 0xF, true);
  return __builtin_bit_cast(double, r);
}
// z[j+1] from the next lane; the row's top lane keeps `keep` (its own value)
__device__ __forceinline__ double shl1_keep(double v, double keep) {
  const long long u = __builtin_bit_cast(long long, v);
  const long long k = __builtin_bit_cast(long long, keep);
  const int lo = __builtin_amdgcn_update_dpp((int)(k & 0xffffffff), (int)(u & 0xffffffff), 0x101, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(k >> 32), (int)(u >> 32), 0x101, 0xF, 0xF, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}

constexpr int N = 96000;
constexpr int BLK = 16;   // samples per register block: x in, y out by vector accesses

// x for a block of 16 (+1 look-ahead) samples from LDS into registers, the
// block's 16 y values out of registers by lane 8 (4 x 32-B stores)
#define BLOCK_LOOP(BODY)                                                        \
  for (int c = 0; c < N; c += 256) {                                            \
    for (int i = lane; i < 256; i += 64) xs[i] = xg[c + i];                     \
    if (lane == 0) xs[256] = c + 256 < N ? xg[c + 256] : 0.0;                   \
    __syncthreads();                                                            \
    for (int ib = 0; ib < 256; ib += BLK) {                                     \
      double xv[BLK + 1], yv[BLK];                                              \
      _Pragma("unroll") for (int q2 = 0; q2 <= BLK; ++q2) xv[q2] = xs[ib + q2]; \
      _Pragma("unroll") for (int ii = 0; ii < BLK; ++ii) {                      \
        const double x = xv[ii];                                                \
        const double xn = xv[ii + 1];                                           \
        (void)xn;                                                               \
        double y;                                                               \
        BODY                                                                    \
        yv[ii] = y;                                                             \
      }                                                                         \
      if (lane == 8) {                                                          \
        _Pragma("unroll") for (int ii = 0; ii < BLK; ++ii) yout[c + ib + ii] = yv[ii]; \
      }                                                                         \
    }                                                                           \
    __syncthreads();                                                            \
  }

template <int MODE>
__global__ __launch_bounds__(64) void k(const double* __restrict__ xg, double* __restrict__ yout, const double* co) {
  const int lane = threadIdx.x & 63;
  const int l = lane & 15;
  const int j = l >= 8 ? l - 8 : 0;
  const double* b = co;
  const double* a = co + 9;
  const double b0 = b[0];
  __shared__ double xs[264];
  if constexpr (MODE == 0) {
    const double cb = b[j + 1], ca = a[j + 1];
    double z = 0.0;
    BLOCK_LOOP({
      const double t = z + b0 * x;
      y = bcast16(t, 8);
      const double zC = shl1_keep(z, -0.0);
      z = (zC + x * cb) - y * ca;
    })
  } else if constexpr (MODE == 1) {
    // lane 8+j owns z[j+1] (j < 7); every lane carries z0
    const double cb2 = j + 2 <= 8 ? b[j + 2] : 0.0, ca2 = j + 2 <= 8 ? a[j + 2] : 0.0;
    const double b1 = b[1], a1 = a[1];
    double z0 = 0.0, zA = 0.0;
    BLOCK_LOOP({
      y = z0 + b0 * x;
      const double z1 = bcast16(zA, 8);
      const double zC = shl1_keep(zA, -0.0);
      z0 = (z1 + x * b1) - y * a1;
      zA = (zC + x * cb2) - y * ca2;
    })
  } else if constexpr (MODE == 2) {
    // lane 8+j: p = z[j] + b[j] x (j = 0..7); the top lane's incoming is b8 x
    const double bj = b[j], aj1 = a[j + 1], b8 = b[8];
    const double x0 = xg[0];
    double p = 0.0 + bj * x0, q = b8 * x0;
    BLOCK_LOOP({
      y = bcast16(p, 8);
      const double inc = shl1_keep(p, q);
      const double zz = inc - y * aj1;
      p = zz + bj * xn;
      q = b8 * xn;
    })
  } else if constexpr (MODE == 3) {
    const double bj = b[j], aj1 = a[j + 1], b8 = b[8], a1 = a[1];
    const double x0 = xg[0];
    double p = 0.0 + bj * x0, q = b8 * x0;
    double yr = 0.0 + b0 * x0;
    BLOCK_LOOP({
      y = yr;
      const double p1 = bcast16(p, 9);
      const double inc = shl1_keep(p, q);
      const double zz = inc - y * aj1;
      yr = (p1 - y * a1) + b0 * xn;
      p = zz + bj * xn;
      q = b8 * xn;
    })
  } else if constexpr (MODE == 4) {
    double zs[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    BLOCK_LOOP({
      y = zs[0] + b[0] * x;
      _Pragma("unroll") for (int m = 0; m < 7; ++m) zs[m] = (zs[m + 1] + x * b[m + 1]) - y * a[m + 1];
      zs[7] = x * b[8] - y * a[8];
    })
  } else {
    double yr = 0.0;
    const double cc = co[3], a1 = a[1];
    BLOCK_LOOP({
      yr = (cc - yr * a1) + b0 * x;
      y = yr;
    })
  }
}

int main() {
  // scipy.signal.butter(4, [0.01, 0.3625], 'band'): QPSK@9600, 96 kHz (modem.py:197)
  double h[18] = {0.031185825959656993, 0.0, -0.12474330383862797, 0.0, 0.18711495575794196, 0.0,
                  -0.12474330383862797, 0.0, 0.031185825959656993, 1.0, -5.052770720381921, 11.123485643730572,
                  -14.212457214051257, 11.765950405233157, -6.511026507791935, 2.3198266936016445,
                  -0.4795625183038954, 0.046554754973477774};
  std::vector<double> x(N), ref(N), got(N);
  unsigned s = 12345;
  for (int i = 0; i < N; ++i) {
    s = s * 1103515245u + 12345u;
    x[i] = ((s >> 8) & 0xffff) / 32768.0 - 1.0;
  }
  {
    double z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < N; ++i) {
      volatile double y = z[0] + h[0] * x[i];
      for (int m = 0; m < 7; ++m) {
        volatile double t = z[m + 1] + x[i] * h[m + 1];
        volatile double u = y * h[9 + m + 1];
        z[m] = t - u;
      }
      volatile double t = x[i] * h[8];
      volatile double u = y * h[17];
      z[7] = t - u;
      ref[i] = y;
    }
  }
  double *dx, *dy, *dc;
  (void)hipMalloc(&dx, N * 8);
  (void)hipMalloc(&dy, N * 8);
  (void)hipMalloc(&dc, sizeof(h));
  (void)hipMemcpy(dx, x.data(), N * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(dc, h, sizeof(h), hipMemcpyHostToDevice);
  const char* names[] = {"row16 (K1r)", "row16 z0-rep", "row16 p-form", "row16 p-form y-rep", "one lane", "chain only"};
  void (*ks[])(const double*, double*, const double*) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>};
  for (int m = 0; m < 6; ++m) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipMemset(dy, 0, N * 8);
    hipLaunchKernelGGL(ks[m], dim3(1), dim3(64), 0, 0, dx, dy, dc);
    (void)hipDeviceSynchronize();
    float best = 1e9f;
    for (int r = 0; r < 5; ++r) {
      (void)hipEventRecord(e0, 0);
      hipLaunchKernelGGL(ks[m], dim3(1), dim3(64), 0, 0, dx, dy, dc);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      best = ms < best ? ms : best;
    }
    (void)hipMemcpy(got.data(), dy, N * 8, hipMemcpyDeviceToHost);
    long bad = 0;
    for (int i = 0; i < N; ++i) bad += std::memcmp(&got[i], &ref[i], 8) != 0;
    printf("%-20s one wave: %7.3f ms for %d samples = %6.2f ns/sample  bit-exact mismatches %ld%s\n", names[m], best, N,
           best * 1e6 / N, bad, m == 5 ? " (not the filter)" : "");
  }
  return 0;
}
