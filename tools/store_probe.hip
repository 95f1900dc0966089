// store_probe.hip -- what a per-sample-pair global store costs a recurrence
// wave (quad 5-tap step, 512 waves, one per SIMD at most):
//   0 no store
//   1 dwordx4 per pair, 64-bit VGPR address + immediate offsets, every lane
//   2 dwordx4 per pair, SGPR base + 32-bit VGPR offset (saddr), every lane
//   3 dwordx2 per sample (y only), saddr, every lane
//   4 as 2 but only lane j==0 of each quad (exec set once per 16 samples)
//   5 lane j keeps pair j of every 4 (v_cndmask), one dwordx4 per 8 samples
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/store_probe.hip -o tools/store_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ unsigned long long now() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long u = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(u & 0xffffffff), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(u >> 32), CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}

template <int ST>
__global__ __launch_bounds__(256) void k(double2* out, unsigned long long* cyc, int iters, const double* co) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int j4 = lane & 3;
  const int wave = blockIdx.x * 4 + wv;
  double z = 0.01 * lane;
  double xs[16], acc = 0;
  for (int i = 0; i < 16; ++i) xs[i] = 0.3 + lane * 1e-3 + i * 0.01;
  const double b0 = co[0], cb = co[j4 + 1], ca = co[10 + j4], cm = j4 == 3 ? 0.0 : 1.0;
  double2* o = out + (size_t)wave * 16 * 8 + (lane >> 2);       // ST 1: per-lane 64-bit pointer
  unsigned off = (unsigned)(wave * 16 * 8 + (lane >> 2)) * 16u;   // ST 2-5: byte offset from the SGPR base
  unsigned long long t0 = now();
  for (int it = 0; it < iters; ++it) {
    double2 keep = make_double2(0, 0);
#pragma unroll
    for (int s = 0; s < 16; s += 2) {
      double y[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        asm volatile("" : "+v"(xs[s + u]));
        const double x = xs[s + u];
        const double t = z + b0 * x;
        y[u] = dpp_f64<0x00>(t);
        const double zC = dpp_f64<0xF9>(z) * cm;
        z = (zC + x * cb) - y[u] * ca;
        if (ST == 3) *reinterpret_cast<double*>(reinterpret_cast<char*>(out) + off + (s + u) * 16 * 16 * 8) = y[u];
      }
      if (ST == 1) o[(s / 2) * 16 * 16] = make_double2(y[0], y[1]);
      if (ST == 2 || (ST == 4 && j4 == 0))
        *reinterpret_cast<double2*>(reinterpret_cast<char*>(out) + off + (s / 2) * 16 * 16 * 16) = make_double2(y[0], y[1]);
      if (ST == 5) {
        const int k = (s / 2) & 3;
        keep.x = j4 == k ? y[0] : keep.x;
        keep.y = j4 == k ? y[1] : keep.y;
        if (k == 3) *reinterpret_cast<double2*>(reinterpret_cast<char*>(out) + off + (s / 8) * 16 * 16 * 16) = keep;
      }
      acc += y[0];
    }
    if (ST == 1) o += 16 * 16 * 8;
    else off += 16 * 16 * 16 * 8;
  }
  unsigned long long t1 = now();
  out[(size_t)(iters + 1) * 8 * 16 * 16 * 64 + wave * 64 + lane] = make_double2(acc, z);
  if (lane == 0) cyc[wave] = t1 - t0;
}

template <int ST>
__global__ __launch_bounds__(256) void k4(double2* out, unsigned long long* cyc, int iters, const double* co) {
  // ST 4 with the lane selection hoisted: only quad lane 0 runs the stores
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int j4 = lane & 3;
  const int wave = blockIdx.x * 4 + wv;
  double z = 0.01 * lane;
  double xs[16], acc = 0;
  for (int i = 0; i < 16; ++i) xs[i] = 0.3 + lane * 1e-3 + i * 0.01;
  const double b0 = co[0], cb = co[j4 + 1], ca = co[10 + j4], cm = j4 == 3 ? 0.0 : 1.0;
  unsigned off = (unsigned)(wave * 16 * 8 + (lane >> 2)) * 16u;
  unsigned long long t0 = now();
  for (int it = 0; it < iters; ++it) {
    double2 ys[8];
#pragma unroll
    for (int s = 0; s < 16; s += 2) {
      double y[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        asm volatile("" : "+v"(xs[s + u]));
        const double x = xs[s + u];
        const double t = z + b0 * x;
        y[u] = dpp_f64<0x00>(t);
        const double zC = dpp_f64<0xF9>(z) * cm;
        z = (zC + x * cb) - y[u] * ca;
      }
      ys[s / 2] = make_double2(y[0], y[1]);
      acc += y[0];
    }
    if (j4 == 0) {
#pragma unroll
      for (int q = 0; q < 8; ++q)
        *reinterpret_cast<double2*>(reinterpret_cast<char*>(out) + off + q * 16 * 16 * 16) = ys[q];
    }
    off += 16 * 16 * 16 * 8;
  }
  unsigned long long t1 = now();
  out[(size_t)(iters + 1) * 8 * 16 * 16 * 64 + wave * 64 + lane] = make_double2(acc, z);
  if (lane == 0) cyc[wave] = t1 - t0;
}

int main() {
  double2* out;
  double* co;
  unsigned long long* cyc;
  const int iters = 64;
  (void)hipMalloc(&out, (size_t)(iters + 2) * 8 * 16 * 16 * 64 * 16);
  (void)hipMalloc(&cyc, 4096 * 8);
  (void)hipMalloc(&co, 18 * 8);
  double h[18] = {0.031, 0, -0.12, 0, 0.187, 0, -0.12, 0, 0.031, 1, -3.9, 7.1, -7.9, 5.9, -2.9, 0.9, -0.2, 0.02};
  (void)hipMemcpy(co, h, sizeof(h), hipMemcpyHostToDevice);
  static unsigned long long c[4096];
  const char* names[] = {"no store", "x4 vaddr64 all lanes", "x4 saddr all lanes", "x2 per sample saddr",
                         "x4 saddr j==0 (per pair)", "x4 1 per 8 samples (cndmask)", "x4 j==0 hoisted"};
  void (*ks[])(double2*, unsigned long long*, int, const double*) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k4<4>};
  for (int m = 0; m < 7; ++m) {
    const int waves = 512, blocks = waves / 4;
    hipLaunchKernelGGL(ks[m], dim3(blocks), dim3(256), 0, 0, out, cyc, iters, co);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(ks[m], dim3(blocks), dim3(256), 0, 0, out, cyc, iters, co);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(c, cyc, 8 * waves, hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < waves; ++i) avg += c[i];
    printf("%-30s cycles/sample=%6.1f\n", names[m], avg / waves / iters / 16);
  }
  return 0;
}
