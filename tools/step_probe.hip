// step_probe.hip -- cycles per sample of the recurrence steps used by the
// kernels (operands in registers, no memory): lane-per-stream 9-tap, quad
// split 9-tap (K1q), pair split 5-tap (K2/K3), lane-per-component 5-tap.
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I audio-modem-radio_amd/csrc tools/step_probe.hip -o tools/step_probe
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

template <int MODE>
__global__ __launch_bounds__(64) void k(double* out, unsigned long long* cyc, int iters, const double* co) {
  const int lane = threadIdx.x, j = lane & 3;
  double b[9], a[9], z[8];
  for (int i = 0; i < 9; ++i) { b[i] = co[i]; a[i] = co[9 + i]; }
  for (int i = 0; i < 8; ++i) z[i] = 0.001 * (lane + i);
  const double cAb = co[j], cAa = co[9 + j], cBb = co[4 + j], cBa = co[13 + j];
  double zA = 0.01 * lane, zB = 0.02 * lane;
  double x = 0.3 + lane * 1e-3, acc = 0;
  const bool top = j == 3, top2 = (j & 1) == 1;
  unsigned long long t0 = now();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      double y;
      if (MODE == 0) {          // lane per stream, 9 taps
        y = z[0] + b[0] * x;
#pragma unroll
        for (int i = 0; i < 7; ++i) z[i] = (z[i + 1] + x * b[i + 1]) - y * a[i + 1];
        z[7] = x * b[8] - y * a[8];
      } else if (MODE == 1) {   // quad split, 9 taps
        const double t = zA + b[0] * x;
        y = dpp_f64<0x00>(t);
        double zC = dpp_f64<0xF9>(zA);
        zC = top ? -0.0 : zC;
        const double nA = (zB + x * cAb) - y * cAa;
        const double nB = (zC + x * cBb) - y * cBa;
        zA = nA; zB = nB;
      } else if (MODE == 2) {   // pair split, 5 taps
        const double t = zA + b[0] * x;
        y = dpp_f64<0xA0>(t);
        double zC = dpp_f64<0xF5>(zA);
        zC = top2 ? -0.0 : zC;
        const double nA = (zB + x * cAb) - y * cAa;
        const double nB = (zC + x * cBb) - y * cBa;
        zA = nA; zB = nB;
      } else {                  // lane per component, 5 taps
        y = z[0] + b[0] * x;
#pragma unroll
        for (int i = 0; i < 3; ++i) z[i] = (z[i + 1] + x * b[i + 1]) - y * a[i + 1];
        z[3] = x * b[4] - y * a[4];
      }
      acc += y;
      x = -x;
    }
  }
  unsigned long long t1 = now();
  out[blockIdx.x * 64 + lane] = acc + zA + zB + z[0];
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  double *out, *co;
  unsigned long long* cyc;
  (void)hipMalloc(&out, 4096 * 64 * 8);
  (void)hipMalloc(&cyc, 4096 * 8);
  (void)hipMalloc(&co, 18 * 8);
  double h[18] = {0.031, 0, -0.12, 0, 0.187, 0, -0.12, 0, 0.031, 1, -3.9, 7.1, -7.9, 5.9, -2.9, 0.9, -0.2, 0.02};
  (void)hipMemcpy(co, h, sizeof(h), hipMemcpyHostToDevice);
  static unsigned long long c[4096];
  const int iters = 2000;
  const char* names[] = {"lane/stream 9-tap", "quad 9-tap (K1q)", "pair 5-tap (K2/K3)", "lane 5-tap"};
  void (*ks[])(double*, unsigned long long*, int, const double*) = {k<0>, k<1>, k<2>, k<3>};
  for (int m = 0; m < 4; ++m)
    for (int blocks : {64, 256, 1024}) {
      hipLaunchKernelGGL(ks[m], dim3(blocks), dim3(64), 0, 0, out, cyc, iters, co);
      (void)hipDeviceSynchronize();
      hipLaunchKernelGGL(ks[m], dim3(blocks), dim3(64), 0, 0, out, cyc, iters, co);
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(c, cyc, 8 * blocks, hipMemcpyDeviceToHost);
      double avg = 0;
      for (int i = 0; i < blocks; ++i) avg += c[i];
      printf("%-22s blocks=%4d cycles/sample=%6.1f\n", names[m], blocks, avg / blocks / iters / 16);
    }
  return 0;
}
