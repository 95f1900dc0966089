// fp64_probe.hip -- measures what bounds a lane-per-stream IIR on gfx950:
// FP64 VALU issue rate and dependent latency for ONE wave on a SIMD, and the
// cost per sample of the real DF-II-T step (9 taps) with operands in
// registers.  Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/fp64_probe.hip -o /tmp/fp64_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ unsigned long long now() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

template <int MODE>
__global__ __launch_bounds__(64) void k_probe(double* out, unsigned long long* cyc, int iters, double seed) {
  double a0 = seed + threadIdx.x, a1 = a0 * 1.1, a2 = a0 * 1.2, a3 = a0 * 1.3, a4 = a0 * 1.4, a5 = a0 * 1.5,
         a6 = a0 * 1.6, a7 = a0 * 1.7;
  const double c = 1.0000001;
  unsigned long long t0 = now();
  for (int i = 0; i < iters; ++i) {
    if (MODE == 0) {  // 8 independent chains of adds: issue rate
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        a0 = a0 + c; a1 = a1 + c; a2 = a2 + c; a3 = a3 + c; a4 = a4 + c; a5 = a5 + c; a6 = a6 + c; a7 = a7 + c;
      }
    } else if (MODE == 1) {  // one dependent chain of adds: latency
#pragma unroll
      for (int k = 0; k < 64; ++k) a0 = a0 + c;
    } else if (MODE == 2) {  // one dependent chain of muls
#pragma unroll
      for (int k = 0; k < 64; ++k) a0 = a0 * c;
    } else if (MODE == 3) {  // 8 independent chains of muls
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        a0 = a0 * c; a1 = a1 * c; a2 = a2 * c; a3 = a3 * c; a4 = a4 * c; a5 = a5 * c; a6 = a6 * c; a7 = a7 * c;
      }
    } else if (MODE == 4) {  // 8 independent fp32 adds (reference)
      float f0 = a0, f1 = a1, f2 = a2, f3 = a3, f4 = a4, f5 = a5, f6 = a6, f7 = a7;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        f0 += 1.f; f1 += 1.f; f2 += 1.f; f3 += 1.f; f4 += 1.f; f5 += 1.f; f6 += 1.f; f7 += 1.f;
      }
      a0 = f0; a1 = f1; a2 = f2; a3 = f3; a4 = f4; a5 = f5; a6 = f6; a7 = f7;
    }
  }
  unsigned long long t1 = now();
  out[blockIdx.x * 64 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// the real band-pass step, 9 taps, zero odd taps, registers only
__global__ __launch_bounds__(64) void k_df2t(double* out, unsigned long long* cyc, int iters, const double* coef) {
  double b[9], a[9], z[8];
  for (int i = 0; i < 9; ++i) { b[i] = coef[i]; a[i] = coef[9 + i]; }
  for (int i = 0; i < 8; ++i) z[i] = 0.001 * (threadIdx.x + i);
  double x = 0.3 + threadIdx.x * 1e-3, acc = 0;
  unsigned long long t0 = now();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const double y = z[0] + b[0] * x;
      const double xz = x * b[1];
#pragma unroll
      for (int i = 0; i < 7; ++i) z[i] = (z[i + 1] + (((i + 1) & 1) ? xz : x * b[i + 1])) - y * a[i + 1];
      z[7] = x * b[8] - y * a[8];
      acc += y;
      x = -x;
    }
  }
  unsigned long long t1 = now();
  out[blockIdx.x * 64 + threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  double* out;
  unsigned long long* cyc;
  double* coef;
  (void)hipMalloc(&out, 4096 * 64 * 8);
  (void)hipMalloc(&cyc, 4096 * 8);
  hipMalloc(&coef, 18 * 8);
  double h[18] = {0.031, 0, -0.12, 0, 0.187, 0, -0.12, 0, 0.031, 1, -3.9, 7.1, -7.9, 5.9, -2.9, 0.9, -0.2, 0.02};
  hipMemcpy(coef, h, sizeof(h), hipMemcpyHostToDevice);
  const int iters = 2000;
  static unsigned long long c[4096];
  auto run = [&](const char* name, void (*k)(double*, unsigned long long*, int, double), int blocks, int threads,
                 double instr_per_iter) {
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters, 1.0);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters, 1.0);
    hipDeviceSynchronize();
    hipMemcpy(c, cyc, 8 * blocks, hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < blocks; ++i) avg += c[i];
    avg /= blocks;
    printf("%-34s blocks=%4d  cycles/iter=%8.1f  cycles/instr=%6.2f\n", name, blocks, avg / iters,
           avg / iters / instr_per_iter);
  };
  for (int blocks : {1, 64, 256, 1024, 2048}) {
    run("8 indep f64 add chains", k_probe<0>, blocks, 64, 64);
    run("1 dep f64 add chain (latency)", k_probe<1>, blocks, 64, 64);
    run("1 dep f64 mul chain (latency)", k_probe<2>, blocks, 64, 64);
    run("8 indep f64 mul chains", k_probe<3>, blocks, 64, 64);
    run("8 indep f32 add chains", k_probe<4>, blocks, 64, 64);
  }
  for (int blocks : {1, 64, 256, 512, 1024, 2048}) {
    hipLaunchKernelGGL(k_df2t, dim3(blocks), dim3(64), 0, 0, out, cyc, iters, coef);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_df2t, dim3(blocks), dim3(64), 0, 0, out, cyc, iters, coef);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(c, cyc, 8 * blocks, hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < blocks; ++i) avg += c[i];
    avg /= blocks;
    printf("df2t 9-tap step: blocks=%4d cycles/sample=%7.1f  wall=%.3f ms  ns/sample=%.2f  eff clock=%.2f GHz\n",
           blocks, avg / iters / 16, ms, ms * 1e6 / (iters * 16.0), avg / (ms * 1e6));
  }
  return 0;
}
