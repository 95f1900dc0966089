// FP64 VALU issue probe (tools/, not part of the library): how many FP64
// wave-instructions per cycle does one SIMD retire at 1, 2, 3, 4 waves per
// SIMD, for (a) independent mul/add streams and (b) the DF-II-T band-pass
// step (psk_lane_kernels.hip df2t_step_zo: 23 FP64 with a 3-deep chain).
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/fp64_probe.hip -o tools/fp64_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_indep(double* out, int iters, double a, double b) {
  double r[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) r[j] = threadIdx.x * 1e-3 + j;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 16; ++j) r[j] = (j & 1) ? r[j] * a : r[j] + b;
  }
  double s = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) s += r[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_df2t(double* out, int iters, const double* cf) {
  double b0 = cf[0], b2 = cf[2], b4 = cf[4];
  double a1 = cf[9], a2 = cf[10], a3 = cf[11], a4 = cf[12], a5 = cf[13], a6 = cf[14], a7 = cf[15], a8 = cf[16];
  double z[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = 0.0;
  double x = threadIdx.x * 1e-3;
  for (int i = 0; i < iters; ++i) {
    const double p0 = b0 * x, p2 = x * b2, p4 = x * b4;
    const double y = z[0] + p0;
    z[0] = z[1] - y * a1;
    z[1] = (z[2] + p2) - y * a2;
    z[2] = z[3] - y * a3;
    z[3] = (z[4] + p4) - y * a4;
    z[4] = z[5] - y * a5;
    z[5] = (z[6] + p2) - y * a6;
    z[6] = z[7] - y * a7;
    z[7] = p0 - y * a8;
    x = y * 0.5;
  }
  double s = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += z[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  int dev = 0, cus = 0, clk = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
  double* out;
  double* cf;
  hipMalloc(&out, (size_t)cus * 1024 * 8 * 4);
  hipMalloc(&cf, 32 * 8);
  double h[32];
  for (int i = 0; i < 32; ++i) h[i] = 0.01 * (i + 1) / (i + 3);
  hipMemcpy(cf, h, sizeof h, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  std::printf("CUs %d, clock %d kHz\n", cus, clk);
  for (int kind = 0; kind < 2; ++kind) {
    for (int wps : {1, 2, 3, 4, 6, 8}) {
      const int block = 256;                       // 4 waves: one per SIMD
      const int grid = cus * wps;                  // wps workgroups per CU -> wps waves per SIMD
      const int iters = kind == 0 ? 20000 : 40000;
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        if (kind == 0) hipLaunchKernelGGL(k_indep, dim3(grid), dim3(block), 0, 0, out, iters, 1.0000001, 1e-9);
        else hipLaunchKernelGGL(k_df2t, dim3(grid), dim3(block), 0, 0, out, iters, cf);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
      }
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double per_wave = kind == 0 ? 16.0 : 24.0;   // FP64 instr per iteration (df2t: 23 + the x update)
      const double wave_instr = (double)grid * 4 * iters * per_wave;
      const double simd_instr_per_s = wave_instr / (ms * 1e-3) / (cus * 4.0);
      std::printf("%s waves/SIMD %d: %.3f ms, %.2f G wave-instr/s per SIMD, %.2f cycles per FP64 wave-instr at %.2f GHz, %.1f TFLOP-ops/s\n",
                  kind == 0 ? "indep" : "df2t ", wps, ms, simd_instr_per_s / 1e9, clk * 1e3 / simd_instr_per_s, clk / 1e6,
                  wave_instr * 64 / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
