// step_probe3.hip -- throughput of lane-efficient DF-II-T layouts (operands in
// registers, no memory traffic), against the round-1 state-per-lane ones.
//   0  lane = stream, 9-tap, every tap computed (33 FP64 / sample)
//   1  lane = stream, 9-tap, zero odd taps skipped + zero detector (25 FP64 + 2)
//   2  2 lanes = stream, 9-tap, 4 states per lane (y quad_perm[0,0,2,2],
//      z[4] quad_perm[1,1,3,3] + top-lane select)
//   3  4 lanes = stream, 9-tap, 2 states per lane
//   4  lane = component, 5-tap + mixer (17 + 1 FP64), LO wave-uniform
//   5  2 lanes = component, 5-tap, 2 states per lane + mixer
//   6  group8 9-tap (round-1 K1g)
//   7  quad 5-tap (round-1 K2q)
// Reported: cycles per sample per wave and stream-samples per ns of the whole
// launch (streams per wave x waves / wall ns per sample).
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/step_probe3.hip -o tools/step_probe3
#include <hip/hip_runtime.h>

#include <cstdio>

struct Co {
  double b[9], a[9];
};

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
__device__ __forceinline__ float tiny_min3(float acc, double a, double b) {
  const float ha = __builtin_bit_cast(float, (unsigned)(__builtin_bit_cast(unsigned long long, a) >> 32));
  const float hb = __builtin_bit_cast(float, (unsigned)(__builtin_bit_cast(unsigned long long, b) >> 32));
  float r;
  asm("v_min3_f32 %0, %1, |%2|, |%3|" : "=v"(r) : "v"(acc), "v"(ha), "v"(hb));
  return r;
}
template <int N>
__device__ __forceinline__ double sel(bool c, double a, double b) { return c ? a : b; }

constexpr int kSpw[8] = {64, 64, 32, 16, 64, 32, 8, 16};   // streams (or components) per wave

template <int MODE>
__global__ __launch_bounds__(256) void k(double* out, unsigned long long* cyc, int iters, Co co, const double* cv) {
  const int lane = threadIdx.x & 63;
  double xs[16], acc = 0;
  for (int i = 0; i < 16; ++i) xs[i] = 0.3 + lane * 1e-3 + i * 0.01;
  double z[8];
  for (int i = 0; i < 8; ++i) z[i] = 0.01 * (lane + i);
  float det = __builtin_inff();
  // per-lane coefficients for the split layouts
  const int p2 = lane & 1, p4 = lane & 3;
  double cb[4], ca[4];
  for (int i = 0; i < 4; ++i) {
    if (MODE == 2) { cb[i] = cv[4 * p2 + i + 1]; ca[i] = cv[9 + 4 * p2 + i + 1]; }
    else if (MODE == 3) { cb[i] = cv[(2 * p4 + i + 1) % 9]; ca[i] = cv[9 + (2 * p4 + i + 1) % 9]; }
    else if (MODE == 5) { cb[i] = cv[(2 * p2 + i + 1) % 5]; ca[i] = cv[9 + (2 * p2 + i + 1) % 5]; }
    else if (MODE == 6) { cb[i] = cv[(lane & 7) + 1]; ca[i] = cv[9 + (lane & 7) + 1]; }
    else if (MODE == 7) { cb[i] = cv[p4 + 1]; ca[i] = cv[9 + p4 + 1]; }
    else { cb[i] = 0; ca[i] = 0; }
  }
  const bool top2 = p2 == 1, top4 = p4 == 3, top8 = (lane & 7) == 7;
  const double cm4 = top4 ? 0.0 : 1.0;
  const double lo = cv[3] * 0.5;
  unsigned long long t0 = now();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      asm volatile("" : "+v"(xs[s]));
      double x = xs[s];
      double y;
      if (MODE == 0) {
        y = z[0] + co.b[0] * x;
#pragma unroll
        for (int i = 0; i < 7; ++i) z[i] = (z[i + 1] + x * co.b[i + 1]) - y * co.a[i + 1];
        z[7] = (-0.0 + x * co.b[8]) - y * co.a[8];
      } else if (MODE == 1) {
        y = z[0] + co.b[0] * x;
        det = tiny_min3(det, z[1], z[3]);
        det = tiny_min3(det, z[5], z[7]);
        z[0] = z[1] - y * co.a[1];
        z[1] = (z[2] + x * co.b[2]) - y * co.a[2];
        z[2] = z[3] - y * co.a[3];
        z[3] = (z[4] + x * co.b[4]) - y * co.a[4];
        z[4] = z[5] - y * co.a[5];
        z[5] = (z[6] + x * co.b[6]) - y * co.a[6];
        z[6] = z[7] - y * co.a[7];
        z[7] = x * co.b[8] - y * co.a[8];
      } else if (MODE == 2) {
        const double t = z[0] + co.b[0] * x;
        y = dpp_f64<0xA0>(t);                     // quad_perm [0,0,2,2]
        double zC = dpp_f64<0xF5>(z[0]);          // quad_perm [1,1,3,3]
        zC = top2 ? -0.0 : zC;
        z[0] = (z[1] + x * cb[0]) - y * ca[0];
        z[1] = (z[2] + x * cb[1]) - y * ca[1];
        z[2] = (z[3] + x * cb[2]) - y * ca[2];
        z[3] = (zC + x * cb[3]) - y * ca[3];
      } else if (MODE == 3) {
        const double t = z[0] + co.b[0] * x;
        y = dpp_f64<0x00>(t);                     // quad_perm [0,0,0,0]
        double zC = dpp_f64<0xF9>(z[0]);          // quad_perm [1,2,3,3]
        zC = top4 ? -0.0 : zC;
        z[0] = (z[1] + x * cb[0]) - y * ca[0];
        z[1] = (zC + x * cb[1]) - y * ca[1];
      } else if (MODE == 4) {
        const double e = x * lo;
        y = z[0] + co.b[0] * e;
        z[0] = (z[1] + e * co.b[1]) - y * co.a[1];
        z[1] = (z[2] + e * co.b[2]) - y * co.a[2];
        z[2] = (z[3] + e * co.b[3]) - y * co.a[3];
        z[3] = e * co.b[4] - y * co.a[4];
        det = tiny_min3(det, e, y);
      } else if (MODE == 5) {
        const double e = x * lo;
        const double t = z[0] + co.b[0] * e;
        y = dpp_f64<0xA0>(t);
        double zC = dpp_f64<0xF5>(z[0]);
        zC = top2 ? -0.0 : zC;
        z[0] = (z[1] + e * cb[0]) - y * ca[0];
        z[1] = (zC + e * cb[1]) - y * ca[1];
        det = tiny_min3(det, e, y);
      } else if (MODE == 6) {
        const double t = z[0] + co.b[0] * x;
        const long u = __builtin_bit_cast(long, t);
        long r = __builtin_amdgcn_update_dpp(0L, u, 0x150, 0xF, 0x3, false);
        r = __builtin_amdgcn_update_dpp(r, u, 0x158, 0xF, 0xC, false);
        y = __builtin_bit_cast(double, r);
        const long long zu = __builtin_bit_cast(long long, z[0]);
        int l0 = __builtin_amdgcn_update_dpp(0, (int)(zu & 0xffffffff), 0x101, 0xF, 0xF, true);
        int h0 = __builtin_amdgcn_update_dpp(0, (int)(zu >> 32), 0x101, 0xF, 0xF, true);
        l0 = top8 ? 0 : l0;
        h0 = top8 ? (int)0x80000000 : h0;
        const double zC = __builtin_bit_cast(double, ((long long)h0 << 32) | (unsigned)l0);
        z[0] = (zC + x * cb[0]) - y * ca[0];
      } else {
        const double e = x * lo;
        const double t = z[0] + co.b[0] * e;
        y = dpp_f64<0x00>(t);
        const double zC = dpp_f64<0xF9>(z[0]) * cm4;
        z[0] = (zC + e * cb[0]) - y * ca[0];
        det = tiny_min3(det, e, y);
      }
      acc += y;
    }
  }
  unsigned long long t1 = now();
  double zs = 0;
  for (int i = 0; i < 8; ++i) zs += z[i];
  out[blockIdx.x * 256 + threadIdx.x] = acc + zs + det;
  if (lane == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

int main() {
  double *out, *cv;
  unsigned long long* cyc;
  (void)hipMalloc(&out, 16384 * 64 * 8);
  (void)hipMalloc(&cyc, 16384 * 8);
  (void)hipMalloc(&cv, 18 * 8);
  Co co;
  double h[18] = {0.031, 0, -0.12, 0, 0.187, 0, -0.12, 0, 0.031, 1, -3.9, 7.1, -7.9, 5.9, -2.9, 0.9, -0.2, 0.02};
  for (int i = 0; i < 9; ++i) { co.b[i] = h[i]; co.a[i] = h[9 + i]; }
  (void)hipMemcpy(cv, h, sizeof(h), hipMemcpyHostToDevice);
  static unsigned long long c[16384];
  const int iters = 400;
  const char* names[] = {"lane 9-tap full", "lane 9-tap zskip", "2-lane 9-tap", "4-lane 9-tap",
                         "lane 5-tap+mix", "2-lane 5-tap+mix", "group8 9-tap (K1g)", "quad 5-tap (K2q)"};
  void (*ks[])(double*, unsigned long long*, int, Co, const double*) = {k<0>, k<1>, k<2>, k<3>,
                                                                        k<4>, k<5>, k<6>, k<7>};
  for (int m = 0; m < 8; ++m)
    for (int waves : {256, 1024, 2048, 4096}) {
      const int blocks = waves / 4;
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0);
      (void)hipEventCreate(&e1);
      hipLaunchKernelGGL(ks[m], dim3(blocks), dim3(256), 0, 0, out, cyc, iters, co, cv);
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0, 0);
      hipLaunchKernelGGL(ks[m], dim3(blocks), dim3(256), 0, 0, out, cyc, iters, co, cv);
      (void)hipEventRecord(e1, 0);
      (void)hipDeviceSynchronize();
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      (void)hipMemcpy(c, cyc, 8 * waves, hipMemcpyDeviceToHost);
      double avg = 0;
      for (int i = 0; i < waves; ++i) avg += c[i];
      const double ns = ms * 1e6 / iters / 16;
      printf("%-22s waves=%5d cycles/sample/wave=%6.1f  stream-samples/ns=%7.1f\n", names[m], waves,
             avg / waves / iters / 16, (double)waves * kSpw[m] / ns);
    }
  return 0;
}
