// step_probe2.hip -- cycles per sample of candidate lane layouts for the
// DF-II-T recurrences (operands in registers, no memory traffic):
//   0  quad 9-tap (current K1q: lane j owns z[2j], z[2j+1])
//   1  row16 9-tap (lane 8+j owns z[j]; y by v_mov_b64 row_newbcast:8,
//      z[j+1] by row_shl:1, the top lane's out-of-row read keeps -0.0)
//   2  pair 5-tap (current K2/K3)
//   3  quad 5-tap (lane j owns z[j]; top-lane zero by a multiply)
//   4  row16 5-tap (lane 12+j owns z[j])
//   5  row16 9-tap, z0 replicated in every lane (lane 8+j owns z[j+1]): y is
//      computed by every lane, so the recurrence chain is add -> mul -> sub
//      with the two DPP moves (z1 broadcast, z[j+2] shift) off the chain
//   6  quad 5-tap, z0 replicated (lane j owns z[j+1])
//   7  8-lane group 9-tap (8 streams per wave): y by two v_mov_b64 row_newbcast
//      (:0 into banks 0-1, :8 into banks 2-3), z[j+1] by row_shl:1 times a 0/1
//      factor (the group's top lane)
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/step_probe2.hip -o tools/step_probe2
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
template <int LANE>
__device__ __forceinline__ double bcast16(double v) {   // v_mov_b64_dpp row_newbcast
  const long u = __builtin_bit_cast(long, v);
  const long r = __builtin_amdgcn_update_dpp(0L, u, 0x150 + LANE, 0xF, 0xF, true);
  return __builtin_bit_cast(double, r);
}
// z[j+1] from the next lane of the row; the last lane of the row keeps the
// previous hi word of its destination (-0.0's 0x80000000) and gets lo = 0
__device__ __forceinline__ double shl1(double v, int& hi_keep) {
  const long long u = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(u & 0xffffffff), 0x101, 0xF, 0xF, true);
  hi_keep = __builtin_amdgcn_update_dpp(hi_keep, (int)(u >> 32), 0x101, 0xF, 0xF, false);
  return __builtin_bit_cast(double, ((long long)hi_keep << 32) | (unsigned)lo);
}

template <int MODE>
__global__ __launch_bounds__(256) void k(double* out, unsigned long long* cyc, int iters, const double* co) {
  const int lane = threadIdx.x & 63;
  const int j4 = lane & 3, j2 = lane & 1, j16 = lane & 15;
  double zA = 0.01 * lane, zB = 0.02 * lane;
  double xs[16], acc = 0;
  for (int i = 0; i < 16; ++i) xs[i] = 0.3 + lane * 1e-3 + i * 0.01;
  double cAb, cAa, cBb, cBa, b0 = co[0], cm = 1.0;
  int hik = (int)0x80000000;
  if (MODE == 0) { cAb = co[2 * j4 + 1]; cAa = co[9 + 2 * j4 + 1]; cBb = co[2 * j4 + 2]; cBa = co[9 + 2 * j4 + 2]; }
  else if (MODE == 1) { const int jj = j16 >= 8 ? j16 - 8 : 0; cAb = co[jj + 1]; cAa = co[10 + jj]; cBb = cBa = 0; }
  else if (MODE == 2) { cAb = co[2 * j2 + 1]; cAa = co[9 + 2 * j2 + 1]; cBb = co[2 * j2 + 2]; cBa = co[9 + 2 * j2 + 2]; }
  else if (MODE == 3) { cAb = co[j4 + 1]; cAa = co[10 + j4]; cBb = cBa = 0; cm = j4 == 3 ? 0.0 : 1.0; }
  else if (MODE == 4) { const int jj = j16 >= 12 ? j16 - 12 : 0; cAb = co[jj + 1]; cAa = co[10 + jj]; cBb = cBa = 0; }
  else if (MODE == 5) { const int jj = j16 >= 8 ? j16 - 8 : 0; cAb = co[jj + 2]; cAa = co[11 + jj]; cBb = co[1]; cBa = co[10]; }
  else if (MODE == 6) { cAb = co[j4 + 2]; cAa = co[11 + j4]; cBb = co[1]; cBa = co[10]; cm = j4 == 3 ? 0.0 : 1.0; }
  else { const int j8 = lane & 7; cAb = co[j8 + 1]; cAa = co[10 + j8]; cBb = cBa = 0; cm = j8 == 7 ? 0.0 : 1.0; }
  double z0r = 0.05;
  const bool top4 = j4 == 3, top2 = j2 == 1;
  unsigned long long t0 = now();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      double y;
      asm volatile("" : "+v"(xs[s]));
      const double x = xs[s];
      if (MODE == 0) {
        const double t = zA + b0 * x;
        y = dpp_f64<0x00>(t);
        double zC = dpp_f64<0xF9>(zA);
        zC = top4 ? -0.0 : zC;
        const double nA = (zB + x * cAb) - y * cAa;
        const double nB = (zC + x * cBb) - y * cBa;
        zA = nA; zB = nB;
      } else if (MODE == 2) {
        const double t = zA + b0 * x;
        y = dpp_f64<0xA0>(t);
        double zC = dpp_f64<0xF5>(zA);
        zC = top2 ? -0.0 : zC;
        const double nA = (zB + x * cAb) - y * cAa;
        const double nB = (zC + x * cBb) - y * cBa;
        zA = nA; zB = nB;
      } else if (MODE == 1 || MODE == 4) {
        const double t = zA + b0 * x;
        y = MODE == 1 ? bcast16<8>(t) : bcast16<12>(t);
        const double zC = shl1(zA, hik);
        zA = (zC + x * cAb) - y * cAa;
      } else if (MODE == 3) {
        const double t = zA + b0 * x;
        y = dpp_f64<0x00>(t);
        const double zC = dpp_f64<0xF9>(zA) * cm;
        zA = (zC + x * cAb) - y * cAa;
      } else if (MODE == 5) {
        y = z0r + b0 * x;
        const double z1b = bcast16<8>(zA);
        const double zC = shl1(zA, hik);
        z0r = (z1b + x * cBb) - y * cBa;
        zA = (zC + x * cAb) - y * cAa;
      } else if (MODE == 7) {
        const double t = zA + b0 * x;
        const long u = __builtin_bit_cast(long, t);
        long r = __builtin_amdgcn_update_dpp(0L, u, 0x150, 0xF, 0x3, false);   // row_newbcast:0, banks 0-1
        r = __builtin_amdgcn_update_dpp(r, u, 0x158, 0xF, 0xC, false);          // row_newbcast:8, banks 2-3
        y = __builtin_bit_cast(double, r);
        const double zC = shl1(zA, hik) * cm;
        zA = (zC + x * cAb) - y * cAa;
      } else {
        y = z0r + b0 * x;
        const double z1b = dpp_f64<0x00>(zA);
        const double zC = dpp_f64<0xF9>(zA) * cm;
        z0r = (z1b + x * cBb) - y * cBa;
        zA = (zC + x * cAb) - y * cAa;
      }
      acc += y;
    }
  }
  unsigned long long t1 = now();
  out[blockIdx.x * 256 + threadIdx.x] = acc + zA + zB + z0r;
  if (lane == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

int main() {
  double *out, *co;
  unsigned long long* cyc;
  (void)hipMalloc(&out, 8192 * 64 * 8);
  (void)hipMalloc(&cyc, 8192 * 8);
  (void)hipMalloc(&co, 18 * 8);
  double h[18] = {0.031, 0, -0.12, 0, 0.187, 0, -0.12, 0, 0.031, 1, -3.9, 7.1, -7.9, 5.9, -2.9, 0.9, -0.2, 0.02};
  (void)hipMemcpy(co, h, sizeof(h), hipMemcpyHostToDevice);
  static unsigned long long c[8192];
  const int iters = 1000;
  const char* names[] = {"quad 9-tap (K1q)", "row16 9-tap", "pair 5-tap (K2/K3)", "quad 5-tap", "row16 5-tap",
                         "row16 9-tap z0-rep", "quad 5-tap z0-rep", "group8 9-tap"};
  void (*ks[])(double*, unsigned long long*, int, const double*) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>, k<7>};
  for (int m = 0; m < 8; ++m)
    for (int waves : {512, 1024, 2048, 3072}) {
      const int blocks = waves / 4;
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0);
      (void)hipEventCreate(&e1);
      hipLaunchKernelGGL(ks[m], dim3(blocks), dim3(256), 0, 0, out, cyc, iters, co);
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0, 0);
      hipLaunchKernelGGL(ks[m], dim3(blocks), dim3(256), 0, 0, out, cyc, iters, co);
      (void)hipEventRecord(e1, 0);
      (void)hipDeviceSynchronize();
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      (void)hipMemcpy(c, cyc, 8 * waves, hipMemcpyDeviceToHost);
      double avg = 0;
      for (int i = 0; i < waves; ++i) avg += c[i];
      printf("%-20s waves=%5d cycles/sample=%6.1f  wall ns/sample=%6.2f\n", names[m], waves,
             avg / waves / iters / 16, ms * 1e6 / iters / 16);
    }
  return 0;
}
