// xcd_exchange_probe.hip -- VERDICT r5 item 3: what one all-to-all exchange
// of a 96000-point complex transform costs when it stays inside one XCD (its
// 4 MiB L2) instead of going through HBM.
//
// 256 workgroups of 256 threads (one per CU: all resident), each reads its
// XCD id (HW_REG_XCC_ID) and takes a rank inside its XCD; the XCD's 32
// workgroups form G-workgroup groups (G = 32: one transform per XCD at a time,
// G = 16: two), each group owning a 1.5 MB scratch (96000 x 16 B).  One PASS
// = every workgroup writes its 1/G slice of the scratch, a group barrier
// (release fence, per-group counter, bounded s_sleep poll, acquire fence),
// every workgroup reads 1/G of EVERY other slice (the four-step transform's
// transpose, 1.5 KB runs), a second barrier.  Timed with s_memrealtime
// (100 MHz) over R passes; no FFT arithmetic, so this is a floor for the
// exchange half of an on-die transform.  Every spin is bounded (a timed-out
// wait sets a flag and the kernel still ends).
// hipcc --offload-arch=gfx950 -O3 tools/xcd_exchange_probe.hip -o tools/xcd_exchange_probe.bin
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kN = 96000;        // complex points per transform
constexpr int kThreads = 256;
constexpr int kWgs = 256;
constexpr int kRounds = 200;

__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 7;
}
__device__ __forceinline__ unsigned long long rt() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

// group barrier number `gen` (1, 2, ...): counter reaches gen * members
__device__ void group_barrier(unsigned* cnt, unsigned target, unsigned* timeout) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    atomicAdd(cnt, 1u);
    unsigned spins = 0;
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 24)) {
        atomicOr(timeout, 1u);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

template <int G, bool DATA>
__global__ __launch_bounds__(kThreads) void k(double2* scratch, unsigned* ctl, unsigned long long* out) {
  // ctl: [0..7] per-XCD rank counters, [8] arrivals, [9] timeout, [16 + g] group counters
  __shared__ unsigned s_rank, s_x;
  if (threadIdx.x == 0) {
    s_x = xcc_id();
    s_rank = atomicAdd(&ctl[s_x], 1u);
    // every workgroup placed before anyone reads the per-XCD counts
    atomicAdd(&ctl[8], 1u);
    unsigned spins = 0;
    while (__hip_atomic_load(&ctl[8], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)kWgs) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 24)) {
        atomicOr(&ctl[9], 1u);
        break;
      }
    }
  }
  __syncthreads();
  const unsigned x = s_x, rank = s_rank;
  const unsigned on_x = __hip_atomic_load(&ctl[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // groups of G by rank; a partial last group (placement not 32 per XCD) sizes itself
  const unsigned grp = rank / G, first = grp * G;
  const unsigned members = on_x - first < (unsigned)G ? on_x - first : (unsigned)G;
  const unsigned me = rank - first;
  const unsigned gid = x * 32 + grp;                       // < 8 * 32 groups
  double2* buf = scratch + (size_t)gid * kN;
  unsigned* cnt = &ctl[16 + gid];
  const int slice = (kN + members - 1) / members;          // elements per member slice
  const int sub = (slice + members - 1) / members;         // elements of each slice a member reads
  double acc = 0.0;
  const unsigned long long t0 = rt();
  for (int r = 0; r < kRounds; ++r) {
    // write my slice
    const int lo = me * slice, hi = lo + slice < kN ? lo + slice : kN;
    if (DATA)
      for (int i = lo + threadIdx.x; i < hi; i += kThreads) buf[i] = make_double2(r + i, acc);
    group_barrier(cnt, (2 * r + 1) * members, &ctl[9]);
    // read 1/members of every slice (the transpose): (slice q, offset t)
    // pairs spread over the threads, every load issued before any is used
    if (DATA) {
      const int total = (int)members * sub;
      for (int base = 0; base < total; base += 16 * kThreads) {
        double v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int kk = base + threadIdx.x + j * kThreads;
          const int q = kk / sub, t = kk - q * sub;
          const int idx = q * slice + (int)me * sub + t;
          v[j] = kk < total && idx < kN ? buf[idx].x : 0.0;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) acc += v[j];
      }
    }
    group_barrier(cnt, (2 * r + 2) * members, &ctl[9]);
  }
  const unsigned long long t1 = rt();
  if (threadIdx.x == 0) {
    out[blockIdx.x * 4 + 0] = t1 - t0;
    out[blockIdx.x * 4 + 1] = x;
    out[blockIdx.x * 4 + 2] = members;
  }
  if (acc == -1.0) out[blockIdx.x * 4 + 3] = 1;            // keep the reads
}

template <int G, bool DATA>
void run(double2* scratch, unsigned* ctl, unsigned long long* out) {
  (void)hipMemset(ctl, 0, 4096);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL((k<G, DATA>), dim3(kWgs), dim3(kThreads), 0, 0, scratch, ctl, out);
  (void)hipEventRecord(e1, 0);
  (void)hipDeviceSynchronize();
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  static unsigned long long h[kWgs * 4];
  unsigned hc[16];
  (void)hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
  (void)hipMemcpy(hc, ctl, sizeof(hc), hipMemcpyDeviceToHost);
  double mx = 0, mean = 0;
  int per_x[8] = {0};
  for (int i = 0; i < kWgs; ++i) {
    const double us = h[i * 4] / 100.0;   // s_memrealtime: 100 MHz
    mx = us > mx ? us : mx;
    mean += us / kWgs;
    per_x[h[i * 4 + 1] & 7]++;
  }
  printf("G=%2d (transforms in flight per XCD: %d) %s  workgroups per XCD:", G, 32 / G, DATA ? "exchange" : "barriers only");
  for (int i = 0; i < 8; ++i) printf(" %d", per_x[i]);
  printf("  timeout=%u\n", hc[9]);
  printf("   %d passes: %.1f us (kernel %.1f us); per pass (write slice + barrier + transpose read + barrier) %.2f us;"
         " per-XCD L2 traffic per pass %.2f MB (x %d groups)\n",
         kRounds, mx, ms * 1e3, mx / kRounds, 2.0 * kN * 16 / 1e6, 32 / G);
  (void)mean;
}

int main() {
  double2* scratch;
  unsigned* ctl;
  unsigned long long* out;
  (void)hipMalloc(&scratch, (size_t)256 * kN * sizeof(double2));
  (void)hipMalloc(&ctl, 4096);
  (void)hipMalloc(&out, kWgs * 4 * 8);
  run<32, false>(scratch, ctl, out);
  run<32, true>(scratch, ctl, out);
  run<16, false>(scratch, ctl, out);
  run<16, true>(scratch, ctl, out);
  run<8, true>(scratch, ctl, out);
  run<32, true>(scratch, ctl, out);
  return 0;
}
