// Wave placement probe (tools/, not part of the library): where do the waves
// of multi-wave workgroups land?  Each wave spins ~1 ms (so a launch's waves
// are co-resident) and records HW_ID (SIMD, CU, SE) and XCC_ID; the host
// prints, per launch shape, the histogram of waves per SIMD over the
// (XCC, SE, CU) slots that hold any wave, and whether one workgroup's waves
// share a SIMD.
//   hipcc -O3 --offload-arch=gfx950 tools/placement_probe.hip -o tools/placement_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <tuple>
#include <vector>

__global__ void k_place(uint32_t* rec, long long spin) {
  extern __shared__ char lds[];
  if (threadIdx.x == 0) lds[0] = 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_REG_HW_ID
  const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < spin) {
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    const size_t i = ((size_t)blockIdx.x * (blockDim.x >> 6) + w) * 2;
    rec[i] = hw;
    rec[i + 1] = xcc;
  }
}

int main() {
  struct Shape { int threads, blocks, lds; const char* what; };
  const Shape shapes[] = {
      {256, 256, 0, "256-thread WGs, 1 per CU"},
      {256, 512, 0, "256-thread WGs, 2 per CU"},
      {256, 512, 65536, "256-thread WGs with 64 KB LDS, 2 per CU (k_bp_lane2 GPB=2)"},
      {64, 1024, 0, "64-thread WGs, 4 per CU"},
      {128, 1024, 0, "128-thread WGs, 4 per CU"},
  };
  uint32_t* rec;
  hipMalloc(&rec, 4096 * 64 * 8);
  for (const Shape& sh : shapes) {
    const int waves = sh.blocks * (sh.threads / 64);
    hipMemset(rec, 0xFF, (size_t)waves * 8);
    hipLaunchKernelGGL(k_place, dim3(sh.blocks), dim3(sh.threads), sh.lds, 0, rec, 100000LL);   // ~1 ms at 100 MHz
    hipDeviceSynchronize();
    std::vector<uint32_t> h((size_t)waves * 2);
    hipMemcpy(h.data(), rec, h.size() * 4, hipMemcpyDeviceToHost);
    std::map<std::tuple<int, int, int, int>, int> per_simd;   // (xcc, se, cu, simd) -> waves
    std::map<std::tuple<int, int, int>, int> per_cu;
    int same = 0, wgs = 0;
    const int wpb = sh.threads / 64;
    for (int b = 0; b < sh.blocks; ++b) {
      std::map<int, int> simds;
      for (int w = 0; w < wpb; ++w) {
        const uint32_t hw = h[((size_t)b * wpb + w) * 2], xcc = h[((size_t)b * wpb + w) * 2 + 1] & 0xF;
        const int simd = (hw >> 4) & 3, cu = (hw >> 8) & 15, se = (hw >> 13) & 7;
        per_simd[{(int)xcc, se, cu, simd}]++;
        per_cu[{(int)xcc, se, cu}]++;
        simds[simd]++;
      }
      ++wgs;
      if (wpb > 1 && (int)simds.size() < wpb) ++same;
    }
    std::map<int, int> hist;        // waves on a SIMD -> number of SIMDs (over CUs with waves)
    for (auto& [cu, n] : per_cu) {
      for (int s = 0; s < 4; ++s) {
        auto it = per_simd.find({std::get<0>(cu), std::get<1>(cu), std::get<2>(cu), s});
        hist[it == per_simd.end() ? 0 : it->second]++;
      }
    }
    // do the workgroups sharing a CU put their wave i on the same SIMD?
    std::map<std::tuple<int, int, int>, std::vector<std::vector<int>>> cu_maps;
    for (int b = 0; b < sh.blocks; ++b) {
      std::vector<int> m;
      std::tuple<int, int, int> key;
      for (int w = 0; w < wpb; ++w) {
        const uint32_t hw = h[((size_t)b * wpb + w) * 2], xcc = h[((size_t)b * wpb + w) * 2 + 1] & 0xF;
        key = {(int)xcc, (int)((hw >> 13) & 7), (int)((hw >> 8) & 15)};
        m.push_back((hw >> 4) & 3);
      }
      cu_maps[key].push_back(m);
    }
    int aligned = 0, multi = 0;
    for (auto& [k, v] : cu_maps) {
      if (v.size() < 2) continue;
      ++multi;
      bool all = true;
      for (size_t j = 1; j < v.size(); ++j) all = all && v[j] == v[0];
      aligned += all;
    }
    std::printf("%-62s CUs with >1 WG: %d, of them wave i on the same SIMD in every WG: %d; first map:", sh.what,
                multi, aligned);
    for (int x : cu_maps.begin()->second[0]) std::printf(" %d", x);
    std::printf("\n");
    if (wpb == 4) {   // k_bp_lane2's roles (role = wave & 1): SIMDs by busy (role 0) waves in the forward phase
      std::map<std::tuple<int, int, int, int>, int> busy;
      for (int b = 0; b < sh.blocks; ++b)
        for (int w = 0; w < wpb; w += 2) {
          const uint32_t hw = h[((size_t)b * wpb + w) * 2], xcc = h[((size_t)b * wpb + w) * 2 + 1] & 0xF;
          busy[{(int)xcc, (int)((hw >> 13) & 7), (int)((hw >> 8) & 15), (int)((hw >> 4) & 3)}]++;
        }
      std::map<int, int> bh;
      for (auto& [cu, n] : per_cu)
        for (int s2 = 0; s2 < 4; ++s2) {
          auto it = busy.find({std::get<0>(cu), std::get<1>(cu), std::get<2>(cu), s2});
          bh[it == busy.end() ? 0 : it->second]++;
        }
      std::printf("%-62s forward phase, SIMDs by role-0 waves:", sh.what);
      for (auto& [k, v] : bh) std::printf(" %d:%d", k, v);
      std::printf("\n");
    }
    std::printf("%-62s CUs used %zu; SIMDs by waves held:", sh.what, per_cu.size());
    for (auto& [k, v] : hist) std::printf(" %d:%d", k, v);
    std::printf("; WGs with waves sharing a SIMD %d/%d\n", same, wgs);
  }
  return 0;
}
