// pocketfft_dev.h -- device restatement of pocketfft's transforms (plans:
// pocketfft.h), bit for bit: every butterfly evaluates pocketfft's expressions
// in its order, without contraction (-ffp-contract=off), so the results equal
// scipy.fft's (oracle/amr_pocketfft.c is the CPU statement of the same
// algorithm, pinned against scipy; tests/test_gpu_pocketfft.py pins these).
//
// Each routine is run by ONE whole workgroup.  Pass by pass over global
// scratch: a pass spreads its independent butterflies (pocketfft's (k, i)
// loop nests) over the workgroup's threads, passes are separated by barriers,
// and the generic passes (radfg / radbg / passg) run their phases between
// barriers, each thread owning the accumulation chains of its outputs (so
// their order is pocketfft's).  Fused (the plans' groups, pocketfft.h): runs
// of consecutive passes go through LDS tiles that are closed under those
// passes' data flow -- cgroup (complex), rfftp_fwd_fused's blocks and
// rgroup_pairs' residue-pair tiles (real forward) -- calling the same
// butterflies, so every value is computed by the same operations.  Every
// thread of the workgroup must call these.
//
// Derived from pocketfft (the FFT library bundled with scipy 1.15.3 as
// scipy.fft's pypocketfft), whose notice follows; the FFTPACK algorithms it
// implements are by Paul N. Swarztrauber (public domain).
//
//   Copyright (C) 2010-2019 Max-Planck-Society
//   All rights reserved.
//
//   Redistribution and use in source and binary forms, with or without
//   modification, are permitted provided that the following conditions are met:
//
//   * Redistributions of source code must retain the above copyright notice,
//     this list of conditions and the following disclaimer.
//   * Redistributions in binary form must reproduce the above copyright notice,
//     this list of conditions and the following disclaimer in the documentation
//     and/or other materials provided with the distribution.
//   * Neither the name of the copyright holder nor the names of its contributors
//     may be used to endorse or promote products derived from this software
//     without specific prior written permission.
//
//   THIS SOFTWARE IS PROVIDED BY THE COPYRIGHT HOLDERS AND CONTRIBUTORS "AS IS"
//   AND ANY EXPRESS OR IMPLIED WARRANTIES, INCLUDING, BUT NOT LIMITED TO, THE
//   IMPLIED WARRANTIES OF MERCHANTABILITY AND FITNESS FOR A PARTICULAR PURPOSE ARE
//   DISCLAIMED. IN NO EVENT SHALL THE COPYRIGHT HOLDER OR CONTRIBUTORS BE LIABLE
//   FOR ANY DIRECT, INDIRECT, INCIDENTAL, SPECIAL, EXEMPLARY, OR CONSEQUENTIAL
//   DAMAGES (INCLUDING, BUT NOT LIMITED TO, PROCUREMENT OF SUBSTITUTE GOODS OR
//   SERVICES; LOSS OF USE, DATA, OR PROFITS; OR BUSINESS INTERRUPTION) HOWEVER
//   CAUSED AND ON ANY THEORY OF LIABILITY, WHETHER IN CONTRACT, STRICT LIABILITY,
//   OR TORT (INCLUDING NEGLIGENCE OR OTHERWISE) ARISING IN ANY WAY OUT OF THE USE
//   OF THIS SOFTWARE, EVEN IF ADVISED OF THE POSSIBILITY OF SUCH DAMAGE.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "pocketfft.h"

namespace amr {
namespace pf {

// 16-byte aligned: LDS and global accesses as one b128 / dwordx4 each (every
// complex array the routines touch starts on a 16-byte boundary: pf_even)
struct alignas(16) Cx {
  double r, i;
};
__device__ __forceinline__ Cx add(Cx a, Cx b) { return {a.r + b.r, a.i + b.i}; }
__device__ __forceinline__ Cx sub(Cx a, Cx b) { return {a.r - b.r, a.i - b.i}; }
__device__ __forceinline__ Cx scale(Cx a, double f) { return {a.r * f, a.i * f}; }
// special_mul<fwd>: v * conj(w) forward, v * w backward
template <bool FWD>
__device__ __forceinline__ Cx smul(Cx v, Cx w) {
  if (FWD) return {v.r * w.r + v.i * w.i, v.i * w.r - v.r * w.i};
  return {v.r * w.r - v.i * w.i, v.r * w.i + v.i * w.r};
}
__device__ __forceinline__ Cx smul(Cx v, Cx w, bool fwd) { return fwd ? smul<true>(v, w) : smul<false>(v, w); }
// ROTX90<fwd>: times -i forward, +i backward
template <bool FWD>
__device__ __forceinline__ Cx rot90(Cx a) {
  if (FWD) return {a.i, -a.r};
  return {-a.i, a.r};
}
template <bool FWD>
__device__ __forceinline__ Cx rot45(Cx a) {
  const double h = 0.707106781186547524400844362104849;
  if (FWD) return {h * (a.r + a.i), h * (a.i - a.r)};
  return {h * (a.r - a.i), h * (a.i + a.r)};
}
template <bool FWD>
__device__ __forceinline__ Cx rot135(Cx a) {
  const double h = 0.707106781186547524400844362104849;
  if (FWD) return {h * (a.i - a.r), h * (-a.r - a.i)};
  return {h * (-a.r - a.i), h * (a.r - a.i)};
}

#define PF_FOR(t, N) for (int t = (int)threadIdx.x; t < (int)(N); t += (int)blockDim.x)

// x / d and x % d for 0 <= x < 2^31 by a uniform divisor d >= 1 (round-up
// multiply-high: m = floor(2^32 (2^l - d) / d) + 1, l = ceil(log2 d), then
// x / d = (umulhi(x, m) + x) >> l, exact for every such x).  The tile loops'
// index splits run on these instead of ~30-instruction integer divisions.
struct FDiv {
  unsigned m;
  int l, d;
  __device__ FDiv(const PfDiv& v) : m(v.m), l(v.l), d(v.d) {}   // host-built (pocketfft.h pf_div)
  __device__ explicit FDiv(int dd) : d(dd) {
    l = 0;
    while ((1 << l) < dd) ++l;
    m = (unsigned)((((uint64_t)1 << 32) * (((uint64_t)1 << l) - (uint64_t)dd)) / (uint64_t)dd + 1);
  }
  __device__ __forceinline__ int div(int x) const { return (int)((__umulhi((unsigned)x, m) + (unsigned)x) >> l); }
  __device__ __forceinline__ int mod(int x) const { return x - div(x) * d; }
};

// ======================= complex passes (cfftp) =============================
// One butterfly of pocketfft's pass of radix IP at index i of a pass with ido:
// v[m] = CC(i, m, k) in, v[m] = CH(i, k, m) out (pass2b / pass3b / pass4b /
// pass5b / pass7 / pass8 / pass11 and their forward twins).  The per-pass
// loops (passk) and the LDS tile executor (cgroup) both run these, so the
// arithmetic is one statement.
#define WA(x, i) wa[(i) - 1 + (x) * (ido - 1)]

template <bool FWD>
__device__ __forceinline__ void bfly2(Cx* v, int i, const Cx* wa, int ido) {
  const Cx a = v[0], b = v[1];
  v[0] = add(a, b);
  const Cx d = sub(a, b);
  v[1] = i == 0 ? d : smul<FWD>(d, WA(0, i));
}

template <bool FWD>
__device__ __forceinline__ void bfly3(Cx* v, int i, const Cx* wa, int ido) {
  const double tw1r = -0.5, tw1i = (FWD ? -1 : 1) * 0.8660254037844386467637231707529362;
  const Cx t0 = v[0], t1 = add(v[1], v[2]), t2 = sub(v[1], v[2]);
  v[0] = add(t0, t1);
  const Cx ca = {t0.r + t1.r * tw1r, t0.i + t1.i * tw1r};
  const Cx cb = {-(t2.i * tw1i), t2.r * tw1i};
  if (i == 0) {
    v[1] = add(ca, cb);
    v[2] = sub(ca, cb);
  } else {
    v[1] = smul<FWD>(add(ca, cb), WA(0, i));
    v[2] = smul<FWD>(sub(ca, cb), WA(1, i));
  }
}

template <bool FWD>
__device__ __forceinline__ void bfly4(Cx* v, int i, const Cx* wa, int ido) {
  const Cx t2 = add(v[0], v[2]), t1 = sub(v[0], v[2]);
  const Cx t3 = add(v[1], v[3]), t4 = rot90<FWD>(sub(v[1], v[3]));
  if (i == 0) {
    v[0] = add(t2, t3);
    v[2] = sub(t2, t3);
    v[1] = add(t1, t4);
    v[3] = sub(t1, t4);
  } else {
    v[0] = add(t2, t3);
    v[1] = smul<FWD>(add(t1, t4), WA(0, i));
    v[2] = smul<FWD>(sub(t2, t3), WA(1, i));
    v[3] = smul<FWD>(sub(t1, t4), WA(2, i));
  }
}

// radices 5, 7, 11 (pocketfft's PREPn / PARTSTEPn): pairs t[j] = CC(j) +
// CC(ip-j), d[j] = CC(j) - CC(ip-j); output u = 1..h:
//   ca = t0 + c(u,1) t[1] + ... + c(u,h) t[h]        (left to right)
//   cb = (-(s(u,1) d[1].i +- ...), s(u,1) d[1].r +- ...)
// with c(u,j), s(u,j) the cos / sin of 2 pi (u j mod ip) / ip, the sin's sign
// flipped (a subtraction in the chain) where u j mod ip lies above ip / 2
template <int IPN>
struct OddTw;
template <>
struct OddTw<5> {
  static constexpr double c[3] = {1.0, 0.3090169943749474241022934171828191, -0.8090169943749474241022934171828191};
  static constexpr double s[3] = {0.0, 0.9510565162951535721164393333793821, 0.5877852522924731291687059546390728};
};
template <>
struct OddTw<7> {
  static constexpr double c[4] = {1.0, 0.6234898018587335305250048840042398, -0.2225209339563144042889025644967948,
                                  -0.9009688679024191262361023195074451};
  static constexpr double s[4] = {0.0, 0.7818314824680298087084445266740578, 0.9749279121818236070181316829939312,
                                  0.433883739117558120475768332848359};
};
template <>
struct OddTw<11> {
  static constexpr double c[6] = {1.0, 0.8412535328311811688618116489193677, 0.4154150130018864255292741492296232,
                                  -0.1423148382732851404437926686163697, -0.6548607339452850640569250724662936,
                                  -0.9594929736144973898903680570663277};
  static constexpr double s[6] = {0.0, 0.5406408174555975821076359543186917, 0.9096319953545183714117153830790285,
                                  0.9898214418809327323760920377767188, 0.7557495743542582837740358439723444,
                                  0.2817325568414296977114179153466169};
};

template <bool FWD, int IPN>
__device__ __forceinline__ void bflyodd(Cx* v, int i, const Cx* wa, int ido) {
  constexpr int H = (IPN - 1) / 2;
  Cx tt[H + 1], dd[H + 1];
  const Cx t0 = v[0];
#pragma unroll
  for (int j = 1; j <= H; ++j) {
    tt[j] = add(v[j], v[IPN - j]);
    dd[j] = sub(v[j], v[IPN - j]);
  }
  Cx s0 = t0;
#pragma unroll
  for (int j = 1; j <= H; ++j) s0.r = s0.r + tt[j].r;
#pragma unroll
  for (int j = 1; j <= H; ++j) s0.i = s0.i + tt[j].i;
  v[0] = s0;
#pragma unroll
  for (int u = 1; u <= H; ++u) {
    Cx ca = t0;
    double cbr = 0.0, cbi = 0.0;
#pragma unroll
    for (int j = 1; j <= H; ++j) {
      int r = (u * j) % IPN;
      const bool neg = r > H;
      if (neg) r = IPN - r;
      const double cr = OddTw<IPN>::c[r], si = (FWD ? -1.0 : 1.0) * OddTw<IPN>::s[r];
      ca.r = ca.r + cr * tt[j].r;
      ca.i = ca.i + cr * tt[j].i;
      if (j == 1) {
        cbi = si * dd[j].r;
        cbr = si * dd[j].i;
      } else if (!neg) {
        cbi = cbi + si * dd[j].r;
        cbr = cbr + si * dd[j].i;
      } else {
        cbi = cbi - si * dd[j].r;
        cbr = cbr - si * dd[j].i;
      }
    }
    const Cx cb = {-cbr, cbi};
    if (i == 0) {
      v[u] = add(ca, cb);
      v[IPN - u] = sub(ca, cb);
    } else {
      v[u] = smul<FWD>(add(ca, cb), WA(u - 1, i));
      v[IPN - u] = smul<FWD>(sub(ca, cb), WA(IPN - u - 1, i));
    }
  }
}

template <bool FWD>
__device__ __forceinline__ void bfly8(Cx* v, int i, const Cx* wa, int ido) {
  Cx a1 = add(v[1], v[5]), a5 = sub(v[1], v[5]);
  Cx a3 = add(v[3], v[7]), a7 = sub(v[3], v[7]);
  Cx u = a1;
  a1 = add(u, a3);
  a3 = rot90<FWD>(sub(u, a3));
  a7 = rot90<FWD>(a7);
  u = a5;
  a5 = rot45<FWD>(add(u, a7));
  a7 = rot135<FWD>(sub(u, a7));
  Cx a0 = add(v[0], v[4]), a4 = sub(v[0], v[4]);
  Cx a2 = add(v[2], v[6]), a6 = sub(v[2], v[6]);
  if (i == 0) {
    const Cx s02 = add(a0, a2), d02 = sub(a0, a2);
    v[0] = add(s02, a1);
    v[4] = sub(s02, a1);
    v[2] = add(d02, a3);
    v[6] = sub(d02, a3);
    a6 = rot90<FWD>(a6);
    const Cx s46 = add(a4, a6), d46 = sub(a4, a6);
    v[1] = add(s46, a5);
    v[5] = sub(s46, a5);
    v[3] = add(d46, a7);
    v[7] = sub(d46, a7);
  } else {
    u = a0;
    a0 = add(u, a2);
    a2 = sub(u, a2);
    v[0] = add(a0, a1);
    v[4] = smul<FWD>(sub(a0, a1), WA(3, i));
    v[2] = smul<FWD>(add(a2, a3), WA(1, i));
    v[6] = smul<FWD>(sub(a2, a3), WA(5, i));
    a6 = rot90<FWD>(a6);
    u = a4;
    a4 = add(u, a6);
    a6 = sub(u, a6);
    v[1] = smul<FWD>(add(a4, a5), WA(0, i));
    v[5] = smul<FWD>(sub(a4, a5), WA(4, i));
    v[3] = smul<FWD>(add(a6, a7), WA(2, i));
    v[7] = smul<FWD>(sub(a6, a7), WA(6, i));
  }
}
#undef WA

template <bool FWD, int IP>
__device__ __forceinline__ void bfly(Cx* v, int i, const Cx* wa, int ido) {
  if constexpr (IP == 2) bfly2<FWD>(v, i, wa, ido);
  else if constexpr (IP == 3) bfly3<FWD>(v, i, wa, ido);
  else if constexpr (IP == 4) bfly4<FWD>(v, i, wa, ido);
  else if constexpr (IP == 8) bfly8<FWD>(v, i, wa, ido);
  else bflyodd<FWD, IP>(v, i, wa, ido);
}

// one whole pass over global memory (the unfused executor)
template <bool FWD, int IP>
__device__ void passk(int ido, int l1, const Cx* __restrict__ cc, Cx* __restrict__ ch, const Cx* wa) {
  PF_FOR(t, l1 * ido) {
    const int k = t / ido, i = t - k * ido;
    Cx v[IP];
#pragma unroll
    for (int m = 0; m < IP; ++m) v[m] = cc[i + ido * (m + IP * k)];
    bfly<FWD, IP>(v, i, wa, ido);
#pragma unroll
    for (int m = 0; m < IP; ++m) ch[i + ido * (k + l1 * m)] = v[m];
  }
}

// generic pass (ip > 11): the result lands in cc
template <bool FWD>
__device__ void passg(int ido, int ip, int l1, Cx* cc, Cx* ch, const Cx* wa, const Cx* csarr) {
  const int cdim = ip, ipph = (ip + 1) / 2, idl1 = ido * l1;
#define CH(a, b, c) ch[(a) + ido * ((b) + l1 * (c))]
#define CC(a, b, c) cc[(a) + ido * ((b) + cdim * (c))]
#define CX(a, b, c) cc[(a) + ido * ((b) + l1 * (c))]
#define CX2(a, b) cc[(a) + idl1 * (b)]
#define CH2(a, b) ch[(a) + idl1 * (b)]
  auto wal = [&](int x) -> Cx {
    if (x == 0) return {1.0, 0.0};
    const Cx c = csarr[x];
    return {c.r, FWD ? -c.i : c.i};
  };
  PF_FOR(t, l1 * ido) {
    const int k = t / ido, i = t - k * ido;
    CH(i, k, 0) = CC(i, 0, k);
    for (int j = 1, jc = ip - 1; j < ipph; ++j, --jc) {
      CH(i, k, j) = add(CC(i, j, k), CC(i, jc, k));
      CH(i, k, jc) = sub(CC(i, j, k), CC(i, jc, k));
    }
  }
  __syncthreads();
  PF_FOR(ik, idl1) {
    Cx tmp = CH2(ik, 0);
    for (int j = 1; j < ipph; ++j) tmp = add(tmp, CH2(ik, j));
    CX2(ik, 0) = tmp;
    for (int l = 1, lc = ip - 1; l < ipph; ++l, --lc) {
      const Cx w1 = wal(l), w2 = wal(2 * l);
      Cx xl, xlc;
      xl.r = CH2(ik, 0).r + w1.r * CH2(ik, 1).r + w2.r * CH2(ik, 2).r;
      xl.i = CH2(ik, 0).i + w1.r * CH2(ik, 1).i + w2.r * CH2(ik, 2).i;
      xlc.r = -(w1.i * CH2(ik, ip - 1).i + w2.i * CH2(ik, ip - 2).i);
      xlc.i = w1.i * CH2(ik, ip - 1).r + w2.i * CH2(ik, ip - 2).r;
      int iwal = 2 * l;
      int j = 3, jc = ip - 3;
      for (; j < ipph - 1; j += 2, jc -= 2) {
        iwal += l;
        if (iwal > ip) iwal -= ip;
        const Cx xw = wal(iwal);
        iwal += l;
        if (iwal > ip) iwal -= ip;
        const Cx xw2 = wal(iwal);
        xl.r += CH2(ik, j).r * xw.r + CH2(ik, j + 1).r * xw2.r;
        xl.i += CH2(ik, j).i * xw.r + CH2(ik, j + 1).i * xw2.r;
        xlc.r -= CH2(ik, jc).i * xw.i + CH2(ik, jc - 1).i * xw2.i;
        xlc.i += CH2(ik, jc).r * xw.i + CH2(ik, jc - 1).r * xw2.i;
      }
      for (; j < ipph; ++j, --jc) {
        iwal += l;
        if (iwal > ip) iwal -= ip;
        const Cx xw = wal(iwal);
        xl.r += CH2(ik, j).r * xw.r;
        xl.i += CH2(ik, j).i * xw.r;
        xlc.r -= CH2(ik, jc).i * xw.i;
        xlc.i += CH2(ik, jc).r * xw.i;
      }
      CX2(ik, l) = xl;
      CX2(ik, lc) = xlc;
    }
  }
  __syncthreads();
  // shuffling and twiddling
  if (ido == 1) {
    PF_FOR(t, (ipph - 1) * idl1) {
      const int j = 1 + t / idl1, ik = t - (j - 1) * idl1, jc = ip - j;
      const Cx t1 = CX2(ik, j), t2 = CX2(ik, jc);
      CX2(ik, j) = add(t1, t2);
      CX2(ik, jc) = sub(t1, t2);
    }
  } else {
    PF_FOR(t, (ipph - 1) * l1 * ido) {
      const int j = 1 + t / (l1 * ido), r = t - (j - 1) * l1 * ido, k = r / ido, i = r - k * ido, jc = ip - j;
      if (i == 0) {
        const Cx t1 = CX(0, k, j), t2 = CX(0, k, jc);
        CX(0, k, j) = add(t1, t2);
        CX(0, k, jc) = sub(t1, t2);
      } else {
        const Cx x1 = add(CX(i, k, j), CX(i, k, jc)), x2 = sub(CX(i, k, j), CX(i, k, jc));
        CX(i, k, j) = smul<FWD>(x1, wa[(j - 1) * (ido - 1) + i - 1]);
        CX(i, k, jc) = smul<FWD>(x2, wa[(jc - 1) * (ido - 1) + i - 1]);
      }
    }
  }
#undef CH
#undef CC
#undef CX
#undef CX2
#undef CH2
}

// c (P.len) in place, scratch ch (P.len): the transform, times fct (not when
// fct == 1), pass by pass over global memory
template <bool FWD>
__device__ void cfftp_passes(const PfPasses& P, const double* pool, Cx* c, Cx* ch, double fct) {
  const int len = P.len;
  if (len == 1) {
    if (threadIdx.x == 0) c[0] = scale(c[0], fct);
    __syncthreads();
    return;
  }
  Cx *p1 = c, *p2 = ch;
  for (int k = 0; k < P.nf; ++k) {
    const PfFact F = P.f[k];
    const Cx* wa = reinterpret_cast<const Cx*>(pool + F.tw);
    switch (F.ip) {
      case 4: passk<FWD, 4>(F.ido, F.l1, p1, p2, wa); break;
      case 8: passk<FWD, 8>(F.ido, F.l1, p1, p2, wa); break;
      case 2: passk<FWD, 2>(F.ido, F.l1, p1, p2, wa); break;
      case 3: passk<FWD, 3>(F.ido, F.l1, p1, p2, wa); break;
      case 5: passk<FWD, 5>(F.ido, F.l1, p1, p2, wa); break;
      case 7: passk<FWD, 7>(F.ido, F.l1, p1, p2, wa); break;
      case 11: passk<FWD, 11>(F.ido, F.l1, p1, p2, wa); break;
      default: {
        passg<FWD>(F.ido, F.ip, F.l1, p1, p2, wa, reinterpret_cast<const Cx*>(pool + F.tws));
        Cx* t = p1;
        p1 = p2;
        p2 = t;
      }
    }
    Cx* t = p1;
    p1 = p2;
    p2 = t;
    __syncthreads();
  }
  if (p1 != c) {
    PF_FOR(i, len) c[i] = fct != 1.0 ? scale(p1[i], fct) : p1[i];
  } else if (fct != 1.0) {
    PF_FOR(i, len) c[i] = scale(c[i], fct);
  }
  __syncthreads();
}

// ------------------------- LDS-fused executor -------------------------------
constexpr int kPfThreadsPre = 512;                      // workgroup size of the prefetching tile loop
constexpr int kPfPreC = kPfTileElems / kPfThreadsPre;    // complex elements per thread of a tile
constexpr int kPfPreR = kPfTileDoubles / kPfThreadsPre;  // real elements per thread of a tile
// One tile pass: radix IP over the tile's Q columns, local sizes idol = ido / D,
// l1l = l1 / L; column uu holds residue i = i0 + uu % Qi of the group's
// global index (the butterfly's twiddle index is i + D * i_loc).
template <bool FWD, int IP>
__device__ __forceinline__ void tile_pass(const Cx* cur, Cx* nxt, const FDiv& fQ, const FDiv& fQi, int qi, int qk,
                                          int i0, int D, const FDiv& fid, int l1l, const Cx* wa, int ido) {
  const int Q = fQ.d, idol = fid.d, nb = Q * idol * l1l;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    const int r = fQ.div(b), uu = b - r * Q;
    const int kk = fQi.div(uu), ii = uu - kk * fQi.d;
    if (ii >= qi || kk >= qk) continue;
    const int k_loc = fid.div(r), i_loc = r - k_loc * idol;
    Cx v[IP];
#pragma unroll
    for (int m = 0; m < IP; ++m) v[m] = cur[(i_loc + idol * (m + IP * k_loc)) * Q + uu];
    bfly<FWD, IP>(v, i0 + ii + D * i_loc, wa, ido);
#pragma unroll
    for (int m = 0; m < IP; ++m) nxt[(i_loc + idol * (k_loc + l1l * m)) * Q + uu] = v[m];
  }
}

// the passes of group G over the whole array: element pos = rd(pos) in,
// wr(pos, v) out (every tile reads i + D (j + P k) and writes i + D (k + L j);
// a group with L == 1 reads and writes the same positions per tile, so it may
// run in place).  lds: 2 * kPfTileElems complex.
template <bool FWD, class Rd, class Wr>
__device__ __forceinline__ void cgroup(const PfPasses& Pl, const PfGroup& G, const double* pool, Rd rd, Wr wr, Cx* lds) {
  const int D = G.D, L = G.L, P = G.P;
  const int Q = G.Q, Qi = G.Qi, Qk = G.Qk;
  const int nti = (D + Qi - 1) / Qi, ntk = (L + Qk - 1) / Qk, nt = nti * ntk;
  // a 512-thread workgroup holds a whole tile in registers (kPfPreC per
  // thread): the next tile's loads are issued before this tile's passes, so
  // their latency hides behind the LDS work and the stores
  const bool pre = blockDim.x == kPfThreadsPre;
  const FDiv fP(G.dv[0]), fQ(G.dv[1]), fQi(G.dv[2]);
  Cx pv[kPfPreC];
  const FDiv fnti(G.dv[6]);
  auto geom = [&](int tile, int& i0, int& k0, int& qi, int& qk) {
    const int tk = fnti.div(tile), ti = tile - tk * nti;
    i0 = ti * Qi;
    k0 = tk * Qk;
    qi = D - i0 < Qi ? D - i0 : Qi;
    qk = L - k0 < Qk ? L - k0 : Qk;
  };
  auto issue = [&](int tile) {
    int i0, k0, qi, qk;
    geom(tile, i0, k0, qi, qk);
    const int ne = qk * P * qi;
    const FDiv fqi(qi == Qi ? G.dv[2] : G.dv[3]);
#pragma unroll
    for (int u = 0; u < kPfPreC; ++u) {
      const int e = (int)threadIdx.x + u * kPfThreadsPre;
      if (e < ne) {
        const int r = fqi.div(e), ii = e - r * qi, kk = fP.div(r), j = r - kk * P;
        pv[u] = rd(i0 + ii + D * (j + P * (k0 + kk)));
      }
    }
  };
  if (pre) issue(0);
  for (int tile = 0; tile < nt; ++tile) {
    int i0, k0, qi, qk;
    geom(tile, i0, k0, qi, qk);
    Cx* cur = lds;
    Cx* nxt = lds + kPfTileElems;
    // load in memory order (k, j, i)
    const int ne = qk * P * qi;
    const FDiv fqi(qi == Qi ? G.dv[2] : G.dv[3]), fqk(qk == Qk ? G.dv[4] : G.dv[5]);
    if (pre) {
#pragma unroll
      for (int u = 0; u < kPfPreC; ++u) {
        const int e = (int)threadIdx.x + u * kPfThreadsPre;
        if (e < ne) {
          const int r = fqi.div(e), ii = e - r * qi, kk = fP.div(r), j = r - kk * P;
          cur[j * Q + kk * Qi + ii] = pv[u];
        }
      }
    } else {
      for (int e = threadIdx.x; e < ne; e += blockDim.x) {
        const int r = fqi.div(e), ii = e - r * qi, kk = fP.div(r), j = r - kk * P;
        cur[j * Q + kk * Qi + ii] = rd(i0 + ii + D * (j + P * (k0 + kk)));
      }
    }
    __syncthreads();
    if (pre && tile + 1 < nt) issue(tile + 1);
    for (int q = G.f0; q < G.f0 + G.nf; ++q) {
      const PfFact F = Pl.f[q];
      const Cx* wa = reinterpret_cast<const Cx*>(pool + F.tw);
      const FDiv fid(F.dv[0]);
      const int l1l = F.l1l;
      switch (F.ip) {
        case 4: tile_pass<FWD, 4>(cur, nxt, fQ, fQi, qi, qk, i0, D, fid, l1l, wa, F.ido); break;
        case 8: tile_pass<FWD, 8>(cur, nxt, fQ, fQi, qi, qk, i0, D, fid, l1l, wa, F.ido); break;
        case 2: tile_pass<FWD, 2>(cur, nxt, fQ, fQi, qi, qk, i0, D, fid, l1l, wa, F.ido); break;
        case 3: tile_pass<FWD, 3>(cur, nxt, fQ, fQi, qi, qk, i0, D, fid, l1l, wa, F.ido); break;
        case 5: tile_pass<FWD, 5>(cur, nxt, fQ, fQi, qi, qk, i0, D, fid, l1l, wa, F.ido); break;
        case 7: tile_pass<FWD, 7>(cur, nxt, fQ, fQi, qi, qk, i0, D, fid, l1l, wa, F.ido); break;
        default: tile_pass<FWD, 11>(cur, nxt, fQ, fQi, qi, qk, i0, D, fid, l1l, wa, F.ido); break;
      }
      __syncthreads();
      Cx* t = cur;
      cur = nxt;
      nxt = t;
    }
    // store in memory order (j, k, i)
    for (int e = threadIdx.x; e < ne; e += blockDim.x) {
      const int r = fqi.div(e), ii = e - r * qi, j = fqk.div(r), kk = r - j * qk;
      wr(i0 + ii + D * (k0 + kk + L * j), cur[j * Q + kk * Qi + ii]);
    }
    __syncthreads();
  }
}

struct RdBuf {
  const Cx* p;
  __device__ Cx operator()(int i) const { return p[i]; }
};
struct WrD {
  double* p;
  __device__ void operator()(int i, double v) const { p[i] = v; }
};
struct RdD {
  const double* p;
  __device__ double operator()(int i) const { return p[i]; }
};
struct WrBuf {
  Cx* p;
  __device__ void operator()(int i, Cx v) const { p[i] = v; }
};

// pocketfft's cfftp transform of the sequence src(0 .. len-1), each result
// handed to fin(pos, v) (unscaled); A, B: len complex of scratch each.  src
// may read A (not B); fin must not write B.  Fused plans run group by group
// (the last one reads B); others materialise src into A, run the passes and
// hand A's entries to fin.  PADB: a two-group plan whose src does not read A
// may run B past len (up to len + len / 8, over A's start): its hand-off rows
// are then padded to whole 128-byte lines.
template <bool FWD, class Src, class Fin, bool LEAN = false, bool PADB = false>
__device__ __forceinline__ void cfftp_x(const PfPasses& P, const double* pool, Src src, Cx* A, Cx* B, Fin fin, Cx* lds) {
  const int len = P.len;
  if (!LEAN && (!P.fused || lds == nullptr)) {
    PF_FOR(i, len) A[i] = src(i);
    __syncthreads();
    cfftp_passes<FWD>(P, pool, A, B, 1.0);
    PF_FOR(i, len) fin(i, A[i]);
    __syncthreads();
    return;
  }
  const int G = P.ng;
  if (G == 1) {   // one group of one tile: every load precedes every store
    cgroup<FWD>(P, P.g[0], pool, src, fin, lds);
    return;
  }
  if (PADB && G == 2 && P.g[0].D >= kPfPadMinD) {
    // group 0's output rows (position p = i + D j, i < D) at i + Dp j, Dp =
    // D rounded up to whole lines: its tiles store line-aligned runs, and
    // group 1 (D = 1) still reads each row as one contiguous run
    const FDiv fD(P.g[0].dv[7]);
    const int pad = (kPfPadC - fD.d % kPfPadC) % kPfPadC;
    cgroup<FWD>(P, P.g[0], pool, src, [=](int p, Cx v) { B[p + fD.div(p) * pad] = v; }, lds);
    cgroup<FWD>(P, P.g[1], pool, [=](int p) { return B[p + fD.div(p) * pad]; }, fin, lds);
    return;
  }
  // outputs: group G-2 -> B, G-3 -> A, ...
  auto outbuf = [&](int g) { return ((G - 2 - g) & 1) == 0 ? B : A; };
  cgroup<FWD>(P, P.g[0], pool, src, WrBuf{outbuf(0)}, lds);
  for (int g = 1; g < G - 1; ++g) cgroup<FWD>(P, P.g[g], pool, RdBuf{outbuf(g - 1)}, WrBuf{outbuf(g)}, lds);
  cgroup<FWD>(P, P.g[G - 1], pool, RdBuf{B}, fin, lds);
}

// c (P.len) in place, scratch ch (P.len): the transform, times fct (not when
// fct == 1); lds (2 * kPfTileElems complex) or nullptr for the unfused passes
template <bool FWD>
__device__ void cfftp(const PfPasses& P, const double* pool, Cx* c, Cx* ch, double fct, Cx* lds) {
  if (P.len == 1 || !P.fused || lds == nullptr) {
    cfftp_passes<FWD>(P, pool, c, ch, fct);
    return;
  }
  cfftp_x<FWD>(P, pool, RdBuf{c}, c, ch,
               [=](int i, Cx v) { c[i] = fct != 1.0 ? scale(v, fct) : v; }, lds);
}

// ========================= real passes (rfftp) ==============================
#define CC(a, b, c) cc[(a) + ido * ((b) + l1 * (c))]
#define WA(x, i) wa[(i) + (x) * (ido - 1)]

// nb sub-arrays at stride bs (the fused executor's tile columns; 1 / 0 for a
// whole-array pass)
__device__ void radf2(int ido, int l1, const double* __restrict__ cc0, double* __restrict__ ch0, const double* wa, int nb = 1,
                      int bs = 0, const PfDiv* dv = nullptr) {
#define CH(a, b, c) ch[(a) + ido * ((b) + 2 * (c))]
  const FDiv fl1 = dv ? FDiv(dv[0]) : FDiv(l1);
  PF_FOR(tb, nb * l1) {
    const int b = fl1.div(tb), k = tb - b * l1;
    const double* cc = cc0 + b * bs;
    double* ch = ch0 + b * bs;
    CH(0, 0, k) = CC(0, k, 0) + CC(0, k, 1);
    CH(ido - 1, 1, k) = CC(0, k, 0) - CC(0, k, 1);
    if ((ido & 1) == 0) {
      CH(0, 1, k) = -CC(ido - 1, k, 1);
      CH(ido - 1, 0, k) = CC(ido - 1, k, 0);
    }
  }
  if (ido <= 2) return;
  const int hi = (ido - 1) / 2;
  const FDiv flh = dv ? FDiv(dv[2]) : FDiv(l1 * hi), fhi = dv ? FDiv(dv[1]) : FDiv(hi);
  PF_FOR(tb, nb * l1 * hi) {
    const int b = flh.div(tb), t = tb - b * (l1 * hi);
    const int k = fhi.div(t), i = 2 + 2 * (t - k * hi), ic = ido - i;
    const double* cc = cc0 + b * bs;
    double* ch = ch0 + b * bs;
    const double tr2 = wa[i - 2] * CC(i - 1, k, 1) + wa[i - 1] * CC(i, k, 1);
    const double ti2 = wa[i - 2] * CC(i, k, 1) - wa[i - 1] * CC(i - 1, k, 1);
    CH(i - 1, 0, k) = CC(i - 1, k, 0) + tr2;
    CH(ic - 1, 1, k) = CC(i - 1, k, 0) - tr2;
    CH(i, 0, k) = ti2 + CC(i, k, 0);
    CH(ic, 1, k) = ti2 - CC(i, k, 0);
  }
#undef CH
}

// nb sub-arrays at stride bs (the fused executor's tile columns; 1 / 0 for a
// whole-array pass)
__device__ void radf3(int ido, int l1, const double* __restrict__ cc0, double* __restrict__ ch0, const double* wa, int nb = 1,
                      int bs = 0, const PfDiv* dv = nullptr) {
  const double taur = -0.5, taui = 0.8660254037844386467637231707529362;
#define CH(a, b, c) ch[(a) + ido * ((b) + 3 * (c))]
  const FDiv fl1 = dv ? FDiv(dv[0]) : FDiv(l1);
  PF_FOR(tb, nb * l1) {
    const int b = fl1.div(tb), k = tb - b * l1;
    const double* cc = cc0 + b * bs;
    double* ch = ch0 + b * bs;
    const double cr2 = CC(0, k, 1) + CC(0, k, 2);
    CH(0, 0, k) = CC(0, k, 0) + cr2;
    CH(0, 2, k) = taui * (CC(0, k, 2) - CC(0, k, 1));
    CH(ido - 1, 1, k) = CC(0, k, 0) + taur * cr2;
  }
  if (ido == 1) return;
  const int hi = (ido - 1) / 2;
  const FDiv flh = dv ? FDiv(dv[2]) : FDiv(l1 * hi), fhi = dv ? FDiv(dv[1]) : FDiv(hi);
  PF_FOR(tb, nb * l1 * hi) {
    const int b = flh.div(tb), t = tb - b * (l1 * hi);
    const int k = fhi.div(t), i = 2 + 2 * (t - k * hi), ic = ido - i;
    const double* cc = cc0 + b * bs;
    double* ch = ch0 + b * bs;
    const double dr2 = WA(0, i - 2) * CC(i - 1, k, 1) + WA(0, i - 1) * CC(i, k, 1);
    const double di2 = WA(0, i - 2) * CC(i, k, 1) - WA(0, i - 1) * CC(i - 1, k, 1);
    const double dr3 = WA(1, i - 2) * CC(i - 1, k, 2) + WA(1, i - 1) * CC(i, k, 2);
    const double di3 = WA(1, i - 2) * CC(i, k, 2) - WA(1, i - 1) * CC(i - 1, k, 2);
    const double cr2 = dr2 + dr3, ci2 = di2 + di3;
    CH(i - 1, 0, k) = CC(i - 1, k, 0) + cr2;
    CH(i, 0, k) = CC(i, k, 0) + ci2;
    const double tr2 = CC(i - 1, k, 0) + taur * cr2, ti2 = CC(i, k, 0) + taur * ci2;
    const double tr3 = taui * (di2 - di3), ti3 = taui * (dr3 - dr2);
    CH(i - 1, 2, k) = tr2 + tr3;
    CH(ic - 1, 1, k) = tr2 - tr3;
    CH(i, 2, k) = ti2 + ti3;
    CH(ic, 1, k) = ti3 - ti2;
  }
#undef CH
}

// nb sub-arrays at stride bs (the fused executor's tile columns; 1 / 0 for a
// whole-array pass)
__device__ void radf4(int ido, int l1, const double* __restrict__ cc0, double* __restrict__ ch0, const double* wa, int nb = 1,
                      int bs = 0, const PfDiv* dv = nullptr) {
  const double hsqt2 = 0.707106781186547524400844362104849;
#define CH(a, b, c) ch[(a) + ido * ((b) + 4 * (c))]
  const FDiv fl1 = dv ? FDiv(dv[0]) : FDiv(l1);
  PF_FOR(tb, nb * l1) {
    const int b = fl1.div(tb), k = tb - b * l1;
    const double* cc = cc0 + b * bs;
    double* ch = ch0 + b * bs;
    const double tr1 = CC(0, k, 3) + CC(0, k, 1);
    CH(0, 2, k) = CC(0, k, 3) - CC(0, k, 1);
    const double tr2 = CC(0, k, 0) + CC(0, k, 2);
    CH(ido - 1, 1, k) = CC(0, k, 0) - CC(0, k, 2);
    CH(0, 0, k) = tr2 + tr1;
    CH(ido - 1, 3, k) = tr2 - tr1;
    if ((ido & 1) == 0) {
      const double ti1 = -hsqt2 * (CC(ido - 1, k, 1) + CC(ido - 1, k, 3));
      const double tr1b = hsqt2 * (CC(ido - 1, k, 1) - CC(ido - 1, k, 3));
      CH(ido - 1, 0, k) = CC(ido - 1, k, 0) + tr1b;
      CH(ido - 1, 2, k) = CC(ido - 1, k, 0) - tr1b;
      CH(0, 3, k) = ti1 + CC(ido - 1, k, 2);
      CH(0, 1, k) = ti1 - CC(ido - 1, k, 2);
    }
  }
  if (ido <= 2) return;
  const int hi = (ido - 1) / 2;
  const FDiv flh = dv ? FDiv(dv[2]) : FDiv(l1 * hi), fhi = dv ? FDiv(dv[1]) : FDiv(hi);
  PF_FOR(tb, nb * l1 * hi) {
    const int b = flh.div(tb), t = tb - b * (l1 * hi);
    const int k = fhi.div(t), i = 2 + 2 * (t - k * hi), ic = ido - i;
    const double* cc = cc0 + b * bs;
    double* ch = ch0 + b * bs;
    const double cr2 = WA(0, i - 2) * CC(i - 1, k, 1) + WA(0, i - 1) * CC(i, k, 1);
    const double ci2 = WA(0, i - 2) * CC(i, k, 1) - WA(0, i - 1) * CC(i - 1, k, 1);
    const double cr3 = WA(1, i - 2) * CC(i - 1, k, 2) + WA(1, i - 1) * CC(i, k, 2);
    const double ci3 = WA(1, i - 2) * CC(i, k, 2) - WA(1, i - 1) * CC(i - 1, k, 2);
    const double cr4 = WA(2, i - 2) * CC(i - 1, k, 3) + WA(2, i - 1) * CC(i, k, 3);
    const double ci4 = WA(2, i - 2) * CC(i, k, 3) - WA(2, i - 1) * CC(i - 1, k, 3);
    const double tr1 = cr4 + cr2, tr4 = cr4 - cr2;
    const double ti1 = ci2 + ci4, ti4 = ci2 - ci4;
    const double tr2 = CC(i - 1, k, 0) + cr3, tr3 = CC(i - 1, k, 0) - cr3;
    const double ti2 = CC(i, k, 0) + ci3, ti3 = CC(i, k, 0) - ci3;
    CH(i - 1, 0, k) = tr2 + tr1;
    CH(ic - 1, 3, k) = tr2 - tr1;
    CH(i, 0, k) = ti1 + ti2;
    CH(ic, 3, k) = ti1 - ti2;
    CH(i - 1, 2, k) = tr3 + ti4;
    CH(ic - 1, 1, k) = tr3 - ti4;
    CH(i, 2, k) = tr4 + ti3;
    CH(ic, 1, k) = tr4 - ti3;
  }
#undef CH
}

// nb sub-arrays at stride bs (the fused executor's tile columns; 1 / 0 for a
// whole-array pass)
__device__ void radf5(int ido, int l1, const double* __restrict__ cc0, double* __restrict__ ch0, const double* wa, int nb = 1,
                      int bs = 0, const PfDiv* dv = nullptr) {
  const double tr11 = 0.3090169943749474241022934171828191, ti11 = 0.9510565162951535721164393333793821;
  const double tr12 = -0.8090169943749474241022934171828191, ti12 = 0.5877852522924731291687059546390728;
#define CH(a, b, c) ch[(a) + ido * ((b) + 5 * (c))]
  const FDiv fl1 = dv ? FDiv(dv[0]) : FDiv(l1);
  PF_FOR(tb, nb * l1) {
    const int b = fl1.div(tb), k = tb - b * l1;
    const double* cc = cc0 + b * bs;
    double* ch = ch0 + b * bs;
    const double cr2 = CC(0, k, 4) + CC(0, k, 1), ci5 = CC(0, k, 4) - CC(0, k, 1);
    const double cr3 = CC(0, k, 3) + CC(0, k, 2), ci4 = CC(0, k, 3) - CC(0, k, 2);
    CH(0, 0, k) = CC(0, k, 0) + cr2 + cr3;
    CH(ido - 1, 1, k) = CC(0, k, 0) + tr11 * cr2 + tr12 * cr3;
    CH(0, 2, k) = ti11 * ci5 + ti12 * ci4;
    CH(ido - 1, 3, k) = CC(0, k, 0) + tr12 * cr2 + tr11 * cr3;
    CH(0, 4, k) = ti12 * ci5 - ti11 * ci4;
  }
  if (ido == 1) return;
  const int hi = (ido - 1) / 2;
  const FDiv flh = dv ? FDiv(dv[2]) : FDiv(l1 * hi), fhi = dv ? FDiv(dv[1]) : FDiv(hi);
  PF_FOR(tb, nb * l1 * hi) {
    const int b = flh.div(tb), t = tb - b * (l1 * hi);
    const int k = fhi.div(t), i = 2 + 2 * (t - k * hi), ic = ido - i;
    const double* cc = cc0 + b * bs;
    double* ch = ch0 + b * bs;
    const double dr2 = WA(0, i - 2) * CC(i - 1, k, 1) + WA(0, i - 1) * CC(i, k, 1);
    const double di2 = WA(0, i - 2) * CC(i, k, 1) - WA(0, i - 1) * CC(i - 1, k, 1);
    const double dr3 = WA(1, i - 2) * CC(i - 1, k, 2) + WA(1, i - 1) * CC(i, k, 2);
    const double di3 = WA(1, i - 2) * CC(i, k, 2) - WA(1, i - 1) * CC(i - 1, k, 2);
    const double dr4 = WA(2, i - 2) * CC(i - 1, k, 3) + WA(2, i - 1) * CC(i, k, 3);
    const double di4 = WA(2, i - 2) * CC(i, k, 3) - WA(2, i - 1) * CC(i - 1, k, 3);
    const double dr5 = WA(3, i - 2) * CC(i - 1, k, 4) + WA(3, i - 1) * CC(i, k, 4);
    const double di5 = WA(3, i - 2) * CC(i, k, 4) - WA(3, i - 1) * CC(i - 1, k, 4);
    const double cr2 = dr5 + dr2, ci5 = dr5 - dr2;
    const double ci2 = di2 + di5, cr5 = di2 - di5;
    const double cr3 = dr4 + dr3, ci4 = dr4 - dr3;
    const double ci3 = di3 + di4, cr4 = di3 - di4;
    CH(i - 1, 0, k) = CC(i - 1, k, 0) + cr2 + cr3;
    CH(i, 0, k) = CC(i, k, 0) + ci2 + ci3;
    const double tr2 = CC(i - 1, k, 0) + tr11 * cr2 + tr12 * cr3;
    const double ti2 = CC(i, k, 0) + tr11 * ci2 + tr12 * ci3;
    const double tr3 = CC(i - 1, k, 0) + tr12 * cr2 + tr11 * cr3;
    const double ti3 = CC(i, k, 0) + tr12 * ci2 + tr11 * ci3;
    const double tr5 = cr5 * ti11 + cr4 * ti12, tr4 = cr5 * ti12 - cr4 * ti11;
    const double ti5 = ci5 * ti11 + ci4 * ti12, ti4 = ci5 * ti12 - ci4 * ti11;
    CH(i - 1, 2, k) = tr2 + tr5;
    CH(ic - 1, 1, k) = tr2 - tr5;
    CH(i, 2, k) = ti2 + ti5;
    CH(ic, 1, k) = ti5 - ti2;
    CH(i - 1, 4, k) = tr3 + tr4;
    CH(ic - 1, 3, k) = tr3 - tr4;
    CH(i, 4, k) = ti3 + ti4;
    CH(ic, 3, k) = ti4 - ti3;
  }
#undef CH
}
#undef CC
#undef WA

// generic forward pass (ip odd > 5, ido odd): the result lands in cc
__device__ void radfg(int ido, int ip, int l1, double* cc, double* ch, const double* wa,
                      const double* csarr) {
  const int cdim = ip, ipph = (ip + 1) / 2, idl1 = ido * l1;
#define CC(a, b, c) cc[(a) + ido * ((b) + cdim * (c))]
#define CH(a, b, c) ch[(a) + ido * ((b) + l1 * (c))]
#define C1(a, b, c) cc[(a) + ido * ((b) + l1 * (c))]
#define C2(a, b) cc[(a) + idl1 * (b)]
#define CH2(a, b) ch[(a) + idl1 * (b)]
  // phase 1: twiddles of the j / jc pairs (i >= 1) and the k column sums (i = 0)
  const int hp = (ido - 1) / 2;
  PF_FOR(t, (ipph - 1) * l1 * (hp + 1)) {
    const int j = 1 + t / (l1 * (hp + 1)), r = t - (j - 1) * l1 * (hp + 1), k = r / (hp + 1),
                  q = r - k * (hp + 1), jc = ip - j;
    if (q == 0) {
      const double t1 = C1(0, k, j), t2 = C1(0, k, jc);
      C1(0, k, j) = t2 + t1;
      C1(0, k, jc) = t2 - t1;
    } else {
      const int i = 2 * q - 1;
      const int idij = (j - 1) * (ido - 1) + (i - 1), idij2 = (jc - 1) * (ido - 1) + (i - 1);
      const double t1 = C1(i, k, j), t2 = C1(i + 1, k, j), t3 = C1(i, k, jc), t4 = C1(i + 1, k, jc);
      const double x1 = wa[idij] * t1 + wa[idij + 1] * t2, x2 = wa[idij] * t2 - wa[idij + 1] * t1,
                   x3 = wa[idij2] * t3 + wa[idij2 + 1] * t4, x4 = wa[idij2] * t4 - wa[idij2 + 1] * t3;
      C1(i, k, j) = x3 + x1;
      C1(i + 1, k, jc) = x3 - x1;
      C1(i + 1, k, j) = x2 + x4;
      C1(i, k, jc) = x2 - x4;
    }
  }
  __syncthreads();
  // phase 2: the ip-point real DFT across columns, per ik
  PF_FOR(ik, idl1) {
    for (int l = 1, lc = ip - 1; l < ipph; ++l, --lc) {
      double a = C2(ik, 0) + csarr[2 * l] * C2(ik, 1) + csarr[4 * l] * C2(ik, 2);
      double b = csarr[2 * l + 1] * C2(ik, ip - 1) + csarr[4 * l + 1] * C2(ik, ip - 2);
      int iang = 2 * l;
      int j = 3, jc = ip - 3;
      for (; j < ipph - 3; j += 4, jc -= 4) {
        iang += l;
        if (iang > ip) iang -= ip;
        const double ar1 = csarr[2 * iang], ai1 = csarr[2 * iang + 1];
        iang += l;
        if (iang > ip) iang -= ip;
        const double ar2 = csarr[2 * iang], ai2 = csarr[2 * iang + 1];
        iang += l;
        if (iang > ip) iang -= ip;
        const double ar3 = csarr[2 * iang], ai3 = csarr[2 * iang + 1];
        iang += l;
        if (iang > ip) iang -= ip;
        const double ar4 = csarr[2 * iang], ai4 = csarr[2 * iang + 1];
        a += ar1 * C2(ik, j) + ar2 * C2(ik, j + 1) + ar3 * C2(ik, j + 2) + ar4 * C2(ik, j + 3);
        b += ai1 * C2(ik, jc) + ai2 * C2(ik, jc - 1) + ai3 * C2(ik, jc - 2) + ai4 * C2(ik, jc - 3);
      }
      for (; j < ipph - 1; j += 2, jc -= 2) {
        iang += l;
        if (iang > ip) iang -= ip;
        const double ar1 = csarr[2 * iang], ai1 = csarr[2 * iang + 1];
        iang += l;
        if (iang > ip) iang -= ip;
        const double ar2 = csarr[2 * iang], ai2 = csarr[2 * iang + 1];
        a += ar1 * C2(ik, j) + ar2 * C2(ik, j + 1);
        b += ai1 * C2(ik, jc) + ai2 * C2(ik, jc - 1);
      }
      for (; j < ipph; ++j, --jc) {
        iang += l;
        if (iang > ip) iang -= ip;
        const double ar = csarr[2 * iang], ai = csarr[2 * iang + 1];
        a += ar * C2(ik, j);
        b += ai * C2(ik, jc);
      }
      CH2(ik, l) = a;
      CH2(ik, lc) = b;
    }
    double s = C2(ik, 0);
    for (int j = 1; j < ipph; ++j) s += C2(ik, j);
    CH2(ik, 0) = s;
  }
  __syncthreads();
  // phase 3: into the halfcomplex layout
  PF_FOR(t, l1 * ido) {
    const int k = t / ido, i = t - k * ido;
    CC(i, 0, k) = CH(i, k, 0);
  }
  PF_FOR(t, (ipph - 1) * l1) {
    const int j = 1 + t / l1, k = t - (j - 1) * l1, jc = ip - j, j2 = 2 * j - 1;
    CC(ido - 1, j2, k) = CH(0, k, j);
    CC(0, j2 + 1, k) = CH(0, k, jc);
  }
  if (ido > 1) {
    PF_FOR(t, (ipph - 1) * l1 * hp) {
      const int j = 1 + t / (l1 * hp), r = t - (j - 1) * l1 * hp, k = r / hp, q = r - k * hp;
      const int jc = ip - j, j2 = 2 * j - 1, i = 1 + 2 * q, ic = ido - i - 2;
      CC(i, j2 + 1, k) = CH(i, k, j) + CH(i, k, jc);
      CC(ic, j2, k) = CH(i, k, j) - CH(i, k, jc);
      CC(i + 1, j2 + 1, k) = CH(i + 1, k, j) + CH(i + 1, k, jc);
      CC(ic + 1, j2, k) = CH(i + 1, k, jc) - CH(i + 1, k, j);
    }
  }
#undef CC
#undef CH
#undef C1
#undef C2
#undef CH2
}

#define CC(a, b, c) cc[(a) + ido * ((b) + IP * (c))]
#define CH(a, b, c) ch[(a) + ido * ((b) + l1 * (c))]
#define WA(x, i) wa[(i) + (x) * (ido - 1)]

__device__ void radb2(int ido, int l1, const double* __restrict__ cc, double* __restrict__ ch, const double* wa) {
  constexpr int IP = 2;
  PF_FOR(k, l1) {
    CH(0, k, 0) = CC(0, 0, k) + CC(ido - 1, 1, k);
    CH(0, k, 1) = CC(0, 0, k) - CC(ido - 1, 1, k);
    if ((ido & 1) == 0) {
      CH(ido - 1, k, 0) = 2 * CC(ido - 1, 0, k);
      CH(ido - 1, k, 1) = -2 * CC(0, 1, k);
    }
  }
  if (ido <= 2) return;
  const int hi = (ido - 1) / 2;
  PF_FOR(t, l1 * hi) {
    const int k = t / hi, i = 2 + 2 * (t - k * hi), ic = ido - i;
    CH(i - 1, k, 0) = CC(i - 1, 0, k) + CC(ic - 1, 1, k);
    const double tr2 = CC(i - 1, 0, k) - CC(ic - 1, 1, k);
    const double ti2 = CC(i, 0, k) + CC(ic, 1, k);
    CH(i, k, 0) = CC(i, 0, k) - CC(ic, 1, k);
    CH(i, k, 1) = WA(0, i - 2) * ti2 + WA(0, i - 1) * tr2;
    CH(i - 1, k, 1) = WA(0, i - 2) * tr2 - WA(0, i - 1) * ti2;
  }
}

__device__ void radb3(int ido, int l1, const double* __restrict__ cc, double* __restrict__ ch, const double* wa) {
  constexpr int IP = 3;
  const double taur = -0.5, taui = 0.8660254037844386467637231707529362;
  PF_FOR(k, l1) {
    const double tr2 = 2 * CC(ido - 1, 1, k);
    const double cr2 = CC(0, 0, k) + taur * tr2;
    CH(0, k, 0) = CC(0, 0, k) + tr2;
    const double ci3 = 2 * taui * CC(0, 2, k);
    CH(0, k, 2) = cr2 + ci3;
    CH(0, k, 1) = cr2 - ci3;
  }
  if (ido == 1) return;
  const int hi = (ido - 1) / 2;
  PF_FOR(t, l1 * hi) {
    const int k = t / hi, i = 2 + 2 * (t - k * hi), ic = ido - i;
    const double tr2 = CC(i - 1, 2, k) + CC(ic - 1, 1, k);
    const double ti2 = CC(i, 2, k) - CC(ic, 1, k);
    const double cr2 = CC(i - 1, 0, k) + taur * tr2;
    const double ci2 = CC(i, 0, k) + taur * ti2;
    CH(i - 1, k, 0) = CC(i - 1, 0, k) + tr2;
    CH(i, k, 0) = CC(i, 0, k) + ti2;
    const double cr3 = taui * (CC(i - 1, 2, k) - CC(ic - 1, 1, k));
    const double ci3 = taui * (CC(i, 2, k) + CC(ic, 1, k));
    const double dr3 = cr2 + ci3, dr2 = cr2 - ci3;
    const double di2 = ci2 + cr3, di3 = ci2 - cr3;
    CH(i, k, 1) = WA(0, i - 2) * di2 + WA(0, i - 1) * dr2;
    CH(i - 1, k, 1) = WA(0, i - 2) * dr2 - WA(0, i - 1) * di2;
    CH(i, k, 2) = WA(1, i - 2) * di3 + WA(1, i - 1) * dr3;
    CH(i - 1, k, 2) = WA(1, i - 2) * dr3 - WA(1, i - 1) * di3;
  }
}

__device__ void radb4(int ido, int l1, const double* __restrict__ cc, double* __restrict__ ch, const double* wa) {
  constexpr int IP = 4;
  const double sqrt2 = 1.414213562373095048801688724209698;
  PF_FOR(k, l1) {
    const double tr2 = CC(0, 0, k) + CC(ido - 1, 3, k), tr1 = CC(0, 0, k) - CC(ido - 1, 3, k);
    const double tr3 = 2 * CC(ido - 1, 1, k);
    const double tr4 = 2 * CC(0, 2, k);
    CH(0, k, 0) = tr2 + tr3;
    CH(0, k, 2) = tr2 - tr3;
    CH(0, k, 3) = tr1 + tr4;
    CH(0, k, 1) = tr1 - tr4;
    if ((ido & 1) == 0) {
      const double ti1 = CC(0, 3, k) + CC(0, 1, k), ti2 = CC(0, 3, k) - CC(0, 1, k);
      const double tr2b = CC(ido - 1, 0, k) + CC(ido - 1, 2, k), tr1b = CC(ido - 1, 0, k) - CC(ido - 1, 2, k);
      CH(ido - 1, k, 0) = tr2b + tr2b;
      CH(ido - 1, k, 1) = sqrt2 * (tr1b - ti1);
      CH(ido - 1, k, 2) = ti2 + ti2;
      CH(ido - 1, k, 3) = -sqrt2 * (tr1b + ti1);
    }
  }
  if (ido <= 2) return;
  const int hi = (ido - 1) / 2;
  PF_FOR(t, l1 * hi) {
    const int k = t / hi, i = 2 + 2 * (t - k * hi), ic = ido - i;
    const double tr2 = CC(i - 1, 0, k) + CC(ic - 1, 3, k), tr1 = CC(i - 1, 0, k) - CC(ic - 1, 3, k);
    const double ti1 = CC(i, 0, k) + CC(ic, 3, k), ti2 = CC(i, 0, k) - CC(ic, 3, k);
    const double tr4 = CC(i, 2, k) + CC(ic, 1, k), ti3 = CC(i, 2, k) - CC(ic, 1, k);
    const double tr3 = CC(i - 1, 2, k) + CC(ic - 1, 1, k), ti4 = CC(i - 1, 2, k) - CC(ic - 1, 1, k);
    CH(i - 1, k, 0) = tr2 + tr3;
    const double cr3 = tr2 - tr3;
    CH(i, k, 0) = ti2 + ti3;
    const double ci3 = ti2 - ti3;
    const double cr4 = tr1 + tr4, cr2 = tr1 - tr4;
    const double ci2 = ti1 + ti4, ci4 = ti1 - ti4;
    CH(i, k, 1) = WA(0, i - 2) * ci2 + WA(0, i - 1) * cr2;
    CH(i - 1, k, 1) = WA(0, i - 2) * cr2 - WA(0, i - 1) * ci2;
    CH(i, k, 2) = WA(1, i - 2) * ci3 + WA(1, i - 1) * cr3;
    CH(i - 1, k, 2) = WA(1, i - 2) * cr3 - WA(1, i - 1) * ci3;
    CH(i, k, 3) = WA(2, i - 2) * ci4 + WA(2, i - 1) * cr4;
    CH(i - 1, k, 3) = WA(2, i - 2) * cr4 - WA(2, i - 1) * ci4;
  }
}

__device__ void radb5(int ido, int l1, const double* __restrict__ cc, double* __restrict__ ch, const double* wa) {
  constexpr int IP = 5;
  const double tr11 = 0.3090169943749474241022934171828191, ti11 = 0.9510565162951535721164393333793821;
  const double tr12 = -0.8090169943749474241022934171828191, ti12 = 0.5877852522924731291687059546390728;
  PF_FOR(k, l1) {
    const double ti5 = CC(0, 2, k) + CC(0, 2, k);
    const double ti4 = CC(0, 4, k) + CC(0, 4, k);
    const double tr2 = CC(ido - 1, 1, k) + CC(ido - 1, 1, k);
    const double tr3 = CC(ido - 1, 3, k) + CC(ido - 1, 3, k);
    CH(0, k, 0) = CC(0, 0, k) + tr2 + tr3;
    const double cr2 = CC(0, 0, k) + tr11 * tr2 + tr12 * tr3;
    const double cr3 = CC(0, 0, k) + tr12 * tr2 + tr11 * tr3;
    const double ci5 = ti5 * ti11 + ti4 * ti12, ci4 = ti5 * ti12 - ti4 * ti11;
    CH(0, k, 4) = cr2 + ci5;
    CH(0, k, 1) = cr2 - ci5;
    CH(0, k, 3) = cr3 + ci4;
    CH(0, k, 2) = cr3 - ci4;
  }
  if (ido == 1) return;
  const int hi = (ido - 1) / 2;
  PF_FOR(t, l1 * hi) {
    const int k = t / hi, i = 2 + 2 * (t - k * hi), ic = ido - i;
    const double tr2 = CC(i - 1, 2, k) + CC(ic - 1, 1, k), tr5 = CC(i - 1, 2, k) - CC(ic - 1, 1, k);
    const double ti5 = CC(i, 2, k) + CC(ic, 1, k), ti2 = CC(i, 2, k) - CC(ic, 1, k);
    const double tr3 = CC(i - 1, 4, k) + CC(ic - 1, 3, k), tr4 = CC(i - 1, 4, k) - CC(ic - 1, 3, k);
    const double ti4 = CC(i, 4, k) + CC(ic, 3, k), ti3 = CC(i, 4, k) - CC(ic, 3, k);
    CH(i - 1, k, 0) = CC(i - 1, 0, k) + tr2 + tr3;
    CH(i, k, 0) = CC(i, 0, k) + ti2 + ti3;
    const double cr2 = CC(i - 1, 0, k) + tr11 * tr2 + tr12 * tr3;
    const double ci2 = CC(i, 0, k) + tr11 * ti2 + tr12 * ti3;
    const double cr3 = CC(i - 1, 0, k) + tr12 * tr2 + tr11 * tr3;
    const double ci3 = CC(i, 0, k) + tr12 * ti2 + tr11 * ti3;
    const double cr5 = tr5 * ti11 + tr4 * ti12, cr4 = tr5 * ti12 - tr4 * ti11;
    const double ci5 = ti5 * ti11 + ti4 * ti12, ci4 = ti5 * ti12 - ti4 * ti11;
    const double dr4 = cr3 + ci4, dr3 = cr3 - ci4;
    const double di3 = ci3 + cr4, di4 = ci3 - cr4;
    const double dr5 = cr2 + ci5, dr2 = cr2 - ci5;
    const double di2 = ci2 + cr5, di5 = ci2 - cr5;
    CH(i, k, 1) = WA(0, i - 2) * di2 + WA(0, i - 1) * dr2;
    CH(i - 1, k, 1) = WA(0, i - 2) * dr2 - WA(0, i - 1) * di2;
    CH(i, k, 2) = WA(1, i - 2) * di3 + WA(1, i - 1) * dr3;
    CH(i - 1, k, 2) = WA(1, i - 2) * dr3 - WA(1, i - 1) * di3;
    CH(i, k, 3) = WA(2, i - 2) * di4 + WA(2, i - 1) * dr4;
    CH(i - 1, k, 3) = WA(2, i - 2) * dr4 - WA(2, i - 1) * di4;
    CH(i, k, 4) = WA(3, i - 2) * di5 + WA(3, i - 1) * dr5;
    CH(i - 1, k, 4) = WA(3, i - 2) * dr5 - WA(3, i - 1) * di5;
  }
}
#undef CC
#undef CH
#undef WA

// generic backward pass (ip odd > 5, ido odd): the result lands in ch
__device__ void radbg(int ido, int ip, int l1, double* cc, double* ch, const double* wa,
                      const double* csarr) {
  const int cdim = ip, ipph = (ip + 1) / 2, idl1 = ido * l1;
#define CC(a, b, c) cc[(a) + ido * ((b) + cdim * (c))]
#define CH(a, b, c) ch[(a) + ido * ((b) + l1 * (c))]
#define C1(a, b, c) cc[(a) + ido * ((b) + l1 * (c))]
#define C2(a, b) cc[(a) + idl1 * (b)]
#define CH2(a, b) ch[(a) + idl1 * (b)]
  const int hp = (ido - 1) / 2;
  // phase 1: unpack the halfcomplex columns into CH
  PF_FOR(t, l1 * ido) {
    const int k = t / ido, i = t - k * ido;
    CH(i, k, 0) = CC(i, 0, k);
  }
  PF_FOR(t, (ipph - 1) * l1 * (hp + 1)) {
    const int j = 1 + t / (l1 * (hp + 1)), r = t - (j - 1) * l1 * (hp + 1), k = r / (hp + 1),
                  q = r - k * (hp + 1), jc = ip - j, j2 = 2 * j - 1;
    if (q == 0) {
      CH(0, k, j) = 2 * CC(ido - 1, j2, k);
      CH(0, k, jc) = 2 * CC(0, j2 + 1, k);
    } else {
      const int i = 2 * q - 1, ic = ido - i - 2;
      CH(i, k, j) = CC(i, j2 + 1, k) + CC(ic, j2, k);
      CH(i, k, jc) = CC(i, j2 + 1, k) - CC(ic, j2, k);
      CH(i + 1, k, j) = CC(i + 1, j2 + 1, k) - CC(ic + 1, j2, k);
      CH(i + 1, k, jc) = CC(i + 1, j2 + 1, k) + CC(ic + 1, j2, k);
    }
  }
  __syncthreads();
  // phase 2: the column DFT (into C2, columns >= 1), then CH2 column 0's sum
  PF_FOR(ik, idl1) {
    for (int l = 1, lc = ip - 1; l < ipph; ++l, --lc) {
      double a = CH2(ik, 0) + csarr[2 * l] * CH2(ik, 1) + csarr[4 * l] * CH2(ik, 2);
      double b = csarr[2 * l + 1] * CH2(ik, ip - 1) + csarr[4 * l + 1] * CH2(ik, ip - 2);
      int iang = 2 * l;
      int j = 3, jc = ip - 3;
      for (; j < ipph - 3; j += 4, jc -= 4) {
        iang += l;
        if (iang > ip) iang -= ip;
        const double ar1 = csarr[2 * iang], ai1 = csarr[2 * iang + 1];
        iang += l;
        if (iang > ip) iang -= ip;
        const double ar2 = csarr[2 * iang], ai2 = csarr[2 * iang + 1];
        iang += l;
        if (iang > ip) iang -= ip;
        const double ar3 = csarr[2 * iang], ai3 = csarr[2 * iang + 1];
        iang += l;
        if (iang > ip) iang -= ip;
        const double ar4 = csarr[2 * iang], ai4 = csarr[2 * iang + 1];
        a += ar1 * CH2(ik, j) + ar2 * CH2(ik, j + 1) + ar3 * CH2(ik, j + 2) + ar4 * CH2(ik, j + 3);
        b += ai1 * CH2(ik, jc) + ai2 * CH2(ik, jc - 1) + ai3 * CH2(ik, jc - 2) + ai4 * CH2(ik, jc - 3);
      }
      for (; j < ipph - 1; j += 2, jc -= 2) {
        iang += l;
        if (iang > ip) iang -= ip;
        const double ar1 = csarr[2 * iang], ai1 = csarr[2 * iang + 1];
        iang += l;
        if (iang > ip) iang -= ip;
        const double ar2 = csarr[2 * iang], ai2 = csarr[2 * iang + 1];
        a += ar1 * CH2(ik, j) + ar2 * CH2(ik, j + 1);
        b += ai1 * CH2(ik, jc) + ai2 * CH2(ik, jc - 1);
      }
      for (; j < ipph; ++j, --jc) {
        iang += l;
        if (iang > ip) iang -= ip;
        const double war = csarr[2 * iang], wai = csarr[2 * iang + 1];
        a += war * CH2(ik, j);
        b += wai * CH2(ik, jc);
      }
      C2(ik, l) = a;
      C2(ik, lc) = b;
    }
    double s = CH2(ik, 0);
    for (int j = 1; j < ipph; ++j) s += CH2(ik, j);
    CH2(ik, 0) = s;
  }
  __syncthreads();
  // phase 3: recombine the pairs into CH, then the twiddles (same thread, same elements)
  PF_FOR(t, (ipph - 1) * l1 * (hp + 1)) {
    const int j = 1 + t / (l1 * (hp + 1)), r = t - (j - 1) * l1 * (hp + 1), k = r / (hp + 1),
                  q = r - k * (hp + 1), jc = ip - j;
    if (q == 0) {
      CH(0, k, jc) = C1(0, k, j) + C1(0, k, jc);
      CH(0, k, j) = C1(0, k, j) - C1(0, k, jc);
    } else {
      const int i = 2 * q - 1;
      const double a = C1(i, k, j) - C1(i + 1, k, jc), b = C1(i, k, j) + C1(i + 1, k, jc);
      const double c = C1(i + 1, k, j) + C1(i, k, jc), d = C1(i + 1, k, j) - C1(i, k, jc);
      const int is = (j - 1) * (ido - 1) + (i - 1), isc = (jc - 1) * (ido - 1) + (i - 1);
      CH(i, k, j) = wa[is] * a - wa[is + 1] * c;
      CH(i + 1, k, j) = wa[is] * c + wa[is + 1] * a;
      CH(i, k, jc) = wa[isc] * b - wa[isc + 1] * d;
      CH(i + 1, k, jc) = wa[isc] * d + wa[isc + 1] * b;
    }
  }
#undef CC
#undef CH
#undef C1
#undef C2
#undef CH2
}

// c (P.len) in place, scratch ch (P.len); r2hc: forward (halfcomplex out), else backward
__device__ void rfftp(const PfPasses& P, const double* pool, double* c, double* ch, double fct, bool r2hc) {
  const int n = P.len;
  if (n == 1) {
    if (threadIdx.x == 0) c[0] *= fct;
    __syncthreads();
    return;
  }
  double *p1 = c, *p2 = ch;
  for (int k1 = 0; k1 < P.nf; ++k1) {
    const int k = r2hc ? P.nf - k1 - 1 : k1;
    const PfFact F = P.f[k];
    const double* wa = pool + (F.tw >= 0 ? F.tw : 0);
    const double* ws = pool + (F.tws >= 0 ? F.tws : 0);
    bool swap = true;
    if (r2hc) {
      switch (F.ip) {
        case 4: radf4(F.ido, F.l1, p1, p2, wa); break;
        case 2: radf2(F.ido, F.l1, p1, p2, wa); break;
        case 3: radf3(F.ido, F.l1, p1, p2, wa); break;
        case 5: radf5(F.ido, F.l1, p1, p2, wa); break;
        default: radfg(F.ido, F.ip, F.l1, p1, p2, wa, ws); swap = false;
      }
    } else {
      switch (F.ip) {
        case 4: radb4(F.ido, F.l1, p1, p2, wa); break;
        case 2: radb2(F.ido, F.l1, p1, p2, wa); break;
        case 3: radb3(F.ido, F.l1, p1, p2, wa); break;
        case 5: radb5(F.ido, F.l1, p1, p2, wa); break;
        default: radbg(F.ido, F.ip, F.l1, p1, p2, wa, ws);
      }
    }
    if (swap) {
      double* t = p1;
      p1 = p2;
      p2 = t;
    }
    __syncthreads();
  }
  // copy_and_norm
  if (p1 != c) {
    PF_FOR(i, n) c[i] = fct != 1.0 ? fct * p1[i] : p1[i];
  } else if (fct != 1.0) {
    PF_FOR(i, n) c[i] *= fct;
  }
  __syncthreads();
}

// one unfused forward real pass over the whole array: in -> out (radfg's
// result lands in its input, then copied)
__device__ inline void radf_whole(const PfPasses& P, const PfFact& F, const double* pool, double* in, double* out) {
  const double* wa = pool + (F.tw >= 0 ? F.tw : 0);
  switch (F.ip) {
    case 4: radf4(F.ido, F.l1, in, out, wa); break;
    case 2: radf2(F.ido, F.l1, in, out, wa); break;
    case 3: radf3(F.ido, F.l1, in, out, wa); break;
    case 5: radf5(F.ido, F.l1, in, out, wa); break;
    default:
      radfg(F.ido, F.ip, F.l1, in, out, wa, pool + (F.tws >= 0 ? F.tws : 0));
      __syncthreads();
      PF_FOR(i, P.len) out[i] = in[i];
  }
  __syncthreads();
}

// ---- "pair" groups: the trailing radf4 / radf2 passes from an even ido D ----
// (pocketfft.h, Q = 2).  A tile holds two runs of residues mod D -- run A
// (slots 0 .. na-1) and run B (slots na .. na+nb-1) -- times all P = n / D
// blocks w, at lds[w * R + slot]; element (a, w) is position a + D w.  Within
// a pass of ido = D B, position a' = res + D blk; the butterflies below are
// radf4 / radf2's own expressions on explicit (residue, block) references.
struct PairTile {
  int a0, na, b0, nb, R;
  __device__ int slot(int res) const { return (res >= a0 && res < a0 + na) ? res - a0 : na + (res - b0); }
};
__device__ inline PairTile pair_tile(int tile, int D, int T) {
  PairTile t;
  if (tile == 0) {   // the class {0, D - 1}
    t.a0 = 0;
    t.na = 1;
    t.b0 = D - 1;
    t.nb = 1;
  } else {
    const int H = D / 2, pmax = H / 2;
    const int p0 = 1 + (tile - 1) * T, p1 = min(p0 + T, pmax + 1);
    const int pe = (2 * (p1 - 1) == H) ? p1 - 1 : p1;   // p = H / 2 pairs with itself
    t.a0 = 2 * p0 - 1;
    t.na = 2 * (p1 - p0);
    t.b0 = 2 * (H - pe) + 1;
    t.nb = 2 * (pe - p0);
  }
  t.R = t.na + t.nb;
  return t;
}
__device__ inline int pair_tiles(int D, int T) { return 1 + ((D / 2) / 2 + T - 1) / T; }

// radf4's butterflies: x[m] = CC(i-1, k, m), y[m] = CC(i, k, m) in; lo[b] =
// CH(i-1, b, k) for b = 0, 2 and CH(ic-1, b, k) for b = 1, 3; hi[b] likewise
// at i / ic
__device__ __forceinline__ void radf4_bf(const double* x, const double* y, int i, int ido, const double* wa,
                                         double* lo, double* hi) {
#define WA(q, j) wa[(j) + (q) * (ido - 1)]
  const double cr2 = WA(0, i - 2) * x[1] + WA(0, i - 1) * y[1];
  const double ci2 = WA(0, i - 2) * y[1] - WA(0, i - 1) * x[1];
  const double cr3 = WA(1, i - 2) * x[2] + WA(1, i - 1) * y[2];
  const double ci3 = WA(1, i - 2) * y[2] - WA(1, i - 1) * x[2];
  const double cr4 = WA(2, i - 2) * x[3] + WA(2, i - 1) * y[3];
  const double ci4 = WA(2, i - 2) * y[3] - WA(2, i - 1) * x[3];
#undef WA
  const double tr1 = cr4 + cr2, tr4 = cr4 - cr2;
  const double ti1 = ci2 + ci4, ti4 = ci2 - ci4;
  const double tr2 = x[0] + cr3, tr3 = x[0] - cr3;
  const double ti2 = y[0] + ci3, ti3 = y[0] - ci3;
  lo[0] = tr2 + tr1;
  lo[3] = tr2 - tr1;
  hi[0] = ti1 + ti2;
  hi[3] = ti1 - ti2;
  lo[2] = tr3 + ti4;
  lo[1] = tr3 - ti4;
  hi[2] = tr4 + ti3;
  hi[1] = tr4 - ti3;
}
// column 0 (c[m] = CC(0, k, m)): z0[b] = CH(0, b, k) for b = 0, 2; zl[b] = CH(ido-1, b, k) for b = 1, 3
__device__ __forceinline__ void radf4_c0(const double* c, double* z0, double* zl) {
  const double tr1 = c[3] + c[1];
  z0[2] = c[3] - c[1];
  const double tr2 = c[0] + c[2];
  zl[1] = c[0] - c[2];
  z0[0] = tr2 + tr1;
  zl[3] = tr2 - tr1;
}
// column ido - 1 (c[m] = CC(ido-1, k, m)): zl[b] = CH(ido-1, b, k) for b = 0, 2; z0[b] = CH(0, b, k) for b = 1, 3
__device__ __forceinline__ void radf4_cl(const double* c, double* z0, double* zl) {
  const double hsqt2 = 0.707106781186547524400844362104849;
  const double ti1 = -hsqt2 * (c[1] + c[3]);
  const double tr1b = hsqt2 * (c[1] - c[3]);
  zl[0] = c[0] + tr1b;
  zl[2] = c[0] - tr1b;
  z0[3] = ti1 + c[2];
  z0[1] = ti1 - c[2];
}
// radf2's: lo[0] = CH(i-1, 0, k), lo[1] = CH(ic-1, 1, k); hi likewise
__device__ __forceinline__ void radf2_bf(const double* x, const double* y, int i, const double* wa, double* lo,
                                         double* hi) {
  const double tr2 = wa[i - 2] * x[1] + wa[i - 1] * y[1];
  const double ti2 = wa[i - 2] * y[1] - wa[i - 1] * x[1];
  lo[0] = x[0] + tr2;
  lo[1] = x[0] - tr2;
  hi[0] = ti2 + y[0];
  hi[1] = ti2 - y[0];
}
__device__ __forceinline__ void radf2_c0(const double* c, double* z0, double* zl) {
  z0[0] = c[0] + c[1];
  zl[1] = c[0] - c[1];
}
__device__ __forceinline__ void radf2_cl(const double* c, double* z0, double* zl) {
  z0[1] = -c[1];
  zl[0] = c[0];
}

// one radf<IP> pass (ido = D B, l1) over a pair tile: cur -> nxt
template <int IP>
__device__ __forceinline__ void rpair_pass(const double* cur, double* nxt, const PairTile& T, bool special, int D,
                                           int B, int l1, const double* wa, const FDiv& fnp, const PfDiv* dvp) {
  const int ido = D * B, R = T.R;
  // input CC(res + D blk, k, m) at w = blk + B (k + l1 m); output CH(res + D blk, b, k) at w = blk + B (b + IP k)
  auto ldx = [&](int res, int blk, int k, int m) { return cur[(blk + B * (k + l1 * m)) * R + T.slot(res)]; };
  auto stx = [&](int res, int blk, int b, int k, double v) { nxt[(blk + B * (b + IP * k)) * R + T.slot(res)] = v; };
  if (!special) {
    const int np = R / 2, nbf = l1 * B * np;
    const FDiv fB(dvp[0]);
    for (int t = threadIdx.x; t < nbf; t += blockDim.x) {
      const int r = fnp.div(t), u = t - r * np, k = fB.div(r), blk = r - k * B;
      const int ae = u < T.na / 2 ? T.a0 + 1 + 2 * u : T.b0 + 1 + 2 * (u - T.na / 2);   // residue of i (even)
      const int i = ae + D * blk, rc = D - ae, bc = B - 1 - blk;                        // ic = rc + D bc
      double x[IP], y[IP], lo[IP], hi[IP];
#pragma unroll
      for (int m = 0; m < IP; ++m) {
        x[m] = ldx(ae - 1, blk, k, m);
        y[m] = ldx(ae, blk, k, m);
      }
      if constexpr (IP == 4) radf4_bf(x, y, i, ido, wa, lo, hi);
      else radf2_bf(x, y, i, wa, lo, hi);
#pragma unroll
      for (int b = 0; b < IP; ++b) {
        if ((b & 1) == 0) {
          stx(ae - 1, blk, b, k, lo[b]);
          stx(ae, blk, b, k, hi[b]);
        } else {
          stx(rc - 1, bc, b, k, lo[b]);
          stx(rc, bc, b, k, hi[b]);
        }
      }
    }
  } else {
    // columns 0 and ido - 1, and the pairs (i - 1, i) = (D - 1 of block c - 1, 0 of block c), c = 1 .. B - 1
    const int nbf = l1 * (B + 1);
    const FDiv fB1(dvp[1]);
    for (int t = threadIdx.x; t < nbf; t += blockDim.x) {
      const int k = fB1.div(t), c = t - k * (B + 1);
      double x[IP], y[IP], lo[IP], hi[IP];
      if (c == 0 || c == B) {
        double z0[IP], zl[IP];
#pragma unroll
        for (int m = 0; m < IP; ++m) x[m] = c == 0 ? ldx(0, 0, k, m) : ldx(D - 1, B - 1, k, m);
        if (c == 0) {
          if constexpr (IP == 4) radf4_c0(x, z0, zl);
          else radf2_c0(x, z0, zl);
        } else {
          if constexpr (IP == 4) radf4_cl(x, z0, zl);
          else radf2_cl(x, z0, zl);
        }
        // column 0 fills CH(0, even b) and CH(ido-1, odd b); column ido-1 the others
#pragma unroll
        for (int b = 0; b < IP; ++b) {
          const bool to0 = ((b & 1) == 0) == (c == 0);
          if (to0) stx(0, 0, b, k, z0[b]);
          else stx(D - 1, B - 1, b, k, zl[b]);
        }
      } else {
        const int i = D * c;   // ic = D (B - c): residue 0 of block B - c, ic - 1 = D - 1 of block B - c - 1
#pragma unroll
        for (int m = 0; m < IP; ++m) {
          x[m] = ldx(D - 1, c - 1, k, m);
          y[m] = ldx(0, c, k, m);
        }
        if constexpr (IP == 4) radf4_bf(x, y, i, ido, wa, lo, hi);
        else radf2_bf(x, y, i, wa, lo, hi);
#pragma unroll
        for (int b = 0; b < IP; ++b) {
          if ((b & 1) == 0) {
            stx(D - 1, c - 1, b, k, lo[b]);
            stx(0, c, b, k, hi[b]);
          } else {
            stx(D - 1, B - c - 1, b, k, lo[b]);
            stx(0, B - c, b, k, hi[b]);
          }
        }
      }
    }
  }
}

// a pair group over the whole array: in (or src, first group) -> out
template <class Src, class Wr>
__device__ __forceinline__ void rgroup_pairs(const PfPasses& P, const PfGroup& Gr, const double* pool, Src src,
                                             bool first, const double* in, Wr wr, double* lds) {
  const int D = Gr.D, Pp = Gr.P, Tn = Gr.Qk;
  const int ntiles = pair_tiles(D, Tn);
  for (int tile = 0; tile < ntiles; ++tile) {
    const PairTile T = pair_tile(tile, D, Tn);
    const int R = T.R, ne = R * Pp;
    double* cur = lds;
    double* nxt = lds + kPfTileDoubles;
    const int kind = tile == 0 ? 0 : (tile == ntiles - 1 ? 4 : 2);   // Gr.dv: R, R / 2 of this tile's kind
    const FDiv fR(Gr.dv[kind]), fnp(Gr.dv[kind + 1]);
    for (int e = threadIdx.x; e < ne; e += blockDim.x) {   // (w, slot): runs A and B of each block
      const int w = fR.div(e), sl = e - w * R;
      const int res = sl < T.na ? T.a0 + sl : T.b0 + (sl - T.na);
      const int pos = res + D * w;
      cur[e] = first ? src(pos) : in[pos];
    }
    __syncthreads();
    int B = 1;
    for (int q = Gr.f0; q > Gr.f0 - Gr.nf; --q) {
      const PfFact F = P.f[q];
      const double* wa = pool + (F.tw >= 0 ? F.tw : 0);
      if (F.ip == 4) rpair_pass<4>(cur, nxt, T, tile == 0, D, B, (int)F.l1, wa, fnp, F.dv);
      else rpair_pass<2>(cur, nxt, T, tile == 0, D, B, (int)F.l1, wa, fnp, F.dv);
      __syncthreads();
      double* t = cur;
      cur = nxt;
      nxt = t;
      B *= (int)F.ip;
    }
    for (int e = threadIdx.x; e < ne; e += blockDim.x) {
      const int w = fR.div(e), sl = e - w * R;
      const int res = sl < T.na ? T.a0 + sl : T.b0 + (sl - T.na);
      wr(res + D * w, cur[e]);
    }
    __syncthreads();
  }
}

// pocketfft's rfftp forward (r2hc, fct 1) of the sequence src(0 .. n-1) into
// f (halfcomplex); tmp: n doubles of scratch; src must read neither f nor
// tmp.  Groups in executed order (pocketfft.h), the last one writing f;
// lds: 2 * kPfTileDoubles doubles.
// fin(i, v): where the halfcomplex result goes (WrD{f}: into f).  A fin
// other than f may alias src's storage element for element: src is read by
// the first group only, fin written by the last (one group: a single tile, or
// pair tiles, each of which reads and writes the same positions).
template <class Src, bool LEAN = false, class Fin = WrD>
__device__ __forceinline__ void rfftp_fwd_fused(const PfPasses& P, const double* pool, Src src, double* f, double* tmp,
                                                double* lds, Fin fin = Fin{nullptr}) {
  const int G = P.ng;
  if constexpr (std::is_same<Fin, WrD>::value)
    if (fin.p == nullptr) fin.p = f;
  auto outbuf = [&](int g) { return ((G - 1 - g) & 1) == 0 ? f : tmp; };
  for (int g = 0; g < G; ++g) {
    const PfGroup& Gr = P.g[g];
    const bool last = g == G - 1;
    double* out = outbuf(g);
    double* in = g == 0 ? nullptr : outbuf(g - 1);
    if (Gr.Q == 2) {
      if (last) rgroup_pairs(P, Gr, pool, src, g == 0, in, fin, lds);
      else rgroup_pairs(P, Gr, pool, src, g == 0, in, WrD{out}, lds);
      continue;
    }
    if (Gr.Q == 0) {
      if (g == 0) {   // materialise the source in the other buffer
        in = out == f ? tmp : f;
        PF_FOR(i, P.len) in[i] = src(i);
        __syncthreads();
      }
      if constexpr (LEAN) {   // hard-coded radices only (pf_hilbert_lean)
        const PfFact& F = P.f[Gr.f0];
        const double* wa = pool + (F.tw >= 0 ? F.tw : 0);
        switch (F.ip) {
          case 4: radf4(F.ido, F.l1, in, out, wa); break;
          case 2: radf2(F.ido, F.l1, in, out, wa); break;
          case 3: radf3(F.ido, F.l1, in, out, wa); break;
          default: radf5(F.ido, F.l1, in, out, wa); break;
        }
        __syncthreads();
      } else {
        radf_whole(P, P.f[Gr.f0], pool, in, out);
      }
      if (last) {
        bool direct = false;
        if constexpr (std::is_same<Fin, WrD>::value) direct = fin.p == out;
        if (!direct) {
          PF_FOR(i, P.len) fin(i, out[i]);
          __syncthreads();
        }
      }
      continue;
    }
    const int D = Gr.D, Pp = Gr.P, Lr = Gr.L, DP = D * Pp;
    const int Qk = Gr.Qk;
    const bool pre = blockDim.x == kPfThreadsPre;
    const FDiv fD(Gr.dv[0]);
    double pv[kPfPreR];
    // global a + D (k + Lr w) -> local k DP + a + D w, in memory order (w, k, a)
    auto issue = [&](int k0) {
      const int qk = Lr - k0 < Qk ? Lr - k0 : Qk, ne = qk * DP;
      const FDiv fqk(qk == Qk ? Gr.dv[1] : Gr.dv[2]);
#pragma unroll
      for (int u = 0; u < kPfPreR; ++u) {
        const int e = (int)threadIdx.x + u * kPfThreadsPre;
        if (e < ne) {
          const int r = fD.div(e), a = e - r * D, w = fqk.div(r), kk = r - w * qk;
          const int pos = a + D * (k0 + kk) + D * Lr * w;
          pv[u] = g == 0 ? src(pos) : in[pos];
        }
      }
    };
    if (pre) issue(0);
    for (int k0 = 0; k0 < Lr; k0 += Qk) {
      const int qk = Lr - k0 < Qk ? Lr - k0 : Qk;
      double* cur = lds;
      double* nxt = lds + kPfTileDoubles;
      const int ne = qk * DP;
      const FDiv fqk(qk == Qk ? Gr.dv[1] : Gr.dv[2]);
      if (pre) {
#pragma unroll
        for (int u = 0; u < kPfPreR; ++u) {
          const int e = (int)threadIdx.x + u * kPfThreadsPre;
          if (e < ne) {
            const int r = fD.div(e), a = e - r * D, w = fqk.div(r), kk = r - w * qk;
            cur[kk * DP + a + D * w] = pv[u];
          }
        }
      } else {
        for (int e = threadIdx.x; e < ne; e += blockDim.x) {
          const int r = fD.div(e), a = e - r * D, w = fqk.div(r), kk = r - w * qk;
          const int pos = a + D * (k0 + kk) + D * Lr * w;
          cur[kk * DP + a + D * w] = g == 0 ? src(pos) : in[pos];
        }
      }
      __syncthreads();
      if (pre && k0 + Qk < Lr) issue(k0 + Qk);
      for (int q = Gr.f0; q > Gr.f0 - Gr.nf; --q) {
        const PfFact F = P.f[q];
        const double* wa = pool + (F.tw >= 0 ? F.tw : 0);
        const int l1l = F.l1l;
        switch (F.ip) {
          case 4: radf4(F.ido, l1l, cur, nxt, wa, qk, DP, F.dv); break;
          case 2: radf2(F.ido, l1l, cur, nxt, wa, qk, DP, F.dv); break;
          case 3: radf3(F.ido, l1l, cur, nxt, wa, qk, DP, F.dv); break;
          default: radf5(F.ido, l1l, cur, nxt, wa, qk, DP, F.dv); break;
        }
        __syncthreads();
        double* t = cur;
        cur = nxt;
        nxt = t;
      }
      // blocks k0 .. k0 + qk - 1 are contiguous in the output
      if (last)
        for (int e = threadIdx.x; e < ne; e += blockDim.x) fin(k0 * DP + e, cur[e]);
      else
        for (int e = threadIdx.x; e < ne; e += blockDim.x) out[k0 * DP + e] = cur[e];
      __syncthreads();
    }
  }
}

// ============================ Bluestein =====================================
template <bool FWD>
__device__ void blue_fft(const PfBlue& B, const double* pool, Cx* c, Cx* akf, Cx* ch, double fct, Cx* lds) {
  const int n = B.n, n2 = B.n2;
  const Cx* bk = reinterpret_cast<const Cx*>(pool + B.bk);
  const Cx* bkf = reinterpret_cast<const Cx*>(pool + B.bkf);
  const Cx zero = scale(smul<FWD>(c[0], bk[0]), 0.);
  PF_FOR(m, n2) akf[m] = m < n ? smul<FWD>(c[m], bk[m]) : zero;
  __syncthreads();
  cfftp<true>(B.plan, pool, akf, ch, 1., lds);
  // the convolution
  PF_FOR(m, n2) akf[m] = smul<!FWD>(akf[m], bkf[2 * m <= n2 ? m : n2 - m]);
  __syncthreads();
  cfftp<false>(B.plan, pool, akf, ch, 1., lds);
  PF_FOR(m, n) c[m] = scale(smul<FWD>(akf[m], bk[m]), fct);
  __syncthreads();
}

// exec_r: real data through the complex Bluestein transform; tmp: n complex
__device__ void blue_r(const PfBlue& B, const double* pool, double* c, Cx* tmp, Cx* akf, Cx* ch, double fct,
                       bool r2hc, Cx* lds) {
  const int n = B.n;
  if (r2hc) {
    const double zero = 0. * c[0];
    PF_FOR(m, n) tmp[m] = {c[m], zero};
    __syncthreads();
    blue_fft<true>(B, pool, tmp, akf, ch, fct, lds);
    PF_FOR(m, n) c[m] = m == 0 ? tmp[0].r : ((m & 1) ? tmp[(m + 1) / 2].r : tmp[m / 2].i);
    __syncthreads();
  } else {
    // tmp[0] = (c0, c0 * 0); tmp[k] = (c[2k-1], c[2k]); n even: tmp[n/2].i = 0 * c0
    PF_FOR(k, n / 2 + 1) {
      Cx v;
      if (k == 0) v = {c[0], c[0] * 0.};
      else if (2 * k == n) v = {c[n - 1], 0. * c[0]};
      else v = {c[2 * k - 1], c[2 * k]};
      tmp[k] = v;
    }
    __syncthreads();
    PF_FOR(m, (n - 1) / 2) {
      const int q = m + 1;   // 2q < n
      tmp[n - q] = {tmp[q].r, -tmp[q].i};
    }
    __syncthreads();
    blue_fft<false>(B, pool, tmp, akf, ch, fct, lds);
    PF_FOR(m, n) c[m] = tmp[m].r;
    __syncthreads();
  }
}

// ============================ entry points ==================================
// per-transform scratch (pocketfft.h pf_scratch_doubles): a (2n), x (2n), and
// for Bluestein akf, ch2 (2 n2 each); lds: the fused executor's tile buffers
// (2 * kPfTileElems complex of the calling kernel's LDS) or nullptr
struct PfScratch {
  double* a;
  Cx* x;
  Cx* akf;
  Cx* ch2;
  Cx* lds;
};
__device__ inline PfScratch pf_scratch(const PfLen& L, double* slot, Cx* lds) {
  PfScratch s;
  s.lds = lds;
  s.a = slot;
  s.x = reinterpret_cast<Cx*>(slot + 2 * L.n);
  s.akf = reinterpret_cast<Cx*>(slot + 4 * L.n);
  s.ch2 = reinterpret_cast<Cx*>(slot + 4 * L.n + 2 * ((L.rblue || L.cblue) ? L.bl.n2 : 0));
  return s;
}

// scipy.fft.rfft's pocketfft_r forward on c (n reals, in place -> halfcomplex)
__device__ inline void pf_r2hc(const PfLen& L, const double* pool, double* c, const PfScratch& s, double fct) {
  if (L.rblue) blue_r(L.bl, pool, c, s.x, s.akf, s.ch2, fct, true, s.lds);
  else rfftp(L.r, pool, c, s.a, fct, true);
}
// pocketfft_r backward on c (halfcomplex in place -> n reals)
__device__ inline void pf_hc2r(const PfLen& L, const double* pool, double* c, const PfScratch& s, double fct) {
  if (L.rblue) blue_r(L.bl, pool, c, s.x, s.akf, s.ch2, fct, false, s.lds);
  else rfftp(L.r, pool, c, s.a, fct, false);
}
// pocketfft_c backward on c (n complex, in place); c must not be s.x when Bluestein
__device__ inline void pf_c2c_bwd(const PfLen& L, const double* pool, Cx* c, const PfScratch& s, double fct) {
  if (L.cblue) blue_fft<false>(L.bl, pool, c, s.akf, s.ch2, fct, s.lds);
  else cfftp<false>(L.c, pool, c, reinterpret_cast<Cx*>(s.a), fct, s.lds);
}

// |scipy.signal.hilbert(f)| of one real row (modem.py:309, 315): f (n) is
// overwritten by its halfcomplex spectrum, env (n) receives the envelope
// (env may be f).  fct = double(1 / long double n).
__device__ inline void pf_hilbert_env(const PfLen& L, const double* pool, double* f, double* env, double* slot,
                                      double fct, Cx* lds) {
  const int n = (int)L.n;
  const PfScratch s = pf_scratch(L, slot, lds);
  pf_r2hc(L, pool, f, s, 1.0);
  // the spectrum as pypocketfft's c2c_sym leaves it (bins 0..n/2 from r2c,
  // conjugated into n - i -- bins 0 and n/2 onto themselves, imaginary -0.0),
  // times scipy's h with numpy's FMA complex multiply
  auto spec = [=](int i) -> Cx {
    double xr, xi;
    if (i == 0) { xr = f[0]; xi = -0.0; }
    else if (2 * i == n) { xr = f[n - 1]; xi = -0.0; }
    else if (2 * i < n) { xr = f[2 * i - 1]; xi = f[2 * i]; }
    else { xr = f[2 * (n - i) - 1]; xi = -f[2 * (n - i)]; }
    const double hr = (i == 0 || 2 * i == n) ? 1.0 : (2 * i < n ? 2.0 : 0.0), hi = 0.0;
    return {__builtin_fma(xr, hr, -(xi * hi)), __builtin_fma(xr, hi, xi * hr)};
  };
  // ifft: pocketfft_c backward, times 1/n; then numpy's complex abs
  auto absw = [=](int i, Cx v) {
    const double ar = fabs(v.r), ai = fabs(v.i);
    const double h = ar > ai ? ar : ai, l = ar > ai ? ai : ar;
    env[i] = h == 0.0 ? 0.0 : h * __builtin_sqrt(__builtin_fma(l / h, l / h, 1.0));
  };
  Cx* X = s.x;
  if (L.cblue) {   // Bluestein scales inside its last chirp multiply
    PF_FOR(i, n) X[i] = spec(i);
    __syncthreads();
    blue_fft<false>(L.bl, pool, X, s.akf, s.ch2, fct, lds);
    PF_FOR(i, n) absw(i, X[i]);
    __syncthreads();
    return;
  }
  // spec reads f, which neither X nor the scratch aliases; the envelope goes
  // straight from the last group's tiles to env (cfftp's copy_and_norm scale
  // first)
  cfftp_x<false>(L.c, pool, spec, X, reinterpret_cast<Cx*>(s.a),
                 [=](int i, Cx v) { absw(i, fct != 1.0 ? scale(v, fct) : v); }, lds);
}

// the same envelope with the row read through src(i) and the envelope handed
// to fin(i, env) -- every transform LDS-fused, no copies in or out.  Needs
// pf_hilbert_fusable(L); slot as pf_hilbert_env's (f = slot, then the
// scratch); src is read before fin is first called.
template <class Src, class Fin, bool LEAN = false>
__device__ __forceinline__ void pf_hilbert_env_x(const PfLen& L, const double* pool, Src src, Fin fin, double* slot, double fct,
                                 Cx* lds, int stage = 0) {
  const int n = (int)L.n;
  double* f = slot;
  const PfScratch s = pf_scratch(L, slot + pf_even(n), lds);
  // stage (diagnostic timing only, AMR_PF_STAGE): 1 the real transform alone
  // (its halfcomplex output handed to fin), 2 the complex half alone (src
  // taken as the halfcomplex spectrum)
  if (stage == 1) {
    rfftp_fwd_fused<Src, LEAN>(L.r, pool, src, f, s.a, reinterpret_cast<double*>(lds));
    for (int i = threadIdx.x; i < n; i += blockDim.x) fin(i, f[i]);
    __syncthreads();
    return;
  }
  if (stage == 2) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) f[i] = src(i);
    __syncthreads();
  } else {
    rfftp_fwd_fused<Src, LEAN>(L.r, pool, src, f, s.a, reinterpret_cast<double*>(lds));
  }
  auto spec = [=](int i) -> Cx {
    double xr, xi;
    if (i == 0) { xr = f[0]; xi = -0.0; }
    else if (2 * i == n) { xr = f[n - 1]; xi = -0.0; }
    else if (2 * i < n) { xr = f[2 * i - 1]; xi = f[2 * i]; }
    else { xr = f[2 * (n - i) - 1]; xi = -f[2 * (n - i)]; }
    const double hr = (i == 0 || 2 * i == n) ? 1.0 : (2 * i < n ? 2.0 : 0.0), hi = 0.0;
    return {__builtin_fma(xr, hr, -(xi * hi)), __builtin_fma(xr, hi, xi * hr)};
  };
  auto envf = [=](int i, Cx v) {
    if (fct != 1.0) v = scale(v, fct);
    const double ar = fabs(v.r), ai = fabs(v.i);
    const double h = ar > ai ? ar : ai, l = ar > ai ? ai : ar;
    fin(i, h == 0.0 ? 0.0 : h * __builtin_sqrt(__builtin_fma(l / h, l / h, 1.0)));
  };
  // (spec reads f only: B = s.a may pad over s.x)
  cfftp_x<false, decltype(spec), decltype(envf), LEAN, true>(L.c, pool, spec, s.x, reinterpret_cast<Cx*>(s.a), envf,
                                                             lds);
}

// The two halves of pf_hilbert_env_x as the bodies of two lean kernels (one
// kernel holding both spills registers): pf_rfft_row -- pocketfft_r forward
// of src into fin (halfcomplex; fin may be src's own storage), scratch slot
// (2n); pf_env_row -- the spectrum read back through fget(j) (halfcomplex
// element j), times h, pocketfft_c backward, 1/n, numpy's abs into fin(i, e),
// scratch slot (4n).  Lean plans only (pf_hilbert_lean).
template <class Src, class Fin>
__device__ __forceinline__ void pf_rfft_row(const PfLen& L, const double* pool, Src src, Fin fin, double* slot,
                                            Cx* lds) {
  rfftp_fwd_fused<Src, true, Fin>(L.r, pool, src, slot, slot + L.n, reinterpret_cast<double*>(lds), fin);
}
template <class Fget, class Fin>
__device__ __forceinline__ void pf_env_row(const PfLen& L, const double* pool, Fget fget, Fin fin, double* slot,
                                           double fct, Cx* lds) {
  const int n = (int)L.n;
  auto spec = [=](int i) -> Cx {
    double xr, xi;
    if (i == 0) { xr = fget(0); xi = -0.0; }
    else if (2 * i == n) { xr = fget(n - 1); xi = -0.0; }
    else if (2 * i < n) { xr = fget(2 * i - 1); xi = fget(2 * i); }
    else { xr = fget(2 * (n - i) - 1); xi = -fget(2 * (n - i)); }
    const double hr = (i == 0 || 2 * i == n) ? 1.0 : (2 * i < n ? 2.0 : 0.0), hi = 0.0;
    return {__builtin_fma(xr, hr, -(xi * hi)), __builtin_fma(xr, hi, xi * hr)};
  };
  auto envf = [=](int i, Cx v) {
    if (fct != 1.0) v = scale(v, fct);
    const double ar = fabs(v.r), ai = fabs(v.i);
    const double h = ar > ai ? ar : ai, l = ar > ai ? ai : ar;
    fin(i, h == 0.0 ? 0.0 : h * __builtin_sqrt(__builtin_fma(l / h, l / h, 1.0)));
  };
  // (B = slot + 2n pads into the slot's tail, >= n doubles past 4n)
  cfftp_x<false, decltype(spec), decltype(envf), true, true>(L.c, pool, spec, reinterpret_cast<Cx*>(slot),
                                                             reinterpret_cast<Cx*>(slot + 2 * (size_t)n), envf, lds);
}

#undef PF_FOR

}  // namespace pf
}  // namespace amr
