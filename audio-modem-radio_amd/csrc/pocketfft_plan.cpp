// pocketfft_plan.cpp -- host construction of the device pocketfft plans
// (pocketfft.h): pocketfft's plan choice, factorisations and twiddle tables
// (sincos_2pibyn), by the rules oracle/amr_pocketfft.c restates and pins
// against scipy 1.15.3.  Host code; compiled by hipcc.
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
#include <hip/hip_runtime.h>

#include <cmath>
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "pocketfft.h"

namespace amr {
namespace {

// pocketfft's sincos_2pibyn(n): W_n^k = v1[k & mask] * v2[k >> shift],
// entries from glibc's sincos by octant, ang = double(0.25L * pi / n)
struct Twid2pi {
  int64_t n = 0, mask = 0, shift = 0;
  std::vector<double2> v1, v2;
  // cos / sin of one argument from glibc's sincos, as scipy's gcc-built
  // pocketfft gets them (gcc merges calc's std::cos / std::sin pair into one
  // sincos call, and sincos differs from sin / cos in the last ulp for some
  // arguments -- oracle/amr_pocketfft.c)
  static double2 cs(double v) {
    double s, c;
    sincos(v, &s, &c);
    return make_double2(c, s);
  }
  static double2 calc(int64_t x, int64_t n, double ang) {
    x <<= 3;
    if (x < 4 * n) {
      if (x < 2 * n) {
        if (x < n) return cs((double)x * ang);
        const double2 t = cs((double)(2 * n - x) * ang);
        return make_double2(t.y, t.x);
      }
      x -= 2 * n;
      if (x < n) {
        const double2 t = cs((double)x * ang);
        return make_double2(-t.y, t.x);
      }
      const double2 t = cs((double)(2 * n - x) * ang);
      return make_double2(-t.x, t.y);
    }
    x = 8 * n - x;
    if (x < 2 * n) {
      if (x < n) {
        const double2 t = cs((double)x * ang);
        return make_double2(t.x, -t.y);
      }
      const double2 t = cs((double)(2 * n - x) * ang);
      return make_double2(t.y, -t.x);
    }
    x -= 2 * n;
    if (x < n) {
      const double2 t = cs((double)x * ang);
      return make_double2(-t.y, -t.x);
    }
    const double2 t = cs((double)(2 * n - x) * ang);
    return make_double2(-t.x, -t.y);
  }
  explicit Twid2pi(int64_t len) : n(len) {
    const double ang = (double)(0.25L * 3.141592653589793238462643383279502884197L / (long double)len);
    const int64_t nval = (len + 2) / 2;
    shift = 1;
    while (((int64_t)1 << shift) * ((int64_t)1 << shift) < nval) ++shift;
    mask = ((int64_t)1 << shift) - 1;
    v1.resize((size_t)(mask + 1));
    v1[0] = make_double2(1.0, 0.0);
    for (int64_t i = 1; i <= mask; ++i) v1[(size_t)i] = calc(i, len, ang);
    v2.resize((size_t)((nval + mask) / (mask + 1)));
    v2[0] = make_double2(1.0, 0.0);
    for (size_t i = 1; i < v2.size(); ++i) v2[i] = calc((int64_t)i * (mask + 1), len, ang);
  }
  double2 operator[](int64_t idx) const {
    const bool hi = 2 * idx > n;
    if (hi) idx = n - idx;
    const double2 a = v1[(size_t)(idx & mask)], b = v2[(size_t)(idx >> shift)];
    const double re = a.x * b.x - a.y * b.y, im = a.x * b.y + a.y * b.x;
    return make_double2(re, hi ? -im : im);
  }
};

int64_t largest_prime_factor(int64_t n) {
  int64_t res = 1;
  while ((n & 1) == 0) {
    res = 2;
    n >>= 1;
  }
  for (int64_t x = 3; x * x <= n; x += 2)
    while (n % x == 0) {
      res = x;
      n /= x;
    }
  if (n > 1) res = n;
  return res;
}

double cost_guess(int64_t n) {
  const double lfp = 1.1;   // pocketfft's penalty for non-hardcoded larger factors
  const int64_t ni = n;
  double result = 0.;
  while ((n & 1) == 0) {
    result += 2;
    n >>= 1;
  }
  for (int64_t x = 3; x * x <= n; x += 2)
    while (n % x == 0) {
      result += (x <= 5) ? (double)x : lfp * (double)x;
      n /= x;
    }
  if (n > 1) result += (n <= 5) ? (double)n : lfp * (double)n;
  return result * (double)ni;
}

// the smallest 2^a 3^b 5^c 7^d 11^e >= n
int64_t good_size_cmplx(int64_t n) {
  if (n <= 12) return n;
  int64_t best = 2 * n;
  for (int64_t f11 = 1; f11 < best; f11 *= 11)
    for (int64_t f117 = f11; f117 < best; f117 *= 7)
      for (int64_t f1175 = f117; f1175 < best; f1175 *= 5) {
        int64_t x = f1175;
        while (x < n) x *= 2;
        for (;;) {
          if (x < n) {
            x *= 3;
          } else if (x > n) {
            if (x < best) best = x;
            if (x & 1) break;
            x >>= 1;
          } else {
            return n;
          }
        }
      }
  return best;
}

bool use_bluestein(int64_t n, bool real) {
  const int64_t tmp = n < 50 ? 0 : largest_prime_factor(n);
  if (tmp * tmp <= n) return false;
  const double comp1 = real ? 0.5 * cost_guess(n) : cost_guess(n);
  const double comp2 = 2 * cost_guess(good_size_cmplx(2 * n - 1)) * 1.5;
  return comp2 < comp1;
}

int factorize(int64_t n, bool with8, int64_t* f) {
  int nf = 0;
  if (with8)
    while ((n & 7) == 0) {
      f[nf++] = 8;
      n >>= 3;
    }
  while ((n & 3) == 0) {
    f[nf++] = 4;
    n >>= 2;
  }
  if ((n & 1) == 0) {
    n >>= 1;
    f[nf++] = 2;
    std::swap(f[0], f[nf - 1]);
  }
  for (int64_t d = 3; d * d <= n; d += 2)
    while (n % d == 0) {
      f[nf++] = d;
      n /= d;
    }
  if (n > 1) f[nf++] = n;
  return nf;
}

void align2(std::vector<double>& pool) {
  if (pool.size() & 1) pool.push_back(0.0);
}

// greedy grouping of a cfftp plan's passes for the LDS-fused executor: runs
// of consecutive passes whose radix product stays <= kPfMaxGroupP; a plan
// with a generic pass (ip > 11) runs unfused
void build_groups(PfPasses& P) {
  P.fused = 0;
  P.ng = 0;
  if (P.nf == 0) return;
  for (int k = 0; k < P.nf; ++k)
    if (P.f[k].ip > 11) return;
  int k = 0;
  while (k < P.nf) {
    PfGroup& G = P.g[P.ng++];
    G.f0 = k;
    G.P = P.f[k].ip;
    G.L = P.f[k].l1;
    ++k;
    while (k < P.nf && G.P * P.f[k].ip <= kPfMaxGroupP) G.P *= P.f[k++].ip;
    G.nf = k - G.f0;
    G.D = P.f[k - 1].ido;
    G.Q = (int)(kPfTileElems / G.P);
    if (G.D >= G.Q) {
      G.Qi = G.Q;
      G.Qk = 1;
    } else {
      G.Qi = (int)G.D;
      G.Qk = (int)(G.Q / G.D);
    }
    const int64_t nti = (G.D + G.Qi - 1) / G.Qi, ntk = (G.L + G.Qk - 1) / G.Qk;
    G.dv[0] = pf_div(G.P);
    G.dv[1] = pf_div(G.Q);
    G.dv[2] = pf_div(G.Qi);
    G.dv[3] = pf_div(G.D - (nti - 1) * G.Qi);
    G.dv[4] = pf_div(G.Qk);
    G.dv[5] = pf_div(G.L - (ntk - 1) * G.Qk);
    G.dv[6] = pf_div(nti);
    G.dv[7] = pf_div(G.D);
    for (int q = G.f0; q < G.f0 + G.nf; ++q) {
      P.f[q].dv[0] = pf_div(P.f[q].ido / G.D);
      P.f[q].l1l = (int32_t)(P.f[q].l1 / G.L);
    }
  }
  P.fused = 1;
}

// pocketfft's cfftp(len): factors and twiddles
bool build_cfftp(int64_t len, PfPasses& P, std::vector<double>& pool) {
  P = PfPasses{};
  P.len = len;
  if (len == 1) return true;
  int64_t f[64];
  const int nf = factorize(len, true, f);
  if (nf > kPfMaxF) return false;
  P.nf = nf;
  const Twid2pi comp(len);
  int64_t l1 = 1;
  for (int k = 0; k < nf; ++k) {
    const int64_t ip = f[k], ido = len / (l1 * ip);
    PfFact& F = P.f[k];
    F.ip = ip;
    F.l1 = l1;
    F.ido = ido;
    align2(pool);
    F.tw = (int64_t)pool.size();
    for (int64_t j = 1; j < ip; ++j)
      for (int64_t i = 1; i < ido; ++i) {
        const double2 w = comp[j * l1 * i];
        pool.push_back(w.x);
        pool.push_back(w.y);
      }
    F.tws = -1;
    if (ip > 11) {
      F.tws = (int64_t)pool.size();
      for (int64_t j = 0; j < ip; ++j) {
        const double2 w = comp[j * l1 * ido];
        pool.push_back(w.x);
        pool.push_back(w.y);
      }
    }
    l1 *= ip;
  }
  build_groups(P);
  return true;
}

// grouping of an rfftp plan's passes in forward (r2hc) order for the fused
// real executor (pocketfft.h)
void build_rgroups(PfPasses& P) {
  P.fused = 0;
  P.ng = 0;
  if (P.nf == 0) return;
  int k = P.nf - 1;
  while (k >= 0) {
    PfGroup& G = P.g[P.ng++];
    G.f0 = k;
    const int64_t D = P.f[k].ido;
    // an even ido: every pass left is radf4 / radf2 (pocketfft executes its
    // 4s and 2 last), and they couple only residue pairs {p, D/2 - p} and
    // {0, D - 1} mod D -- one "pair" group to the end, tiles of T pair
    // classes times all n / D blocks (pocketfft_dev.h rgroup_pairs)
    if (D % 2 == 0 && P.len / D <= kPfTileDoubles / 4) {
      G.nf = k + 1;
      G.D = D;
      G.P = P.len / D;
      G.L = 1;
      G.Q = 2;
      G.Qi = 0;
      G.Qk = (int)(kPfTileDoubles / (4 * G.P));   // T: pair classes per tile (<= 4 T residues)
      {
        // R (and R / 2) of the special tile {0, D - 1}, a full tile (4 T
        // residues, or 4 T - 2 when it ends on the self-paired p = D / 4) and
        // the last tile
        const int64_t H = D / 2, pmax = H / 2, T = G.Qk, nt = (pmax + T - 1) / T;
        auto rtile = [&](int64_t tile) {
          const int64_t p0 = 1 + (tile - 1) * T, p1 = std::min(p0 + T, pmax + 1);
          const int64_t pe = (2 * (p1 - 1) == H) ? p1 - 1 : p1;
          return 2 * (p1 - p0) + 2 * (pe - p0);
        };
        G.dv[0] = pf_div(2);
        G.dv[1] = pf_div(1);
        G.dv[2] = pf_div(nt >= 1 ? rtile(1) : 2);
        G.dv[3] = pf_div(nt >= 1 ? rtile(1) / 2 : 1);
        G.dv[4] = pf_div(nt >= 1 ? rtile(nt) : 2);
        G.dv[5] = pf_div(nt >= 1 ? rtile(nt) / 2 : 1);
        int64_t B = 1;
        for (int q = k; q >= 0; --q) {
          P.f[q].dv[0] = pf_div(B);
          P.f[q].dv[1] = pf_div(B + 1);
          B *= P.f[q].ip;
        }
      }
      k = -1;
      break;
    }
    const int64_t qmin = std::max<int64_t>(1, (kPfMinRun + D - 1) / D);
    G.D = D;
    G.P = P.f[k].ip;
    const bool hard = G.P <= 5;
    --k;
    if (hard)
      while (k >= 0 && P.f[k].ip <= 5 && D * G.P * P.f[k].ip * qmin <= kPfTileDoubles) G.P *= P.f[k--].ip;
    G.nf = G.f0 - k;
    G.L = P.f[k + 1].l1;
    G.Qi = 0;
    if (hard && D * G.P * qmin <= kPfTileDoubles) {
      G.Q = 1;
      G.Qk = (int)std::min<int64_t>(G.L, kPfTileDoubles / (D * G.P));
      const int64_t ntk = (G.L + G.Qk - 1) / G.Qk;
      G.dv[0] = pf_div(D);
      G.dv[1] = pf_div(G.Qk);
      G.dv[2] = pf_div(G.L - (ntk - 1) * G.Qk);
      for (int q = G.f0; q > G.f0 - G.nf; --q) {
        const int64_t l1l = P.f[q].l1 / G.L, hi = (P.f[q].ido - 1) / 2;
        P.f[q].dv[0] = pf_div(l1l);
        P.f[q].dv[1] = pf_div(hi);
        P.f[q].dv[2] = pf_div(l1l * hi);
        P.f[q].l1l = (int32_t)l1l;
      }
    } else {
      G.Q = 0;
      G.Qk = 0;
    }
  }
  P.fused = 1;
}

// pocketfft's rfftp(len): factors, twiddles and the generic passes' tables
bool build_rfftp(int64_t len, PfPasses& P, std::vector<double>& pool) {
  P = PfPasses{};
  P.len = len;
  if (len == 1) return true;
  int64_t f[64];
  const int nf = factorize(len, false, f);
  if (nf > kPfMaxF) return false;
  P.nf = nf;
  const Twid2pi twid(len);
  int64_t l1 = 1;
  for (int k = 0; k < nf; ++k) {
    const int64_t ip = f[k], ido = len / (l1 * ip);
    PfFact& F = P.f[k];
    F.ip = ip;
    F.l1 = l1;
    F.ido = ido;
    F.tw = F.tws = -1;
    if (k < nf - 1) {   // the last factor needs no twiddles
      F.tw = (int64_t)pool.size();
      std::vector<double> t((size_t)((ip - 1) * (ido - 1)), 0.0);
      for (int64_t j = 1; j < ip; ++j)
        for (int64_t i = 1; i <= (ido - 1) / 2; ++i) {
          const double2 w = twid[j * l1 * i];
          t[(size_t)((j - 1) * (ido - 1) + 2 * i - 2)] = w.x;
          t[(size_t)((j - 1) * (ido - 1) + 2 * i - 1)] = w.y;
        }
      pool.insert(pool.end(), t.begin(), t.end());
    }
    if (ip > 5) {   // the generic passes' factors
      F.tws = (int64_t)pool.size();
      std::vector<double> t((size_t)(2 * ip), 0.0);
      t[0] = 1.;
      t[1] = 0.;
      for (int64_t i = 2, ic = 2 * ip - 2; i <= ic; i += 2, ic -= 2) {
        const double2 w = twid[i / 2 * (len / ip)];
        t[(size_t)i] = w.x;
        t[(size_t)(i + 1)] = w.y;
        t[(size_t)ic] = w.x;
        t[(size_t)(ic + 1)] = -w.y;
      }
      pool.insert(pool.end(), t.begin(), t.end());
    }
    l1 *= ip;
  }
  build_rgroups(P);
  return true;
}

// pocketfft's fftblue(n) without bkf (pf_finish)
bool build_blue(int64_t n, PfBlue& B, std::vector<double>& pool) {
  B = PfBlue{};
  B.n = n;
  B.n2 = good_size_cmplx(n * 2 - 1);
  if (!build_cfftp(B.n2, B.plan, pool)) return false;
  const Twid2pi tmp(2 * n);
  align2(pool);
  B.bk = (int64_t)pool.size();
  pool.push_back(1.0);
  pool.push_back(0.0);
  int64_t coeff = 0;
  for (int64_t m = 1; m < n; ++m) {
    coeff += 2 * m - 1;
    if (coeff >= 2 * n) coeff -= 2 * n;
    const double2 w = tmp[coeff];
    pool.push_back(w.x);
    pool.push_back(w.y);
  }
  B.bkf = (int64_t)pool.size();
  pool.resize(pool.size() + (size_t)(2 * (B.n2 / 2 + 1)), 0.0);
  return true;
}

}  // namespace

void pf_hilbert_shape(int64_t n, bool* blue, int64_t* n2, int64_t* maxp) {
  const bool b = use_bluestein(n, true) || use_bluestein(n, false);
  const int64_t m = b ? good_size_cmplx(2 * n - 1) : n;
  if (blue) *blue = b;
  if (n2) *n2 = m;
  if (maxp) *maxp = m > 1 ? largest_prime_factor(m) : 1;
}

bool pf_fuse_on() {
  static const bool on = [] {
    const char* e = getenv("AMR_PF_FUSE");
    return !(e && e[0] == '0');
  }();
  return on;
}

bool pf_len_build(int64_t n, PfLen& L, std::vector<double>& pool) {
  // the device transforms index in 32 bits (a row and its Bluestein scratch
  // stay below 2^31 doubles)
  if (n < 1 || n > kPfMaxLen) return false;
  L = PfLen{};
  L.n = n;
  L.rblue = use_bluestein(n, true);
  L.cblue = use_bluestein(n, false);
  if (!L.rblue && !build_rfftp(n, L.r, pool)) return false;
  if (!L.cblue && !build_cfftp(n, L.c, pool)) return false;
  if ((L.rblue || L.cblue) && !build_blue(n, L.bl, pool)) return false;
  align2(pool);
  return true;
}

int64_t pf_scratch_doubles(const PfLen& L) {
  return 4 * L.n + ((L.rblue || L.cblue) ? 4 * L.bl.n2 : 0);
}

int64_t pf_scratch_doubles_n(int64_t n) {
  const bool blue = use_bluestein(n, true) || use_bluestein(n, false);
  return 4 * n + (blue ? 4 * good_size_cmplx(2 * n - 1) : 0);
}

namespace {
int64_t cfftp_doubles(int64_t len) {
  if (len == 1) return 0;
  int64_t f[64];
  const int nf = factorize(len, true, f);
  int64_t d = 0, l1 = 1;
  for (int k = 0; k < nf; ++k) {
    const int64_t ip = f[k], ido = len / (l1 * ip);
    d += 1 + 2 * (ip - 1) * (ido - 1) + (ip > 11 ? 2 * ip : 0);
    l1 *= ip;
  }
  return d;
}
int64_t rfftp_doubles(int64_t len) {
  if (len == 1) return 0;
  int64_t f[64];
  const int nf = factorize(len, false, f);
  int64_t d = 0, l1 = 1;
  for (int k = 0; k < nf; ++k) {
    const int64_t ip = f[k], ido = len / (l1 * ip);
    d += (k < nf - 1 ? (ip - 1) * (ido - 1) : 0) + (ip > 5 ? 2 * ip : 0);
    l1 *= ip;
  }
  return d;
}
}  // namespace

int64_t pf_pool_doubles_bound(int64_t n) {
  const bool rb = use_bluestein(n, true), cb = use_bluestein(n, false);
  int64_t d = 8 + (rb ? 0 : rfftp_doubles(n)) + (cb ? 0 : cfftp_doubles(n));
  if (rb || cb) {
    const int64_t n2 = good_size_cmplx(2 * n - 1);
    d += cfftp_doubles(n2) + 2 + 2 * n + 2 * (n2 / 2 + 1);
  }
  return d;
}

int64_t pf_resample_slot_doubles(const PfLen& Lx, const PfLen& Ly) {
  // the row (max n) + one transform's scratch at a time
  return pf_even(std::max(Lx.n, Ly.n)) + std::max(pf_scratch_doubles(Lx), pf_scratch_doubles(Ly));
}

}  // namespace amr
