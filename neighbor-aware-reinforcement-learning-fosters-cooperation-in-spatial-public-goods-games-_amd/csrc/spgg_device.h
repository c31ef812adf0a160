// spgg_device.h — device helpers shared by the SPGG kernels (gfx950, wave64).
#pragma once

#include <hip/hip_runtime.h>

#include <stdint.h>

#include "spgg_abi.h"

namespace spgg {

// Threads per step-kernel workgroup (a tile holds up to 1024 agents: 4 per
// thread at 256, 2 at 512).  Build knob for A/B timing: -DSPGG_BLOCK=512.
#ifndef SPGG_BLOCK
#define SPGG_BLOCK 256
#endif
constexpr int kBlock = SPGG_BLOCK;
static_assert(kBlock == 256 || kBlock == 512, "SPGG_BLOCK must be 256 or 512");
constexpr int kWaves = kBlock / 64;

__device__ __forceinline__ int wrap(int x, int L) {
  while (x < 0) x += L;
  while (x >= L) x -= L;
  return x;
}

// ---------------------------------------------------------------------------
// Workgroup reduction of K per-thread f64 partials (K a power of two <= 64).
// Butterfly "transpose" reduce: at each level a lane keeps one half of its
// values and receives the other half from a partner lane, so K values cost
// ~K exchanges instead of 6K.  Afterwards lane l holds the wave sum of value
// (l >> log2(64/K)).  Exchanges run on the VALU, never through the LDS pipe:
//   bit 5 / bit 4: v_permlane32_swap / v_permlane16_swap (gfx950) swap the
//                  kept and the shipped half in one instruction per dword
//   bit 3 .. 0:    DPP row_ror:8, row_half_mirror, quad_perm — partners
//                  l^8, l^7, l^2, l^1: each flips the level's bit and keeps
//                  the higher bits, and together they span the 16-lane row.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double x) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), CTRL, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}

// (a, b) -> (a', b') with a' + b' = the partner-summed kept value (MASK 32/16).
template <int MASK>
__device__ __forceinline__ double swap_sum(double a, double b) {
  int alo = __double2loint(a), ahi = __double2hiint(a), blo = __double2loint(b), bhi = __double2hiint(b);
  if constexpr (MASK == 32) {
    const auto l = __builtin_amdgcn_permlane32_swap(alo, blo, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(ahi, bhi, false, false);
    alo = l[0]; blo = l[1]; ahi = h[0]; bhi = h[1];
  } else {
    const auto l = __builtin_amdgcn_permlane16_swap(alo, blo, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(ahi, bhi, false, false);
    alo = l[0]; blo = l[1]; ahi = h[0]; bhi = h[1];
  }
  return __hiloint2double(ahi, alo) + __hiloint2double(bhi, blo);
}

// Same exchanges for packed integer counters (one dword per value).
template <int MASK>
__device__ __forceinline__ uint32_t swap_sum(uint32_t a, uint32_t b) {
  const auto s = MASK == 32 ? __builtin_amdgcn_permlane32_swap((int)a, (int)b, false, false)
                            : __builtin_amdgcn_permlane16_swap((int)a, (int)b, false, false);
  return (uint32_t)s[0] + (uint32_t)s[1];
}

template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xf, 0xf, false);
}

template <int MASK, typename T>
__device__ __forceinline__ T partner(T x) {
  if constexpr (sizeof(T) == 8) {
    if constexpr (MASK == 8) return dpp_f64<0x128>(x);        // row_ror:8      -> l^8
    else if constexpr (MASK == 4) return dpp_f64<0x141>(x);   // row_half_mirror -> l^7
    else if constexpr (MASK == 2) return dpp_f64<0x4E>(x);    // quad_perm [2,3,0,1]
    else return dpp_f64<0xB1>(x);                             // quad_perm [1,0,3,2]
  } else {
    if constexpr (MASK == 8) return dpp_u32<0x128>(x);
    else if constexpr (MASK == 4) return dpp_u32<0x141>(x);
    else if constexpr (MASK == 2) return dpp_u32<0x4E>(x);
    else return dpp_u32<0xB1>(x);
  }
}

template <int CNT, int MASK, int K, typename T>
__device__ __forceinline__ void transpose_level(T (&v)[K], int lane) {
  if constexpr (MASK >= 1) {
    constexpr int h = CNT > 1 ? CNT / 2 : 1;
    if constexpr (MASK >= 16) {
      if constexpr (CNT > 1) {
#pragma unroll
        for (int i = 0; i < h; ++i) v[i] = swap_sum<MASK>(v[i], v[i + h]);
      } else {
        v[0] = swap_sum<MASK>(v[0], v[0]);
      }
    } else {
      if constexpr (CNT > 1) {
        const bool upper = (lane & MASK) != 0;
#pragma unroll
        for (int i = 0; i < h; ++i) {
          const T send = upper ? v[i] : v[i + h];
          const T keep = upper ? v[i + h] : v[i];
          v[i] = keep + partner<MASK>(send);
        }
      } else {
        v[0] += partner<MASK>(v[0]);
      }
    }
    transpose_level<(CNT > 1 ? CNT / 2 : 1), MASK / 2, K, T>(v, lane);
  }
}

// Reduce v over the workgroup; thread k < K then returns the total of value k.
// lds must hold kWaves*K doubles.
template <int K>
__device__ __forceinline__ double block_reduce(double (&v)[K], double* lds) {
  static_assert(K >= 1 && K <= 64 && (K & (K - 1)) == 0, "K must be a power of two");
  transpose_level<K, 32, K, double>(v, threadIdx.x & 63);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int per = 64 / K;
  if ((lane & (per - 1)) == 0) lds[wave * K + lane / per] = v[0];
  __syncthreads();
  double tot = 0.0;
  if (threadIdx.x < K) {
#pragma unroll
    for (int w = 0; w < kWaves; ++w) tot += lds[w * K + threadIdx.x];
  }
  return tot;
}

// Workgroup-uniform values computed on the VALU (f64 has no scalar ALU) moved back
// to SGPRs: held in VGPRs they cost every lane two registers for the whole kernel.
__device__ __forceinline__ double uniform_f64(double x) {
  return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(x)),
                          __builtin_amdgcn_readfirstlane(__double2loint(x)));
}
__device__ __forceinline__ uint64_t uniform_u64(uint64_t x) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(x >> 32)) << 32 |
         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
}

// max of two non-NaN doubles as ONE v_max_f64.  fmax() in IEEE mode first quiets
// each operand that is not provably canonical (v_max_f64 x, x, x), three f64 ops in
// all; no value here is ever a NaN, and quieting changes no other value (f64
// denormals are preserved), so the result is the same double.
__device__ __forceinline__ double max_f64(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// Max over the wave, in every lane: permlane32/16 swaps, then DPP partners
// l^8, l^7, l^2, l^1 (together they span the 16-lane row), no LDS.
template <int MASK>
__device__ __forceinline__ double swap_max(double x) {
  const int lo = __double2loint(x), hi = __double2hiint(x);
  const auto l = MASK == 32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false)
                            : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h = MASK == 32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false)
                            : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return max_f64(__hiloint2double(h[0], l[0]), __hiloint2double(h[1], l[1]));
}

__device__ __forceinline__ double wave_max(double v) {
  v = swap_max<32>(v);
  v = swap_max<16>(v);
  v = max_f64(v, partner<8>(v));
  v = max_f64(v, partner<4>(v));
  v = max_f64(v, partner<2>(v));
  v = max_f64(v, partner<1>(v));
  return v;
}

// ---------------------------------------------------------------------------
// numpy legacy random_sample: 53-bit double from two 32-bit words.
__device__ __forceinline__ double mt_double(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) / 9007199254740992.0;
}

// Philox2x32-10 (Salmon et al. 2011; Crush-resistant at 10 rounds): 64 bits
// per (counter, key) at half the cost of the 4x32 variant.
__device__ __forceinline__ uint2 philox2x32_10(uint2 c, uint32_t k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) k += 0x9E3779B9u;
    const uint64_t p = (uint64_t)0xD256D193u * c.x;  // one v_mad_u64_u32 for lo and hi
    c = make_uint2((uint32_t)(p >> 32) ^ k ^ c.y, (uint32_t)p);
  }
  return c;
}

// u < thr for u = k / 2^53 (k < 2^53, numpy's random_sample) and a threshold
// in [0, 1] given as T = ceil(thr * 2^53): the scaling by 2^53 is exact, and
// for an integer k, k < x <=> k < ceil(x).  One 64-bit integer compare.
__host__ __device__ inline uint64_t u53_threshold(double thr) {
  return (uint64_t)__builtin_ceil(thr * 9007199254740992.0);
}

// Philox mode: agents 2m and 2m+1 share one Philox2x32-10 block, counter (m, t),
// key = replica seed mixed with the replica index; the even agent takes w.x, the
// odd one w.y.  Of an agent's 32 bits, bits 31..1 give u = k / 2^31 (numpy's
// random_sample has 53 bits: statistical parity only) and bit 0 the random action.
__device__ __forceinline__ uint2 philox_block(int idx, int t, uint32_t key) {
  return philox2x32_10(make_uint2((uint32_t)idx >> 1, (uint32_t)t), key);
}
// explore = u < eps given thr53 = ceil(eps * 2^53): k * 2^22 < thr53 <=> k / 2^31 < eps
// (an integer below a ceiling is below the real), and for the integer k < 2^31 that is
// k < ceil(thr53 / 2^22) <= 2^31: one 32-bit compare against a workgroup-uniform bound;
// rbit = bit 0 (algorithms.py:105-108)
__device__ __forceinline__ void philox_decide(uint32_t bits, uint64_t thr53, int* explore, int* rbit) {
  const uint32_t thr31 = (uint32_t)((thr53 + ((1ull << 22) - 1)) >> 22);
  *explore = (bits >> 1) < thr31 ? 1 : 0;
  *rbit = (int)(bits & 1u);
}
__device__ __forceinline__ void philox_draw(int idx, int t, uint32_t key, uint64_t thr53, int* explore,
                                            int* rbit) {
  const uint2 w = philox_block(idx, t, key);
  philox_decide((idx & 1) ? w.y : w.x, thr53, explore, rbit);
}

// q[4] accessors with a run-time index e = 2s + a, kept in registers (no scratch).
__device__ __forceinline__ double q_get(const double (&q)[4], int e) {
  const double lo = (e & 1) ? q[1] : q[0], hi = (e & 1) ? q[3] : q[2];
  return (e & 2) ? hi : lo;
}
__device__ __forceinline__ void q_set(double (&q)[4], int e, double x) {
  q[0] = e == 0 ? x : q[0];
  q[1] = e == 1 ? x : q[1];
  q[2] = e == 2 ? x : q[2];
  q[3] = e == 3 ? x : q[3];
}

// x / d rounded to nearest for a workgroup-uniform d, given r = RN(1/d):
// q = RN(x*r), e = x - q*d (exact by FMA), RN(q + e*r) is the correctly
// rounded quotient (Markstein's theorem; no over/underflow in our ranges).
// Bit-identical to the IEEE division at 3 f64 ops instead of ~11.
__device__ __forceinline__ double div_uniform(double x, double d, double r) {
  const double q = x * r;
  const double e = __builtin_fma(-q, d, x);
  return __builtin_fma(e, r, q);
}

// Reputation state threshold: (acc / n) > 0  <=>  acc >= k * 2^-1074 with
// k = 3 (n = 5) or 7 (n = 13): the smallest sums whose quotient does not
// round to zero.  Exact for every double acc, no division (spgg.py:306-307).
__device__ __forceinline__ double rep_threshold(bool m2) {
  return __longlong_as_double(m2 ? 7LL : 3LL);  // 7*2^-1074 / 3*2^-1074 (subnormals)
}

// ---------------------------------------------------------------------------
// Payoff of one agent given the cooperator indicators of the 13 cells around
// it (spgg.py:230-259, 373-377): group counts N_k at the centre and the four
// axial neighbours, P_k = S0 ? (r*c*N_k)/5 - cost : (r*c*N_k)/5 (table lookups
// with host-computed entries, equal in value to the reference's
// (t-cost)*S0 + t*S1), summed in the reference's group order, normalised.
struct Cells13 {
  int c00, cm0, cp0, c0m, c0p, cmm, cmp, cpm, cpp, cM0, cP0, c0M, c0P;
};

// tab: LDS copy of pay_c[6] followed by pay_d[6]; norm_rcp = RN(1/norm_den).
__device__ __forceinline__ double payoff13(const Cells13& c, const double* tab, double norm_min,
                                           double norm_den, double norm_rcp) {
  const int N0 = c.c00 + c.cm0 + c.cp0 + c.c0m + c.c0p;  // group (0,0)  -> N0[i,j]
  const int N1 = c.cm0 + c.cM0 + c.c00 + c.cmm + c.cmp;  // group (1,0)  -> N0[i-1,j]
  const int N2 = c.cp0 + c.c00 + c.cP0 + c.cpm + c.cpp;  // group (-1,0) -> N0[i+1,j]
  const int N3 = c.c0m + c.cmm + c.cpm + c.c0M + c.c00;  // group (1,1)  -> N0[i,j-1]
  const int N4 = c.c0p + c.cmp + c.cpp + c.c00 + c.c0P;  // group (-1,1) -> N0[i,j+1]
  const double* t = tab + (c.c00 ? 0 : 6);
  double tot = t[N0];
  tot = tot + t[N1];
  tot = tot + t[N2];
  tot = tot + t[N3];
  tot = tot + t[N4];
  return div_uniform(tot - norm_min, norm_den, norm_rcp);  // (tot - (r-5)) / (4r - (r-5))
}

}  // namespace spgg
