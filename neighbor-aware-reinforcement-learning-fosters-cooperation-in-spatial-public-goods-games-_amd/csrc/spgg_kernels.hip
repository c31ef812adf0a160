// spgg_kernels.hip — MI355X (gfx950) kernels for the SPGG per-iteration hot path.
//
// One iteration t of the reference's run loop (src/model/spgg.py:368-592) is
// two launches over every replica in the batch:
//
//   act(t)   per agent: [finalize the deferred neighbor-influence (NI) term of
//            iteration t-1 + its Q statistics] -> payoff P from S_t (13-cell
//            stencil) -> iteration-start record -> absorbing-stop check ->
//            state s from R_t -> eps-greedy action -> R_{t+1}, S_{t+1}, reward
//   learn(t) per agent: state s' from R_{t+1} -> Q-learning TD update ->
//            diagnostic TD -> NI max/argmax over the 4 (M=1) / 12 (M=2)
//            neighbor rewards -> pending NI record + lattice-wide max |diff|
//
// The NI term divides by the lattice-wide max (spgg.py:488), so it cannot be
// applied in the pass that produces the rewards; it is applied by the NEXT
// act launch (or spgg_flush), reproducing the reference's arithmetic exactly:
//   Q[s,a] = (qc + alpha*td) + (kappa*max(0,md))/(gmax+lambda_eps) * (+-1).
//
// Every float op is f64 and written in the reference's evaluation order; the
// file is compiled with -ffp-contract=off so no FMA contraction changes a bit.
// Per-step history values are reduced per workgroup (wave butterfly +
// LDS) and added with one f64 atomic per value per workgroup.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>

#include "spgg_abi.h"

namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
constexpr int kMtThreads = 640;  // >= 624 MT19937 words, 10 waves

struct KArgs {
  const uint8_t* S_cur;  // S_t
  uint8_t* S_nxt;        // S_{t+1}
  const double* R_cur;   // R_t
  double* R_nxt;         // R_{t+1}
  double* Q;             // [rep][n][4]
  double* reward;
  uint8_t* aux;
  double* ni_md;
  double* ni_atd;
  const uint8_t* explore;
  const uint8_t* rbit;
  const double* eps;
  double* stats;
  int* stop_iter;
  const spgg_rep_params* params;
  int L;
  int n;
  int chunk;  // agents per workgroup
  int slots;  // iterations + 2
};

__device__ __forceinline__ int wrap(int x, int L) {
  while (x < 0) x += L;
  while (x >= L) x -= L;
  return x;
}

// ---------------------------------------------------------------------------
// Workgroup reduction of K per-thread f64 partials (K a power of two <= 64).
// Butterfly "transpose" reduce: at each xor level a lane keeps one half of its
// values and ships the other half, so K values cost ~K shuffles instead of
// 6K.  Afterwards lane l holds the wave sum of value (l >> log2(64/K)).
template <int CNT, int MASK, int K>
__device__ __forceinline__ void transpose_level(double (&v)[K], int lane) {
  if constexpr (MASK >= 1) {
    if constexpr (CNT > 1) {
      constexpr int h = CNT / 2;
      const bool upper = (lane & MASK) != 0;
#pragma unroll
      for (int i = 0; i < h; ++i) {
        const double send = upper ? v[i] : v[i + h];
        const double keep = upper ? v[i + h] : v[i];
        v[i] = keep + __shfl_xor(send, MASK);
      }
      transpose_level<h, MASK / 2, K>(v, lane);
    } else {
      v[0] += __shfl_xor(v[0], MASK);
      transpose_level<1, MASK / 2, K>(v, lane);
    }
  }
}

template <int K>
__device__ __forceinline__ double wave_transpose_reduce(double (&v)[K]) {
  static_assert(K >= 1 && K <= 64 && (K & (K - 1)) == 0, "K must be a power of two");
  transpose_level<K, 32, K>(v, threadIdx.x & 63);
  return v[0];
}

// q[4] accessors with a run-time index, kept in registers (no scratch).
__device__ __forceinline__ double q_get(const double (&q)[4], int e) {
  return e == 0 ? q[0] : (e == 1 ? q[1] : (e == 2 ? q[2] : q[3]));
}
__device__ __forceinline__ void q_set(double (&q)[4], int e, double x) {
  q[0] = e == 0 ? x : q[0];
  q[1] = e == 1 ? x : q[1];
  q[2] = e == 2 ? x : q[2];
  q[3] = e == 3 ? x : q[3];
}

// Reduce v over the workgroup; thread k < K then returns the total of value k.
template <int K>
__device__ __forceinline__ double block_reduce(double (&v)[K], double* lds) {
  const double s = wave_transpose_reduce<K>(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int per = 64 / K;
  if ((lane & (per - 1)) == 0) lds[wave * K + lane / per] = s;
  __syncthreads();
  double tot = 0.0;
  if (threadIdx.x < K) {
#pragma unroll
    for (int w = 0; w < kWaves; ++w) tot += lds[w * K + threadIdx.x];
  }
  return tot;
}

__device__ __forceinline__ double block_reduce_max(double v, double* lds) {
#pragma unroll
  for (int mask = 32; mask >= 1; mask >>= 1) v = fmax(v, __shfl_xor(v, mask));
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) lds[wave] = v;
  __syncthreads();
  double m = 0.0;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 0; w < kWaves; ++w) m = fmax(m, lds[w]);
  }
  return m;
}

// ---------------------------------------------------------------------------
// Philox4x32-10 (counter-based): performance-mode eps-greedy draws.
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
  }
  return c;
}

// numpy legacy random_sample: 53-bit double from two 32-bit words.
__device__ __forceinline__ double mt_double(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) / 9007199254740992.0;
}

// ---------------------------------------------------------------------------
// Payoff of agent (i,j) from S_t: 5 groups (spgg.py:373-377), each
// P_k = ((r*c*N_k)/5 - cost)*S0 + ((r*c*N_k)/5)*S1 (spgg.py:256-257), with
// N_k the cooperator count of the group centred at (i,j),(i-1,j),(i+1,j),
// (i,j-1),(i,j+1) (group offsets read as (shift, axis), spgg.py:201).
__device__ __forceinline__ double payoff(const uint8_t* S, int i, int j, int L,
                                         const spgg_rep_params& p) {
  const int im1 = wrap(i - 1, L), ip1 = wrap(i + 1, L), im2 = wrap(i - 2, L), ip2 = wrap(i + 2, L);
  const int jm1 = wrap(j - 1, L), jp1 = wrap(j + 1, L), jm2 = wrap(j - 2, L), jp2 = wrap(j + 2, L);
#define C0(r, c) (S[(r) * L + (c)] == 0 ? 1 : 0)
  const int c_00 = C0(i, j), c_m0 = C0(im1, j), c_p0 = C0(ip1, j), c_0m = C0(i, jm1), c_0p = C0(i, jp1);
  const int c_mm = C0(im1, jm1), c_mp = C0(im1, jp1), c_pm = C0(ip1, jm1), c_pp = C0(ip1, jp1);
  const int c_M0 = C0(im2, j), c_P0 = C0(ip2, j), c_0M = C0(i, jm2), c_0P = C0(i, jp2);
#undef C0
  const int N[5] = {
      c_00 + c_m0 + c_p0 + c_0m + c_0p,   // group (0,0)       -> N0[i,j]
      c_m0 + c_M0 + c_00 + c_mm + c_mp,   // group (1,0)       -> N0[i-1,j]
      c_p0 + c_00 + c_P0 + c_pm + c_pp,   // group (-1,0)      -> N0[i+1,j]
      c_0m + c_mm + c_pm + c_0M + c_00,   // group (1,1)       -> N0[i,j-1]
      c_0p + c_mp + c_pp + c_00 + c_0P};  // group (-1,1)      -> N0[i,j+1]
  const double s0 = (double)c_00, s1 = (double)(1 - c_00);
  double tot = 0.0;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const double tk = (p.rc * (double)N[k]) / 5.0;
    const double pk = (tk - p.cost) * s0 + tk * s1;
    tot = (k == 0) ? pk : tot + pk;
  }
  return (tot - p.norm_min) / p.norm_den;
}

// Reputation state (spgg.py:292-307): mean of R over 5 / 13 offsets > 0,
// summed in the reference's offset order, starting from 0.0.
template <bool M2>
__device__ __forceinline__ int rep_state(const double* R, int i, int j, int L) {
  const int im1 = wrap(i - 1, L), ip1 = wrap(i + 1, L);
  const int jm1 = wrap(j - 1, L), jp1 = wrap(j + 1, L);
  // roll(R, (dx,dy))[i,j] = R[i-dx, j-dy]
  double acc = 0.0;
  acc += R[i * L + j];      // (0,0)
  acc += R[im1 * L + j];    // (1,0)
  acc += R[ip1 * L + j];    // (-1,0)
  acc += R[i * L + jm1];    // (0,1)
  acc += R[i * L + jp1];    // (0,-1)
  if constexpr (M2) {
    const int im2 = wrap(i - 2, L), ip2 = wrap(i + 2, L);
    const int jm2 = wrap(j - 2, L), jp2 = wrap(j + 2, L);
    acc += R[im2 * L + j];    // (2,0)
    acc += R[ip2 * L + j];    // (-2,0)
    acc += R[i * L + jm2];    // (0,2)
    acc += R[i * L + jp2];    // (0,-2)
    acc += R[im1 * L + jm1];  // (1,1)
    acc += R[im1 * L + jp1];  // (1,-1)
    acc += R[ip1 * L + jm1];  // (-1,1)
    acc += R[ip1 * L + jp1];  // (-1,-1)
    return (acc / 13.0) > 0.0 ? 1 : 0;
  } else {
    return (acc / 5.0) > 0.0 ? 1 : 0;
  }
}

// Value slots of the act reduction.
enum {
  V_PCT = 0, V_Q = 1, V_QC = 5, V_QD = 9,                 // -> slot t-1
  V_SUMP = 13, V_SUMP_C, V_SUMP_D, V_SUMR,                // -> slot t
  V_SWCD, V_SWDC, V_WPP, V_WRR, V_REWC, V_REWD, V_RATIO,  // -> slot t
  V_NCOOP1,                                               // -> slot t+1
  V_ACT_N
};
static_assert(V_ACT_N <= 32, "act reduction holds 32 values");

__device__ __forceinline__ int act_stat_index(int k, int* slot_delta) {
  if (k == V_PCT) { *slot_delta = -1; return SPGG_ST_SUM_PCT; }
  if (k < V_QC) { *slot_delta = -1; return SPGG_ST_SUMQ + (k - V_Q); }
  if (k < V_QD) { *slot_delta = -1; return SPGG_ST_SUMQ_C + (k - V_QC); }
  if (k < V_SUMP) { *slot_delta = -1; return SPGG_ST_SUMQ_D + (k - V_QD); }
  *slot_delta = 0;
  switch (k) {
    case V_SUMP: return SPGG_ST_SUMP;
    case V_SUMP_C: return SPGG_ST_SUMP_C;
    case V_SUMP_D: return SPGG_ST_SUMP_D;
    case V_SUMR: return SPGG_ST_SUMR;
    case V_SWCD: return SPGG_ST_SW_CD;
    case V_SWDC: return SPGG_ST_SW_DC;
    case V_WPP: return SPGG_ST_SUM_WPP;
    case V_WRR: return SPGG_ST_SUM_WRR;
    case V_REWC: return SPGG_ST_SUM_REW_C;
    case V_REWD: return SPGG_ST_SUM_REW_D;
    case V_RATIO: return SPGG_ST_SUM_RATIO_C;
    case V_NCOOP1: *slot_delta = 1; return SPGG_ST_NCOOP;
    default: return -1;
  }
}

// ---------------------------------------------------------------------------
template <bool M2, bool ACTION_STATE, int RNG>
__global__ __launch_bounds__(kBlock) void spgg_act_kernel(KArgs a, int t, int finalize_only) {
  __shared__ double lds[kWaves * 32];
  const int rep = blockIdx.y;
  const int st = a.stop_iter[rep];
  if (st != 0 && st < t) return;  // replica absorbed before t: nothing to do
  const spgg_rep_params p = a.params[rep];
  const int L = a.L, n = a.n;
  const size_t rb = (size_t)rep * n;
  double* srow = a.stats + (size_t)rep * a.slots * SPGG_NSTAT;
  const bool has_pending = t > 1;
  bool stop_now = false;
  if (!finalize_only) {
    const double nc = srow[(size_t)t * SPGG_NSTAT + SPGG_ST_NCOOP];
    stop_now = (nc == 0.0) || (nc == (double)n);  // spgg.py:405
    if (stop_now && blockIdx.x == 0 && threadIdx.x == 0) a.stop_iter[rep] = t;
  }
  double lam_den = 0.0;
  if (has_pending) lam_den = srow[(size_t)(t - 1) * SPGG_NSTAT + SPGG_ST_GMAX] + p.lambda_eps;
  const double eps_t = a.eps[(size_t)rep * a.slots + t];

  double v[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) v[k] = 0.0;

  const int beg = blockIdx.x * a.chunk;
  const int end = min(beg + a.chunk, n);
  for (int idx = beg + (int)threadIdx.x; idx < end; idx += kBlock) {
    const size_t g = rb + idx;
    const int i = idx / L, j = idx - (idx / L) * L;
    const int s_t = a.S_cur[g];
    double2* qp = reinterpret_cast<double2*>(a.Q + g * 4);
    const double2 q01 = qp[0], q23 = qp[1];
    double q[4] = {q01.x, q01.y, q23.x, q23.y};

    if (has_pending) {  // NI of iteration t-1, spgg.py:489-509 + 511-513, 561-583
      const int ax = a.aux[g];
      const int so = ax & 1, ps = (ax >> 1) & 1, dp = (ax >> 2) & 1;
      const double md = a.ni_md[g], atd = a.ni_atd[g];
      const double lam = (p.kappa * md) / lam_den;
      const double nu = lam * (dp ? 1.0 : -1.0);
      const int e = so * 2 + s_t;  // S_t is the action of iteration t-1
      const double qn = q_get(q, e) + nu;
      q_set(q, e, qn);
      a.Q[g * 4 + e] = qn;
      const double anu = fabs(nu);
      v[V_PCT] += anu / ((atd + anu) + 1e-8) * 100.0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[V_Q + k] += q[k];
        if (ps == 0) v[V_QC + k] += q[k]; else v[V_QD + k] += q[k];
      }
    }
    if (finalize_only) continue;

    // iteration-start record, spgg.py:373-394
    const double P = payoff(a.S_cur + rb, i, j, L, p);
    const double r_t = a.R_cur[g];
    v[V_SUMP] += P;
    if (s_t == 0) v[V_SUMP_C] += P; else v[V_SUMP_D] += P;
    v[V_SUMR] += r_t;
    if (stop_now) continue;

    // old state, spgg.py:409
    int so;
    if constexpr (ACTION_STATE) so = (s_t == 0) ? 1 : 0;
    else so = rep_state<M2>(a.R_cur + rb, i, j, L);

    // eps-greedy, algorithms.py:105-109
    int explore, rb_bit;
    if constexpr (RNG == SPGG_RNG_PHILOX) {
      const uint4 w = philox4x32_10(make_uint4((uint32_t)idx, (uint32_t)t, (uint32_t)rep, 0x53504747u),
                                    (uint32_t)p.seed, (uint32_t)(p.seed >> 32));
      explore = mt_double(w.x, w.y) < eps_t ? 1 : 0;
      rb_bit = (int)(w.z & 1u);
    } else {
      explore = a.explore[g];
      rb_bit = a.rbit[g];
    }
    const double qs0 = so ? q[2] : q[0], qs1 = so ? q[3] : q[1];
    const int greedy = (qs0 >= qs1) ? 0 : 1;  // argmax, ties -> 0
    const int act = explore ? rb_bit : greedy;

    // reputation, spgg.py:319-323
    double rn = r_t + (act == 0 ? p.rep_gain_c : p.neg_delta_r_d);
    rn = fmin(fmax(rn, p.r_min), p.r_max);
    a.R_nxt[g] = rn;
    a.S_nxt[g] = (uint8_t)act;

    // reward, spgg.py:424-427
    const double rr = (act == 0) ? 0.5 : 0.0;
    const double wpp = p.w_p * P, wrr = p.w_rep * rr;
    const double rew = wpp + wrr;
    a.reward[g] = rew;
    a.aux[g] = (uint8_t)(so | (s_t << 1));

    v[V_SWCD] += (s_t == 0 && act == 1) ? 1.0 : 0.0;
    v[V_SWDC] += (s_t == 1 && act == 0) ? 1.0 : 0.0;
    v[V_NCOOP1] += (act == 0) ? 1.0 : 0.0;
    v[V_WPP] += wpp;
    v[V_WRR] += wrr;
    if (act == 0) {
      v[V_REWC] += rew;
      v[V_RATIO] += (fabs(wrr) / (fabs(rew) + 1e-9)) * 100.0;
    } else {
      v[V_REWD] += rew;
    }
  }

  const double tot = block_reduce<32>(v, lds);
  if (threadIdx.x < V_ACT_N) {
    int dslot;
    const int k = act_stat_index(threadIdx.x, &dslot);
    const bool used = (dslot < 0) ? has_pending : !finalize_only;
    if (used && tot != 0.0) atomicAdd(&srow[(size_t)(t + dslot) * SPGG_NSTAT + k], tot);
  }
}

// ---------------------------------------------------------------------------
template <bool M2, bool ACTION_STATE>
__global__ __launch_bounds__(kBlock) void spgg_learn_kernel(KArgs a, int t) {
  __shared__ double lds[kWaves * 8 + kWaves];
  const int rep = blockIdx.y;
  const int st = a.stop_iter[rep];
  if (st != 0 && st <= t) return;
  const spgg_rep_params p = a.params[rep];
  const int L = a.L, n = a.n;
  const size_t rb = (size_t)rep * n;
  const uint8_t* S1 = a.S_nxt + rb;
  const double* rw = a.reward + rb;
  double* srow = a.stats + (size_t)rep * a.slots * SPGG_NSTAT;

  double v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = 0.0;
  double bmax = 0.0;

  const int beg = blockIdx.x * a.chunk;
  const int end = min(beg + a.chunk, n);
  for (int idx = beg + (int)threadIdx.x; idx < end; idx += kBlock) {
    const size_t g = rb + idx;
    const int i = idx / L, j = idx - (idx / L) * L;
    const int act = S1[idx];
    const int ax = a.aux[g];
    const int so = ax & 1;
    int sn;  // new state, spgg.py:423
    if constexpr (ACTION_STATE) sn = (act == 0) ? 1 : 0;
    else sn = rep_state<M2>(a.R_nxt + rb, i, j, L);
    const double rew = rw[idx];

    // Q-learning TD update, algorithms.py:121-131
    double2* qp = reinterpret_cast<double2*>(a.Q + g * 4);
    const double2 q01 = qp[0], q23 = qp[1];
    double q[4] = {q01.x, q01.y, q23.x, q23.y};
    const int e = so * 2 + act;
    const double qc = q_get(q, e);
    const double m = sn ? fmax(q[2], q[3]) : fmax(q[0], q[1]);
    const double td = (rew + p.gamma * m) - qc;
    const double q1 = qc + p.alpha * td;
    q_set(q, e, q1);
    a.Q[g * 4 + e] = q1;
    // diagnostic TD on the updated table, spgg.py:446-473
    const double m2 = sn ? fmax(q[2], q[3]) : fmax(q[0], q[1]);
    const double td2 = (rew + p.diag_gamma * m2) - q1;
    const double atd = fabs(p.diag_alpha * td2);

    // neighbor influence, spgg.py:477-494: d_k = roll(rew, o_k) - rew,
    // roll(X,(dx,dy))[i,j] = X[i-dx, j-dy]; first argmax wins ties.
    const int im1 = wrap(i - 1, L), ip1 = wrap(i + 1, L);
    const int jm1 = wrap(j - 1, L), jp1 = wrap(j + 1, L);
    constexpr int K = M2 ? 12 : 4;
    int nb[K];
    nb[0] = im1 * L + j;  // (1,0)
    nb[1] = ip1 * L + j;  // (-1,0)
    nb[2] = i * L + jm1;  // (0,1)
    nb[3] = i * L + jp1;  // (0,-1)
    if constexpr (M2) {
      const int im2 = wrap(i - 2, L), ip2 = wrap(i + 2, L);
      const int jm2 = wrap(j - 2, L), jp2 = wrap(j + 2, L);
      nb[4] = im2 * L + j;    // (2,0)
      nb[5] = ip2 * L + j;    // (-2,0)
      nb[6] = i * L + jm2;    // (0,2)
      nb[7] = i * L + jp2;    // (0,-2)
      nb[8] = im1 * L + jm1;  // (1,1)
      nb[9] = im1 * L + jp1;  // (1,-1)
      nb[10] = ip1 * L + jm1; // (-1,1)
      nb[11] = ip1 * L + jp1; // (-1,-1)
    }
    double md = rw[nb[0]] - rew;
    int ks = 0;
#pragma unroll
    for (int k = 1; k < K; ++k) {
      const double d = rw[nb[k]] - rew;
      if (d > md) { md = d; ks = k; }
    }
    int ksel = nb[0];
#pragma unroll
    for (int k = 1; k < K; ++k) ksel = (ks == k) ? nb[k] : ksel;
    const int dp = (S1[ksel] == act) ? 1 : 0;
    const double mdp = md > 0.0 ? md : 0.0;
    a.ni_md[g] = mdp;
    a.ni_atd[g] = atd;
    a.aux[g] = (uint8_t)(ax | (dp << 2));
    bmax = fmax(bmax, mdp);

    // group composition on S_{t+1}, spgg.py:585-592
    const int nd = act + S1[im1 * L + j] + S1[ip1 * L + j] + S1[i * L + jm1] + S1[i * L + jp1];
#pragma unroll
    for (int d = 0; d < 6; ++d) v[d] += (nd == d) ? 1.0 : 0.0;
    if (md > 0.0) {  // spgg.py:520-523
      v[6] += 1.0;
      if (ks >= 4) v[7] += 1.0;
    }
  }

  const double tot = block_reduce<8>(v, lds);
  double* slot = srow + (size_t)t * SPGG_NSTAT;
  if (threadIdx.x < 8 && tot != 0.0) {
    const int k = threadIdx.x < 6 ? SPGG_ST_GC0 + threadIdx.x
                                  : (threadIdx.x == 6 ? SPGG_ST_NMD_POS : SPGG_ST_NMD_POS2);
    atomicAdd(&slot[k], tot);
  }
  __syncthreads();
  const double bm = block_reduce_max(bmax, lds + kWaves * 8);
  if (threadIdx.x == 0 && bm > 0.0) {
    // non-negative doubles order like their bit patterns (spgg.py:488)
    atomicMax(reinterpret_cast<unsigned long long*>(&slot[SPGG_ST_GMAX]),
              (unsigned long long)__double_as_longlong(bm));
  }
}

// ---------------------------------------------------------------------------
// Device MT19937, bit-identical to numpy.random.RandomState (legacy seeding,
// randomkit mt19937_gen + tempering).  One workgroup per replica owns its
// 624-word key in LDS; the twist runs in three dependency phases.
// Per executed iteration the reference draws rand(L,L) (2 words per double,
// algorithms.py:105) then randint(0,2,(L,L)) (1 word each, algorithms.py:108).
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

__device__ __forceinline__ uint32_t mt_mix(uint32_t hi, uint32_t lo, uint32_t far) {
  const uint32_t y = (hi & 0x80000000u) | (lo & 0x7fffffffu);
  return far ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

__device__ void mt_twist(uint32_t* mt) {
  const int i = threadIdx.x;
  uint32_t o_i = 0, o_i1 = 0, o_far = 0;
  if (i < 624) {
    o_i = mt[i];
    if (i < 623) o_i1 = mt[i + 1];
    if (i < 227) o_far = mt[i + 397];
  }
  __syncthreads();
  if (i < 227) mt[i] = mt_mix(o_i, o_i1, o_far);
  __syncthreads();
  if (i >= 227 && i < 454) mt[i] = mt_mix(o_i, o_i1, mt[i - 227]);
  __syncthreads();
  if (i >= 454 && i < 624) mt[i] = mt_mix(o_i, (i == 623) ? mt[0] : o_i1, mt[i - 227]);
  __syncthreads();
}

__global__ __launch_bounds__(kMtThreads) void spgg_mt_draw_kernel(
    uint32_t* mt_state, uint8_t* explore, uint8_t* rbit, const double* eps, const double* stats,
    const int* stop_iter, int n, int slots, int t) {
  __shared__ uint32_t mt[624];
  __shared__ uint32_t carry;
  const int rep = blockIdx.x;
  const int st = stop_iter[rep];
  if (st != 0 && st < t) return;
  const double nc = stats[((size_t)rep * slots + t) * SPGG_NSTAT + SPGG_ST_NCOOP];
  if (nc == 0.0 || nc == (double)n) return;  // absorbing: no draw this iteration
  uint32_t* gstate = mt_state + (size_t)rep * 625;
  const int tid = threadIdx.x;
  if (tid < 624) mt[tid] = gstate[tid];
  int pos = (int)gstate[624];
  __syncthreads();
  const double e = eps[(size_t)rep * slots + t];
  uint8_t* ex = explore + (size_t)rep * n;
  uint8_t* rb = rbit + (size_t)rep * n;
  const long long total = 3LL * n, nu = 2LL * n;
  long long produced = 0;
  while (produced < total) {
    if (pos == 624) {
      mt_twist(mt);
      pos = 0;
    }
    const int avail = (int)min((long long)(624 - pos), total - produced);
    if (tid >= pos && tid < pos + avail) {
      const long long w = produced + (tid - pos);
      const uint32_t y = mt_temper(mt[tid]);
      if (w < nu) {
        if ((w & 1) == 0) {
          if (tid + 1 < pos + avail) ex[w >> 1] = mt_double(y, mt_temper(mt[tid + 1])) < e ? 1 : 0;
          else carry = y;  // pair straddles the key block
        } else if (tid == pos) {
          ex[w >> 1] = mt_double(carry, y) < e ? 1 : 0;
        }
      } else {
        rb[w - nu] = (uint8_t)(y & 1u);
      }
    }
    produced += avail;
    pos += avail;
    __syncthreads();
  }
  if (tid < 624) gstate[tid] = mt[tid];
  if (tid == 0) gstate[624] = (uint32_t)pos;
}

// P of every agent from S_t (epilogue: SPGG.P / run()'s mean(P), spgg.py:378, 637).
__global__ __launch_bounds__(kBlock) void spgg_payoff_kernel(const uint8_t* S, const spgg_rep_params* params,
                                                             double* out, int L, int n) {
  const int rep = blockIdx.y;
  const int idx = blockIdx.x * kBlock + threadIdx.x;
  if (idx >= n) return;
  const spgg_rep_params p = params[rep];
  const int i = idx / L, j = idx - (idx / L) * L;
  out[(size_t)rep * n + idx] = payoff(S + (size_t)rep * n, i, j, L, p);
}

}  // namespace

// ===========================================================================
// C ABI
struct spgg_ctx {
  spgg_config cfg{};
  spgg_buffers buf{};
  bool bound = false;
  bool params_set = false;
  spgg_rep_params* d_params = nullptr;
  int n = 0;
  int chunk = kBlock;
  int blocks_x = 1;
  std::string err;
};

namespace {

int fail(spgg_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

int hip_check(spgg_ctx* c, hipError_t e, const char* what) {
  if (e == hipSuccess) return SPGG_OK;
  return fail(c, SPGG_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

KArgs make_args(const spgg_ctx* c, int t) {
  KArgs a{};
  const int cur = (t - 1) & 1, nxt = t & 1;
  a.S_cur = c->buf.S[cur];
  a.S_nxt = c->buf.S[nxt];
  a.R_cur = c->buf.R[cur];
  a.R_nxt = c->buf.R[nxt];
  a.Q = c->buf.Q;
  a.reward = c->buf.reward;
  a.aux = c->buf.aux;
  a.ni_md = c->buf.ni_md;
  a.ni_atd = c->buf.ni_atd;
  a.explore = c->buf.explore;
  a.rbit = c->buf.rbit;
  a.eps = c->buf.eps;
  a.stats = c->buf.stats;
  a.stop_iter = c->buf.stop_iter;
  a.params = c->d_params;
  a.L = c->cfg.L;
  a.n = c->n;
  a.chunk = c->chunk;
  a.slots = c->cfg.iterations + 2;
  return a;
}

template <bool M2, bool AS, int RNG>
void launch_act(const KArgs& a, dim3 grid, int t, int fin, hipStream_t s) {
  hipLaunchKernelGGL((spgg_act_kernel<M2, AS, RNG>), grid, dim3(kBlock), 0, s, a, t, fin);
}

template <bool M2, bool AS>
void launch_act_rng(const KArgs& a, dim3 grid, int t, int fin, int rng, hipStream_t s) {
  if (rng == SPGG_RNG_PHILOX) launch_act<M2, AS, SPGG_RNG_PHILOX>(a, grid, t, fin, s);
  else launch_act<M2, AS, SPGG_RNG_MT19937>(a, grid, t, fin, s);  // INJECT reads the same bytes
}

void launch_act_any(const spgg_ctx* c, const KArgs& a, dim3 grid, int t, int fin, hipStream_t s) {
  const bool m2 = c->cfg.second_order != 0;
  const bool as = c->cfg.state_mode == SPGG_STATE_ACTION;
  const int rng = c->cfg.rng_mode;
  if (m2) {
    if (as) launch_act_rng<true, true>(a, grid, t, fin, rng, s);
    else launch_act_rng<true, false>(a, grid, t, fin, rng, s);
  } else {
    if (as) launch_act_rng<false, true>(a, grid, t, fin, rng, s);
    else launch_act_rng<false, false>(a, grid, t, fin, rng, s);
  }
}

void launch_learn_any(const spgg_ctx* c, const KArgs& a, dim3 grid, int t, hipStream_t s) {
  const bool m2 = c->cfg.second_order != 0;
  const bool as = c->cfg.state_mode == SPGG_STATE_ACTION;
  if (m2) {
    if (as) hipLaunchKernelGGL((spgg_learn_kernel<true, true>), grid, dim3(kBlock), 0, s, a, t);
    else hipLaunchKernelGGL((spgg_learn_kernel<true, false>), grid, dim3(kBlock), 0, s, a, t);
  } else {
    if (as) hipLaunchKernelGGL((spgg_learn_kernel<false, true>), grid, dim3(kBlock), 0, s, a, t);
    else hipLaunchKernelGGL((spgg_learn_kernel<false, false>), grid, dim3(kBlock), 0, s, a, t);
  }
}

void launch_draw(const spgg_ctx* c, int t, hipStream_t s) {
  hipLaunchKernelGGL(spgg_mt_draw_kernel, dim3(c->cfg.n_rep), dim3(kMtThreads), 0, s,
                     c->buf.mt_state, c->buf.explore, c->buf.rbit, c->buf.eps, c->buf.stats,
                     c->buf.stop_iter, c->n, c->cfg.iterations + 2, t);
}

}  // namespace

extern "C" {

int spgg_abi_version(void) { return SPGG_ABI_VERSION; }

const char* spgg_last_error(const spgg_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int spgg_create(spgg_ctx** out, const spgg_config* cfg) {
  if (!out || !cfg) return SPGG_E_ARG;
  *out = nullptr;
  if (cfg->n_rep < 1 || cfg->L < 1 || cfg->iterations < 0 || (long long)cfg->L * cfg->L > (1LL << 30))
    return SPGG_E_ARG;
  if (cfg->state_mode != SPGG_STATE_REPUTATION && cfg->state_mode != SPGG_STATE_ACTION) return SPGG_E_ARG;
  if (cfg->rng_mode < SPGG_RNG_INJECT || cfg->rng_mode > SPGG_RNG_PHILOX) return SPGG_E_ARG;
  if (cfg->n_rep > 65535) return SPGG_E_ARG;
  spgg_ctx* c = new (std::nothrow) spgg_ctx();
  if (!c) return SPGG_E_ARG;
  c->cfg = *cfg;
  c->n = cfg->L * cfg->L;
  // Agents per workgroup: grow while the batch still fills >= 2048 workgroups.
  int apt = 1;
  while (apt < 8) {
    const long long per = (long long)kBlock * apt * 2;
    const long long blocks = (long long)cfg->n_rep * ((c->n + per - 1) / per);
    if (blocks < 2048) break;
    apt *= 2;
  }
  c->chunk = kBlock * apt;
  c->blocks_x = (c->n + c->chunk - 1) / c->chunk;
  int rc = hip_check(c, hipSetDevice(cfg->device), "hipSetDevice");
  if (rc) { delete c; return rc; }
  *out = c;
  return SPGG_OK;
}

int spgg_set_params(spgg_ctx* c, const spgg_rep_params* params) {
  if (!c || !params) return fail(c, SPGG_E_ARG, "null argument");
  int rc = hip_check(c, hipSetDevice(c->cfg.device), "hipSetDevice");
  if (rc) return rc;
  const size_t bytes = sizeof(spgg_rep_params) * c->cfg.n_rep;
  if (!c->d_params) {
    rc = hip_check(c, hipMalloc(&c->d_params, bytes), "hipMalloc(params)");
    if (rc) return rc;
  }
  rc = hip_check(c, hipMemcpy(c->d_params, params, bytes, hipMemcpyHostToDevice), "hipMemcpy(params)");
  if (rc) return rc;
  c->params_set = true;
  return SPGG_OK;
}

int spgg_bind(spgg_ctx* c, const spgg_buffers* b) {
  if (!c || !b) return fail(c, SPGG_E_ARG, "null argument");
  if (!b->S[0] || !b->S[1] || !b->R[0] || !b->R[1] || !b->Q || !b->reward || !b->aux || !b->ni_md ||
      !b->ni_atd || !b->eps || !b->stats || !b->stop_iter)
    return fail(c, SPGG_E_ARG, "spgg_bind: a required buffer is null");
  if (c->cfg.rng_mode != SPGG_RNG_PHILOX && (!b->explore || !b->rbit))
    return fail(c, SPGG_E_ARG, "spgg_bind: explore/rbit buffers required for INJECT/MT19937");
  if (c->cfg.rng_mode == SPGG_RNG_MT19937 && !b->mt_state)
    return fail(c, SPGG_E_ARG, "spgg_bind: mt_state required for MT19937");
  if ((reinterpret_cast<uintptr_t>(b->Q) & 15) != 0)
    return fail(c, SPGG_E_ARG, "spgg_bind: Q must be 16-byte aligned");
  c->buf = *b;
  c->bound = true;
  return SPGG_OK;
}

int spgg_step(spgg_ctx* c, int32_t t0, int32_t n_steps, void* stream) {
  if (!c) return SPGG_E_ARG;
  if (!c->bound || !c->params_set) return fail(c, SPGG_E_STATE, "spgg_step before bind/set_params");
  if (t0 < 1 || n_steps < 0 || (long long)t0 + n_steps - 1 > c->cfg.iterations)
    return fail(c, SPGG_E_ARG, "spgg_step: iteration range outside [1, iterations]");
  if (c->cfg.rng_mode == SPGG_RNG_INJECT && n_steps > 1)
    return fail(c, SPGG_E_ARG, "spgg_step: INJECT mode steps one iteration per call");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid(c->blocks_x, c->cfg.n_rep);
  for (int t = t0; t < t0 + n_steps; ++t) {
    const KArgs a = make_args(c, t);
    if (c->cfg.rng_mode == SPGG_RNG_MT19937) launch_draw(c, t, s);
    launch_act_any(c, a, grid, t, 0, s);
    launch_learn_any(c, a, grid, t, s);
  }
  return hip_check(c, hipGetLastError(), "spgg_step launch");
}

int spgg_flush(spgg_ctx* c, int32_t t_last, void* stream) {
  if (!c) return SPGG_E_ARG;
  if (!c->bound || !c->params_set) return fail(c, SPGG_E_STATE, "spgg_flush before bind/set_params");
  if (t_last < 1 || t_last > c->cfg.iterations) return fail(c, SPGG_E_ARG, "spgg_flush: bad t_last");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid(c->blocks_x, c->cfg.n_rep);
  launch_act_any(c, make_args(c, t_last + 1), grid, t_last + 1, 1, s);
  return hip_check(c, hipGetLastError(), "spgg_flush launch");
}

int spgg_draw(spgg_ctx* c, int32_t t, void* stream) {
  if (!c) return SPGG_E_ARG;
  if (!c->bound || c->cfg.rng_mode != SPGG_RNG_MT19937)
    return fail(c, SPGG_E_STATE, "spgg_draw needs a bound MT19937 context");
  if (t < 1 || t > c->cfg.iterations) return fail(c, SPGG_E_ARG, "spgg_draw: bad t");
  launch_draw(c, t, reinterpret_cast<hipStream_t>(stream));
  return hip_check(c, hipGetLastError(), "spgg_draw launch");
}

int spgg_payoff(spgg_ctx* c, int32_t t, double* out, void* stream) {
  if (!c || !out) return fail(c, SPGG_E_ARG, "null argument");
  if (!c->bound || !c->params_set) return fail(c, SPGG_E_STATE, "spgg_payoff before bind/set_params");
  if (t < 1) return fail(c, SPGG_E_ARG, "spgg_payoff: bad t");
  const dim3 grid((c->n + kBlock - 1) / kBlock, c->cfg.n_rep);
  hipLaunchKernelGGL(spgg_payoff_kernel, grid, dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream),
                     c->buf.S[(t - 1) & 1], c->d_params, out, c->cfg.L, c->n);
  return hip_check(c, hipGetLastError(), "spgg_payoff launch");
}

int spgg_destroy(spgg_ctx* c) {
  if (!c) return SPGG_OK;
  if (c->d_params) {
    (void)hipSetDevice(c->cfg.device);
    (void)hipFree(c->d_params);
  }
  delete c;
  return SPGG_OK;
}

}  // extern "C"
