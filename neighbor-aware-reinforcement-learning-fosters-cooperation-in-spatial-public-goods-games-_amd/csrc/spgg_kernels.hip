// spgg_kernels.hip — MI355X (gfx950) kernels for the SPGG per-iteration hot path.
//
// ONE launch per iteration t of the reference's run loop
// (src/model/spgg.py:368-592) covers every replica of the batch.  A
// workgroup owns a TH x TW tile of one replica's periodic L x L lattice:
//
//   phase 0  stage S_t (halo M+2) and R_t (halo 2M) of the tile in LDS; load
//            the owned agents' Q and pending neighbor-influence (NI) record
//   phase 1  owned agents: apply the deferred NI term of iteration t-1
//            (+ its Q statistics) -> payoff P (13-cell stencil) -> iteration
//            start record -> absorbing-stop check -> state s from R_t ->
//            eps-greedy action -> R_{t+1}, reward.  The ring of neighbours at
//            distance <= M (owned by other workgroups) is recomputed the same
//            way, so every reward/action the tile's NI needs is in LDS.
//   phase 2  owned agents: s' from R_{t+1} -> Q-learning TD -> diagnostic TD
//            -> NI max/argmax over 4 (M=1) / 12 (M=2) neighbour rewards ->
//            pending NI record, lattice-wide max |diff| (atomic), S_{t+1}.
//
// The NI term divides by a lattice-wide max (spgg.py:488), so it is applied
// one launch later (or by spgg_flush) with the reference's exact arithmetic:
//   Q[s,a] = (qc + alpha*td) + (kappa*max(0,md))/(gmax+lambda_eps) * (+-1).
// Q and the pending max_diff are ping-ponged by iteration parity: a launch
// reads only buffers the previous launch wrote, so the ring recompute never
// races another workgroup's writes.
//
// Every float op that feeds the simulation is f64 in the reference's
// evaluation order; compiled with -ffp-contract=off (no FMA contraction).
// History values are reduced per workgroup (wave butterfly + LDS) and added
// with one f64 atomic per value per workgroup.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <numeric>
#include <type_traits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "spgg_abi.h"
#include "spgg_test.h"
#include "spgg_device.h"
#include "spgg_mt.h"

using namespace spgg;

// Timing-only ablation builds (-DSPGG_ABLATE=mask; results are WRONG):
//   1 = cheap hash instead of Philox, 2 = no history atomics, 4 = no ring recompute,
//   8 = no history reductions (NCOOP kept constant), 64 = empty workgroups (launch floor),
//   16 = no workgroup totals (final barrier + epilogue), 512 = no per-agent Q / md / atd loads
//   (synthetic values), 2048 = no per-agent Q / md / atd stores, 8192 = no md loads / stores (the
//   pending NI term reads +0), 16384 (with 8) = the lattice-wide max still recorded (the dynamics
//   of the product), 32768 = no NI percent (its |alpha*td'| dead), 65536 = no phase-1b value
//   reductions, 131072 = no counter reductions (NCOOP kept constant), 4096 = Q plane 0 read only (plane 1's
//   entries copied from it), 128 = memory only (the owned loads,
//   staging and stores, no compute)
#ifndef SPGG_ABLATE
#define SPGG_ABLATE 0
#endif
#ifndef SPGG_PRIO  // A/B probe: s_setprio of the load phase
#define SPGG_PRIO 0
#endif
#ifndef SPGG_QNT  // A/B probe: bit 0 Q loads, bit 1 Q stores non-temporal (not for Double-Q)
#define SPGG_QNT 0
#endif
#ifndef SPGG_QSTORE  // A/B probe: 0 changed rows, 1 both rows, 2 rows changed anywhere in the 8-agent line, 3 in the lane pair, 4 in the 8-lane group (DPP)
#define SPGG_QSTORE 0
#endif
// (Rejected A/B knobs -- reward-code pending records, partial Q stores, non-temporal
// per-agent streams, wave priorities -- live in profiles/r02/rejected_knobs.patch with
// their measurements.)

// Build layout: this file is compiled once per RL operator with
// -DSPGG_TU=<SPGG_ALG_*> (that operator's step kernels only) and once with
// -DSPGG_TU=9 (C ABI, MT19937 and payoff kernels); without SPGG_TU it is one
// translation unit with everything.  The pieces meet in spgg_impl.
#ifndef SPGG_TU
#define SPGG_TU (-1)
#endif
#define SPGG_TU_HAS_ALG(k) (SPGG_TU == -1 || SPGG_TU == (k))
#define SPGG_TU_HAS_HOST (SPGG_TU == -1 || SPGG_TU == 9)

namespace spgg_impl {

struct TileArgs {
  const uint8_t* S_in;    // S_t   (bit0 strategy, bits1-4 bookkeeping of iteration t-1)
  uint8_t* S_out;         // S_{t+1}
  const void* R_in;       // f64, or int8 units of rep_unit (compact reputation)
  void* R_out;
  double* Q;              // [rep][state plane s][n][QW/2], IN PLACE: after TD of t-1, before its NI term
  double* md;             // [rep][n], IN PLACE: max(0, max_diff) of iteration t-1
  const double* pub_in;   // border records of iteration t-1 (ring recompute reads them)
  double* pub_out;        // border records of iteration t
  float* atd;             // [rep][n], IN PLACE: |alpha*td'| of iteration t-1 (diagnostic)
  const uint32_t* draws;  // draw record of THIS iteration (INJECT / MT19937): [rep][word][plane] bits
  int draw_words;         // u32 words per replica (draw_words_of: 32-agent words x planes)
  int planes;             // draw planes per iteration (draw_planes)
  const double* eps;
  double* stats;          // [rep][stripe][slot][NSTAT]: a workgroup adds to stripe tile % stripes
  int* stop_iter;
  const spgg_rep_params* params;
  const int2* ring;       // [tiles_per_rep][ring_max]: {agent index, border-record offset}, then the
                          // border-slot table: [4 tile shapes][kBlock] x 4 int16 (border_slot_table)
  int L, n, TW, TH, tiles_x, tiles_per_rep, n_rep, slots;
  int PB;                 // border-record slots per tile (pub_slots)
  int ring_max;
  int stripes;            // history-record stripes per replica (spgg_stat_stripes)
  int rep_stride;         // replica of the launch's j-th tile range: (j * rep_stride) % n_rep (rep_stride_for)
};

// What a step launch needs to pick and size the kernel instance.
struct LaunchCfg {
  int m2, as, rq, rng, twc, total_tiles;
  int apt;  // agents per thread: apt_of(alg), or 1 for small batches
  size_t lds_bytes;
};

// A persistent launch (spgg_persist_kernel): iterations t0 .. t_end in one launch.  The buffers
// a neighbouring workgroup reads are ping-ponged by iteration parity as between launches (S, R,
// border records), so the kernel picks them per iteration from both halves; the draw record of
// iteration t is ring slot (t-1) % draw_slots.  Between two iterations each workgroup arrives at
// its replica's counters (one per shard: tile % shards) and waits for every tile of the replica:
// counter j reaches tiles_in_shard(j) x (base + k) after the k-th barrier of this launch (base:
// the barriers this run's earlier persistent launches completed; the counters are zeroed at the
// run's first one).
struct PersistArgs {
  uint8_t* S[2];
  void* R[2];
  double* pub[2];
  const uint32_t* draws0;  // draw ring slot 0 (INJECT / MT19937; null for Philox)
  long long draw_stride;   // u32 words between ring slots
  int draw_slots;
  int t_end;               // last iteration of the launch
  uint32_t* bar;           // arrival counters [n_rep][shards][kBarWords] (one 64-byte line each)
  int shards;
  uint32_t base;
  uint32_t* err;           // error word: SPGG_STEP_ERR_BARRIER when a wait ran out of its bound
  uint32_t* err_host;      // its pinned host copy (device-mapped), set by the failing workgroup itself:
                           // spgg_status reads it without a copy enqueued after every launch
};
constexpr int kBarWords = 16;

// Enqueue one step-kernel launch of operator ALG (defined in that operator's TU): iteration t
// (pa == nullptr), or the persistent launch of iterations t .. pa->t_end.
template <int ALG>
void launch_alg(const LaunchCfg& lc, const TileArgs& a, int t, int fin, hipStream_t s,
                const PersistArgs* pa = nullptr);
// Workgroups of the persistent instance for lc that one CU holds at once (0: no such instance).
template <int ALG>
int persist_blocks_per_cu(const LaunchCfg& lc);

// Agents per thread of operator ALG's kernel: tiles of up to 1024 agents
// (Double-Q, holding two tables in registers: 512).
constexpr int apt_of(int alg) { return (alg == SPGG_ALG_DOUBLE_Q ? 512 : 1024) / kBlock; }
// Per-thread register windows of the flattened staging walk (S / R halos of a
// tile of <= 1024 agents; host-checked).
constexpr int js_of(bool m2) { return kBlock == 256 ? (m2 ? 8 : 7) : 4; }
constexpr int jr_of() { return kBlock == 256 ? 6 : 3; }
// Ring cells per thread: ring = (tw+2M)(th+2M) - tw*th <= 4M*(56+64)/2 + 4M^2 for
// tiles of <= 1024 agents (host-checked against ring_max).
constexpr int ring_per_thread(bool m2) { return kBlock == 256 && m2 ? 2 : 1; }
// Doubles per agent in Q and fields per border record (Double-Q: both tables).
constexpr int qw_of(int alg) { return alg == SPGG_ALG_DOUBLE_Q ? 8 : 4; }
constexpr int pf_of(int alg) { return alg == SPGG_ALG_DOUBLE_Q ? 5 : 3; }

// Border records.  An agent within HA cells of its tile's edge is read by the
// ring recompute of a neighbouring tile (every ring cell of a tile is a border
// cell of its owner, for any tiling and wrap).  Slots of a th x tw tile: the
// HA top rows, the HA bottom rows, then HA left + HA right cells of each
// middle row (row-major within each part, so tile edges read coalesced).
__host__ __device__ inline int pub_slots(int TW, int TH, int HA) {
  return 2 * HA * TW + (TH > 2 * HA ? (TH - 2 * HA) * 2 * HA : 0);
}
__host__ __device__ inline bool is_border(int r, int c, int th, int tw, int HA) {
  return r < HA || r >= th - HA || c < HA || c >= tw - HA;
}
__host__ __device__ inline int border_slot(int r, int c, int th, int tw, int HA) {
  if (r < HA) return r * tw + c;
  if (r >= th - HA) return (r - th + 2 * HA) * tw + c;
  const int cc = c < HA ? c : c - tw + 2 * HA;
  return 2 * HA * tw + (r - HA) * 2 * HA + cc;
}
// The same slot, or -1 for an interior cell, without branches (the host tabulates it per
// tile shape and thread for the step kernel's store phase: border_slot_table).
__host__ __device__ inline int border_slot_or_none(int r, int c, int th, int tw, int HA) {
  const bool top = r < HA, bot = r >= th - HA;
  const bool left = c < HA, right = c >= tw - HA;
  const int band = (top ? r : r - th + 2 * HA) * tw + c;
  const int side = 2 * HA * tw + (r - HA) * 2 * HA + (left ? c : c - tw + 2 * HA);
  return (top || bot) ? band : ((left || right) ? side : -1);
}

// Ring cell k of a th x tw tile in region coordinates (ay, ax) of the
// (th + 2HA) x (tw + 2HA) window: the HA rows above, the HA rows below, then
// HA cells left and right of each tile row.  k < (tw+2HA)(th+2HA) - th*tw.
__host__ __device__ inline void ring_cell(int k, int th, int tw, int HA, int* ay, int* ax) {
  const int aw = tw + 2 * HA, band = HA * aw;
  if (k < band) {
    *ay = k / aw;
    *ax = k - *ay * aw;
  } else if (k < 2 * band) {
    const int k2 = k - band;
    *ay = HA + th + k2 / aw;
    *ax = k2 - (k2 / aw) * aw;
  } else {
    const int k3 = k - 2 * band;
    *ay = HA + k3 / (2 * HA);
    const int cc = k3 - (k3 / (2 * HA)) * (2 * HA);
    *ax = cc < HA ? cc : tw + cc;
  }
}

}  // namespace spgg_impl

using spgg_impl::TileArgs;

namespace {


struct LdsLayout {
  int sw, sh, aw, ah;
  int off_Rew, off_R, off_Rn, off_S, off_D, off_A, off_PC, off_DR, off_DP, bytes;
};

// Staged draw bits (MT19937 / inject, compile-time-width tiles): per region row, the draw-record
// words (planes 0, 1) of kDrawSlots 32-agent groups -- 3 from the row's first cell (x0 - HA),
// 3 from column 0 (the cells past the periodic wrap) -- and, repacked, the row's 64 region cells.
constexpr int kDrawSlots = 6;

// Pitch of the plus-count plane: one 64-lane wave row per region row.
constexpr int kPcPitch = 64;

// 16-byte aligned carve: f64 first, then the R planes (rsz = 8 or 1), then bytes.
// S and defector-bit planes: tile + halo HS (payoffs over tile + HA); the
// plus-count plane: tile + HA + 1 rows of kPcPitch; everything else tile + HA.
// dword_rows (compile-time-width kernels): every plane has one dword-aligned
// pitch wide enough for a window staged as aligned dwords (window column j at
// plane column j + its 0..3-byte misalignment).
__host__ __device__ inline LdsLayout lds_layout(int tw, int th, int HS, int HA, int rsz, bool dword_rows = false,
                                                bool draws = false) {
  LdsLayout l;
  l.sw = tw + 2 * HS; l.sh = th + 2 * HS;
  l.aw = tw + 2 * HA; l.ah = th + 2 * HA;
  if (dword_rows) l.sw = l.aw = (tw + 2 * HS + 3 + 3) / 4 * 4;
  const int na = l.aw * l.ah;
  int off = (12 + kWaves * 64) * 8;  // payoff table + reduction scratch
  l.off_Rew = off;  off += ((na * 8 + 15) / 16) * 16;
  l.off_R = off;    off += ((na * rsz + 15) / 16) * 16;
  l.off_Rn = off;   off += ((na * rsz + 15) / 16) * 16;
  l.off_S = off;    off += ((l.sw * l.sh + 15) / 16) * 16;
  l.off_D = off;    off += ((l.sw * l.sh + kPcPitch + 15) / 16) * 16;  // + slack: full-wave row reads
  l.off_A = off;    off += ((na + 15) / 16) * 16;
  l.off_PC = off;   off += (l.ah + 2) * kPcPitch;
  off = (off + 15) / 16 * 16;
  l.off_DR = off;   off += draws ? l.ah * kDrawSlots * 2 * 4 : 0;
  l.off_DP = off;   off += draws ? l.ah * 2 * 2 * 4 : 0;
  l.bytes = off;
  return l;
}

// Element i of a per-replica array: scalar base + zero-extended 32-bit byte
// offset, so every access is one global_load/store in saddr form with no
// 64-bit address arithmetic (the host keeps each per-replica array < 4 GiB).
// (char-pointer arithmetic, not an integer round trip: the compiler must still
// see a global pointer, or it falls back to flat instructions.)
template <typename T>
__device__ __forceinline__ T* at(T* base, uint32_t i) {
  using B = typename std::conditional<std::is_const<T>::value, const char, char>::type;
  return reinterpret_cast<T*>(reinterpret_cast<B*>(base) + (size_t)(i * (uint32_t)sizeof(T)));
}

// A load / store of element p, plain or (SC1: inside a persistent launch, for bytes another
// workgroup reads) write-through / past the CU's L1 -- relaxed agent-scope atomics, lowered to
// global_load / global_store ... sc1 (the hand-off rules: replica_barrier below).
#ifndef SPGG_PERSIST_PLAIN  // timing variant: plain hand-off accesses (results may be stale: WRONG)
#define SPGG_PERSIST_PLAIN 0
#endif
#ifndef SPGG_PERSIST_STAGGER  // timing variant: s_sleep(16) x this per stagger rank after each barrier
#define SPGG_PERSIST_STAGGER 0
#endif
#ifndef SPGG_PERSIST_NORECOMP  // timing variant: see step_impl's CARRY
#define SPGG_PERSIST_NORECOMP 0
#endif
template <bool SC1, typename T>
__device__ __forceinline__ T hload(const T* p) {
  if constexpr (SC1 && !SPGG_PERSIST_PLAIN) return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}
template <bool SC1, typename T>
__device__ __forceinline__ void hstore(T* p, T v) {
  if constexpr (SC1 && !SPGG_PERSIST_PLAIN) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

// Compact reputation: when rep_gain_C, delta_R_D, R_min, R_max are multiples
// of a dyadic unit u with |R/u| <= 127 (host-checked), every R the reference
// can produce is k*u exactly, its f64 sums and clip are exact, and
// (sum/n > 0) <=> (sum of k > 0): int8 storage is bit-identical.
template <bool RQ>
using RStore = typename std::conditional<RQ, int8_t, double>::type;
template <bool RQ>
using RVal = typename std::conditional<RQ, int, double>::type;

template <bool RQ, typename PT>
__device__ __forceinline__ RVal<RQ> rep_next(RVal<RQ> r, int act, const PT& p) {
  if constexpr (RQ) {  // spgg.py:321-323 in units of rep_unit
    const int k = r + (act == 0 ? p.rk_gain : -p.rk_loss);
    return min(max(k, p.rk_min), p.rk_max);
  } else {             // spgg.py:321-323
    const double x = r + (act == 0 ? p.rep_gain_c : p.neg_delta_r_d);
    return fmin(fmax(x, p.r_min), p.r_max);
  }
}

template <bool M2>
__device__ __forceinline__ int rep_state_lds(const int8_t* R, int c, int w) {
  int acc = R[c] + R[c - w] + R[c + w] + R[c - 1] + R[c + 1];
  if constexpr (M2)
    acc += R[c - 2 * w] + R[c + 2 * w] + R[c - 2] + R[c + 2] + R[c - w - 1] + R[c - w + 1] + R[c + w - 1] +
           R[c + w + 1];
  return acc > 0 ? 1 : 0;
}

// Reputation sum in the reference's offset order (spgg.py:296-305):
// roll(R,(dx,dy))[i,j] = R[i-dx, j-dy]; acc starts at 0.0.
template <bool M2>
__device__ __forceinline__ int rep_state_lds(const double* R, int c, int w) {
  double acc = 0.0;
  acc += R[c];          // (0,0)
  acc += R[c - w];      // (1,0)
  acc += R[c + w];      // (-1,0)
  acc += R[c - 1];      // (0,1)
  acc += R[c + 1];      // (0,-1)
  if constexpr (M2) {
    acc += R[c - 2 * w];  // (2,0)
    acc += R[c + 2 * w];  // (-2,0)
    acc += R[c - 2];      // (0,2)
    acc += R[c + 2];      // (0,-2)
    acc += R[c - w - 1];  // (1,1)
    acc += R[c - w + 1];  // (1,-1)
    acc += R[c + w - 1];  // (-1,1)
    acc += R[c + w + 1];  // (-1,-1)
  }
  return acc >= rep_threshold(M2) ? 1 : 0;
}

// The deferred NI term nu of iteration t-1 (spgg.py:489-509): lambda times
// +-1 by whether the best neighbour's action matched (S_t bit 2).
__device__ __forceinline__ double pending_nu(uint8_t b, double md, double kappa, double lam_den, double lam_rcp) {
  const double lam = div_uniform(kappa * md, lam_den, lam_rcp);  // (kappa*max(0,md))/(gmax+eps)
  return ((b >> 2) & 1) ? lam : -lam;  // lam * (+-1.0): exact sign flip
}

// (s_old, a) entry index of iteration t-1 recorded in S_t bits 0-1.
__device__ __forceinline__ int pending_entry(uint8_t b) { return ((b >> 1) & 1) * 2 + (b & 1); }

// Wave sums of K values into red[wave*64 + base + k] (f64, or packed integer
// counters stored as exact doubles).
// (tid: the thread's index -- threadIdx.x, passed in so that a persistent launch's loop can make it
// opaque per iteration: derived lane values are then recomputed instead of held across iterations)
template <int K, typename T>
__device__ __forceinline__ void wave_partials(T (&v)[K], double* red, int base, int tid) {
  transpose_level<K, 32, K, T>(v, tid & 63);
  const int lane = tid & 63, wave = tid >> 6;
  constexpr int per = 64 / K;
  if ((lane & (per - 1)) == 0) red[wave * 64 + base + lane / per] = (double)v[0];
}

// Periodic index for x in [-L, 2L) (every halo offset here is <= 4 < L
// once L >= 8); tiny lattices take the general loop.
__device__ __forceinline__ int wrap1(int x, int L, bool tiny) {
  if (tiny) return wrap(x, L);
  x += x < 0 ? L : 0;
  x -= x >= L ? L : 0;
  return x;
}

// Register type of a staged element: sub-dword values are held one per VGPR
// (packing bytes with v_perm would make every load wait for the previous one).
template <typename T>
using StageReg = typename std::conditional<(sizeof(T) < 4), int, T>::type;

// Copy an h x w window of a periodic L x L plane (origin y0, x0; may wrap)
// into LDS, flattened over all threads (tiles of run-time width).  Every
// global load of the thread is issued before the first LDS store: one memory
// round trip (J >= h*w/kBlock; host-checked).  dbit (S windows): also the
// defector-bit plane (bit0 of each byte) at the same pitch.
template <int J, typename T>
__device__ __forceinline__ void stage_region(T* dst, int pitch, const T* src, int h, int w, int y0, int x0,
                                             int L, bool tiny, uint8_t* dbit = nullptr) {
  const int total = h * w;
  const int tid = threadIdx.x;
  const int dr = kBlock / w, dc = kBlock - (kBlock / w) * w;
  int r = tid / w, c = tid - (tid / w) * w;
  StageReg<T> buf[J];
  int di[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    di[j] = r * pitch + c;
    // unconditional load (tail rows clamped into the window): conditional loads
    // make the compiler wait on each one before the next is issued
    buf[j] = *at(src, (uint32_t)(wrap1(y0 + min(r, h - 1), L, tiny) * L + wrap1(x0 + c, L, tiny)));
    r += dr;
    c += dc;
    if (c >= w) {
      c -= w;
      ++r;
    }
  }
#pragma unroll
  for (int j = 0; j < J; ++j)
    if (tid + j * kBlock < total) {
      dst[di[j]] = (T)buf[j];
      if constexpr (sizeof(T) == 1) {
        if (dbit) dbit[di[j]] = (uint8_t)(buf[j] & 1);
      }
    }
}

// Row-per-wave window for a compile-time width W <= 64 (TWC kernels, L >= 2W):
// wave w holds rows w, w+4, ...; the row index and its wrap are wave-uniform
// (scalar ALU), the column wrap is computed once per lane.  load() issues the
// window's loads into registers, store() (later, after other loads were
// issued) writes them to LDS -- for S windows also the defector-bit plane.
template <int J, int W, typename T>
struct RowWindow {
  StageReg<T> buf[J];
  template <bool SC1 = false>
  __device__ __forceinline__ void load(const T* src, int h, int y0, int x0, int L, int tid) {
    static_assert(W <= 64, "one row per wave instruction");
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int gx = x0 + (lane < W ? lane : W - 1);
    gx += gx < 0 ? L : 0;
    gx -= gx >= L ? L : 0;
#pragma unroll
    for (int j = 0; j < J; ++j) {  // unconditional loads (rows clamped)
      const int row = min(wave + j * kWaves, h - 1);
      int gy = y0 + row;
      gy += gy < 0 ? L : 0;
      gy -= gy >= L ? L : 0;
      buf[j] = hload<SC1>(at(src, (uint32_t)(gy * L + gx)));
    }
  }
  template <int PITCH>
  __device__ __forceinline__ void store(T* dst, int h, uint8_t* dbit, int tid) {
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool in_row = lane < W;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int row = wave + j * kWaves;
      if (in_row && row < h) {
        dst[row * PITCH + lane] = (T)buf[j];
        if constexpr (sizeof(T) == 1) {
          if (dbit) dbit[row * PITCH + lane] = (uint8_t)(buf[j] & 1);
        }
      }
    }
  }
};

// x mod L for x in [-L, 2L) in four unsigned ops: min(x, x + L) takes x + L exactly when
// x < 0 (x reads as a huge unsigned), min(y, y - L) takes y - L exactly when y >= L.
__device__ __forceinline__ uint32_t wrap_once(int x, int L) {
  const uint32_t y = min((uint32_t)x, (uint32_t)x + (uint32_t)L);
  return min(y, y - (uint32_t)L);
}

// Window of h rows staged as aligned dwords (TWC kernels, L % 4 == 0, tile
// columns multiples of 4): xb = the window's first global column rounded down
// to a multiple of 4 (may be negative: periodic), DW dwords per row.  Thread t <
// RPP*DW holds column t % DW of rows t / DW + j*RPP (RPP = kBlock / DW rows per
// pass; J passes cover h, host-checked via TH <= 25), so the column, its wrap and
// the first row are computed once and each pass adds a constant row (and a
// constant LDS offset); rows and columns are wrapped by wrap_once.  A 46-byte row
// costs 12-13 lanes instead of 46 byte loads, one VGPR per J.
template <int J, int DW>
struct DwordWindow {
  static constexpr int RPP = kBlock / DW;
  uint32_t buf[J];
  template <bool SC1 = false>
  __device__ __forceinline__ void load(const void* plane, int h, int y0, int xb, int L, int tid) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(plane);
    const int Ld = L >> 2;
    const int r0 = tid / DW, col = tid - (tid / DW) * DW;  // idle threads (r0 >= RPP) load clamped rows
    const uint32_t gx = wrap_once((xb >> 2) + col, Ld);
#pragma unroll
    for (int j = 0; j < J; ++j) {  // unconditional loads (rows clamped)
      const uint32_t gy = wrap_once(y0 + min(r0 + j * RPP, h - 1), L);
      buf[j] = hload<SC1>(at(src, __umul24(gy, (uint32_t)Ld) + gx));  // gy, Ld < 2^24
    }
  }
  // dst (pitch bytes, a multiple of 4): the window's dwords; dbit: bit0 of each byte.
  __device__ __forceinline__ void store(uint8_t* dst, int pitch, int h, uint8_t* dbit, int tid) {
    const int r0 = tid / DW, col = tid - (tid / DW) * DW;
    const int o0 = r0 * pitch + col * 4;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      if (r0 < RPP && r0 + j * RPP < h) {
        const int o = o0 + j * RPP * pitch;
        *reinterpret_cast<uint32_t*>(dst + o) = buf[j];
        if (dbit) *reinterpret_cast<uint32_t*>(dbit + o) = buf[j] & 0x01010101u;
      }
    }
  }
};

// Plus-shaped defector counts over the region + 1 ring, x8 (byte offsets into
// a payoff table indexed by defector count): pc[(y)*64 + x] for region cell
// (y - 1, x - 1) = defector bits of S-window cells (y+1, x+1) and its four
// neighbours.  One wave row per region row; lanes past the row width compute
// unused cells (the D plane carries read slack).
__device__ __forceinline__ void build_plus_counts(uint8_t* pc, const uint8_t* d, int sw, int rows, int tid) {
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int y = wave; y < rows; y += kWaves) {
    const uint8_t* p = d + y * sw + lane;
    const int cnt = p[1] + p[sw] + p[sw + 1] + p[sw + 2] + p[2 * sw + 1];
    pc[y * kPcPitch + lane] = (uint8_t)(cnt << 3);
  }
}

// The same plane for compile-time-width tiles, four cells per lane: the defector plane
// (window column j at physical column j + soff, soff <= 1, rows dword-aligned) is read
// as aligned dwords and the five neighbour bytes of four consecutive cells are funnel
// shifts of two of them (v_alignbit).  Each byte sum is <= 5 and x8 <= 40, so no byte
// carries into the next; bytes past the window (uninitialised) feed only higher, unused
// bytes.  DWPR = dwords per plane row (>= the region width + 2, / 4).
template <int DWPR>
__device__ __forceinline__ void build_plus_counts_dw(uint8_t* pc, const uint8_t* dplane, int sw, int rows,
                                                     int soff, int tid) {
  const uint32_t s0 = 8u * soff, s1 = s0 + 8u, s2 = s0 + 16u;
  const int swd = sw >> 2;
  for (int task = tid; task < rows * DWPR; task += kBlock) {
    const int y = task / DWPR, xd = task - (task / DWPR) * DWPR;
    const uint32_t* r0 = reinterpret_cast<const uint32_t*>(dplane) + y * swd + xd;
    const uint32_t a0 = r0[0], a1 = r0[1];                    // row y    (the cell above)
    const uint32_t b0 = r0[swd], b1 = r0[swd + 1];            // row y+1  (left, centre, right)
    const uint32_t c0 = r0[2 * swd], c1 = r0[2 * swd + 1];    // row y+2  (the cell below)
    const uint32_t cnt = __builtin_amdgcn_alignbit(a1, a0, s1) + __builtin_amdgcn_alignbit(b1, b0, s0) +
                         __builtin_amdgcn_alignbit(b1, b0, s1) + __builtin_amdgcn_alignbit(b1, b0, s2) +
                         __builtin_amdgcn_alignbit(c1, c0, s1);
    *reinterpret_cast<uint32_t*>(pc + y * kPcPitch + xd * 4) = cnt << 3;
  }
}

// The plus-count plane of the PREVIOUS strategies S_{t-1}: bit 3 of every S_t byte (the
// strategy its owner started iteration t-1 with), from the staged S window itself -- the
// payoffs of iteration t-1 recomputed for the pending NI record (recomputed_record).
__device__ __forceinline__ void build_plus_counts_prev(uint8_t* pc, const uint8_t* s, int sw, int rows, int tid) {
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int y = wave; y < rows; y += kWaves) {
    const uint8_t* p = s + y * sw + lane;
    const int cnt = ((p[1] >> 3) & 1) + ((p[sw] >> 3) & 1) + ((p[sw + 1] >> 3) & 1) + ((p[sw + 2] >> 3) & 1) +
                    ((p[2 * sw + 1] >> 3) & 1);
    pc[y * kPcPitch + lane] = (uint8_t)(cnt << 3);
  }
}
template <int DWPR>
__device__ __forceinline__ void build_plus_counts_prev_dw(uint8_t* pc, const uint8_t* splane, int sw, int rows,
                                                          int soff, int tid) {
  const uint32_t s0 = 8u * soff, s1 = s0 + 8u, s2 = s0 + 16u;
  const int swd = sw >> 2;
  constexpr uint32_t kB3 = 0x01010101u;
  for (int task = tid; task < rows * DWPR; task += kBlock) {
    const int y = task / DWPR, xd = task - (task / DWPR) * DWPR;
    const uint32_t* r0 = reinterpret_cast<const uint32_t*>(splane) + y * swd + xd;
    const uint32_t a0 = (r0[0] >> 3) & kB3, a1 = (r0[1] >> 3) & kB3;
    const uint32_t b0 = (r0[swd] >> 3) & kB3, b1 = (r0[swd + 1] >> 3) & kB3;
    const uint32_t c0 = (r0[2 * swd] >> 3) & kB3, c1 = (r0[2 * swd + 1] >> 3) & kB3;
    const uint32_t cnt = __builtin_amdgcn_alignbit(a1, a0, s1) + __builtin_amdgcn_alignbit(b1, b0, s0) +
                         __builtin_amdgcn_alignbit(b1, b0, s1) + __builtin_amdgcn_alignbit(b1, b0, s2) +
                         __builtin_amdgcn_alignbit(c1, c0, s1);
    *reinterpret_cast<uint32_t*>(pc + y * kPcPitch + xd * 4) = cnt << 3;
  }
}

// Payoff of the region cell (ry, rx) (spgg.py:230-259, 373-377): the five
// group defector counts are plus counts at the cell and its four axial
// neighbours, each a byte offset into tb = the table of the cell's own
// strategy indexed by defector count; summed in the reference's group order,
// normalised.
#define T_AT(t, o) (*reinterpret_cast<const double*>((t) + (o)))
__device__ __forceinline__ double payoff_pc(const uint8_t* pc, int ry, int rx, const double* tb, double norm_min,
                                            double norm_den, double norm_rcp) {
  const uint8_t* p = pc + ry * kPcPitch + rx + 1;  // plus count of N0[i-1, j]
  const char* t = reinterpret_cast<const char*>(tb);
  const uint32_t x0 = p[kPcPitch], x1 = p[0], x2 = p[2 * kPcPitch], x3 = p[kPcPitch - 1], x4 = p[kPcPitch + 1];
  double tot = T_AT(t, x0);                   // group (0,0)  -> N0[i,j]
  tot = tot + T_AT(t, x1);                     // group (1,0)  -> N0[i-1,j]
  tot = tot + T_AT(t, x2);                     // group (-1,0) -> N0[i+1,j]
  tot = tot + T_AT(t, x3);                     // group (1,1)  -> N0[i,j-1]
  tot = tot + T_AT(t, x4);                     // group (-1,1) -> N0[i,j+1]
  return div_uniform(tot - norm_min, norm_den, norm_rcp);  // (tot - (r-5)) / (4r - (r-5))
}

#undef T_AT

// 1/x to full f64 precision for DIAGNOSTIC quotients only (history values,
// tolerance 1e-5): hardware estimate + two Newton steps, no IEEE division.
__device__ __forceinline__ double rcp_diag(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = __builtin_fma(r, __builtin_fma(-x, r, 1.0), r);
  r = __builtin_fma(r, __builtin_fma(-x, r, 1.0), r);
  return r;
}

// Eight signed bytes packed little-endian into a 64-bit immediate.
constexpr uint64_t stat_bytes(int a, int b, int c, int d, int e, int f, int g, int h) {
  return (uint64_t)(uint8_t)a | (uint64_t)(uint8_t)b << 8 | (uint64_t)(uint8_t)c << 16 | (uint64_t)(uint8_t)d << 24 |
         (uint64_t)(uint8_t)e << 32 | (uint64_t)(uint8_t)f << 40 | (uint64_t)(uint8_t)g << 48 |
         (uint64_t)(uint8_t)h << 56;
}

// History counters as 16-bit fields f = 0..10, two per dword (word f>>1,
// half f&1; a workgroup counts at most 1024 agents, so fields never carry):
//   SW_CD, SW_DC, NCOOP, NMD_POS, NMD_POS2, GC0, GC1, ..., GC5.
// Per thread the group-composition counts GC0..5 are nibbles of one word
// (<= APT agents each) until they are spread into the fields.

// Q table helpers.  QB = 1 for Double Q-learning (second table qb), else the
// qb arrays are dead and the compiler drops them.
enum { ALG_Q = SPGG_ALG_QLEARNING, ALG_SARSA = SPGG_ALG_SARSA, ALG_ES = SPGG_ALG_EXPECTED_SARSA,
       ALG_DQ = SPGG_ALG_DOUBLE_Q };

// argmax over the two actions of a Q row, ties -> action 0 (np.argmax, algorithms.py:106-107)
__device__ __forceinline__ int greedy2(double v0, double v1) { return v0 >= v1 ? 0 : 1; }

// Double-Q's combined table entry (q1 + q2) / 2 (algorithms.py:262-266); the
// halving is exact, so * 0.5 is the same double.
__device__ __forceinline__ double mean2(double x, double y) { return (x + y) * 0.5; }

// E[Q(s', .)] under the eps-greedy policy: probabilities eps/2 and
// (1 - eps) + eps/2 on the greedy action, summed p0*q0 + p1*q1
// (algorithms.py:205-222, spgg.py:455-462).
__device__ __forceinline__ double expected_q(double v0, double v1, double eps) {
  const double po = eps * 0.5;            // eps / num_actions
  const double pgr = (1.0 - eps) + po;    // (1 - eps) + eps / num_actions
  const int g = greedy2(v0, v1);
  return (g == 0 ? pgr : po) * v0 + (g == 1 ? pgr : po) * v1;
}

// Draw pair k of agent g at iteration t: explore flag (rand < thr) and the
// randint bit.  Philox: the agent's half of block (agent pair, t + k*2^26) under the replica key;
// device MT19937 / inject: planes 2k, 2k+1 of the draw record.
// Bit g of plane p in this iteration's draw record of replica `rep` (words of 32 agents,
// the planes of one word interleaved: spgg_abi.h, spgg_buffers.draws).
__device__ __forceinline__ int draw_bit(const TileArgs& a, int rep, int g, int p) {
  const uint32_t w = *at(a.draws, (uint32_t)(rep * a.draw_words + (g >> 5) * a.planes + p));
  return (int)((w >> (g & 31)) & 1u);
}

template <int RNG>
__device__ __forceinline__ void draw_pair(const TileArgs& a, int rep, int g, int t, uint32_t key, uint64_t thr,
                                          int k, int* ex, int* rbt) {
  if constexpr (RNG == SPGG_RNG_PHILOX) {
#if SPGG_ABLATE & 1
    *ex = ((g * 2654435761u + t + k) >> 7) % 50 == 0; *rbt = (g ^ t ^ k) & 1;
#else
    philox_draw(g, t + (k << 26), key, thr, ex, rbt);
#endif
  } else {
    *ex = draw_bit(a, rep, g, 2 * k);
    *rbt = draw_bit(a, rep, g, 2 * k + 1);
  }
}

// Draw pair 0 of region cell (ry, rx) from the staged bits (spgg_step_kernel, DSTAGE).
__device__ __forceinline__ void staged_draw(const uint2* sDP, int ry, int rx, int* ex, int* rbt) {
  const uint2 w = sDP[ry * 2 + (rx >> 5)];
  *ex = (int)((w.x >> (rx & 31)) & 1u);
  *rbt = (int)((w.y >> (rx & 31)) & 1u);
}

// Double-Q's table choice (rand < 0.5, algorithms.py:302): plane 2, or Philox pair 1.
template <int RNG>
__device__ __forceinline__ int draw_table1(const TileArgs& a, int rep, int g, int t, uint32_t key) {
  if constexpr (RNG == SPGG_RNG_PHILOX) {
    int ex, rbt;
    philox_draw(g, t + (1 << 26), key, 1ull << 52, &ex, &rbt);  // rand < 0.5
    return ex;
  } else {
    return draw_bit(a, rep, g, 2);
  }
}

typedef double vd2 __attribute__((ext_vector_type(2)));

// Q in state planes (spgg_abi.h): a replica's table is [s][n][QH] -- plane s holds every
// agent's row s, (Q[s,0], Q[s,1]) (Double-Q: then q_table_2's row s).  An iteration
// changes at most the rows of its own state and of the pending NI entry (the state of
// t-1), mostly one and the same, so the other plane's lines stay clean in the caches and
// are not written back (the (L,L,2,2) layout dirtied every agent's whole 32 bytes).
// vd2 index of agent g's row s: (s * n + g) * (QH / 2).
template <int QB>
__device__ __forceinline__ void load_q(const double* Qr, uint32_t n, uint32_t agent, double (&q)[4],
                                       double (&qb)[QB ? 4 : 1]) {
  const vd2* q0 = at(reinterpret_cast<const vd2*>(Qr), agent * (QB ? 2 : 1));
  const vd2* q1 = at(reinterpret_cast<const vd2*>(Qr), (n + agent) * (QB ? 2 : 1));
#if SPGG_QNT & 1  // A/B probe: Q rows loaded non-temporally
  const vd2 q01 = __builtin_nontemporal_load(q0), q23 = __builtin_nontemporal_load(q1);
#else
  const vd2 q01 = q0[0], q23 = (SPGG_ABLATE & 4096) ? q01 : q1[0];  // 4096: one plane's reads only
#endif
  q[0] = q01.x; q[1] = q01.y; q[2] = q23.x; q[3] = q23.y;
  if constexpr (QB) {
    const vd2 b01 = q0[1], b23 = q1[1];
    qb[0] = b01.x; qb[1] = b01.y; qb[2] = b23.x; qb[3] = b23.y;
  }
}

// Store the rows of `rows` (bit s: row s changed).
template <int QB>
__device__ __forceinline__ void store_q(double* Qr, uint32_t n, uint32_t agent, const double (&q)[4],
                                        const double (&qb)[QB ? 4 : 1], uint32_t rows = 3u) {
  vd2* q0 = at(reinterpret_cast<vd2*>(Qr), agent * (QB ? 2 : 1));
  vd2* q1 = at(reinterpret_cast<vd2*>(Qr), (n + agent) * (QB ? 2 : 1));
#if SPGG_QNT & 2  // A/B probe: Q rows stored non-temporally
  if constexpr (!QB) {
    if (rows & 1u) __builtin_nontemporal_store(vd2{q[0], q[1]}, q0);
    if (rows & 2u) __builtin_nontemporal_store(vd2{q[2], q[3]}, q1);
    return;
  }
#endif
  if (rows & 1u) {
    q0[0] = vd2{q[0], q[1]};
    if constexpr (QB) q0[1] = vd2{qb[0], qb[1]};
  }
  if (rows & 2u) {
    q1[0] = vd2{q[2], q[3]};
    if constexpr (QB) q1[1] = vd2{qb[2], qb[3]};
  }
}

// Q row of state s the eps-greedy select reads (Double-Q: the mean table).
template <int QB>
__device__ __forceinline__ void select_row(const double (&q)[4], const double (&qb)[QB ? 4 : 1], int s,
                                           double* v0, double* v1) {
  if constexpr (QB) {
    const double m00 = mean2(q[0], qb[0]), m01 = mean2(q[1], qb[1]);
    const double m10 = mean2(q[2], qb[2]), m11 = mean2(q[3], qb[3]);
    *v0 = s ? m10 : m00;
    *v1 = s ? m11 : m01;
  } else {
    // the row select written out (one compare, four 32-bit selects): as C++ selects of two
    // entries of q it was folded into one load at a computed index of q, which keeps q in
    // scratch memory (and an empty asm barrier on the entries cost four 64-bit copies)
    uint32_t a0, a1, b0, b1;
    asm("v_cmp_ne_u32_e32 vcc, 0, %4\n\t"
        "v_cndmask_b32_e32 %0, %5, %6, vcc\n\t"
        "v_cndmask_b32_e32 %1, %7, %8, vcc\n\t"
        "v_cndmask_b32_e32 %2, %9, %10, vcc\n\t"
        "v_cndmask_b32_e32 %3, %11, %12, vcc"
        : "=&v"(a0), "=&v"(a1), "=&v"(b0), "=&v"(b1)
        : "v"(s), "v"(__double2loint(q[0])), "v"(__double2loint(q[2])), "v"(__double2hiint(q[0])),
          "v"(__double2hiint(q[2])), "v"(__double2loint(q[1])), "v"(__double2loint(q[3])),
          "v"(__double2hiint(q[1])), "v"(__double2hiint(q[3]))
        : "vcc");
    *v0 = __hiloint2double((int)a1, (int)a0);
    *v1 = __hiloint2double((int)b1, (int)b0);
  }
}

// Diagnostic TD on the UPDATED table (spgg.py:446-473), Double-Q: on the mean
// table, |diag_alpha*td'| with e = (s_old, a) and sn the new state.
template <typename PT>
__device__ __forceinline__ float diag_td_dq(const double (&q)[4], const double (&qb)[4], int e, int sn, double rew,
                                            const PT& pg) {
  const double m00 = mean2(q[0], qb[0]), m01 = mean2(q[1], qb[1]);
  const double m10 = mean2(q[2], qb[2]), m11 = mean2(q[3], qb[3]);
  const double m0 = sn ? m10 : m00, m1 = sn ? m11 : m01;
  const double td2 = (rew + pg.diag_gamma * max_f64(m0, m1)) - mean2(q_get(q, e), q_get(qb, e));
  return (float)fabs(pg.diag_alpha * td2);
}

// TD update of the operator for one agent (algorithms.py:112-341) and the
// diagnostic TD on the updated table (spgg.py:446-473).  Returns |diag_alpha*td'|.
// diag = false (kappa == 0: the NI percent it feeds is exactly 0) skips the
// diagnostic and returns 0.
template <int ALG, int RNG, typename PT>
__device__ __forceinline__ float td_update(const TileArgs& a, const PT& pg, int rep, int g, int t,
                                           uint32_t key, double eps, uint64_t eps53, bool diag, double rew,
                                           int so, int act, int sn, double (&q)[4],
                                           double (&qb)[ALG == ALG_DQ ? 4 : 1], double* rn0, double* rn1) {
  const double alpha = pg.alpha, gamma = pg.gamma, dgamma = pg.diag_gamma;
  const int e = so * 2 + act;
  if constexpr (ALG == ALG_DQ) {
    // scalar copies: value selects only (pointer selects into the tables
    // would keep them out of registers)
    double x[4] = {q[0], q[1], q[2], q[3]}, y[4] = {qb[0], qb[1], qb[2], qb[3]};
    const int up1 = draw_table1<RNG>(a, rep, g, t, key);
    const double qc1 = q_get(x, e), qc2 = q_get(y, e);
    const double y0 = y[0], y1 = y[1], y2 = y[2], y3 = y[3];
    const double x0 = x[0], x1 = x[1], x2 = x[2], x3 = x[3];
    const double b0 = sn ? y2 : y0, b1 = sn ? y3 : y1;  // q_table_2[s']
    const double c0 = sn ? x2 : x0, c1 = sn ? x3 : x1;  // q_table_1[s']
    const double n1 = b0 >= b1 ? b0 : b1;  // q2 at its argmax (algorithms.py:317-323)
    const double n2 = c0 >= c1 ? c0 : c1;
    const double u1 = qc1 + alpha * ((rew + gamma * n1) - qc1);
    const double u2 = qc2 + alpha * ((rew + gamma * n2) - qc2);
    const double nq1 = up1 ? u1 : qc1, nq2 = up1 ? qc2 : u2;
    q[0] = e == 0 ? nq1 : x0; q[1] = e == 1 ? nq1 : x1; q[2] = e == 2 ? nq1 : x2; q[3] = e == 3 ? nq1 : x3;
    qb[0] = e == 0 ? nq2 : y0; qb[1] = e == 1 ? nq2 : y1; qb[2] = e == 2 ? nq2 : y2; qb[3] = e == 3 ? nq2 : y3;
    *rn0 = sn ? q[2] : q[0];
    *rn1 = sn ? q[3] : q[1];
    return diag ? diag_td_dq(q, qb, e, sn, rew, pg) : 0.f;
  } else {
    // rows of the old and the new state; the updated entry is (so, act)
    const double o0 = so ? q[2] : q[0], o1 = so ? q[3] : q[1];
    const double v0 = sn ? q[2] : q[0], v1 = sn ? q[3] : q[1];
    const double qc = act ? o1 : o0;
    double target;
    if constexpr (ALG == ALG_Q) {
      target = max_f64(v0, v1);                                      // algorithms.py:124-127
    } else if constexpr (ALG == ALG_SARSA) {
      int ex, rbt;                                                   // next action, spgg.py:434
      draw_pair<RNG>(a, rep, g, t, key, eps53, 1, &ex, &rbt);
      target = (ex ? rbt : greedy2(v0, v1)) ? v1 : v0;               // algorithms.py:168-171
    } else {
      target = expected_q(v0, v1, eps);                              // algorithms.py:205-222
    }
    const double td = (rew + gamma * target) - qc;
    const double q1 = qc + alpha * td;
    // entry (so, act) <- q1: lane masks of so and act combined on the scalar unit (four
    // v_cmp of e against 0..3 would each take a VALU issue slot)
    const bool s1 = so != 0, a1 = act != 0;
    q[0] = (!s1 && !a1) ? q1 : q[0];
    q[1] = (!s1 && a1) ? q1 : q[1];
    q[2] = (s1 && !a1) ? q1 : q[2];
    q[3] = (s1 && a1) ? q1 : q[3];
    const double w0 = sn ? q[2] : q[0], w1 = sn ? q[3] : q[1];       // updated table, row s'
    *rn0 = w0;  // (also the border record's row)
    *rn1 = w1;
    if (!diag) return 0.f;
    double target2;
    if constexpr (ALG == ALG_SARSA) {
      int ex, rbt;                                                   // diagnostic select, spgg.py:452
      draw_pair<RNG>(a, rep, g, t, key, eps53, 2, &ex, &rbt);
      target2 = (ex ? rbt : greedy2(w0, w1)) ? w1 : w0;
    } else {
      target2 = ALG == ALG_ES ? expected_q(w0, w1, eps) : max_f64(w0, w1);
    }
    return (float)fabs(pg.diag_alpha * ((rew + dgamma * target2) - q1));  // Q'[s,a] = q1
  }
}

// The pending NI record of iteration t-1 RECOMPUTED in launch t (every operator but SARSA,
// whose diagnostic select draws again, spgg.py:452): instead of storing max(0, max_diff) (f64)
// and |alpha*td'| (f32) per agent in launch t-1 and loading them here (24 B per agent-step of a
// kappa != 0 replica), launch t rebuilds the rewards of iteration t-1 over its region from the
// S_t window's bit 3 (S_{t-1}: the payoffs) and bit 0 (a_{t-1}: the reputation reward), and
// from them and the Q rows it holds (the table after the TD update of t-1, before its NI term)
// the same two values, bit for bit (the same f64 operations on the same operands).
template <bool M2>
__device__ __forceinline__ double prev_max_diff(const double* rew, int ca, int w) {
  // spgg.py:486-489 restated as phase 2 computes it: max over the 4 / 12 offsets of
  // rew[nb] - rew[ca] (max is exact and order-free on non-NaN, never -0 rewards), then max(0, .)
  const double r0 = rew[ca];
  constexpr int KN = M2 ? 12 : 4;
  const int nb[12] = {ca - w, ca + w, ca - 1, ca + 1, ca - 2 * w, ca + 2 * w, ca - 2, ca + 2,
                      ca - w - 1, ca - w + 1, ca + w - 1, ca + w + 1};
  double rw[KN];
#pragma unroll
  for (int k = 0; k < KN; ++k) rw[k] = rew[nb[k]];
  // max_k RN(rw_k - r0) = RN(max_k rw_k - r0): x -> RN(x - r0) is non-decreasing and the maximum
  // attains it, so one subtraction gives phase 2's value bit for bit (phase 2 needs every
  // difference: its argmax keeps the first of equal rounded differences)
  double m = rw[0];
#pragma unroll
  for (int k = 1; k < KN; ++k) m = max_f64(m, rw[k]);
  return max_f64(m - r0, 0.0);  // max(0, md): one v_max_f64 (md is never -0)
}

// |diag_alpha * td'| of iteration t-1 (spgg.py:446-475) from the table after its TD update
// (q, qb: before the NI term), its entry e = (s_old, a), its new state sn and reward rew --
// what td_update returned in launch t-1.  eps_prev: eps of iteration t-1 (Expected SARSA).
template <int ALG, typename PT>
__device__ __forceinline__ float prev_diag_td(const double (&q)[4], const double (&qb)[ALG == ALG_DQ ? 4 : 1],
                                              int e, int sn, double rew, const PT& pg, double eps_prev) {
  if constexpr (ALG == ALG_DQ) {
    return diag_td_dq(q, qb, e, sn, rew, pg);
  } else {
    double w0, w1, o0, o1;
    select_row<0>(q, qb, sn, &w0, &w1);        // row s' of the updated table
    select_row<0>(q, qb, e >> 1, &o0, &o1);    // row s_old: Q'[s, a] = q1
    const double q1 = (e & 1) ? o1 : o0;
    const double target2 = ALG == ALG_ES ? expected_q(w0, w1, eps_prev) : max_f64(w0, w1);
    return (float)fabs(pg.diag_alpha * ((rew + pg.diag_gamma * target2) - q1));
  }
}

// ---- persistent launches: hand-offs between the workgroups of one replica ----------------
// Inside one persistent launch every byte that another workgroup reads (the S / R halo
// windows, the border records, the history record's NCOOP / lattice max) is stored
// write-through and loaded past the CU's vector L1: relaxed agent-scope atomic stores and loads,
// which gfx950 lowers to global_store / global_load ... sc1.  With each storing wave's
// vmcnt(0), one arrival per workgroup after its barrier, an sc1 poll and a workgroup barrier
// before the loads, no acquire / release fence is needed (MI355X_MICROARCH.md, inter-workgroup
// visibility: an agent-scope acquire costs ~6.5 us per phase at 4 workgroups per CU).  The
// per-launch form (SC1 = false) keeps plain accesses: a launch boundary orders them.
// (hload / hstore: the accessors above, sc1 in persistent launches)

// Sum / max of one f64 per lane over the wave, in every lane (permlane swaps + DPP, no LDS).
__device__ __forceinline__ double wave_sum(double v) {
  {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    v = __hiloint2double(h[0], l[0]) + __hiloint2double(h[1], l[1]);
  }
  {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    v = __hiloint2double(h[0], l[0]) + __hiloint2double(h[1], l[1]);
  }
  v += partner<8>(v);
  v += partner<4>(v);
  v += partner<2>(v);
  v += partner<1>(v);
  return v;
}

#ifndef SPGG_BAR_DEBUG
#define SPGG_BAR_DEBUG 0
#endif
// Bound of a persistent launch's wait for its replica's other tiles, in polls (each an sc1
// load round trip, >= ~0.5 us, plus s_sleep): >= ~1 s.  Every tile of a persistent launch is
// co-resident (the host checks the batch against the instance's occupancy), so a wait that
// runs out means a tile never arrived: the launch records SPGG_STEP_ERR_BARRIER and stops
// instead of hanging the GPU.
constexpr uint32_t kBarrierPolls = 1u << 21;

// The replica barrier between two iterations of a persistent launch: every tile of replica rep
// has finished its k-th iteration of the launch (its S / R / border-record stores and history
// atomics drained).  Returns false when this wait, or another workgroup's, ran out of its bound.
__device__ __forceinline__ bool replica_barrier(const spgg_impl::PersistArgs& pa, int rep, int tile,
                                                int tiles_per_rep, uint32_t k,
                                                unsigned long long* arrive_stamp = nullptr) {
  __shared__ int bar_ok;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores and atomics have landed
  __syncthreads();                                  // ... and every other wave's
  if (arrive_stamp && threadIdx.x == 0) *arrive_stamp = __builtin_amdgcn_s_memrealtime();  // (SPGG_STAMPS)
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x, S = pa.shards;
    uint32_t* ctr = pa.bar + (size_t)rep * S * spgg_impl::kBarWords;
    if (lane == 0)
      __hip_atomic_fetch_add(ctr + (tile % S) * spgg_impl::kBarWords, 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    // lane j < S polls shard j (the others repeat shard 0): one load instruction per poll
    const int j = lane < S ? lane : 0;
    const uint32_t want = (uint32_t)((tiles_per_rep - j + S - 1) / S) * (pa.base + k);
    bool ok = false;
    for (uint32_t poll = 0; poll < kBarrierPolls; ++poll) {
      const uint32_t have = __hip_atomic_load(ctr + j * spgg_impl::kBarWords, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t err = __hip_atomic_load(pa.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__builtin_amdgcn_readfirstlane(err) != 0) break;
      if (__all((int32_t)(have - want) >= 0)) {
        ok = true;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (!ok && lane == 0) {
      atomicOr(pa.err, (uint32_t)SPGG_STEP_ERR_BARRIER);
      __hip_atomic_fetch_or(pa.err_host, (uint32_t)SPGG_STEP_ERR_BARRIER, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
#if SPGG_BAR_DEBUG  // diagnostic build: which shard fell short
    if (!ok) {
      const uint32_t have = __hip_atomic_load(ctr + j * spgg_impl::kBarWords, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((int32_t)(have - want) < 0)
        printf("spgg barrier: rep %d tile %d k %u shard %d have %u want %u base %u\n", rep, tile, k, j, have, want,
               pa.base);
    }
#endif
    if (lane == 0) bar_ok = ok ? 1 : 0;
  }
  __syncthreads();
  return bar_ok != 0;
}

// ONE launch = iteration t of every replica (or, fin_only, the final deferred
// NI term).  TWC > 0: compile-time tile width, every tile full width (host:
// L % TWC == 0), so LDS pitches and region divisions are immediates.
//
// Buffers: S and R ping-pong by parity (neighbours read their halos while the
// owner writes the next ones); Q, max_diff and |alpha*td'| IN PLACE (an
// agent's entries are read and written only by its owner; the ring recompute
// reads the owner's border record instead), border records ping-pong.  Per
// agent-step HBM/Infinity-Cache traffic: Q 32 B read + 16 B written (the changed state
// plane's row; 32 when the NI row and the TD row differ), md 8 + 8,
// atd 4 + 4, S/R ~5 B, border records ~6 B; the working set of cfg3 (~235 MB)
// stays within the 256 MB Infinity Cache (a ping-ponged Q alone was 270 MB).
//
// Diagnostic build (-DSPGG_STAMPS=1, one stream): workgroups stamp s_memrealtime
// (100 MHz) at phase boundaries of iteration SPGG_STAMP_T into spgg_stamps
// [logical][10] (slots 8, 9: HW_ID, XCC_ID); read by spgg_stamps_read.
#ifndef SPGG_STAMPS
#define SPGG_STAMPS 0
#endif
#if SPGG_STAMPS
#ifndef SPGG_STAMP_T
#define SPGG_STAMP_T 30
#endif
// slots per workgroup: 0-7 phases, 8 HW_ID, 9 XCC_ID; persistent launches: 10 = the replica
// barrier's stores drained (arrival), 11 = its wait passed
constexpr int kStampWG = 8192, kStampSlots = 12;
__device__ unsigned long long spgg_stamps[kStampWG * kStampSlots];
#define STAMP(k)                                                                            \
  do {                                                                                      \
    if (t == SPGG_STAMP_T && tid == 0 && stamp_id < kStampWG)                               \
      spgg_stamps[stamp_id * kStampSlots + (k)] = __builtin_amdgcn_s_memrealtime();         \
  } while (0)
#else
#define STAMP(k) \
  do {           \
  } while (0)
#endif
//
// Occupancy floor (waves per SIMD): 4 (<= 128 VGPRs) where that allocates
// without spilling (first-order Philox kernels of compile-time width, the
// bench path); elsewhere the compiler's choice.  SPGG_MIN_WAVES overrides.
constexpr int min_waves(bool m2, int rng, int twc, int alg) {
#ifdef SPGG_MIN_WAVES
  return SPGG_MIN_WAVES;
#else
#ifdef SPGG_MT_MIN_WAVES
  if (!m2 && rng == SPGG_RNG_MT19937 && twc > 0 && alg != SPGG_ALG_DOUBLE_Q) return SPGG_MT_MIN_WAVES;
#endif
  return (!m2 && rng == SPGG_RNG_PHILOX && twc > 0 && alg != SPGG_ALG_DOUBLE_Q) ? 4 : 1;
#endif
}

//
// PERSIST (spgg_persist_kernel): the launch steps iterations t0 .. pa.t_end of replicas whose
// tiles are all co-resident, each thread keeping its agents' Q rows (and, where the kernel
// stores it, the pending NI record) in registers from one iteration to the next: they are
// loaded at the launch's first iteration and stored after its last (or at the absorbing
// iteration), so an iteration moves only the halo windows, border records and outputs.
// Between two iterations replica_barrier stands in for the launch boundary (the lattice max
// and NCOOP of the replica's history record, spgg.py:405,488, and the neighbours' S / R /
// border records); those hand-offs are sc1 (hload / hstore).  Every workgroup of a replica takes the
// same absorbing decision at the same iteration (NCOOP), so none waits for a stopped tile.
template <bool M2, bool AS, bool RQ, int RNG, int APT, int TWC, int ALG, bool PERSIST>
__device__ __forceinline__ void step_impl(const TileArgs& a0, const int t0, const int fin_only,
                                          const spgg_impl::PersistArgs& pa) {
  static_assert(!PERSIST || TWC > 0, "persistent launches use the compile-time-width kernels");
  using RT = RStore<RQ>;
  constexpr int HA = M2 ? 2 : 1;  // neighbour radius of the NI / action ring
  constexpr int HS = HA + 2;      // S halo: payoffs over tile + HA
  constexpr int QB = ALG == ALG_DQ ? 1 : 0;
  constexpr int QW = QB ? 8 : 4;
  constexpr int PF = spgg_impl::pf_of(ALG);
  // pending NI record recomputed from S_t's bits (prev_max_diff / prev_diag_td), not stored: in
  // the large-batch kernels (the operator's most agents per thread), where the 24 B per agent-step
  // it saves bound the launch (cfg3 65.5 -> 64.1 us/step in the driver's window, 54.2 -> 53.2
  // steady); the latency-bound small batches (two / one agent per thread) keep the stored record,
  // where the region pass's VALU sits on the critical path (cfg4 steady 12.2 -> 14.9 us/step)
  constexpr bool RECOMP = ALG != ALG_SARSA && APT == spgg_impl::apt_of(ALG) && !(PERSIST && SPGG_PERSIST_NORECOMP);
  // PERSIST: the stored pending record (md, atd) of the owned agents carried in registers from one
  // iteration to the next (timing variant SPGG_PERSIST_NORECOMP: through global memory instead)
  constexpr bool CARRY = PERSIST && !SPGG_PERSIST_NORECOMP;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  // XCD-aware placement: blocks b, b+8, b+16... share an XCD (round-robin
  // dispatch), so give them consecutive tiles of one replica (shared halos).
  const int total = a0.n_rep * a0.tiles_per_rep;
  const int per_xcd = (total + 7) / 8;
  const int logical = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  if (logical >= total) return;
  if (SPGG_ABLATE & 64) return;
  const int lrep = logical / a0.tiles_per_rep;
  const int tile = logical - lrep * a0.tiles_per_rep;
  // the XCDs take consecutive tile ranges; a stride over the replicas spreads the cheap ones
  // (kappa == 0) evenly over them (rep_stride_for)
  const int rep = a0.rep_stride > 1 ? (int)(((uint32_t)lrep * (uint32_t)a0.rep_stride) % (uint32_t)a0.n_rep) : lrep;
#if SPGG_STAMPS
  // the workgroup's stamp slot: the batch-wide replica id (stream_id) and tile, so the launches of
  // every replica group (stream) of a batch stamp disjoint slots
  const int stamp_id = (int)a0.params[rep].stream_id * a0.tiles_per_rep + tile;
#endif

  const int L = a0.L, n = a0.n;
  const bool tiny = TWC ? false : L < 8;  // TWC => L % TWC == 0
  const int tyi = tile / a0.tiles_x, txi = tile - (tile / a0.tiles_x) * a0.tiles_x;
  const int y0 = tyi * a0.TH, x0 = txi * a0.TW;
  const int th = min(a0.TH, L - y0), tw = TWC ? TWC : min(a0.TW, L - x0);
  // LDS pitches from the full tile width (constants when TWC > 0); edge tiles
  // use the top-left part of each region
  // draw bits staged through LDS (one load round trip with the windows) instead of a record
  // load per agent at the point of use (MT19937 steps 8 us slower than Philox before this)
  constexpr bool DSTAGE = RNG != SPGG_RNG_PHILOX && TWC > 0;
  const LdsLayout ly = TWC ? lds_layout(TWC, a0.TH, HS, HA, (int)sizeof(RT), true, DSTAGE)
                           : lds_layout(tw, th, HS, HA, (int)sizeof(RT));
  double* tab = reinterpret_cast<double*>(smem);
  double* red = tab + 12;
  double* sRew = reinterpret_cast<double*>(smem + ly.off_Rew);
  RT* sR = reinterpret_cast<RT*>(smem + ly.off_R);
  RT* sRn = reinterpret_cast<RT*>(smem + ly.off_Rn);
  uint8_t* sS = smem + ly.off_S;
  uint8_t* sD = smem + ly.off_D;
  uint8_t* sA = smem + ly.off_A;
  uint8_t* sPC = smem + ly.off_PC;
  // the plus-count plane of S_{t-1} (recomputed NI record) shares the ring records' space past
  // ly.bytes: it is dead before phase 1a writes the records (the host sizes the larger of the two;
  // a plane of its own took the step workgroup's LDS past the room a generator workgroup needs
  // beside five of them: cfg3 MT19937 whole run 71.4-72.2 -> 70.5-71.2 us/iter)
  uint8_t* sPP = smem + ly.bytes;
  uint32_t* sDR = reinterpret_cast<uint32_t*>(smem + ly.off_DR);  // [row][slot][plane]
  uint2* sDP = reinterpret_cast<uint2*>(smem + ly.off_DP);         // [row][half] (plane 0, plane 1)
  // this replica's arrays: scalar bases, 32-bit element offsets (at())
  const size_t rb = (size_t)rep * n;
  double* Qr = a0.Q + rb * QW;
  double* mdr = a0.md + rb;
  float* atdr = a0.atd + rb;
  const int aw = tw + 2 * HA, ah = th + 2 * HA;  // region: tile + ring

  // Owned agent u of this thread: tile-local k = tid + u*kBlock, (r, c) packed.
  // Agent slots are branch-free: a slot past the tile's last agent SHADOWS the
  // tile's first agent (same inputs, so every value it computes and stores is
  // bit-identical to the owner's); only its history contributions are masked
  // (vm = 0).  Per-slot branches cost more in exec-mask and copy instructions.
  // slot u: (r << 16) | (c << 8) | its action bits (a | s_old << 1 | dp << 2 | s_t << 3 | s' << 4, set
  // from phase 1b on); the agent index is agent_of(rc[u]) (recomputed, not held)
  // (PERSIST: q, qb, md_own, atd_own and the slots carry over from one iteration to the next)
  int rc[APT];
  unsigned vbits = 0;  // bit u: slot u holds an owned agent
  double q[APT][4];
  double qb[APT][QB ? 4 : 1];
  double md_own[APT];
  float atd_own[APT];
  const int n_own = th * tw;
  const uint32_t g00 = (uint32_t)(y0 * L + x0);
  // (row < 256, L < 2^24: a full-rate 24-bit multiply instead of the quarter-rate 32-bit one)
  auto agent_of = [&](int rcu) { return g00 + __umul24((uint32_t)(rcu >> 16), (uint32_t)L) + ((rcu >> 8) & 0xff); };
  bool stored = false;  // PERSIST: the table is in memory (absorbing iteration, or a failed wait)
  int t = t0;
  for (;; ++t) {
  // the iteration's arguments: the halves of the ping-pong buffers and the draw record of t
  TileArgs a = a0;
  if constexpr (PERSIST) {
    const int cur = (t - 1) & 1, nxt = t & 1;
    a.S_in = pa.S[cur];
    a.S_out = pa.S[nxt];
    a.R_in = pa.R[cur];
    a.R_out = pa.R[nxt];
    a.pub_in = pa.pub[cur];
    a.pub_out = pa.pub[nxt];
    if (pa.draws0) a.draws = pa.draws0 + (size_t)((t - 1) % pa.draw_slots) * pa.draw_stride;
  }
  const bool first = !PERSIST || t == t0;  // the launch's first iteration: load the carried state
  // the thread index, opaque per iteration in a persistent launch: values derived from it (window
  // and record addresses, slot tables) are recomputed each iteration instead of being hoisted out
  // of the loop and held -- or spilled -- across it (the carried Q rows need those registers)
  int tid = threadIdx.x;
  if constexpr (PERSIST) asm volatile("" : "+v"(tid));
  const uint8_t* Sin = a.S_in + rb;
  uint8_t* Sout = a.S_out + rb;
  const RT* Rin = reinterpret_cast<const RT*>(a.R_in) + rb;
  RT* Rout = reinterpret_cast<RT*>(a.R_out) + rb;
  const bool pending = t > 1;
  STAMP(0);
#if SPGG_PRIO  // A/B probe: the load phase at a raised wave priority (back to 0 after staging)
  if constexpr (!PERSIST) __builtin_amdgcn_s_setprio(SPGG_PRIO);
#endif
#if SPGG_STAMPS
  if (t == SPGG_STAMP_T && tid == 0 && stamp_id < kStampWG) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    spgg_stamps[stamp_id * kStampSlots + 8] = hw;
    spgg_stamps[stamp_id * kStampSlots + 9] = xcc;
  }
#endif

  // ---- phase 0: every vector load first, then the replica's state ---------
  // None of these loads depends on the replica's state, so they are all in
  // flight together (one memory round trip) while the scalar reads below
  // (stop flag, counters, parameters) resolve.
  if (!first) {
#pragma unroll
    for (int u = 0; u < APT; ++u) rc[u] &= ~0xff;  // the last iteration's action bits
  } else {
    const int dr = kBlock / tw, dc = kBlock - (kBlock / tw) * tw;
    int r = tid / tw, c = tid - (tid / tw) * tw;
#pragma unroll
    for (int u = 0; u < APT; ++u) {
      const int k = tid + u * kBlock;
      const bool own = k < n_own;
      // (TWC tiles: odd lanes shadow the tile's second agent, so lane pairs keep holding
      // agent pairs (2m, 2m+1) -- the Philox blocks of phase 1b are shared per lane pair)
      rc[u] = own ? (r << 16) | (c << 8) : (TWC ? (tid & 1) << 8 : 0);
      vbits |= own ? 1u << u : 0u;
      // loads unconditional (threads without a u-th agent read the tile's
      // first one and drop it; md/atd are read even at t = 1, unused there):
      // conditional loads serialise on each other
      const uint32_t g = own ? g00 + __umul24((uint32_t)r, (uint32_t)L) + (uint32_t)c : g00 + (TWC ? (tid & 1) : 0);
      if (SPGG_ABLATE & 512) {  // compute-floor probe: no per-agent loads
#pragma unroll
        for (int k = 0; k < 4; ++k) q[u][k] = (double)((g + k) & 15) * 1e-3;
        if constexpr (QB) for (int k = 0; k < 4; ++k) qb[u][QB ? k : 0] = q[u][k];
        md_own[u] = 0.0;
        atd_own[u] = 0.f;
      } else {
        load_q<QB>(Qr, (uint32_t)n, g, q[u], qb[u]);
      }
      r += dr;
      c += dc;
      if (c >= tw) {
        c -= tw;
        ++r;
      }
    }
  }
  // ring cells of this thread (k = tid + j*kBlock): agent index + border-record offset
  constexpr int RP = spgg_impl::ring_per_thread(M2);
  const int ring = aw * ah - n_own;
  int2 re[RP];
  {
    const int2* rtab = a.ring + (size_t)tile * a.ring_max;
#pragma unroll
    for (int j = 0; j < RP; ++j) re[j] = *at(rtab, (uint32_t)min(tid + j * kBlock, ring - 1));
  }
  // halo windows into registers (TWC: aligned dwords, or rows of f64 R per
  // wave; rows <= TH + 2*halo, TH <= 25 host-checked)
  constexpr int JRR = (25 + 2 * HA + kWaves - 1) / kWaves;
  constexpr int JSF = spgg_impl::js_of(M2), JRF = spgg_impl::jr_of();
  constexpr int DWS = (TWC + 2 * HS + 3 + 3) / 4, DWR = (TWC + 2 * HA + 3 + 3) / 4;
  constexpr int JSD = (25 + 2 * HS + kBlock / DWS - 1) / (kBlock / DWS);  // passes of kBlock / DW rows
  constexpr int JRD = (25 + 2 * HA + kBlock / DWR - 1) / (kBlock / DWR);
  // window column j lives at plane column j + its misalignment (views below)
  const int soffS = TWC ? ((x0 - HS) & 3) : 0, soffR = TWC && RQ ? ((x0 - HA) & 3) : 0;
  uint8_t* sSv = sS + soffS;  // S / defector planes indexed by window coordinates
  uint8_t* sDv = sD + soffS;
  RT* sRv = sR + soffR;
  DwordWindow<JSD, DWS> winS;
  DwordWindow<JRD, DWR> winRd;
  RowWindow<JRR, TWC + 2 * HA, RT> winR;
  if constexpr (TWC > 0) {
    winS.template load<PERSIST>(Sin, th + 2 * HS, y0 - HS, (x0 - HS) & ~3, L, tid);
    if constexpr (!AS) {
      if constexpr (RQ) winRd.template load<PERSIST>(Rin, ah, y0 - HA, (x0 - HA) & ~3, L, tid);
      else winR.template load<PERSIST>(Rin, ah, y0 - HA, x0 - HA, L, tid);
    }
  }

  // the pending NI record after every other load (its address waits for the replica's kappa): a
  // replica with kappa == 0 never uses it (phase 1a skips the NI term), so all its lanes read
  // the replica's first entry -- one cache line per wave instead of 12 B per agent
  if (!(SPGG_ABLATE & 512) && !RECOMP && (first || !CARRY)) {
    const bool ni_rec = __builtin_amdgcn_readfirstlane((int)(a.params[rep].kappa != 0.0)) != 0;
#pragma unroll
    for (int u = 0; u < APT; ++u) {
      const uint32_t g = ni_rec ? agent_of(rc[u]) : 0u;
      md_own[u] = (SPGG_ABLATE & 8192) ? 0.0 : *at(mdr, g);  // 8192: md traffic floor probe
      atd_own[u] = (SPGG_ABLATE & 256) ? 0.f : *at(atdr, g);  // 256: atd traffic floor probe
    }
  }
  // draw-record words of the region rows (DSTAGE): row ry, slot sl: 32-agent group
  // (gy*L + (sl < 3 ? xA : 0)) / 32 + sl % 3, planes 0 and 1 (adjacent words)
  const uint32_t xA = wrap_once(x0 - HA, L);        // the region's first column
  const int a_len = min(aw, L - (int)xA);           // region cells before the periodic wrap
  uint32_t dw0 = 0, dw1 = 0;
  if constexpr (DSTAGE) {
    const int i = min(tid, ah * kDrawSlots - 1), ry = i / kDrawSlots, sl = i - ry * kDrawSlots;
    const uint32_t gy = wrap_once(y0 - HA + ry, L);
    const uint32_t grp = min((gy * (uint32_t)L + (sl < 3 ? xA : 0u)) / 32u + (uint32_t)(sl % 3),
                             (uint32_t)(a.draw_words / a.planes - 1));
    const uint32_t wi = (uint32_t)rep * a.draw_words + grp * a.planes;
    dw0 = *at(a.draws, wi);
    dw1 = *at(a.draws, wi + 1);
  }
  // replica state (scalar loads)
  const int st = first ? a.stop_iter[rep] : 0;  // (PERSIST: stops within the launch end its loop)
  const bool dead = st != 0 && st < t;  // absorbed before t: nothing to do
  const spgg_rep_params& pg = a.params[rep];
  // the replica's parameters (per-agent fields read from LDS: through a reference into global
  // memory the compiler must assume the agents' stores alias them) and its payoff tables
  // indexed by defector count, one 8-byte word per thread (a one-lane copy took ~40 VALU
  // moves of one wave); loaded unconditionally (clamped) with the windows, stored with them
  __shared__ spgg_rep_params hps;
  static_assert(sizeof(spgg_rep_params) % 8 == 0, "spgg_rep_params: whole 8-byte words");
  constexpr int kParamWords = (int)(sizeof(spgg_rep_params) / 8);
  constexpr int kPayWord = (int)(offsetof(spgg_rep_params, pay_c) / 8);  // pay_d follows pay_c
  const uint64_t pword = *at(reinterpret_cast<const uint64_t*>(&pg),
                             (uint32_t)(tid < kParamWords ? tid
                                        : tid < kParamWords + 6 ? kPayWord + 5 - (tid - kParamWords)
                                        : kPayWord + 17 - min(tid - kParamWords, 11)));
  const spgg_rep_params& hp = hps;
  const double kappa = pg.kappa, w_p = pg.w_p, w_rep = pg.w_rep;
  // the replica's history record: slot values are sums over its stripes (max for GMAX);
  // this workgroup adds to stripe tile % stripes (bounded atomic contention per address)
  const size_t stripe_len = (size_t)a.slots * SPGG_NSTAT;
  const double* rrow = a.stats + (size_t)rep * a.stripes * stripe_len;
  double* srow = a.stats + ((size_t)rep * a.stripes + tile % a.stripes) * stripe_len;
  bool stop_now = false;
  double gmax_prev = 0.0;
  if constexpr (PERSIST) {
    // written by this launch's previous iteration (other workgroups' atomics): sc1 vector loads,
    // stripe k in lane k; NCOOP sums integers (exact in any order), the maximum is order-free
    const int lane = tid & 63, k = lane < a.stripes ? lane : 0;
    const double ncv = hload<true>(rrow + k * stripe_len + (size_t)t * SPGG_NSTAT + SPGG_ST_NCOOP);
    const double gmv = pending ? hload<true>(rrow + k * stripe_len + (size_t)(t - 1) * SPGG_NSTAT + SPGG_ST_GMAX) : 0.0;
    const double nc = uniform_f64(wave_sum(lane < a.stripes ? ncv : 0.0));
    stop_now = (nc == 0.0) || (nc == (double)n);  // spgg.py:405
    gmax_prev = uniform_f64(max_f64(wave_max(gmv), 0.0));
  } else {
    if (!fin_only) {
      double nc = 0.0;
      for (int k = 0; k < a.stripes; ++k) nc += rrow[k * stripe_len + (size_t)t * SPGG_NSTAT + SPGG_ST_NCOOP];
      stop_now = (nc == 0.0) || (nc == (double)n);  // spgg.py:405
    }
    if (pending)
      for (int k = 0; k < a.stripes; ++k)
        gmax_prev = fmax(gmax_prev, rrow[k * stripe_len + (size_t)(t - 1) * SPGG_NSTAT + SPGG_ST_GMAX]);
  }
  const bool acting = !fin_only && !stop_now;
  const double lam_den = uniform_f64(pending ? gmax_prev + pg.lambda_eps : 1.0);
  const double lam_rcp = uniform_f64(1.0 / lam_den);  // IEEE, once per workgroup
  const double eps_t = a.eps[(size_t)rep * a.slots + t];
  const double eps_prev = ALG == ALG_ES && pending ? a.eps[(size_t)rep * a.slots + t - 1] : 0.0;
  const uint64_t eps53 = uniform_u64(u53_threshold(eps_t));  // rand < eps_t as an integer compare
  // Philox key: 64-bit seed folded with the global replica id (distinct streams per replica)
  const uint32_t pkey = (uint32_t)pg.seed ^ (uint32_t)(pg.seed >> 32) * 0x85EBCA6Bu ^
                        (uint32_t)pg.stream_id * 0xC2B2AE35u;

  // windows -> LDS (waits for the loads above)
  if (tid < kParamWords) reinterpret_cast<uint64_t*>(&hps)[tid] = pword;
  else if (tid < kParamWords + 12) reinterpret_cast<uint64_t*>(tab)[tid - kParamWords] = pword;
  if constexpr (TWC > 0) {
    winS.store(sS, ly.sw, th + 2 * HS, sD, tid);
    if constexpr (!AS) {
      if constexpr (RQ) winRd.store(reinterpret_cast<uint8_t*>(sR), ly.aw, ah, nullptr, tid);
      else winR.template store<(TWC + 2 * HS + 6) / 4 * 4>(sR, ah, nullptr, tid);
    }
  } else {
    stage_region<JSF>(sS, ly.sw, Sin, th + 2 * HS, tw + 2 * HS, y0 - HS, x0 - HS, L, tiny, sD);
    if (!AS) stage_region<JRF>(sR, ly.aw, Rin, ah, aw, y0 - HA, x0 - HA, L, tiny);
  }
  if constexpr (DSTAGE) {
    if (tid < ah * kDrawSlots) {
      sDR[tid * 2] = dw0;
      sDR[tid * 2 + 1] = dw1;
    }
  }
  if (dead) return;  // workgroup-uniform; no vector load is outstanding here
  if (stop_now && tile == 0 && tid == 0) a.stop_iter[rep] = t;
  // border records of this thread's ring cells: in flight during phases 1a / 1b
  // (unconditional: every offset is valid, and a load under a branch makes the
  // compiler wait for it at the join)
  double rv[RP][PF];
  {
    const double* pin = a.pub_in + (size_t)rep * a.tiles_per_rep * PF * a.PB;
#pragma unroll
    for (int j = 0; j < RP; ++j)
#pragma unroll
      for (int f = 0; f < PF; ++f) rv[j][f] = hload<PERSIST>(at(pin, (uint32_t)(re[j].y + f * a.PB)));
  }
  __syncthreads();
  STAMP(1);
#if SPGG_PRIO
  if constexpr (!PERSIST) __builtin_amdgcn_s_setprio(0);
#endif
  if (SPGG_ABLATE & 128) {  // memory floor: write back what was read
#pragma unroll
    for (int u = 0; u < APT; ++u) {
      const int r = rc[u] >> 16, c = (rc[u] >> 8) & 0xff;
      store_q<QB>(Qr, (uint32_t)n, agent_of(rc[u]), q[u], qb[u]);
      if (!RECOMP) {
        *at(mdr, agent_of(rc[u])) = md_own[u];
        *at(atdr, agent_of(rc[u])) = atd_own[u];
      }
      *at(Sout, agent_of(rc[u])) = sSv[(r + HS) * ly.sw + (c + HS)];
      if (!AS) *at(Rout, agent_of(rc[u])) = sRv[(r + HA) * ly.aw + (c + HA)];
    }
    return;
  }
  // plus counts for the payoffs of phases 1b / 1c (their barrier: after phase 1a)
  if (!fin_only) {
    if constexpr (TWC > 0) build_plus_counts_dw<(TWC + 2 * HA + 2 + 3) / 4>(sPC, sD, ly.sw, ah + 2, soffS, tid);
    else build_plus_counts(sPC, sDv, ly.sw, ah + 2, tid);
  }
  // the rewards of iteration t-1 over the region (tile + ring), into sRew (phase 1a reads them;
  // phases 1b / 1c overwrite them with iteration t's after the barrier that ends phase 1a)
  const bool rec_prev = RECOMP && pending && kappa != 0.0;  // workgroup-uniform
  if (rec_prev) {
    if constexpr (TWC > 0) build_plus_counts_prev_dw<(TWC + 2 * HA + 2 + 3) / 4>(sPP, sS, ly.sw, ah + 2, soffS, tid);
    else build_plus_counts_prev(sPP, sSv, ly.sw, ah + 2, tid);
    __syncthreads();  // both plus-count planes
    const int dr = kBlock / aw, dc = kBlock - (kBlock / aw) * aw;
    int ry = tid / aw, rx = tid - (tid / aw) * aw;
    for (int k = tid; k < aw * ah; k += kBlock) {
      const uint8_t b = sSv[(ry + (HS - HA)) * ly.sw + (rx + (HS - HA))];
      const double P = payoff_pc(sPP, ry, rx, tab + (((b >> 3) & 1) ? 6 : 0), hp.norm_min, hp.norm_den, hp.norm_rcp);
      const double rr = (b & 1) ? 0.0 : 0.5;                    // a_{t-1} = S_t (spgg.py:424-427)
      const double wpp = w_p * P, wrr = w_rep * rr;
      sRew[ry * ly.aw + rx] = wpp + wrr;
      ry += dr;
      rx += dc;
      if (rx >= aw) {
        rx -= aw;
        ++ry;
      }
    }
    __syncthreads();  // rewards of iteration t-1
  }
  // draw bits repacked to the region (DSTAGE): word (row ry, half h) holds cells rx = 32h ..
  // 32h+31 -- bit offA + rx of the row's first three groups for rx < a_len, bit offB + rx -
  // a_len of the three from column 0 past the wrap (read in phases 1b / 1c, after the barrier)
  if constexpr (DSTAGE) {
    if (!fin_only && tid < ah * 2) {
      const int ry = tid >> 1, r0 = (tid & 1) * 32;
      const uint32_t gyL = wrap_once(y0 - HA + ry, L) * (uint32_t)L;
      const int offA = (int)((gyL + xA) & 31u), offB = (int)(gyL & 31u);
      const uint32_t* W = sDR + ry * kDrawSlots * 2;
      auto bits32 = [&](int slot0, int bitpos, int p) {  // 32 bits from bitpos of slots slot0..slot0+2
        const int w = bitpos >> 5;
        const uint32_t lo = W[(slot0 + min(w, 2)) * 2 + p], hi = W[(slot0 + min(w + 1, 2)) * 2 + p];
        return __builtin_amdgcn_alignbit(hi, lo, (uint32_t)(bitpos & 31));
      };
      uint32_t out[2] = {0u, 0u};
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        if (r0 < a_len) out[p] = bits32(0, offA + r0, p);
        if (a_len < r0 + 32) {  // cells from the wrapped part
          const int rs = max(r0, a_len), sh = rs - r0;
          const uint32_t mB = ~0u << sh;
          out[p] = (out[p] & ~mB) | ((bits32(3, offB + rs - a_len, p) << sh) & mB);
        }
      }
      sDP[ry * 2 + (r0 >> 5)] = make_uint2(out[0], out[1]);
    }
  }

  // ---- phase 1a: finalize iteration t-1 for owned agents -----------------
  // value slots (-> slot t-1): red 0-3 sum Q, 4-7 sum Q over prev C; the NI percent
  // (pct_t1) is reduced with phase 1b's values
  float pct_t1 = 0.f;
  uint32_t ni_rows = 0;  // 2 bits per slot: the Q row (state plane) the NI term of t-1 changed
  {
    double v[8];
    float pct = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = 0.0;
    uint8_t sb[APT];  // S_t bytes of the owned agents: s_t (bit 0) and the state (bit 4) go to rc
#pragma unroll
    for (int u = 0; u < APT; ++u) {
      const int r = rc[u] >> 16, c = (rc[u] >> 8) & 0xff;
      sb[u] = sSv[(r + HS) * ly.sw + (c + HS)];
      rc[u] |= (AS ? 0 : ((sb[u] >> 4) & 1) << 1) | ((sb[u] & 1) << 3);
    }
    if (pending) {
#pragma unroll
      for (int u = 0; u < APT; ++u) {
        const double vmu = (vbits >> u) & 1 ? 1.0 : 0.0;
        const uint8_t b = sb[u];
        const int e = pending_entry(b);
        // kappa == 0 (a replica-uniform skip): nu = +0, q + 0 == q (Q never holds -0.0:
        // U(-0.01,0.01) draws and TD sums of finite values give +0 for exact zeros),
        // and the NI percent is exactly 0
        if (kappa != 0.0) {
          double mdp;
          float atdv;
          if constexpr (RECOMP) {  // the record of t-1 from its rewards and the held table
            const int r = rc[u] >> 16, c = (rc[u] >> 8) & 0xff;
            const int ca = (r + HA) * ly.aw + (c + HA);
            mdp = prev_max_diff<M2>(sRew, ca, ly.aw);
            atdv = prev_diag_td<ALG>(q[u], qb[u], e, (b >> 4) & 1, sRew[ca], hp, eps_prev);
          } else {
            mdp = md_own[u];
            atdv = atd_own[u];
          }
          const double nu = pending_nu(b, mdp, kappa, lam_den, lam_rcp);
          // Q[s,a] += nu as exact masked FMAs: fma(1, nu, x) = x + nu, fma(0, nu, x) = x
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const double m = e == k ? 1.0 : 0.0;
            q[u][k] = __builtin_fma(m, nu, q[u][k]);
            if constexpr (QB) qb[u][k] = __builtin_fma(m, nu, qb[u][QB ? k : 0]);  // both tables (spgg.py:496-502)
          }
          ni_rows |= (1u << (e >> 1)) << (2 * u);
          // NI percent (spgg.py:512; x100 applied to the workgroup total), in f32:
          // a history mean (tolerance 1e-5), each term a ratio in [0, 1]
          const float anu = fabsf((float)nu);
          pct = (SPGG_ABLATE & 32768) ? 0.f : __builtin_fmaf(anu * __builtin_amdgcn_rcpf((atdv + anu) + 1e-8f), (float)vmu, pct);
        }
        const double cm = ((b >> 3) & 1) ? 0.0 : vmu;                  // prev_S of t-1 == C
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {                                 // spgg.py:562-583
          const double qv = QB ? mean2(q[u][e2], qb[u][QB ? e2 : 0]) : q[u][e2];
          v[e2] = __builtin_fma(qv, vmu, v[e2]);                        // x*0/1 exact: one rounding
          v[4 + e2] = __builtin_fma(qv, cm, v[4 + e2]);
        }
      }
    }
    wave_partials<8>(v, red, 0, tid);
    pct_t1 = pct;  // reduced with phase 1b's values
  }
  if (!acting) {  // flush launch or absorbing iteration: persist the finalized Q
#pragma unroll
    for (int u = 0; u < APT; ++u) store_q<QB>(Qr, (uint32_t)n, agent_of(rc[u]), q[u], qb[u]);
    stored = true;
  }
  // the ring cells' border records (landed during phase 1a) to LDS for phase 1c:
  // held in registers across phase 1b they cost the occupancy of a fifth wave
  double* sRec = reinterpret_cast<double*>(smem + ly.bytes);  // [ring cell][PF]
#pragma unroll
  for (int j = 0; j < RP; ++j) {
    const int k = tid + j * kBlock;
    if (k < ring) {
#pragma unroll
      for (int f = 0; f < PF; ++f) sRec[k * PF + f] = rv[j][f];
    }
  }
  STAMP(2);
  __syncthreads();  // plus counts and ring records complete

  // ---- phase 1b: iteration start + action select for owned agents --------
  // f64 value slots: 0 sum R (slot t), 1 sum reward over C actions (slot t), 2 sum
  // reputation-reward ratio over C actions (slot t), 3 NI percent (slot t-1, phase 1a).
  // The payoff sums (sum P, over C / D, sum w_P*P), sum w_rep*rr and the reward sum
  // over D are NOT accumulated per agent: spgg_history_finalize derives them from the
  // group-composition and cooperator counts (a group with d defectors pays its members
  // (5-d)*pay_c + d*pay_d in total, so sum P over the lattice is a 6-bin histogram dot
  // a table; history means, tolerance 1e-5).
  uint32_t cw0 = 0, cw1 = 0;
  // Philox bits of the owned slots, one block per lane pair and slot pair: lane pairs
  // hold agent pairs (2m, 2m+1) in every slot (TWC: even L, x0 and width), so the even
  // lane computes the blocks of slots j < APT/2, the odd lane those of j + APT/2, and
  // each hands the partner its half (one DPP swap): half the Philox work per agent
  // (the blocks of slots 2j and 2j+1 are made just before slot 2j: two bit words live, not APT)
  constexpr bool PAIRED = RNG == SPGG_RNG_PHILOX && TWC > 0 && APT % 2 == 0 && !(SPGG_ABLATE & 1);
  uint32_t pbits[APT];
  {
    double va[4] = {0.0, 0.0, 0.0, 0.0};
    RVal<RQ> rsum = 0;  // sum R_t (int8 units: an exact integer sum)
#pragma unroll
    for (int u = 0; u < APT; ++u) {
      if (fin_only) continue;
      const int r = rc[u] >> 16, c = (rc[u] >> 8) & 0xff;
      const uint32_t one = (vbits >> u) & 1;
      const double vmu = one ? 1.0 : 0.0;
      const int cs = (r + HS) * ly.sw + (c + HS);
      const int ca = (r + HA) * ly.aw + (c + HA);
      const int s_t = (rc[u] >> 3) & 1;                     // (S_t bits, recorded in phase 1a)
      const double P = payoff_pc(sPC, r + HA, c + HA, tab + (s_t ? 6 : 0), hp.norm_min, hp.norm_den,
                                 hp.norm_rcp);
      const RVal<RQ> r_t = AS ? hload<PERSIST>(at(Rin, agent_of(rc[u]))) : sRv[ca];
      if constexpr (RQ) rsum += one ? r_t : 0;             // spgg.py:394 (units)
      else rsum = __builtin_fma(r_t, vmu, rsum);
      if (!acting) continue;
      if constexpr (PAIRED) {
        if (u % 2 == 0) {  // even lane: block of slot u, odd lane: slot u+1; swap halves
          const bool odd = tid & 1;
          const uint2 w = philox_block((int)agent_of(rc[odd ? u + 1 : u]), t, pkey);
          const uint32_t keep = odd ? w.y : w.x, recv = partner<1>(odd ? w.x : w.y);
          pbits[u] = odd ? recv : keep;
          pbits[u + 1] = odd ? keep : recv;
        }
      }
      int so;                                               // spgg.py:409
      if constexpr (AS) so = s_t == 0 ? 1 : 0;
      else so = (rc[u] >> 1) & 1;                           // = the state phase 2 of t-1 derived from
                                                            // R_t (S_t bit 4; iteration 1: the prologue)
      int ex, rbt;                                          // algorithms.py:105-109
      if constexpr (PAIRED) philox_decide(pbits[u], eps53, &ex, &rbt);
      else if constexpr (DSTAGE) staged_draw(sDP, r + HA, c + HA, &ex, &rbt);
      else draw_pair<RNG>(a, rep, agent_of(rc[u]), t, pkey, eps53, 0, &ex, &rbt);
      double qs0, qs1;
      select_row<QB>(q[u], qb[u], so, &qs0, &qs1);
      const int act = ex ? rbt : greedy2(qs0, qs1);         // argmax ties -> 0
      const RVal<RQ> rn = rep_next<RQ>(r_t, act, hp);
      const double rr = act == 0 ? 0.5 : 0.0;               // spgg.py:424-427
      const double wpp = w_p * P, wrr = w_rep * rr;
      const double rew = wpp + wrr;
      sA[ca] = (uint8_t)act;
      sRn[ca] = (RT)rn;
      sRew[ca] = rew;  // (R_{t+1} is stored in phase 2: a store here would make the ring's
                       // record loads wait for it)
      rc[u] |= act | (AS ? so << 1 : 0);                    // (state and s_t bits: phase 1a)
      cw0 += (s_t == 0 && act == 1) ? one : 0u;            // C->D, spgg.py:419 (D->C is derived
                                                            // in spgg_history_finalize)
      cw1 += act == 0 ? one : 0u;
      const double am = act ? 0.0 : vmu;
      va[1] = __builtin_fma(rew, am, va[1]);                // spgg.py:542
      // reputation-reward ratio (x100 applied to the total): exactly 0 when w_rep == 0
      if (w_rep != 0.0) va[2] = __builtin_fma(fabs(wrr) * rcp_diag(fabs(rew) + 1e-9), am, va[2]);
    }
    va[0] = (double)rsum;
    va[3] = (double)pct_t1;
    // red[wave*64 + 16..19]: va[0..3] (reduced here: frees their registers for phases 1c / 2)
    if (!(SPGG_ABLATE & (8 | 65536))) wave_partials<4>(va, red, 16, tid);
  }
  STAMP(3);

  // ---- phase 1c: recompute the ring of neighbours (distance <= M) --------
  // Their Q row of state s_t (S_t bit 4) and max_diff come from the owner's
  // border record of iteration t-1; the owner applies the same NI term to
  // the same entry, so both agree bit for bit.
  if (acting && !(SPGG_ABLATE & 4)) {
#pragma unroll
    for (int j = 0; j < RP; ++j) {
      const int k = tid + j * kBlock;
      if (k >= ring) break;
      int ay, ax;
      spgg_impl::ring_cell(k, th, tw, HA, &ay, &ax);
      const int g = re[j].x;
      const int cs = (ay + (HS - HA)) * ly.sw + (ax + (HS - HA));
      const uint8_t b = sSv[cs];
      const double* rec = sRec + k * PF;
      double v0 = rec[0], v1 = rec[1], w0 = 0.0, w1 = 0.0;
      if constexpr (QB) {
        w0 = rec[QB ? 2 : 0];
        w1 = rec[QB ? 3 : 0];
      }
      if (pending && kappa != 0.0) {  // kappa == 0: nu = +0 (see phase 1a)
        const int e = pending_entry(b);
        if ((e >> 1) == ((b >> 4) & 1)) {  // the NI entry lies in the published row
          const double nu = pending_nu(b, rec[PF - 1], kappa, lam_den, lam_rcp);
          if (e & 1) v1 = v1 + nu; else v0 = v0 + nu;
          if constexpr (QB) {
            if (e & 1) w1 = w1 + nu; else w0 = w0 + nu;
          }
        }
      }
      const double P = payoff_pc(sPC, ay, ax, tab + ((b & 1) ? 6 : 0), hp.norm_min, hp.norm_den, hp.norm_rcp);
      const RVal<RQ> r_t = AS ? RVal<RQ>(0) : RVal<RQ>(sRv[ay * ly.aw + ax]);
      int ex, rbt;
      if constexpr (DSTAGE) staged_draw(sDP, ay, ax, &ex, &rbt);
      else draw_pair<RNG>(a, rep, g, t, pkey, eps53, 0, &ex, &rbt);
      const int act = ex ? rbt : (QB ? greedy2(mean2(v0, w0), mean2(v1, w1)) : greedy2(v0, v1));
      const RVal<RQ> rn = rep_next<RQ>(r_t, act, hp);
      const double rr = act == 0 ? 0.5 : 0.0;
      const int ca = ay * ly.aw + ax;
      sA[ca] = (uint8_t)act;
      sRn[ca] = (RT)rn;
      const double wpp = w_p * P, wrr = w_rep * rr;
      sRew[ca] = wpp + wrr;
    }
  }
  __syncthreads();
  STAMP(4);

  // ---- phase 2: learn for owned agents -----------------------------------
  double bmax = 0.0;
  uint32_t gcn = 0, nmd2 = 0;  // group composition nibbles GC0..5; NMD_POS2
  if (acting) {
    double* pout = a.pub_out + (size_t)(rep * a.tiles_per_rep + tile) * PF * a.PB;
    // border-record slots of this thread's agents (-1: interior or shadow slot), one 16-bit
    // field per slot from the host table of the tile's shape: ~13 VALU per agent less than
    // border_slot_or_none, and the load lands while the first agent is processed
    // (border_slot_table: the host's build_ring_table)
    const uint64_t bsw = *at(reinterpret_cast<const uint64_t*>(a.ring + (size_t)a.tiles_per_rep * a.ring_max),
                             (uint32_t)(((th != a.TH ? 2 : 0) + (tw != a.TW ? 1 : 0)) * kBlock + tid));
    // the stored diagnostic |alpha*td'| (kappa == 0: the NI percent it feeds is exactly 0), as a
    // scalar flag (an f64 compare has no scalar form and was repeated on the VALU per agent)
    const bool ni_on = __builtin_amdgcn_readfirstlane((int)(kappa != 0.0)) != 0;
    const bool diag_on = ni_on && !RECOMP;
#pragma unroll
    for (int u = 0; u < APT; ++u) {
      const int r = rc[u] >> 16, c = (rc[u] >> 8) & 0xff;
      const int ca = (r + HA) * ly.aw + (c + HA);
      const uint32_t one = (vbits >> u) & 1;
      const int act = rc[u] & 1, so = (rc[u] >> 1) & 1;
      const double rew = sRew[ca];
      int sn;                                               // spgg.py:423
      if constexpr (AS) sn = act == 0 ? 1 : 0;
      else sn = rep_state_lds<M2>(sRn, ca, ly.aw);
      double rn0, rn1;  // row s_{t+1} of the updated table (the border record's)
      const float atd = td_update<ALG, RNG>(a, hp, rep, agent_of(rc[u]), t, pkey, eps_t, eps53, diag_on, rew, so,
                                            act, sn, q[u], qb[u], &rn0, &rn1);
      if constexpr (CARRY) atd_own[u] = atd;  // (carried to the next iteration's phase 1a)
      else if (diag_on && !(SPGG_ABLATE & (256 | 2048))) *at(atdr, agent_of(rc[u])) = atd;  // read only for the NI percent (0 when kappa == 0)
      // the rows this launch changed: the TD row (so) and the NI row of t-1 (phase 1a)
      if (!PERSIST && !(SPGG_ABLATE & 2048)) {
        uint32_t rows = ((ni_rows >> (2 * u)) & 3u) | (1u << so);
#if SPGG_QSTORE == 1
        rows = 3u;
#elif SPGG_QSTORE == 2
        rows |= (uint32_t)__shfl_xor((int)rows, 1);
        rows |= (uint32_t)__shfl_xor((int)rows, 2);
        rows |= (uint32_t)__shfl_xor((int)rows, 4);
#elif SPGG_QSTORE == 3
        if constexpr (TWC > 0 && TWC % 2 == 0) rows |= partner<1>(rows);
#elif SPGG_QSTORE == 4
        if constexpr (TWC > 0 && TWC % 8 == 0) {
          rows |= partner<1>(rows);
          rows |= partner<2>(rows);
          rows |= partner<4>(rows);
        }
#endif
        store_q<QB>(Qr, (uint32_t)n, agent_of(rc[u]), q[u], qb[u], rows);
      }
      // neighbour influence, spgg.py:477-494: first argmax wins ties
      const int w = ly.aw;
      constexpr int KN = M2 ? 12 : 4;
      const int nb[12] = {ca - w, ca + w, ca - 1, ca + 1,
                          ca - 2 * w, ca + 2 * w, ca - 2, ca + 2,
                          ca - w - 1, ca - w + 1, ca + w - 1, ca + w + 1};
      // every neighbour's reward and action read up front (unconditional LDS loads, in
      // flight together): a select of a load inside the scan was compiled into a load under
      // an exec mask per neighbour, each waiting for the one before
      double rw[KN];
      int an[KN];
#pragma unroll
      for (int kk = 0; kk < KN; ++kk) {
        rw[kk] = sRew[nb[kk]];
        an[kk] = sA[nb[kk]];
      }
      double md = rw[0] - rew;
      int abest = an[0], ks = 0;      // best neighbour's action (and offset index, M=2)
#pragma unroll
      for (int kk = 1; kk < KN; ++kk) {
        const double d = rw[kk] - rew;
        const bool better = d > md;
        md = max_f64(md, d);  // = better ? d : md (equal values are equal doubles: rewards are never -0)
        abest = better ? an[kk] : abest;
        if constexpr (M2) ks = better ? kk : ks;
      }
      const int dp = abest == act ? 1 : 0;
      const double mdp = max_f64(md, 0.0);  // max(0, md), one op (md is never -0: rewards are never -0)
      bmax = max_f64(bmax, mdp);
      // max(0, max_diff) feeds only the next launch's NI term, which is +0 when kappa == 0
      // (phase 1a and the ring skip it): not stored then (-8 B/agent-step for those replicas)
      if constexpr (CARRY) md_own[u] = mdp;
      else if (ni_on && !RECOMP && !(SPGG_ABLATE & (2048 | 8192))) *at(mdr, agent_of(rc[u])) = mdp;
      hstore<PERSIST>(at(Sout, agent_of(rc[u])), (uint8_t)((rc[u] & 0xff) | (dp << 2) | (sn << 4)));
      hstore<PERSIST>(at(Rout, agent_of(rc[u])), (RT)sRn[ca]);
      const int bslot = (int)(int16_t)(uint16_t)(bsw >> (16 * u));  // (table: border_slot_table)
      if (bslot >= 0) {  // row s_{t+1} + max_diff for the neighbours' ring
        double* rec = pout + bslot;
        hstore<PERSIST>(rec, rn0);
        hstore<PERSIST>(rec + a.PB, rn1);
        if constexpr (QB) {
          hstore<PERSIST>(rec + 2 * a.PB, sn ? qb[u][QB ? 2 : 0] : qb[u][0]);
          hstore<PERSIST>(rec + 3 * a.PB, sn ? qb[u][QB ? 3 : 0] : qb[u][QB ? 1 : 0]);
        }
        if (ni_on) hstore<PERSIST>(rec + (PF - 1) * a.PB, mdp);
      }
      // group composition on S_{t+1}, spgg.py:585-592: nibble nd of gcn
      const int nd = act + an[0] + an[1] + an[2] + an[3];   // (the four axial neighbours, loaded above)
      gcn += one << (4 * nd);
      if (md > 0.0) {                                       // spgg.py:520-523
        cw1 += one << 16;
        if (M2 && ks >= 4) nmd2 += one;
      }
    }
  }
  STAMP(5);
  if (!(SPGG_ABLATE & (8 | 131072))) {  // red[wave*64 + 24..29]: counter words (fields of the layout above)
    uint32_t cw[8] = {cw0,
                      cw1,
                      nmd2 | ((gcn & 0xfu) << 16),
                      ((gcn >> 4) & 0xfu) | (((gcn >> 8) & 0xfu) << 16),
                      ((gcn >> 12) & 0xfu) | (((gcn >> 16) & 0xfu) << 16),
                      (gcn >> 20) & 0xfu,
                      0u,
                      0u};
    wave_partials<8>(cw, red, 24, tid);
  }
  {  // the tile's max(0, max_diff): wave maxima -> red[wave*64 + 12]
    const double wm = wave_max(bmax);
    if ((tid & 63) == 0) red[(tid >> 6) * 64 + 12] = wm;
  }
  if (SPGG_ABLATE & 16) {  // timing probe: no workgroup totals (barrier + epilogue); NCOOP kept constant
    if (tid == 0 && tile == 0 && acting) srow[(size_t)(t + 1) * SPGG_NSTAT] = n / 2;
    return;
  }
  __syncthreads();
  STAMP(6);

  // ---- workgroup totals -> per-iteration history record ------------------
  if ((SPGG_ABLATE & (8 | 131072)) && tid == 0 && tile == 0 && acting) srow[(size_t)(t + 1) * SPGG_NSTAT] = n / 2;
  if ((SPGG_ABLATE & 16392) == 16392 && tid == 40 && acting) {  // 8 + 16384: the lattice max kept (dynamics unchanged)
    double bm = 0.0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) bm = max_f64(bm, red[w * 64 + 12]);
    if (bm > 0.0)
      atomicMax(reinterpret_cast<unsigned long long*>(&srow[(size_t)t * SPGG_NSTAT + SPGG_ST_GMAX]),
                (unsigned long long)__double_as_longlong(bm));
  }
  if (tid < 64 && !(SPGG_ABLATE & 8)) {
    // lane -> record value: source word src of every wave's red[] (and, for derived values, its
    // "C" partner src_c); lane 40 reads the wave maxima (word 12) for the lattice-wide max
    int slot = -1, k = -1, src = 12, src_c = -1;
    bool counter = false;
    // Finalize group (slot t-1): sums over prev-D are total - prev-C.
    if (tid < 13) {
      if (pending) {
        slot = t - 1;
        if (tid < 4) { k = SPGG_ST_SUMQ + tid; src = tid; }
        else if (tid < 8) { k = SPGG_ST_SUMQ_C + tid - 4; src = tid; }
        else if (tid == 8) { k = SPGG_ST_SUM_PCT; src = 16 + 3; }
        else { k = SPGG_ST_SUMQ_D + tid - 9; src = tid - 9; src_c = tid - 5; }
      }
    } else if (tid >= 16 && tid < 16 + 14 && !fin_only) {
      const int j = tid - 16;  // 0-2 va, 3-13 counters
      // record index of value j, one byte each in two 64-bit immediates (a
      // constant-memory table would cost the epilogue a memory round trip)
      // (j = 4, cw0's high half, counts nothing: SW_DC is written by spgg_history_finalize alone)
      constexpr uint64_t km0 = stat_bytes(SPGG_ST_SUMR, SPGG_ST_SUM_REW_C, SPGG_ST_SUM_RATIO_C, SPGG_ST_SW_CD,
                                          -1, SPGG_ST_NCOOP, SPGG_ST_NMD_POS, SPGG_ST_NMD_POS2);
      constexpr uint64_t km1 = stat_bytes(SPGG_ST_GC0, SPGG_ST_GC0 + 1, SPGG_ST_GC0 + 2, SPGG_ST_GC0 + 3,
                                          SPGG_ST_GC0 + 4, SPGG_ST_GC0 + 5, -1, -1);
      k = (int)(int8_t)(uint8_t)((j < 8 ? km0 : km1) >> (8 * (j & 7)));
      counter = j >= 3;
      src = counter ? 24 + ((j - 3) >> 1) : 16 + j;
      const bool start_val = j == 0;                   // recorded on the absorbing iteration too
      if ((acting || start_val) && k >= 0) slot = (j == 5) ? t + 1 : t;
    }
    if ((SPGG_ABLATE & 131072) && tid >= 19 && tid <= 29) slot = -1;  // (counter fields)
    // every word of the four waves read at once, unconditionally: one LDS round trip (the reads
    // chained under the derived values' branches held the workgroup's last wave, and with it the
    // CU's slot for the next workgroup, ~0.9 us)
    const int sc = src_c >= 0 ? src_c : src;
    double x[kWaves], y[kWaves];
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
      x[w] = red[w * 64 + src];
      y[w] = red[w * 64 + sc];
    }
    const double rep_unit = hp.rep_unit;  // (from LDS: a global read here would wait for every store of the tile)
    if (tid == 40 && acting) {  // lattice-wide max |diff| (spgg.py:488)
      double bm = 0.0;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) bm = max_f64(bm, x[w]);
      // non-negative doubles order like their bit patterns
      if (bm > 0.0)
        atomicMax(reinterpret_cast<unsigned long long*>(&srow[(size_t)t * SPGG_NSTAT + SPGG_ST_GMAX]),
                  (unsigned long long)__double_as_longlong(bm));
    }
    if (slot >= 0) {
      const int j = tid - 16;
      double tot0 = 0.0, tot1 = 0.0;  // this slot and (for derived values) its "C" partner
#pragma unroll
      for (int w = 0; w < kWaves; ++w) {
        tot0 += x[w];
        tot1 += y[w];
      }
      double val = src_c >= 0 ? tot0 - tot1 : tot0;
      if (counter) val = (double)(((unsigned long long)tot0 >> (16 * ((j - 3) & 1))) & 0xffffu);
      if (RQ && k == SPGG_ST_SUMR) val *= rep_unit;
      if (k == SPGG_ST_SUM_PCT || k == SPGG_ST_SUM_RATIO_C) val *= 100.0;  // percent sums
      if (val != 0.0 && (!(SPGG_ABLATE & 2) || k == SPGG_ST_NCOOP))
        atomicAdd(&srow[(size_t)slot * SPGG_NSTAT + k], val);
    }
  }
  STAMP(7);
  if constexpr (!PERSIST) {
    break;
  } else {
    if (!acting || t == pa.t_end) break;  // absorbed (the table stored in phase 1a), or done
    unsigned long long* arrive = nullptr;
#if SPGG_STAMPS
    if (t == SPGG_STAMP_T && stamp_id < kStampWG) arrive = &spgg_stamps[stamp_id * kStampSlots + 10];
#endif
    if (!replica_barrier(pa, rep, tile, a0.tiles_per_rep, (uint32_t)(t - t0 + 1), arrive)) {
      stored = true;  // a tile never arrived: stop here (SPGG_STEP_ERR_BARRIER; the state is void)
      break;
    }
    STAMP(11);
#if SPGG_PERSIST_STAGGER  // timing variant: workgroups start the next iteration staggered by (blockIdx/8)%4
    for (int z = 0; z < ((blockIdx.x >> 3) & 3) * SPGG_PERSIST_STAGGER; ++z) __builtin_amdgcn_s_sleep(16);
#endif
  }
  }  // iterations
  if constexpr (PERSIST) {
    if (!stored) {  // the carried state after the launch's last iteration, as a launch leaves it
      const bool ni_rec = __builtin_amdgcn_readfirstlane((int)(a0.params[rep].kappa != 0.0)) != 0;
#pragma unroll
      for (int u = 0; u < APT; ++u) {
        store_q<QB>(Qr, (uint32_t)n, agent_of(rc[u]), q[u], qb[u]);
        if (CARRY && !RECOMP && ni_rec) {
          *at(mdr, agent_of(rc[u])) = md_own[u];
          *at(atdr, agent_of(rc[u])) = atd_own[u];
        }
      }
    }
  }
}

template <bool M2, bool AS, bool RQ, int RNG, int APT, int TWC, int ALG>
__global__ __launch_bounds__(kBlock, min_waves(M2, RNG, TWC, ALG)) void spgg_step_kernel(TileArgs a, int t,
                                                                                         int fin_only) {
  step_impl<M2, AS, RQ, RNG, APT, TWC, ALG, false>(a, t, fin_only, spgg_impl::PersistArgs{});
}

// The persistent form: four workgroups per CU at most 128 VGPRs (cfg5's 1000 tiles of 1024
// agents must all be resident on 256 CUs).
template <bool M2, bool AS, bool RQ, int RNG, int APT, int TWC, int ALG>
__global__ __launch_bounds__(kBlock, 4) void spgg_persist_kernel(TileArgs a, int t0, spgg_impl::PersistArgs pa) {
  step_impl<M2, AS, RQ, RNG, APT, TWC, ALG, true>(a, t0, 0, pa);
}

// Prologue of iteration 1: state s_1 of every agent into S_1 bit 4 and the
// border records of the initial table (row s_1; no pending NI), so launch 1's
// ring recompute reads the same records as every later launch.
template <bool M2, bool AS, bool RQ, int ALG>
__global__ __launch_bounds__(kBlock) void spgg_publish_init_kernel(TileArgs a) {
  using RT = RStore<RQ>;
  constexpr int HA = M2 ? 2 : 1;
  constexpr int QB = ALG == ALG_DQ ? 1 : 0;
  constexpr int PF = spgg_impl::pf_of(ALG);
  const int rep = blockIdx.y;
  const int g = blockIdx.x * kBlock + threadIdx.x;
  const int L = a.L;
  const int y = g / L, x = g - (g / L) * L;
  const size_t rb = (size_t)rep * a.n;
  uint8_t* S = a.S_out;  // S_1, updated in place (bit 4; bit 0 is only read)
  // group composition of S_1 (defectors in each agent's 5-cell plus, spgg.py:585-592
  // restated on S_1) -> history slot 0, from which spgg_history_finalize derives
  // iteration 1's payoff sums (later iterations: the step kernel's counts)
  __shared__ int gc1[6];
  if (threadIdx.x < 6) gc1[threadIdx.x] = 0;
  __syncthreads();
  if (g < a.n) {
    const uint8_t* s = S + rb;
    const int d = (s[g] & 1) + (s[wrap(y - 1, L) * L + x] & 1) + (s[wrap(y + 1, L) * L + x] & 1) +
                  (s[y * L + wrap(x - 1, L)] & 1) + (s[y * L + wrap(x + 1, L)] & 1);
    atomicAdd(&gc1[d], 1);
  }
  __syncthreads();
  if (threadIdx.x < 6 && gc1[threadIdx.x] != 0)
    atomicAdd(&a.stats[(size_t)rep * a.stripes * a.slots * SPGG_NSTAT + SPGG_ST_GC0 + threadIdx.x],
              (double)gc1[threadIdx.x]);
  if (g >= a.n) return;
  int s1;
  if constexpr (AS) {
    s1 = (S[rb + g] & 1) ? 0 : 1;
  } else {  // spgg.py:296-307 over R_1, offsets in the reference's order
    const RT* R = reinterpret_cast<const RT*>(a.R_in) + rb;
    const int ym = wrap(y - 1, L), yp = wrap(y + 1, L), xm = wrap(x - 1, L), xp = wrap(x + 1, L);
    RT cell[13];
    cell[0] = R[y * L + x]; cell[1] = R[ym * L + x]; cell[2] = R[yp * L + x];
    cell[3] = R[y * L + xm]; cell[4] = R[y * L + xp];
    int nc = 5;
    if constexpr (M2) {
      const int yM = wrap(y - 2, L), yP = wrap(y + 2, L), xM = wrap(x - 2, L), xP = wrap(x + 2, L);
      cell[5] = R[yM * L + x]; cell[6] = R[yP * L + x]; cell[7] = R[y * L + xM]; cell[8] = R[y * L + xP];
      cell[9] = R[ym * L + xm]; cell[10] = R[ym * L + xp]; cell[11] = R[yp * L + xm]; cell[12] = R[yp * L + xp];
      nc = 13;
    }
    if constexpr (RQ) {
      int acc = 0;
      for (int i = 0; i < nc; ++i) acc += cell[i];
      s1 = acc > 0 ? 1 : 0;
    } else {
      double acc = 0.0;
      for (int i = 0; i < nc; ++i) acc += cell[i];
      s1 = acc >= rep_threshold(M2) ? 1 : 0;
    }
  }
  S[rb + g] = (uint8_t)((S[rb + g] & 0x0f) | (s1 << 4));
  const int ty = y / a.TH, tx = x / a.TW;
  const int r = y - ty * a.TH, c = x - tx * a.TW;
  const int th = min(a.TH, L - ty * a.TH), tw = min(a.TW, L - tx * a.TW);
  if (!spgg_impl::is_border(r, c, th, tw, HA)) return;
  constexpr int QH = QB ? 4 : 2;  // doubles per agent and state plane (load_q)
  const double* Q = a.Q + rb * 2 * QH + ((size_t)s1 * a.n + g) * QH;  // row s_1
  double* rec = a.pub_out + (size_t)(rep * a.tiles_per_rep + ty * a.tiles_x + tx) * PF * a.PB +
                spgg_impl::border_slot(r, c, th, tw, HA);
  rec[0] = Q[0];
  rec[a.PB] = Q[1];
  if constexpr (QB) {
    rec[2 * a.PB] = Q[2];
    rec[3 * a.PB] = Q[3];
  }
  rec[(PF - 1) * a.PB] = 0.0;
}

}  // namespace

namespace spgg_impl {

// The persistent instance for lc (compile-time-width tiles: the operator's maximum agents per
// thread at width 40, or two at width 20), or null.
template <bool M2, bool AS, bool RQ, int RNG, int ALG>
const void* persist_fn_t(const LaunchCfg& lc) {
  constexpr int APT = apt_of(ALG);
  if constexpr (APT > 2) {
    if (lc.apt == 2 && lc.twc == 20)
      return reinterpret_cast<const void*>(&spgg_persist_kernel<M2, AS, RQ, RNG, 2, 20, ALG>);
  }
  if (lc.apt == APT && lc.twc == 40)
    return reinterpret_cast<const void*>(&spgg_persist_kernel<M2, AS, RQ, RNG, APT, 40, ALG>);
  return nullptr;
}

template <int ALG>
const void* persist_fn(const LaunchCfg& lc) {
  if (lc.rng == SPGG_RNG_INJECT) return nullptr;  // (one iteration per call)
  const bool ph = lc.rng == SPGG_RNG_PHILOX;
#define SPGG_PF(X, Y, Z)                                                                             \
  if (lc.m2 == X && lc.as == Y && lc.rq == Z)                                                        \
    return ph ? persist_fn_t<X, Y, Z, SPGG_RNG_PHILOX, ALG>(lc) : persist_fn_t<X, Y, Z, SPGG_RNG_MT19937, ALG>(lc);
  SPGG_PF(0, 0, 0) SPGG_PF(0, 0, 1) SPGG_PF(0, 1, 0) SPGG_PF(0, 1, 1)
  SPGG_PF(1, 0, 0) SPGG_PF(1, 0, 1) SPGG_PF(1, 1, 0) SPGG_PF(1, 1, 1)
#undef SPGG_PF
  return nullptr;
}

template <int ALG>
int persist_blocks_per_cu(const LaunchCfg& lc) {
  const void* f = persist_fn<ALG>(lc);
  int nb = 0;
  if (!f || hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, kBlock, lc.lds_bytes) != hipSuccess) return 0;
  return nb;
}

template <bool M2, bool AS, bool RQ, int RNG, int ALG>
void launch_t(const LaunchCfg& lc, const TileArgs& a, int t, int fin, hipStream_t s) {
  constexpr int APT = apt_of(ALG);
  const dim3 grid(((lc.total_tiles + 7) / 8) * 8);
  if (lc.apt == 1) {  // small batch: one agent per thread (tiles of <= 256 agents, run-time width)
    hipLaunchKernelGGL((spgg_step_kernel<M2, AS, RQ, RNG, 1, 0, ALG>), grid, dim3(kBlock), lc.lds_bytes, s, a, t,
                       fin);
    return;
  }
  if constexpr (APT > 2) {
    if (lc.apt == 2) {  // two agents per thread (tiles of <= 512 agents: 20 x 25 when 20 divides L)
      if (lc.twc == 20)
        hipLaunchKernelGGL((spgg_step_kernel<M2, AS, RQ, RNG, 2, 20, ALG>), grid, dim3(kBlock), lc.lds_bytes, s, a,
                           t, fin);
      else
        hipLaunchKernelGGL((spgg_step_kernel<M2, AS, RQ, RNG, 2, 0, ALG>), grid, dim3(kBlock), lc.lds_bytes, s, a,
                           t, fin);
      return;
    }
  }
#ifndef SPGG_NO_TWC
  if (lc.twc == 40)  // the tile every L that is a multiple of 40 gets (L = 200, 1000)
    hipLaunchKernelGGL((spgg_step_kernel<M2, AS, RQ, RNG, APT, 40, ALG>), grid, dim3(kBlock), lc.lds_bytes, s, a,
                       t, fin);
  else
#endif
    hipLaunchKernelGGL((spgg_step_kernel<M2, AS, RQ, RNG, APT, 0, ALG>), grid, dim3(kBlock), lc.lds_bytes, s, a,
                       t, fin);
}

template <bool M2, bool AS, bool RQ, int ALG>
void launch_rng(const LaunchCfg& lc, const TileArgs& a, int t, int fin, hipStream_t s) {
  if (t == 0) {  // prologue of iteration 1 (border records of the initial table)
    const dim3 grid((a.n + kBlock - 1) / kBlock, a.n_rep);
    hipLaunchKernelGGL((spgg_publish_init_kernel<M2, AS, RQ, ALG>), grid, dim3(kBlock), 0, s, a);
    return;
  }
  if (lc.rng == SPGG_RNG_PHILOX) launch_t<M2, AS, RQ, SPGG_RNG_PHILOX, ALG>(lc, a, t, fin, s);
  else launch_t<M2, AS, RQ, SPGG_RNG_MT19937, ALG>(lc, a, t, fin, s);  // INJECT reads the same planes
}

template <bool M2, bool AS, int ALG>
void launch_rq(const LaunchCfg& lc, const TileArgs& a, int t, int fin, hipStream_t s) {
  if (lc.rq) launch_rng<M2, AS, true, ALG>(lc, a, t, fin, s);
  else launch_rng<M2, AS, false, ALG>(lc, a, t, fin, s);
}

template <int ALG>
void launch_alg(const LaunchCfg& lc, const TileArgs& a, int t, int fin, hipStream_t s, const PersistArgs* pa) {
  if (pa) {  // iterations t .. pa->t_end in one launch (the host checked the instance and residency)
    const void* f = persist_fn<ALG>(lc);
    if (!f) return;  // (spgg_step only asks for instances persist_blocks_per_cu found)
    TileArgs ka = a;
    int kt = t;
    PersistArgs kp = *pa;
    void* args[] = {&ka, &kt, &kp};
    (void)hipLaunchKernel(f, dim3(((lc.total_tiles + 7) / 8) * 8), dim3(kBlock), args, lc.lds_bytes, s);
    return;
  }
  if (lc.m2) {
    if (lc.as) launch_rq<true, true, ALG>(lc, a, t, fin, s);
    else launch_rq<true, false, ALG>(lc, a, t, fin, s);
  } else {
    if (lc.as) launch_rq<false, true, ALG>(lc, a, t, fin, s);
    else launch_rq<false, false, ALG>(lc, a, t, fin, s);
  }
}

// Explicit instantiation in the operator's own translation unit; elsewhere
// an extern declaration keeps the kernels from being instantiated again.
#define SPGG_LAUNCH_INST(k, name)                                                                   \
  template void launch_alg<name>(const LaunchCfg&, const TileArgs&, int, int, hipStream_t, const PersistArgs*); \
  template int persist_blocks_per_cu<name>(const LaunchCfg&);
#define SPGG_LAUNCH_EXTERN(k, name)                                                                 \
  extern template void launch_alg<name>(const LaunchCfg&, const TileArgs&, int, int, hipStream_t,   \
                                        const PersistArgs*);                                        \
  extern template int persist_blocks_per_cu<name>(const LaunchCfg&);
#if SPGG_TU_HAS_ALG(0)
#if SPGG_STAMPS
}  // namespace spgg_impl
extern "C" int spgg_stamps_read(void* dst, size_t bytes) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(spgg_stamps), bytes < sizeof(spgg_stamps) ? bytes : sizeof(spgg_stamps));
}
namespace spgg_impl {
#endif
SPGG_LAUNCH_INST(0, SPGG_ALG_QLEARNING)
#else
SPGG_LAUNCH_EXTERN(0, SPGG_ALG_QLEARNING)
#endif
#if SPGG_TU_HAS_ALG(1)
SPGG_LAUNCH_INST(1, SPGG_ALG_SARSA)
#else
SPGG_LAUNCH_EXTERN(1, SPGG_ALG_SARSA)
#endif
#if SPGG_TU_HAS_ALG(2)
SPGG_LAUNCH_INST(2, SPGG_ALG_EXPECTED_SARSA)
#else
SPGG_LAUNCH_EXTERN(2, SPGG_ALG_EXPECTED_SARSA)
#endif
#if SPGG_TU_HAS_ALG(3)
SPGG_LAUNCH_INST(3, SPGG_ALG_DOUBLE_Q)
#else
SPGG_LAUNCH_EXTERN(3, SPGG_ALG_DOUBLE_Q)
#endif

}  // namespace spgg_impl

#if SPGG_TU_HAS_HOST
namespace {

// ---------------------------------------------------------------------------
// Device MT19937, bit-identical to numpy.random.RandomState (legacy seeding,
// randomkit mt19937_gen + tempering), generating the draw records of whole
// chunks of iterations ahead of the step kernels (spgg_step runs it on its own
// stream; the draws depend on nothing but the key and the eps schedule).
//
// The raw word stream obeys x[k+624] = x[k+397] ^ twist(x[k], x[k+1]), so the 227
// words of a block [F, F+227) depend only on words >= 227 back: block-parallel.
// One workgroup per chain, no barrier after the prologue:
//   wave 0, the recurrence: the 227 positions of a block in 4 slots of lanes
//     (gen_slot_base), x[F+j] from x[F+j-227] (the lane's previous word of the slot, a
//     register) and x[F+j-624], x[F+j-623] (the LDS ring, 2-3 blocks old; read one block
//     ahead).  It publishes its completed blocks (gen_done) every kGenPub blocks; one
//     wave's LDS operations complete in order.  The ring holds kGenNB blocks at fixed positions (block b at 256*(b % kGenNB),
//     + a mirror of block 0 behind the last one), so with the block loop unrolled kGenNB
//     times every LDS address is a lane constant plus an immediate offset, and no LDS
//     operation of the recurrence sits under a branch;
//   the other kGenOut waves: temper + threshold + pack the finished words (below the
//     frontier 624 + 227*min(gen_done)): 64 draws per wave instruction, one __ballot, two
//     32-bit stores -- the draw record holds one BIT per draw (spgg_abi.h).  They publish
//     the first word they still need (gen_need), which the recurrence must not overwrite.
// Per executed iteration the reference draws rand(L,L) (2 words per double,
// algorithms.py:105) then randint(0,2,(L,L)) (1 word each, algorithms.py:108);
// SARSA twice more (spgg.py:434, 452), Double-Q then rand(L,L) < 0.5
// (algorithms.py:307).  After each iteration the key (the 624-word block holding
// the last consumed word, + pos) is saved to a snapshot ring, from which
// spgg_flush restores the key the reference would hold (spgg_mt_final_kernel).
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

using spgg_mt::mt_next;

// bit 0 of mt_temper(y) as a function of y: y0 ^ y3 ^ y14 ^ y18 ^ y22 ^ y29 (the tempering
// shifts and masks of mt_temper composed; tests/test_mt_jump_cpu.py checks it on numpy)
constexpr uint32_t kTemperBit0 = 0x20444009u;

// Draw program of one iteration, in the reference's order: plane i is rand(L,L)
// compared with a threshold (2 words per value, i even) or randint(0,2,(L,L))
// (1 word, i odd).
//   Q-learning / Expected SARSA: D(eps) I            (algorithms.py:105,108)
//   SARSA:   D(eps) I D(eps) I D(eps) I              (+ spgg.py:434, 452)
//   Double-Q: D(eps) I D(0.5)                        (+ algorithms.py:307)
__host__ __device__ inline int draw_planes(int alg) {
  return alg == SPGG_ALG_SARSA ? 6 : alg == SPGG_ALG_DOUBLE_Q ? 3 : 2;
}
// MT words one iteration consumes, and the first word of plane p within them.
__host__ __device__ inline int64_t draw_mt_words(int64_t n, int planes) { return n * (planes / 2 * 3 + (planes & 1) * 2); }
__host__ __device__ inline uint32_t plane_word0(uint32_t n, int p) { return n * (uint32_t)(p / 2 * 3 + (p & 1) * 2); }
// u32 words of one replica's draw record: 64-draw chunks (two words each) x planes.
__host__ __device__ inline int64_t draw_words_of(int n, int alg) {
  return (int64_t)((n + 63) / 64) * 2 * draw_planes(alg);
}

// One recurrence wave and three output waves per chain: the A/B variants of this layout
// (2 recurrence waves, 1-3 output waves, publication periods, wave priorities, VGPR caps,
// timing ablations) were measured in round 3 and live in profiles/r03/rejected_gen_knobs.patch.
#ifndef SPGG_GEN_OUT
#define SPGG_GEN_OUT 3
#endif
constexpr int kGenOut = SPGG_GEN_OUT;            // output waves
constexpr int kGenSPW = 4;                       // slots of the lone recurrence wave
// Blocks between two progress publications of the recurrence wave (each publication waits
// for the wave's LDS writes: one exposed LDS round trip per period).
constexpr int kGenPub = 4;

// Chunks an output wave handles per batch (one wait, one need publication, one store of the
// batch's draw words; the ring coordinates stepped, not divided, from one chunk to the next).
constexpr int kGenU = 4;
constexpr int kGenThreads = 64 * (1 + kGenOut);
constexpr int kMtBlock = 227;                    // 624 - 397: words one dependency step produces
// Ring words per block: none of padding, so a chunk's words are contiguous across a block
// boundary (and into the mirror of block 0 past the last block): one lane address per read.
constexpr int kGenPitch = kMtBlock;
// Ring blocks.  Not a lever: 8 or 12 (10 / 14 KB of LDS instead of 18) measured the same whole runs
// (profiles/r04/generator_groups.txt) -- with the generator resident, the step kernel's occupancy
// is bound by VGPRs, not LDS.
#ifndef SPGG_GEN_NB
#define SPGG_GEN_NB 16
#endif
constexpr int kGenNB = SPGG_GEN_NB;
static_assert(kGenNB == 16 || kGenNB == 8, "the block loop is unrolled kGenNB times");
static_assert(kGenNB % kGenPub == 0, "publication period divides the unrolled block loop");
// an output wave reads at most kGenU x kGenOut x 128 - 1 words past its published need (a batch);
// the frontier it is guaranteed to see lies (kGenNB - kGenPub) x 227 + 1 words past the smallest need
static_assert(kGenU * kGenOut * 128 - 1 < (kGenNB - kGenPub) * kMtBlock + 1, "output waves' progress");
constexpr int kGenRingWords = kGenPitch * kGenNB;
constexpr int kGenRing = kGenRingWords + kGenPitch;  // + a mirror of block 0 behind the last one
// Progress a failed recurrence wave publishes: every output wave's wait then ends at once.
constexpr uint32_t kGenDoneAbort = (0xffffffffu - 624u) / kMtBlock;
// Bound of every wait loop between the generator's waves (0.2-0.5 s of s_sleep): a wait that
// long means a defect.  The wave then records SPGG_GEN_ERR_SPIN in the context's error word,
// which spgg_flush / spgg_status report (SPGG_E_STATE: the draws of such a run are not the
// reference's), releases the other waves (need 0xffffffff / progress kGenDoneAbort) and
// stops, so the kernel ends instead of hanging the GPU.  (The recurrence wave stops through its
// last-block path: an early return there took the kernel from 51 to 74 VGPRs.)
constexpr uint32_t kGenSpinMax = 1u << 23;
#ifndef SPGG_GEN_SLEEP_OUT  // s_sleep argument of a polling output wave (x 64 clocks)
#define SPGG_GEN_SLEEP_OUT 1
#endif
#ifndef SPGG_GEN_SLEEP_REC  // s_sleep argument of the recurrence wave waiting for the output waves
#define SPGG_GEN_SLEEP_REC 2
#endif

// The 227 positions of a block in 4 slots of 64 lanes: slot s holds positions
// base(s) + lane for lane < len(s).  Positions 169-226 need positions 0-57 of the block two
// back (every other position only blocks three back), so slots 0 and 1 -- the same wave --
// hold both: a wave reads another wave's words only from blocks >= 2 behind, which leaves
// each wave a block of slack.  The lanes past len(s) (29 = 256 - 227 of them) DUPLICATE lane
// (lane - len(s)) of their slot -- the same position, operands and previous word, so they compute
// and write the same value to the same address -- so every LDS write is unconditional and the
// ring has no padding.
__host__ __device__ constexpr int gen_slot_base(int s) { return s == 0 ? 0 : s == 1 ? 169 : s == 2 ? 58 : 122; }
__host__ __device__ constexpr int gen_slot_len(int s) { return s == 0 ? 58 : s == 1 ? 58 : s == 2 ? 64 : 47; }
__device__ __forceinline__ int gen_position(int s, int lane) {
  return gen_slot_base(s) + (lane < gen_slot_len(s) ? lane : lane - gen_slot_len(s));
}

struct GenArgs {
  const uint32_t* key_in;  // [rep][625] chain 0's key + pos: mt_state, or the chunk's key buffer
  uint32_t* key_out;       // [rep][625] the key after the launch's last iteration (its last chain)
  const uint32_t* parts;   // chains >= 1: start windows, [rep][chain][kSplits][624] XOR parts
  const uint32_t* run_pos0;  // [rep] first word of the run's iteration 1 in its key block
  int chains, per_chain;   // chain c: iterations t0 + c*per_chain .. (+ per_chain - 1)
  uint32_t* snap;          // snapshot slot s of replica rep: snap + s*snap_stride + rep*625
  int64_t snap_stride;
  int snap_slots;
  uint32_t* draws;         // draw record of iteration t: draws + ((t-1) % draw_slots)*draw_stride
  int64_t draw_stride;
  int draw_slots;
  int draw_words;          // per replica (draw_words_of)
  const double* eps;       // [rep][eps_slots]
  int eps_slots;
  const int* stop_iter;
  uint32_t* err;           // the context's error word (SPGG_GEN_ERR_*), OR-ed on a failed wait
  int n, alg;
};

// A wait between the generator's waves ran out of its bound: recorded for the host (one lane,
// a vector global atomic).
__device__ __forceinline__ void gen_fail(const GenArgs& g) {
  if ((threadIdx.x & 63) == 0) atomicOr(g.err, (uint32_t)SPGG_GEN_ERR_SPIN);
}

// Flags shared through LDS between the generator's waves: relaxed workgroup-scope atomics
// on the __shared__ array itself (plain ds_read / ds_write; through a generic pointer they
// become flat accesses with system-scope waits).  Every lane of a wave writes its own copy
// (no branch around the store); readers read lane 0's.  A flag store is a release: it waits
// until every earlier LDS access of the wave has completed (lgkmcnt(0); issue order alone
// does not order another wave's view of two writes), and the compiler may not move an
// access across it; a reader only touches the ring after its flag read returned.
#define LDS_LD(x) __hip_atomic_load(&(x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
// after a wait on a flag: no memory access of the wave may be moved above the wait by the
// compiler (relaxed atomics do not order the plain ring accesses; the hardware does)
#define GEN_FENCE() asm volatile("" ::: "memory")
#define LDS_ST(x, v)                                                          \
  do {                                                                        \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                        \
    __hip_atomic_store(&(x), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); \
  } while (0)

// Word k of a launch (the key block = words 0..623) lives in ring block (k + 57) / 227 - 3
// (mod kGenNB), at offset (k + 57) % 227: blocks b >= 0 hold words 624 + 227 b ..
// (blocks are contiguous, so that is ring position (k - 624) mod kGenRingWords)
__device__ __forceinline__ uint32_t gen_word_pos(uint32_t k) {
  static_assert(kGenPitch == kMtBlock, "contiguous ring blocks");
  return (k + (uint32_t)(kGenRingWords - 624)) % (uint32_t)kGenRingWords;
}

// Iterations t0..t1 of every replica, from its key; writes the draw records, the key
// snapshots (slot t % snap_slots = the key after iteration t; t0 == 1 also slot 0 = the
// initial key) and the advanced key.  blockIdx.x = rep * chains + c: chain c runs
// iterations t0 + c*per_chain .. (+ per_chain - 1) from its window -- chain 0 from key_in
// (an aligned key block + pos), chain c >= 1 from the XOR of its parts: the window that
// starts at its first draw word, whose offset within the reference's 624-word key blocks
// is ph.  Word indices are relative to the chain's window (the host keeps a chain below
// 2^31 words).  skip_stopped: replicas already absorbed are left alone (their draws are
// never read).
__global__ __launch_bounds__(kGenThreads) void spgg_mt_gen_kernel(GenArgs g, int t0, int t1, int skip_stopped) {
  __shared__ uint32_t ring[kGenRing];
  __shared__ uint32_t gen_done[64];           // blocks the recurrence wave has published (per lane)
  __shared__ uint32_t gen_need[kGenOut][64];  // output wave w reads no word below this (per lane)
  __shared__ uint32_t pos_sh;
  const int rep = blockIdx.x / g.chains, ch = blockIdx.x - rep * g.chains, tid = threadIdx.x;
  bool last_chain;  // the chain whose iterations end the launch: it writes key_out
  {
    const int ct0 = t0 + ch * g.per_chain;
    if (ct0 > t1) return;
    last_chain = ct0 + g.per_chain - 1 >= t1;
    t1 = min(t1, ct0 + g.per_chain - 1);
    t0 = ct0;
  }
  if (skip_stopped && g.stop_iter[rep] != 0) return;
  const int planes = draw_planes(g.alg);
  const uint32_t W = (uint32_t)draw_mt_words(g.n, planes);
  uint32_t ph = 0;  // offset of the window's first word within a key block
  if (ch == 0) {
    const uint32_t* key = g.key_in + (size_t)rep * 625;
    for (int i = tid; i < 624; i += kGenThreads) ring[gen_word_pos(i)] = key[i];
    if (tid == 0) pos_sh = key[624];  // next word to consume (624: the block is exhausted)
    if (t0 == 1) {
      uint32_t* s0 = g.snap + (size_t)rep * 625;
      for (int i = tid; i < 625; i += kGenThreads) s0[i] = key[i];
    }
  } else {
    const uint32_t* pp = g.parts + (size_t)(rep * g.chains + ch) * spgg_mt::kSplits * 624;
    for (int i = tid; i < 624; i += kGenThreads) {
      uint32_t v = 0;
#pragma unroll
      for (int p = 0; p < spgg_mt::kSplits; ++p) v ^= pp[p * 624 + i];
      ring[gen_word_pos(i)] = v;
    }
    if (tid == 0) pos_sh = 0;
    ph = (uint32_t)(((uint64_t)g.run_pos0[rep] + (uint64_t)(t0 - 1) * W) % 624u);
  }
  if (tid < 64) gen_done[tid] = 0;
  if (tid < 64 * kGenOut) gen_need[tid >> 6][tid & 63] = 0;
  __syncthreads();
  const uint32_t pos0 = pos_sh;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  // first word of the key block holding word E - 1 (window-relative; >= 0: W >= 624 for chains)
  auto key_block = [ph](uint32_t E) { return ((E - 1 + ph) / 624) * 624 - ph; };
  // blocks of 227 words this launch generates: through the key block of its last iteration
  uint32_t nblk;
  {
    const uint32_t E_last = pos0 + (uint32_t)(t1 - t0 + 1) * W;
    const uint32_t target_last = key_block(E_last) + 624;
    nblk = target_last > 624 ? (target_last - 624 + kMtBlock - 1) / kMtBlock : 0;
  }
  if (wave == 0) {
    // ---- the recurrence: every slot of every block ------------------------------------------
    __builtin_amdgcn_s_setprio(3);  // the critical path
    uint32_t prev[kGenSPW], ca[kGenSPW], cb[kGenSPW];
    uint32_t *wp[kGenSPW], *pa[kGenSPW], *pb[kGenSPW];  // lane addresses: own word, its two operands
#pragma unroll
    for (int i = 0; i < kGenSPW; ++i) {
      const int j = gen_position(i, lane);
      wp[i] = ring + j;
      pa[i] = ring + j + 57;  // (a word past 227 is the next block's: contiguous ring)
      pb[i] = ring + j + 58;
      prev[i] = wp[i][(kGenNB - 1) * kGenPitch];  // x[397 + j]: block -1
      ca[i] = pa[i][(kGenNB - 3) * kGenPitch];    // operands of block 0: block -3
      cb[i] = pb[i][(kGenNB - 3) * kGenPitch];
    }
    uint32_t E = pos0 + W;
    uint32_t mb = key_block(E), target = mb + 624;
    uint32_t lim = 0;   // largest F whose block may be written (output waves' reads)
    int t = t0;
    uint32_t key_mb = 0, key_pos = pos0;
    uint32_t b = 0;     // blocks completed
    bool aborted = false;  // a flow-control wait ran out of its bound
    // key after iteration t (words [mb, mb+624) and pos), to the snapshot ring; then the next
    auto retire = [&]() {
      uint32_t* sn = g.snap + (size_t)(t % g.snap_slots) * g.snap_stride + (size_t)rep * 625;
#pragma unroll 1
      for (int m = 0; m < 10; ++m) {
        const uint32_t i = lane + 64 * m;
        if (i < 624) sn[i] = ring[gen_word_pos(mb + i)];
      }
      if (lane == 0) sn[624] = E - mb;
      key_mb = mb;
      key_pos = E - mb;
      ++t;
      E += W;
      mb = key_block(E);
      target = mb + 624;
    };
    // one block: b % kGenNB == U; operands ca/cb were read one block ahead
#define SPGG_GEN_BLOCK(U)                                                                                 \
  {                                                                                                       \
    if (b == nblk) goto rec_done;                                                                         \
    while (t <= t1 && 624u + kMtBlock * b >= target) retire();                                            \
    const uint32_t F = 624u + kMtBlock * b;                                                               \
    uint32_t spin = 0;                                                                                    \
    for (; F > lim && spin < kGenSpinMax; ++spin) { /* flow control: no output wave still reads the     \
                                                       positions written */                               \
      uint32_t m = 0xffffffffu;                                                                           \
      _Pragma("unroll") for (int w = 0; w < kGenOut; ++w) m = min(m, LDS_LD(gen_need[w][0]));             \
      m = __builtin_amdgcn_readfirstlane(m);                                                              \
      /* (saturating: finished output waves publish 0xffffffff) */                                       \
      lim = m > 0xffffffffu - (kGenNB - 1) * kMtBlock ? 0xffffffffu : m + (kGenNB - 1) * kMtBlock;        \
      if (F > lim) __builtin_amdgcn_s_sleep(SPGG_GEN_SLEEP_REC);                                          \
    }                                                                                                     \
    if (F > lim) { /* the bound ran out (the condition, not the counter: a last poll that succeeds    \
                      is no failure); this block is the last: rec_done publishes kGenDoneAbort */       \
      gen_fail(g);                                                                                        \
      aborted = true;                                                                                     \
      nblk = b + 1;                                                                                       \
    }                                                                                                     \
    GEN_FENCE();                                                                                          \
    uint32_t na[kGenSPW], nb[kGenSPW];                                                                    \
    _Pragma("unroll") for (int i = 0; i < kGenSPW; ++i) {                                                 \
      constexpr int rb = ((U + 1 + kGenNB - 3) % kGenNB) * kGenPitch;                                     \
      na[i] = pa[i][rb];                                                                                  \
      nb[i] = pb[i][rb];                                                                                  \
    }                                                                                                     \
    _Pragma("unroll") for (int i = 0; i < kGenSPW; ++i) {                                                 \
      const uint32_t x = mt_next(prev[i], ca[i], cb[i]);                                                  \
      prev[i] = x;                                                                                        \
      wp[i][U * kGenPitch] = x;                                                                           \
      if (U == 0) wp[i][kGenNB * kGenPitch] = x; /* mirror of block 0 */                                  \
      ca[i] = na[i];                                                                                      \
      cb[i] = nb[i];                                                                                      \
    }                                                                                                     \
    ++b;                                                                                                  \
    if ((U + 1) % kGenPub == 0) LDS_ST(gen_done[lane], b);                                                \
  }
    for (;;) {
      SPGG_GEN_BLOCK(0) SPGG_GEN_BLOCK(1) SPGG_GEN_BLOCK(2) SPGG_GEN_BLOCK(3)
      SPGG_GEN_BLOCK(4) SPGG_GEN_BLOCK(5) SPGG_GEN_BLOCK(6) SPGG_GEN_BLOCK(7)
#if SPGG_GEN_NB == 16
      SPGG_GEN_BLOCK(8) SPGG_GEN_BLOCK(9) SPGG_GEN_BLOCK(10) SPGG_GEN_BLOCK(11)
      SPGG_GEN_BLOCK(12) SPGG_GEN_BLOCK(13) SPGG_GEN_BLOCK(14) SPGG_GEN_BLOCK(15)
#endif
    }
#undef SPGG_GEN_BLOCK
  rec_done:
    LDS_ST(gen_done[lane], aborted ? kGenDoneAbort : b);  // (published every kGenPub blocks: the rest)
    GEN_FENCE();
    while (t <= t1) retire();  // (the frontier covers every remaining target)
    if (last_chain) {
      uint32_t* key = g.key_out + (size_t)rep * 625;
      for (int i = lane; i < 624; i += 64) key[i] = ring[gen_word_pos(key_mb + i)];
      if (lane == 0) key[624] = key_pos;
    }
    return;
  }
  // ---- output waves: chunks ow, ow + kGenOut, ... of every plane of every iteration --------
  // (per chunk: one ring read per lane, the temper / parity, one ballot; per batch of kGenU
  // chunks: one wait, the batch's first word published as the wave's need, one store)
  const int ow = wave - 1;
  const uint64_t thr_half = u53_threshold(0.5);
  const int nchunk = (g.n + 63) / 64;
  uint32_t kpos = pos0;
  uint32_t seen = 624;  // the frontier as last read
  // lane 2u + h of a batch's store: half h of the draw word of the batch's chunk u
  // (the record's word of chunk c, plane p, half h: 2 c planes + h planes + p, spgg_abi.h)
  const uint32_t lane_off = (uint32_t)(((lane >> 1) * kGenOut * 2 + (lane & 1)) * planes);
  // the draws of the plane's last chunk (n % 64 of them when partial)
  const uint64_t tail = (g.n & 63) ? (1ull << (g.n & 63)) - 1ull : ~0ull;
  for (int t = t0; t <= t1; ++t) {
    const uint64_t thr = u53_threshold(g.eps[(size_t)rep * g.eps_slots + t]);
    uint32_t* rec_out = g.draws + (size_t)((t - 1) % g.draw_slots) * g.draw_stride + (size_t)rep * g.draw_words;
    for (int p = 0; p < planes; ++p) {
      const bool dbl = (p & 1) == 0;
      // rand() < th: ((a>>5) * 2^26 + (b>>6)) / 2^53 < th as a 53-bit integer compare, decided
      // by a alone unless its 27 bits equal th's (p = 2^-27: b is read only then)
      const uint64_t th = (g.alg == SPGG_ALG_DOUBLE_Q && p == 2) ? thr_half : thr;
      const uint32_t th_hi = __builtin_amdgcn_readfirstlane((uint32_t)(th >> 26));
      const uint32_t th_lo = __builtin_amdgcn_readfirstlane((uint32_t)th & ((1u << 26) - 1u));
      const uint32_t base = kpos + plane_word0((uint32_t)g.n, p);
      // (the chunk loop is instantiated per plane kind: the kind's branches leave the loop)
      auto chunks = [&](auto dbl_c) -> bool {
        constexpr bool dbl = decltype(dbl_c)::value;
        constexpr uint32_t wmul = dbl ? 2u : 1u;           // words per draw
        constexpr uint32_t cstep = 64u * wmul * kGenOut;    // words from one chunk of this wave to its next
        static_assert(cstep * kGenU < (uint32_t)kGenRingWords, "a batch stays within one turn of the ring");
        const uint32_t wlane = wmul * (uint32_t)lane;
        // the current chunk's first word and its ring position, stepped per chunk: word k sits at
        // (k - 624) mod kGenRingWords (gen_word_pos; the blocks are contiguous)
        uint32_t first = base + 64u * wmul * (uint32_t)ow;
        uint32_t rpos = gen_word_pos(first);
        for (int c = ow; c < nchunk; c += kGenOut * kGenU) {
          const int nb = min(kGenU, (nchunk - 1 - c) / kGenOut + 1);  // chunks of this batch
          const int cl = c + (nb - 1) * kGenOut;
          const uint32_t last = first + cstep * (uint32_t)(nb - 1) + wmul * (uint32_t)min(64, g.n - 64 * cl) - 1u;
          LDS_ST(gen_need[ow][lane], first);
          if (seen <= last) {  // wait for the recurrence (the check of its bound only on this path)
            uint32_t spin = 0;
            for (; seen <= last && spin < kGenSpinMax; ++spin) {
              seen = 624u + kMtBlock * __builtin_amdgcn_readfirstlane(LDS_LD(gen_done[0]));
              if (seen <= last) __builtin_amdgcn_s_sleep(SPGG_GEN_SLEEP_OUT);
            }
            if (seen <= last) {  // (the condition itself: a last poll that succeeds is no failure)
              gen_fail(g);
              LDS_ST(gen_need[ow][lane], 0xffffffffu);
              return false;
            }
          }
          GEN_FENCE();
          // the batch's words first (one LDS round trip; a chunk past the batch reads a ring word
          // it drops), then per chunk: the chunk's <= 128 words are contiguous from its ring position
          // (past the last block: the mirror of block 0)
          uint32_t rp[kGenU], x[kGenU];
#pragma unroll
          for (int u = 0; u < kGenU; ++u) {
            rp[u] = u == 0 ? rpos : rp[u - 1] + cstep;
            if (u > 0) rp[u] -= rp[u] >= (uint32_t)kGenRingWords ? (uint32_t)kGenRingWords : 0u;
            x[u] = ring[rp[u] + wlane];
          }
          uint32_t val = 0;
#pragma unroll
          for (int u = 0; u < kGenU; ++u) {
            if (u < nb) {
              bool flag;
              if (dbl) {
                const uint32_t ah = mt_temper(x[u]) >> 5;
                flag = ah < th_hi;
                if (ah == th_hi) flag = (mt_temper(ring[rp[u] + wlane + 1]) >> 6) < th_lo;
              } else {  // randint(0, 2) = the tempered word's low bit = parity of raw bits 0,3,14,18,22,29
                flag = (__builtin_popcount(x[u] & kTemperBit0) & 1) != 0;
              }
              // (lanes past n read stale words: masked)
              const uint64_t bits = __builtin_amdgcn_ballot_w64(flag) & (c + u * kGenOut == nchunk - 1 ? tail : ~0ull);
              val = lane == 2 * u ? (uint32_t)bits : lane == 2 * u + 1 ? (uint32_t)(bits >> 32) : val;
            }
          }
          rpos += cstep * (uint32_t)nb;
          rpos -= rpos >= (uint32_t)kGenRingWords ? (uint32_t)kGenRingWords : 0u;
          if (lane < 2 * nb) *at(rec_out, (uint32_t)(2 * c * planes + p) + lane_off) = val;
          first += cstep * (uint32_t)nb;
        }
        return true;
      };
      if (!(dbl ? chunks(std::true_type{}) : chunks(std::false_type{}))) return;
    }
    kpos += W;
  }
  LDS_ST(gen_need[ow][lane], 0xffffffffu);  // done: never blocks the recurrence
}

// spgg_test_set_error: ORs flags into a context's generator error word, on the generator's
// stream, as a failing wait does (tests of the error path).
__global__ void spgg_set_err_kernel(uint32_t* err, uint32_t flags) {
  if (threadIdx.x == 0) atomicOr(err, flags);
}

// spgg_flush (MT19937): the key the reference holds after the run -- after the last
// iteration a replica executed (its absorbing iteration draws nothing) -- from the ring.
__global__ void spgg_mt_final_kernel(GenArgs g, int t_last) {
  const int rep = blockIdx.x;
  const int st = g.stop_iter[rep];
  const int src = st ? st - 1 : t_last;
  const uint32_t* sn = g.snap + (size_t)(src % g.snap_slots) * g.snap_stride + (size_t)rep * 625;
  uint32_t* key = g.key_out + (size_t)rep * 625;
  for (int i = threadIdx.x; i < 625; i += blockDim.x) key[i] = sn[i];
}

// History values derived from device counts (spgg_history_finalize), for iterations
// t = 1 .. last of each replica (last = its absorbing iteration, else t_last), into
// stripe 0 (the step kernel adds nothing to these slots):
//   start of t (spgg.py:383-394): SUMP, SUMP_C, SUMP_D from the group composition of S_t
//     (slot t-1; slot 0 = S_1, written by the prologue): a group centred on a cell with d
//     defectors pays its 5-d cooperators pay_c[5-d] and its d defectors pay_d[5-d], so
//     sum Praw = sum_d GC_d ((5-d) pay_c + d pay_d), over C: sum_d GC_d (5-d) pay_c, and
//     sum P = (sum Praw - n (r-5)) / (4r - (r-5)) (spgg.py:373-378);
//   step t (executed steps only, spgg.py:419-420, 425-426, 529-545): SUM_WPP = w_P sum P,
//     SUM_WRR = (C actions = NCOOP of slot t+1) * w_rep * 0.5, SUM_REW_D = SUM_WPP + SUM_WRR
//     - SUM_REW_C, SW_DC = SW_CD + NCOOP(t+1) - NCOOP(t) (cooperators gained = D->C - C->D).
// History means: the regrouped sums differ from per-agent accumulation in rounding only.
__global__ __launch_bounds__(kBlock) void spgg_history_finalize_kernel(double* stats, const int* stop_iter,
                                                                       const spgg_rep_params* params, int n,
                                                                       int slots, int stripes, int t_last) {
  const int rep = blockIdx.y;
  const int t = blockIdx.x * kBlock + threadIdx.x + 1;
  const int st = stop_iter[rep];
  const int last = st ? st : t_last, m = st ? st - 1 : t_last;
  if (t > last || t + 1 >= slots) return;
  const size_t stripe_len = (size_t)slots * SPGG_NSTAT;
  const double* rec = stats + (size_t)rep * stripes * stripe_len;
  auto total = [&](int slot, int k) {
    double v = 0.0;
    for (int sp = 0; sp < stripes; ++sp) v += rec[sp * stripe_len + (size_t)slot * SPGG_NSTAT + k];
    return v;
  };
  const spgg_rep_params& p = params[rep];
  double praw = 0.0, praw_c = 0.0;
#pragma unroll
  for (int d = 0; d <= 5; ++d) {
    const double gc = total(t - 1, SPGG_ST_GC0 + d);
    praw_c += gc * ((5 - d) * p.pay_c[5 - d]);
    praw += gc * ((5 - d) * p.pay_c[5 - d] + d * p.pay_d[5 - d]);
  }
  const double nc = total(t, SPGG_ST_NCOOP);
  const double sump = (praw - n * p.norm_min) / p.norm_den;
  const double sump_c = (praw_c - nc * p.norm_min) / p.norm_den;
  double* out = stats + (size_t)rep * stripes * stripe_len + (size_t)t * SPGG_NSTAT;
  out[SPGG_ST_SUMP] = sump;
  out[SPGG_ST_SUMP_C] = sump_c;
  out[SPGG_ST_SUMP_D] = sump - sump_c;
  if (t <= m) {
    const double nc1 = total(t + 1, SPGG_ST_NCOOP);
    const double wpp = p.w_p * sump;
    const double wrr = nc1 * (p.w_rep * 0.5);
    out[SPGG_ST_SUM_WPP] = wpp;
    out[SPGG_ST_SUM_WRR] = wrr;
    out[SPGG_ST_SUM_REW_D] = (wpp + wrr) - total(t, SPGG_ST_SUM_REW_C);
    out[SPGG_ST_SW_DC] = total(t, SPGG_ST_SW_CD) + nc1 - nc;   // exact integers
  }
}

// P of every agent from S_t (epilogue: SPGG.P / run()'s mean(P), spgg.py:378, 637).
__global__ __launch_bounds__(kBlock) void spgg_payoff_kernel(const uint8_t* S, const spgg_rep_params* params,
                                                             double* out, int L, int n) {
  __shared__ double tab[12];
  const int rep = blockIdx.y;
  if (threadIdx.x < 12)
    tab[threadIdx.x] = threadIdx.x < 6 ? params[rep].pay_c[threadIdx.x] : params[rep].pay_d[threadIdx.x - 6];
  __syncthreads();
  const int idx = blockIdx.x * kBlock + threadIdx.x;
  if (idx >= n) return;
  const uint8_t* s = S + (size_t)rep * n;
  const int i = idx / L, j = idx - (idx / L) * L;
  const int im1 = wrap(i - 1, L), ip1 = wrap(i + 1, L), im2 = wrap(i - 2, L), ip2 = wrap(i + 2, L);
  const int jm1 = wrap(j - 1, L), jp1 = wrap(j + 1, L), jm2 = wrap(j - 2, L), jp2 = wrap(j + 2, L);
#define CO(r, c) ((s[(r) * L + (c)] & 1) ? 0 : 1)
  Cells13 c;
  c.c00 = CO(i, j); c.cm0 = CO(im1, j); c.cp0 = CO(ip1, j); c.c0m = CO(i, jm1); c.c0p = CO(i, jp1);
  c.cmm = CO(im1, jm1); c.cmp = CO(im1, jp1); c.cpm = CO(ip1, jm1); c.cpp = CO(ip1, jp1);
  c.cM0 = CO(im2, j); c.cP0 = CO(ip2, j); c.c0M = CO(i, jm2); c.c0P = CO(i, jp2);
#undef CO
  out[(size_t)rep * n + idx] = payoff13(c, tab, params[rep].norm_min, params[rep].norm_den, params[rep].norm_rcp);
}

}  // namespace

// ===========================================================================
// C ABI
struct spgg_ctx {
  spgg_config cfg{};
  spgg_buffers buf{};
  bool bound = false;
  bool params_set = false;
  // MT19937 draw pipeline: the generator runs gen_chunk iterations per launch on its own
  // stream, one chunk ahead of the steps; draw records in a ring of draw_slots = 2 chunks,
  // key snapshots in a ring of snap_slots (spgg_draw_layout).  A chunk is chains x
  // per_chain iterations: chain c of replica rep is workgroup rep*chains + c, started from
  // the window its jump produced (spgg_mt.h)
  int gen_chunk = 8, draw_slots = 16, snap_slots = 25;
  int chains = 1, per_chain = 8, jump_levels = 0;  // jump_levels = log2(chains)
  uint32_t* d_parts[2] = {nullptr, nullptr};  // chain start windows of chunks q (q & 1)
  uint32_t* d_keybuf[2] = {nullptr, nullptr}; // chain 0's key of chunk q ([q & 1]; chunk 0: mt_state)
  uint32_t* d_run_pos0 = nullptr;
  uint32_t* d_polys = nullptr;                // x^(2^j per_chain W - 1) mod phi, j = 0..jump_levels
  int64_t draw_words = 0;            // u32 words of one replica's draw record
  hipStream_t gen_stream = nullptr;  // the generator's stream (library-owned unless set)
  bool own_gen_stream = false;
  hipEvent_t gen_done[2] = {nullptr, nullptr}, step_done[2] = {nullptr, nullptr}, gen_idle = nullptr;
  hipEvent_t caller_ready = nullptr;  // the caller's stream at a run's first generator chunk
  uint32_t* d_err = nullptr;         // generator error word (SPGG_GEN_ERR_*, sticky per context)
  volatile uint32_t* h_err = nullptr;  // its pinned host copy, refreshed after every chunk
  int gen_upto = 0;                  // iterations whose generation is enqueued
  std::vector<spgg_rep_params> params_host;  // the replicas' parameters as last set
  bool params_moved = false;  // a replica's parameters changed since the run's iteration 1
  spgg_rep_params* d_params = nullptr;
  int2* d_ring = nullptr;   // ring table (geometry of the tiling)
  int ring_max = 0;
  int n = 0;
  int TW = 0, TH = 0, tiles_x = 0, tiles_per_rep = 0, apt = 4, PB = 0;
  int stripes = 1;  // history-record stripes per replica
  int rep_stride = 1;  // replica order of the step launches over the XCDs (rep_stride_for)
  size_t lds_bytes = 0;
  // persistent launches (spgg_persist_kernel): decided at spgg_create from the whole batch's
  // tiles and the instance's occupancy; arrival counters [n_rep][stripes][kBarWords]
  bool persist = false;
  int persist_capacity = 0;      // workgroups the device holds at once (occupancy x CUs)
  uint32_t* d_bar = nullptr;
  uint32_t bar_base = 0;         // barrier rounds of this run's earlier persistent launches
  std::string err;
};

namespace {

// Compile-time tile width of the step kernel (0: run-time width): every tile
// full width, L >= 2 * window width (L % 4 == 0 for the aligned-dword window
// staging), window rows within the staging register budget (TH <= 25).
int twc_of(const spgg_config& cfg, int TW, int TH) {
  if (TW == 40 && cfg.L % 40 == 0 && cfg.L >= 120 && TH <= 25) return 40;
  // two agents per thread (spgg_create): 20 x 25 tiles, kernels of compile-time width 20
  if (TW == 20 && cfg.L % 20 == 0 && cfg.L >= 60 && TH <= 25 && cfg.algorithm != SPGG_ALG_DOUBLE_Q) return 20;
  return 0;
}

// spgg_last_error(NULL): the calling thread's last spgg_create failure
thread_local std::string g_create_err;

int fail(spgg_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

int create_fail(int code, const std::string& msg) {
  g_create_err = msg;
  return code;
}

int hip_check(spgg_ctx* c, hipError_t e, const char* what) {
  if (e == hipSuccess) return SPGG_OK;
  return fail(c, SPGG_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

// A tuning knob's value (spgg_abi.h, "Environment knobs"), read only when SPGG_TUNING=1: a stray
// variable in a user's environment never changes the layout or the schedule of a production run.
const char* tuning_env(const char* name) {
  const char* on = getenv("SPGG_TUNING");
  return on && !strcmp(on, "1") ? getenv(name) : nullptr;
}

// Below this many workgroups per launch (at the operator's agents per thread)
// a batch runs one agent per thread (4x the workgroups, each a quarter as long).
// Measured with the striped history record (which keeps the atomics per address
// at <= 64 per iteration): one L=200 replica (40 tiles) 10.8 -> 10.2 us/step with
// one agent per thread, 8 replicas (320 tiles, M=2) 16.2 -> 17.0, one L=1000
// replica (1000 tiles) 28.1 -> 53.9.  SPGG_APT=1 / =<max> forces either.
constexpr long long kSmallBatchTiles = 128;
// Below this many 1024-agent tiles, two agents per thread (20 x 25 tiles, compile-time width
// 20: where 20 divides L >= 60) -- twice the workgroups of half the length (round 4, L=200,
// us/step at 1 / 2 replica groups, profiles/r04/plan_sweep.txt: one replica 8.38 vs 10.65 at
// one agent per thread; run100 7.78 vs 9.34; 8 replicas M=2 action 12.43 vs 14.17 at four
// agents per thread; 16 replicas 13.89 vs 14.18 (M=1); 32 replicas 23.90 vs 23.07 and one
// L=1000 replica, 1000 tiles, 33.4 vs 26.3: four agents per thread from here on).
constexpr long long kTwoPerThreadTiles = 800;

// MT19937 generator layout (spgg_mt_chains).  One chain generates a replica's draws at
// ~200 ns per 227 words (measured: 119-215 ns with the steps running), i.e. ~W/227*0.2 us
// per iteration of W words; the steps take ~15 ps per agent of the batch (cfg3: 62 us for
// 4.2e6 agents), >= ~8 us.  Chains per replica: a power of two with kGenRateMargin x the needed rate; a
// chain covers >= ~1e6 words (a jump costs ~20 us on 8 workgroups) and a chunk >= 128
// iterations (cfg3, 105 x L=200, us/step by chains x iterations per chain: 16x4 86.0,
// 32x2 96.4 -- 64-iteration chunks; 16x9 71.2, 8x18 72.7, 32x4 74.0, 64x2 74.8 -- 128-144;
// profiles/r03/mt_chain_layouts.txt); the draw ring (2 chunks) stays <= 512 MB.  Lattices
// under 4096 words per iteration keep one chain.
// Chains generate at kGenRateMargin x the rate the steps consume: each generator workgroup beyond
// the one a CU holds beside five step workgroups displaces a step workgroup for its whole chunk,
// so more chains cost more than they hide (cfg3 MT19937 whole run, 3000 iterations, per-process:
// 2 chains 69.4 us/iter -- too slow to keep up -- 4 chains 65.6-66.0, 8 (round 4's 4x) 69.5-70.1,
// 16 72.3; profiles/r05/mt_chains_cfg3.txt).
constexpr double kGenRateMargin = 2.0;

void choose_mt_chains(spgg_ctx* c) {
  const spgg_config& cfg = c->cfg;
  const long long W = draw_mt_words(c->n, draw_planes(cfg.algorithm));
  int chains = 1, per = 8;
  const long long batch = cfg.batch_reps > 0 ? cfg.batch_reps : cfg.n_rep;
  if (W >= 4096) {
    const double gen_ns = W / 227.0 * 200.0;
    const double step_ns = std::max(8000.0, (double)batch * c->n * 0.015);
    const double need = kGenRateMargin * gen_ns / step_ns;
    while (chains < 256 && chains < need) chains *= 2;
    if (chains > 1)
      per = (int)std::max((1000000 + W - 1) / W, (long long)((128 + chains - 1) / chains));
    // bytes per iteration of the WHOLE batch: every context of one batch (replica groups of
    // different sizes) must get the same layout, since the caller sizes the shared draw and
    // snapshot buffers from one of them (spgg_draw_layout)
    const double rec = draw_words_of(c->n, cfg.algorithm) * 4.0 * batch;
    while (chains > 1 && 2.0 * chains * per * rec > 512e6) {
      if (per > 1) per = std::max(1, per / 2);
      else chains /= 2;
    }
  }
  if (const char* e = tuning_env("SPGG_MT_CHAINS")) {
    int v = atoi(e), p2 = 1;
    while (p2 < 256 && p2 < v) p2 *= 2;
    chains = W >= 624 ? std::max(1, p2) : 1;  // (a chain's first key block must lie in its window)
  }
  if (const char* e = tuning_env("SPGG_MT_PER_CHAIN")) per = std::max(1, std::min(4096, atoi(e)));
  if (chains == 1)
    if (const char* e = tuning_env("SPGG_MT_CHUNK")) per = std::max(1, std::min(256, atoi(e)));
  // a chain indexes its words in 32 bits (below 2^31)
  per = (int)std::max(1LL, std::min((long long)per, ((1LL << 31) - (1LL << 16)) / W));
  c->chains = chains;
  c->per_chain = per;
  c->gen_chunk = chains * per;
  c->jump_levels = 0;
  while ((1 << c->jump_levels) < chains) ++c->jump_levels;
  if (chains > 1) {
    // the jump polynomials the first spgg_step needs (mt_lazy_init), computed now on a thread of
    // their own: jump_poly caches them per exponent under its lock, so the step's calls find them
    // ready, or wait for this computation instead of repeating it
    const uint64_t D = (uint64_t)per * (uint64_t)W;
    const int J = c->jump_levels;
    try {
      std::thread([D, J] {
        uint32_t tmp[624];
        for (int j = 0; j <= J; ++j) spgg_mt::jump_poly((D << j) - 1, tmp);
      }).detach();
    } catch (...) {  // no thread: computed by the first step
    }
  }
}

// Workgroups per history-record stripe (spgg_stat_stripes).
constexpr int kTilesPerStripe = 64;

// Tile shape: <= max_agents (256 threads x agents per thread), rows >= 16
// wide when L allows; minimise padded lanes + halo recompute per agent
// (L=200 -> 40x25, L=1000 -> 40x25 at 1024 agents).
void choose_tile(int L, int max_agents, int* TW, int* TH) {
  int best_w = std::min(L, 32), best_h = std::min(L, 32);
  double best = 1e300;
  for (int w = std::min(L, 16); w <= std::min(L, 56); ++w) {
    for (int h = 1; h <= std::min(L, 64); ++h) {
      if (w * h > max_agents) break;
      const int tx = (L + w - 1) / w, ty = (L + h - 1) / h;
      const double slots = (double)tx * ty * ((w * h + kBlock - 1) / kBlock) * kBlock;
      const double halo = (double)tx * ty * ((w + 4) * (h + 4) - w * h);
      const double cost = (slots + 2.0 * halo) / ((double)L * L);
      if (cost < best - 1e-12 || (cost <= best + 1e-12 && w > best_w)) {  // ties: wider rows
        best = cost;
        best_w = w;
        best_h = h;
      }
    }
  }
  *TW = best_w;
  *TH = best_h;
}

// For every tile, the ring cells in the kernel's enumeration order: the
// agent index and the offset of its owner's border record (owner tile *
// PF * PB + slot) within a replica's record buffer.
int build_ring_table(spgg_ctx* c) {
  const int L = c->cfg.L, HA = c->cfg.second_order ? 2 : 1;
  const int PF = spgg_impl::pf_of(c->cfg.algorithm);
  auto wrapL = [L](int x) { return ((x % L) + L) % L; };
  int rmax = 1;
  for (int tile = 0; tile < c->tiles_per_rep; ++tile) {
    const int ty = tile / c->tiles_x, tx = tile % c->tiles_x;
    const int th = std::min(c->TH, L - ty * c->TH), tw = std::min(c->TW, L - tx * c->TW);
    rmax = std::max(rmax, (tw + 2 * HA) * (th + 2 * HA) - th * tw);
  }
  // + the border-slot table (border_slot_table, kernel phase 2): per tile shape (th < TH: +2, tw < TW: +1) and
  // thread, the border-record slot of each agent slot u < 4 (agent tid + u*kBlock), -1 for an
  // interior cell or a slot past the tile (its shadow agent's owner writes the record)
  std::vector<int2> tab((size_t)c->tiles_per_rep * rmax + 4 * kBlock, make_int2(0, 0));
  {
    const int ty_last = (L - 1) / c->TH, tx_last = (L - 1) / c->TW;
    for (int shape = 0; shape < 4; ++shape) {
      const int th = (shape & 2) ? L - ty_last * c->TH : c->TH, tw = (shape & 1) ? L - tx_last * c->TW : c->TW;
      for (int tid = 0; tid < kBlock; ++tid) {
        uint64_t w = 0;
        for (int u = 0; u < 4; ++u) {
          const int k = tid + u * kBlock;
          const int slot = k < th * tw ? spgg_impl::border_slot_or_none(k / tw, k % tw, th, tw, HA) : -1;
          w |= (uint64_t)(uint16_t)(int16_t)slot << (16 * u);
        }
        tab[(size_t)c->tiles_per_rep * rmax + shape * kBlock + tid] = make_int2((int)(uint32_t)w, (int)(uint32_t)(w >> 32));
      }
    }
  }
  for (int tile = 0; tile < c->tiles_per_rep; ++tile) {
    const int ty = tile / c->tiles_x, tx = tile % c->tiles_x;
    const int y0 = ty * c->TH, x0 = tx * c->TW;
    const int th = std::min(c->TH, L - y0), tw = std::min(c->TW, L - x0);
    const int ring = (tw + 2 * HA) * (th + 2 * HA) - th * tw;
    for (int k = 0; k < ring; ++k) {
      int ay, ax;
      spgg_impl::ring_cell(k, th, tw, HA, &ay, &ax);
      const int gy = wrapL(y0 - HA + ay), gx = wrapL(x0 - HA + ax);
      const int oty = gy / c->TH, otx = gx / c->TW;
      const int oth = std::min(c->TH, L - oty * c->TH), otw = std::min(c->TW, L - otx * c->TW);
      const int slot = spgg_impl::border_slot(gy - oty * c->TH, gx - otx * c->TW, oth, otw, HA);
      tab[(size_t)tile * rmax + k] = make_int2(gy * L + gx, (oty * c->tiles_x + otx) * PF * c->PB + slot);
    }
  }
  if (rmax > spgg_impl::ring_per_thread(c->cfg.second_order != 0) * kBlock)
    return fail(c, SPGG_E_ARG, "tile ring exceeds the kernel's ring cells per thread");
  c->ring_max = rmax;
  int rc = hip_check(c, hipMalloc(&c->d_ring, tab.size() * sizeof(int2)), "hipMalloc(ring)");
  if (rc) return rc;
  return hip_check(c, hipMemcpy(c->d_ring, tab.data(), tab.size() * sizeof(int2), hipMemcpyHostToDevice),
                   "hipMemcpy(ring)");
}

// Iteration t reads S_t, R_t, records [(t-1)&1] and writes [t&1]; Q, md,
// atd in place.  t = 0 addresses the iteration-1 prologue (S_1 and R_1 in,
// records [0] out).
TileArgs make_args(const spgg_ctx* c, int t) {
  TileArgs a{};
  if (t == 0) {
    a.S_out = c->buf.S[0];
    a.R_in = c->buf.R[0];
    a.pub_out = c->buf.pub[0];
  } else {
    const int cur = (t - 1) & 1, nxt = t & 1;
    a.S_in = c->buf.S[cur];    a.S_out = c->buf.S[nxt];
    a.R_in = c->buf.R[cur];    a.R_out = c->buf.R[nxt];
    a.pub_in = c->buf.pub[cur];  a.pub_out = c->buf.pub[nxt];
  }
  a.Q = c->buf.Q;
  a.md = c->buf.md;
  a.atd = c->buf.atd;
  // this iteration's draw record (ring slot (t-1) % draw_slots)
  a.draws = c->buf.draws ? c->buf.draws + (size_t)((t >= 1 ? t - 1 : 0) % c->draw_slots) * c->buf.draw_slot_stride
                         : nullptr;
  a.draw_words = (int)c->draw_words;
  a.planes = draw_planes(c->cfg.algorithm);
  a.eps = c->buf.eps;
  a.stats = c->buf.stats;
  a.stop_iter = c->buf.stop_iter;
  a.params = c->d_params;
  a.L = c->cfg.L;
  a.n = c->n;
  a.TW = c->TW;
  a.TH = c->TH;
  a.tiles_x = c->tiles_x;
  a.tiles_per_rep = c->tiles_per_rep;
  a.n_rep = c->cfg.n_rep;
  a.slots = c->cfg.iterations + 2;
  a.PB = c->PB;
  a.ring = c->d_ring;
  a.ring_max = c->ring_max;
  a.stripes = c->stripes;
  a.rep_stride = c->rep_stride;
  return a;
}

spgg_impl::LaunchCfg launch_cfg(const spgg_ctx* c) {
  spgg_impl::LaunchCfg lc;
  lc.m2 = c->cfg.second_order != 0;
  lc.as = c->cfg.state_mode == SPGG_STATE_ACTION;
  lc.rq = c->cfg.rep_int8 != 0;
  lc.rng = c->cfg.rng_mode;
  lc.twc = twc_of(c->cfg, c->TW, c->TH);
  lc.apt = c->apt;
  lc.total_tiles = c->cfg.n_rep * c->tiles_per_rep;
  lc.lds_bytes = c->lds_bytes;
  return lc;
}

void launch_step(const spgg_ctx* c, int t, int fin, hipStream_t s, const spgg_impl::PersistArgs* pa = nullptr) {
  const TileArgs a = make_args(c, t);
  const spgg_impl::LaunchCfg lc = launch_cfg(c);
  switch (c->cfg.algorithm) {
    case SPGG_ALG_SARSA: spgg_impl::launch_alg<SPGG_ALG_SARSA>(lc, a, t, fin, s, pa); break;
    case SPGG_ALG_EXPECTED_SARSA: spgg_impl::launch_alg<SPGG_ALG_EXPECTED_SARSA>(lc, a, t, fin, s, pa); break;
    case SPGG_ALG_DOUBLE_Q: spgg_impl::launch_alg<SPGG_ALG_DOUBLE_Q>(lc, a, t, fin, s, pa); break;
    default: spgg_impl::launch_alg<SPGG_ALG_QLEARNING>(lc, a, t, fin, s, pa); break;
  }
}

// Workgroups of the context's persistent instance one CU holds (0: none for this layout).
int persist_blocks(const spgg_ctx* c) {
  const spgg_impl::LaunchCfg lc = launch_cfg(c);
  switch (c->cfg.algorithm) {
    case SPGG_ALG_SARSA: return spgg_impl::persist_blocks_per_cu<SPGG_ALG_SARSA>(lc);
    case SPGG_ALG_EXPECTED_SARSA: return spgg_impl::persist_blocks_per_cu<SPGG_ALG_EXPECTED_SARSA>(lc);
    case SPGG_ALG_DOUBLE_Q: return spgg_impl::persist_blocks_per_cu<SPGG_ALG_DOUBLE_Q>(lc);
    default: return spgg_impl::persist_blocks_per_cu<SPGG_ALG_QLEARNING>(lc);
  }
}

// Error word (and its pinned host copy) of a context, for the generator and persistent launches.
int err_word_init(spgg_ctx* c) {
  int rc = SPGG_OK;
  if (!c->d_err) {
    rc = hip_check(c, hipMalloc(&c->d_err, 4), "hipMalloc(err)");
    if (!rc) rc = hip_check(c, hipMemset(c->d_err, 0, 4), "hipMemset(err)");
  }
  if (!rc && !c->h_err) {
    void* h = nullptr;
    // (mapped: a persistent launch's failing workgroup sets it directly, no copy per launch)
    rc = hip_check(c, hipHostMalloc(&h, 4, hipHostMallocMapped), "hipHostMalloc(err)");
    if (!rc) {
      c->h_err = static_cast<volatile uint32_t*>(h);
      *c->h_err = 0;
    }
  }
  return rc;
}

// The persistent launch's arrival counters and error word (once per context).
int persist_lazy_init(spgg_ctx* c) {
  int rc = err_word_init(c);
  if (rc || c->d_bar) return rc;
  const size_t bytes = (size_t)c->cfg.n_rep * c->stripes * spgg_impl::kBarWords * 4;
  rc = hip_check(c, hipMalloc(&c->d_bar, bytes), "hipMalloc(barrier counters)");
  if (!rc) rc = hip_check(c, hipMemset(c->d_bar, 0, bytes), "hipMemset(barrier counters)");
  return rc;
}

// Iterations t .. t1 (t1 > t) as ONE persistent launch; a run's first one zeroes the counters.
void launch_persist(spgg_ctx* c, int t, int t1, hipStream_t s) {
  if (t == 1) {
    (void)hipMemsetAsync(c->d_bar, 0, (size_t)c->cfg.n_rep * c->stripes * spgg_impl::kBarWords * 4, s);
    c->bar_base = 0;
  }
  spgg_impl::PersistArgs pa{};
  for (int i = 0; i < 2; ++i) {
    pa.S[i] = c->buf.S[i];
    pa.R[i] = c->buf.R[i];
    pa.pub[i] = c->buf.pub[i];
  }
  pa.draws0 = c->cfg.rng_mode == SPGG_RNG_PHILOX ? nullptr : c->buf.draws;
  pa.draw_stride = c->buf.draw_slot_stride;
  pa.draw_slots = c->draw_slots;
  pa.t_end = t1;
  pa.bar = c->d_bar;
  pa.shards = c->stripes;
  pa.base = c->bar_base;
  pa.err = c->d_err;
  void* hd = nullptr;
  pa.err_host = hipHostGetDevicePointer(&hd, (void*)c->h_err, 0) == hipSuccess ? static_cast<uint32_t*>(hd)
                                                                                 : const_cast<uint32_t*>(c->h_err);
  launch_step(c, t, 0, s, &pa);
  c->bar_base += (uint32_t)(t1 - t);
  // (no copy of the error word after the launch: a D2H copy in the stream cost a 20-iteration window
  // ~150 us; the failing workgroup writes the pinned host word itself, which spgg_status reads)
}

// q: the chunk a pipelined launch generates (-1: a single-chain launch in place on mt_state)
GenArgs gen_args(const spgg_ctx* c, int q = -1) {
  GenArgs g{};
  g.key_in = q <= 0 ? c->buf.mt_state : c->d_keybuf[q & 1];
  g.key_out = q < 0 ? c->buf.mt_state : c->d_keybuf[(q + 1) & 1];
  g.parts = q < 0 ? nullptr : c->d_parts[q & 1];
  g.run_pos0 = c->d_run_pos0;
  g.chains = q < 0 ? 1 : c->chains;
  g.per_chain = q < 0 ? c->gen_chunk : c->per_chain;
  g.snap = c->buf.mt_snap;
  g.snap_stride = c->buf.mt_snap_stride;
  g.snap_slots = c->snap_slots;
  g.draws = c->buf.draws;
  g.draw_stride = c->buf.draw_slot_stride;
  g.draw_slots = c->draw_slots;
  g.draw_words = (int)c->draw_words;
  g.eps = c->buf.eps;
  g.eps_slots = c->cfg.iterations + 2;
  g.stop_iter = c->buf.stop_iter;
  g.err = c->d_err;
  g.n = c->n;
  g.alg = c->cfg.algorithm;
  return g;
}

void launch_gen(const spgg_ctx* c, int t0, int t1, int skip_stopped, hipStream_t s, int q = -1) {
  const GenArgs g = gen_args(c, q);
  hipLaunchKernelGGL(spgg_mt_gen_kernel, dim3(c->cfg.n_rep * g.chains), dim3(kGenThreads), 0, s, g, t0, t1,
                     skip_stopped);
}

// A stream for the library's generator (gen) or the caller's replica groups (spgg_stream_create).
// HIP maps streams onto a few hardware queues (GPU_MAX_HW_QUEUES, 4), and streams that share
// one are serialised; SPGG_STREAM_MODE: 0 = hipStreamCreateWithFlags, 1 = greatest priority,
// 2 (default) = a CU mask of every CU (a queue of its own), 3 = CU-masked and partitioned: the
// generator on every SPGG_GEN_CU_STRIDE-th CU (default 8: 32 of 256), the groups on the rest.
// The generator's stream (SPGG_GEN_STREAM_MODE): plain non-blocking (mode 0).  CU-masked streams
// are BLOCKING -- every operation on the legacy null stream then waits for the generator's queued
// chunks (round 3, when the engine synced on the null stream: cfg2 11.1 vs 15.8 us/iter, cfg5 32.3
// vs 52.1, but cfg3 84.0 vs 99.9 in favour of the CU mask; profiles/r03/streams.txt).  Since the
// engine's run loop left the null stream (round 4), mode 0 is the faster one at every batch size
// (cfg3 MT19937 whole run 71.4 vs 74.1 us/iter, cfg5 36.0 vs 41.3; an idle CU-masked generator
// stream alone slowed the steps: 59.7 vs 65.6; profiles/r04/generator_stream_modes.txt).
hipError_t make_stream(hipStream_t* s, bool gen) {
  const char* e = tuning_env(gen ? "SPGG_GEN_STREAM_MODE" : "SPGG_STREAM_MODE");
  const int mode = e ? atoi(e) : gen ? 0 : 2;
  if (mode == 1 || mode == 4) {  // 1: greatest priority, 4: least (non-blocking)
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess)
      return hipStreamCreateWithPriority(s, hipStreamNonBlocking, mode == 1 ? hi : lo);
  } else if (mode == 2 || mode == 3) {
    int dev = 0, cus = 0;
    hipError_t r = hipGetDevice(&dev);
    if (r == hipSuccess) r = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (r == hipSuccess && cus > 0) {
      const char* st = tuning_env("SPGG_GEN_CU_STRIDE");
      const int stride = std::max(2, st ? atoi(st) : 8);
      std::vector<uint32_t> mask((cus + 31) / 32, 0u);
      for (int i = 0; i < cus; ++i)
        if (mode == 2 || ((i % stride == 0) == gen)) mask[i / 32] |= 1u << (i % 32);
      return hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data());
    }
  }
  return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

// MT19937 pipeline: generation of chunk q (iterations q*K+1 .. (q+1)*K) waits for the steps
// of chunk q-2 (whose ring slots it reuses) and is enqueued when chunk q-1 starts, so it
// overlaps the steps of chunk q-1; the steps of chunk q wait for it.
int mt_lazy_init(spgg_ctx* c) {
  if (c->gen_done[0] && c->h_err) return SPGG_OK;
  int rc = SPGG_OK;
  if (!c->gen_stream) {
    rc = hip_check(c, make_stream(&c->gen_stream, true), "hipStreamCreate(gen)");
    if (rc) return rc;
    c->own_gen_stream = true;
  }
  for (int i = 0; i < 2 && !rc; ++i) {
    rc = hip_check(c, hipEventCreateWithFlags(&c->gen_done[i], hipEventDisableTiming), "hipEventCreate");
    if (!rc) rc = hip_check(c, hipEventCreateWithFlags(&c->step_done[i], hipEventDisableTiming), "hipEventCreate");
  }
  if (!rc) rc = hip_check(c, hipEventCreateWithFlags(&c->gen_idle, hipEventDisableTiming), "hipEventCreate");
  if (!rc) rc = hip_check(c, hipEventCreateWithFlags(&c->caller_ready, hipEventDisableTiming), "hipEventCreate");
  if (!rc) rc = err_word_init(c);
  if (rc || c->chains == 1) return rc;
  // chained generator: start windows, chunk keys, and the jump polynomials
  const size_t R = c->cfg.n_rep, win = R * c->chains * spgg_mt::kSplits * 624;
  for (int i = 0; i < 2 && !rc; ++i) {
    rc = hip_check(c, hipMalloc(&c->d_parts[i], win * 4), "hipMalloc(mt parts)");
    if (!rc) rc = hip_check(c, hipMalloc(&c->d_keybuf[i], R * 625 * 4), "hipMalloc(mt keys)");
  }
  if (!rc) rc = hip_check(c, hipMalloc(&c->d_run_pos0, R * 4), "hipMalloc(mt pos)");
  if (!rc) rc = hip_check(c, hipMalloc(&c->d_polys, (size_t)(c->jump_levels + 1) * 624 * 4), "hipMalloc(mt polys)");
  if (rc) return rc;
  const uint64_t W = (uint64_t)draw_mt_words(c->n, draw_planes(c->cfg.algorithm));
  std::vector<uint32_t> polys((size_t)(c->jump_levels + 1) * 624);
  for (int j = 0; j <= c->jump_levels; ++j) {
    spgg_mt::jump_poly(((uint64_t)c->per_chain * W << j) - 1, polys.data() + (size_t)j * 624);
    bool nz = false;
    for (int i = 0; i < 624; ++i) nz |= polys[(size_t)j * 624 + i] != 0;
    if (!nz) return fail(c, SPGG_E_STATE, "MT19937 jump polynomial unavailable");
  }
  return hip_check(c, hipMemcpy(c->d_polys, polys.data(), polys.size() * 4, hipMemcpyHostToDevice),
                   "hipMemcpy(mt polys)");
}

// Chained generator (chains > 1): before chunk 0, every chain's window is seeded with the
// window at iteration 1's first word and jumped by (its chain index) x per_chain iterations,
// one jump level per bit of the index; after chunk q's generation, chains >= 1 jump one
// chunk ahead (chain 0 continues from chunk q's last chain: key_out).
void enqueue_gen_chunk(spgg_ctx* c, int q) {
  const int K = c->gen_chunk;
  const int t0 = q * K + 1, t1 = std::min((q + 1) * K, c->cfg.iterations);
  const int J = c->jump_levels, R = c->cfg.n_rep;
  if (q >= 2) (void)hipStreamWaitEvent(c->gen_stream, c->step_done[q & 1], 0);
  if (c->chains > 1 && q == 0) {
    spgg_mt::launch_seed(c->buf.mt_state, c->d_run_pos0, c->d_parts[J & 1], R, c->chains, c->gen_stream);
    for (int j = 0; j < J; ++j)
      spgg_mt::launch_jump(c->d_parts[(J - j) & 1], c->d_parts[(J - j - 1) & 1], c->d_polys + (size_t)j * 624, R,
                           c->chains, j, nullptr, c->gen_stream);
  }
  launch_gen(c, t0, t1, 1, c->gen_stream, c->chains > 1 ? q : -1);
  (void)hipEventRecord(c->gen_done[q & 1], c->gen_stream);
  // the error word after this chunk, for spgg_status (no host sync)
  (void)hipMemcpyAsync((void*)c->h_err, c->d_err, 4, hipMemcpyDeviceToHost, c->gen_stream);
  if (c->chains > 1 && t1 < c->cfg.iterations)
    spgg_mt::launch_jump(c->d_parts[q & 1], c->d_parts[(q + 1) & 1], c->d_polys + (size_t)J * 624, R, c->chains, -1,
                         c->buf.stop_iter, c->gen_stream);
  c->gen_upto = t1;
}

}  // namespace

#ifndef SPGG_TIMING
#define SPGG_TIMING 0
#endif

#ifndef SPGG_BUILD_ID
#define SPGG_BUILD_ID "unversioned"
#endif

extern "C" {

int spgg_abi_version(void) { return SPGG_ABI_VERSION; }

// "spgg-build:<id>" also lets build.py read the id from the file without loading it
static const char kBuildTag[] = "spgg-build:" SPGG_BUILD_ID;
const char* spgg_build_id(void) { return kBuildTag + 11; }

int spgg_draw_planes(int32_t algorithm) {
  if (algorithm < SPGG_ALG_QLEARNING || algorithm > SPGG_ALG_DOUBLE_Q) return SPGG_E_ARG;
  return draw_planes(algorithm);
}

const char* spgg_last_error(const spgg_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_err.c_str(); }

int spgg_create(spgg_ctx** out, const spgg_config* cfg) {
  if (!out || !cfg) return create_fail(SPGG_E_ARG, "spgg_create: null argument");
  *out = nullptr;
  g_create_err.clear();
  if (cfg->n_rep < 1 || cfg->L < 1 || cfg->iterations < 0 || (long long)cfg->L * cfg->L > (1LL << 30))
    return create_fail(SPGG_E_ARG, "spgg_create: n_rep >= 1, 1 <= L <= 32768, iterations >= 0 required");
  if (cfg->state_mode != SPGG_STATE_REPUTATION && cfg->state_mode != SPGG_STATE_ACTION)
    return create_fail(SPGG_E_ARG, "spgg_create: unknown state_mode");
  if (cfg->rng_mode < SPGG_RNG_INJECT || cfg->rng_mode > SPGG_RNG_PHILOX)
    return create_fail(SPGG_E_ARG, "spgg_create: unknown rng_mode");
  if (cfg->algorithm < SPGG_ALG_QLEARNING || cfg->algorithm > SPGG_ALG_DOUBLE_Q)
    return create_fail(SPGG_E_ARG, "spgg_create: unknown algorithm");
  if (cfg->iterations >= (1 << 26))  // Philox counter: t + pair*2^26
    return create_fail(SPGG_E_ARG, "spgg_create: iterations >= 2^26");
  if (cfg->batch_reps != 0 && cfg->batch_reps < cfg->n_rep)
    return create_fail(SPGG_E_ARG, "spgg_create: batch_reps < n_rep");
  if ((long long)cfg->n_rep * cfg->L * cfg->L > (1LL << 31) - 1)
    return create_fail(SPGG_E_ARG, "spgg_create: n_rep * L * L >= 2^31");
  // the step kernel addresses a replica's arrays with 32-bit byte offsets (Q: qw doubles per agent)
  if ((long long)cfg->L * cfg->L * spgg_impl::qw_of(cfg->algorithm) * 8 > 0xFFFFFFFFLL)
    return create_fail(SPGG_E_ARG, "spgg_create: a replica's Q table exceeds 4 GiB (32-bit offsets)");
  // Agents per thread: the operator's maximum (tiles of up to 1024 agents); two for a
  // batch of fewer than kTwoPerThreadTiles such tiles where 20 x 25 tiles fit L; else one
  // for a batch that would launch fewer than kSmallBatchTiles workgroups (4x the
  // workgroups, each a quarter as long).  Decided from the WHOLE batch
  // (batch_reps), so the replica groups of one batch share one tiling: their
  // border-record and history-record strides must agree.  SPGG_APT = 1 / max forces either.
  const int apt_max = spgg_impl::apt_of(cfg->algorithm);
  int apt = apt_max;
  {
    int tw4, th4;
    choose_tile(cfg->L, kBlock * apt_max, &tw4, &th4);
    const long long reps = cfg->batch_reps > 0 ? cfg->batch_reps : cfg->n_rep;
    const long long tiles4 = reps * ((cfg->L + tw4 - 1) / tw4) * ((cfg->L + th4 - 1) / th4);
    if (const char* e = tuning_env("SPGG_APT")) {
      if (!strcmp(e, "max") || atoi(e) == apt_max) apt = apt_max;
      else if (!strcmp(e, "1")) apt = 1;
      else if (!strcmp(e, "2")) apt = 2;
      else
        return create_fail(SPGG_E_ARG, std::string("SPGG_APT=") + e + ": expected 1, 2 or max (" +
                                           std::to_string(apt_max) + " agents per thread for this operator)");
    } else if (tiles4 < kTwoPerThreadTiles && apt_max > 2 && cfg->L % 20 == 0 && cfg->L >= 60) {
      apt = 2;
    } else if (tiles4 < kSmallBatchTiles) {
      apt = 1;
    }
  }
  spgg_ctx* c = new (std::nothrow) spgg_ctx();
  if (!c) return create_fail(SPGG_E_ARG, "spgg_create: out of host memory");
  c->cfg = *cfg;
  c->n = cfg->L * cfg->L;
  c->apt = apt;
  if (cfg->rng_mode == SPGG_RNG_MT19937) choose_mt_chains(c);
  c->draw_slots = 2 * c->gen_chunk;
  c->snap_slots = 3 * c->gen_chunk + 1;
  c->draw_words = draw_words_of(c->n, cfg->algorithm);
  choose_tile(cfg->L, kBlock * c->apt, &c->TW, &c->TH);
  // two agents per thread: 20 x 25 (500 agents) where 20 divides L -- the same cost as the
  // chooser's 25 x 20 (a transpose), with a compile-time tile width (aligned-dword windows)
  if (c->apt == 2 && c->apt < spgg_impl::apt_of(cfg->algorithm) && cfg->L % 20 == 0 && cfg->L >= 60) {
    c->TW = 20;
    c->TH = 25;
  }
  if (const char* e = tuning_env("SPGG_TILE")) {  // tuning knob: "<TW>x<TH>"
    int w = 0, h = 0;
    if (sscanf(e, "%dx%d", &w, &h) == 2 && w >= 1 && h >= 1 && w <= std::min(cfg->L, 56) &&
        h <= std::min(cfg->L, 64) && w * h <= kBlock * c->apt) {
      c->TW = w;
      c->TH = h;
    }
  }
  c->tiles_x = (cfg->L + c->TW - 1) / c->TW;
  c->tiles_per_rep = c->tiles_x * ((cfg->L + c->TH - 1) / c->TH);
  // history-record stripes: <= kTilesPerStripe workgroups add to one record address per
  // iteration (a single record of an L=1000 replica took 1000 atomics per address: ~12 us)
  int tiles_per_stripe = kTilesPerStripe;
  if (const char* e = tuning_env("SPGG_TILES_PER_STRIPE")) tiles_per_stripe = std::max(1, atoi(e));
  while (c->stripes < 32 && (c->tiles_per_rep + c->stripes - 1) / c->stripes > tiles_per_stripe) c->stripes *= 2;
  const int HA = cfg->second_order ? 2 : 1;
  const bool twc = twc_of(*cfg, c->TW, c->TH) > 0;
  const LdsLayout ly = lds_layout(c->TW, c->TH, HA + 2, HA, cfg->rep_int8 ? 1 : 8, twc,
                                  twc && cfg->rng_mode != SPGG_RNG_PHILOX);  // (the kernel's DSTAGE)
  c->lds_bytes = (size_t)ly.bytes;
  c->PB = spgg_impl::pub_slots(c->TW, c->TH, HA);
  // stage_region's per-thread register window must cover the S and R halos
  const int js = spgg_impl::js_of(cfg->second_order != 0), jr = spgg_impl::jr_of();
  if (c->lds_bytes > 160 * 1024 || ly.sw * ly.sh > js * kBlock || ly.aw * ly.ah > jr * kBlock) {
    delete c;
    return create_fail(SPGG_E_ARG, "spgg_create: tile windows exceed the kernel's LDS / staging budget");
  }
  int rc = hip_check(c, hipSetDevice(cfg->device), "hipSetDevice");
  if (!rc) rc = build_ring_table(c);
  if (!rc) {  // + the ring cells' border records (or the S_{t-1} plus-count plane that shares them)
    c->lds_bytes += std::max((size_t)c->ring_max * spgg_impl::pf_of(cfg->algorithm) * sizeof(double),
                             (size_t)(ly.ah + 2) * kPcPitch);
    if (c->lds_bytes > 160 * 1024) rc = fail(c, SPGG_E_ARG, "tile LDS footprint exceeds 160 KB");
  }
  // persistent launches (opt-in, SPGG_PERSIST=1): when the whole batch's tiles (every replica
  // group of it, which run concurrently) fit the device at once -- the persistent instance's
  // occupancy x CUs; MT19937: one workgroup per CU fewer, the room a generator workgroup of the
  // next chunk takes beside them (with every slot counted, a cfg5 launch waited > 1 s for three
  // tiles that the generator's workgroups kept from being dispatched) -- each spgg_step call (each
  // generator chunk, MT19937) is one launch instead of one per iteration.  Off by default: measured
  // slower on every BASELINE shape ("Persistent launches")
  if (!rc && cfg->rng_mode != SPGG_RNG_INJECT) {
    const char* e = tuning_env("SPGG_PERSIST");
    const int nb = (e && !strcmp(e, "1")) ? persist_blocks(c) : 0;
    int cus = 0;
    if (nb > 0 && hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, cfg->device) == hipSuccess) {
      const long long reps = cfg->batch_reps > 0 ? cfg->batch_reps : cfg->n_rep;
      c->persist_capacity = (nb - (cfg->rng_mode == SPGG_RNG_MT19937 ? 1 : 0)) * cus;
      c->persist = reps * c->tiles_per_rep <= (long long)c->persist_capacity;
    }
  }
  if (rc) {
    g_create_err = c->err;
    spgg_destroy(c);
    return rc;
  }
  *out = c;
  return SPGG_OK;
}

// The step kernel hands each XCD a consecutive range of logical tiles (blockIdx remap), so the
// replicas of a launch split over the XCDs in index order.  A replica with kappa == 0 costs ~0.82
// of another (no NI term: its recomputed record and NI percent are skipped; phase stamps,
// profiles/r05/phase_stamps_t15_t450.txt), and a batch ordered like the reference's sweeps (kappa in
// blocks of seeds) gives some XCDs more of them: cfg3's groups 5-7 % above the mean on their
// busiest XCD.  Logical replica j runs replica (j * stride) % n_rep: the stride (coprime to n_rep)
// that minimises the busiest XCD's share of that estimate, or 1 when no stride gains >= 1 %.
// Results do not depend on it (every replica is computed alone).
static int rep_stride_for(const spgg_ctx* c, const spgg_rep_params* params) {
  const int R = c->cfg.n_rep, tiles = c->tiles_per_rep;
  if (R < 3 || tiles < 1) return 1;
  if (const char* e = tuning_env("SPGG_REP_STRIDE")) {  // tuning knob (a stride not coprime to R: 1)
    const int st = atoi(e) % R;
    return st > 1 && std::gcd(st, R) == 1 ? st : 1;
  }
  const long long total = (long long)R * tiles, per = (total + 7) / 8;
  auto busiest = [&](int stride) {
    double load[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < R; ++j) {
      const int r = (int)(((long long)j * stride) % R);
      const double w = params[r].kappa == 0.0 ? 0.82 : 1.0;
      for (long long k = (long long)j * tiles; k < (long long)(j + 1) * tiles;) {  // tiles of j per XCD
        const int x = (int)(k / per);
        const long long k1 = std::min((long long)(j + 1) * tiles, (x + 1) * per);
        load[x] += w * (double)(k1 - k);
        k = k1;
      }
    }
    return *std::max_element(load, load + 8);
  };
  const double base = busiest(1);
  int best = 1;
  double best_load = base;
  for (int st = 2; st < R; ++st) {
    if (std::gcd(st, R) != 1) continue;
    const double l = busiest(st);
    if (l < best_load - 1e-9) { best_load = l; best = st; }
  }
  return best_load <= 0.99 * base ? best : 1;
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
  // parameters are fixed for a run: kappa == 0 replicas keep no pending NI record (md / atd), and
  // the large-batch kernels rebuild iteration t-1's rewards and |alpha*td'| from the parameters
  // in force at launch t (recomputed record) -- a change between two spgg_step calls of one run
  // would apply the deferred NI term with other rewards (spgg_step / spgg_flush refuse to go on)
  if (c->params_host.size() == (size_t)c->cfg.n_rep)
    c->params_moved |= memcmp(c->params_host.data(), params, bytes) != 0;
  c->params_host.assign(params, params + c->cfg.n_rep);
  c->rep_stride = rep_stride_for(c, params);
  c->params_set = true;
  return SPGG_OK;
}

int spgg_bind(spgg_ctx* c, const spgg_buffers* b) {
  if (!c || !b) return fail(c, SPGG_E_ARG, "null argument");
  for (int i = 0; i < 2; ++i)
    if (!b->S[i] || !b->R[i] || !b->pub[i])
      return fail(c, SPGG_E_ARG, "spgg_bind: an S / R / border-record buffer is null");
  if (!b->Q || !b->md || !b->atd || !b->eps || !b->stats || !b->stop_iter)
    return fail(c, SPGG_E_ARG, "spgg_bind: a required buffer is null");
  if (c->cfg.rng_mode != SPGG_RNG_PHILOX &&
      (!b->draws || b->draw_slot_stride < (int64_t)c->cfg.n_rep * c->draw_words))
    return fail(c, SPGG_E_ARG, "spgg_bind: draw records (spgg_draw_layout slots, stride >= n_rep*words) required "
                               "for INJECT/MT19937");
  if (c->cfg.rng_mode == SPGG_RNG_MT19937 &&
      (!b->mt_state || !b->mt_snap || b->mt_snap_stride < (int64_t)c->cfg.n_rep * 625))
    return fail(c, SPGG_E_ARG, "spgg_bind: mt_state and mt_snap (stride >= n_rep*625) required for MT19937");
  if ((reinterpret_cast<uintptr_t>(b->Q) & 15) != 0)
    return fail(c, SPGG_E_ARG, "spgg_bind: the Q buffer must be 16-byte aligned");
  c->buf = *b;
  c->bound = true;
  return SPGG_OK;
}

// spgg_step's argument and state checks (no side effects: spgg_step_groups checks every
// context before it enqueues anything).
static int step_check(spgg_ctx* c, int32_t t0, int32_t n_steps) {
  if (!c) return SPGG_E_ARG;
  if (!c->bound || !c->params_set) return fail(c, SPGG_E_STATE, "spgg_step before bind/set_params");
  if (t0 < 1 || n_steps < 0 || (long long)t0 + n_steps - 1 > c->cfg.iterations)
    return fail(c, SPGG_E_ARG, "spgg_step: iteration range outside [1, iterations]");
  if (c->cfg.rng_mode == SPGG_RNG_INJECT && n_steps > 1)
    return fail(c, SPGG_E_ARG, "spgg_step: INJECT mode steps one iteration per call");
  if (t0 != 1 && c->params_moved)
    return fail(c, SPGG_E_STATE, "spgg_step: replica parameters changed mid-run (spgg_set_params after "
                                 "iteration 1: e.g. a kappa woken from 0 has no pending NI record)");
  return SPGG_OK;
}

// Run setup of a checked spgg_step call: the iteration-1 prologue and the generator's start.
// The fallible setup a step needs (allocations, the generator's jump polynomials), idempotent.
static int step_setup(spgg_ctx* c) {
  int rc = SPGG_OK;
  if (c->cfg.rng_mode == SPGG_RNG_MT19937) rc = mt_lazy_init(c);
  if (!rc && c->persist) rc = persist_lazy_init(c);
  return rc;
}

static int step_begin(spgg_ctx* c, int32_t t0, int32_t n_steps, hipStream_t s) {
  if (t0 == 1) c->params_moved = false;  // a new run
  const bool mt = c->cfg.rng_mode == SPGG_RNG_MT19937;
  int rc = step_setup(c);
  if (rc) return rc;
  if (mt && t0 == 1) c->gen_upto = 0;  // a new run: generation restarts from mt_state
  if (t0 == 1 && n_steps > 0) launch_step(c, 0, 0, s);  // iteration-1 prologue
  if (mt && n_steps > 0 && c->gen_upto == 0) {
    // a run's first generator chunks read mt_state, eps and stop_iter and write the draw and
    // snapshot rings, which the caller may have just written on its own stream (e.g. torch's
    // zero fills): the generator's stream waits for it (later chunks wait for the steps)
    (void)hipEventRecord(c->caller_ready, s);
    (void)hipStreamWaitEvent(c->gen_stream, c->caller_ready, 0);
  }
  return SPGG_OK;
}

// The last iteration of the segment of a spgg_step call that starts at t (the call ends before
// end): a persistent context runs to the call's end -- MT19937: to the end of the generator chunk
// holding t, whose generation the segment's launch waits for -- in one launch; otherwise the
// segment is iteration t alone.
static int seg_end(const spgg_ctx* c, int t, int end) {
  if (!c->persist) return t;
  int t1 = end - 1;
  if (c->cfg.rng_mode == SPGG_RNG_MT19937) t1 = std::min(t1, ((t - 1) / c->gen_chunk + 1) * c->gen_chunk);
  return t1;
}

// Iterations t .. t1 of a spgg_step call that began at t0: their generator chunks (MT19937) and
// the step launch(es) -- one per iteration, or one persistent launch.
static void step_seg(spgg_ctx* c, int t, int t1, int32_t t0, hipStream_t s) {
  const bool mt = c->cfg.rng_mode == SPGG_RNG_MT19937;
  const int K = c->gen_chunk, T = c->cfg.iterations;
  // timing-only builds (-DSPGG_TIMING=1: the step launches skipped, the generator alone; =2: the
  // generator launches skipped, steps on stale draws; results are WRONG); 0 in the product
  constexpr int timing = SPGG_TIMING;
  if (mt) {
    const int q = (t - 1) / K;
    // this chunk and the next one enqueued (the next overlaps this chunk's steps)
    while (timing != 2 && c->gen_upto < std::min(T, (q + 2) * K)) enqueue_gen_chunk(c, c->gen_upto / K);
    if (timing != 2 && (t == q * K + 1 || t == t0)) (void)hipStreamWaitEvent(s, c->gen_done[q & 1], 0);
  }
  if (timing != 1) {
    if (t1 > t) launch_persist(c, t, t1, s);
    else launch_step(c, t, 0, s);
  }
  if (mt && (t1 % K == 0 || t1 == T)) (void)hipEventRecord(c->step_done[((t1 - 1) / K) & 1], s);
}

int spgg_step(spgg_ctx* c, int32_t t0, int32_t n_steps, void* stream) {
  int rc = step_check(c, t0, n_steps);
  if (rc) return rc;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if ((rc = step_begin(c, t0, n_steps, s))) return rc;
  const int end = t0 + n_steps;
  for (int t = t0; t < end;) {
    const int t1 = seg_end(c, t, end);
    step_seg(c, t, t1, t0, s);
    t = t1 + 1;
  }
  return hip_check(c, hipGetLastError(), "spgg_step launch");
}

int spgg_step_groups(spgg_ctx* const* ctxs, void* const* streams, int32_t n_ctx, int32_t t0, int32_t n_steps) {
  if (!ctxs || !streams || n_ctx < 1) return SPGG_E_ARG;
  for (int i = 0; i < n_ctx; ++i) {
    if (!ctxs[i]) return SPGG_E_ARG;
    for (int j = 0; j < i; ++j)
      if (ctxs[j] == ctxs[i]) return fail(ctxs[i], SPGG_E_ARG, "spgg_step_groups: a context listed twice");
    if (ctxs[i]->cfg.rng_mode == SPGG_RNG_INJECT)
      return fail(ctxs[i], SPGG_E_ARG, "spgg_step_groups: INJECT mode steps through spgg_step");
    int rc = step_check(ctxs[i], t0, n_steps);
    // the fallible part of step_begin (the generator's lazy setup: allocations, the jump
    // polynomials) runs here too, so that nothing is enqueued on any context unless every one
    // of them can start; a failure is reported on that context and on ctxs[0], which callers read
    if (!rc) rc = step_setup(ctxs[i]);
    if (rc) {
      if (i > 0) fail(ctxs[0], rc, "spgg_step_groups: context " + std::to_string(i) + ": " + ctxs[i]->err);
      return rc;
    }
  }
  for (int i = 0; i < n_ctx; ++i) {
    int rc = step_begin(ctxs[i], t0, n_steps, reinterpret_cast<hipStream_t>(streams[i]));
    if (rc) return rc;  // (cannot fail: step_setup above already succeeded)
  }
  // segments of context 0 (every context of one batch has the same layout, generator chunk and
  // persistent decision -- all decided from the whole batch); one iteration at a time otherwise
  bool same = true;
  for (int i = 1; i < n_ctx; ++i)
    same &= ctxs[i]->persist == ctxs[0]->persist && ctxs[i]->gen_chunk == ctxs[0]->gen_chunk &&
            ctxs[i]->cfg.rng_mode == ctxs[0]->cfg.rng_mode;
  const int end = t0 + n_steps;
  for (int t = t0; t < end;) {
    int t1 = same ? seg_end(ctxs[0], t, end) : t;
    for (int i = 0; i < n_ctx; ++i)
      step_seg(ctxs[i], t, ctxs[i]->persist ? t1 : t, t0, reinterpret_cast<hipStream_t>(streams[i]));
    t = t1 + 1;
  }
  const int rc = hip_check(ctxs[0], hipGetLastError(), "spgg_step_groups launch");
  for (int i = 1; i < n_ctx && rc; ++i) ctxs[i]->err = ctxs[0]->err;
  return rc;
}

int spgg_flush(spgg_ctx* c, int32_t t_last, void* stream) {
  if (!c) return SPGG_E_ARG;
  if (!c->bound || !c->params_set) return fail(c, SPGG_E_STATE, "spgg_flush before bind/set_params");
  if (t_last < 1 || t_last > c->cfg.iterations) return fail(c, SPGG_E_ARG, "spgg_flush: bad t_last");
  if (c->params_moved)  // the NI term would read a pending record that was never written
    return fail(c, SPGG_E_STATE, "spgg_flush: replica parameters changed mid-run (e.g. a kappa woken "
                                 "from 0 has no pending NI record)");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (c->cfg.rng_mode == SPGG_RNG_MT19937 && c->gen_done[0]) {
    // the generator ran ahead: wait for it, then restore each replica's key to the one the
    // reference holds (after its last executed iteration) from the snapshot ring
    (void)hipMemcpyAsync((void*)c->h_err, c->d_err, 4, hipMemcpyDeviceToHost, c->gen_stream);
    (void)hipEventRecord(c->gen_idle, c->gen_stream);
    (void)hipStreamWaitEvent(s, c->gen_idle, 0);
    c->gen_upto = 0;
    // every chunk of the run has been generated once the generator's stream drains: a wait
    // that exhausted its bound there means wrong draws, reported instead of a silent result
    int rc = hip_check(c, hipEventSynchronize(c->gen_idle), "spgg_flush: generator");
    if (rc) return rc;
    if (*c->h_err)
      return fail(c, SPGG_E_STATE, "spgg_flush: the MT19937 draw generator failed (error word " +
                                       std::to_string(*c->h_err) + "): a wait between its waves ran out of "
                                       "its bound, so this run's draws are not the reference's");
    hipLaunchKernelGGL(spgg_mt_final_kernel, dim3(c->cfg.n_rep), dim3(256), 0, s, gen_args(c), t_last);
  }
  launch_step(c, t_last + 1, 1, s);
  return hip_check(c, hipGetLastError(), "spgg_flush launch");
}

int spgg_history_finalize(spgg_ctx* c, int32_t t_last, void* stream) {
  if (!c) return SPGG_E_ARG;
  if (!c->bound || !c->params_set) return fail(c, SPGG_E_STATE, "spgg_history_finalize before bind/set_params");
  if (t_last < 0 || t_last > c->cfg.iterations) return fail(c, SPGG_E_ARG, "spgg_history_finalize: bad t_last");
  const int slots = c->cfg.iterations + 2;
  const dim3 grid((slots + kBlock - 1) / kBlock, c->cfg.n_rep);
  hipLaunchKernelGGL(spgg_history_finalize_kernel, grid, dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream),
                     c->buf.stats, c->buf.stop_iter, c->d_params, c->n, slots, c->stripes, t_last);
  return hip_check(c, hipGetLastError(), "spgg_history_finalize launch");
}

int spgg_draw(spgg_ctx* c, int32_t t, void* stream) { return spgg_draw_range(c, t, t, stream); }

int spgg_draw_range(spgg_ctx* c, int32_t t0, int32_t t1, void* stream) {
  if (!c) return SPGG_E_ARG;
  if (!c->bound || c->cfg.rng_mode != SPGG_RNG_MT19937)
    return fail(c, SPGG_E_STATE, "spgg_draw needs a bound MT19937 context");
  if (t0 < 1 || t1 < t0 || t1 > c->cfg.iterations || t1 - t0 + 1 > c->gen_chunk ||
      (long long)(t1 - t0 + 2) * draw_mt_words(c->n, draw_planes(c->cfg.algorithm)) >= (1LL << 31))
    return fail(c, SPGG_E_ARG, "spgg_draw_range: 1 <= t0 <= t1 <= iterations, t1 - t0 < gen chunk, < 2^31 words");
  const int rc = mt_lazy_init(c);  // (the error word)
  if (rc) return rc;
  launch_gen(c, t0, t1, 0, reinterpret_cast<hipStream_t>(stream));
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

int spgg_status(const spgg_ctx* c, uint32_t* flags) {
  if (!c || !flags) return SPGG_E_ARG;
  *flags = c->h_err ? *c->h_err : 0u;
  return SPGG_OK;
}

int spgg_test_set_error(spgg_ctx* c, uint32_t flags) {
  if (!c) return SPGG_E_ARG;
  if (c->cfg.rng_mode != SPGG_RNG_MT19937) return fail(c, SPGG_E_STATE, "spgg_test_set_error: MT19937 only");
  int rc = hip_check(c, hipSetDevice(c->cfg.device), "hipSetDevice");
  if (!rc) rc = mt_lazy_init(c);
  if (rc) return rc;
  hipLaunchKernelGGL(spgg_set_err_kernel, dim3(1), dim3(64), 0, c->gen_stream, c->d_err, flags);
  return hip_check(c, hipGetLastError(), "spgg_test_set_error launch");
}

int spgg_pub_doubles(const spgg_ctx* c, int64_t* per_rep) {
  if (!c || !per_rep) return SPGG_E_ARG;
  *per_rep = (int64_t)c->tiles_per_rep * spgg_impl::pf_of(c->cfg.algorithm) * c->PB;
  return SPGG_OK;
}

int spgg_stat_stripes(const spgg_ctx* c, int32_t* stripes) {
  if (!c || !stripes) return SPGG_E_ARG;
  *stripes = c->stripes;
  return SPGG_OK;
}

int spgg_persistent(const spgg_ctx* c, int32_t* on, int32_t* capacity) {
  if (!c || !on || !capacity) return SPGG_E_ARG;
  *on = c->persist ? 1 : 0;
  *capacity = c->persist_capacity;
  return SPGG_OK;
}

int spgg_tile_shape(const spgg_ctx* c, int32_t* tw, int32_t* th) {
  if (!c || !tw || !th) return SPGG_E_ARG;
  *tw = c->TW;
  *th = c->TH;
  return SPGG_OK;
}

int spgg_draw_layout(const spgg_ctx* c, int32_t* slots, int64_t* words_per_rep, int32_t* snap_slots) {
  if (!c || !slots || !words_per_rep || !snap_slots) return SPGG_E_ARG;
  *slots = c->draw_slots;
  *words_per_rep = c->draw_words;
  *snap_slots = c->snap_slots;
  return SPGG_OK;
}

int spgg_mt_chains(const spgg_ctx* c, int32_t* chains, int32_t* per_chain) {
  if (!c || !chains || !per_chain) return SPGG_E_ARG;
  const bool mt = c->cfg.rng_mode == SPGG_RNG_MT19937;
  *chains = mt ? c->chains : 1;
  *per_chain = mt ? c->per_chain : 1;
  return SPGG_OK;
}

int spgg_stream_create(int32_t device, void** stream) {
  if (!stream) return SPGG_E_ARG;
  *stream = nullptr;
  if (hipSetDevice(device) != hipSuccess) return SPGG_E_HIP;
  hipStream_t s = nullptr;
  if (make_stream(&s, false) != hipSuccess) return SPGG_E_HIP;
  *stream = s;
  return SPGG_OK;
}

int spgg_stream_destroy(void* stream) {
  if (!stream) return SPGG_E_ARG;
  return hipStreamDestroy(reinterpret_cast<hipStream_t>(stream)) == hipSuccess ? SPGG_OK : SPGG_E_HIP;
}

int spgg_set_draw_stream(spgg_ctx* c, void* stream) {
  if (!c) return SPGG_E_ARG;
  if (c->cfg.rng_mode != SPGG_RNG_MT19937) return fail(c, SPGG_E_STATE, "spgg_set_draw_stream: MT19937 only");
  if (c->gen_done[0] || c->gen_stream) return fail(c, SPGG_E_STATE, "spgg_set_draw_stream: set it before spgg_step");
  c->gen_stream = reinterpret_cast<hipStream_t>(stream);
  c->own_gen_stream = false;
  return SPGG_OK;
}

int spgg_destroy(spgg_ctx* c) {
  if (!c) return SPGG_OK;
  if (c->d_params || c->d_ring || c->gen_stream || c->gen_done[0] || c->d_err || c->d_bar) {
    (void)hipSetDevice(c->cfg.device);
    if (c->gen_stream) (void)hipStreamSynchronize(c->gen_stream);  // no generator writes after return
    if (c->d_params) (void)hipFree(c->d_params);
    if (c->d_ring) (void)hipFree(c->d_ring);
    for (int i = 0; i < 2; ++i) {
      if (c->gen_done[i]) (void)hipEventDestroy(c->gen_done[i]);
      if (c->step_done[i]) (void)hipEventDestroy(c->step_done[i]);
    }
    if (c->gen_idle) (void)hipEventDestroy(c->gen_idle);
    if (c->caller_ready) (void)hipEventDestroy(c->caller_ready);
    if (c->d_err) (void)hipFree(c->d_err);
    if (c->h_err) (void)hipHostFree((void*)c->h_err);
    for (int i = 0; i < 2; ++i) {
      if (c->d_parts[i]) (void)hipFree(c->d_parts[i]);
      if (c->d_keybuf[i]) (void)hipFree(c->d_keybuf[i]);
    }
    if (c->d_run_pos0) (void)hipFree(c->d_run_pos0);
    if (c->d_bar) (void)hipFree(c->d_bar);
    if (c->d_polys) (void)hipFree(c->d_polys);
    if (c->own_gen_stream) (void)hipStreamDestroy(c->gen_stream);
  }
  delete c;
  return SPGG_OK;
}

}  // extern "C"
#endif  // SPGG_TU_HAS_HOST
