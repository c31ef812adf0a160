// spgg_mt.hip — MT19937 jump-ahead: the characteristic polynomial and x^e mod phi (host),
// chain seeding and the jump kernel (device).  See spgg_mt.h.
//
// The jump is a GF(2) correlation: window(B+D)[j] = XOR over the set coefficients i of
// g = x^(D-1) mod phi of x[B+1+i+j], j < 624 -- ~10^4 set coefficients x 624 words.  A
// jump is spread over kSplits workgroups, one range of coefficients each: every workgroup
// regenerates the stream words its range touches (one wave, 227-word dependency blocks in
// an LDS ring), then XORs shifted copies of them from LDS (three output words per thread),
// and writes its part; the consumer XORs the kSplits parts.
#include "spgg_mt.h"

#include <cstring>
#include <map>
#include <mutex>
#include <vector>

namespace spgg_mt {

// ---------------------------------------------------------------------------------------
// Host: GF(2) polynomials, bit i of word i/64 = coefficient of x^i.
namespace {

constexpr int kPW = (kDeg + 1 + 63) / 64;  // 312 words hold degree <= 19967

using Poly = std::vector<uint64_t>;

inline int bit_of(const uint64_t* p, int i) { return (int)((p[i >> 6] >> (i & 63)) & 1u); }

// p ^= q << sh   (q has nq words; p must hold them)
inline void xor_shifted(uint64_t* p, const uint64_t* q, int nq, int sh) {
  const int w = sh >> 6, b = sh & 63;
  if (b == 0) {
    for (int i = 0; i < nq; ++i) p[w + i] ^= q[i];
  } else {
    for (int i = 0; i < nq; ++i) {
      p[w + i] ^= q[i] << b;
      p[w + i + 1] ^= q[i] >> (64 - b);
    }
  }
}

// MT19937's characteristic polynomial by Berlekamp-Massey on bit 0 of the raw
// (untempered) words of init_genrand(5489)'s stream: the sequence's minimal polynomial,
// which is phi itself when its degree is 19937 (phi is irreducible).  Empty on failure.
Poly derive_phi() {
  constexpr int N = 2 * kDeg + 64;  // bits of the sequence
  std::vector<uint32_t> x(N + 2 + kKey);
  x[0] = 5489u;
  for (int i = 1; i < kKey; ++i) x[i] = 1812433253u * (x[i - 1] ^ (x[i - 1] >> 30)) + (uint32_t)i;
  for (size_t k = kKey; k < x.size(); ++k) x[k] = mt_next(x[k - 227], x[k - kKey], x[k - kKey + 1]);
  // s[n] = bit 0 of x[n + 1]; u = s reversed (u[k] = s[N-1-k]), packed with slack words
  const int NW = N / 64 + 4;  // C, B hold 2*NW words: x^m B (m <= N) never leaves them
  std::vector<uint64_t> u(NW, 0), C(2 * NW, 0), B(2 * NW, 0), T;
  std::vector<uint8_t> s(N);
  for (int n = 0; n < N; ++n) {
    s[n] = (uint8_t)(x[n + 1] & 1u);
    if (s[n]) u[(N - 1 - n) >> 6] |= 1ull << ((N - 1 - n) & 63);
  }
  C[0] = B[0] = 1;
  int L = 0, m = 1;
  for (int n = 0; n < N; ++n) {
    // d = sum_{i=0..L} C_i s[n-i] = sum_i C_i u[N-1-n+i]
    const int off = N - 1 - n;
    uint64_t acc = 0;
    for (int w = 0; w <= L / 64; ++w) {
      const int pos = off + 64 * w, pw = pos >> 6, sh = pos & 63;
      const uint64_t uw = sh ? (u[pw] >> sh) | (u[pw + 1] << (64 - sh)) : u[pw];
      acc ^= C[w] & uw;
    }
    const int d = __builtin_popcountll(acc) & 1;
    if (!d) {
      ++m;
    } else if (2 * L <= n) {
      T = C;
      xor_shifted(C.data(), B.data(), NW, m);  // C += x^m B
      L = n + 1 - L;
      B.swap(T);
      m = 1;
    } else {
      xor_shifted(C.data(), B.data(), NW, m);
      ++m;
    }
  }
  if (L != kDeg) return Poly();
  Poly phi(kPW, 0);  // phi_k = C_{L-k}
  for (int k = 0; k <= L; ++k)
    if (bit_of(C.data(), L - k)) phi[k >> 6] |= 1ull << (k & 63);
  return phi;
}

// (heap objects never freed: spgg_create's prefetch thread may still run at process exit)
const Poly& phi() {
  static const Poly* p = new Poly(derive_phi());
  return *p;
}

// Reduction table: T[v] (v < 256) = the multiple m * phi (deg m < 8) whose coefficients at
// degrees kDeg .. kDeg+7 are the bits of v and whose other coefficients lie below kDeg:
// XOR-ing T[v] << s clears the eight coefficients kDeg+s .. kDeg+s+7 of a product at once
// (a bit at a time took ~35 ms per exponentiation)
constexpr int kTW = kPW + 1;  // words of a table entry (degree <= kDeg + 7)
const std::vector<uint64_t>& red_table() {
  static const std::vector<uint64_t>* T = new std::vector<uint64_t>([] {
    const Poly& f = phi();
    std::vector<uint64_t> t(256 * kTW, 0);
    // single bits first: phi << i, its coefficients kDeg .. kDeg+i-1 cleared with lower bits
    for (int i = 0; i < 8; ++i) {
      uint64_t* e = t.data() + (size_t)(1 << i) * kTW;
      xor_shifted(e, f.data(), kPW, i);
      for (int j = i - 1; j >= 0; --j)
        if (bit_of(e, kDeg + j))
          for (int w = 0; w < kTW; ++w) e[w] ^= t[(size_t)(1 << j) * kTW + w];
    }
    for (int v = 1; v < 256; ++v) {  // linear: T[v] = XOR of its single-bit entries
      if ((v & (v - 1)) == 0) continue;
      const int lo = v & -v;
      for (int w = 0; w < kTW; ++w) t[(size_t)v * kTW + w] = t[(size_t)lo * kTW + w] ^ t[(size_t)(v ^ lo) * kTW + w];
    }
    return t;
  }());
  return *T;
}

// (phi, ~30 ms of Berlekamp-Massey, and the reduction table are built by the first jump_poly
// call: spgg_create's prefetch thread of an MT19937 context with chains, so no thread starts
// when the library loads -- a fork() while one held these statics' guards would leave the child
// blocked on its first jump)

// q (degree <= 2 (kDeg - 1), 2 kPW + 2 words) mod phi, eight coefficients at a time from the top
void reduce_mod(std::vector<uint64_t>& q) {
  const std::vector<uint64_t>& T = red_table();
  for (int s = 2 * (kDeg - 1) - kDeg - 7; s > -8; s -= 8) {
    const int lo = s < 0 ? 0 : s;               // (the last chunk is narrower)
    const int d = kDeg + lo, nb = s < 0 ? 8 + s : 8;
    uint32_t v = 0;
    for (int b = 0; b < nb; ++b) v |= (uint32_t)bit_of(q.data(), d + b) << b;
    if (v) xor_shifted(q.data(), T.data() + (size_t)v * kTW, kTW, lo);
  }
}

// p (degree < 19937) squared mod phi
void sqr_mod(Poly& p) {
  std::vector<uint64_t> q(2 * kPW + 2, 0);
  for (int w = 0; w < kPW; ++w) {
    uint64_t lo = 0, hi = 0;
    const uint64_t v = p[w];
    for (int b = 0; b < 32; ++b) {
      lo |= ((v >> b) & 1ull) << (2 * b);
      hi |= ((v >> (b + 32)) & 1ull) << (2 * b);
    }
    q[2 * w] = lo;
    q[2 * w + 1] = hi;
  }
  reduce_mod(q);
  for (int w = 0; w < kPW; ++w) p[w] = q[w];
}

// p * x mod phi
void mulx_mod(Poly& p) {
  uint64_t carry = 0;
  for (int w = 0; w < kPW; ++w) {
    const uint64_t v = p[w];
    p[w] = (v << 1) | carry;
    carry = v >> 63;
  }
  if (bit_of(p.data(), kDeg))
    for (int w = 0; w < kPW; ++w) p[w] ^= phi()[w];
}

// x^e mod phi (square and multiply from the top bit)
Poly pow_x(uint64_t e) {
  Poly p(kPW, 0);
  p[0] = 1;
  for (int b = 63; b >= 0; --b) {
    sqr_mod(p);
    if ((e >> b) & 1u) mulx_mod(p);
  }
  return p;
}

}  // namespace

void jump_poly(uint64_t e, uint32_t* out) {
  // (never destroyed: a prefetching thread, spgg_create's, may still hold them at process exit)
  static std::mutex* mu_p = new std::mutex;
  static std::map<uint64_t, Poly>* cache_p = new std::map<uint64_t, Poly>;
  std::mutex& mu = *mu_p;
  std::map<uint64_t, Poly>& cache = *cache_p;
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(e);
  if (it == cache.end()) {
    if (phi().empty()) {  // cannot happen for MT19937; the caller checks for an all-zero g
      std::memset(out, 0, kKey * sizeof(uint32_t));
      return;
    }
    // the generator's jump levels are e_{j+1} = 2 e_j + 1 (jumps of D << j words, minus one):
    // x^(2e+1) = (x^e)^2 x mod phi, one squaring instead of a whole exponentiation (~35 ms each)
    auto half = (e & 1u) ? cache.find(e >> 1) : cache.end();
    if (half != cache.end()) {
      Poly p = half->second;
      sqr_mod(p);
      mulx_mod(p);
      it = cache.emplace(e, std::move(p)).first;
    } else {
      it = cache.emplace(e, pow_x(e)).first;
    }
  }
  std::memcpy(out, it->second.data(), kKey * sizeof(uint32_t));  // 312 u64 = 624 u32 (little endian)
}

// ---------------------------------------------------------------------------------------
// Device
namespace {

constexpr int kThreads = 256;
constexpr int kBlk = 227;                                        // words one dependency step yields
constexpr int kRingW = 1024;                                     // recurrence ring (> 624 + 227)
constexpr int kSpan = ((kDeg + kSplits - 1) / kSplits + 31) / 32 * 32;  // coefficients per split
constexpr int kCap = kSpan + 3 * kThreads;                       // captured words (+ slack lanes)

__global__ __launch_bounds__(kThreads) void mt_seed_kernel(const uint32_t* mt_state, uint32_t* run_pos0,
                                                          uint32_t* parts, int chains) {
  __shared__ uint32_t X[2 * kKey];
  const int rep = blockIdx.x, tid = threadIdx.x;
  const uint32_t* key = mt_state + (size_t)rep * (kKey + 1);
  for (int i = tid; i < kKey; i += kThreads) X[i] = key[i];
  const int P = (int)min(key[kKey], (uint32_t)kKey);  // 0..624: next word to draw
  if (tid == 0) run_pos0[rep] = (uint32_t)P;
  __syncthreads();
  for (int f = 0; f < P; f += kBlk) {  // X[624 + m], m < P, in dependency blocks
    for (int m = f + tid; m < min(f + kBlk, P); m += kThreads) X[kKey + m] = mt_next(X[m + 397], X[m], X[m + 1]);
    __syncthreads();
  }
  for (int c = 0; c < chains; ++c) {
    uint32_t* o = parts + (size_t)(rep * chains + c) * kSplits * kKey;
    for (int i = tid; i < kSplits * kKey; i += kThreads) o[i] = i < kKey ? X[P + i] : 0u;
  }
}

__global__ __launch_bounds__(kThreads) void mt_jump_kernel(const uint32_t* in, uint32_t* out, const uint32_t* poly,
                                                          int chains, int bit, const int* stop_iter) {
  __shared__ uint32_t ring[kRingW];
  __shared__ uint32_t cap[kCap];  // cap[u] = X[1 + i0 + u]
  const int tid = threadIdx.x;
  const int s = blockIdx.x % kSplits, cc = (blockIdx.x / kSplits) % chains, rep = blockIdx.x / (kSplits * chains);
  if (bit < 0 && cc == 0) return;
  if (stop_iter && stop_iter[rep] != 0) return;
  const size_t base = (size_t)(rep * chains + cc) * kSplits * kKey;
  uint32_t* o = out + base + (size_t)s * kKey;
  if (bit >= 0 && !((cc >> bit) & 1)) {  // not jumped this round: carried over
    for (int j = tid; j < kKey; j += kThreads) o[j] = in[base + (size_t)s * kKey + j];
    return;
  }
  for (int j = tid; j < kKey; j += kThreads) {
    uint32_t v = 0;
#pragma unroll
    for (int p = 0; p < kSplits; ++p) v ^= in[base + (size_t)p * kKey + j];
    ring[j] = v;  // X[j] = x[B + j]
  }
  const int i0 = s * kSpan, i1 = min(kDeg, i0 + kSpan);
  const int ncap = i1 - i0 + kKey - 1;  // X[1 + i0 .. i1 + 623]
  __syncthreads();
  for (int u = tid; u < ncap; u += kThreads)
    if (1 + i0 + u < kKey) cap[u] = ring[1 + i0 + u];
  // the copy above reads ring[1 .. 623]; the extension below overwrites those words once it
  // wraps (m >= kRingW), so every wave's copy must be done first
  __syncthreads();
  if (tid < 64) {  // one wave extends the stream: its LDS accesses complete in order
    const int lane = tid, mmax = i1 + kKey - 1;
    for (int F = kKey; F <= mmax; F += kBlk) {
      uint32_t v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = F + lane + 64 * q;
        v[q] = mt_next(ring[(m - 227) & (kRingW - 1)], ring[(m - kKey) & (kRingW - 1)],
                       ring[(m - kKey + 1) & (kRingW - 1)]);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = F + lane + 64 * q, u = m - 1 - i0;
        if (lane + 64 * q < kBlk) {
          ring[m & (kRingW - 1)] = v[q];
          if (u >= 0 && u < ncap) cap[u] = v[q];
        }
      }
    }
  }
  __syncthreads();
  // out[j] = XOR_{i in [i0, i1), g_i} X[1 + i + j] = cap[i - i0 + j], j = tid, tid+256, tid+512
  uint32_t a0 = 0, a1 = 0, a2 = 0;
  for (int w = i0 / 32; w < (i1 + 31) / 32; ++w) {
    uint32_t bits = poly[w];
    if (32 * w + 32 > i1) bits &= (1u << (i1 - 32 * w)) - 1u;
    while (bits) {
      const int u = 32 * w + __builtin_ctz(bits) - i0 + tid;
      bits &= bits - 1u;
      a0 ^= cap[u];
      a1 ^= cap[u + kThreads];
      a2 ^= cap[u + 2 * kThreads];  // (threads past 624 - 512 read slack, discarded)
    }
  }
  o[tid] = a0;
  o[tid + kThreads] = a1;
  if (tid + 2 * kThreads < kKey) o[tid + 2 * kThreads] = a2;
}

}  // namespace

void launch_seed(const uint32_t* mt_state, uint32_t* run_pos0, uint32_t* parts, int n_rep, int chains,
                 hipStream_t s) {
  hipLaunchKernelGGL(mt_seed_kernel, dim3(n_rep), dim3(kThreads), 0, s, mt_state, run_pos0, parts, chains);
}

void launch_jump(const uint32_t* parts_in, uint32_t* parts_out, const uint32_t* poly, int n_rep, int chains,
                 int bit, const int* stop_iter, hipStream_t s) {
  hipLaunchKernelGGL(mt_jump_kernel, dim3(n_rep * chains * kSplits), dim3(kThreads), 0, s, parts_in, parts_out,
                     poly, chains, bit, stop_iter);
}

}  // namespace spgg_mt

// Test hook (spgg_abi.h): g = x^e mod phi
extern "C" int spgg_mt_jump_poly(int64_t e, uint32_t* out) {
  if (e < 0 || !out) return -1;
  spgg_mt::jump_poly((uint64_t)e, out);
  for (int i = 0; i < spgg_mt::kKey; ++i)
    if (out[i]) return 0;
  return -5;  // SPGG_E_STATE: no characteristic polynomial
}
