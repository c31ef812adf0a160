// spgg_mt.h — MT19937 jump-ahead for the device draw generator (spgg_kernels.hip).
//
// A replica's draws are one MT19937 stream (numpy RandomState, the reference's global RNG:
// src/model/algorithms.py:105,108, spgg.py:434,452).  Its recurrence is serial per stream, so
// the generator splits the stream into CHAINS: chain c of a generator chunk starts at the
// first word of its own iterations, reached by jumping ahead from an earlier window with
// polynomial arithmetic over GF(2) (spgg_mt.hip).
//
// Window(B) = the 624 words x[B .. B+623] of the stream (x[k+624] = x[k+397] ^
// twist(x[k], x[k+1])).  With g = x^(D-1) mod phi (phi: MT19937's characteristic
// polynomial, degree 19937):  x[B+D+j] = XOR_{i : g_i = 1} x[B+1+i+j]  for every j >= 0,
// since x[B+1+m] = C A^m state(B) for the 19937-bit state of window B.  The low 31 bits of
// x[B] never enter (only its top bit is state), so any window can be jumped.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace spgg_mt {

constexpr int kDeg = 19937;      // degree of phi
constexpr int kKey = 624;        // words of a window / key
constexpr int kSplits = 8;       // workgroups per jump, each a range of g's coefficients

// x[k+624] = x[k+397] ^ twist(x[k], x[k+1]): upper bit of x[k], lower 31 of x[k+1]
__host__ __device__ __forceinline__ uint32_t mt_next(uint32_t far, uint32_t lo_k, uint32_t lo_k1) {
  const uint32_t y = (lo_k & 0x80000000u) | (lo_k1 & 0x7fffffffu);
  return far ^ (y >> 1) ^ ((lo_k1 & 1u) ? 0x9908b0dfu : 0u);
}

// g = x^e mod phi as 624 u32 words (bit i of word i/32 = coefficient of x^i, i < 19937).
// Host; phi is derived once per process (Berlekamp-Massey on the stream), results cached.
void jump_poly(uint64_t e, uint32_t* out);

// Start windows of a run's chains, layout [rep][chain][kSplits][624] (a window is the XOR
// of its kSplits parts):
//   seed: every chain of replica rep gets window(P1) in part 0 (P1 = key[624], the first
//   word iteration 1 draws, relative to the key block mt_state[rep]); run_pos0[rep] = P1.
void launch_seed(const uint32_t* mt_state, uint32_t* run_pos0, uint32_t* parts, int n_rep, int chains,
                 hipStream_t s);
//   jump: window(B) -> window(B+D) with poly = jump_poly(D-1), for chain c iff bit < 0 (then
//   every chain c >= 1; chain 0 is left alone) or bit `bit` of c is set (others are copied).
//   Replicas with stop_iter != 0 (stop_iter may be null) are skipped.
void launch_jump(const uint32_t* parts_in, uint32_t* parts_out, const uint32_t* poly, int n_rep, int chains,
                 int bit, const int* stop_iter, hipStream_t s);

}  // namespace spgg_mt
