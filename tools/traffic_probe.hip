// Memory-only probe with the step kernel's tiling and per-agent traffic:
// stage S/R halos in LDS, read Q/md/atd of owned + ring agents, write
// Q/md/atd/S/R of owned agents.  No simulation compute.  Timing tool only.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
constexpr int kBlock = 256;
__device__ __forceinline__ int wrap1(int x, int L) { x += x < 0 ? L : 0; x -= x >= L ? L : 0; return x; }

template <int APT>
__device__ __forceinline__ void probe_tile(int logical,const uint8_t* S_in, uint8_t* S_out, const int8_t* R_in, int8_t* R_out,
                                                const double* Q_in, double* Q_out, const double* md_in, double* md_out,
                                                float* atd, int L, int TW, int TH, int tiles_x, int tiles_per_rep,
                                                int n_rep, int mode) {
  __shared__ uint8_t sS[64 * 40];
  __shared__ int8_t sR[64 * 40];
  const int total = n_rep * tiles_per_rep;
  if (logical >= total) return;
  const int rep = logical / tiles_per_rep, tile = logical % tiles_per_rep;
  const int y0 = (tile / tiles_x) * TH, x0 = (tile % tiles_x) * TW;
  const int th = min(TH, L - y0), tw = min(TW, L - x0);
  const size_t n = (size_t)L * L, rb = rep * n;
  const int tid = threadIdx.x;
  double q[APT][4], md[APT];
  float at[APT];
  int g[APT];
#pragma unroll
  for (int u = 0; u < APT; ++u) {
    const int k = tid + u * kBlock;
    g[u] = -1;
    if (k < th * tw) {
      g[u] = (y0 + k / tw) * L + x0 + k % tw;
      const double2* qp = reinterpret_cast<const double2*>(Q_in + (rb + g[u]) * 4);
      const double2 a = qp[0], b = qp[1];
      q[u][0] = a.x; q[u][1] = a.y; q[u][2] = b.x; q[u][3] = b.y;
      md[u] = md_in[rb + g[u]];
      at[u] = atd[rb + g[u]];
    }
  }
  // ring (M=1): 2*(tw+2+th) agents
  const int ring = 2 * (tw + 2 + th);
  double rq = 0.0;
  if (tid < ring) {
    const int ay = tid < tw + 2 ? -1 : (tid < 2 * (tw + 2) ? th : (tid - 2 * (tw + 2)) / 2);
    const int ax = tid < 2 * (tw + 2) ? (tid % (tw + 2)) - 1 : ((tid & 1) ? tw : -1);
    const int gg = wrap1(y0 + ay, L) * L + wrap1(x0 + ax, L);
    const double2* qp = reinterpret_cast<const double2*>(Q_in + (rb + gg) * 4);
    const double2 a = qp[0], b = qp[1];
    rq = a.x + a.y + b.x + b.y + md_in[rb + gg];
  }
  const int sw = tw + 6, sh = th + 6, rw = tw + 4, rh = th + 4;
  for (int k = tid; k < sh * sw; k += kBlock) sS[k] = S_in[rb + wrap1(y0 - 3 + k / sw, L) * L + wrap1(x0 - 3 + k % sw, L)];
  for (int k = tid; k < rh * rw; k += kBlock) sR[k] = R_in[rb + wrap1(y0 - 2 + k / rw, L) * L + wrap1(x0 - 2 + k % rw, L)];
  __syncthreads();
  if (mode & 1) {  // no stores: keep the loads alive
    double acc = rq;
#pragma unroll
    for (int u = 0; u < APT; ++u) if (g[u] >= 0) acc += q[u][0] + q[u][1] + q[u][2] + q[u][3] + md[u] + at[u];
    if (acc == 12345.678) md_out[0] = acc;
    return;
  }
#pragma unroll
  for (int u = 0; u < APT; ++u) {
    if (g[u] < 0) continue;
    const int k = tid + u * kBlock, r = k / tw, c = k % tw;
    const uint8_t s = sS[(r + 3) * sw + c + 3];
    const int8_t rr = sR[(r + 2) * rw + c + 2];
    double2* qo = reinterpret_cast<double2*>(Q_out + (rb + g[u]) * 4);
    qo[0] = make_double2(q[u][0] + rq, q[u][1]);
    qo[1] = make_double2(q[u][2], q[u][3] + md[u]);
    md_out[rb + g[u]] = md[u] * 0.5;
    atd[rb + g[u]] = at[u] + 1.f;
    S_out[rb + g[u]] = s ^ 1;
    R_out[rb + g[u]] = rr + 1;
  }
}
template <int APT>
__global__ __launch_bounds__(kBlock) void probe(const uint8_t* S_in, uint8_t* S_out, const int8_t* R_in, int8_t* R_out,
                                                const double* Q_in, double* Q_out, const double* md_in, double* md_out,
                                                float* atd, int L, int TW, int TH, int tiles_x, int tiles_per_rep,
                                                int n_rep, int mode) {
  const int total = n_rep * tiles_per_rep;
  if (mode & 32) {  // persistent: static grid-stride over tiles
    for (int logical = blockIdx.x; logical < total; logical += gridDim.x) {
      probe_tile<APT>(logical, S_in, S_out, R_in, R_out, Q_in, Q_out, md_in, md_out, atd, L, TW, TH, tiles_x,
                      tiles_per_rep, n_rep, mode);
      __syncthreads();
    }
    return;
  }
  const int per_xcd = (total + 7) / 8;
  const int logical = (mode & 4) ? (int)blockIdx.x : (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  probe_tile<APT>(logical, S_in, S_out, R_in, R_out, Q_in, Q_out, md_in, md_out, atd, L, TW, TH, tiles_x,
                  tiles_per_rep, n_rep, mode);
}
}  // namespace

extern "C" int probe_launch(const void* S_in, void* S_out, const void* R_in, void* R_out, const void* Q_in, void* Q_out,
                            const void* md_in, void* md_out, void* atd, int L, int TW, int TH, int n_rep, int mode,
                            void* stream) {
  const int tiles_x = (L + TW - 1) / TW, tiles_per_rep = tiles_x * ((L + TH - 1) / TH);
  const int total = n_rep * tiles_per_rep;
  const size_t nn = (size_t)n_rep * L * L;
  const int grid = (mode & 32) ? ((mode >> 8) ? (mode >> 8) * 256 : 1024)
                 : (mode & 16) ? (int)((nn + 1023) / 1024) : (mode & 8) ? (int)((nn + 255) / 256)
                 : (mode & 2) ? 256 * 8 : (total + 7) / 8 * 8;
  hipLaunchKernelGGL(probe<4>, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream,
                     (const uint8_t*)S_in, (uint8_t*)S_out, (const int8_t*)R_in, (int8_t*)R_out, (const double*)Q_in,
                     (double*)Q_out, (const double*)md_in, (double*)md_out, (float*)atd, L, TW, TH, tiles_x,
                     tiles_per_rep, n_rep, mode);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
