// Memory-pattern probe (timing tool only): the step kernel's tiling and
// per-agent traffic with parts switched off by `flags`:
//   1 ring Q/md reads, 2 md/atd traffic, 4 S/R staging + writes, 8 Q in place,
//   16 md/atd packed into a 48-B agent record with Q (needs 2), 32 S/R staged and
//   written as dwords (needs 4; L, TW multiples of 4), 64 tile-blocked layout
//   (each tile's agents contiguous, tile stride 1024 agents; no 16/32)
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
constexpr int kBlock = 256;
__device__ __forceinline__ int wrap1(int x, int L) { x += x < 0 ? L : 0; x -= x >= L ? L : 0; return x; }
// agent (y, x) -> storage index; blocked: tile-major, stride 1024 per tile
__device__ __forceinline__ int sidx(int y, int x, int L, int TW, int TH, int tiles_x, bool blk) {
  if (!blk) return y * L + x;
  const int ty = y / TH, tx = x / TW;
  return (ty * tiles_x + tx) * 1024 + (y - ty * TH) * TW + (x - tx * TW);
}

__global__ __launch_bounds__(kBlock) void pprobe(const uint8_t* S_in, uint8_t* S_out, const int8_t* R_in,
                                                 int8_t* R_out, const double* Q_in, double* Q_out,
                                                 const double* md_in, double* md_out, float* atd, int L, int TW,
                                                 int TH, int tiles_x, int tiles_per_rep, int n_rep, int flags) {
  __shared__ uint8_t sS[64 * 64];
  __shared__ int8_t sR[64 * 64];
  const int total = n_rep * tiles_per_rep;
  const int per_xcd = (total + 7) / 8;
  const int logical = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  if (logical >= total) return;
  const int rep = logical / tiles_per_rep, tile = logical % tiles_per_rep;
  const int y0 = (tile / tiles_x) * TH, x0 = (tile % tiles_x) * TW;
  const int th = min(TH, L - y0), tw = min(TW, L - x0);
  const size_t n = (flags & 64) ? (size_t)tiles_per_rep * 1024 : (size_t)L * L, rb = rep * n;
  const int tid = threadIdx.x;
  if (flags & 8) Q_out = const_cast<double*>(Q_in);
  double q[4][4], md[4];
  float at[4];
  int g[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int k = tid + u * kBlock;
    g[u] = -1;
    md[u] = 0.0;
    at[u] = 0.f;
    if (k < th * tw) {
      g[u] = (flags & 64) ? tile * 1024 + k : (y0 + k / tw) * L + x0 + k % tw;
      const int rs = (flags & 16) ? 6 : 4;
      const double2* qp = reinterpret_cast<const double2*>(Q_in + (rb + g[u]) * rs);
      const double2 a = qp[0], b = qp[1];
      q[u][0] = a.x; q[u][1] = a.y; q[u][2] = b.x; q[u][3] = b.y;
      if (flags & 16) {
        const double2 c = qp[2];
        md[u] = c.x;
        at[u] = (float)c.y;
      } else if (flags & 2) {
        md[u] = md_in[rb + g[u]];
        at[u] = atd[rb + g[u]];
      }
    }
  }
  double rq = 0.0;
  const int ring = 2 * (tw + 2 + th);
  if ((flags & 1) && tid < ring) {
    const int ay = tid < tw + 2 ? -1 : (tid < 2 * (tw + 2) ? th : (tid - 2 * (tw + 2)) / 2);
    const int ax = tid < 2 * (tw + 2) ? (tid % (tw + 2)) - 1 : ((tid & 1) ? tw : -1);
    const int gg = sidx(wrap1(y0 + ay, L), wrap1(x0 + ax, L), L, TW, TH, tiles_x, flags & 64);
    const int rs = (flags & 16) ? 6 : 4;
    const double2* qp = reinterpret_cast<const double2*>(Q_in + (rb + gg) * rs);
    const double2 a = qp[0], b = qp[1];
    rq = a.x + a.y + b.x + b.y + ((flags & 16) ? qp[2].x : (flags & 2) ? md_in[rb + gg] : 0.0);
  }
  const int sw = tw + 6, sh = th + 6, rw = tw + 4, rh = th + 4;
  if ((flags & 36) == 36) {  // dword staging: aligned 4-byte columns [x0-4, x0+tw+4)
    const int cw = (tw + 8) / 4, L4 = L / 4;
    const uint32_t* S4 = reinterpret_cast<const uint32_t*>(S_in + rb);
    const uint32_t* R4 = reinterpret_cast<const uint32_t*>(R_in + rb);
    uint32_t* sS4 = reinterpret_cast<uint32_t*>(sS);
    uint32_t* sR4 = reinterpret_cast<uint32_t*>(sR);
    for (int k = tid; k < (th + 6) * cw; k += kBlock) {
      const int r = k / cw, c = k % cw;
      sS4[k] = S4[wrap1(y0 - 3 + r, L) * L4 + wrap1(x0 / 4 - 1 + c, L4)];
    }
    for (int k = tid; k < (th + 4) * cw; k += kBlock) {
      const int r = k / cw, c = k % cw;
      sR4[k] = R4[wrap1(y0 - 2 + r, L) * L4 + wrap1(x0 / 4 - 1 + c, L4)];
    }
  } else if (flags & 4) {
    const bool blk = flags & 64;
    for (int k = tid; k < sh * sw; k += kBlock)
      sS[k] = S_in[rb + sidx(wrap1(y0 - 3 + k / sw, L), wrap1(x0 - 3 + k % sw, L), L, TW, TH, tiles_x, blk)];
    for (int k = tid; k < rh * rw; k += kBlock)
      sR[k] = R_in[rb + sidx(wrap1(y0 - 2 + k / rw, L), wrap1(x0 - 2 + k % rw, L), L, TW, TH, tiles_x, blk)];
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    if (g[u] < 0) continue;
    const int k = tid + u * kBlock, r = k / tw, c = k % tw;
    const int rs = (flags & 16) ? 6 : 4;
    double2* qo = reinterpret_cast<double2*>(Q_out + (rb + g[u]) * rs);
    qo[0] = make_double2(q[u][0] + rq, q[u][1]);
    qo[1] = make_double2(q[u][2], q[u][3] + md[u]);
    if (flags & 16) {
      qo[2] = make_double2(md[u] * 0.5, (double)(at[u] + 1.f));
    } else if (flags & 2) {
      md_out[rb + g[u]] = md[u] * 0.5;
      atd[rb + g[u]] = at[u] + 1.f;
    }
    if ((flags & 36) == 4) {
      S_out[rb + g[u]] = sS[(r + 3) * sw + c + 3] ^ 1;
      R_out[rb + g[u]] = sR[(r + 2) * rw + c + 2] + 1;
    }
  }
  if ((flags & 36) == 36) {  // bytes via LDS, dword stores
    const int cw = (tw + 8) / 4, tw4 = tw / 4;
    __shared__ uint32_t oS[64 * 16], oR[64 * 16];
    for (int k = tid; k < th * tw4; k += kBlock) {
      const int r = k / tw4, c = k % tw4;
      oS[k] = reinterpret_cast<const uint32_t*>(sS)[(r + 3) * cw + c + 1] ^ 0x01010101u;
      oR[k] = reinterpret_cast<const uint32_t*>(sR)[(r + 2) * cw + c + 1] + 0x01010101u;
    }
    __syncthreads();
    uint32_t* S4 = reinterpret_cast<uint32_t*>(S_out + rb);
    uint32_t* R4 = reinterpret_cast<uint32_t*>(R_out + rb);
    for (int k = tid; k < th * tw4; k += kBlock) {
      const int r = k / tw4, c = k % tw4;
      S4[(y0 + r) * (L / 4) + x0 / 4 + c] = oS[k];
      R4[(y0 + r) * (L / 4) + x0 / 4 + c] = oR[k];
    }
  }
}
}  // namespace

extern "C" int pprobe_launch(const void* S_in, void* S_out, const void* R_in, void* R_out, const void* Q_in,
                             void* Q_out, const void* md_in, void* md_out, void* atd, int L, int TW, int TH,
                             int n_rep, int flags, void* stream) {
  const int tiles_x = (L + TW - 1) / TW, tiles_per_rep = tiles_x * ((L + TH - 1) / TH);
  const int total = n_rep * tiles_per_rep;
  hipLaunchKernelGGL(pprobe, dim3((total + 7) / 8 * 8), dim3(kBlock), 0, (hipStream_t)stream,
                     (const uint8_t*)S_in, (uint8_t*)S_out, (const int8_t*)R_in, (int8_t*)R_out,
                     (const double*)Q_in, (double*)Q_out, (const double*)md_in, (double*)md_out, (float*)atd, L, TW,
                     TH, tiles_x, tiles_per_rep, n_rep, flags);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
