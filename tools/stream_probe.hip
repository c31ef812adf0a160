// Streaming probe (timing tool only): per-agent read+write of the step
// kernel's arrays with no stencil, to price each array's access width.
//   flags: 1 Q (32 B AoS), 2 md (f64), 4 atd (f32), 8 S+R (u8 x2),
//          16 vectorised narrow arrays (thread owns 4 consecutive agents),
//          32 Q as 4 SoA planes
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
constexpr int kBlock = 256;
__global__ __launch_bounds__(kBlock) void sprobe(const double* Qi, double* Qo, const double* mi, double* mo,
                                                 float* at, const uint8_t* Si, uint8_t* So, const int8_t* Ri,
                                                 int8_t* Ro, int n, int flags) {
  const int base = blockIdx.x * 1024;
  const int tid = threadIdx.x;
  if (flags & 16) {
    const int a0 = base + tid * 4;
    if (a0 + 3 >= n) return;
    double acc = 0.0;
    if (flags & 1) {
      const double2* q = reinterpret_cast<const double2*>(Qi + (size_t)a0 * 4);
      double2 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = q[j];
      double2* qo = reinterpret_cast<double2*>(Qo + (size_t)a0 * 4);
#pragma unroll
      for (int j = 0; j < 8; ++j) qo[j] = make_double2(v[j].x + 1.0, v[j].y);
    }
    if (flags & 2) {
      const double2* m = reinterpret_cast<const double2*>(mi + a0);
      double2 a = m[0], b = m[1];
      double2* o = reinterpret_cast<double2*>(mo + a0);
      o[0] = make_double2(a.x * 0.5, a.y);
      o[1] = make_double2(b.x, b.y * 0.5);
    }
    if (flags & 4) {
      float4* p = reinterpret_cast<float4*>(at + a0);
      float4 v = *p;
      v.x += 1.f;
      *p = v;
    }
    if (flags & 8) {
      const uint32_t s = *reinterpret_cast<const uint32_t*>(Si + a0);
      const uint32_t r = *reinterpret_cast<const uint32_t*>(Ri + a0);
      *reinterpret_cast<uint32_t*>(So + a0) = s ^ 0x01010101u;
      *reinterpret_cast<uint32_t*>(Ro + a0) = r + 0x01010101u;
    }
    (void)acc;
    return;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int a = base + tid + u * kBlock;
    if (a >= n) continue;
    if (flags & 1) {
      if (flags & 32) {
        double v[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) v[p] = Qi[(size_t)p * n + a];
#pragma unroll
        for (int p = 0; p < 4; ++p) Qo[(size_t)p * n + a] = v[p] + 1.0;
      } else {
        const double2* q = reinterpret_cast<const double2*>(Qi + (size_t)a * 4);
        const double2 x = q[0], y = q[1];
        double2* qo = reinterpret_cast<double2*>(Qo + (size_t)a * 4);
        qo[0] = make_double2(x.x + 1.0, x.y);
        qo[1] = y;
      }
    }
    if (flags & 2) mo[a] = mi[a] * 0.5;
    if (flags & 4) at[a] += 1.f;
    if (flags & 8) {
      So[a] = Si[a] ^ 1;
      Ro[a] = Ri[a] + 1;
    }
  }
}
}  // namespace

extern "C" int sprobe_launch(const void* Qi, void* Qo, const void* mi, void* mo, void* at, const void* Si, void* So,
                             const void* Ri, void* Ro, int n, int flags, void* stream) {
  hipLaunchKernelGGL(sprobe, dim3((n + 1023) / 1024), dim3(kBlock), 0, (hipStream_t)stream, (const double*)Qi,
                     (double*)Qo, (const double*)mi, (double*)mo, (float*)at, (const uint8_t*)Si, (uint8_t*)So,
                     (const int8_t*)Ri, (int8_t*)Ro, n, flags);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
