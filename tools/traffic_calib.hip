// Calibration of the L2's memory-side request counters (TCC_EA0_*) on gfx950 against known byte
// counts, for the access widths the step kernel uses.  MI355X_MICROARCH.md (HBM section): FETCH_SIZE
// reports half of a 16-B-per-lane streaming read; "other access widths are uncalibrated".
//
// Each pattern is its own kernel (rocprofv3 names it), moves exactly kBytes of data (reads or writes)
// in a region of its own, and is preceded by a flush kernel that streams a separate 256 MiB region
// (so the pattern starts with a cold L2 and the flush collects any dirty lines the previous pattern
// left).  Timing/measurement tool only:
//   hipcc --offload-arch=gfx950 -O3 -o build_probe/traffic_calib tools/traffic_calib.hip
//   rocprofv3 --kernel-trace --pmc <counters> -- build_probe/traffic_calib
// tools/traffic_split.py turns the counter CSVs into bytes per pattern.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

namespace {
constexpr size_t kBytes = 128ull << 20;   // bytes moved per pattern
constexpr size_t kFlush = 256ull << 20;
constexpr int kGrid = 2048, kBlock = 256;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <typename T>
__device__ __forceinline__ uint32_t fold(const T& v) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&v);
  uint32_t a = 0;
  for (unsigned i = 0; i < (sizeof(T) + 3) / 4; ++i) a ^= w[i];
  return a;
}
__device__ __forceinline__ uint32_t fold(const uint8_t& v) { return v * 0x01000193u; }

// contiguous reads, W bytes per lane
template <typename T>
__global__ __launch_bounds__(kBlock) void rd_stream(const T* __restrict__ p, size_t n, uint32_t* sink) {
  uint32_t a = 0;
  for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)kGrid * kBlock) a ^= fold(p[i]);
  if (a == 0x9e3779b9u) sink[0] = a;
}
// contiguous writes, W bytes per lane
template <typename T>
__global__ __launch_bounds__(kBlock) void wr_stream(T* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)kGrid * kBlock) {
    T v;
    uint8_t* b = reinterpret_cast<uint8_t*>(&v);
    for (unsigned k = 0; k < sizeof(T); ++k) b[k] = (uint8_t)(i + k);
    p[i] = v;
  }
}
// 16-B writes to every other 16-B slot: half of each 32-B sector written (the Q-plane row of one
// agent whose plane neighbour is in the other state).  Moves kBytes of data over 2*kBytes of lines.
__global__ __launch_bounds__(kBlock) void wr16_half(uint4* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)kGrid * kBlock)
    p[2 * i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}
// 16-B writes at a 64-B stride: one 32-B sector of each 64-B block half written (32 vs 64-B write
// granularity).  Moves kBytes / 4 of data over kBytes of lines.
__global__ __launch_bounds__(kBlock) void wr16_quarter(uint4* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)kGrid * kBlock)
    p[4 * i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}
// 4-B reads of 48-B row segments at a 200-B pitch (an L=200 lattice's S/R window rows: 12 lanes
// per row): only the segment's bytes are wanted; kBytes / 4 of segments (over ~kBytes of rows).
__global__ __launch_bounds__(kBlock) void rd_rows48(const uint32_t* __restrict__ p, size_t rows, uint32_t* sink) {
  uint32_t a = 0;
  for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < rows * 12; i += (size_t)kGrid * kBlock)
    a ^= p[(i / 12) * 50 + (i % 12)];
  if (a == 0x9e3779b9u) sink[0] = a;
}
__global__ __launch_bounds__(kBlock) void flush(const uint4* __restrict__ p, size_t n, uint32_t* sink) {
  uint32_t a = 0;
  for (size_t i = blockIdx.x * (size_t)kBlock + threadIdx.x; i < n; i += (size_t)kGrid * kBlock) a ^= p[i].x ^ p[i].w;
  if (a == 0x9e3779b9u) sink[0] = a;
}
}  // namespace

int main() {
  const int kPatterns = 11;
  uint8_t *base = nullptr, *fl = nullptr;
  uint32_t* sink = nullptr;
  const size_t region = 2 * kBytes + (256ull << 10);
  CK(hipMalloc(&base, region * kPatterns));
  CK(hipMalloc(&fl, kFlush));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(base, 0x5a, region * kPatterns));
  CK(hipMemset(fl, 0x33, kFlush));
  CK(hipDeviceSynchronize());
  auto R = [&](int k) { return base + region * k; };
  auto F = [&]() { hipLaunchKernelGGL(flush, dim3(kGrid), dim3(kBlock), 0, 0, (const uint4*)fl, kFlush / 16, sink); };
  F();
  hipLaunchKernelGGL(rd_stream<uint4>, dim3(kGrid), dim3(kBlock), 0, 0, (const uint4*)R(0), kBytes / 16, sink); F();
  hipLaunchKernelGGL(rd_stream<uint2>, dim3(kGrid), dim3(kBlock), 0, 0, (const uint2*)R(1), kBytes / 8, sink); F();
  hipLaunchKernelGGL(rd_stream<uint32_t>, dim3(kGrid), dim3(kBlock), 0, 0, (const uint32_t*)R(2), kBytes / 4, sink); F();
  hipLaunchKernelGGL(rd_stream<uint8_t>, dim3(kGrid), dim3(kBlock), 0, 0, (const uint8_t*)R(3), kBytes, sink); F();
  hipLaunchKernelGGL(rd_rows48, dim3(kGrid), dim3(kBlock), 0, 0, (const uint32_t*)R(4), kBytes / 192, sink); F();
  hipLaunchKernelGGL(wr_stream<uint4>, dim3(kGrid), dim3(kBlock), 0, 0, (uint4*)R(5), kBytes / 16); F();
  hipLaunchKernelGGL(wr_stream<uint2>, dim3(kGrid), dim3(kBlock), 0, 0, (uint2*)R(6), kBytes / 8); F();
  hipLaunchKernelGGL(wr_stream<uint32_t>, dim3(kGrid), dim3(kBlock), 0, 0, (uint32_t*)R(7), kBytes / 4); F();
  hipLaunchKernelGGL(wr_stream<uint8_t>, dim3(kGrid), dim3(kBlock), 0, 0, (uint8_t*)R(8), kBytes); F();
  hipLaunchKernelGGL(wr16_half, dim3(kGrid), dim3(kBlock), 0, 0, (uint4*)R(9), kBytes / 16); F();
  hipLaunchKernelGGL(wr16_quarter, dim3(kGrid), dim3(kBlock), 0, 0, (uint4*)R(10), kBytes / 64); F();
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  std::printf("traffic_calib: 11 patterns of %zu bytes each, flush %zu bytes between\n", kBytes, kFlush);
  CK(hipFree(base));
  CK(hipFree(fl));
  CK(hipFree(sink));
  return 0;
}
