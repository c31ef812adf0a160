// Clock probe (timing tool only): one wave on its own stream records the shader clock
// (s_memtime) and the 100 MHz constant clock (s_memrealtime) over a spin of `us`
// microseconds, so the chip's effective clock while other kernels run beside it is
// delta(memtime) / delta(memrealtime) x 100 MHz (MI355X_MICROARCH.md, DVFS give-back (6)).
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void clock_probe_kernel(unsigned long long* out, int slot, unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long r = r0;
  while (r - r0 < ticks) {
    __builtin_amdgcn_s_sleep(8);
    r = __builtin_amdgcn_s_memrealtime();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x < 2) out[2 * slot + threadIdx.x] = threadIdx.x ? (r - r0) : (t1 - t0);  // vector stores
}

extern "C" int clock_probe_launch(unsigned long long* out, int slot, int us, hipStream_t s) {
  hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, s, out, slot, (unsigned long long)us * 100ull);
  return (int)hipGetLastError();
}
