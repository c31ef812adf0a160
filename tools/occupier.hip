// Occupancy probe: workgroups that hold a chosen VGPR / LDS footprint and SLEEP for a given time
// (s_sleep loops on the constant-clock s_memrealtime, ~no issue slots), launched beside the step
// kernels to separate the cost of a co-resident generator's RESOURCES from that of its WORK.
// Built by tools/occupier_probe.py:  hipcc --offload-arch=gfx950 -O3 -shared -fPIC
#include <hip/hip_runtime.h>
#include <stdint.h>

template <int V>
__global__ __launch_bounds__(256) void occupy(uint64_t ticks, int spin_valu) {
  extern __shared__ uint32_t lds[];
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  float acc = (float)threadIdx.x;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    if (spin_valu) {
#pragma unroll
      for (int k = 0; k < 16; ++k) acc = __builtin_fmaf(acc, 1.0001f, 0.5f);
    } else {
      __builtin_amdgcn_s_sleep(8);
    }
  }
  if (V == 56) asm volatile("" ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12",
                            "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25",
                            "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38",
                            "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51",
                            "v52", "v53", "v54", "v55");
  if (acc == -1.f) lds[threadIdx.x] = 1;  // never: keeps acc live
}

extern "C" int occupier_launch(void* stream, int nwg, int lds_bytes, int vgpr56, double us, int spin_valu) {
  const uint64_t ticks = (uint64_t)(us * 100.0);  // s_memrealtime: 100 MHz
  if (vgpr56)
    hipLaunchKernelGGL(occupy<56>, dim3(nwg), dim3(256), lds_bytes, (hipStream_t)stream, ticks, spin_valu);
  else
    hipLaunchKernelGGL(occupy<0>, dim3(nwg), dim3(256), lds_bytes, (hipStream_t)stream, ticks, spin_valu);
  return (int)hipGetLastError();
}
