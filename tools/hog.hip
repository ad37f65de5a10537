// CU hog for the contention A/B (tools/lib_ab.py LIB_AB_HOG): `blocks` workgroups that each hold one CU (96 KB of
// LDS, so no 128-KB GEMM block fits beside one) for `ns` nanoseconds of wall clock, standing in for the RCCL kernels
// of a data-parallel step that share the GPU with the GEMMs.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/hog.hip -o tools/ab/libhog.so
#include <hip/hip_runtime.h>

__global__ __launch_bounds__(256) void hog_kernel(long long ticks) {
  __shared__ float pad[24 * 1024];
  const long long t0 = wall_clock64();
  float acc = 0.f;
  while (wall_clock64() - t0 < ticks) acc += 1.f;
  pad[threadIdx.x] = acc;  // keeps the LDS allocation live
}

extern "C" int hog(int blocks, long long ns, void* stream) {
  // wall_clock64 runs at 100 MHz on gfx9
  hog_kernel<<<blocks, 256, 0, static_cast<hipStream_t>(stream)>>>(ns / 10);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
