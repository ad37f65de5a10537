// Prices VERDICT r4's in-kernel split-K fix-up for the block weight gradients before building it: in that scheme the
// LAST-arriving split block of each 256x256 output tile sums the tile's S fp32 slabs (split order, the same bits as
// splitk_reduce) and writes it, so the reduction runs on one block per tile, at the end of a single-round launch
// (243-252 blocks on 256 CUs: every tile's last block arrives within the same few microseconds). Measured here:
//   reduce : splitk_reduce's grid-stride pass (2048 x 256 threads) over the S slabs, as the step runs it now;
//   fixup  : one 512-thread block per tile (the GEMM's block size) summing that tile's S slabs: the tail the fix-up
//            would add after the last main loop;
//   both after a writer pass that stores the slabs (the GEMM epilogue's bytes), so that they start MALL-hot.
// hipcc --offload-arch=gfx950 -O3 tools/fixup_probe.hip -o /tmp/fixup_probe && /tmp/fixup_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(256) void writer(float* slab, size_t n4, float v) {
  f32x4* s = reinterpret_cast<f32x4*>(slab);
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
    s[i] = f32x4{v, v + 1.f, v + 2.f, (float)(i & 7)};
}

// splitk_reduce_kernel's body (gemm256.hip), non-accumulating
__global__ __launch_bounds__(256) void reduce(const float* __restrict__ slab, int splits, size_t n4, float* __restrict__ out) {
  const f32x4* s4 = reinterpret_cast<const f32x4*>(slab);
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    for (int z = 0; z < splits; z += 8) {
      const int nz = min(8, splits - z);
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (u < nz) v[u] = s4[(size_t)(z + u) * n4 + i];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (u < nz) s += v[u];
    }
    reinterpret_cast<f32x4*>(out)[i] = s;
  }
}

// one block per 256x256 tile of C[M][N]: rows r = 8*it + (tid >> 6), columns 4*(tid & 63) .. +3; the S slabs' loads of
// a row group in flight together (8 at a time), added in split order
__global__ __launch_bounds__(512) void fixup(const float* __restrict__ slab, int splits, int M, int N,
                                             float* __restrict__ out) {
  const int tn = N / 256;
  const int m0 = (blockIdx.x / tn) * 256, n0 = (blockIdx.x % tn) * 256;
  const size_t plane = (size_t)M * N;
  const int c = n0 + 4 * (threadIdx.x & 63);
  for (int it = 0; it < 32; ++it) {
    const int r = m0 + 8 * it + (threadIdx.x >> 6);
    const size_t o = (size_t)r * N + c;
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    for (int z = 0; z < splits; z += 8) {
      const int nz = min(8, splits - z);
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (u < nz) v[u] = *reinterpret_cast<const f32x4*>(slab + (size_t)(z + u) * plane + o);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (u < nz) s += v[u];
    }
    *reinterpret_cast<f32x4*>(out + o) = s;
  }
}

int main() {
  struct Shape { const char* name; int M, N, S; };
  // the block weight gradients of GPT-2 124M at B=64, T=1024 with their default split counts (_lib.wgrad_splits)
  const Shape shapes[] = {{"qkv  768x2304 S=9", 768, 2304, 9}, {"proj 768x768 S=27", 768, 768, 27},
                          {"fc1  768x3072 S=7", 768, 3072, 7}, {"fc2  3072x768 S=7", 3072, 768, 7}};
  size_t maxf = 0;
  for (const Shape& s : shapes) maxf = std::max(maxf, (size_t)s.S * s.M * s.N);
  float *slab, *out, *ref;
  CK(hipMalloc(&slab, maxf * 4));
  CK(hipMalloc(&out, (size_t)3072 * 3072 * 4));
  CK(hipMalloc(&ref, (size_t)3072 * 3072 * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 20;
  printf("%-20s %10s %10s %10s %10s %10s\n", "shape", "write us", "w+reduce", "w+fixup", "reduce", "fixup");
  for (const Shape& s : shapes) {
    const size_t n = (size_t)s.M * s.N, tot = n * s.S;
    const int tiles = (s.M / 256) * (s.N / 256);
    float tw = 0, twr = 0, twf = 0;
    for (int mode = 0; mode < 3; ++mode) {
      for (int w = 0; w < 3; ++w) {  // warm-up
        writer<<<2048, 256>>>(slab, tot / 4, 1.f);
        if (mode == 1) reduce<<<2048, 256>>>(slab, s.S, n / 4, ref);
        if (mode == 2) fixup<<<tiles, 512>>>(slab, s.S, s.M, s.N, out);
      }
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int r = 0; r < reps; ++r) {
        writer<<<2048, 256>>>(slab, tot / 4, (float)r);
        if (mode == 1) reduce<<<2048, 256>>>(slab, s.S, n / 4, ref);
        if (mode == 2) fixup<<<tiles, 512>>>(slab, s.S, s.M, s.N, out);
      }
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      (mode == 0 ? tw : mode == 1 ? twr : twf) = ms * 1e3f / reps;
    }
    // same bits
    std::vector<float> a(n), b(n);
    CK(hipMemcpy(a.data(), ref, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), out, n * 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < n; ++i) bad += a[i] != b[i];
    printf("%-20s %10.1f %10.1f %10.1f %10.1f %10.1f   (%d tiles, mismatches %zu)\n", s.name, tw, twr, twf, twr - tw,
           twf - tw, tiles, bad);
  }
  return 0;
}
