// LDS-DMA (global_load_lds_dwordx4) streaming probe: how fast does one 1-KiB wave-instruction land for
// the two operand image shapes of gemm_pp.hip?
//   pattern 0 (k-contiguous operand): an instruction covers 8 rows x 128 B of a [rows][ld] matrix
//   pattern 1 (m-contiguous operand): an instruction covers 4 rows x 256 B
//   pattern 2 (m-contiguous, interleaved half): 4 rows x 4 x 64 B
// 256 blocks x 512 threads stream a 1 GiB bf16 matrix once into a 4-slot LDS ring (counted vmcnt),
// no compute. Build: hipcc --offload-arch=gfx950 -O3 tools/dma_probe.hip -o tools/dma_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef __attribute__((address_space(3))) void lds_void;

template <int PAT>
__global__ __launch_bounds__(512, 1) void dma_kernel(const char* __restrict__ src, long rows, int ld_bytes, int iters,
                                                      int* sink) {
  __shared__ __attribute__((aligned(1024))) char smem[64 * 1024];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // each block owns a column band of 256 B (pattern 1/2) or 128 B x 2 (pattern 0) and walks the rows
  const long band = blockIdx.x;
  for (int it = 0; it < iters; ++it) {
    // 8 waves x 2 instructions = 16 KiB per step (one "half-tile")
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int ins = wid * 2 + t;
      long row;
      int col;
      if (PAT == 0) {
        row = (long)it * 128 + 8 * ins + (lane >> 3);
        col = (lane & 7) * 16;
      } else if (PAT == 1) {
        row = (long)it * 64 + 4 * ins + (lane >> 4);
        col = (lane & 15) * 16;
      } else {
        row = (long)it * 64 + 4 * ins + (lane >> 4);
        const int c = lane & 15;  // 4 segments of 64 B, 128 B apart
        col = (c >> 2) * 128 + (c & 3) * 16;
      }
      const char* g = src + (row % rows) * ld_bytes + band * 512 + col;
      __builtin_amdgcn_global_load_lds((const void*)g, (lds_void*)(smem + ((it & 3) * 16 + ins) * 1024), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) sink[blockIdx.x] = smem[lane];
}

int main() {
  const long bytes = 1L << 30;
  char* d;
  hipMalloc(&d, bytes);
  hipMemset(d, 1, bytes);
  int* sink;
  hipMalloc(&sink, 4096 * 4);
  const int ld = 256 * 512;  // 128 KiB rows: 256 column bands of 512 B
  const long rows = bytes / ld;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int cfg = 0; cfg < 6; ++cfg) {
    const int pat = cfg % 3;
    const long rmod = cfg < 3 ? rows : 256;  // cfg >= 3: a 256-row window re-read (L2-resident per XCD)
    const int per_step_rows = pat == 0 ? 128 : 64;
    const int iters = (int)(rows / per_step_rows);
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(a);
      if (pat == 0) dma_kernel<0><<<256, 512>>>(d, rmod, ld, iters, sink);
      if (pat == 1) dma_kernel<1><<<256, 512>>>(d, rmod, ld, iters, sink);
      if (pat == 2) dma_kernel<2><<<256, 512>>>(d, rmod, ld, iters, sink);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double moved = 256.0 * iters * 16384;
      if (rep == 2)
        printf("pattern %d %s: %.3f ms, %.0f GB/s (%.2f GiB moved)\n", pat, cfg < 3 ? "HBM stream" : "L2 window ",
               ms, moved / ms / 1e6, moved / (1 << 30));
    }
  }
  return 0;
}
