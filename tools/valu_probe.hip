// Issue cost of integer VALU ops on gfx950 (the dropout hash's multiplies): one kernel per op, 8
// independent chains per lane, 4096 iterations, timed with s_memtime (100 MHz) around the loop by lane 0 of
// each wave; blocks of `waves` waves, one block per CU.  hipcc --offload-arch=gfx950 -O3 tools/valu_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHAIN8(INS)                                                                                         \
  asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS " %3, %3, %8\n\t" INS \
               " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS " %6, %6, %8\n\t" INS " %7, %7, %8"               \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)             \
               : "v"(k))

template <int OP>
__global__ void probe(uint32_t* out, uint64_t* cyc, uint32_t seed) {
  uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
           a7 = a0 + 7, k = seed | 1;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 4096; ++i) {
    if constexpr (OP == 0) CHAIN8("v_add_u32");
    if constexpr (OP == 1) CHAIN8("v_mul_lo_u32");
    if constexpr (OP == 2) CHAIN8("v_mul_u32_u24");
    if constexpr (OP == 3) CHAIN8("v_xor_b32");
    if constexpr (OP == 4) CHAIN8("v_mul_hi_u32");
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

int main() {
  const char* names[] = {"v_add_u32", "v_mul_lo_u32", "v_mul_u32_u24", "v_xor_b32", "v_mul_hi_u32"};
  uint32_t* out;
  uint64_t* cyc;
  hipMalloc(&out, 256 * 1024 * 4);
  hipMalloc(&cyc, 256 * 16 * 8);
  for (int waves : {4, 8, 16}) {
    for (int op = 0; op < 5; ++op) {
      auto run = [&]() {
        switch (op) {
          case 0: probe<0><<<256, 64 * waves>>>(out, cyc, 7); break;
          case 1: probe<1><<<256, 64 * waves>>>(out, cyc, 7); break;
          case 2: probe<2><<<256, 64 * waves>>>(out, cyc, 7); break;
          case 3: probe<3><<<256, 64 * waves>>>(out, cyc, 7); break;
          case 4: probe<4><<<256, 64 * waves>>>(out, cyc, 7); break;
        }
      };
      run();
      hipDeviceSynchronize();
      hipEvent_t s, e;
      hipEventCreate(&s);
      hipEventCreate(&e);
      hipEventRecord(s);
      run();
      hipEventRecord(e);
      hipEventSynchronize(e);
      float ms;
      hipEventElapsedTime(&ms, s, e);
      // per SIMD: waves/4 waves x 256 x 8 instructions; clock 2.4 GHz assumed for the cycle estimate
      const double inst_per_simd = (waves / 4.0) * 4096 * 8;
      printf("waves/CU %2d %-14s %8.1f us  ~%.2f cycles per wave-instruction per SIMD\n", waves, names[op],
             ms * 1e3, ms * 1e-3 * 2.4e9 / inst_per_simd);
    }
  }
  return 0;
}
