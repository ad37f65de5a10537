// Issue cost of the integer multiplies a dropout hash can use on gfx950 (round 6): v_mul_lo_u32 (today's second
// round), v_mul_hi_u32, v_mad_u64_u32 (a 64-bit product: two 32-bit hash words per instruction) and, for scale,
// v_add_u32 / v_xor_b32: one kernel per op, 8 independent chains per lane, 2048 iterations, s_memtime around the loop;
// cycles per instruction per wave at 1 / 2 / 3 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_probe3.hip -o /tmp/valu_probe3 && /tmp/valu_probe3
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define V8(INS)                                                                                                   \
  asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS " %3, %3, %8\n\t" INS     \
               " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS " %6, %6, %8\n\t" INS " %7, %7, %8"                 \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)              \
               : "v"(k))
#define M64(I)                                                                                   \
  asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(w##I) : "v"(a##I), "v"(k) : "vcc")

template <int OP>
__global__ void probe(uint32_t* out, uint64_t* cyc, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
           a7 = a0 + 7, k = seed | 1u;
  uint64_t w0 = a0, w1 = a1, w2 = a2, w3 = a3, w4 = a4, w5 = a5, w6 = a6, w7 = a7;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 2048; ++i) {
    if constexpr (OP == 0) V8("v_mul_lo_u32");
    if constexpr (OP == 1) V8("v_mul_hi_u32");
    if constexpr (OP == 2) { M64(0); M64(1); M64(2); M64(3); M64(4); M64(5); M64(6); M64(7); }
    if constexpr (OP == 3) V8("v_add_u32");
    if constexpr (OP == 4) V8("v_xor_b32");
    if constexpr (OP == 5) V8("v_mul_u32_u24");
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 +
                                               (uint32_t)(w0 + w1 + w2 + w3 + w4 + w5 + w6 + w7);
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int OP>
double run(int waves, uint32_t* out, uint64_t* cyc) {
  const int blocks = 256;
  for (int r = 0; r < 2; ++r) {
    probe<OP><<<blocks, 64 * waves>>>(out, cyc, 12345u);
    hipDeviceSynchronize();
  }
  std::vector<uint64_t> h(blocks * waves);
  hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  return (double)h[h.size() / 2] / (2048.0 * 8);
}

int main() {
  uint32_t* out;
  uint64_t* cyc;
  hipMalloc(&out, 256 * 1024 * 4);
  hipMalloc(&cyc, 256 * 16 * 8);
  const char* names[] = {"v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32", "v_add_u32", "v_xor_b32", "v_mul_u32_u24"};
  for (int waves : {4, 8, 12}) {
    double c[6] = {run<0>(waves, out, cyc), run<1>(waves, out, cyc), run<2>(waves, out, cyc),
                   run<3>(waves, out, cyc), run<4>(waves, out, cyc), run<5>(waves, out, cyc)};
    printf("%2d waves/CU (%d per SIMD):", waves, waves / 4);
    for (int i = 0; i < 6; ++i) printf("  %s %.2f", names[i], c[i]);
    printf("  (cyc per instruction per wave)\n");
  }
  return 0;
}
