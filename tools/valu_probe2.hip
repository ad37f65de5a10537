// Issue cost of packed vs scalar f32 VALU on gfx950 (the softmax affine pairs and the GEMM epilogues' f32x4 math): one
// kernel per op, 8 independent chains per lane (16 floats: the packed ops work on register pairs), 2048 iterations,
// timed with s_memtime around the loop by lane 0 of each wave; one block of `waves` waves per CU. Cycles are per
// instruction per wave; "per float" divides the packed ops by 2.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_probe2.hip -o /tmp/valu_probe2 && /tmp/valu_probe2
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef float f32x2 __attribute__((ext_vector_type(2)));

#define P8(INS)                                                                                                     \
  asm volatile(INS " %0, %0, %8, %8\n\t" INS " %1, %1, %8, %8\n\t" INS " %2, %2, %8, %8\n\t" INS " %3, %3, %8, %8\n\t" \
               INS " %4, %4, %8, %8\n\t" INS " %5, %5, %8, %8\n\t" INS " %6, %6, %8, %8\n\t" INS " %7, %7, %8, %8"     \
               : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3), "+v"(p4), "+v"(p5), "+v"(p6), "+v"(p7)                     \
               : "v"(k2))
#define P8_2(INS)                                                                                        \
  asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS " %3, %3, %8\n\t" INS \
               " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS " %6, %6, %8\n\t" INS " %7, %7, %8"             \
               : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3), "+v"(p4), "+v"(p5), "+v"(p6), "+v"(p7)          \
               : "v"(k2))
#define S8(INS)                                                                                                   \
  asm volatile(INS " %0, %0, %8, %8\n\t" INS " %1, %1, %8, %8\n\t" INS " %2, %2, %8, %8\n\t" INS " %3, %3, %8, %8\n\t" \
               INS " %4, %4, %8, %8\n\t" INS " %5, %5, %8, %8\n\t" INS " %6, %6, %8, %8\n\t" INS " %7, %7, %8, %8"     \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)                     \
               : "v"(k))
#define S8_2(INS)                                                                                        \
  asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS " %3, %3, %8\n\t" INS \
               " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS " %6, %6, %8\n\t" INS " %7, %7, %8"             \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)          \
               : "v"(k))

template <int OP>
__global__ void probe(float* out, uint64_t* cyc, float seed) {
  float a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
        a7 = a0 + 7, k = seed * 0.5f;
  f32x2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}, p4 = p0 + 1.f, p5 = p1 + 1.f, p6 = p2 + 1.f,
        p7 = p3 + 1.f, k2 = {k, k};
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 2048; ++i) {
    if constexpr (OP == 0) S8("v_fma_f32");
    if constexpr (OP == 1) P8("v_pk_fma_f32");
    if constexpr (OP == 2) S8_2("v_mul_f32");
    if constexpr (OP == 3) P8_2("v_pk_mul_f32");
    if constexpr (OP == 4) S8_2("v_add_f32");
    if constexpr (OP == 5) P8_2("v_pk_add_f32");
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const float r = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0[0] + p1[1] + p2[0] + p3[1] + p4[0] + p5[1] + p6[0] + p7[1];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int OP>
double run(int waves, float* out, uint64_t* cyc) {
  const int blocks = 256;
  probe<OP><<<blocks, 64 * waves>>>(out, cyc, 1e-7f);
  hipDeviceSynchronize();
  probe<OP><<<blocks, 64 * waves>>>(out, cyc, 1e-7f);
  hipDeviceSynchronize();
  std::vector<uint64_t> h(blocks * waves);
  hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  return (double)h[h.size() / 2] / (2048.0 * 8);  // per instruction, one wave
}

int main() {
  float* out;
  uint64_t* cyc;
  hipMalloc(&out, 256 * 1024 * 4);
  hipMalloc(&cyc, 256 * 16 * 8);
  const char* names[] = {"v_fma_f32", "v_pk_fma_f32", "v_mul_f32", "v_pk_mul_f32", "v_add_f32", "v_pk_add_f32"};
  for (int waves : {4, 8, 12}) {
    double c[6] = {run<0>(waves, out, cyc), run<1>(waves, out, cyc), run<2>(waves, out, cyc),
                   run<3>(waves, out, cyc), run<4>(waves, out, cyc), run<5>(waves, out, cyc)};
    printf("%2d waves/CU (%d per SIMD):", waves, waves / 4);
    for (int i = 0; i < 6; ++i) printf("  %s %.2f cyc/ins (%.2f per float)", names[i], c[i], i & 1 ? c[i] / 2 : c[i]);
    printf("\n");
  }
  return 0;
}
