// Shared device/host helpers for the gfx950 (MI355X, CDNA4) kernels of libgpt2mi.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define GPT2MI_EXPORT extern "C" __attribute__((visibility("default")))

// A/B knobs (the -D macros tools/variant_lib.sh, tools/wgrad_ablation.sh and `make timing` build experiment libraries
// with; some of them compile stores out or redirect them, i.e. give wrong outputs): the product library is built with
// every knob at its product value, and a knob set to anything else without -DGPT2MI_AB_BUILD is a compile error, so
// one stray -D cannot silently change what the step computes.
#ifdef GPT2MI_AB_BUILD
#define GPT2MI_PRODUCT_KNOB(name, value) static_assert(true, "")
#else
#define GPT2MI_PRODUCT_KNOB(name, value) \
  static_assert((name) == (value), #name " is an A/B knob: build experiments with -DGPT2MI_AB_BUILD")
#endif

// ---- error reporting (C ABI: every entry returns 0 on success) ------------------------------
namespace gpt2mi {
void set_error(const char* fmt, ...);
int check_launch(const char* what);
}  // namespace gpt2mi

#define GPT2MI_REQUIRE(cond, ...)                  \
  do {                                             \
    if (!(cond)) {                                 \
      gpt2mi::set_error(__VA_ARGS__);              \
      return 22; /* EINVAL */                      \
    }                                              \
  } while (0)

// ---- bf16 helpers -----------------------------------------------------------------------------
__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }  // RNE; v_cvt_pk_bf16_f32 on gfx950

__device__ __forceinline__ float u16_to_f(uint16_t u) { return __uint_as_float(((uint32_t)u) << 16); }

// ---- wave (64-lane) reductions ------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- counter-based dropout RNG -------------------------------------------------------------------
// keep(i) is a pure function of (seed, element index), so backward regenerates the forward mask
// without storing it. One 32-bit multiply-xorshift hash yields TWO 16-bit uniforms: element pairs
// share a hash (GEMM/LN/embedding sites: elements 2j, 2j+1; attention: queries q, q^16 of one key,
// which sit in the same lane in every attention kernel). keep = int16(uniform16) >= round(p * 2^16) - 2^15.
// All element / pair indices fit in 32 bits for every BASELINE config (attention B*H*T*T < 2^32).
// The 64-bit site seed holds two words: s32 (low) enters the first round additively, the odd multiplier of the
// second round is the high word (a vetted per-site constant, gpt_2_distributed_amd/dropout_keys.py). With one
// multiplier for every site, each site's mask would be a translate of ONE 2^32-long sequence (site s at counter x =
// site s' at x + s - s'), and a step draws ~6.7e9 counters at cfg 2, so sites would reuse each other's decisions;
// distinct multipliers make the sites' sequences distinct functions (tests/test_oracle.py: decision correlation
// between sites at equal and shifted counters). Free: the multiply takes an SGPR instead of a literal.
__device__ __forceinline__ uint32_t seed32(uint64_t seed) { return (uint32_t)seed; }
// (a seed with a zero high word, e.g. a small integer, takes murmur3's 0x85EBCA6B)
constexpr uint32_t kDropC2 = 0x85EBCA6Bu;
__device__ __forceinline__ uint32_t seed_kx(uint64_t seed) {
  const uint32_t hi = (uint32_t)(seed >> 32);
  return hi ? hi | 1u : kDropC2;
}
// Two rounds of multiply-xorshift (murmur3 fmix32 without its closing rounds). The first round is linear in the
// counter, (x + s32) * C1, so a kernel walking counters x + c (c a per-element constant) forms it as
// drop_pre(s32, x) + c * C1: one v_add instead of an add, xor and v_mul_lo_u32 (half the VALU rate, measured by
// tools/valu_probe.hip) per hash.
constexpr uint32_t kDropC1 = 0x9E3779B1u;
__device__ __forceinline__ uint32_t drop_pre(uint32_t s32, uint32_t x) { return (x + s32) * kDropC1; }
// The second round ends at the multiply (by the site's multiplier kx): a closing xorshift (murmur3's h ^= h >> 13)
// leaves the 16-bit decisions statistically unchanged (tests/test_oracle.py: decision correlations over the
// kernels' counter strides) and costs three instructions per hash in the attention kernels.
__device__ __forceinline__ uint32_t drop_fin(uint32_t h, uint32_t kx) {
  h ^= h >> 16;
  return h * kx;
}
__device__ __forceinline__ uint32_t drop_hash(uint32_t s32, uint32_t kx, uint32_t x) {
  return drop_fin(drop_pre(s32, x), kx);
}
// keep iff the 16-bit half, read as a signed int16, is >= thr - 32768 (P(keep) = 1 - thr / 2^16): a signed
// threshold, so packed-int16 arithmetic can form the decisions of a pair at once from the sign bits of
// (thr - 32769) -sat- half (drop_keep_mask2)
__device__ __forceinline__ bool drop_keep16(uint32_t h, int half, uint32_t thr) {
  // h opaque (no instruction): otherwise sext(low half of x * C2) becomes a second multiply, by C2 << 16
  asm("" : "+v"(h));
  return (int)(int16_t)(half ? (h >> 16) : h) >= (int)thr - 32768;
}
// Both decisions of hash h at once, for the packed path: bit 15 / bit 31 of the result are set iff half 0 / 1
// is kept. tk2 = drop_tk2(thr) (thr >= 1): (thr - 32769) in both int16 halves; saturation keeps the sign exact.
typedef short s16x2 __attribute__((ext_vector_type(2)));
__host__ __device__ __forceinline__ uint32_t drop_tk2(uint32_t thr) {
  const uint32_t t = (uint32_t)(uint16_t)(int16_t)((int)thr - 32769);
  return t | (t << 16);
}
__device__ __forceinline__ uint32_t drop_keep_mask2(uint32_t tk2, uint32_t h) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(__builtin_bit_cast(s16x2, tk2), __builtin_bit_cast(s16x2, h)));
}
// Both decisions of hash h as 32-bit lane masks (all ones = keep), for selects done as bit operations (v_and_b32 /
// v_bfi_b32) instead of a compare into an SGPR pair and v_cndmask (whose SGPR read hazard costs an s_nop per pair)
__device__ __forceinline__ void drop_keep_masks(uint32_t tk2, uint32_t h, uint32_t& m0, uint32_t& m1) {
  const uint32_t r = drop_keep_mask2(tk2, h);
  m0 = (uint32_t)__builtin_amdgcn_sbfe((int)r, 15, 1);
  m1 = (uint32_t)((int)r >> 31);
}
// keep ? a : b for a lane mask m from drop_keep_masks: one v_bitop3_b32 (gfx950's 3-input bit operation; truth table
// 0xCA = S0 ? S1 : S2 bitwise) through its builtin. Not inline asm: the compiler does not apply the MFMA-result read
// hazard (its wait states) to an asm operand, and the attention backward feeds this select straight from MFMA
// accumulators — an asm v_bfi_b32 there read stale dP values once the dQ tile was software-pipelined
// (nondeterministic dK at p > 0, tools/attn_determinism.py). Nor the C bit expression: in the kernels hipcc expands it
// to 2-3 instructions (+156 per dK/dV tile body)
__device__ __forceinline__ float sel_mask(uint32_t m, float a, float b) {
  return __uint_as_float(__builtin_amdgcn_bitop3_b32(m, __float_as_uint(a), __float_as_uint(b), 0xCA));
}
// element-indexed form: element i uses half (i & 1) of hash(i >> 1)
__device__ __forceinline__ bool drop_keep(uint64_t seed, uint64_t idx, uint32_t thr) {
  return drop_keep16(drop_hash(seed32(seed), seed_kx(seed), (uint32_t)(idx >> 1)), (int)(idx & 1), thr);
}

static inline uint32_t drop_threshold(float p) {
  if (p <= 0.f) return 0u;
  double t = (double)p * 65536.0 + 0.5;
  return (uint32_t)(t > 65536.0 ? 65536.0 : t);
}

// ---- XCD-aware block remap (blocks b and b+8 share an XCD; give each XCD a contiguous range) ----
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8, idx = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// ---- LDS-DMA issued by inline asm --------------------------------------------------------------------------
// hipcc's waitcnt pass cannot tell which LDS bytes an LDS-DMA (global_load_lds / buffer_load ... lds) writes, so
// after one it drains ALL vector memory (s_waitcnt vmcnt(0)) before the next LDS read of any address: in a
// multi-stage GEMM that waits for the DMAs just issued for a LATER K-tile and serialises the operand feed with
// the MFMAs. Issued from asm the DMAs are invisible to that pass; the kernels retire them with their own
// counted s_waitcnt vmcnt(N) + s_barrier (RAW) and restage a slot only after a barrier that follows its last
// read (WAR). The compiler's own waits for its ordinary loads stay correct: vector memory loads retire in issue
// order, so extra (asm) loads in flight only make a counted wait wait longer.
// M0 = the LDS destination of the wave's 64 x 16 B (lane-linear; an operand bound to m0). The hazard recognizer
// does not look inside asm: s_nop 4 covers the M0-write -> LDS-DMA (1) and VALU-SGPR-write -> VMEM-read (5) wait
// states of the SGPR operands (descriptor, soffset, M0).
typedef __attribute__((address_space(3))) void lds_void;
// generic pointer into LDS -> LDS byte address: the shared aperture is 4 GiB aligned, so the low 32 bits of a
// flat LDS address are the LDS offset (a plain truncation; the address-space cast would add a null check per DMA)
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)p);
}
__device__ __forceinline__ void lds_dma16(const void* gptr, const void* lds_dst) {
  const uint32_t m0 = lds_addr(lds_dst);
  asm volatile("s_nop 4\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gptr), "{m0}"(m0) : "memory");
}
// raw buffer descriptor over [base, base + 2 GiB) (the same words __builtin_amdgcn_make_buffer_rsrc forms on gfx950)
__device__ __forceinline__ u32x4 buf_desc(const void* base) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  return u32x4{(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a),
               (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32) & 0xffffu), 0x7fffffffu, 0x00020000u};
}
__device__ __forceinline__ void lds_dma16_buf(u32x4 desc, uint32_t voff, int soff, const void* lds_dst) {
  const uint32_t m0 = lds_addr(lds_dst);
  asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(desc), "s"(soff), "{m0}"(m0)
               : "memory");
}
