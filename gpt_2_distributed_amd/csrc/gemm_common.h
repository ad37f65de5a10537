// Shared GEMM parameter block and fused epilogue ops (gemm.hip: 128x128 kernel; gemm256.hip).
#pragma once
#include "common.h"

enum Epi : int {
  EPI_BF16 = 0,      // C_bf16 = alpha*acc (+bias)
  EPI_F32 = 1,       // C_f32 (+)= alpha*acc (+bias)           (accumulate flag)
  EPI_RESID = 2,     // C_f32 = resid_f32 + drop(alpha*acc + bias)          (proj / fc2 + residual)
  EPI_GELU = 3,      // u = acc+bias: C = drop(gelu_tanh(u)), aux = keep/(1-p) * gelu'(u)  (fc1 + NewGELU + drop1)
  EPI_GELU_BWD = 4,  // C = alpha*acc * aux          (fc2 dgrad -> fc1 pre-activation grad: mask and gelu'
                     //                               were folded into aux by the forward epilogue)
  EPI_ATOMIC = 5,    // atomicAdd(C_f32, alpha*acc)            (split-K wgrad into the grad arena)
  EPI_SLAB = 6,      // split-K partial tile -> fp32 slab[blockIdx.y] (gemm256 wgrad; summed by splitk_reduce)
  EPI_SLAB16 = 7,    // the same partial tile rounded to a bf16 slab (GPT2MI_SCHED_BF16_SLABS; splitk_reduce16)
};

struct GemmParams {
  const bf16* A;
  const bf16* B;
  void* C;
  const float* bias;
  const float* resid;
  void* aux;  // EPI_GELU: masked GELU derivative out; EPI_GELU_BWD: the same, in (element type = TE)
  const float* alpha_dev;
  float* dbias;  // optional: dbias[n] += sum_m C[m][n] of the stored output (bias grad of the next op)
  int M, N, K, lda, ldb, ldc, ldaux;
  int k_per_split;
  float alpha;
  int accumulate;
  uint64_t seed;
  uint32_t thr;
  float inv_keep;
  int qslot;  // persistent schedule: this launch's work-queue slot (gemm_pp.hip g_pp_queue; set by the dispatcher)
};

// keep mask of the 4 dropout elements 2*pidx .. 2*pidx+3 as multipliers keep/(1-p) or 0 (x * m is the
// dropout of x, as torch's fused dropout forms it): two hashes, 16 bits per element
__device__ __forceinline__ f32x4 drop_scale4(const GemmParams& P, uint32_t pidx) {
  const uint32_t s = seed32(P.seed), kx = seed_kx(P.seed);
  const uint32_t pre = drop_pre(s, pidx);
  const uint32_t h0 = drop_fin(pre, kx), h1 = drop_fin(pre + kDropC1, kx);
  const float k = P.inv_keep;
  return f32x4{drop_keep16(h0, 0, P.thr) ? k : 0.f, drop_keep16(h0, 1, P.thr) ? k : 0.f,
               drop_keep16(h1, 0, P.thr) ? k : 0.f, drop_keep16(h1, 1, P.thr) ? k : 0.f};
}

// NewGELU (model.py:63-77): 0.5u(1 + tanh(z)), z = sqrt(2/pi)(u + 0.044715u^3), evaluated in the
// equivalent sigmoid form u * s with s = 1/(1 + exp(-2z)) (v_exp_f32 + v_rcp_f32, no division).
// Of 4 pre-activations times the dropout multipliers m, and its derivative times m, in
// packed-f32 pairs (v_pk_mul/fma/add_f32 issue two lanes' worth per instruction; the epilogue of the
// fc1 GEMM is VALU-issue bound):
//   s = 1/(1 + 2^(u (A + B u^2))), h = u s m, d = gelu'(u) m = s m + s m * u (1 - s) (2 k0 + 6 k0 k1 u^2)
__device__ __forceinline__ void gelu4(f32x4 u, f32x4 m, f32x4& h, f32x4& d) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f, m2log2e = -2.0f * 1.4426950408889634f;
  const f32x2 A = {k0 * m2log2e, k0 * m2log2e}, B = {k0 * k1 * m2log2e, k0 * k1 * m2log2e};
  const f32x2 Q0 = {2.f * k0, 2.f * k0}, Q1 = {6.f * k0 * k1, 6.f * k0 * k1}, one = {1.f, 1.f};
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const f32x2 x = {u[2 * p], u[2 * p + 1]}, mm = {m[2 * p], m[2 * p + 1]};
    const f32x2 x2 = x * x;
    const f32x2 arg = x * __builtin_elementwise_fma(x2, B, A);
    const f32x2 e = {__builtin_amdgcn_exp2f(arg[0]), __builtin_amdgcn_exp2f(arg[1])};
    const f32x2 den = e + one;
    const f32x2 sg = {__builtin_amdgcn_rcpf(den[0]), __builtin_amdgcn_rcpf(den[1])};
    const f32x2 r = x * (one - sg) * __builtin_elementwise_fma(x2, Q1, Q0);
    const f32x2 sm = sg * mm;
    const f32x2 hh = x * sm, dd = __builtin_elementwise_fma(r, sm, sm);
    h[2 * p] = hh[0];
    h[2 * p + 1] = hh[1];
    d[2 * p] = dd[0];
    d[2 * p + 1] = dd[1];
  }
}

// GELU_MOVE_EXP (A/B timing builds only): 1 = the fc1 epilogue stores u (bf16) in aux instead of
// keep/(1-p) * gelu'(u), and the fc2 dgrad epilogue forms keep/(1-p) * gelu'(u) from it (sigmoid, derivative, the
// site's dropout hash at p = 0.1) before its multiply: the derivative's VALU moved from the fc1 epilogue to the fc2 dgrad's
#ifndef GELU_MOVE_EXP
#define GELU_MOVE_EXP 0
#endif
GPT2MI_PRODUCT_KNOB(GELU_MOVE_EXP, 0);
// h only (GELU_MOVE_EXP): h = u s m
__device__ __forceinline__ f32x4 gelu4h(f32x4 u, f32x4 m) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f, m2log2e = -2.0f * 1.4426950408889634f;
  const f32x2 A = {k0 * m2log2e, k0 * m2log2e}, B = {k0 * k1 * m2log2e, k0 * k1 * m2log2e}, one = {1.f, 1.f};
  f32x4 h;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const f32x2 x = {u[2 * p], u[2 * p + 1]}, mm = {m[2 * p], m[2 * p + 1]};
    const f32x2 arg = x * __builtin_elementwise_fma(x * x, B, A);
    const f32x2 e = {__builtin_amdgcn_exp2f(arg[0]), __builtin_amdgcn_exp2f(arg[1])};
    const f32x2 den = e + one;
    const f32x2 sg = {__builtin_amdgcn_rcpf(den[0]), __builtin_amdgcn_rcpf(den[1])};
    const f32x2 hh = x * (sg * mm);
    h[2 * p] = hh[0];
    h[2 * p + 1] = hh[1];
  }
  return h;
}

// 4-element vector load/store of the activation element type TE (bf16 under autocast, fp32 in the
// fp32 / no-autocast mode of the reference).
// Epilogue stores are non-temporal (global_store ... nt): the outputs stream to HBM without displacing the
// operand tiles the other blocks still read from L2 (step A/B: 65.04 -> 64.39 ms of GPU time; qkv / lm_head
// forward 5-9 % faster in isolation)
// GEMM_STORE_EXP (A/B builds only, tools/variant_lib.sh): 1 = epilogue stores compiled out (values kept live),
// 2 = every tile's stores land in rows / columns 0..255 of the output (an L2-resident 128-KB window)
#ifndef GEMM_STORE_EXP
#define GEMM_STORE_EXP 0
#endif
GPT2MI_PRODUCT_KNOB(GEMM_STORE_EXP, 0);
__device__ __forceinline__ size_t out_idx(int gm, int ld, int gn) {
  if constexpr (GEMM_STORE_EXP == 2) return (size_t)(gm & 255) * ld + (gn & 255);
  return (size_t)gm * ld + gn;
}
template <typename TE>
__device__ __forceinline__ void store4(TE* p, f32x4 v) {
  if constexpr (GEMM_STORE_EXP == 1) {
    asm volatile("" ::"v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));
    return;
  }
  if constexpr (sizeof(TE) == 2)
    __builtin_nontemporal_store(bf16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])}, reinterpret_cast<bf16x4*>(p));
  else __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
}
// v as stored in TE (bf16 rounding)
template <typename TE>
__device__ __forceinline__ f32x4 round4(f32x4 v) {
  if constexpr (sizeof(TE) == 2) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = bf2f(f2bf(v[j]));
  }
  return v;
}
template <typename TE>
__device__ __forceinline__ f32x4 load4(const TE* p) {
  if constexpr (sizeof(TE) == 2) {
    bf16x4 t = *reinterpret_cast<const bf16x4*>(p);
    return f32x4{bf2f(t[0]), bf2f(t[1]), bf2f(t[2]), bf2f(t[3])};
  } else {
    return *reinterpret_cast<const f32x4*>(p);
  }
}

// The epilogue's input operand at C[gm][gn..gn+3]: the residual (RESID), the stored pre-activation
// (GELU_BWD) or the old C (F32 with accumulate); zeros otherwise. Separate from the apply step so a
// kernel can issue these loads early (gemm_pp.hip prefetches a whole pass of them).
template <int EPI, typename TE = bf16>
__device__ __forceinline__ f32x4 epilogue_operand(const GemmParams& P, int gm, int gn) {
  if constexpr (EPI == EPI_RESID) {
    return *reinterpret_cast<const f32x4*>(P.resid + (size_t)gm * P.ldc + gn);
  } else if constexpr (EPI == EPI_GELU_BWD) {
    return load4<TE>(reinterpret_cast<const TE*>(P.aux) + (size_t)gm * P.ldaux + gn);
  } else if constexpr (EPI == EPI_F32) {
    if (P.accumulate) return *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(P.C) + (size_t)gm * P.ldc + gn);
    return f32x4{0.f, 0.f, 0.f, 0.f};
  } else {
    return f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

// Apply the fused epilogue to 4 consecutive outputs C[gm][gn..gn+3]; v = alpha*acc (+bias), opnd =
// epilogue_operand(gm, gn). TE = element type of the bf16-or-fp32 outputs (C of BF16/GELU/GELU_BWD, aux).
// Returns the primary output as stored for BF16 / GELU_BWD (for fused column sums), v otherwise.
// DROPM: -1 tests P.thr per call; 0 / 1 = dropout known off / on (a caller that branches once per tile: the
// per-row test otherwise splits a pass into exec-masked blocks that cannot interleave).
template <int EPI, typename TE = bf16, int DROPM = -1>
__device__ __forceinline__ f32x4 epilogue_apply(const GemmParams& P, int gm, int gn, f32x4 v, f32x4 opnd) {
  const bool drop = DROPM < 0 ? P.thr != 0u : DROPM == 1;
  const size_t cidx = out_idx(gm, P.ldc, gn);
  // dropout pair index: element gm*N + gn of the logical [M,N] over 2, mod 2^32 (N and gn are multiples of 4
  // in every kernel: N is a multiple of the tile width, host-checked)
  const uint32_t pidx = (uint32_t)gm * (uint32_t)(P.N >> 1) + (uint32_t)(gn >> 1);
  if constexpr (EPI == EPI_BF16) {
    store4<TE>(reinterpret_cast<TE*>(P.C) + cidx, v);
    return round4<TE>(v);
  } else if constexpr (EPI == EPI_F32) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] += opnd[j];
    store4<float>(reinterpret_cast<float*>(P.C) + cidx, v);
  } else if constexpr (EPI == EPI_RESID) {
    // x + drop(y) rounded as two operations (the reference's dropout multiply, then the residual add): never
    // contracted to an fma, so every kernel (and schedule) that applies this epilogue stores the same bits. Vector
    // operations: v_pk_mul_f32 / v_pk_add_f32 (two lanes' worth per instruction, each rounded on its own) whether
    // or not the SLP pass runs (gemm_pp.hip is built without it)
#pragma clang fp contract(off)
    if (drop) v = v * drop_scale4(P, pidx);
    opnd = opnd + v;
    store4<float>(reinterpret_cast<float*>(P.C) + cidx, opnd);
  } else if constexpr (EPI == EPI_GELU) {
    // the forward also emits what the backward needs of this site: dL/du = dL/dh * keep/(1-p) * gelu'(u),
    // so the fc2 dgrad epilogue is one multiply (no dropout hash, no GELU math, no pre-activation)
    f32x4 h, dg, m = {1.f, 1.f, 1.f, 1.f};
    if (drop) m = drop_scale4(P, pidx);
    gelu4(v, m, h, dg);
    store4<TE>(reinterpret_cast<TE*>(P.aux) + out_idx(gm, P.ldaux, gn), dg);
    store4<TE>(reinterpret_cast<TE*>(P.C) + cidx, h);
  } else if constexpr (EPI == EPI_GELU_BWD) {
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = v[j] * opnd[j];
    store4<TE>(reinterpret_cast<TE*>(P.C) + cidx, o);
    return round4<TE>(o);
  } else if constexpr (EPI == EPI_ATOMIC) {
    float* C = reinterpret_cast<float*>(P.C);
#pragma unroll
    for (int j = 0; j < 4; ++j) atomicAdd(C + cidx + j, v[j]);
  }
  return v;
}

// The bf16-output epilogues (BF16, GELU, GELU_BWD) on 8 consecutive outputs C[gm][gn..gn+7] (v0: gn..gn+3,
// v1: gn+4..gn+7; op: the GELU_BWD operand as loaded), every output array written by ONE 16-B store per lane: the
// epilogue's store tail is store-issue bound (per instruction, not per byte; cdna_hip_programming.md T21), so
// half the instructions of the 4-wide form for the same bytes. Bitwise the same results as epilogue_apply.
// r0 / r1: the primary output as stored (bf16-rounded), for fused column sums.
// Returns the stored bf16 values: the as-stored column sums widen these bits instead of converting again.
__device__ __forceinline__ bf16x8 store8_bf16(bf16* p, f32x4 a, f32x4 b) {
  const bf16x8 v = {f2bf(a[0]), f2bf(a[1]), f2bf(a[2]), f2bf(a[3]), f2bf(b[0]), f2bf(b[1]), f2bf(b[2]), f2bf(b[3])};
  if constexpr (GEMM_STORE_EXP == 1) {
    asm volatile("" ::"v"(__builtin_bit_cast(u32x4, v)));
    return v;
  }
  __builtin_nontemporal_store(v, reinterpret_cast<bf16x8*>(p));
  return v;
}
__device__ __forceinline__ void widen8(bf16x8 v, f32x4& r0, f32x4& r1) {
  r0 = f32x4{bf2f(v[0]), bf2f(v[1]), bf2f(v[2]), bf2f(v[3])};
  r1 = f32x4{bf2f(v[4]), bf2f(v[5]), bf2f(v[6]), bf2f(v[7])};
}
template <int EPI, int DROPM = -1>
__device__ __forceinline__ void epilogue8(const GemmParams& P, int gm, int gn, f32x4 v0, f32x4 v1, bf16x8 op, f32x4& r0,
                                          f32x4& r1) {
  static_assert(EPI == EPI_BF16 || EPI == EPI_GELU || EPI == EPI_GELU_BWD, "bf16-output epilogues only");
  const bool drop = DROPM < 0 ? P.thr != 0u : DROPM == 1;
  bf16* C = reinterpret_cast<bf16*>(P.C) + out_idx(gm, P.ldc, gn);
  if constexpr (EPI == EPI_BF16) {
    widen8(store8_bf16(C, v0, v1), r0, r1);
  } else if constexpr (EPI == EPI_GELU) {
    const uint32_t pidx = (uint32_t)gm * (uint32_t)(P.N >> 1) + (uint32_t)(gn >> 1);
    f32x4 h0, d0, h1, d1, m0 = {1.f, 1.f, 1.f, 1.f}, m1 = {1.f, 1.f, 1.f, 1.f};
    if (drop) {
      m0 = drop_scale4(P, pidx);
      m1 = drop_scale4(P, pidx + 2);
    }
    if constexpr (GELU_MOVE_EXP == 1) {
      h0 = gelu4h(v0, m0);
      h1 = gelu4h(v1, m1);
      d0 = v0;
      d1 = v1;
    } else {
      gelu4(v0, m0, h0, d0);
      gelu4(v1, m1, h1, d1);
    }
    store8_bf16(reinterpret_cast<bf16*>(P.aux) + out_idx(gm, P.ldaux, gn), d0, d1);
    store8_bf16(C, h0, h1);
    r0 = h0;
    r1 = h1;
  } else if constexpr (GELU_MOVE_EXP == 1) {
    const uint32_t pidx = (uint32_t)gm * (uint32_t)(P.N >> 1) + (uint32_t)(gn >> 1);
    GemmParams Q = P;
    Q.thr = 6554u;  // the fc1 site's p = 0.1 (timing build)
    Q.inv_keep = 1.f / 0.9f;
    const f32x4 m0 = drop_scale4(Q, pidx), m1 = drop_scale4(Q, pidx + 2);
    f32x4 h0, d0, h1, d1;
    gelu4(f32x4{bf2f(op[0]), bf2f(op[1]), bf2f(op[2]), bf2f(op[3])}, m0, h0, d0);
    gelu4(f32x4{bf2f(op[4]), bf2f(op[5]), bf2f(op[6]), bf2f(op[7])}, m1, h1, d1);
    widen8(store8_bf16(C, v0 * d0, v1 * d1), r0, r1);
  } else {
    // vector products: packed (v_pk_mul_f32) whether or not the compiler's SLP pass runs
    const f32x4 o0 = v0 * f32x4{bf2f(op[0]), bf2f(op[1]), bf2f(op[2]), bf2f(op[3])};
    const f32x4 o1 = v1 * f32x4{bf2f(op[4]), bf2f(op[5]), bf2f(op[6]), bf2f(op[7])};
    widen8(store8_bf16(C, o0, o1), r0, r1);
  }
}

template <int EPI, typename TE = bf16>
__device__ __forceinline__ void epilogue_store(const GemmParams& P, int gm, int gn, f32x4 v) {
  epilogue_apply<EPI, TE>(P, gm, gn, v, epilogue_operand<EPI, TE>(P, gm, gn));
}

// Grouped weight gradients: kGroupMax problems at most, one launch (gemm_pp.hip gemm_pp_grouped_kernel); prefix[g] =
// output tiles of problems 0 .. g-1 (prefix[count] = tiles)
constexpr int kGroupMax = 4;
struct GemmGroup {
  GemmParams p[kGroupMax];
  int prefix[kGroupMax + 1];
  int count, tiles;
};

namespace gpt2mi {
int gemm_pp_grouped(const GemmGroup& G, hipStream_t s);
// out_g[i] (+)= sum_z slab_g[z][i] for every problem g of a grouped launch (fp32 slabs)
int splitk_reduce_grouped(const float* const* slab, float* const* out, const size_t* n, int count, int splits,
                          int accumulate, hipStream_t s);
int gemm256_dispatch(int layout, int epilogue, const GemmParams& P, hipStream_t s, int splits);
// persistent_ok: the caller allows the persistent (one block per CU) schedule (gpt2mi.h GPT2MI_SCHED_NO_PERSISTENT);
// shared_cus: other kernels (RCCL) may hold CUs: the persistent shapes take their tiles from work queues
// (GPT2MI_SCHED_SHARED_CUS)
int gemm_pp_dispatch(int layout, int epilogue, const GemmParams& P, hipStream_t s, int splits, int map = 0,
                     bool persistent_ok = true, bool shared_cus = false);
int splitk_reduce(const float* slab, int splits, size_t n, float* out, int accumulate, hipStream_t s);
// the same sums over bf16 slabs (each element widened to fp32, then added in split order)
int splitk_reduce16(const bf16* slab, int splits, size_t n, float* out, int accumulate, hipStream_t s);
// out[c][r] (+)= sum_z slab[z][r][c]: slabs [splits][rows][cols] summed in split order and written transposed
int splitk_reduce_t(const float* slab, int splits, int rows, int cols, float* out, int accumulate, hipStream_t s);
int splitk_reduce16_t(const bf16* slab, int splits, int rows, int cols, float* out, int accumulate, hipStream_t s);
}
