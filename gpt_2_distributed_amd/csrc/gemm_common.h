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
};

// NewGELU (model.py:63-77): 0.5u(1 + tanh(z)), z = sqrt(2/pi)(u + 0.044715u^3), evaluated in the
// equivalent sigmoid form u * s with s = 1/(1 + exp(-2z)) (v_exp_f32 + v_rcp_f32: the epilogues run
// this on every fc1 output, where a division-based tanh made them VALU-bound).
//   gelu'(u) = s * (1 + 2*sqrt(2/pi) * u * (1 - s) * (1 + 3*0.044715*u^2))
__device__ __forceinline__ float gelu_sig(float u) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f, m2log2e = -2.0f * 1.4426950408889634f;
  const float z = k0 * u * (1.f + k1 * u * u);
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(m2log2e * z));
}
__device__ __forceinline__ float gelu_f(float u) { return u * gelu_sig(u); }
__device__ __forceinline__ float gelu_grad_from_sig(float u, float sg) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return sg * (1.f + 2.f * k0 * u * (1.f - sg) * (1.f + 3.f * k1 * u * u));
}
__device__ __forceinline__ float gelu_grad_f(float u) { return gelu_grad_from_sig(u, gelu_sig(u)); }

// keep mask of the 4 dropout elements didx..didx+3 (didx even): two hashes, 16 bits per element
__device__ __forceinline__ void drop4(const GemmParams& P, uint64_t didx, bool keep[4]) {
  const uint32_t s = seed32(P.seed);
  const uint32_t h0 = drop_hash(s, (uint32_t)(didx >> 1)), h1 = drop_hash(s, (uint32_t)(didx >> 1) + 1u);
  keep[0] = drop_keep16(h0, 0, P.thr);
  keep[1] = drop_keep16(h0, 1, P.thr);
  keep[2] = drop_keep16(h1, 0, P.thr);
  keep[3] = drop_keep16(h1, 1, P.thr);
}

// 4-element vector load/store of the activation element type TE (bf16 under autocast, fp32 in the
// fp32 / no-autocast mode of the reference).
template <typename TE>
__device__ __forceinline__ void store4(TE* p, f32x4 v) {
  if constexpr (sizeof(TE) == 2) *reinterpret_cast<bf16x4*>(p) = bf16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
  else *reinterpret_cast<f32x4*>(p) = v;
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
template <int EPI, typename TE = bf16>
__device__ __forceinline__ f32x4 epilogue_apply(const GemmParams& P, int gm, int gn, f32x4 v, f32x4 opnd) {
  const size_t cidx = (size_t)gm * P.ldc + gn;
  const uint64_t didx = (uint64_t)gm * P.N + gn;  // dropout element index in the logical [M,N] (even)
  bool keep[4] = {true, true, true, true};
  if (EPI == EPI_RESID || EPI == EPI_GELU)
    if (P.thr) drop4(P, didx, keep);
  if constexpr (EPI == EPI_BF16) {
    store4<TE>(reinterpret_cast<TE*>(P.C) + cidx, v);
    return round4<TE>(v);
  } else if constexpr (EPI == EPI_F32) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] += opnd[j];
    *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(P.C) + cidx) = v;
  } else if constexpr (EPI == EPI_RESID) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float y = v[j];
      if (P.thr) y = keep[j] ? y * P.inv_keep : 0.f;
      opnd[j] += y;
    }
    *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(P.C) + cidx) = opnd;
  } else if constexpr (EPI == EPI_GELU) {
    // the forward also emits what the backward needs of this site: dL/du = dL/dh * keep/(1-p) * gelu'(u),
    // so the fc2 dgrad epilogue is one multiply (no dropout hash, no GELU math, no pre-activation)
    f32x4 h, dg;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float sg = gelu_sig(v[j]);
      float a = v[j] * sg;
      float d = gelu_grad_from_sig(v[j], sg);
      if (P.thr) {
        a = keep[j] ? a * P.inv_keep : 0.f;
        d = keep[j] ? d * P.inv_keep : 0.f;
      }
      h[j] = a;
      dg[j] = d;
    }
    store4<TE>(reinterpret_cast<TE*>(P.aux) + (size_t)gm * P.ldaux + gn, dg);
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

template <int EPI, typename TE = bf16>
__device__ __forceinline__ void epilogue_store(const GemmParams& P, int gm, int gn, f32x4 v) {
  epilogue_apply<EPI, TE>(P, gm, gn, v, epilogue_operand<EPI, TE>(P, gm, gn));
}

namespace gpt2mi {
int gemm256_dispatch(int layout, int epilogue, const GemmParams& P, hipStream_t s, int splits);
int gemm_pp_dispatch(int layout, int epilogue, const GemmParams& P, hipStream_t s, int splits, int map = 0);
int splitk_reduce(const float* slab, int splits, size_t n, float* out, int accumulate, hipStream_t s);
}
