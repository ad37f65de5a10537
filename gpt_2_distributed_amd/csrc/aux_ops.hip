// Small bandwidth kernels around the step: the gradient entering through the returned logits, the
// residual-branch gradient of a stand-alone sub-module backward, dtype casts, the data-parallel gradient
// pre-scale, and the FSDP shard pack/unpack passes. gfx950, wave64, 16-B vector accesses where aligned.
//
// Replaces: autograd's accumulation of a user loss's dlogits into the lm_head
// backward (model.py:351, logits returned to the caller), the dropout+bias-grad backward of a branch
// output (model.py:158,191), DDP's bucket division by world size (torch/nn/parallel/distributed.py
// reducer, train_gpt2_distributed.py:163) and FSDP's bf16 flat-parameter all-gather / grad
// reduce-scatter casts (train_gpt2_distributed.py:146-161, MixedPrecision(param=bf16, reduce=bf16)).
#include "common.h"

namespace {

template <typename T>
__device__ __forceinline__ float ld_f(const T* p) {
  if constexpr (sizeof(T) == 2) return bf2f(*p);
  else return *p;
}
template <typename T>
__device__ __forceinline__ T st_v(float v) {
  if constexpr (sizeof(T) == 2) return f2bf(v);
  else return v;
}

// dl[b*Tp + t][n] = (init ? 0 : alpha*dl) + g[b*Tv + t][n] for t < Tv, n < V; columns [V, ldd) = 0;
// rows t >= Tv (sequence padding) = (init ? 0 : unchanged). One block per row.
template <typename T>
__global__ __launch_bounds__(256) void dlogits_accum_kernel(T* __restrict__ dl, int ldd, const T* __restrict__ g,
                                                            int ldg, int Tp, int Tv, int V,
                                                            const float* __restrict__ alpha_dev, int init) {
  const int row = blockIdx.x;
  const int b = row / Tp, t = row % Tp;
  T* d = dl + (size_t)row * ldd;
  const float a = init ? 0.f : (alpha_dev ? alpha_dev[0] : 1.f);
  if (t >= Tv) {
    if (init)
      for (int c = threadIdx.x; c < ldd; c += 256) d[c] = st_v<T>(0.f);
    return;
  }
  const T* gr = g + ((size_t)b * Tv + t) * ldg;
  for (int c = threadIdx.x; c < ldd; c += 256) {
    float v = 0.f;
    if (c < V) v = (init ? 0.f : a * ld_f(d + c)) + ld_f(gr + c);
    d[c] = st_v<T>(v);
  }
}

// Residual-branch gradient of a sub-module backward: out = bf16/fp32(dres * keep/(1-p)) and
// dbias += colsum(out as stored) — what the LayerNorm backward emits for the branch below it in the
// fused step (norm_embed.hip ln_bwd_kernel), for a caller that hands the branch output grad directly.
// Each thread owns 4 adjacent columns; blockIdx.y splits rows; one atomic per column per block.
template <typename TO>
__global__ __launch_bounds__(256) void branch_bwd_kernel(const float* __restrict__ dres, TO* __restrict__ out,
                                                         float* __restrict__ dbias, int M, int C, int rows_per_block,
                                                         uint64_t seed, uint32_t thr, float inv_keep) {
  const int col = (blockIdx.x * 64 + (threadIdx.x & 63)) * 4;
  const int sub = threadIdx.x >> 6;
  const int r0 = blockIdx.y * rows_per_block, r1 = min(M, r0 + rows_per_block);
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  if (col < C) {
    for (int r = r0 + sub; r < r1; r += 4) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(dres + (size_t)r * C + col);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float x = v[j];
        if (thr) x = drop_keep(seed, (uint64_t)r * C + col + j, thr) ? x * inv_keep : 0.f;
        const TO o = st_v<TO>(x);
        out[(size_t)r * C + col + j] = o;
        s[j] += ld_f(&o);
      }
    }
  }
  __shared__ float red[4][256];
#pragma unroll
  for (int j = 0; j < 4; ++j) red[sub][(threadIdx.x & 63) * 4 + j] = s[j];
  __syncthreads();
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (dbias && c < C) atomicAdd(dbias + c, red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x]);
}

__global__ __launch_bounds__(256) void cast_bf16_f32_kernel(const bf16* __restrict__ x, float* __restrict__ y, size_t n) {
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) y[i] = bf2f(x[i]);
}

// x *= s over n floats (n % 4 == 0, 16-B aligned)
__global__ __launch_bounds__(256) void scale_kernel(float* __restrict__ x, size_t n4, float s) {
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    f32x4 v = reinterpret_cast<f32x4*>(x)[i];
    reinterpret_cast<f32x4*>(x)[i] = v * s;
  }
}

// FSDP unpack of a gathered flat unit: dst_f32 = src, dst_bf16 = bf16(src) (src bf16 or fp32)
template <typename TS>
__global__ __launch_bounds__(256) void unpack_kernel(const TS* __restrict__ src, float* __restrict__ dst,
                                                     bf16* __restrict__ dst_bf, size_t n) {
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const float v = ld_f(src + i);
    if (dst) dst[i] = v;
    if (dst_bf) dst_bf[i] = f2bf(v);
  }
}

// FSDP: dst (fp32 grad shard) (+)= src (reduce-scattered shard, bf16 or fp32)
template <typename TS>
__global__ __launch_bounds__(256) void accum_kernel(const TS* __restrict__ src, float* __restrict__ dst, size_t n,
                                                    int accumulate) {
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    dst[i] = (accumulate ? dst[i] : 0.f) + ld_f(src + i);
}

// FSDP pack: dst[i] = TD(src[i]) for i < n, 0 for n <= i < n_pad (a unit's grad range into the padded
// reduce-scatter input)
template <typename TD>
__global__ __launch_bounds__(256) void pack_kernel(const float* __restrict__ src, TD* __restrict__ dst, size_t n,
                                                   size_t n_pad) {
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n_pad; i += (size_t)gridDim.x * 256)
    dst[i] = st_v<TD>(i < n ? src[i] : 0.f);
}

// 8 consecutive elements as fp32 (one 16-B load of bf16, two of fp32) / stored from fp32 (16-B stores). The FSDP
// passes below run on them where every pointer is 16-B aligned (the flat units are): the per-element 2-B accesses ran
// at 2-3 TB/s (profiles/r4f/summary_fsdp.txt: unpack 31 us for a 7.1 M-parameter block)
template <typename T>
__device__ __forceinline__ void ld8(const T* p, float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    const bf16x8 x = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = bf2f(x[e]);
  } else {
    const f32x4 a = reinterpret_cast<const f32x4*>(p)[0], b = reinterpret_cast<const f32x4*>(p)[1];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = a[e], v[4 + e] = b[e];
  }
}
template <typename T>
__device__ __forceinline__ void st8(T* p, const float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    bf16x8 x;
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = f2bf(v[e]);
    *reinterpret_cast<bf16x8*>(p) = x;
  } else {
    reinterpret_cast<f32x4*>(p)[0] = f32x4{v[0], v[1], v[2], v[3]};
    reinterpret_cast<f32x4*>(p)[1] = f32x4{v[4], v[5], v[6], v[7]};
  }
}
template <typename TS>
__global__ __launch_bounds__(256) void unpack8_kernel(const TS* __restrict__ src, float* __restrict__ dst,
                                                      bf16* __restrict__ dst_bf, size_t n8) {
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n8; i += (size_t)gridDim.x * 256) {
    float v[8];
    ld8(src + 8 * i, v);
    if (dst) st8(dst + 8 * i, v);
    if (dst_bf) st8(dst_bf + 8 * i, v);
  }
}
template <typename TS>
__global__ __launch_bounds__(256) void accum8_kernel(const TS* __restrict__ src, float* __restrict__ dst, size_t n8,
                                                     int accumulate) {
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n8; i += (size_t)gridDim.x * 256) {
    float v[8], d[8];
    ld8(src + 8 * i, v);
    if (accumulate) {
      ld8(dst + 8 * i, d);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = d[e] + v[e];
    }
    st8(dst + 8 * i, v);
  }
}
template <typename TD>
__global__ __launch_bounds__(256) void pack8_kernel(const float* __restrict__ src, TD* __restrict__ dst, size_t n8) {
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n8; i += (size_t)gridDim.x * 256) {
    float v[8];
    ld8(src + 8 * i, v);
    st8(dst + 8 * i, v);
  }
}
bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

int grid_for(size_t n) {
  const size_t g = (n + 255) / 256;
  return (int)(g > 4096 ? 4096 : (g == 0 ? 1 : g));
}

}  // namespace

template <typename T>
static int dlogits_accum_t(T* dl, int ldd, const T* g, int ldg, int B, int Tp, int Tv, int V, const float* alpha_dev,
                           int init, void* stream) {
  GPT2MI_REQUIRE(B > 0 && Tp > 0 && Tv > 0 && Tv <= Tp && V > 0 && ldd >= V && ldg >= V,
                 "dlogits_accum: bad shape B=%d Tp=%d Tv=%d V=%d ldd=%d ldg=%d", B, Tp, Tv, V, ldd, ldg);
  dlogits_accum_kernel<T><<<B * Tp, 256, 0, (hipStream_t)stream>>>(dl, ldd, g, ldg, Tp, Tv, V, alpha_dev, init);
  return gpt2mi::check_launch("dlogits_accum");
}

GPT2MI_EXPORT int gpt2mi_dlogits_accum(uint16_t* dl, int ldd, const uint16_t* g, int ldg, int B, int Tp, int Tv, int V,
                                       const float* alpha_dev, int init, void* stream) {
  return dlogits_accum_t<bf16>((bf16*)dl, ldd, (const bf16*)g, ldg, B, Tp, Tv, V, alpha_dev, init, stream);
}

GPT2MI_EXPORT int gpt2mi_dlogits_accum_f32(float* dl, int ldd, const float* g, int ldg, int B, int Tp, int Tv, int V,
                                           const float* alpha_dev, int init, void* stream) {
  return dlogits_accum_t<float>(dl, ldd, g, ldg, B, Tp, Tv, V, alpha_dev, init, stream);
}

template <typename TO>
static int branch_bwd_t(const float* dres, TO* out, float* dbias, int M, int C, float p, uint64_t seed, void* stream) {
  GPT2MI_REQUIRE(M > 0 && C > 0 && C % 4 == 0, "branch_bwd: C=%d must be a multiple of 4", C);
  GPT2MI_REQUIRE(p <= 0.f || (size_t)M * C < (1ull << 33), "branch_bwd: M*C=%zu exceeds the 32-bit dropout pair index",
                 (size_t)M * C);
  const int gx = (C + 255) / 256;
  const int want_y = (1024 + gx - 1) / gx;
  const int rpb = std::max(8, std::min(256, (M + want_y - 1) / want_y));
  dim3 grid(gx, (M + rpb - 1) / rpb);
  const uint32_t thr = drop_threshold(p);
  branch_bwd_kernel<TO><<<grid, 256, 0, (hipStream_t)stream>>>(dres, out, dbias, M, C, rpb, seed, thr,
                                                               p > 0.f ? 1.f / (1.f - p) : 1.f);
  return gpt2mi::check_launch("branch_bwd");
}

GPT2MI_EXPORT int gpt2mi_branch_bwd(const float* dres, uint16_t* out, float* dbias, int M, int C, float p, uint64_t seed,
                                    void* stream) {
  return branch_bwd_t<bf16>(dres, (bf16*)out, dbias, M, C, p, seed, stream);
}

GPT2MI_EXPORT int gpt2mi_branch_bwd_f32(const float* dres, float* out, float* dbias, int M, int C, float p,
                                        uint64_t seed, void* stream) {
  return branch_bwd_t<float>(dres, out, dbias, M, C, p, seed, stream);
}

GPT2MI_EXPORT int gpt2mi_cast_bf16_f32(const uint16_t* x, float* y, size_t n, void* stream) {
  cast_bf16_f32_kernel<<<grid_for(n), 256, 0, (hipStream_t)stream>>>((const bf16*)x, y, n);
  return gpt2mi::check_launch("cast_bf16_f32");
}

GPT2MI_EXPORT int gpt2mi_scale_f32(float* x, size_t n, float s, void* stream) {
  GPT2MI_REQUIRE(n % 4 == 0 && ((uintptr_t)x & 15) == 0, "scale_f32: n=%zu must be a multiple of 4, x 16-B aligned", n);
  scale_kernel<<<grid_for(n / 4), 256, 0, (hipStream_t)stream>>>(x, n / 4, s);
  return gpt2mi::check_launch("scale_f32");
}

// The FSDP passes: 8 elements per lane over the 16-B aligned prefix of multiples of 8, the element kernels over the
// rest (and over everything when a pointer is not 16-B aligned)
template <typename TS>
static void unpack_t(const TS* src, float* dst, bf16* dst_bf, size_t n, hipStream_t s) {
  const size_t n8 = al16(src) && al16(dst) && al16(dst_bf) ? n / 8 : 0;
  if (n8) unpack8_kernel<TS><<<grid_for(n8), 256, 0, s>>>(src, dst, dst_bf, n8);
  if (n > 8 * n8)
    unpack_kernel<TS><<<grid_for(n - 8 * n8), 256, 0, s>>>(src + 8 * n8, dst ? dst + 8 * n8 : nullptr,
                                                          dst_bf ? dst_bf + 8 * n8 : nullptr, n - 8 * n8);
}
template <typename TS>
static void accum_t(const TS* src, float* dst, size_t n, int accumulate, hipStream_t s) {
  const size_t n8 = al16(src) && al16(dst) ? n / 8 : 0;
  if (n8) accum8_kernel<TS><<<grid_for(n8), 256, 0, s>>>(src, dst, n8, accumulate);
  if (n > 8 * n8) accum_kernel<TS><<<grid_for(n - 8 * n8), 256, 0, s>>>(src + 8 * n8, dst + 8 * n8, n - 8 * n8, accumulate);
}
template <typename TD>
static void pack_t(const float* src, TD* dst, size_t n, size_t n_pad, hipStream_t s) {
  const size_t n8 = al16(src) && al16(dst) ? n / 8 : 0;
  if (n8) pack8_kernel<TD><<<grid_for(n8), 256, 0, s>>>(src, dst, n8);
  if (n_pad > 8 * n8)
    pack_kernel<TD><<<grid_for(n_pad - 8 * n8), 256, 0, s>>>(src + 8 * n8, dst + 8 * n8, n - 8 * n8, n_pad - 8 * n8);
}

GPT2MI_EXPORT int gpt2mi_fsdp_unpack(const void* src, int src_f32, float* dst_f32, uint16_t* dst_bf16, size_t n,
                                     void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (src_f32)
    unpack_t<float>((const float*)src, dst_f32, (bf16*)dst_bf16, n, s);
  else
    unpack_t<bf16>((const bf16*)src, dst_f32, (bf16*)dst_bf16, n, s);
  return gpt2mi::check_launch("fsdp_unpack");
}

GPT2MI_EXPORT int gpt2mi_fsdp_pack(const float* src, void* dst, int dst_f32, size_t n, size_t n_pad, void* stream) {
  GPT2MI_REQUIRE(n_pad >= n, "fsdp_pack: n_pad=%zu < n=%zu", n_pad, n);
  hipStream_t s = (hipStream_t)stream;
  if (dst_f32)
    pack_t<float>(src, (float*)dst, n, n_pad, s);
  else
    pack_t<bf16>(src, (bf16*)dst, n, n_pad, s);
  return gpt2mi::check_launch("fsdp_pack");
}

GPT2MI_EXPORT int gpt2mi_fsdp_accum(const void* src, int src_f32, float* dst, size_t n, int accumulate, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (src_f32)
    accum_t<float>((const float*)src, dst, n, accumulate, s);
  else
    accum_t<bf16>((const bf16*)src, dst, n, accumulate, s);
  return gpt2mi::check_launch("fsdp_accum");
}
