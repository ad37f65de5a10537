// LayerNorm fwd/bwd, token+position embedding fwd/bwd, bias column sums. gfx950, wave64.
//
// Replaces: K1 embedding+dropout (model.py:295-304), K2 native_layer_norm fwd/bwd
// (model.py:204,210,247), embedding_dense_backward, and the bias-grad reductions of addmm backward.
// All are HBM-bound: one wave per row, 16-B vector accesses, two-pass statistics in registers.
#include "common.h"

namespace {

constexpr int kWaves = 4;  // 256-thread blocks

// Row held in registers: lane owns elements e = VEC*(lane + 64*i), i < nv (C = 64*VEC*nv).
template <int VEC>
__device__ __forceinline__ void load_vec(const float* p, float* d) {
  if constexpr (VEC == 4) {
    f32x4 t = *reinterpret_cast<const f32x4*>(p);
    d[0] = t[0]; d[1] = t[1]; d[2] = t[2]; d[3] = t[3];
  } else if constexpr (VEC == 2) {
    float2 t = *reinterpret_cast<const float2*>(p);
    d[0] = t.x; d[1] = t.y;
  } else {
    d[0] = *p;
  }
}
template <int VEC>
__device__ __forceinline__ void store_vec(float* p, const float* d) {
  if constexpr (VEC == 4) {
    *reinterpret_cast<f32x4*>(p) = f32x4{d[0], d[1], d[2], d[3]};
  } else if constexpr (VEC == 2) {
    *reinterpret_cast<float2*>(p) = make_float2(d[0], d[1]);
  } else {
    *p = d[0];
  }
}
template <int VEC>
__device__ __forceinline__ void store_bf(bf16* p, const float* d) {
  if constexpr (VEC == 4) {
    *reinterpret_cast<bf16x4*>(p) = bf16x4{f2bf(d[0]), f2bf(d[1]), f2bf(d[2]), f2bf(d[3])};
  } else if constexpr (VEC == 2) {
    p[0] = f2bf(d[0]); p[1] = f2bf(d[1]);
  } else {
    *p = f2bf(d[0]);
  }
}
template <int VEC>
__device__ __forceinline__ void load_bf(const bf16* p, float* d) {
  if constexpr (VEC == 4) {
    bf16x4 t = *reinterpret_cast<const bf16x4*>(p);
    d[0] = bf2f(t[0]); d[1] = bf2f(t[1]); d[2] = bf2f(t[2]); d[3] = bf2f(t[3]);
  } else if constexpr (VEC == 2) {
    d[0] = bf2f(p[0]); d[1] = bf2f(p[1]);
  } else {
    d[0] = bf2f(*p);
  }
}

template <int VEC, typename T>
__device__ __forceinline__ void load_t(const T* p, float* d) {
  if constexpr (sizeof(T) == 2) load_bf<VEC>(p, d);
  else load_vec<VEC>(p, d);
}
template <int VEC, typename T>
__device__ __forceinline__ void store_t(T* p, const float* d) {
  if constexpr (sizeof(T) == 2) store_bf<VEC>(p, d);
  else store_vec<VEC>(p, d);
}
// value as stored in T (bf16 rounding), for column sums of what the next GEMM actually reads
template <typename T>
__device__ __forceinline__ float as_stored(float v) {
  if constexpr (sizeof(T) == 2) return bf2f(f2bf(v));
  else return v;
}

// ---------------------------------------------------------------------------------------------
// LayerNorm forward: y = (x-mu)*rstd*w + b, biased variance (nn.LayerNorm). x fp32 [M,C];
// y bf16 (what autocast feeds the next linear) and/or fp32; mean/rstd fp32 [M] for backward.
template <int VEC, int NV>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                     const float* __restrict__ b, bf16* __restrict__ y,
                                                     float* __restrict__ yf, float* __restrict__ mean,
                                                     float* __restrict__ rstd, int M, int C, int nv, float eps) {
  const int lane = threadIdx.x & 63;
  const int row0 = blockIdx.x * kWaves + (threadIdx.x >> 6);
  const int stride = gridDim.x * kWaves;
  for (int row = row0; row < M; row += stride) {
    const float* xr = x + (size_t)row * C;
    float v[NV * VEC];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
      {
        load_vec<VEC>(xr + VEC * (lane + 64 * i), v + VEC * i);
#pragma unroll
        for (int j = 0; j < VEC; ++j) s += v[VEC * i + j];
      }
    const float mu = wave_sum(s) / (float)C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          float d = v[VEC * i + j] - mu;
          q += d * d;
        }
    const float rs = rsqrtf(wave_sum(q) / (float)C + eps);
#pragma unroll
    for (int i = 0; i < NV; ++i)
      {
        const int e = VEC * (lane + 64 * i);
        float wv[VEC], bv[VEC], o[VEC];
        load_vec<VEC>(w + e, wv);
        load_vec<VEC>(b + e, bv);
#pragma unroll
        for (int j = 0; j < VEC; ++j) o[j] = (v[VEC * i + j] - mu) * rs * wv[j] + bv[j];
        if (y) store_bf<VEC>(y + (size_t)row * C + e, o);
        if (yf) store_vec<VEC>(yf + (size_t)row * C + e, o);
      }
    if (lane == 0) {
      mean[row] = mu;
      rstd[row] = rs;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// LayerNorm backward fused with the residual-stream gradient:
//   g = dy (bf16 [M,C], the grad of the LN output as autocast hands it back);
//   dres[m] += rstd*(g*w - mean(g*w) - xhat*mean(g*w*xhat))       (residual grad, fp32, in place)
//   dw += sum_m g*xhat ; db += sum_m g                               (LN param grads, fp32 +=)
// and, for the NEXT backward GEMM of the residual branch below this LN, emits
//   out_bf[m] = bf16(dres_new[m] * keep/(1-p))  and  dbias_out += colsum(out_bf)
// (the branch's dropout mask regenerated from (seed,row*C+c); dbias_out = that branch's bias grad).
template <int VEC, int NV, typename TG>
__global__ __launch_bounds__(256) void ln_bwd_kernel(
    const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ mean,
    const float* __restrict__ rstd, const TG* __restrict__ dy, float* __restrict__ dres,
    float* __restrict__ dw, float* __restrict__ db, TG* __restrict__ out_bf, float* __restrict__ dbias_out,
    int M, int C, int nv, uint64_t seed, uint32_t thr, float inv_keep, int dres_init) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int row0 = blockIdx.x * kWaves + wid;
  const int stride = gridDim.x * kWaves;
  float adw[NV * VEC], adb[NV * VEC], abo[NV * VEC];
#pragma unroll
  for (int i = 0; i < NV * VEC; ++i) adw[i] = adb[i] = abo[i] = 0.f;

  float wv[NV * VEC];  // gamma: the lane's columns, loop-invariant
#pragma unroll
  for (int i = 0; i < NV; ++i) load_vec<VEC>(w + VEC * (lane + 64 * i), wv + VEC * i);
  for (int row = row0; row < M; row += stride) {
    const float mu = mean[row], rs = rstd[row];
    const float* xr = x + (size_t)row * C;
    const TG* gr = dy + (size_t)row * C;
    float* dr = dres + (size_t)row * C;
    float xh[NV * VEC], g[NV * VEC], rd[NV * VEC];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {  // every load of the row first (the residual grad too): one round trip
      const int e = VEC * (lane + 64 * i);
      load_vec<VEC>(xr + e, xh + VEC * i);
      load_t<VEC, TG>(gr + e, g + VEC * i);
      if (dres_init) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) rd[VEC * i + j] = 0.f;
      } else {
        load_vec<VEC>(dr + e, rd + VEC * i);
      }
    }
#pragma unroll
    for (int i = 0; i < NV; ++i)
      {
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const int k = VEC * i + j;
          xh[k] = (xh[k] - mu) * rs;
          adw[k] += g[k] * xh[k];
          adb[k] += g[k];
          const float gw = g[k] * wv[k];
          g[k] = gw;
          s1 += gw;
          s2 += gw * xh[k];
        }
      }
    const float m1 = wave_sum(s1) / (float)C;
    const float m2 = wave_sum(s2) / (float)C;
#pragma unroll
    for (int i = 0; i < NV; ++i)
      {
        const int e = VEC * (lane + 64 * i);
        float r[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const int k = VEC * i + j;
          r[j] = rd[k] + rs * (g[k] - m1 - xh[k] * m2);
        }
        store_vec<VEC>(dr + e, r);
        if (out_bf) {
          float o[VEC];
#pragma unroll
          for (int j = 0; j < VEC; ++j) {
            float val = r[j];
            if (thr) val = drop_keep(seed, (uint64_t)row * C + e + j, thr) ? val * inv_keep : 0.f;
            o[j] = val;
          }
          store_t<VEC, TG>(out_bf + (size_t)row * C + e, o);
          if (dbias_out) {
#pragma unroll
            for (int j = 0; j < VEC; ++j) abo[VEC * i + j] += as_stored<TG>(o[j]);
          }
        }
      }
  }
  // Block reduction of the column partials through LDS, then one atomic per column per block.
  extern __shared__ float smem[];  // [kWaves][C]
  auto flush = [&](float* acc, float* dst) {
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
        for (int j = 0; j < VEC; ++j) smem[wid * C + VEC * (lane + 64 * i) + j] = acc[VEC * i + j];
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < kWaves; ++q) s += smem[q * C + c];
      atomicAdd(dst + c, s);
    }
    __syncthreads();
  };
  if (dw) flush(adw, dw);
  if (db) flush(adb, db);
  if (dbias_out && out_bf) flush(abo, dbias_out);
}

// ---------------------------------------------------------------------------------------------
// Embedding forward (model.py:295-304): x[b,t,:] = drop(wte[idx[b,t],:] + wpe[t,:]), fp32.
template <int VEC, int NV>
__global__ __launch_bounds__(256) void embed_fwd_kernel(const int64_t* __restrict__ idx, const float* __restrict__ wte,
                                                        const float* __restrict__ wpe, float* __restrict__ x,
                                                        int M, int T, int T_valid, int C, int nv, uint64_t seed,
                                                        uint32_t thr, float inv_keep) {
  const int lane = threadIdx.x & 63;
  for (int row = blockIdx.x * kWaves + (threadIdx.x >> 6); row < M; row += gridDim.x * kWaves) {
    const int t = row % T;
    if (t >= T_valid) {  // sequence padding (T rounded up to the attention tile): zero rows, no table reads
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        float z[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) z[j] = 0.f;
        store_vec<VEC>(x + (size_t)row * C + VEC * (lane + 64 * i), z);
      }
      continue;
    }
    const int64_t tok = idx[row];
#pragma unroll
    for (int i = 0; i < NV; ++i)
      {
        const int e = VEC * (lane + 64 * i);
        float a[VEC], p[VEC];
        load_vec<VEC>(wte + (size_t)tok * C + e, a);
        load_vec<VEC>(wpe + (size_t)t * C + e, p);
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          a[j] += p[j];
          if (thr) a[j] = drop_keep(seed, (uint64_t)row * C + e + j, thr) ? a[j] * inv_keep : 0.f;
        }
        store_vec<VEC>(x + (size_t)row * C + e, a);
      }
  }
}

// Embedding backward (model.py:295-304 reversed), both tables in one pass over the residual gradient, the dropout
// mask hashed once per element: one thread per (t, c) walks the batch,
//   g = dres[b,t,c]*keep/(1-p);  dwte[idx[b,t],c] += g (fp32 atomics, 256 contiguous bytes per wave instruction;
//   the tied lm_head wgrad has already written those rows);  dwpe[t,c] += sum_b g (no atomics, batch order).
// (Two kernels before: the token-table one and the position-table one each re-hashed every element: 169 + 66 us.)
__global__ __launch_bounds__(256) void embed_bwd_kernel(const int64_t* __restrict__ idx, const float* __restrict__ dres,
                                                        float* __restrict__ dwte, float* __restrict__ dwpe, int B,
                                                        int T, int T_valid, int C, uint64_t seed, uint32_t thr,
                                                        float inv_keep) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= T_valid * C) return;  // rows of wpe past T_valid are not touched (they may not exist)
  const int t = i / C, c = i % C;
  float s = 0.f;
  auto one = [&](int b, float g, int64_t tok) {
    const size_t row = (size_t)b * T + t;
    if (thr) g = drop_keep(seed, row * C + c, thr) ? g * inv_keep : 0.f;
    s += g;
    atomicAdd(dwte + (size_t)tok * C + c, g);
  };
  int b = 0;
  for (; b + 4 <= B; b += 4) {  // the four rows' loads first
    float g[4];
    int64_t tok[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t row = (size_t)(b + u) * T + t;
      g[u] = dres[row * C + c];
      tok[u] = idx[row];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) one(b + u, g[u], tok[u]);
  }
  for (; b < B; ++b) one(b, dres[((size_t)b * T + t) * C + c], idx[(size_t)b * T + t]);
  dwpe[i] += s;
}

// Column sums of a bf16 [M,N] matrix with row stride ld: db[n] += sum_m g[m,n]. Each thread owns
// 4 adjacent columns (8-B loads); blockIdx.y splits rows; one atomic per column per block-row-chunk.
template <typename TG>
__global__ __launch_bounds__(256) void colsum_kernel(const TG* __restrict__ g, float* __restrict__ db, int M,
                                                          int N, int ld, int rows_per_block) {
  const int col4 = (blockIdx.x * 64 + (threadIdx.x & 63)) * 4;
  const int sub = threadIdx.x >> 6;  // 4 row groups per block
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  if (col4 < N) {
    for (int r = r0 + sub; r < r1; r += 4) {
      float v[4];
      load_t<4, TG>(g + (size_t)r * ld + col4, v);
#pragma unroll
      for (int j = 0; j < 4; ++j) s[j] += v[j];
    }
  }
  __shared__ float red[4][256];
#pragma unroll
  for (int j = 0; j < 4; ++j) red[sub][(threadIdx.x & 63) * 4 + j] = s[j];
  __syncthreads();
  if (threadIdx.x < 256) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c < N) atomicAdd(db + c, red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x]);
  }
}

int grid_rows(int M) {
  int g = (M + kWaves - 1) / kWaves;
  return g > 8192 ? 8192 : g;
}

}  // namespace



// Row-width dispatch: VEC=4 when C%256==0, VEC=2 when C%128==0, else VEC=1 (C%64==0); NV = C/(64*VEC)
// must be one of the instantiated widths (covers C = 128..2048 incl. 768, 1024 and 1600).
#define GPT2MI_ROW_CASES(X) X(4, 1) X(4, 2) X(4, 3) X(4, 4) X(4, 5) X(4, 6) X(4, 7) X(4, 8) \
  X(2, 1) X(2, 3) X(2, 5) X(2, 7) X(1, 1) X(1, 3) X(1, 25)

static bool row_shape(int C, int* vec, int* nv) {
  if (C <= 0 || C % 64 != 0) return false;
  *vec = (C % 256 == 0) ? 4 : (C % 128 == 0) ? 2 : 1;
  *nv = C / (64 * *vec);
#define X(V, N) if (*vec == V && *nv == N) return true;
  GPT2MI_ROW_CASES(X)
#undef X
  return false;
}

GPT2MI_EXPORT int gpt2mi_layernorm_fwd(const float* x, const float* w, const float* b, uint16_t* y_bf16, float* y_f32,
                                       float* mean, float* rstd, int M, int C, float eps, void* stream) {
  int vec, nv;
  GPT2MI_REQUIRE(row_shape(C, &vec, &nv), "layernorm_fwd: unsupported C=%d", C);
  hipStream_t s = (hipStream_t)stream;
  const int g = grid_rows(M);
#define X(V, N) if (vec == V && nv == N) ln_fwd_kernel<V, N><<<g, 256, 0, s>>>(x, w, b, (bf16*)y_bf16, y_f32, mean, rstd, M, C, nv, eps);
  GPT2MI_ROW_CASES(X)
#undef X
  return gpt2mi::check_launch("layernorm_fwd");
}

template <typename TG>
static int layernorm_bwd_t(const float* x, const float* w, const float* mean, const float* rstd, const TG* dy,
                           float* dres, float* dw, float* db, TG* out, float* dbias_out, int M, int C, float p_out,
                           uint64_t seed_out, int dres_init, void* stream) {
  int vec, nv;
  GPT2MI_REQUIRE(row_shape(C, &vec, &nv), "layernorm_bwd: unsupported C=%d", C);
  GPT2MI_REQUIRE(p_out <= 0.f || (size_t)M * C < (1ull << 33),
                 "layernorm_bwd: M*C exceeds the 32-bit dropout pair index");
  hipStream_t s = (hipStream_t)stream;
#ifndef LN_BWD_MAX_BLOCKS
#define LN_BWD_MAX_BLOCKS 512
#endif
GPT2MI_PRODUCT_KNOB(LN_BWD_MAX_BLOCKS, 512);
  // the column-sum flush is one atomic per column per block: fewer blocks, fewer atomics (tools/ln_probe.py at cfg 2:
  // 2048 blocks 157-158 us, 1024 158, 512 153 — 8 waves per CU still stream at the HBM limit)
  const int g = grid_rows(M) > LN_BWD_MAX_BLOCKS ? LN_BWD_MAX_BLOCKS : grid_rows(M);
  const size_t sh = (size_t)kWaves * C * sizeof(float);
  const uint32_t thr = drop_threshold(p_out);
  const float ik = p_out > 0.f ? 1.f / (1.f - p_out) : 1.f;
#define X(V, N) if (vec == V && nv == N) ln_bwd_kernel<V, N, TG><<<g, 256, sh, s>>>(x, w, mean, rstd, dy, dres, dw, db, out, dbias_out, M, C, nv, seed_out, thr, ik, dres_init);
  GPT2MI_ROW_CASES(X)
#undef X
  return gpt2mi::check_launch("layernorm_bwd");
}

GPT2MI_EXPORT int gpt2mi_layernorm_bwd(const float* x, const float* w, const float* mean, const float* rstd,
                                       const uint16_t* dy, float* dres, float* dw, float* db, uint16_t* out_bf16,
                                       float* dbias_out, int M, int C, float p_out, uint64_t seed_out, int dres_init,
                                       void* stream) {
  return layernorm_bwd_t<bf16>(x, w, mean, rstd, (const bf16*)dy, dres, dw, db, (bf16*)out_bf16, dbias_out, M, C,
                               p_out, seed_out, dres_init, stream);
}

GPT2MI_EXPORT int gpt2mi_layernorm_bwd_f32(const float* x, const float* w, const float* mean, const float* rstd,
                                           const float* dy, float* dres, float* dw, float* db, float* out_f32,
                                           float* dbias_out, int M, int C, float p_out, uint64_t seed_out,
                                           int dres_init, void* stream) {
  return layernorm_bwd_t<float>(x, w, mean, rstd, dy, dres, dw, db, out_f32, dbias_out, M, C, p_out, seed_out,
                                dres_init, stream);
}

GPT2MI_EXPORT int gpt2mi_embed_fwd(const int64_t* idx, const float* wte, const float* wpe, float* x, int B, int T,
                                   int T_valid, int C, float p, uint64_t seed, void* stream) {
  int vec, nv;
  GPT2MI_REQUIRE(row_shape(C, &vec, &nv), "embed_fwd: unsupported C=%d", C);
  GPT2MI_REQUIRE(T_valid > 0 && T_valid <= T, "embed_fwd: T_valid=%d not in [1, T=%d]", T_valid, T);
  GPT2MI_REQUIRE(p <= 0.f || (size_t)B * T * C < (1ull << 33), "embed_fwd: B*T*C exceeds the 32-bit dropout pair index");
  hipStream_t s = (hipStream_t)stream;
  const int M = B * T;
  const uint32_t thr = drop_threshold(p);
  const float ik = p > 0.f ? 1.f / (1.f - p) : 1.f;
#define X(V, N) if (vec == V && nv == N) embed_fwd_kernel<V, N><<<grid_rows(M), 256, 0, s>>>(idx, wte, wpe, x, M, T, T_valid, C, nv, seed, thr, ik);
  GPT2MI_ROW_CASES(X)
#undef X
  return gpt2mi::check_launch("embed_fwd");
}

GPT2MI_EXPORT int gpt2mi_embed_bwd(const int64_t* idx, const float* dres, float* dwte, float* dwpe, int B, int T,
                                   int T_valid, int C, float p, uint64_t seed, void* stream) {
  GPT2MI_REQUIRE(T_valid > 0 && T_valid <= T, "embed_bwd: T_valid=%d not in [1, T=%d]", T_valid, T);
  hipStream_t s = (hipStream_t)stream;
  const uint32_t thr = drop_threshold(p);
  const float ik = p > 0.f ? 1.f / (1.f - p) : 1.f;
  embed_bwd_kernel<<<(T_valid * C + 255) / 256, 256, 0, s>>>(idx, dres, dwte, dwpe, B, T, T_valid, C, seed, thr, ik);
  return gpt2mi::check_launch("embed_bwd");
}

template <typename TG>
static int colsum_t(const TG* g, float* db, int M, int N, int ld, void* stream) {
  GPT2MI_REQUIRE(N % 4 == 0 && ld % 4 == 0, "colsum: N=%d and ld=%d must be multiples of 4", N, ld);
  hipStream_t s = (hipStream_t)stream;
  // >= ~1024 blocks (the 32-token partial sums of the attention backward are only M/32 rows)
  const int gx = (N + 255) / 256;
  const int want_y = (1024 + gx - 1) / gx;
  const int rpb = std::max(8, std::min(256, (M + want_y - 1) / want_y));
  dim3 grid(gx, (M + rpb - 1) / rpb);
  colsum_kernel<TG><<<grid, 256, 0, s>>>(g, db, M, N, ld, rpb);
  return gpt2mi::check_launch("colsum");
}

GPT2MI_EXPORT int gpt2mi_colsum_bf16(const uint16_t* g, float* db, int M, int N, int ld, void* stream) {
  return colsum_t<bf16>((const bf16*)g, db, M, N, ld, stream);
}

GPT2MI_EXPORT int gpt2mi_colsum_f32(const float* g, float* db, int M, int N, int ld, void* stream) {
  return colsum_t<float>(g, db, M, N, ld, stream);
}
