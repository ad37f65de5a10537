// fp32 mode: the reference model run WITHOUT torch.autocast (model.py in plain fp32 — the CPU
// trajectory of SURVEY §6 and the north star's "fp32-mode loss within 1e-4" gate).
//
// Same entry points and fused epilogues as the bf16 path (gemm.hip / attention.hip), with every
// activation, weight and product in fp32:
//  * GEMM: v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulation — gfx950 has no
//    reduced-precision fp32 MFMA mode), 128x128x16 block tile, 4 waves of 64x64, register-staged
//    double-buffered LDS. Operand images are k-major [16][128+16] floats: a fragment read is 16
//    consecutive floats on each of 4 k-rows whose bank offsets differ by 16 -> conflict-free.
//    As in the bf16 kernels the MFMA is issued as D^T = B.A^T so a lane owns 4 consecutive
//    output columns (16-B epilogue stores, shared epilogue code with the bf16 kernels).
//  * attention: flash-style fwd / dK-dV / dQ kernels on the VALU (fp32 FMA): four lanes per
//    query (key) row, each owning 16 of the 64 head dims, scores reduced with two xor-shuffles;
//    K/V (Q/dO) tiles of 64 rows staged in LDS and broadcast to the 16 rows of a wave.
//    Dropout masks are the bf16 kernel's (seed, head, query-pair, key) hash, so both precisions
//    drop the same probabilities.
#include "common.h"
#include "gemm_common.h"
#include "gpt2mi.h"

namespace {

// ============================== GEMM ==============================================================
constexpr int FBM = 128, FBN = 128, FBK = 16;
constexpr int kFThreads = 256;
constexpr int kFLd = FBM + 16;                 // floats per k-row of an operand image
constexpr int kFOp = FBK * kFLd;               // floats per operand image
constexpr int kFStage = 2 * kFOp;              // A + B

// Loads one operand K-tile into 2 float4 registers per thread.
//   TRANS=0: src[row][k] (k contiguous): thread -> (row id>>2, k 4*(id&3))
//   TRANS=1: src[k][row] (row contiguous): thread -> (k id>>5, row 4*(id&31))
template <bool TRANS>
__device__ __forceinline__ void f_load(f32x4* r, const float* __restrict__ src, int ld, int row0, int k0, int rmax) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int id = threadIdx.x + kFThreads * i;
    const float* p;
    if constexpr (!TRANS) {
      p = src + (size_t)min(row0 + (id >> 2), rmax) * ld + k0 + 4 * (id & 3);
    } else {
      p = src + (size_t)(k0 + (id >> 5)) * ld + min(row0 + 4 * (id & 31), rmax - 3);
    }
    r[i] = *reinterpret_cast<const f32x4*>(p);
  }
}
template <bool TRANS>
__device__ __forceinline__ void f_store(float* img, const f32x4* r) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int id = threadIdx.x + kFThreads * i;
    if constexpr (!TRANS) {
      const int row = id >> 2, k = 4 * (id & 3);
#pragma unroll
      for (int j = 0; j < 4; ++j) img[(k + j) * kFLd + row] = r[i][j];
    } else {
      *reinterpret_cast<f32x4*>(img + (id >> 5) * kFLd + 4 * (id & 31)) = r[i];
    }
  }
}

template <bool A_T, bool B_T, int EPI>
__global__ __launch_bounds__(kFThreads, 2) void gemm_f32_kernel(GemmParams P, const float* __restrict__ A,
                                                                const float* __restrict__ B) {
  __shared__ __attribute__((aligned(16))) float smem[2 * kFStage];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles_m = (P.M + FBM - 1) / FBM, tiles_n = (P.N + FBN - 1) / FBN;
  const int pid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tm = pid / tiles_n, tn = pid % tiles_n;
  const int m0 = tm * FBM, n0 = tn * FBN;
  const int kbeg = blockIdx.z * P.k_per_split;
  const int nk = P.k_per_split / FBK;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  f32x4 ra[2], rb[2];
  f_load<A_T>(ra, A, P.lda, m0, kbeg, P.M - 1);
  f_load<B_T>(rb, B, P.ldb, n0, kbeg, P.N - 1);
  f_store<A_T>(smem, ra);
  f_store<B_T>(smem + kFOp, rb);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const float* As = smem + (kt & 1) * kFStage;
    const float* Bs = As + kFOp;
    if (kt + 1 < nk) {
      f_load<A_T>(ra, A, P.lda, m0, kbeg + (kt + 1) * FBK, P.M - 1);
      f_load<B_T>(rb, B, P.ldb, n0, kbeg + (kt + 1) * FBK, P.N - 1);
    }
#pragma unroll
    for (int kk = 0; kk < FBK / 4; ++kk) {
      const int krow = (4 * kk + (lane >> 4)) * kFLd + (lane & 15);
      float af[4], bfr[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        af[f] = As[krow + wm * 64 + 16 * f];
        bfr[f] = Bs[krow + wn * 64 + 16 * f];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      float* nxt = smem + ((kt + 1) & 1) * kFStage;
      f_store<A_T>(nxt, ra);
      f_store<B_T>(nxt + kFOp, rb);
    }
    __syncthreads();
  }

  float alpha = P.alpha;
  if (P.alpha_dev) alpha *= P.alpha_dev[0];
  // acc[i][j][r] = C[m0 + wm*64 + 16i + (l&15)][n0 + wn*64 + 16j + 4(l>>4) + r]
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int gm = m0 + wm * 64 + 16 * i + (lane & 15);
    if (gm >= P.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int gn = n0 + wn * 64 + 16 * j + 4 * (lane >> 4);
      if (gn >= P.N) continue;
      f32x4 v;
      f32x4 b = (P.bias && EPI != EPI_GELU_BWD) ? *reinterpret_cast<const f32x4*>(P.bias + gn)
                                                 : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] * alpha + b[r];
      epilogue_store<EPI, float>(P, gm, gn, v);
    }
  }
}

template <bool A_T, bool B_T, int EPI>
int f_launch(const GemmParams& P, const float* A, const float* B, int splits, hipStream_t s) {
  dim3 grid(((P.M + FBM - 1) / FBM) * ((P.N + FBN - 1) / FBN), 1, splits);
  gemm_f32_kernel<A_T, B_T, EPI><<<grid, kFThreads, 0, s>>>(P, A, B);
  return gpt2mi::check_launch("gemm_f32");
}

// ============================== attention =========================================================
constexpr int HD = 64;       // head dim
constexpr int RT = 64;       // rows (queries or keys) per tile / per workgroup
constexpr int kAThreads = 256;  // 4 lanes per row

__device__ __forceinline__ bool attn_keep(uint32_t s32, uint32_t kx, int bh, int T, int q, int key, uint32_t thr) {
  const uint32_t hh = drop_hash(s32, kx, ((uint32_t)bh * T + (q & ~16)) * (uint32_t)T + key);
  return drop_keep16(hh, (q >> 4) & 1, thr);
}

// sum over the 4 lanes of a row (lanes 4r..4r+3 of a wave)
__device__ __forceinline__ float quad_sum(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  return v;
}

// [64 rows][64] fp32 tile of a strided matrix -> LDS (4 float4 per thread)
__device__ __forceinline__ void a_tile(float* dst, const float* __restrict__ src, size_t ld) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int id = threadIdx.x + kAThreads * i;
    *reinterpret_cast<f32x4*>(dst + (id >> 4) * HD + 4 * (id & 15)) =
        *reinterpret_cast<const f32x4*>(src + (size_t)(id >> 4) * ld + 4 * (id & 15));
  }
}

__device__ __forceinline__ void ld16(float* d, const float* p) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x4 t = *reinterpret_cast<const f32x4*>(p + 4 * i);
    d[4 * i] = t[0]; d[4 * i + 1] = t[1]; d[4 * i + 2] = t[2]; d[4 * i + 3] = t[3];
  }
}
__device__ __forceinline__ void st16(float* p, const float* d, float scale) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
    *reinterpret_cast<f32x4*>(p + 4 * i) = f32x4{d[4 * i] * scale, d[4 * i + 1] * scale, d[4 * i + 2] * scale,
                                                 d[4 * i + 3] * scale};
}

// Forward: workgroup = (64 queries, one head); out = softmax(q k^T * scale, causal) (dropout) v.
__global__ __launch_bounds__(kAThreads) void attn_fwd_f32_kernel(const float* __restrict__ qkv, float* __restrict__ out,
                                                                 float* __restrict__ lse, int T, int H, float scale,
                                                                 uint64_t seed, uint32_t thr, float inv_keep) {
  __shared__ __attribute__((aligned(16))) float kv[2][RT * HD];
  const int qt = gridDim.x - 1 - blockIdx.x, bh = blockIdx.y, b = bh / H, h = bh % H;
  const int C = H * HD;
  const size_t ld = 3 * (size_t)C;
  const float* base = qkv + (size_t)b * T * ld;
  const int r = threadIdx.x >> 2, qd = threadIdx.x & 3;
  const int q = qt * RT + r;
  const uint32_t s32 = seed32(seed), kx = seed_kx(seed);
  float qv[16], acc[16];
  ld16(qv, base + (size_t)q * ld + h * HD + 16 * qd);
#pragma unroll
  for (int d = 0; d < 16; ++d) acc[d] = 0.f;
  float m = -INFINITY, l = 0.f;
  for (int kt = 0; kt <= qt; ++kt) {
    __syncthreads();
    a_tile(kv[0], base + (size_t)kt * RT * ld + C + h * HD, ld);
    a_tile(kv[1], base + (size_t)kt * RT * ld + 2 * C + h * HD, ld);
    __syncthreads();
    // online softmax over chunks of 16 keys (fully unrolled: the scores stay in registers)
#pragma unroll 1
    for (int jc = 0; jc < RT; jc += 16) {
      float s[16];
      float tmax = -INFINITY;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const float* kr = kv[0] + (jc + j) * HD + 16 * qd;
        float p = 0.f;
#pragma unroll
        for (int d = 0; d < 16; ++d) p += qv[d] * kr[d];
        p = quad_sum(p) * scale;
        if (kt * RT + jc + j > q) p = -INFINITY;
        s[j] = p;
        tmax = fmaxf(tmax, p);
      }
      const float mn = fmaxf(m, tmax);
      if (mn == -INFINITY) continue;  // whole chunk masked and nothing seen yet: cannot happen at jc = 0
      const float corr = __expf(m - mn);
      l *= corr;
#pragma unroll
      for (int d = 0; d < 16; ++d) acc[d] *= corr;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        float p = __expf(s[j] - mn);
        l += p;
        if (thr) p = attn_keep(s32, kx, bh, T, q, kt * RT + jc + j, thr) ? p * inv_keep : 0.f;
        const float* vr = kv[1] + (jc + j) * HD + 16 * qd;
#pragma unroll
        for (int d = 0; d < 16; ++d) acc[d] += p * vr[d];
      }
      m = mn;
    }
  }
  st16(out + ((size_t)b * T + q) * C + h * HD + 16 * qd, acc, 1.f / l);
  if (qd == 0) lse[(size_t)bh * T + q] = m + __logf(l);
}

// delta[bh, q] = sum_d dout[q, h, d] * out[q, h, d]
__global__ __launch_bounds__(256) void attn_delta_f32_kernel(const float* __restrict__ out, const float* __restrict__ dout,
                                                             float* __restrict__ delta, int B, int T, int H) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);  // (b, t, h) row
  if (i >= B * T * H) return;
  const int lane = threadIdx.x & 63;
  const int h = i % H, bt = i / H, b = bt / T, t = bt % T;
  const size_t off = (size_t)bt * H * HD + h * HD + lane;
  const float v = wave_sum(out[off] * dout[off]);
  if (lane == 0) delta[((size_t)b * H + h) * T + t] = v;
}

// dK, dV: workgroup = (64 keys, one head), loops over the query tiles at or after its key tile.
__global__ __launch_bounds__(kAThreads) void attn_bwd_dkdv_f32_kernel(
    const float* __restrict__ qkv, const float* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, float* __restrict__ dqkv, int T, int H, float scale, uint64_t seed, uint32_t thr,
    float inv_keep) {
  __shared__ __attribute__((aligned(16))) float qo[2][RT * HD];
  __shared__ float sl[RT], sd[RT];
  const int kt = blockIdx.x, bh = blockIdx.y, b = bh / H, h = bh % H;
  const int C = H * HD;
  const size_t ld = 3 * (size_t)C;
  const float* base = qkv + (size_t)b * T * ld;
  const float* dbase = dout + (size_t)b * T * C;
  const int r = threadIdx.x >> 2, qd = threadIdx.x & 3;
  const int key = kt * RT + r;
  const uint32_t s32 = seed32(seed), kx = seed_kx(seed);
  float kr[16], vr[16], dk[16], dv[16];
  ld16(kr, base + (size_t)key * ld + C + h * HD + 16 * qd);
  ld16(vr, base + (size_t)key * ld + 2 * C + h * HD + 16 * qd);
#pragma unroll
  for (int d = 0; d < 16; ++d) dk[d] = dv[d] = 0.f;
  const int nqt = T / RT;
  for (int qt = kt; qt < nqt; ++qt) {
    __syncthreads();
    a_tile(qo[0], base + (size_t)qt * RT * ld + h * HD, ld);
    a_tile(qo[1], dbase + (size_t)qt * RT * C + h * HD, C);
    if (threadIdx.x < RT) {
      sl[threadIdx.x] = lse[(size_t)bh * T + qt * RT + threadIdx.x];
      sd[threadIdx.x] = delta[(size_t)bh * T + qt * RT + threadIdx.x];
    }
    __syncthreads();
#pragma unroll 4
    for (int i = 0; i < RT; ++i) {
      const int q = qt * RT + i;
      if (q < key) continue;  // row-uniform within the 4 lanes
      const float* qr = qo[0] + i * HD + 16 * qd;
      const float* gr = qo[1] + i * HD + 16 * qd;
      float s = 0.f, dp = 0.f;
#pragma unroll
      for (int d = 0; d < 16; ++d) {
        s += qr[d] * kr[d];
        dp += gr[d] * vr[d];
      }
      s = quad_sum(s) * scale;
      dp = quad_sum(dp);
      const float p = __expf(s - sl[i]);
      float pd = p;
      if (thr) {
        const bool keep = attn_keep(s32, kx, bh, T, q, key, thr);
        pd = keep ? p * inv_keep : 0.f;
        dp = keep ? dp * inv_keep : 0.f;
      }
      const float ds = p * (dp - sd[i]) * scale;
#pragma unroll
      for (int d = 0; d < 16; ++d) {
        dv[d] += pd * gr[d];
        dk[d] += ds * qr[d];
      }
    }
  }
  float* orow = dqkv + ((size_t)b * T + key) * ld + h * HD + 16 * qd;
  st16(orow + C, dk, 1.f);
  st16(orow + 2 * C, dv, 1.f);
}

// dQ: workgroup = (64 queries, one head), loops over the key tiles at or before its query tile.
__global__ __launch_bounds__(kAThreads) void attn_bwd_dq_f32_kernel(
    const float* __restrict__ qkv, const float* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, float* __restrict__ dqkv, int T, int H, float scale, uint64_t seed, uint32_t thr,
    float inv_keep) {
  __shared__ __attribute__((aligned(16))) float kv[2][RT * HD];
  const int qt = gridDim.x - 1 - blockIdx.x, bh = blockIdx.y, b = bh / H, h = bh % H;
  const int C = H * HD;
  const size_t ld = 3 * (size_t)C;
  const float* base = qkv + (size_t)b * T * ld;
  const int r = threadIdx.x >> 2, qd = threadIdx.x & 3;
  const int q = qt * RT + r;
  const uint32_t s32 = seed32(seed), kx = seed_kx(seed);
  float qv[16], gv[16], dq[16];
  ld16(qv, base + (size_t)q * ld + h * HD + 16 * qd);
  ld16(gv, dout + ((size_t)b * T + q) * C + h * HD + 16 * qd);
#pragma unroll
  for (int d = 0; d < 16; ++d) dq[d] = 0.f;
  const float lq = lse[(size_t)bh * T + q], dl = delta[(size_t)bh * T + q];
  for (int kt = 0; kt <= qt; ++kt) {
    __syncthreads();
    a_tile(kv[0], base + (size_t)kt * RT * ld + C + h * HD, ld);
    a_tile(kv[1], base + (size_t)kt * RT * ld + 2 * C + h * HD, ld);
    __syncthreads();
#pragma unroll 4
    for (int j = 0; j < RT; ++j) {
      const int key = kt * RT + j;
      if (key > q) break;  // row-uniform
      const float* kr = kv[0] + j * HD + 16 * qd;
      const float* vr = kv[1] + j * HD + 16 * qd;
      float s = 0.f, dp = 0.f;
#pragma unroll
      for (int d = 0; d < 16; ++d) {
        s += qv[d] * kr[d];
        dp += gv[d] * vr[d];
      }
      s = quad_sum(s) * scale;
      dp = quad_sum(dp);
      const float p = __expf(s - lq);
      if (thr) dp = attn_keep(s32, kx, bh, T, q, key, thr) ? dp * inv_keep : 0.f;
      const float ds = p * (dp - dl) * scale;
#pragma unroll
      for (int d = 0; d < 16; ++d) dq[d] += ds * kr[d];
    }
  }
  st16(dqkv + ((size_t)b * T + q) * ld + h * HD + 16 * qd, dq, 1.f);
}

}  // namespace

// fp32 GEMM: same contract as gpt2mi_gemm (layouts, epilogues, alpha, dropout) with fp32 A, B and fp32
// outputs everywhere (C and aux of the BF16/GELU/GELU_BWD epilogues are fp32 here).
GPT2MI_EXPORT int gpt2mi_gemm_f32(int layout, int epilogue, int M, int N, int K, const float* A, int lda, const float* B,
                                  int ldb, void* C, int ldc, const float* bias, const float* resid, float* aux,
                                  int ldaux, float alpha, const float* alpha_dev, int accumulate, int splits,
                                  float p_drop, uint64_t seed, float* dbias, void* stream) {
  GPT2MI_REQUIRE(dbias == nullptr || ((epilogue == EPI_BF16 || epilogue == EPI_GELU_BWD) && layout <= 1),
                 "gemm_f32: dbias (fused column sum) needs the BF16 or GELU_BWD epilogue of layout 0/1");
  if (dbias) {
    const int rc = gpt2mi_gemm_f32(layout, epilogue, M, N, K, A, lda, B, ldb, C, ldc, bias, resid, aux, ldaux, alpha,
                                   alpha_dev, accumulate, splits, p_drop, seed, nullptr, stream);
    if (rc) return rc;
    return gpt2mi_colsum_f32((const float*)C, dbias, M, N, ldc, stream);
  }
  GPT2MI_REQUIRE(M > 0 && N >= 4 && N % 4 == 0 && K % FBK == 0, "gemm_f32: need N=%d %% 4 == 0 and K=%d %% 16 == 0",
                 N, K);
  GPT2MI_REQUIRE(p_drop <= 0.f || (size_t)M * N < (1ull << 33),
                 "gemm_f32: M*N=%zu exceeds the 32-bit dropout pair index", (size_t)M * N);
  GPT2MI_REQUIRE(layout >= 0 && layout <= 2, "gemm_f32: bad layout %d", layout);
  GPT2MI_REQUIRE(layout != 2 || M >= 4, "gemm_f32: wgrad needs M >= 4");
  GPT2MI_REQUIRE(splits >= 1 && K % (FBK * splits) == 0, "gemm_f32: K=%d must be a multiple of 16*splits(%d)", K, splits);
  GPT2MI_REQUIRE(splits == 1 || epilogue == EPI_ATOMIC, "gemm_f32: split-K needs the atomic epilogue");
  GPT2MI_REQUIRE(ldc % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0 && (ldaux % 4 == 0 || aux == nullptr),
                 "gemm_f32: leading dimensions must be multiples of 4");
  GemmParams P{};
  P.C = C;
  P.bias = bias;
  P.resid = resid;
  P.aux = aux;
  P.alpha_dev = alpha_dev;
  P.M = M; P.N = N; P.K = K;
  P.lda = lda; P.ldb = ldb; P.ldc = ldc; P.ldaux = ldaux;
  P.k_per_split = K / splits;
  P.alpha = alpha;
  P.accumulate = accumulate;
  P.seed = seed;
  P.thr = drop_threshold(p_drop);
  P.inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  hipStream_t s = (hipStream_t)stream;
  switch (layout * 16 + epilogue) {
    case 0 * 16 + EPI_BF16: return f_launch<false, false, EPI_BF16>(P, A, B, splits, s);
    case 0 * 16 + EPI_F32: return f_launch<false, false, EPI_F32>(P, A, B, splits, s);
    case 0 * 16 + EPI_RESID: return f_launch<false, false, EPI_RESID>(P, A, B, splits, s);
    case 0 * 16 + EPI_GELU: return f_launch<false, false, EPI_GELU>(P, A, B, splits, s);
    case 1 * 16 + EPI_BF16: return f_launch<false, true, EPI_BF16>(P, A, B, splits, s);
    case 1 * 16 + EPI_F32: return f_launch<false, true, EPI_F32>(P, A, B, splits, s);
    case 1 * 16 + EPI_GELU_BWD: return f_launch<false, true, EPI_GELU_BWD>(P, A, B, splits, s);
    case 2 * 16 + EPI_F32: return f_launch<true, true, EPI_F32>(P, A, B, splits, s);
    case 2 * 16 + EPI_ATOMIC: return f_launch<true, true, EPI_ATOMIC>(P, A, B, splits, s);
    default:
      gpt2mi::set_error("gemm_f32: unsupported layout %d / epilogue %d combination", layout, epilogue);
      return 22;
  }
}

GPT2MI_EXPORT int gpt2mi_attn_fwd_f32(const float* qkv, float* out, float* lse, int B, int T, int H, int head_dim,
                                      float p_drop, uint64_t seed, void* stream) {
  GPT2MI_REQUIRE(head_dim == HD, "attn_fwd_f32: head_dim=%d (only 64 is built)", head_dim);
  GPT2MI_REQUIRE(p_drop <= 0.f || (size_t)B * H * T * T < (1ull << 32),
                 "attn_fwd_f32: B*H*T*T exceeds the 32-bit dropout hash index");
  GPT2MI_REQUIRE(T % RT == 0 && T > 0, "attn_fwd_f32: T=%d must be a multiple of 64", T);
  attn_fwd_f32_kernel<<<dim3(T / RT, B * H), kAThreads, 0, (hipStream_t)stream>>>(
      qkv, out, lse, T, H, 1.f / sqrtf((float)head_dim), seed, drop_threshold(p_drop),
      p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f);
  return gpt2mi::check_launch("attn_fwd_f32");
}

GPT2MI_EXPORT int gpt2mi_attn_bwd_f32(const float* qkv, const float* out, const float* dout, const float* lse,
                                      float* delta, float* dqkv, float* dqkv_colsum, int B, int T, int H,
                                      int head_dim, float p_drop, uint64_t seed, void* stream) {
  GPT2MI_REQUIRE(head_dim == HD, "attn_bwd_f32: head_dim=%d (only 64 is built)", head_dim);
  GPT2MI_REQUIRE(p_drop <= 0.f || (size_t)B * H * T * T < (1ull << 32),
                 "attn_bwd_f32: B*H*T*T exceeds the 32-bit dropout hash index");
  GPT2MI_REQUIRE(dqkv_colsum == nullptr, "attn_bwd_f32: the fused bias-gradient partials are bf16-path only");
  GPT2MI_REQUIRE(T % RT == 0 && T > 0, "attn_bwd_f32: T=%d must be a multiple of 64", T);
  hipStream_t s = (hipStream_t)stream;
  const float scale = 1.f / sqrtf((float)head_dim);
  const uint32_t thr = drop_threshold(p_drop);
  const float ik = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  attn_delta_f32_kernel<<<(B * T * H + 3) / 4, 256, 0, s>>>(out, dout, delta, B, T, H);
  int rc = gpt2mi::check_launch("attn_delta_f32");
  if (rc) return rc;
  attn_bwd_dkdv_f32_kernel<<<dim3(T / RT, B * H), kAThreads, 0, s>>>(qkv, dout, lse, delta, dqkv, T, H, scale, seed,
                                                                      thr, ik);
  rc = gpt2mi::check_launch("attn_bwd_dkdv_f32");
  if (rc) return rc;
  attn_bwd_dq_f32_kernel<<<dim3(T / RT, B * H), kAThreads, 0, s>>>(qkv, dout, lse, delta, dqkv, T, H, scale, seed, thr,
                                                                    ik);
  return gpt2mi::check_launch("attn_bwd_dq_f32");
}
