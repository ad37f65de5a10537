// bf16 MFMA GEMM for gfx950 with fused epilogues — every Linear of the GPT-2 step.
//
//   C[m,n] (op)= epilogue( alpha * sum_k A(m,k) * B(n,k) )
//
// Operand layouts (template):
//   A_T=0: A stored [M][K] (row m, k contiguous)     A_T=1: A stored [K][M] (m contiguous)
//   B_T=0: B stored [N][K] (nn.Linear weight [out][in]) B_T=1: B stored [K][N]
// forward (x @ W^T)       : A_T=0, B_T=0   (model.py:95-96,174-177,326 under autocast bf16)
// dgrad   (dY @ W)        : A_T=0, B_T=1
// wgrad   (dY^T @ X)      : A_T=1, B_T=1   (split-K over tokens, fp32 atomics into the grad arena)
//
// Structure: 256 threads = 4 waves (2x2), 128x128 block tile, BK=64, v_mfma_f32_16x16x32_bf16,
// register-staged global->LDS double buffer (next tile's loads issued before the MFMAs, written
// after them, one barrier per K-tile). LDS images:
//   k-contiguous operand : [rows][64] bf16 (128-B rows), 16-B chunk c stored at c ^ (row & 7)
//                          -> fragment reads are conflict-free ds_read_b128;
//   m-contiguous operand : [64 k][128] bf16 (256-B rows), chunk c stored at c ^ 2*((k&3)|((k>>3&1)<<2))
//                          -> fragments by two conflict-free ds_read_b64_tr_b16 (hardware transpose).
// Epilogue: accumulators -> LDS (fp32, padded rows) -> row-contiguous 16-B chunks -> fused op -> HBM.
#include "common.h"
#include "gemm_common.h"
#include "gpt2mi.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int kThreads = 256;
constexpr int kStageBytes = (BM + BN) * BK * 2;           // 32 KiB
constexpr int kEpiLd = BN + 4;                            // fp32 epilogue row stride (floats)
constexpr int kLdsBytes = (2 * kStageBytes > BM * kEpiLd * 4) ? 2 * kStageBytes : BM * kEpiLd * 4;

__device__ __forceinline__ int kc_off(int row, int chunk) { return row * 128 + 16 * (chunk ^ (row & 7)); }
__device__ __forceinline__ int mc_swz(int k) { return 2 * ((k & 3) | (((k >> 3) & 1) << 2)); }
__device__ __forceinline__ int mc_off(int k, int chunk) { return k * 256 + 16 * ((chunk ^ mc_swz(k)) & 15); }

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ bf16x8 read_frag_kc(const char* base, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(base + kc_off(row, chunk));
}

// tr read of the m-contiguous image: lane (g=l>>4, q=(l&15)>>2, p=l&3) gives A[m0+(l&15)][k0+8g+j]
__device__ __forceinline__ bf16x8 read_frag_mc(const char* base, int k0, int m0, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int k1 = k0 + 8 * g + q;
  const int chunk = (m0 >> 3) + (p >> 1);
  const int off1 = mc_off(k1, chunk) + 8 * (p & 1);
  const int off2 = mc_off(k1 + 4, chunk) + 8 * (p & 1);
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + off1));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + off2));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

// Tile loader: 4 x 16-B chunks per thread per operand per K-tile.
template <bool TRANS, int ROWS>
struct Loader {
  // TRANS=0: tile is [ROWS][BK] from src[row*ld + k]; TRANS=1: tile is [BK][ROWS] from src[k*ld + row]
  __device__ __forceinline__ static void load(u32x4* r, const bf16* src, int ld, int row0, int k0, int rmax) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int id = threadIdx.x + kThreads * i;
      const bf16* p;
      if constexpr (!TRANS) {
        p = src + (size_t)min(row0 + id / 8, rmax) * ld + k0 + 8 * (id % 8);
      } else {  // partial last tile (extent % 128 == 64): clamp the 8-column chunk into the row (rmax+1 is a
                // multiple of 64); the clamped columns only feed outputs the epilogue discards
        p = src + (size_t)(k0 + id / (ROWS / 8)) * ld + min(row0 + 8 * (id % (ROWS / 8)), rmax - 7);
      }
      r[i] = *reinterpret_cast<const u32x4*>(p);
    }
  }
  __device__ __forceinline__ static void store(char* base, const u32x4* r) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int id = threadIdx.x + kThreads * i;
      int off;
      if constexpr (!TRANS) {
        off = kc_off(id / 8, id % 8);
      } else {
        off = mc_off(id / (ROWS / 8), id % (ROWS / 8));
      }
      *reinterpret_cast<u32x4*>(base + off) = r[i];
    }
  }
};

template <bool A_T, bool B_T, int EPI>
__global__ __launch_bounds__(kThreads, 2) void gemm_kernel(GemmParams P) {
  __shared__ __attribute__((aligned(16))) char smem[kLdsBytes];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  // tile scheduling: XCD-contiguous ranges, grouped-M ordering for L2 reuse
  const int tiles_m = (P.M + BM - 1) / BM, tiles_n = (P.N + BN - 1) / BN;
  const int ntiles = tiles_m * tiles_n;
  const int pid = xcd_remap(blockIdx.x, ntiles);
  constexpr int GM = 8;
  const int group = pid / (GM * tiles_n);
  const int first_m = group * GM;
  const int gsz = min(tiles_m - first_m, GM);
  const int tm = first_m + (pid % (GM * tiles_n)) % gsz;
  const int tn = (pid % (GM * tiles_n)) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = blockIdx.z * P.k_per_split;
  const int nk = P.k_per_split / BK;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 ra[4], rb[4];
  using LA = Loader<A_T, BM>;
  using LB = Loader<B_T, BN>;
  LA::load(ra, P.A, P.lda, m0, kbeg, P.M - 1);
  LB::load(rb, P.B, P.ldb, n0, kbeg, P.N - 1);
  LA::store(smem, ra);
  LB::store(smem + BM * BK * 2, rb);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const char* As = smem + cur * kStageBytes;
    const char* Bs = As + BM * BK * 2;
    if (kt + 1 < nk) {
      LA::load(ra, P.A, P.lda, m0, kbeg + (kt + 1) * BK, P.M - 1);
      LB::load(rb, P.B, P.ldb, n0, kbeg + (kt + 1) * BK, P.N - 1);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        if constexpr (!A_T) af[f] = read_frag_kc(As, wm * 64 + 16 * f + (lane & 15), 4 * kk + (lane >> 4));
        else af[f] = read_frag_mc(As, 32 * kk, wm * 64 + 16 * f, lane);
        if constexpr (!B_T) bfr[f] = read_frag_kc(Bs, wn * 64 + 16 * f + (lane & 15), 4 * kk + (lane >> 4));
        else bfr[f] = read_frag_mc(Bs, 32 * kk, wn * 64 + 16 * f, lane);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      char* nxt = smem + (cur ^ 1) * kStageBytes;
      LA::store(nxt, ra);
      LB::store(nxt + BM * BK * 2, rb);
    }
    __syncthreads();
  }

  // ---- epilogue: accumulators -> LDS fp32 [BM][kEpiLd] ----
  float* ep = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * 64 + 16 * i + 4 * (lane >> 4) + r;
        const int col = wn * 64 + 16 * j + (lane & 15);
        ep[row * kEpiLd + col] = acc[i][j][r];
      }
  __syncthreads();

  float alpha = P.alpha;
  if (P.alpha_dev) alpha *= P.alpha_dev[0];

  if constexpr (EPI == EPI_ATOMIC) {
    float* C = reinterpret_cast<float*>(P.C);
#pragma unroll 4
    for (int it = 0; it < (BM * BN) / kThreads; ++it) {
      const int id = threadIdx.x + kThreads * it;
      const int row = id / BN, col = id % BN;
      if (m0 + row >= P.M || n0 + col >= P.N) continue;
      atomicAdd(C + (size_t)(m0 + row) * P.ldc + n0 + col, alpha * ep[row * kEpiLd + col]);
    }
    return;
  } else {
#pragma unroll 2
    for (int it = 0; it < (BM * BN) / (4 * kThreads); ++it) {
      const int id = threadIdx.x + kThreads * it;
      const int row = id / (BN / 4), c4 = 4 * (id % (BN / 4));
      const int gm = m0 + row, gn = n0 + c4;
      if (gm >= P.M || gn >= P.N) continue;
      f32x4 v = *reinterpret_cast<const f32x4*>(ep + row * kEpiLd + c4);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] *= alpha;
      if (P.bias && EPI != EPI_GELU_BWD) {
        f32x4 b = *reinterpret_cast<const f32x4*>(P.bias + gn);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] += b[j];
      }
      epilogue_store<EPI>(P, gm, gn, v);
    }
  }
}

template <bool A_T, bool B_T, int EPI>
int launch(const GemmParams& P, int splits, hipStream_t s) {
  dim3 grid(((P.M + BM - 1) / BM) * ((P.N + BN - 1) / BN), 1, splits);
  gemm_kernel<A_T, B_T, EPI><<<grid, kThreads, 0, s>>>(P);
  return gpt2mi::check_launch("gemm");
}

}  // namespace

// layout: 0 = forward (A[M][K], B[N][K]); 1 = dgrad (A[M][K], B[K][N]); 2 = wgrad (A[K][M], B[K][N]).
GPT2MI_EXPORT int gpt2mi_gemm(int layout, int epilogue, int M, int N, int K, const uint16_t* A, int lda,
                              const uint16_t* B, int ldb, void* C, int ldc, const float* bias, const float* resid,
                              uint16_t* aux, int ldaux, float alpha, const float* alpha_dev, int accumulate,
                              int splits, float p_drop, uint64_t seed, float* dbias, int sched, void* stream) {
  GPT2MI_REQUIRE(dbias == nullptr || ((epilogue == EPI_BF16 || epilogue == EPI_GELU_BWD) && layout <= 1),
                 "gemm: dbias (fused column sum) needs the BF16 or GELU_BWD epilogue of layout 0/1");
  // 128-wide tiles with a half-width last tile in N (and in M for the transposed A of wgrad): C = 1600
  // (GPT-2 1.5B) gives N = 1600 / 4800
  GPT2MI_REQUIRE(N % 64 == 0 && N > 0 && M % 64 == 0 && M > 0, "gemm: N=%d and M=%d must be multiples of 64", N, M);
  GPT2MI_REQUIRE(splits >= 1 && K % (BK * splits) == 0, "gemm: K=%d must be a multiple of %d*splits(%d)", K, BK,
                 splits);
  GPT2MI_REQUIRE(splits == 1 || epilogue == EPI_ATOMIC, "gemm: split-K needs the atomic epilogue");
  GPT2MI_REQUIRE(layout >= 0 && layout <= 2, "gemm: bad layout %d", layout);
  GPT2MI_REQUIRE((sched & ~(GPT2MI_SCHED_NO_PERSISTENT | GPT2MI_SCHED_SHARED_CUS | 0xff)) == 0 && (sched & 0xff) <= 8, "gemm: bad sched %#x",
                 sched);
  const int impl = sched & 0xff;
  GPT2MI_REQUIRE(ldc % 4 == 0 && (ldaux % 4 == 0 || aux == nullptr), "gemm: ldc/ldaux must be multiples of 4");
  GPT2MI_REQUIRE(p_drop <= 0.f || (size_t)M * N < (1ull << 33),
                 "gemm: M*N=%zu exceeds the 32-bit dropout pair index", (size_t)M * N);
  GemmParams P{};
  P.A = (const bf16*)A;
  P.B = (const bf16*)B;
  P.C = C;
  P.bias = bias;
  P.resid = resid;
  P.aux = aux;
  P.alpha_dev = alpha_dev;
  P.dbias = dbias;
  P.M = M; P.N = N; P.K = K;
  P.lda = lda; P.ldb = ldb; P.ldc = ldc; P.ldaux = ldaux;
  P.k_per_split = K / splits;
  P.alpha = alpha;
  P.accumulate = accumulate;
  P.seed = seed;
  P.thr = drop_threshold(p_drop);
  P.inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  hipStream_t s = (hipStream_t)stream;
  // the ping-pong kernel takes any M, N multiple of 64 (a partial last tile; GPT-2 1.5B's 1600 / 4800) and any K-tile
  // count >= 2; the 2-stage 256x256 kernel full column tiles only
  // (transposed operands — layouts 1 / 2 — full column tiles only here; since ABI v11 a partial tile's m-contiguous
  // reads stop at the operand's last element (gemm_pp.hip BND), which only gpt2mi_gemm_wgrad's launches exercise)
  const bool pp_ok = splits == 1 && epilogue != EPI_ATOMIC &&
                     (layout == 0 || (N % 256 == 0 && (layout == 1 || M % 256 == 0)));
  const bool big_ok = pp_ok && N % 256 == 0 && (layout <= 1 || M % 256 == 0);
  if (pp_ok && (impl == 0 || impl >= 3)) {
    // impl 6: the ping-pong kernel without its persistent schedule (A/B)
    const int map = impl == 6 ? -1 : impl == 7 ? 7 : (impl >= 3 && impl <= 5) ? impl - 2 : 0;
    const int rc = gpt2mi::gemm_pp_dispatch(layout, epilogue, P, s, 1, map, !(sched & GPT2MI_SCHED_NO_PERSISTENT),
                                            (sched & GPT2MI_SCHED_SHARED_CUS) != 0);
    if (rc >= 0) return rc;  // the ping-pong kernel fuses dbias
  }
  if (dbias) {  // other kernels: the GEMM, then the column sums of its output
    P.dbias = nullptr;
    const int rc = gpt2mi_gemm(layout, epilogue, M, N, K, A, lda, B, ldb, C, ldc, bias, resid, aux, ldaux, alpha,
                               alpha_dev, accumulate, splits, p_drop, seed, nullptr, sched, stream);
    if (rc) return rc;
    return gpt2mi_colsum_bf16((const uint16_t*)C, dbias, M, N, ldc, stream);
  }
  if (big_ok && impl != 1) {
    const int rc = gpt2mi::gemm256_dispatch(layout, epilogue, P, s, 1);
    if (rc >= 0) return rc;
  }
  switch (layout * 16 + epilogue) {
    case 0 * 16 + EPI_BF16: return launch<false, false, EPI_BF16>(P, splits, s);
    case 0 * 16 + EPI_F32: return launch<false, false, EPI_F32>(P, splits, s);
    case 0 * 16 + EPI_RESID: return launch<false, false, EPI_RESID>(P, splits, s);
    case 0 * 16 + EPI_GELU: return launch<false, false, EPI_GELU>(P, splits, s);
    case 0 * 16 + EPI_GELU_BWD: return launch<false, false, EPI_GELU_BWD>(P, splits, s);
    case 1 * 16 + EPI_BF16: return launch<false, true, EPI_BF16>(P, splits, s);
    case 1 * 16 + EPI_F32: return launch<false, true, EPI_F32>(P, splits, s);
    case 1 * 16 + EPI_GELU_BWD: return launch<false, true, EPI_GELU_BWD>(P, splits, s);
    case 2 * 16 + EPI_F32: return launch<true, true, EPI_F32>(P, splits, s);
    case 2 * 16 + EPI_ATOMIC: return launch<true, true, EPI_ATOMIC>(P, splits, s);
    default:
      gpt2mi::set_error("gemm: unsupported layout %d / epilogue %d combination", layout, epilogue);
      return 22;
  }
}

// Weight gradient C[M][N] (+)= alpha * A^T B with A stored [K][M], B stored [K][N] (dW = dY^T X over
// K = tokens), on the 256x256 kernel: `splits` K ranges write fp32 partial slabs into `workspace`
// (splits*M*N floats), then one pass sums them in fixed order into C (deterministic; no atomics).
GPT2MI_EXPORT int gpt2mi_gemm_wgrad(int M, int N, int K, const uint16_t* A, int lda, const uint16_t* B, int ldb,
                                    float* C, int ldc, int accumulate, float alpha, const float* alpha_dev,
                                    float* workspace, size_t workspace_floats, int splits, int sched,
                                    void* stream) {
  GPT2MI_REQUIRE(M % 64 == 0 && N % 64 == 0 && K % 64 == 0 && M > 0 && N > 0 && K > 0,
                 "gemm_wgrad: M=%d N=%d K=%d must be multiples of 64", M, N, K);
  GPT2MI_REQUIRE(ldc == N, "gemm_wgrad: C must be dense (ldc == N)");
  GPT2MI_REQUIRE(splits >= 1 && splits <= K / 64, "gemm_wgrad: bad splits %d", splits);
  GPT2MI_REQUIRE((sched & ~(GPT2MI_SCHED_NO_PERSISTENT | GPT2MI_SCHED_SHARED_CUS | GPT2MI_SCHED_BF16_SLABS | 0xff)) == 0 && (sched & 0xff) <= 8,
                 "gemm_wgrad: bad sched %#x", sched);
  const int impl = sched & 0xff;  // 2: the 2-stage 256x256 kernel (A/B); 0 / 8: the ping-pong kernel
  const bool slab16 = (sched & GPT2MI_SCHED_BF16_SLABS) != 0;
  hipStream_t s = (hipStream_t)stream;
  GemmParams P{};
  P.A = (const bf16*)A;
  P.B = (const bf16*)B;
  P.M = M; P.N = N; P.K = K; P.lda = lda; P.ldb = ldb; P.ldc = ldc;
  P.alpha = alpha;
  P.alpha_dev = alpha_dev;
  P.accumulate = accumulate;
  const int ktiles = K / 64;
  // the ping-pong kernel (default; impl 8) walks K-tile pairs: an even tile count per split (the last split's
  // count is then even too when ktiles is)
  const bool pp = (impl == 0 || impl == 8) && ktiles % 2 == 0;
  if (!pp && (M % 256 != 0 || N % 256 != 0 || impl == 1)) {
    // an odd token-tile count with a partial output tile: the 128x128 kernel (accumulates into / writes C, one pass)
    // (impl 1 keeps forcing the 128x128 kernel there: gpt2mi_gemm would otherwise pick the ping-pong one)
    return gpt2mi_gemm(2, EPI_F32, M, N, K, A, lda, B, ldb, C, ldc, nullptr, nullptr, nullptr, 0, alpha, alpha_dev,
                       accumulate, 1, 0.f, 0, nullptr, (impl == 1 ? 1 : GPT2MI_SCHED_AUTO) |
                           (sched & (GPT2MI_SCHED_NO_PERSISTENT | GPT2MI_SCHED_SHARED_CUS)),
                       stream);
  }
  int tiles_per = (ktiles + splits - 1) / splits;
  if (pp) tiles_per += tiles_per & 1;
  P.k_per_split = tiles_per * 64;
  splits = (K + P.k_per_split - 1) / P.k_per_split;
  if (splits == 1) {
    P.C = C;
    if (pp) {
      const int rc = gpt2mi::gemm_pp_dispatch(2, EPI_F32, P, s, 1, 0);
      if (rc >= 0) return rc;
    }
    return gpt2mi::gemm256_dispatch(2, EPI_F32, P, s, 1);
  }
  GPT2MI_REQUIRE(workspace != nullptr && workspace_floats >= (size_t)splits * M * N,
                 "gemm_wgrad: workspace of %zu floats < splits*M*N = %zu", workspace_floats, (size_t)splits * M * N);
  P.C = workspace;
  P.accumulate = 0;
  // bf16 slabs on the ping-pong kernel only (the 2-stage fallback writes fp32 ones)
  int rc = pp ? gpt2mi::gemm_pp_dispatch(2, slab16 ? EPI_SLAB16 : EPI_SLAB, P, s, splits, 0) : -1;
  const bool b16 = slab16 && rc >= 0;
  if (rc < 0) rc = gpt2mi::gemm256_dispatch(2, EPI_SLAB, P, s, splits);
  if (rc) return rc;
  if (b16) return gpt2mi::splitk_reduce16((const bf16*)workspace, splits, (size_t)M * N, C, accumulate, s);
  return gpt2mi::splitk_reduce(workspace, splits, (size_t)M * N, C, accumulate, s);
}

// Up to four weight gradients over the same K tokens as ONE split-K launch plus one reduction launch (a GPT2Block's qkv /
// proj / fc1 / fc2 weight gradients, issued together at the end of the block's backward): C_g[M_g][N_g] (+)= alpha *
// A_g^T B_g for g < count, every M_g and N_g a multiple of 256. Each problem's `splits` slabs are summed in split
// order, so each C_g holds the same bits as gpt2mi_gemm_wgrad(M_g, N_g, K, ..., splits) with fp32 slabs.
GPT2MI_EXPORT int gpt2mi_gemm_wgrad_grouped(int count, const int* M, const int* N, int K, const uint16_t* const* A,
                                            const int* lda, const uint16_t* const* B, const int* ldb, float* const* C,
                                            int accumulate, float alpha, const float* alpha_dev, float* workspace,
                                            size_t workspace_floats, int splits, int sched, void* stream) {
  GPT2MI_REQUIRE(count >= 1 && count <= kGroupMax, "gemm_wgrad_grouped: count=%d (1..%d)", count, kGroupMax);
  GPT2MI_REQUIRE(K % 128 == 0 && K > 0, "gemm_wgrad_grouped: K=%d must be a multiple of 128", K);
  GPT2MI_REQUIRE(splits >= 1 && splits <= K / 128, "gemm_wgrad_grouped: bad splits %d", splits);
  GPT2MI_REQUIRE((sched & ~(GPT2MI_SCHED_NO_PERSISTENT | GPT2MI_SCHED_SHARED_CUS)) == 0,
                 "gemm_wgrad_grouped: bad sched %#x (fp32 slabs on the ping-pong kernel only)", sched);
  GemmGroup G{};
  G.count = count;
  const int ktiles = K / 64;
  int tiles_per = (ktiles + splits - 1) / splits;
  tiles_per += tiles_per & 1;  // even K-tile counts per split (the ping-pong kernel walks K-tile pairs)
  const int kps = tiles_per * 64;
  splits = (K + kps - 1) / kps;
  size_t off = 0;
  const float* slab[kGroupMax];
  float* out[kGroupMax];
  size_t n[kGroupMax];
  for (int g = 0; g < count; ++g) {
    GPT2MI_REQUIRE(M[g] > 0 && N[g] > 0 && M[g] % 256 == 0 && N[g] % 256 == 0,
                   "gemm_wgrad_grouped: problem %d is %d x %d (multiples of 256 only)", g, M[g], N[g]);
    GemmParams& P = G.p[g];
    P.A = (const bf16*)A[g];
    P.B = (const bf16*)B[g];
    P.M = M[g]; P.N = N[g]; P.K = K; P.lda = lda[g]; P.ldb = ldb[g]; P.ldc = N[g];
    P.alpha = alpha;
    P.alpha_dev = alpha_dev;
    P.k_per_split = kps;
    P.C = workspace + off;
    slab[g] = workspace + off;
    out[g] = C[g];
    n[g] = (size_t)M[g] * N[g];
    off += (size_t)splits * n[g];
    G.prefix[g + 1] = G.prefix[g] + (M[g] / 256) * (N[g] / 256);
  }
  G.tiles = G.prefix[count];
  GPT2MI_REQUIRE(workspace != nullptr && workspace_floats >= off,
                 "gemm_wgrad_grouped: workspace of %zu floats < %zu (splits x the problems' outputs)", workspace_floats, off);
  hipStream_t s = (hipStream_t)stream;
  int rc = gpt2mi::gemm_pp_grouped(G, s);
  if (rc) return rc;
  return gpt2mi::splitk_reduce_grouped(slab, out, n, count, splits, accumulate, s);
}

// The same weight gradient with the second operand given TRANSPOSED, k-contiguous: Bt stored [N][K] (X^T, e.g. the
// final LayerNorm's output transposed once per step). Runs the ping-pong kernel in layout 1 on C^T[N][M] = Bt . A
// (k-contiguous A operand, m-contiguous B operand: one transposed fragment stream instead of two; the lm_head wgrad
// split 1.75 -> 1.42 ms, tools/lmwg_ab.py) into split-K slabs, then sums them transposed into C[M][N].
GPT2MI_EXPORT int gpt2mi_gemm_wgrad_kt(int M, int N, int K, const uint16_t* A, int lda, const uint16_t* Bt, int ldbt,
                                       float* C, int ldc, int accumulate, float alpha, const float* alpha_dev,
                                       float* workspace, size_t workspace_floats, int splits, int sched,
                                       void* stream) {
  GPT2MI_REQUIRE(M % 64 == 0 && N % 64 == 0 && K % 128 == 0 && M > 0 && N > 0 && K > 0,
                 "gemm_wgrad_kt: M=%d N=%d must be multiples of 64, K=%d of 128", M, N, K);
  GPT2MI_REQUIRE(M % 256 == 0, "gemm_wgrad_kt: M=%d must be a multiple of 256 (the transposed operand's full tiles)", M);
  GPT2MI_REQUIRE(ldc == N, "gemm_wgrad_kt: C must be dense (ldc == N)");
  GPT2MI_REQUIRE(splits >= 1 && splits <= K / 128, "gemm_wgrad_kt: bad splits %d", splits);
  GPT2MI_REQUIRE((sched & ~(GPT2MI_SCHED_NO_PERSISTENT | GPT2MI_SCHED_SHARED_CUS | GPT2MI_SCHED_BF16_SLABS | 0xff)) == 0,
                 "gemm_wgrad_kt: bad sched %#x", sched);
  const bool slab16 = (sched & GPT2MI_SCHED_BF16_SLABS) != 0;
  GPT2MI_REQUIRE(workspace != nullptr, "gemm_wgrad_kt: needs a workspace (splits*M*N floats)");
  hipStream_t s = (hipStream_t)stream;
  GemmParams P{};
  P.A = (const bf16*)Bt;  // C^T[N][M] = Bt[N][K] . A[K][M]
  P.B = (const bf16*)A;
  P.M = N; P.N = M; P.K = K; P.lda = ldbt; P.ldb = lda; P.ldc = M;
  P.alpha = alpha;
  P.alpha_dev = alpha_dev;
  const int ktiles = K / 64;
  int tiles_per = (ktiles + splits - 1) / splits;
  tiles_per += tiles_per & 1;  // even K-tile counts per split (the ping-pong kernel walks K-tile pairs)
  P.k_per_split = tiles_per * 64;
  splits = (K + P.k_per_split - 1) / P.k_per_split;
  GPT2MI_REQUIRE(workspace_floats >= (size_t)splits * M * N, "gemm_wgrad_kt: workspace of %zu floats < %zu",
                 workspace_floats, (size_t)splits * M * N);
  P.C = workspace;
  // one split: an fp32 slab, as gpt2mi_gemm_wgrad writes one split straight into C (the same bits)
  const bool b16 = slab16 && splits > 1;
  const int rc = gpt2mi::gemm_pp_dispatch(1, b16 ? EPI_SLAB16 : EPI_SLAB, P, s, splits, 0);
  if (rc < 0) {
    gpt2mi::set_error("gemm_wgrad_kt: no kernel for M=%d N=%d K=%d splits=%d", M, N, K, splits);
    return 22;
  }
  if (rc) return rc;
  if (b16) return gpt2mi::splitk_reduce16_t((const bf16*)workspace, splits, N, M, C, accumulate, s);
  return gpt2mi::splitk_reduce_t(workspace, splits, N, M, C, accumulate, s);
}

