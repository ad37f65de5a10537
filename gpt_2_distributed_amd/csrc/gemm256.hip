// bf16 MFMA GEMM, 256x256 block tile — the forward / dgrad workhorse (see gemm.hip for the API).
//
// 512 threads = 8 waves as 2 (M) x 4 (N), 128x64 outputs per wave (8x4 v_mfma_f32_16x16x32_bf16
// accumulators, 128 registers), BK = 32, one workgroup per CU, 4-stage LDS ring (4 x 32 KiB).
// Global->LDS by global_load_lds_dwordx4 (LDS-DMA, no register staging), 4 instructions per wave
// per K-tile. Three K-tiles are in flight while one is consumed: each iteration waits with a
// COUNTED vmcnt for its own tile only (never vmcnt(0) in the loop), crosses one raw s_barrier
// (which also frees the stage read in the previous iteration) and refills that stage with tile
// kt+3 before issuing its 32 MFMAs. The DMA destination is lane-linear, so the bank-conflict XOR
// swizzle is applied on the SOURCE address and undone on the ds_read:
//   k-contiguous operand image [256][32] : chunk c of row r at (c ^ ((r>>3 & 1) << 1))  (ds_read_b128)
//   m-contiguous operand image [32][256] : chunk c of k-row k at (c ^ 2((k&3)|((k>>3&1)<<2)))
//                                          (two ds_read_b64_tr_b16 per fragment)
// Epilogue straight from registers: the MFMA is issued as D^T = B.A^T, so each lane holds FOUR
// CONSECUTIVE output columns of one row -> 8-B (bf16) / 16-B (fp32) stores and 16-B bias /
// residual / pre-activation loads, no LDS round trip.
#include "common.h"
#include "gemm_common.h"

namespace {

constexpr int BM = 256, BN = 256, BK = 32;
constexpr int kThreads = 512;
constexpr int kStages = 4;
constexpr int kOpBytes = BM * BK * 2;             // 16 KiB per operand per stage
constexpr int kStageBytes = 2 * kOpBytes;         // 32 KiB
constexpr int kLdsBytes = kStages * kStageBytes;  // 128 KiB

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ int kc_swz(int row) { return ((row >> 3) & 1) << 1; }
__device__ __forceinline__ int kc_off(int row, int chunk) { return row * 64 + 16 * (chunk ^ kc_swz(row)); }
__device__ __forceinline__ int mc_swz(int k) { return 2 * ((k & 3) | (((k >> 3) & 1) << 2)); }
__device__ __forceinline__ int mc_off(int k, int chunk) { return k * 512 + 16 * (chunk ^ mc_swz(k)); }

// One operand's K-tile by LDS-DMA: 16 x 1 KiB instructions per tile, 2 per wave.
template <bool TRANS>
__device__ __forceinline__ void dma_tile(const bf16* __restrict__ src, int ld, int row0, int k0, int rmax, char* tile,
                                         int wid, int lane) {
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int ins = wid * 2 + t;
    const bf16* g;
    if constexpr (!TRANS) {  // instruction covers rows 16*ins .. +16 (64 B each)
      const int row = 16 * ins + (lane >> 2);
      const int c = (lane & 3) ^ kc_swz(row);
      g = src + (size_t)min(row0 + row, rmax) * ld + k0 + 8 * c;
    } else {  // instruction covers k-rows 2*ins, 2*ins+1 (512 B each)
      const int k = 2 * ins + (lane >> 5);
      const int c = (lane & 31) ^ mc_swz(k);
      g = src + (size_t)(k0 + k) * ld + row0 + 8 * c;
    }
    __builtin_amdgcn_global_load_lds((const void*)g, (lds_void*)(tile + ins * 1024), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8 frag_kc(const char* base, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(base + kc_off(row, chunk));
}
__device__ __forceinline__ bf16x8 frag_mc(const char* base, int k0, int m0, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int k1 = k0 + 8 * g + q;
  const int chunk = (m0 >> 3) + (p >> 1);
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + mc_off(k1, chunk) + 8 * (p & 1)));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + mc_off(k1 + 4, chunk) + 8 * (p & 1)));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

template <bool A_T, bool B_T, int EPI>
__global__ __launch_bounds__(kThreads, 1) void gemm256_kernel(GemmParams P) {
  __shared__ __attribute__((aligned(16))) char smem[kLdsBytes];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 2, wn = wid & 3;

  const int tiles_m = (P.M + BM - 1) / BM, tiles_n = P.N / BN;
  const int ntiles = tiles_m * tiles_n;
  const int pid = xcd_remap(blockIdx.x, ntiles);
  constexpr int GM = 4;
  const int group = pid / (GM * tiles_n);
  const int first_m = group * GM;
  const int gsz = min(tiles_m - first_m, GM);
  const int tm = first_m + (pid % (GM * tiles_n)) % gsz;
  const int tn = (pid % (GM * tiles_n)) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = P.K / BK;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int t) {
    char* st = smem + (t & (kStages - 1)) * kStageBytes;
    dma_tile<A_T>(P.A, P.lda, m0, t * BK, P.M - 1, st, wid, lane);
    dma_tile<B_T>(P.B, P.ldb, n0, t * BK, P.N - 1, st + kOpBytes, wid, lane);
  };
#pragma unroll
  for (int t = 0; t < kStages - 1; ++t)
    if (t < nk) issue(t);

  for (int kt = 0; kt < nk; ++kt) {
    // retire this wave's DMAs of tile kt (4 per tile; tiles kt+1, kt+2 may stay in flight)
    // (wait + barrier in ONE asm statement: no LDS access can be scheduled between them)
    if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
    else if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    if (kt + kStages - 1 < nk) issue(kt + kStages - 1);
    const char* As = smem + (kt & (kStages - 1)) * kStageBytes;
    const char* Bs = As + kOpBytes;
    bf16x8 bf[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (!B_T) bf[j] = frag_kc(Bs, wn * 64 + 16 * j + (lane & 15), lane >> 4);
      else bf[j] = frag_mc(Bs, 0, wn * 64 + 16 * j, lane);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      bf16x8 af;
      if constexpr (!A_T) af = frag_kc(As, wm * 128 + 16 * i + (lane & 15), lane >> 4);
      else af = frag_mc(As, 0, wm * 128 + 16 * i, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af, acc[i][j], 0, 0, 0);
    }
  }

  // ---- epilogue from registers: acc[i][j][r] = C[m0 + wm*128 + 16i + (l&15)][n0 + wn*64 + 16j + 4(l>>4) + r]
  float alpha = P.alpha;
  if (P.alpha_dev) alpha *= P.alpha_dev[0];
  const int gcol0 = n0 + wn * 64 + 4 * (lane >> 4);
  f32x4 bias[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    bias[j] = (P.bias && EPI != EPI_GELU_BWD) ? *reinterpret_cast<const f32x4*>(P.bias + gcol0 + 16 * j)
                                              : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int gm = m0 + wm * 128 + 16 * i + (lane & 15);
    if (gm >= P.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int gn = gcol0 + 16 * j;
      f32x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] * alpha + bias[j][r];
      epilogue_store<EPI>(P, gm, gn, v);
    }
  }
}

template <bool A_T, bool B_T, int EPI>
int launch(const GemmParams& P, hipStream_t s) {
  dim3 grid(((P.M + BM - 1) / BM) * (P.N / BN));
  gemm256_kernel<A_T, B_T, EPI><<<grid, kThreads, 0, s>>>(P);
  return gpt2mi::check_launch("gemm256");
}

}  // namespace

namespace gpt2mi {
// Layouts 0 (forward) and 1 (dgrad); N % 256 == 0, M % 64 == 0, K % 32 == 0, no split-K.
int gemm256_dispatch(int layout, int epilogue, const GemmParams& P, hipStream_t s) {
  switch (layout * 16 + epilogue) {
    case 0 * 16 + EPI_BF16: return launch<false, false, EPI_BF16>(P, s);
    case 0 * 16 + EPI_F32: return launch<false, false, EPI_F32>(P, s);
    case 0 * 16 + EPI_RESID: return launch<false, false, EPI_RESID>(P, s);
    case 0 * 16 + EPI_GELU: return launch<false, false, EPI_GELU>(P, s);
    case 1 * 16 + EPI_BF16: return launch<false, true, EPI_BF16>(P, s);
    case 1 * 16 + EPI_F32: return launch<false, true, EPI_F32>(P, s);
    case 1 * 16 + EPI_GELU_BWD: return launch<false, true, EPI_GELU_BWD>(P, s);
    default: return -1;  // not built for this kernel: caller falls back to the 128x128 kernel
  }
}
}  // namespace gpt2mi
