// bf16 MFMA GEMM, 256x256 block tile — the forward / dgrad workhorse (see gemm.hip for the API).
//
// 512 threads = 8 waves as 2 (M) x 4 (N), 128x64 outputs per wave (8x4 v_mfma_f32_16x16x32_bf16
// accumulators, 128 registers), BK = 64, one workgroup per CU, 2 LDS stages (2 x 64 KiB).
// Global->LDS by global_load_lds_dwordx4 (LDS-DMA, no register staging), 8 instructions per wave
// per K-tile, issued for tile kt+1 before the MFMAs of tile kt and retired by one vmcnt(0) +
// barrier per K-tile. Measured alternatives that were slower on MI355X (tools/kbench.py): a 4-stage
// BK=32 ring with counted vmcnt (twice the barriers per MFMA) and register double-buffering of
// the fragments (the compiler already overlaps the ds_reads; +70 VGPRs).
// Split-K (wgrad): the block's item index selects a K range; each split writes its fp32 partial tile to a slab
// and gpt2mi_gemm_wgrad sums the slabs into the gradient in a second, deterministic pass.
// The DMA destination is lane-linear, so the bank-conflict XOR swizzle is applied on the SOURCE
// address and undone on the ds_read:
//   k-contiguous operand image [256][64] : chunk c of row r at (c ^ (r & 7))            (ds_read_b128)
//   m-contiguous operand image [64][256] : chunk c of k-row k at (c ^ 2((k&3)|((k>>3&1)<<2)))
//                                          (two ds_read_b64_tr_b16 per fragment)
// Epilogue straight from registers: the MFMA is issued as D^T = B.A^T, so each lane holds FOUR
// CONSECUTIVE output columns of one row -> 8-B (bf16) / 16-B (fp32) stores and 16-B bias /
// residual / pre-activation loads, no LDS round trip.
#include "common.h"
#include "gemm_common.h"

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int kThreads = 512;
constexpr int kOpBytes = BM * BK * 2;       // 32 KiB per operand per stage
constexpr int kStageBytes = 2 * kOpBytes;   // 64 KiB
constexpr int kLdsBytes = 2 * kStageBytes;  // 128 KiB

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ int kc_off(int row, int chunk) { return row * 128 + 16 * (chunk ^ (row & 7)); }
__device__ __forceinline__ int mc_swz(int k) { return 2 * ((k & 3) | (((k >> 3) & 1) << 2)); }
__device__ __forceinline__ int mc_off(int k, int chunk) { return k * 512 + 16 * (chunk ^ mc_swz(k)); }

// One operand's K-tile by LDS-DMA: 32 x 1 KiB instructions per tile, 4 per wave.
template <bool TRANS>
__device__ __forceinline__ void dma_tile(const bf16* __restrict__ src, int ld, int row0, int k0, int rmax, char* tile,
                                         int wid, int lane) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int ins = wid * 4 + t;
    const bf16* g;
    if constexpr (!TRANS) {  // instruction covers rows 8*ins .. +8 (128 B each)
      const int row = 8 * ins + (lane >> 3);
      const int c = (lane & 7) ^ (row & 7);
      g = src + (size_t)min(row0 + row, rmax) * ld + k0 + 8 * c;
    } else {  // instruction covers k-rows 2*ins, 2*ins+1 (512 B each)
      const int k = 2 * ins + (lane >> 5);
      const int c = (lane & 31) ^ mc_swz(k);
      g = src + (size_t)(k0 + k) * ld + row0 + 8 * c;
    }
    lds_dma16(g, tile + ins * 1024);
  }
}

// The m-contiguous operand's K-tile by BUFFER LDS-DMA (WG_BUFDMA): the descriptor is rebased on the K-tile
// (k0 * ld elements, scalar registers), so the per-lane part of the source offset — k-row parity (l >> 5)
// and the swizzled 16-B chunk — takes two VGPRs for every K-tile (instruction t and t + 2 share a
// swizzle) and the k-row / column block is a wave-uniform soffset: no 64-bit address math per DMA.
#ifndef WG_BUFDMA
#define WG_BUFDMA 1
#endif
GPT2MI_PRODUCT_KNOB(WG_BUFDMA, 1);
#ifndef WG_ABL
#define WG_ABL 0
#endif
GPT2MI_PRODUCT_KNOB(WG_ABL, 0);
__device__ __forceinline__ uint32_t mc_lane_off(int ld, int wid, int par, int lane) {
  const int k = 8 * (wid & 1) + 2 * par + (lane >> 5);  // k-row mod 16 of instruction t = par (mod 2)
  return (uint32_t)(((lane >> 5) * ld + 8 * ((lane & 31) ^ mc_swz(k))) * (int)sizeof(bf16));
}
__device__ __forceinline__ void dma_tile_mc_buf(const bf16* __restrict__ src, int ld, int row0, int k0,
                                                const uint32_t (&loff)[2], char* tile, int wid) {
  const u32x4 rs = buf_desc(src + (size_t)k0 * ld);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int ins = wid * 4 + t;
    const int soff = ((2 * ins) * ld + row0) * (int)sizeof(bf16);
    lds_dma16_buf(rs, loff[t & 1], soff, tile + ins * 1024);
  }
}

typedef short s16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ s16x8 s16x8v(int v) {
  const short x = (short)v;
  return s16x8{x, x, x, x, x, x, x, x};
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
  // 1-D grid over (split, tile) items, split-major: the XCD remap gives each XCD a contiguous item range,
  // so the blocks of one K split (which share its A and B token rows) run out of one L2
  const int nsplit = (P.K + P.k_per_split - 1) / P.k_per_split;
  const int item = xcd_remap(blockIdx.x, ntiles * nsplit);
  const int split = item / ntiles;
  const int pid = item - split * ntiles;
  constexpr int GM = 4;
  const int group = pid / (GM * tiles_n);
  const int first_m = group * GM;
  const int gsz = min(tiles_m - first_m, GM);
  const int tm = first_m + (pid % (GM * tiles_n)) % gsz;
  const int tn = (pid % (GM * tiles_n)) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = split * P.k_per_split;
  const int nk = (min(P.K, kbeg + P.k_per_split) - kbeg) / BK;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr bool kBufDma = WG_BUFDMA && A_T && B_T;  // the weight-gradient instantiation
  // WG_ABL (tools/wgrad_ablation.sh; never set in the product build): the wgrad main loop with parts removed
  // (1: MFMAs, 2: fragment reads, 4: next-tile DMAs) to time what bounds it. Results are garbage.
  constexpr int kAbl = WG_ABL;
  [[maybe_unused]] uint32_t loff_a[2] = {0, 0}, loff_b[2] = {0, 0};
  if constexpr (kBufDma) {
    loff_a[0] = mc_lane_off(P.lda, wid, 0, lane);
    loff_a[1] = mc_lane_off(P.lda, wid, 1, lane);
    loff_b[0] = mc_lane_off(P.ldb, wid, 0, lane);
    loff_b[1] = mc_lane_off(P.ldb, wid, 1, lane);
  }
  auto stage = [&](int k0, char* dst) {
    if constexpr (kBufDma) {
      dma_tile_mc_buf(P.A, P.lda, m0, k0, loff_a, dst, wid);
      dma_tile_mc_buf(P.B, P.ldb, n0, k0, loff_b, dst + kOpBytes, wid);
    } else {
      dma_tile<A_T>(P.A, P.lda, m0, k0, P.M - 1, dst, wid, lane);
      dma_tile<B_T>(P.B, P.ldb, n0, k0, P.N - 1, dst + kOpBytes, wid, lane);
    }
  };
  stage(kbeg, smem);
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");

  for (int kt = 0; kt < nk; ++kt) {
    const char* As = smem + (kt & 1) * kStageBytes;
    const char* Bs = As + kOpBytes;
    if (!(kAbl & 4) && kt + 1 < nk) stage(kbeg + (kt + 1) * BK, smem + ((kt + 1) & 1) * kStageBytes);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 bf[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (!B_T) bf[j] = frag_kc(Bs, wn * 64 + 16 * j + (lane & 15), 4 * kk + (lane >> 4));
        else bf[j] = frag_mc(Bs, 32 * kk, wn * 64 + 16 * j, lane);
      }
      if constexpr (A_T && B_T) {
        bf16x8 af[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) af[i] = frag_mc(As, 32 * kk, wm * 128 + 16 * i, lane);
        if constexpr (kAbl & 2) {
#pragma unroll
          for (int i = 0; i < 8; ++i) af[i] = __builtin_bit_cast(bf16x8, s16x8v(lane + i + kt));
#pragma unroll
          for (int j = 0; j < 4; ++j) bf[j] = __builtin_bit_cast(bf16x8, s16x8v(lane - j - kt));
        }
        if constexpr (kAbl & 1) {
#pragma unroll
          for (int i = 0; i < 8; ++i) asm volatile("" ::"v"(af[i]));
#pragma unroll
          for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(bf[j]));
        } else {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[i][j], 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          bf16x8 af;
          if constexpr (!A_T) af = frag_kc(As, wm * 128 + 16 * i + (lane & 15), 4 * kk + (lane >> 4));
          else af = frag_mc(As, 32 * kk, wm * 128 + 16 * i, lane);
          if constexpr (kAbl & 2) {
            af = __builtin_bit_cast(bf16x8, s16x8v(lane + i + kt));
            if (i == 0) {
#pragma unroll
              for (int j = 0; j < 4; ++j) bf[j] = __builtin_bit_cast(bf16x8, s16x8v(lane - j - kt));
            }
          }
          if constexpr (kAbl & 1) {
            asm volatile("" ::"v"(af));
            if (i == 0) {
#pragma unroll
              for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(bf[j]));
            }
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af, acc[i][j], 0, 0, 0);
          }
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
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
      if constexpr (EPI == EPI_SLAB) {  // split-K partial: plain 16-B store into slab blockIdx.y
        float* slab = reinterpret_cast<float*>(P.C) + (size_t)split * P.M * P.ldc;
        *reinterpret_cast<f32x4*>(slab + (size_t)gm * P.ldc + gn) = v;
      } else {
        epilogue_store<EPI>(P, gm, gn, v);
      }
    }
  }
}

template <bool A_T, bool B_T, int EPI>
int launch(const GemmParams& P, hipStream_t s, int splits) {
  dim3 grid(((P.M + BM - 1) / BM) * (P.N / BN) * splits);
  gemm256_kernel<A_T, B_T, EPI><<<grid, kThreads, 0, s>>>(P);
  return gpt2mi::check_launch("gemm256");
}

// out[i] (+)= sum_z slab[z][i]   (fixed summation order: deterministic). The slabs' loads go out in groups of 8 before
// their adds (in split order: the same bits as one load per add), so a thread keeps 8 loads in flight instead of one
// (the 27-split proj reduction was latency-bound)
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ slab, int splits, size_t n4,
                                                            float* __restrict__ out, int accumulate) {
  const f32x4* s4 = reinterpret_cast<const f32x4*>(slab);
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    f32x4 s = accumulate ? reinterpret_cast<const f32x4*>(out)[i] : f32x4{0.f, 0.f, 0.f, 0.f};
    for (int z = 0; z < splits; z += 8) {
      const int nz = min(8, splits - z);  // (uniform)
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (u < nz) v[u] = s4[(size_t)(z + u) * n4 + i];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (u < nz) s += v[u];
    }
    reinterpret_cast<f32x4*>(out)[i] = s;
  }
}

// The same sums for the problems of a grouped weight-gradient launch (gpt2mi_gemm_wgrad_grouped): blockIdx.y is the
// problem, whose slabs / output / length come from the kernel arguments; the same per-element order as above
struct ReduceGroup {
  const float* slab[kGroupMax];
  float* out[kGroupMax];
  size_t n4[kGroupMax];
};
__global__ __launch_bounds__(256) void splitk_reduce_grouped_kernel(ReduceGroup R, int splits, int accumulate) {
  const int g = blockIdx.y;
  const f32x4* s4 = reinterpret_cast<const f32x4*>(R.slab[g]);
  f32x4* o4 = reinterpret_cast<f32x4*>(R.out[g]);
  const size_t n4 = R.n4[g];
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    f32x4 s = accumulate ? o4[i] : f32x4{0.f, 0.f, 0.f, 0.f};
    for (int z = 0; z < splits; z += 8) {
      const int nz = min(8, splits - z);  // (uniform)
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (u < nz) v[u] = s4[(size_t)(z + u) * n4 + i];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (u < nz) s += v[u];
    }
    o4[i] = s;
  }
}

// bf16 slabs (GPT2MI_SCHED_BF16_SLABS): 8 elements per thread (one 16-B load per slab), each widened to fp32 and added
// in the order above (the old value first when accumulating, then the slabs in split order)
__global__ __launch_bounds__(256) void splitk_reduce16_kernel(const bf16* __restrict__ slab, int splits, size_t n8,
                                                              float* __restrict__ out, int accumulate) {
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n8; i += (size_t)gridDim.x * 256) {
    f32x4* o = reinterpret_cast<f32x4*>(out) + 2 * i;
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0;
    if (accumulate) {
      s0 = o[0];
      s1 = o[1];
    }
    for (int z = 0; z < splits; ++z) {
      const bf16x8 v = reinterpret_cast<const bf16x8*>(slab + (size_t)z * n8 * 8)[i];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s0[e] += bf2f(v[e]);
        s1[e] += bf2f(v[4 + e]);
      }
    }
    o[0] = s0;
    o[1] = s1;
  }
}

// 64 x 64 tile of the slabs per block, summed as splitk_reduce sums (the old value first when accumulating, then the
// slabs in split order: the same bits), staged through LDS and written transposed: 16-B loads and stores, 16 lanes per
// 256-B row segment on both sides
template <typename TS>  // slab element: float, or bf16 (GPT2MI_SCHED_BF16_SLABS)
__global__ __launch_bounds__(256) void splitk_reduce_t_kernel(const TS* __restrict__ slab, int splits, int rows,
                                                              int cols, float* __restrict__ out, int accumulate) {
  __shared__ float t[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int q = threadIdx.x & 15, p = threadIdx.x >> 4;  // 16 lanes x 4 floats per 64-float segment, 16 segments / pass
  const size_t plane = (size_t)rows * cols;
  if (accumulate) {  // t[r][c] = out[c][r]
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = 16 * i + p;
      const f32x4 v = *reinterpret_cast<const f32x4*>(out + (size_t)(c0 + c) * rows + r0 + 4 * q);
#pragma unroll
      for (int e = 0; e < 4; ++e) t[4 * q + e][c] = v[e];
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 16 * i + p;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (accumulate) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = t[r][4 * q + e];
    }
    const TS* src = slab + (size_t)(r0 + r) * cols + c0 + 4 * q;
    for (int z = 0; z < splits; ++z) {
      const f32x4 w = load4<TS>(src + z * plane);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] += w[e];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) t[r][4 * q + e] = v[e];  // (the lane's own elements: read above, by it alone)
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = 16 * i + p;
    const f32x4 v = {t[4 * q][c], t[4 * q + 1][c], t[4 * q + 2][c], t[4 * q + 3][c]};
    *reinterpret_cast<f32x4*>(out + (size_t)(c0 + c) * rows + r0 + 4 * q) = v;
  }
}

}  // namespace

namespace gpt2mi {
// Layouts 0 (forward) and 1 (dgrad); N % 256 == 0, M % 64 == 0, K % 32 == 0, no split-K.
int gemm256_dispatch(int layout, int epilogue, const GemmParams& P, hipStream_t s, int splits) {
  switch (layout * 16 + epilogue) {
    case 0 * 16 + EPI_BF16: return launch<false, false, EPI_BF16>(P, s, 1);
    case 0 * 16 + EPI_F32: return launch<false, false, EPI_F32>(P, s, 1);
    case 0 * 16 + EPI_RESID: return launch<false, false, EPI_RESID>(P, s, 1);
    case 0 * 16 + EPI_GELU: return launch<false, false, EPI_GELU>(P, s, 1);
    case 0 * 16 + EPI_GELU_BWD: return launch<false, false, EPI_GELU_BWD>(P, s, 1);
    case 1 * 16 + EPI_BF16: return launch<false, true, EPI_BF16>(P, s, 1);
    case 1 * 16 + EPI_F32: return launch<false, true, EPI_F32>(P, s, 1);
    case 1 * 16 + EPI_GELU_BWD: return launch<false, true, EPI_GELU_BWD>(P, s, 1);
    case 2 * 16 + EPI_F32: return launch<true, true, EPI_F32>(P, s, 1);
    case 2 * 16 + EPI_SLAB: return launch<true, true, EPI_SLAB>(P, s, splits);
    default: return -1;  // not built for this kernel: caller falls back to the 128x128 kernel
  }
}

int splitk_reduce_t(const float* slab, int splits, int rows, int cols, float* out, int accumulate, hipStream_t s) {
  splitk_reduce_t_kernel<float><<<dim3(cols / 64, rows / 64), 256, 0, s>>>(slab, splits, rows, cols, out, accumulate);
  return check_launch("splitk_reduce_t");
}
int splitk_reduce16_t(const bf16* slab, int splits, int rows, int cols, float* out, int accumulate, hipStream_t s) {
  splitk_reduce_t_kernel<bf16><<<dim3(cols / 64, rows / 64), 256, 0, s>>>(slab, splits, rows, cols, out, accumulate);
  return check_launch("splitk_reduce16_t");
}
int splitk_reduce16(const bf16* slab, int splits, size_t n, float* out, int accumulate, hipStream_t s) {
  splitk_reduce16_kernel<<<2048, 256, 0, s>>>(slab, splits, n / 8, out, accumulate);
  return check_launch("splitk_reduce16");
}
int splitk_reduce_grouped(const float* const* slab, float* const* out, const size_t* n, int count, int splits,
                          int accumulate, hipStream_t s) {
  ReduceGroup R{};
  for (int g = 0; g < count; ++g) {
    R.slab[g] = slab[g];
    R.out[g] = out[g];
    R.n4[g] = n[g] / 4;
  }
  splitk_reduce_grouped_kernel<<<dim3(2048 / count, count), 256, 0, s>>>(R, splits, accumulate);
  return check_launch("splitk_reduce_grouped");
}
int splitk_reduce(const float* slab, int splits, size_t n, float* out, int accumulate, hipStream_t s) {
  splitk_reduce_kernel<<<2048, 256, 0, s>>>(slab, splits, n / 4, out, accumulate);
  return check_launch("splitk_reduce");
}
}  // namespace gpt2mi
