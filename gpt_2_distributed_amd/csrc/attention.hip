// Causal flash attention forward/backward for gfx950, head_dim 64, bf16 in/out, fp32 softmax.
//
// Replaces (model.py:124-155): the [B,H,T,T] bmm -> /sqrt(D) ->
// masked_fill(tril==0,-1e4) -> softmax(fp32) -> dropout -> bmm chain and its backward, with no
// T x T tensor and no mask buffer (causality from tile indices; -1e4 and -inf give the same fp32
// softmax since no row is fully masked).
//
// Layout in HBM (no view/transpose copies): q,k,v are read straight out of the qkv GEMM output
// [B*T, 3C] (cols [0,C)=q, [C,2C)=k, [2C,3C)=v, head h at h*64), y is written head-merged into
// [B*T, C], dq/dk/dv into the same [B*T, 3C] layout so the qkv backward GEMMs consume them as-is.
//
// Work split: a wave owns 32 queries (fwd, dQ) or 32 keys (dK/dV) as two 16-lane MFMA groups, so
// every K/V (Q/dO) fragment read from LDS feeds two MFMAs; 4 waves per workgroup; heavy (late
// query / early key) blocks are dispatched first for the causal imbalance; key tiles that are fully
// masked for a wave are skipped wave-uniformly.
// MFMA formulation (v_mfma_f32_16x16x32_bf16), "key on the lane" / "query on the lane":
//   forward / dQ : S^T = K Q^T  -> lane l holds 16 keys of query l&15: softmax stats per lane;
//                  O^T += V^T P^T with P^T taken from the S^T accumulators IN REGISTERS (the MFMA
//                  k-index is permuted consistently on both operands), V^T by ds_read_b64_tr_b16.
//   dK/dV        : S = Q K^T    -> lane holds 16 queries of key l&15; dV^T += dO^T P, dK^T += Q^T dS
//                  with P/dS from registers and dO^T/Q^T by transposed LDS reads.
// LDS tiles are [64 rows][64 bf16] (128-B rows), 16-B chunk c stored at c ^ (row & 6): conflict-
// free for both the ds_read_b128 row reads and the permuted transposed reads.
#include <type_traits>

#include "common.h"

namespace {

constexpr int D = 64;
constexpr int BQ = 128;  // queries per workgroup in fwd / dQ (32 per wave = two 16-query MFMA groups)
constexpr int BKV = 64;  // keys per K/V tile in fwd / dQ
#ifndef ATTN_FWD_OCC
#define ATTN_FWD_OCC 3  // forward waves per SIMD the register budget is cut for (launch bounds)
#endif
#ifndef ATTN_FWD_LMAX
#define ATTN_FWD_LMAX 1  // forward rescale test on each lane's own scores (0: cross-lane max every tile, A/B builds)
#endif
GPT2MI_PRODUCT_KNOB(ATTN_FWD_OCC, 3);
GPT2MI_PRODUCT_KNOB(ATTN_FWD_LMAX, 1);
constexpr int BKB = 128;  // keys per workgroup in dK/dV (4 waves of 32)
#ifndef ATTN_DKDV_PIPE
#define ATTN_DKDV_PIPE 0  // dK/dV tile body: 0 phases in separate blocks; 1-3 one block per DIAG variant (A/B builds)
#endif
#ifndef ATTN_DKDV_FILL
#define ATTN_DKDV_FILL 10  // ATTN_DKDV_PIPE 3: VALU instructions placed after each MFMA
#endif
GPT2MI_PRODUCT_KNOB(ATTN_DKDV_PIPE, 0);
#ifndef ATTN_HASH_ANCHOR
#define ATTN_HASH_ANCHOR 0  // dK/dV dropout hash: 1 = the opaque anchor on the counter sum (no v_mov per hash; A/B)
#endif
GPT2MI_PRODUCT_KNOB(ATTN_HASH_ANCHOR, 0);
#ifndef ATTN_DQ_SGB
#define ATTN_DQ_SGB 0  // dQ tile: 1 = sched_group_barrier interleave of each half's MFMAs with the other half's VALU (A/B)
#endif
#ifndef ATTN_DQ_FA
#define ATTN_DQ_FA 6  // ATTN_DQ_SGB: VALU instructions after each S / dP MFMA of the second half
#endif
#ifndef ATTN_DQ_FB
#define ATTN_DQ_FB 12  // ATTN_DQ_SGB: VALU instructions after each dQ MFMA of the first half
#endif
GPT2MI_PRODUCT_KNOB(ATTN_DQ_SGB, 0);
constexpr int kThreads = 256;
constexpr float kLog2e = 1.4426950408889634f;

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef short s16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int t_off(int row, int chunk) { return row * 128 + 16 * (chunk ^ (row & 6)); }

// row read: lane gets tile[row0 + (l&15)][32kk + 8g + 0..7]
__device__ __forceinline__ bf16x8 row_frag(const char* base, int row0, int kk, int lane) {
  return *reinterpret_cast<const bf16x8*>(base + t_off(row0 + (lane & 15), 4 * kk + (lane >> 4)));
}

// permuted transposed read: lane (g=l>>4, i=l&15) gets, for j = 0..7,
//   tile[16*(2kk + (j>>2)) + 4g + (j&3)][c0 + i]
__device__ __forceinline__ bf16x8 tr_frag(const char* base, int kk, int c0, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int chunk = (c0 >> 3) + (p >> 1);
  const int r1 = 32 * kk + 4 * g + q;
  const int r2 = r1 + 16;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + t_off(r1, chunk) + 8 * (p & 1)));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + t_off(r2, chunk) + 8 * (p & 1)));
  s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

// max / sum over the 4 lanes l, l^16, l^32, l^48 (one query's keys in the S^T accumulators) with
// the VALU lane swaps of gfx950 (no LDS round trip): op(swap[0], swap[1]) = op(own, partner)
__device__ __forceinline__ float xor_max(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float xor_sum(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
// max of a lane's 16 scores as a v_max3 tree: 8 instructions (5 + 2 + 1)
__device__ __forceinline__ float max3f(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }

__device__ __forceinline__ float max16(const f32x4 (&s)[4]) {
  const float t0 = max3f(s[0][0], s[0][1], s[0][2]), t1 = max3f(s[0][3], s[1][0], s[1][1]);
  const float t2 = max3f(s[1][2], s[1][3], s[2][0]), t3 = max3f(s[2][1], s[2][2], s[2][3]);
  const float t4 = max3f(s[3][0], s[3][1], s[3][2]);
  return fmaxf(max3f(t0, t1, t2), max3f(t3, t4, s[3][3]));
}
// Sum over the 16 lanes of a DPP row (lanes with the same l >> 4): every lane gets the row total.
__device__ __forceinline__ float row16_sum(float x) {
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xF, 0xF, false));   // quad_perm 1,0,3,2
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xF, 0xF, false));   // quad_perm 2,3,0,1
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x141, 0xF, 0xF, false));  // row_half_mirror
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x140, 0xF, 0xF, false));  // row_mirror
  return x;
}

// Column sums of a wave's [32 rows][64 cols] output tile as stored (bf16-rounded), held as
// v[grp][fd][r] = row 16grp + (l & 15), col 16fd + 4(l >> 4) + r. Returns lane l's share: the total of
// column 16((l & 15) >> 2) + 4(l >> 4) + (l & 3), so one 64-lane store writes the tile's 64 sums.
// (The qkv bias gradient: partial sums per 32 tokens, reduced over tokens by gpt2mi_colsum_f32.)
__device__ __forceinline__ float tile_colsum(const f32x4 (&v)[2][4], float scale, int lane) {
  const int j = lane & 15;
  float mine = 0.f;
#pragma unroll
  for (int fd = 0; fd < 4; ++fd)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float t = row16_sum(bf2f(f2bf(v[0][fd][r] * scale)) + bf2f(f2bf(v[1][fd][r] * scale)));
      mine = j == 4 * fd + r ? t : mine;
    }
  return mine;
}
__device__ __forceinline__ int tile_colsum_col(int lane) { return 16 * ((lane & 15) >> 2) + 4 * (lane >> 4) + (lane & 3); }

// One 64-wide output row (head_dim) of a wave's MFMA accumulators, v[fd][r] = row value at d = 16fd + 4g + r
// (g = lane >> 4), scaled by sc and stored as bf16 with two 16-B stores per lane instead of four 8-B ones (the
// output tail is store-issue bound; cdna_hip_programming.md T21): a permlane16 swap per dword hands lane group g
// the 8 contiguous d of the pair (fd, fd + 1) it stores — d 16(g & 1) + 8(g >> 1) .. +8 of the pair's 32.
__device__ __forceinline__ void store_row64(bf16* row, const f32x4 (&v)[4], float sc, int lane) {
  const int g = lane >> 4;
#pragma unroll
  for (int pr = 0; pr < 2; ++pr) {
    const bf16x4 a = {f2bf(v[2 * pr][0] * sc), f2bf(v[2 * pr][1] * sc), f2bf(v[2 * pr][2] * sc), f2bf(v[2 * pr][3] * sc)};
    const bf16x4 b = {f2bf(v[2 * pr + 1][0] * sc), f2bf(v[2 * pr + 1][1] * sc), f2bf(v[2 * pr + 1][2] * sc),
                      f2bf(v[2 * pr + 1][3] * sc)};
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 ua = __builtin_bit_cast(u32x2, a), ub = __builtin_bit_cast(u32x2, b);
    // rows 1 / 3 of the first operand <-> rows 0 / 2 of the second
    const auto x = __builtin_amdgcn_permlane16_swap(ua[0], ub[0], false, false);
    const auto y = __builtin_amdgcn_permlane16_swap(ua[1], ub[1], false, false);
    *reinterpret_cast<u32x4*>(row + 32 * pr + 16 * (g & 1) + 8 * (g >> 1)) = u32x4{x[0], y[0], x[1], y[1]};
  }
}

constexpr float kRescaleThr = 8.f;  // log2 units: P <= 256 between rescales (bf16-exact exponent range)
// exp2(a x + b) of a pair: the affine part as ONE packed FMA (v_pk_fma_f32, two lanes' worth per issue; each component
// the same fused fma as fmaf, so the same bits), the exponentials one by one (no packed transcendental)
__device__ __forceinline__ f32x2 exp2_affine2(float x0, float x1, float a, float b) {
  const f32x2 t = __builtin_elementwise_fma(f32x2{x0, x1}, f32x2{a, a}, f32x2{b, b});
  return f32x2{__builtin_amdgcn_exp2f(t[0]), __builtin_amdgcn_exp2f(t[1])};
}

// pack accumulator registers acc[2kk + (j>>2)][j&3] (j = 0..7) to a bf16 operand fragment
__device__ __forceinline__ bf16x8 pack_perm(const f32x4* acc, int kk) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = f2bf(acc[2 * kk + (j >> 2)][j & 3]);
  return r;
}

typedef __attribute__((address_space(3))) void lds_void;
// 64 rows x 128 B tiles arrive by LDS-DMA (buffer_load_dwordx4 ... lds, no register staging): instruction
// `ins` (of wave w: ins = 2w, 2w+1) writes LDS bytes [1024*ins, +1024) = rows 8*ins .. 8*ins+7, and the
// t_off swizzle is applied on the source side (slot s of row r holds chunk s ^ (r & 6)). A lane's source
// offset is the same for every instruction (one VGPR); the tile / row-group position is a wave-uniform
// byte offset (SGPR soffset) into a raw buffer over one batch row's qkv (or dO).
__device__ __forceinline__ uint32_t tile_dma_off(size_t ld, int lane) {
  const int r = lane >> 3;
  return (uint32_t)((r * ld + 8 * ((lane & 7) ^ (r & 6))) * sizeof(bf16));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t qkv_rsrc(const bf16* base) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7fffffff, 0x00020000);
}
// rows [row0, row0 + 64) x cols [col0, col0 + 64) of the buffer (row stride ld elements)
template <int NW = 4>  // waves of the workgroup sharing the tile's 8 instructions
__device__ __forceinline__ void tile_dma(char* lds, __amdgpu_buffer_rsrc_t rs, int row0, int col0, int ld,
                                         uint32_t loff, int w) {
#pragma unroll
  for (int i = 0; i < 8 / NW; ++i) {
    const int ins = (8 / NW) * w + i;
    const int soff = ((row0 + 8 * ins) * ld + col0) * (int)sizeof(bf16);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(lds + ins * 1024), 16, loff, soff, 0, 0);
  }
}

// Block -> (head, query/key block) map: globally heaviest first. Block L takes head L % BH and block L / BH, so
// every head's heaviest block (the last query block in fwd / dQ, the first key block in dK/dV: its causal work is
// the longest) is dispatched before any head's second-heaviest, and the lightest blocks fill the tail. A 2-D grid
// sends block L to XCD L % 8, so head bh stays on XCD bh % 8 (BH % 8 == 0) across its blocks: those run at
// different times, and its K/V or Q/dO tiles come back from the 256 MB MALL rather than that XCD's L2. The
// previous map (the 8 blocks of a head together on one XCD, head groups in dispatch order) left a tail of heavy
// blocks dispatched last: forward 236 -> 183 us, backward 692 -> 594 us per layer at cfg 2 (same-process A/B,
// bitwise equal outputs).
__device__ __forceinline__ void attn_block(int& bh, int& blk) {
  const int BH = gridDim.y;
  const int L = blockIdx.y * gridDim.x + blockIdx.x;
  bh = L % BH;
  blk = L / BH;
}

// Dropout of attention probability (q, key) of head bh: 16-bit half (q >> 4) & 1 of
// drop_hash(seed, (bh*T + (q & ~16))*T + key) — queries q and q^16 of one key share a hash.

// ---------------------------------------------------------------------------------------------
template <bool DROP>
__global__ __launch_bounds__(kThreads, ATTN_FWD_OCC) void attn_fwd_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out,
                                                               float* __restrict__ lse, int T, int H, float scale,
                                                               uint64_t seed, uint32_t thr, float inv_keep) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * BKV * 128];  // 2 stages x (K, V)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4;
  const int nqb = (T + BQ - 1) / BQ;
  int bh, blk;
  attn_block(bh, blk);
  const int qb = nqb - 1 - blk;  // heavy (late) query blocks first
  const int b = bh / H, h = bh % H;
  const int C = H * D;
  const size_t ld = 3 * (size_t)C;
  const bf16* base = qkv + (size_t)b * T * ld;
  const int q_lo = qb * BQ + 32 * w;  // first query of this wave
  const bool wave_valid = q_lo < T;    // T % 64 == 0: a wave's 32 queries are all valid or all not

  bf16x8 qf[2][2];
#pragma unroll
  for (int qg = 0; qg < 2; ++qg)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      qf[qg][kk] = *reinterpret_cast<const bf16x8*>(
          base + (size_t)min(q_lo + 16 * qg + (lane & 15), T - 1) * ld + h * D + 32 * kk + 8 * g);
  const float sl2 = scale * kLog2e;
  float m[2] = {-INFINITY, -INFINITY};
  // o[qg][4] holds the row sums l = P.1 of the group's queries: one more PV-shaped MFMA against a
  // ones operand (the MFMA pipe has slack; 32 VALU adds per tile do not). Every row of it is l.
  f32x4 o[2][5];
#pragma unroll
  for (int qg = 0; qg < 2; ++qg)
#pragma unroll
    for (int f = 0; f < 5; ++f) o[qg][f] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bf16 one = (bf16)1.f;
  const bf16x8 ones = {one, one, one, one, one, one, one, one};

  const int nkv = min((qb + 1) * BQ, T) / BKV;
  const uint32_t loff = tile_dma_off(ld, lane);
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const __amdgpu_buffer_rsrc_t rs = qkv_rsrc(base);
  tile_dma(smem, rs, 0, C + h * D, (int)ld, loff, wu);
  tile_dma(smem + BKV * 128, rs, 0, 2 * C + h * D, (int)ld, loff, wu);
  __syncthreads();  // waits for this wave's DMAs (vmcnt(0)), then for every wave's

  for (int j = 0; j < nkv; ++j) {
    const int cur = j & 1;
    const char* Ks = smem + cur * 2 * BKV * 128;
    const char* Vs = Ks + BKV * 128;
    const int k_lo = j * BKV;
    // wave-uniform: a key of the tile is visible to a query of the wave
    const bool active = wave_valid && k_lo <= q_lo + 31;
    f32x4 s[2][4];
    if (active) {
#pragma unroll
      for (int fi = 0; fi < 4; ++fi) {
        s[0][fi] = s[1][fi] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const bf16x8 kf = row_frag(Ks, 16 * fi, kk, lane);
          s[0][fi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[0][kk], s[0][fi], 0, 0, 0);
          s[1][fi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[1][kk], s[1][fi], 0, 0, 0);
        }
      }
    }
    // next K/V tile straight into the other LDS stage (read last in tile j-1, released by its barrier),
    // issued behind S = K Q^T; it lands while this tile's softmax and P.V run
    if (j + 1 < nkv) {
      char* nxt = smem + (cur ^ 1) * 2 * BKV * 128;
      tile_dma(nxt, rs, (j + 1) * BKV, C + h * D, (int)ld, loff, wu);
      tile_dma(nxt + BKV * 128, rs, (j + 1) * BKV, 2 * C + h * D, (int)ld, loff, wu);
    }
    if (active) {
      const bool diag = k_lo + BKV - 1 > q_lo;
      if (diag) {  // causal mask only on the diagonal tiles (wave-uniform branch)
#pragma unroll
        for (int qg = 0; qg < 2; ++qg)
#pragma unroll
          for (int fi = 0; fi < 4; ++fi)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (k_lo + 16 * fi + 4 * g + r > q_lo + 16 * qg + (lane & 15)) s[qg][fi][r] = -INFINITY;
      }
#pragma unroll
      for (int qg = 0; qg < 2; ++qg) {
        // thresholded rescale (defer-max): keep the running max unless some row of the wave grew by
        // more than kRescaleThr (log2 units); P then stays below 2^kRescaleThr. Wave-uniform decision,
        // taken before this tile is exponentiated, so O, l and P all see the same max.
#if ATTN_FWD_LMAX
        // The test needs no max across the 4 lanes of a query: they share m, and x -> x * sl2 is monotonic, so
        // "every lane's own 16 keys pass" is the same decision as "every query's 64 keys pass". The cross-lane
        // max is formed only when a rescale is taken (same cand, same bits as the all-lanes form).
        const float lmax = max16(s[qg]);
        if (!__all(lmax * sl2 <= m[qg] + kRescaleThr)) {
          const float cand = xor_max(lmax) * sl2;
#else
        float tmax = -INFINITY;  // max of the raw scores (scale > 0)
#pragma unroll
        for (int fi = 0; fi < 4; ++fi)
          tmax = fmaxf(tmax, fmaxf(fmaxf(s[qg][fi][0], s[qg][fi][1]), fmaxf(s[qg][fi][2], s[qg][fi][3])));
        tmax = xor_max(tmax);
        const float cand = tmax * sl2;
        if (!__all(cand <= m[qg] + kRescaleThr)) {
#endif
          const float mn = fmaxf(m[qg], cand);  // finite: tile 0 holds key 0, visible to every query
          const float corr = __builtin_amdgcn_exp2f(m[qg] - mn);
#pragma unroll
          for (int f = 0; f < 4; ++f)
#pragma unroll
            for (int r = 0; r < 4; ++r) o[qg][f][r] *= corr;
          o[qg][4][0] *= corr;  // only row 0 of the row-sum accumulator is read
          m[qg] = mn;
        }
#pragma unroll
        for (int fi = 0; fi < 4; ++fi)
#pragma unroll
          for (int r = 0; r < 4; r += 2) {
            const f32x2 e = exp2_affine2(s[qg][fi][r], s[qg][fi][r + 1], sl2, -m[qg]);
            s[qg][fi][r] = e[0];
            s[qg][fi][r + 1] = e[1];
          }
      }
      // P packed to bf16 once per 32-key half (kk): the row sums (before dropout: the normaliser is the undropped
      // softmax denominator) and P.V read the same fragments. Dropout on the packed P (its 1/(1-p) goes into the
      // final scale): one hash per (q, q^16) pair of a key, both decisions from one packed int16 subtract.
      [[maybe_unused]] uint32_t pre = 0, tk2 = 0;
      if constexpr (DROP) {
        pre = drop_pre(seed32(seed), ((uint32_t)bh * T + q_lo + (lane & 15)) * (uint32_t)T + k_lo + 4 * g);
        tk2 = drop_tk2(thr);
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 p0 = pack_perm(s[0], kk), p1 = pack_perm(s[1], kk);
        o[0][4] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, p0, o[0][4], 0, 0, 0);
        o[1][4] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, p1, o[1][4], 0, 0, 0);
        if constexpr (DROP) {
          u32x4 w0 = __builtin_bit_cast(u32x4, p0), w1 = __builtin_bit_cast(u32x4, p1);
#pragma unroll
          for (int d = 0; d < 4; ++d) {  // dword d: keys (fi, r), (fi, r + 1) with fi = 2kk + (d >> 1), r = 2(d & 1)
            const uint32_t c = 16 * (2 * kk + (d >> 1)) + 2 * (d & 1);
            const uint32_t ka = drop_keep_mask2(tk2, drop_fin(pre + c * kDropC1, seed_kx(seed)));
            const uint32_t kb = drop_keep_mask2(tk2, drop_fin(pre + (c + 1) * kDropC1, seed_kx(seed)));
            // the bytes of each bf16 = the sign (keep bit) of key r's / key r+1's decision for query group 0 / 1
            w0[d] &= __builtin_amdgcn_perm(kb, ka, 0x0A0A0808u);
            w1[d] &= __builtin_amdgcn_perm(kb, ka, 0x0B0B0909u);
          }
          p0 = __builtin_bit_cast(bf16x8, w0);
          p1 = __builtin_bit_cast(bf16x8, w1);
        }
#pragma unroll
        for (int fd = 0; fd < 4; ++fd) {
          const bf16x8 vt = tr_frag(Vs, kk, 16 * fd, lane);
          o[0][fd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vt, p0, o[0][fd], 0, 0, 0);
          o[1][fd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vt, p1, o[1][fd], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  if (!wave_valid) return;
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    const int q = q_lo + 16 * qg + (lane & 15);
    const float lq = o[qg][4][0];
    const float il = (DROP ? inv_keep : 1.f) / lq;
    const f32x4 ov[4] = {o[qg][0], o[qg][1], o[qg][2], o[qg][3]};
    store_row64(out + ((size_t)b * T + q) * C + h * D, ov, il, lane);
    if (g == 0) lse[(size_t)bh * T + q] = (m[qg] + log2f(lq)) / kLog2e;  // natural-log LSE of scaled scores
  }
}

// ---------------------------------------------------------------------------------------------
// dQ: query-outer; recomputes P from the saved LSE. dS^T = P^T o (dP^T - delta), dQ^T += K^T dS^T.
// delta = rowsum(dO o O) of the wave's own queries is formed here (no separate pass) and written out for
// the dK/dV kernel, which runs after this one. A 64-key tile runs as two 32-key halves, the second half's S / dP MFMAs
// issued ahead of the first half's dQ MFMAs so that those run beside the second half's elementwise VALU work (a
// software pipeline inside one wave; the half-size S / dP registers also bring the kernel to 160 VGPRs: 3 waves / SIMD).
template <bool DROP>
__global__ __launch_bounds__(kThreads, 3) void attn_bwd_dq_kernel(const bf16* __restrict__ qkv,
                                                                  const bf16* __restrict__ out,
                                                                  const bf16* __restrict__ dout,
                                                                  const float* __restrict__ lse,
                                                                  float* __restrict__ delta,
                                                                  bf16* __restrict__ dqkv, float* __restrict__ csum,
                                                                  int T, int H, float scale, uint64_t seed,
                                                                  uint32_t thr, float inv_keep) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * BKV * 128];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4;
  const int nqb = (T + BQ - 1) / BQ;
  int bh, blk;
  attn_block(bh, blk);
  const int qb = nqb - 1 - blk;
  const int b = bh / H, h = bh % H;
  const int C = H * D;
  const size_t ld = 3 * (size_t)C;
  const bf16* base = qkv + (size_t)b * T * ld;
  const int q_lo = qb * BQ + 32 * w;
  const bool wave_valid = q_lo < T;
  bf16x8 qf[2][2], df[2][2];
  float lse2[2], dl[2];
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    const int q = min(q_lo + 16 * qg + (lane & 15), T - 1);
    float dsum = 0.f;  // this lane's 16 of the 64 dims of dO . O
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const size_t row = ((size_t)b * T + q) * C + h * D + 32 * kk + 8 * g;
      qf[qg][kk] = *reinterpret_cast<const bf16x8*>(base + (size_t)q * ld + h * D + 32 * kk + 8 * g);
      df[qg][kk] = *reinterpret_cast<const bf16x8*>(dout + row);
      const bf16x8 of = *reinterpret_cast<const bf16x8*>(out + row);
#pragma unroll
      for (int e = 0; e < 8; ++e) dsum = fmaf(bf2f(df[qg][kk][e]), bf2f(of[e]), dsum);
      if (DROP) {  // dP' = (dO/(1-p)).V: the keep-scale of dropout folded into dO once per wave
#pragma unroll
        for (int e = 0; e < 8; ++e) df[qg][kk][e] = f2bf(bf2f(df[qg][kk][e]) * inv_keep);
      }
    }
    lse2[qg] = lse[(size_t)bh * T + q] * kLog2e;
    dl[qg] = xor_sum(dsum);  // delta = dO . O (the dropped, normalised output), over the 4 lane groups
    if (wave_valid && g == 0) delta[(size_t)bh * T + q] = dl[qg];
  }
  const float sl2 = scale * kLog2e;
  [[maybe_unused]] const uint32_t tk2 = drop_tk2(thr > 0u ? thr : 1u);
  f32x4 dq[2][4];
#pragma unroll
  for (int qg = 0; qg < 2; ++qg)
#pragma unroll
    for (int f = 0; f < 4; ++f) dq[qg][f] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nkv = min((qb + 1) * BQ, T) / BKV;
  const uint32_t loff = tile_dma_off(ld, lane);
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const __amdgpu_buffer_rsrc_t rs = qkv_rsrc(base);
  tile_dma(smem, rs, 0, C + h * D, (int)ld, loff, wu);
  tile_dma(smem + BKV * 128, rs, 0, 2 * C + h * D, (int)ld, loff, wu);
  __syncthreads();
  for (int j = 0; j < nkv; ++j) {
    const int cur = j & 1;
    const char* Ks = smem + cur * 2 * BKV * 128;
    const char* Vs = Ks + BKV * 128;
    if (j + 1 < nkv) {  // next K/V tile by LDS-DMA into the stage released by tile j-1's barrier
      char* nxt = smem + (cur ^ 1) * 2 * BKV * 128;
      tile_dma(nxt, rs, (j + 1) * BKV, C + h * D, (int)ld, loff, wu);
      tile_dma(nxt + BKV * 128, rs, (j + 1) * BKV, 2 * C + h * D, (int)ld, loff, wu);
    }
    const int k_lo = j * BKV;
    if (wave_valid && k_lo <= q_lo + 31) {
      const bool diag = k_lo + BKV - 1 > q_lo;
      [[maybe_unused]] uint32_t pre = 0;
      if constexpr (DROP)
        pre = drop_pre(seed32(seed), ((uint32_t)bh * T + q_lo + (lane & 15)) * (uint32_t)T + k_lo + 4 * g);
      // S / dP of the 32 keys of half kk (fi = 2kk + f): s, dp [qg][f]
      auto sdp = [&](int kk, f32x4 (&s)[2][2], f32x4 (&dp)[2][2]) {
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          const int fi = 2 * kk + f;
          s[0][f] = s[1][f] = f32x4{0.f, 0.f, 0.f, 0.f};
          dp[0][f] = f32x4{-dl[0], -dl[0], -dl[0], -dl[0]};
          dp[1][f] = f32x4{-dl[1], -dl[1], -dl[1], -dl[1]};
#pragma unroll
          for (int k2 = 0; k2 < 2; ++k2) {
            const bf16x8 kf = row_frag(Ks, 16 * fi, k2, lane);
            const bf16x8 vf = row_frag(Vs, 16 * fi, k2, lane);
#pragma unroll
            for (int qg = 0; qg < 2; ++qg) {
              s[qg][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[qg][k2], s[qg][f], 0, 0, 0);
              dp[qg][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, df[qg][k2], dp[qg][f], 0, 0, 0);
            }
          }
        }
      };
      // dS of half kk, packed per query group
      auto elem = [&](auto diag_c, int kk, f32x4 (&s)[2][2], const f32x4 (&dp)[2][2], bf16x8 (&pk)[2]) {
        constexpr bool DIAG = decltype(diag_c)::value;
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          const int fi = 2 * kk + f;
#pragma unroll
          for (int r = 0; r < 4; r += 2) {  // keys r, r + 1: packed FMA / product pairs
            uint32_t km[2][2] = {{~0u, ~0u}, {~0u, ~0u}};
            if constexpr (DROP) {
#pragma unroll
              for (int e = 0; e < 2; ++e)
                drop_keep_masks(tk2, drop_fin(pre + (uint32_t)(16 * fi + r + e) * kDropC1, seed_kx(seed)), km[e][0],
                                km[e][1]);
            }
#pragma unroll
            for (int qg = 0; qg < 2; ++qg) {
              f32x2 p = exp2_affine2(s[qg][f][r], s[qg][f][r + 1], sl2, -lse2[qg]);
              f32x2 d = {dp[qg][f][r], dp[qg][f][r + 1]};
#pragma unroll
              for (int e = 0; e < 2; ++e) {
                if constexpr (DIAG) p[e] = (k_lo + 16 * fi + 4 * g + r + e > q_lo + 16 * qg + (lane & 15)) ? 0.f : p[e];
                if constexpr (DROP) d[e] = sel_mask(km[e][qg], d[e], -dl[qg]);
              }
              const f32x2 v = p * d;
              s[qg][f][r] = v[0];
              s[qg][f][r + 1] = v[1];
            }
          }
        }
        pk[0] = pack_perm(s[0], 0);
        pk[1] = pack_perm(s[1], 0);
      };
      auto dqm = [&](int kk, const bf16x8 (&pk)[2]) {
#pragma unroll
        for (int fd = 0; fd < 4; ++fd) {
          const bf16x8 kt = tr_frag(Ks, kk, 16 * fd, lane);
          dq[0][fd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kt, pk[0], dq[0][fd], 0, 0, 0);
          dq[1][fd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kt, pk[1], dq[1][fd], 0, 0, 0);
        }
      };
      auto tile = [&](auto diag_c) {
        f32x4 sa[2][2], dpa[2][2], sb[2][2], dpb[2][2];
        bf16x8 pa[2], pb[2];
        sdp(0, sa, dpa);
#if ATTN_DQ_SGB
        // A/B: the second half's S / dP MFMAs placed one by one among the first half's dS chain, then the first half's
        // dQ MFMAs among the second half's chain (fragment reads first in each region)
        __builtin_amdgcn_sched_barrier(0);
        elem(diag_c, 0, sa, dpa, pa);
        sdp(1, sb, dpb);
        __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, ATTN_DQ_FA, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        dqm(0, pa);
        elem(diag_c, 1, sb, dpb, pb);
        __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, ATTN_DQ_FB, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
#else
        elem(diag_c, 0, sa, dpa, pa);
        sdp(1, sb, dpb);
        __builtin_amdgcn_sched_barrier(0);
        dqm(0, pa);
        elem(diag_c, 1, sb, dpb, pb);
        __builtin_amdgcn_sched_barrier(0);
#endif
        dqm(1, pb);
      };
      if (diag) tile(std::true_type{});
      else tile(std::false_type{});
    }
    __syncthreads();
  }
  if (!wave_valid) return;
#pragma unroll
  for (int qg = 0; qg < 2; ++qg) {
    const int q = q_lo + 16 * qg + (lane & 15);
    const f32x4 qv[4] = {dq[qg][0], dq[qg][1], dq[qg][2], dq[qg][3]};
    store_row64(dqkv + ((size_t)b * T + q) * ld + h * D, qv, scale, lane);
  }
  if (csum) {  // partial qkv-bias gradient: row (b*T + q_lo)/32 of csum [B*T/32][3C], q columns
    const float cs = tile_colsum(dq, scale, lane);
    csum[((size_t)b * T + q_lo) / 32 * 3 * C + h * D + tile_colsum_col(lane)] = cs;
  }
}

// ---------------------------------------------------------------------------------------------
// dK, dV: key-outer (128 keys per workgroup, 32 per wave) over 32-query Q / dO tiles at or after the keys. The
// workgroup's K and V rows live in LDS (loaded once, V prescaled by 1/(1-p)) and the waves read their fragments per
// tile, instead of holding them in registers: 166 VGPRs, 3 waves / SIMD (the round-3 kernel held K / V in 32 VGPRs
// and took 64-query tiles at 224 VGPRs, 2 waves / SIMD: 339-354 -> 315 us per layer in the step, profiles/r4s/).
constexpr int BQ3 = 32;
template <bool DROP>
__global__ __launch_bounds__(256, 3) void attn_bwd_dkdv_kernel(const bf16* __restrict__ qkv,
                                                                 const bf16* __restrict__ dout,
                                                                 const float* __restrict__ lse,
                                                                 const float* __restrict__ delta,
                                                                 bf16* __restrict__ dqkv, float* __restrict__ csum,
                                                                 int T, int H, float scale, uint64_t seed,
                                                                 uint32_t thr, float inv_keep) {
  constexpr int kKV = BKB * 128;            // [128 keys][64 d] bf16
  constexpr int kTile = BQ3 * 128;          // [32 queries][64 d] bf16
  constexpr int kStage = 2 * kTile + 2 * BQ3 * 4;  // Q, dO, lse, delta
  __shared__ __attribute__((aligned(16))) char smem[2 * kKV + 2 * kStage];
  char* const Kl = smem;
  char* const Vl = smem + kKV;
  char* const stg = smem + 2 * kKV;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4;
  const int nqt = T / BQ3;
  int bh, kb;
  attn_block(bh, kb);
  const int b = bh / H, h = bh % H;
  const int C = H * D;
  const size_t ld = 3 * (size_t)C;
  const bf16* base = qkv + (size_t)b * T * ld;
#if ATTN_DKDV_PIPE == 0
  const int k_lo = kb * 128 + 32 * w;
#else
  const int k_lo = kb * 128 + 32 * __builtin_amdgcn_readfirstlane(w);  // wave-uniform: scalar branches on it
#endif
  const bool wave_valid = k_lo < T;
  // K and V rows kb*128 .. +128 (clamped to T - 1 past the end: only invalid waves read those) into LDS, swizzled as
  // every tile (t_off); 4 chunks of 16 B per thread and array
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = threadIdx.x + 256 * i, row = idx >> 3, ch = idx & 7;
    const size_t src = (size_t)min(kb * 128 + row, T - 1) * ld + h * D + 8 * ch;
    const bf16x8 kv = *reinterpret_cast<const bf16x8*>(base + src + C);
    bf16x8 vv = *reinterpret_cast<const bf16x8*>(base + src + 2 * C);
    if (DROP) {
#pragma unroll
      for (int e = 0; e < 8; ++e) vv[e] = f2bf(bf2f(vv[e]) * inv_keep);
    }
    *reinterpret_cast<bf16x8*>(Kl + t_off(row, ch)) = kv;
    *reinterpret_cast<bf16x8*>(Vl + t_off(row, ch)) = vv;
  }
  const float sl2 = scale * kLog2e;
  [[maybe_unused]] const uint32_t tk2 = drop_tk2(thr > 0u ? thr : 1u);
  f32x4 dk[2][4], dv[2][4];
#pragma unroll
  for (int kg = 0; kg < 2; ++kg)
#pragma unroll
    for (int f = 0; f < 4; ++f) dk[kg][f] = dv[kg][f] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float* lrow = lse + (size_t)bh * T;
  const float* drow = delta + (size_t)bh * T;
  float rl = 0.f, rdl = 0.f;
  const uint32_t qoff = tile_dma_off(ld, lane), doff = tile_dma_off(C, lane);
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const __amdgpu_buffer_rsrc_t rsq = qkv_rsrc(base), rsd = qkv_rsrc(dout + (size_t)b * T * C);
  // Q / dO tiles (32 rows: one DMA instruction per wave and array); lse / delta by registers
  auto gload = [&](int i, char* st) {
    tile_dma<8>(st, rsq, i * BQ3, h * D, (int)ld, qoff, wu);
    tile_dma<8>(st + kTile, rsd, i * BQ3, h * D, C, doff, wu);
    if (threadIdx.x < BQ3) {
      rl = lrow[i * BQ3 + threadIdx.x];
      rdl = drow[i * BQ3 + threadIdx.x];
    }
  };
  auto sstore = [&](char* st) {
    if (threadIdx.x < BQ3) {
      // both negated: the FMA addend and the dropped-key value of dP - delta as stored (no per-tile negations)
      reinterpret_cast<float*>(st + 2 * kTile)[threadIdx.x] = -(rl * kLog2e);
      reinterpret_cast<float*>(st + 2 * kTile + BQ3 * 4)[threadIdx.x] = -rdl;
    }
  };
  const int i0 = kb * 128 / BQ3;
  gload(i0, stg);
  sstore(stg);
  __syncthreads();
  const char* Kw = Kl + 32 * w * 128;  // this wave's 32 keys
  const char* Vw = Vl + 32 * w * 128;
#if ATTN_DKDV_PIPE == 0
  for (int i = i0; i < nqt; ++i) {
    const int cur = (i - i0) & 1;
    const char* Qs = stg + cur * kStage;
    const char* Ds = Qs + kTile;
    const float* Ls = reinterpret_cast<const float*>(Qs + 2 * kTile);
    const float* Dl = Ls + BQ3;
    if (i + 1 < nqt) gload(i + 1, stg + (cur ^ 1) * kStage);
    const int q0 = i * BQ3;
    if (wave_valid && q0 + BQ3 - 1 >= k_lo) {
      const bool diag = q0 < k_lo + 31;
      const uint32_t pre_t = DROP ? drop_pre(seed32(seed), ((uint32_t)bh * T + q0 + 4 * g) * (uint32_t)T + k_lo + (lane & 15)) : 0u;
      f32x4 s[2][2], dp[2][2];  // [kg][fl]: S[q = q0 + 16fl + 4g + r][key = k_lo + 16kg + (l&15)]
      f32x4 nl4[2], nd4[2];  // -lse * log2(e), -delta of the tile's queries
#pragma unroll
      for (int fl = 0; fl < 2; ++fl) {
        nl4[fl] = *reinterpret_cast<const f32x4*>(Ls + 16 * fl + 4 * g);
        nd4[fl] = *reinterpret_cast<const f32x4*>(Dl + 16 * fl + 4 * g);
        s[0][fl] = s[1][fl] = f32x4{0.f, 0.f, 0.f, 0.f};
        dp[0][fl] = dp[1][fl] = nd4[fl];
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 kfr[2], vfr[2];
#pragma unroll
        for (int kg = 0; kg < 2; ++kg) {
          kfr[kg] = row_frag(Kw, 16 * kg, kk, lane);
          vfr[kg] = row_frag(Vw, 16 * kg, kk, lane);
        }
#pragma unroll
        for (int fl = 0; fl < 2; ++fl) {
          const bf16x8 qa = row_frag(Qs, 16 * fl, kk, lane);
          const bf16x8 da = row_frag(Ds, 16 * fl, kk, lane);
#pragma unroll
          for (int kg = 0; kg < 2; ++kg) {
            s[kg][fl] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa, kfr[kg], s[kg][fl], 0, 0, 0);
            dp[kg][fl] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da, vfr[kg], dp[kg][fl], 0, 0, 0);
          }
        }
      }
      auto elementwise = [&](auto diag_c) {
        constexpr bool DIAG = decltype(diag_c)::value;
#pragma unroll
        for (int kg = 0; kg < 2; ++kg) {
          const int key = k_lo + 16 * kg + (lane & 15);
          // the scores' affine part in place, as packed FMA pairs (v_pk_fma_f32; no register beyond s): x = s * sl2 - lse
#pragma unroll
          for (int fl = 0; fl < 2; ++fl)
#pragma unroll
            for (int r = 0; r < 4; r += 2) {
              const f32x2 t = __builtin_elementwise_fma(f32x2{s[kg][fl][r], s[kg][fl][r + 1]}, f32x2{sl2, sl2},
                                                        f32x2{nl4[fl][r], nl4[fl][r + 1]});
              s[kg][fl][r] = t[0];
              s[kg][fl][r + 1] = t[1];
            }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            uint32_t km[2] = {~0u, ~0u};
            if constexpr (DROP) {
#if ATTN_HASH_ANCHOR
              // the counter of this (r, kg) formed, then made opaque: hashed here, not hoisted ahead of the tile (its
              // masks would not fit), and the add writes a fresh register (no copy of pre_t per hash)
              const uint32_t off = __builtin_amdgcn_readfirstlane(((uint32_t)r * (uint32_t)T + 16u * kg) * kDropC1);
              uint32_t pv;
              asm volatile("v_add_u32 %0, %1, %2" : "=v"(pv) : "s"(off), "v"(pre_t));
              drop_keep_masks(tk2, drop_fin(pv, seed_kx(seed)), km[0], km[1]);
#else
              uint32_t pv = pre_t;
              asm volatile("" : "+v"(pv));  // hashed here, not hoisted ahead of the tile (its masks would not fit)
              drop_keep_masks(tk2, drop_fin(pv + ((uint32_t)r * (uint32_t)T + 16u * kg) * kDropC1, seed_kx(seed)),
                              km[0], km[1]);
#endif
            }
#pragma unroll
            for (int fl = 0; fl < 2; ++fl) {
              float p = __builtin_amdgcn_exp2f(s[kg][fl][r]);
              if constexpr (DIAG) p = (q0 + 16 * fl + 4 * g + r < key) ? 0.f : p;
              float pdv = p, d = dp[kg][fl][r];
              if constexpr (DROP) {
                pdv = __uint_as_float(km[fl] & __float_as_uint(p));
                d = sel_mask(km[fl], d, nd4[fl][r]);
              }
              dp[kg][fl][r] = pdv;
              s[kg][fl][r] = p * d;
            }
          }
        }
      };
      if (diag) elementwise(std::true_type{});
      else elementwise(std::false_type{});
      const bf16x8 p0 = pack_perm(dp[0], 0), p1 = pack_perm(dp[1], 0);
      const bf16x8 s0 = pack_perm(s[0], 0), s1 = pack_perm(s[1], 0);
#pragma unroll
      for (int fd = 0; fd < 4; ++fd) {
        const bf16x8 dot = tr_frag(Ds, 0, 16 * fd, lane);
        const bf16x8 qt = tr_frag(Qs, 0, 16 * fd, lane);
        dv[0][fd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dot, p0, dv[0][fd], 0, 0, 0);
        dv[1][fd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dot, p1, dv[1][fd], 0, 0, 0);
        dk[0][fd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qt, s0, dk[0][fd], 0, 0, 0);
        dk[1][fd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qt, s1, dk[1][fd], 0, 0, 0);
      }
    }
    if (i + 1 < nqt) sstore(stg + (cur ^ 1) * kStage);
    __syncthreads();
  }
#else
  // one query tile: Q / dO / lse / delta of tile i are in stage (i - i0) & 1; the next tile is staged under it
  auto step = [&](int i, auto work) {
    const int cur = (i - i0) & 1;
    const char* Qs = stg + cur * kStage;
    const char* Ds = Qs + kTile;
    const float* Ls = reinterpret_cast<const float*>(Qs + 2 * kTile);
    const float* Dl = Ls + BQ3;
    if (i + 1 < nqt) gload(i + 1, stg + (cur ^ 1) * kStage);
    work(i * BQ3, Qs, Ds, Ls, Dl);
    if (i + 1 < nqt) sstore(stg + (cur ^ 1) * kStage);
    __syncthreads();
  };
  // the general tile: a wave may be inactive (its keys after the tile's queries) or on the causal diagonal
  auto general = [&](const int q0, const char* Qs, const char* Ds, const float* Ls, const float* Dl) {
      if (wave_valid && q0 + BQ3 - 1 >= k_lo) {
        const bool diag = q0 < k_lo + 31;
        const uint32_t pre_t = DROP ? drop_pre(seed32(seed), ((uint32_t)bh * T + q0 + 4 * g) * (uint32_t)T + k_lo + (lane & 15)) : 0u;
        f32x4 s[2][2], dp[2][2];  // [kg][fl]: S[q = q0 + 16fl + 4g + r][key = k_lo + 16kg + (l&15)]
        f32x4 nl4[2], nd4[2];  // -lse * log2(e), -delta of the tile's queries
#pragma unroll
        for (int fl = 0; fl < 2; ++fl) {
          nl4[fl] = *reinterpret_cast<const f32x4*>(Ls + 16 * fl + 4 * g);
          nd4[fl] = *reinterpret_cast<const f32x4*>(Dl + 16 * fl + 4 * g);
          s[0][fl] = s[1][fl] = f32x4{0.f, 0.f, 0.f, 0.f};
          dp[0][fl] = dp[1][fl] = nd4[fl];
        }
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          bf16x8 kfr[2], vfr[2];
#pragma unroll
          for (int kg = 0; kg < 2; ++kg) {
            kfr[kg] = row_frag(Kw, 16 * kg, kk, lane);
            vfr[kg] = row_frag(Vw, 16 * kg, kk, lane);
          }
#pragma unroll
          for (int fl = 0; fl < 2; ++fl) {
            const bf16x8 qa = row_frag(Qs, 16 * fl, kk, lane);
            const bf16x8 da = row_frag(Ds, 16 * fl, kk, lane);
#pragma unroll
            for (int kg = 0; kg < 2; ++kg) {
              s[kg][fl] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa, kfr[kg], s[kg][fl], 0, 0, 0);
              dp[kg][fl] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da, vfr[kg], dp[kg][fl], 0, 0, 0);
            }
          }
        }
        auto elementwise = [&](auto diag_c) {
          constexpr bool DIAG = decltype(diag_c)::value;
#pragma unroll
          for (int kg = 0; kg < 2; ++kg) {
            const int key = k_lo + 16 * kg + (lane & 15);
            // the scores' affine part in place, as packed FMA pairs (v_pk_fma_f32; no register beyond s): x = s * sl2 - lse
#pragma unroll
            for (int fl = 0; fl < 2; ++fl)
#pragma unroll
              for (int r = 0; r < 4; r += 2) {
                const f32x2 t = __builtin_elementwise_fma(f32x2{s[kg][fl][r], s[kg][fl][r + 1]}, f32x2{sl2, sl2},
                                                          f32x2{nl4[fl][r], nl4[fl][r + 1]});
                s[kg][fl][r] = t[0];
                s[kg][fl][r + 1] = t[1];
              }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              uint32_t km[2] = {~0u, ~0u};
              if constexpr (DROP) {
                uint32_t pv = pre_t;
                asm volatile("" : "+v"(pv));  // hashed here, not hoisted ahead of the tile (its masks would not fit)
                drop_keep_masks(tk2, drop_fin(pv + ((uint32_t)r * (uint32_t)T + 16u * kg) * kDropC1, seed_kx(seed)),
                                km[0], km[1]);
              }
#pragma unroll
              for (int fl = 0; fl < 2; ++fl) {
                float p = __builtin_amdgcn_exp2f(s[kg][fl][r]);
                if constexpr (DIAG) p = (q0 + 16 * fl + 4 * g + r < key) ? 0.f : p;
                float pdv = p, d = dp[kg][fl][r];
                if constexpr (DROP) {
                  pdv = __uint_as_float(km[fl] & __float_as_uint(p));
                  d = sel_mask(km[fl], d, nd4[fl][r]);
                }
                dp[kg][fl][r] = pdv;
                s[kg][fl][r] = p * d;
              }
            }
          }
        };
        if (diag) elementwise(std::true_type{});
        else elementwise(std::false_type{});
        const bf16x8 p0 = pack_perm(dp[0], 0), p1 = pack_perm(dp[1], 0);
        const bf16x8 s0 = pack_perm(s[0], 0), s1 = pack_perm(s[1], 0);
#pragma unroll
        for (int fd = 0; fd < 4; ++fd) {
          const bf16x8 dot = tr_frag(Ds, 0, 16 * fd, lane);
          const bf16x8 qt = tr_frag(Qs, 0, 16 * fd, lane);
          dv[0][fd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dot, p0, dv[0][fd], 0, 0, 0);
          dv[1][fd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dot, p1, dv[1][fd], 0, 0, 0);
          dk[0][fd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qt, s0, dk[0][fd], 0, 0, 0);
          dk[1][fd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qt, s1, dk[1][fd], 0, 0, 0);
        }
      }
  };
  // Tiles i0 .. i0 + 3 hold every wave's diagonal tile (wave w: i0 + w) and the inactive waves; from i0 + 4 on every
  // wave of the workgroup is active and off the diagonal, and the tile is ONE basic block: the S / dP MFMAs, the
  // elementwise chain and the dV / dK MFMAs scheduled together (key group kg = 0 finished first, its dS formed while
  // kg = 1's S / dP MFMAs run, its dV / dK MFMAs issued beside kg = 1's elementwise). The Q / dO row fragments are
  // read per key group (re-read for kg = 1: 8 more ds_read_b128 per tile) instead of held for both (32 VGPRs past
  // the 3-waves / SIMD budget).
  for (int i = i0; i < min(i0 + 4, nqt); ++i) step(i, general);
  auto steady = [&](const int q0, const char* Qs, const char* Ds, const float* Ls, const float* Dl) {
    const uint32_t pre_t = DROP ? drop_pre(seed32(seed), ((uint32_t)bh * T + q0 + 4 * g) * (uint32_t)T + k_lo + (lane & 15)) : 0u;
    auto tile = [&]() {
      constexpr bool DIAG = false;
      f32x4 s[2][2], dp[2][2];  // [kg][fl]: S[q = q0 + 16fl + 4g + r][key = k_lo + 16kg + (l&15)]
      f32x4 nl4[2], nd4[2];  // -lse * log2(e), -delta of the tile's queries
#pragma unroll
      for (int fl = 0; fl < 2; ++fl) {
        nl4[fl] = *reinterpret_cast<const f32x4*>(Ls + 16 * fl + 4 * g);
        nd4[fl] = *reinterpret_cast<const f32x4*>(Dl + 16 * fl + 4 * g);
      }
      auto sdp = [&](int kg) {
#pragma unroll
        for (int fl = 0; fl < 2; ++fl) {
          s[kg][fl] = f32x4{0.f, 0.f, 0.f, 0.f};
          dp[kg][fl] = nd4[fl];
        }
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const bf16x8 kf = row_frag(Kw, 16 * kg, kk, lane), vf = row_frag(Vw, 16 * kg, kk, lane);
#pragma unroll
          for (int fl = 0; fl < 2; ++fl) {
            const bf16x8 qa = row_frag(Qs, 16 * fl, kk, lane);
            const bf16x8 da = row_frag(Ds, 16 * fl, kk, lane);
            s[kg][fl] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa, kf, s[kg][fl], 0, 0, 0);
            dp[kg][fl] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da, vf, dp[kg][fl], 0, 0, 0);
          }
        }
      };
      auto elem = [&](int kg) {
        const int key = k_lo + 16 * kg + (lane & 15);
#pragma unroll
        for (int fl = 0; fl < 2; ++fl)
#pragma unroll
          for (int r = 0; r < 4; r += 2) {
            const f32x2 t = __builtin_elementwise_fma(f32x2{s[kg][fl][r], s[kg][fl][r + 1]}, f32x2{sl2, sl2},
                                                      f32x2{nl4[fl][r], nl4[fl][r + 1]});
            s[kg][fl][r] = t[0];
            s[kg][fl][r + 1] = t[1];
          }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          uint32_t km[2] = {~0u, ~0u};
          if constexpr (DROP) {
            uint32_t pv = pre_t;
            asm volatile("" : "+v"(pv));  // hashed here, not hoisted ahead of the tile (its masks would not fit)
            drop_keep_masks(tk2, drop_fin(pv + ((uint32_t)r * (uint32_t)T + 16u * kg) * kDropC1, seed_kx(seed)),
                            km[0], km[1]);
          }
#pragma unroll
          for (int fl = 0; fl < 2; ++fl) {
            float p = __builtin_amdgcn_exp2f(s[kg][fl][r]);
            if constexpr (DIAG) p = (q0 + 16 * fl + 4 * g + r < key) ? 0.f : p;
            float pdv = p, d = dp[kg][fl][r];
            if constexpr (DROP) {
              pdv = __uint_as_float(km[fl] & __float_as_uint(p));
              d = sel_mask(km[fl], d, nd4[fl][r]);
            }
            dp[kg][fl][r] = pdv;
            s[kg][fl][r] = p * d;
          }
        }
      };
      auto dvdk = [&](int kg) {
        const bf16x8 pp = pack_perm(dp[kg], 0), ss = pack_perm(s[kg], 0);
#pragma unroll
        for (int fd = 0; fd < 4; ++fd) {
          const bf16x8 dot = tr_frag(Ds, 0, 16 * fd, lane);
          const bf16x8 qt = tr_frag(Qs, 0, 16 * fd, lane);
          dv[kg][fd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dot, pp, dv[kg][fd], 0, 0, 0);
          dk[kg][fd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qt, ss, dk[kg][fd], 0, 0, 0);
        }
      };
#if ATTN_DKDV_PIPE == 1  // program order by phase, the scheduler free within the block
      sdp(0);
      sdp(1);
      elem(0);
      elem(1);
      dvdk(0);
      dvdk(1);
#elif ATTN_DKDV_PIPE == 2  // program order by key group
      sdp(0);
      sdp(1);
      elem(0);
      dvdk(0);
      elem(1);
      dvdk(1);
#elif ATTN_DKDV_PIPE == 4  // phases fenced (register-pressure check)
      sdp(0);
      __builtin_amdgcn_sched_barrier(0);
      sdp(1);
      __builtin_amdgcn_sched_barrier(0);
      elem(0);
      __builtin_amdgcn_sched_barrier(0);
      dvdk(0);
      __builtin_amdgcn_sched_barrier(0);
      elem(1);
      __builtin_amdgcn_sched_barrier(0);
      dvdk(1);
#else  // 3: key-group pipeline with the MFMAs of one group spread through the other group's elementwise
      sdp(0);
      __builtin_amdgcn_sched_barrier(0);
      sdp(1);
      elem(0);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, ATTN_DKDV_FILL, 0);  // VALU
      }
      __builtin_amdgcn_sched_barrier(0);
      dvdk(0);
      elem(1);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);
        __builtin_amdgcn_sched_group_barrier(0x002, ATTN_DKDV_FILL, 1);
      }
      __builtin_amdgcn_sched_barrier(0);
      dvdk(1);
#endif
    };
    tile();
  };
  for (int i = i0 + 4; i < nqt; ++i) step(i, steady);
#endif
  if (!wave_valid) return;
#pragma unroll
  for (int kg = 0; kg < 2; ++kg) {
    const int key = k_lo + 16 * kg + (lane & 15);
    bf16* kout = dqkv + ((size_t)b * T + key) * ld + C + h * D;
    const f32x4 kv[4] = {dk[kg][0], dk[kg][1], dk[kg][2], dk[kg][3]};
    const f32x4 vv[4] = {dv[kg][0], dv[kg][1], dv[kg][2], dv[kg][3]};
    store_row64(kout, kv, scale, lane);
    store_row64(kout + C, vv, DROP ? inv_keep : 1.f, lane);
  }
  if (csum) {
    float* crow = csum + ((size_t)b * T + k_lo) / 32 * 3 * C + C + h * D + tile_colsum_col(lane);
    const float ck = tile_colsum(dk, scale, lane);
    const float cv = tile_colsum(dv, DROP ? inv_keep : 1.f, lane);
    crow[0] = ck;
    crow[C] = cv;
  }
}

}  // namespace

GPT2MI_EXPORT int gpt2mi_attn_fwd(const uint16_t* qkv, uint16_t* out, float* lse, int B, int T, int H, int head_dim,
                                  float p_drop, uint64_t seed, void* stream) {
  GPT2MI_REQUIRE(head_dim == D, "attn_fwd: head_dim=%d (only 64 is built)", head_dim);
  GPT2MI_REQUIRE(p_drop <= 0.f || (size_t)B * H * T * T < (1ull << 32),
                 "attn_fwd: B*H*T*T exceeds the 32-bit dropout hash index");
  GPT2MI_REQUIRE(T % 64 == 0 && T > 0, "attn_fwd: T=%d must be a multiple of 64", T);
  GPT2MI_REQUIRE((size_t)T * 3 * H * D * sizeof(bf16) < (1ull << 31),
                 "attn_fwd: T*3C too large for the 32-bit buffer offsets of one batch row (T=%d)", T);
  const float scale = 1.f / sqrtf((float)head_dim);
  dim3 grid((T + BQ - 1) / BQ, B * H);
  const uint32_t thr = drop_threshold(p_drop);
  const float ik = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  if (thr)
    attn_fwd_kernel<true><<<grid, kThreads, 0, (hipStream_t)stream>>>((const bf16*)qkv, (bf16*)out, lse, T, H, scale,
                                                                      seed, thr, ik);
  else
    attn_fwd_kernel<false><<<grid, kThreads, 0, (hipStream_t)stream>>>((const bf16*)qkv, (bf16*)out, lse, T, H, scale,
                                                                       seed, thr, ik);
  return gpt2mi::check_launch("attn_fwd");
}

GPT2MI_EXPORT int gpt2mi_attn_bwd(const uint16_t* qkv, const uint16_t* out, const uint16_t* dout, const float* lse,
                                  float* delta, uint16_t* dqkv, float* dqkv_colsum, int B, int T, int H,
                                  int head_dim, float p_drop, uint64_t seed, void* stream) {
  GPT2MI_REQUIRE(head_dim == D, "attn_bwd: head_dim=%d (only 64 is built)", head_dim);
  GPT2MI_REQUIRE(p_drop <= 0.f || (size_t)B * H * T * T < (1ull << 32),
                 "attn_bwd: B*H*T*T exceeds the 32-bit dropout hash index");
  GPT2MI_REQUIRE(T % 64 == 0 && T > 0, "attn_bwd: T=%d must be a multiple of 64", T);
  GPT2MI_REQUIRE((size_t)T * 3 * H * D * sizeof(bf16) < (1ull << 31),
                 "attn_bwd: T*3C too large for the 32-bit buffer offsets of one batch row (T=%d)", T);
  hipStream_t s = (hipStream_t)stream;
  const float scale = 1.f / sqrtf((float)head_dim);
  const uint32_t thr = drop_threshold(p_drop);
  const float ik = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  // dQ first: it forms delta (dO . O per query) for the dK/dV kernel
  const dim3 gq((T + BQ - 1) / BQ, B * H);
  if (thr)
    attn_bwd_dq_kernel<true><<<gq, kThreads, 0, s>>>((const bf16*)qkv, (const bf16*)out, (const bf16*)dout, lse, delta,
                                                     (bf16*)dqkv, dqkv_colsum, T, H, scale, seed, thr, ik);
  else
    attn_bwd_dq_kernel<false><<<gq, kThreads, 0, s>>>((const bf16*)qkv, (const bf16*)out, (const bf16*)dout, lse,
                                                      delta, (bf16*)dqkv, dqkv_colsum, T, H, scale, seed, thr, ik);
  int rc = gpt2mi::check_launch("attn_bwd_dq");
  if (rc) return rc;
  const dim3 gkv((T + BKB - 1) / BKB, B * H);
  if (thr)
    attn_bwd_dkdv_kernel<true><<<gkv, 256, 0, s>>>((const bf16*)qkv, (const bf16*)dout, lse, delta, (bf16*)dqkv,
                                                    dqkv_colsum, T, H, scale, seed, thr, ik);
  else
    attn_bwd_dkdv_kernel<false><<<gkv, 256, 0, s>>>((const bf16*)qkv, (const bf16*)dout, lse, delta, (bf16*)dqkv,
                                                     dqkv_colsum, T, H, scale, seed, thr, ik);
  return gpt2mi::check_launch("attn_bwd_dkdv");
}
