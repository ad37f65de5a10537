// bf16 matrix transpose for the transposed weight shadow (engine.py): every nn.Linear weight W[out][in]
// is also kept as W^T[in][out], so the backward dgrad dX = dY.W runs as the forward-layout GEMM
// dY.(W^T)^T with both operands k-contiguous (ds_read_b128 fragments instead of the transposed
// ds_read_b64_tr_b16 pairs: measured 1590 vs 1231 TF at 8192^3, tools/gemm_probe.py).
// 64x64 tiles through LDS (+2-element row pad: conflict-free column reads), 16-B global accesses.
#include "common.h"

namespace {

constexpr int TT = 64;

// one 64x64 tile (r0, c0) of src[R][C] (leading dim lds) into dst[C][R] (leading dim ldd)
__device__ __forceinline__ void transpose_tile(const bf16* __restrict__ src, bf16* __restrict__ dst, int r0, int c0,
                                               int lds, int ldd) {
  __shared__ bf16 tile[TT][TT + 2];
  const int t = threadIdx.x;
  // load: 64 rows x 8 chunks of 8 elements = 512 chunks, 2 per thread
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int id = t + 256 * k, r = id >> 3, ch = id & 7;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(src + (size_t)(r0 + r) * lds + c0 + 8 * ch);
#pragma unroll
    for (int j = 0; j < 8; ++j) tile[r][8 * ch + j] = v[j];
  }
  __syncthreads();
  // store: output row c (= input column), 8 consecutive input rows per chunk
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int id = t + 256 * k, c = id >> 3, ch = id & 7;
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = tile[8 * ch + j][c];
    *reinterpret_cast<bf16x8*>(dst + (size_t)(c0 + c) * ldd + r0 + 8 * ch) = v;
  }
}

__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16* __restrict__ src, bf16* __restrict__ dst,
                                                            int R, int C, int lds, int ldd) {
  transpose_tile(src, dst, blockIdx.y * TT, blockIdx.x * TT, lds, ldd);
}

// Every weight of the shadow arena in one launch: desc[i] = {element offset, R, C, first tile} (dense
// [R][C] at src + offset -> [C][R] at dst + offset), blocks walk the flat tile range.
__global__ __launch_bounds__(256) void transpose_bf16_batched_kernel(const bf16* __restrict__ src,
                                                                    bf16* __restrict__ dst,
                                                                    const int64_t* __restrict__ desc, int n) {
  const int64_t tile = blockIdx.x;
  // the matrix holding this tile: the last i with first_tile(i) <= tile (binary search over the sorted first tiles:
  // GPT-2 1.5B has 193 matrices, and a linear scan of dependent scalar loads per block took the 1.5B refresh to 2.8 ms,
  // 2.1 TB/s, against 4.6 TB/s at 124M's 49)
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (desc[4 * mid + 3] <= tile) lo = mid;
    else hi = mid - 1;
  }
  const int i = lo;
  const int64_t off = desc[4 * i], R = desc[4 * i + 1], C = desc[4 * i + 2], t = tile - desc[4 * i + 3];
  const int tc = (int)(C / TT);
  transpose_tile(src + off, dst + off, (int)(t / tc) * TT, (int)(t % tc) * TT, (int)C, (int)R);
}

}  // namespace

GPT2MI_EXPORT int gpt2mi_transpose_bf16(const uint16_t* src, uint16_t* dst, int R, int C, int ld_src, int ld_dst,
                                        void* stream) {
  GPT2MI_REQUIRE(R > 0 && C > 0 && R % TT == 0 && C % TT == 0, "transpose_bf16: R=%d and C=%d must be multiples of 64",
                 R, C);
  GPT2MI_REQUIRE(ld_src % 8 == 0 && ld_dst % 8 == 0 && ld_src >= C && ld_dst >= R,
                 "transpose_bf16: bad leading dimensions %d / %d", ld_src, ld_dst);
  transpose_bf16_kernel<<<dim3(C / TT, R / TT), 256, 0, (hipStream_t)stream>>>((const bf16*)src, (bf16*)dst, R, C,
                                                                               ld_src, ld_dst);
  return gpt2mi::check_launch("transpose_bf16");
}

GPT2MI_EXPORT int gpt2mi_transpose_bf16_batched(const uint16_t* src, uint16_t* dst, const int64_t* desc, int n,
                                                int64_t total_tiles, void* stream) {
  GPT2MI_REQUIRE(n > 0 && total_tiles > 0 && total_tiles < (1ll << 31), "transpose_bf16_batched: n=%d tiles=%lld", n,
                 (long long)total_tiles);
  transpose_bf16_batched_kernel<<<dim3((unsigned)total_tiles), 256, 0, (hipStream_t)stream>>>(
      (const bf16*)src, (bf16*)dst, desc, n);
  return gpt2mi::check_launch("transpose_bf16_batched");
}
