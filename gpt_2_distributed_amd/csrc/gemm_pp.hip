// bf16 MFMA GEMM, 256x256x64 block tile, "ping-pong" 4-phase K-step — the main GEMM of the step.
//
// Same contract and epilogues as gemm.hip / gemm256.hip (C = epi(alpha * A.B^T), layouts 0/1/2).
//
// Structure (CDNA4 idiom: 2 waves per SIMD that alternate MFMA and memory work):
//  * 512 threads = 8 waves = 2 groups of 4 (group g = wave>>2, one wave of each group per SIMD).
//    Wave (g, c) owns a 2x2 grid of 64x32 quadrants (mi, ni): rows mi*128 + g*64..+64, columns
//    ni*128 + c*32..+32; a quadrant x K=64 is 16 v_mfma_f32_16x16x32_bf16.
//  * A K-tile is staged as four 16 KiB "half-tiles" A_0/A_1 (rows 0-127 / 128-255) and B_0/B_1
//    (columns 0-127 / 128-255): contiguous 256-B global segments for m-contiguous operands. Two
//    K-tile buffers = 128 KiB LDS, filled only by LDS-DMA (global_load_lds_dwordx4, 2 per wave per
//    half-tile).
//  * One K-tile = 4 phases; phase p: ds_read the quadrant's new operands, issue one half-tile DMA,
//    s_waitcnt vmcnt(8), s_barrier, MFMA the quadrant at s_setprio 1, s_barrier. Group 1 starts one
//    barrier late, so in every barrier interval one group runs MFMAs while the other reads LDS /
//    issues DMA. B_0 stays in registers from phase 1 to phase 4, so every slot dies early:
//        phase  quadrant   reads        DMA issued (into)
//          1    (0,0)      A_0, B_0     B_1 of tile t+1   (buffer t+1; last read 3 phases ago)
//          2    (0,1)      B_1          A_1 of tile t+1   (buffer t+1; last read 3 phases ago)
//          3    (1,1)      A_1          A_0 of tile t+2   (buffer t, read last in phase 1)
//          4    (1,0)      -            B_0 of tile t+2   (buffer t, read last in phase 1)
//    Every slot is restaged >= 2 phases after its last read (WAR across the group stagger) and
//    each half-tile is issued 5-6 phases before its first read: the counted `vmcnt(8)` of every
//    phase keeps 4 half-tiles (64 KiB per CU) in flight across the barrier and retires exactly the
//    half-tile the next phase reads (RAW: wait in phase p, read in phase p+1).
//    The last K-tile pair issues no DMA past the end and counts its waits down instead.
//  * Operand images: k-contiguous operands [128][64] bf16 (128-B rows, 16-B chunk c at c^(row&7),
//    ds_read_b128); m-contiguous operands [64][128] (256-B rows, chunk c at c^swz(k),
//    ds_read_b64_tr_b16). The swizzle is applied on the DMA source address (the LDS side of an
//    LDS-DMA is lane-linear) and undone on the read.
//  * Epilogue through LDS: the MFMA is issued as D^T = B.A^T (a lane owns 4 consecutive columns);
//    the block writes its fp32 accumulators into a [128][256] row-major LDS image (two passes of
//    128 rows, 16-B chunk c of row r at c ^ (r & 15): conflict-free both ways), then every wave
//    reads back whole rows and applies the fused epilogue with full-row coalesced stores (one
//    store instruction = one 256-column output row).
#include <atomic>
#include <type_traits>

#include "common.h"
#include "gemm_common.h"

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
// The B fragments of the next K-tile read in phase 4 (kEarly in gemm_pp_kernel; PP_B0_EARLY=0: the round-2 schedule
// everywhere, for A/B builds)
#ifndef PP_B0_EARLY
#define PP_B0_EARLY 1
#endif
GPT2MI_PRODUCT_KNOB(PP_B0_EARLY, 1);
constexpr int kThreads = 512;
constexpr int kHalf = 128 * BK * 2;  // 16 KiB
constexpr int kBuf = 4 * kHalf;      // A_0, A_1, B_0, B_1
constexpr int kLds = 2 * kBuf;       // 128 KiB
constexpr int SA0 = 0, SA1 = kHalf, SB0 = 2 * kHalf, SB1 = 3 * kHalf;

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ int mc_swz(int k) { return 2 * ((k & 3) | (((k >> 3) & 1) << 2)); }

// image row/col ir (0..127) of half `h` -> offset inside the 256-wide block dimension
//   contiguous (default): A_h / B_h = rows / columns h*128 + ir
//   interleaved (A/B experiments): A_h = 64-row slice h of each 128-row group, B_h = 32-column slice
//   h of each 64-column group
template <bool INTERLEAVED, bool IS_A>
__device__ __forceinline__ int half_map(int ir, int h) {
  if constexpr (!INTERLEAVED) return (h << 7) + ir;
  else if constexpr (IS_A) return ((ir >> 6) << 7) + (h << 6) + (ir & 63);
  else return ((ir >> 5) << 6) + (h << 5) + (ir & 31);
}

// One half-tile by LDS-DMA: 16 x 1 KiB instructions, 2 per wave.
//   TRANS=0 (k-contiguous, src[row][k]): instruction covers image rows 8*ins..+8; per-lane 64-bit addresses
//     (global_load_lds), rows clamped to rmax (the operand's last row) for a partial last tile. (A buffer DMA with a
//     descriptor per instruction ran these shapes 10-20 % slower: lm_head dgrad 3.64 -> 4.09 ms.)
//   TRANS=1 (m-contiguous, src[k][row]): instruction covers k-rows 4*ins..+4, by buffer DMA: a lane's source offset
//     is the same for every instruction, half and K-tile (one VGPR, dma_lane_off) and the instruction's position a
//     wave-uniform 64-bit base in its descriptor (SALU), so the wgrad keeps no per-lane 64-bit pointers across the
//     main loop (fits its 256 VGPRs with the phase-4 B reads, kEarly). A partial last tile (extent % 256 != 0, a
//     multiple of 64) reads past the row's end — the next row's elements, which only feed outputs the epilogue does
//     not store; with BND (the launch has such a partial tile) the descriptor's num_records ends at the operand's last
//     element ((K - 1) * ld + extent), so lanes past the last row read zeros instead of whatever follows the operand in
//     memory. Full tiles never read past their rows: BND = false skips the bound, whose per-DMA scalar arithmetic cost
//     the weight gradients 10-15 % (qkv 199 -> 236 us, tools/lib_ab.py, round 4).
// zero: the zero K-tile of an odd K-tile count (TRANS=0: every lane reads 16 zero bytes; TRANS=1: num_records 0).
// 16 zero bytes: the source of every lane of a zero K-tile's flat DMAs
__device__ const u32x4 g_zero16 = {0u, 0u, 0u, 0u};

template <bool TRANS, bool IS_A, bool IL>
__device__ __forceinline__ uint32_t dma_lane_off(int ld, int lane, int wid) {
  if constexpr (!TRANS) {
    return 0u;  // (flat DMA: per-lane addresses)
  } else {
    // k = 4 ins + (lane >> 4) with ins = 2 wid + t: k & 3 = lane >> 4 and (k >> 3) & 1 = wid & 1 for both t, so
    // mc_swz(k) = 2 ((lane >> 4) | (wid & 1) << 2)
    const int l4 = lane >> 4;
    const int c = (lane & 15) ^ (2 * (l4 | ((wid & 1) << 2)));
    return (uint32_t)((l4 * ld + half_map<IL, IS_A>(8 * c, 0)) * (int)sizeof(bf16));
  }
}
__device__ __forceinline__ u32x4 buf_desc_n(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  return u32x4{(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a),
               (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32) & 0xffffu),
               (uint32_t)__builtin_amdgcn_readfirstlane(bytes), 0x00020000u};
}
template <bool TRANS, bool IS_A, bool IL, bool BND>
__device__ __forceinline__ void dma_half(const bf16* __restrict__ src, int ld, int base, int h, int k0, int rmax,
                                         char* slot, int wid, int lane, uint32_t loff, int kdim,
                                         bool zero = false) {
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int ins = wid * 2 + t;
    if constexpr (!TRANS) {
      const int ir = 8 * ins + (lane >> 3);
      const int c = (lane & 7) ^ (ir & 7);
      const bf16* g = src + (size_t)min(base + half_map<IL, IS_A>(ir, h), rmax) * ld + k0 + 8 * c;
      if (zero) {  // branch-free select of the zero source (zero is wave-uniform)
        const uintptr_t zm = (uintptr_t)0 - (uintptr_t)zero;
        g = reinterpret_cast<const bf16*>((reinterpret_cast<uintptr_t>(g) & ~zm) |
                                          (reinterpret_cast<uintptr_t>(&g_zero16) & zm));
      }
      lds_dma16(g, slot + ins * 1024);
    } else {
      // bytes from this instruction's base to the operand's last element ((kdim - 1) * ld + rmax + 1; uniform)
      const int row = k0 + 4 * ins, col = base + half_map<IL, IS_A>(0, h);
      const size_t off = (size_t)row * ld + col;
      if constexpr (BND) {
        const size_t rem = 2 * ((size_t)(kdim - 1 - row) * ld + (rmax + 1 - col));
        lds_dma16_buf(buf_desc_n(src + off, zero ? 0u : (uint32_t)min(rem, (size_t)0x7fffffffu)), loff, 0,
                      slot + ins * 1024);
      } else {
        lds_dma16_buf(buf_desc_n(src + off, zero ? 0u : 0x7fffffffu), loff, 0, slot + ins * 1024);
      }
    }
  }
}

// The same half-tile of a k-contiguous operand by BUFFER LDS-DMA (the persistent kernel): the lane part of
// the source offset, row (l >> 3) of an instruction's 8 rows and 16-B chunk (l & 7) ^ (l >> 3), is the same
// for every instruction, half and tile (one VGPR per operand); the row-group / K-tile position is a
// wave-uniform byte offset (soffset). Rows past the operand's end read as zeros (buffer range check).
__device__ __forceinline__ uint32_t kc_lane_off(int ld, int lane) {
  return (uint32_t)(((lane >> 3) * ld + 8 * ((lane & 7) ^ (lane >> 3))) * (int)sizeof(bf16));
}
__device__ __forceinline__ void dma_half_buf(u32x4 rs, int ld, int row0, int k0, uint32_t loff, char* slot, int wid) {
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int ins = wid * 2 + t;
    const int soff = ((row0 + 8 * ins) * ld + k0) * (int)sizeof(bf16);
    lds_dma16_buf(rs, loff, soff, slot + ins * 1024);
  }
}

// fragment reads: lane gets operand[ir0 + (l&15)][32kk + 8(l>>4) + 0..7]
template <bool TRANS>
__device__ __forceinline__ bf16x8 frag(const char* slot, int ir0, int kk, int lane) {
  if constexpr (!TRANS) {
    const int ir = ir0 + (lane & 15), c = 4 * kk + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(slot + ir * 128 + 16 * (c ^ (ir & 7)));
  } else {
    // k-rows k1 = 32kk + 8g + q and k1 + 4 share one swizzle (mc_swz ignores bits 2 and 5 of k), and
    // ir0 is a multiple of 16, so the lane part of the address is one VGPR per 16-row fragment
    // (the kk / hi offsets are immediates): keeps the wgrad (both operands transposed) under 256 VGPRs
    const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
    const int kl = 8 * g + q;
    const int phys = (((ir0 >> 3) + (p >> 1)) ^ mc_swz(kl)) & 15;
    const char* a0 = slot + kl * 256 + 16 * phys + 8 * (p & 1) + kk * (32 * 256);
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a0);
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * 256));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, r);
  }
}

struct Frags {
  bf16x8 a[2][4];   // [kk][row frag] of the current A half
  bf16x8 b[2][2][2];  // [ni][kk][col frag]: B_0 (kept for the whole K-tile) and B_1
};

template <bool A_T>
__device__ __forceinline__ void read_a(Frags& f, const char* slot, int wr, int lane) {  // image rows wr*64..+64
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int i = 0; i < 4; ++i) f.a[kk][i] = frag<A_T>(slot, wr * 64 + 16 * i, kk, lane);
}
template <bool B_T, int NI>
__device__ __forceinline__ void read_b(Frags& f, const char* slot, int wc, int lane) {
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int j = 0; j < 2; ++j) f.b[NI][kk][j] = frag<B_T>(slot, wc * 32 + 16 * j, kk, lane);
}

template <int NI>
__device__ __forceinline__ void mfma_quadrant(f32x4 (&acc)[4][2], const Frags& f) {
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.b[NI][kk][j], f.a[kk][i], acc[i][j], 0, 0, 0);
}

// s_waitcnt vmcnt takes 0..63: a count past that waits for a few more of the oldest operations (safe)
constexpr int vm_cap(int n) { return n > 63 ? 63 : n; }

// end of a phase's memory segment: retire the half-tile the next phase reads, then the ping-pong
// MFMA segment between two barriers
// PP_LGKM_AFTER_BARRIER=0 (A/B builds): no explicit lgkmcnt(0) ahead of the MFMA segment; the compiler's own counted
// waits retire each fragment read before its first MFMA, and every fragment a memory segment reads is consumed by the
// MFMA segment that follows it, so all reads still complete before the barrier that ends that segment
#ifndef PP_LGKM_AFTER_BARRIER
#define PP_LGKM_AFTER_BARRIER 1
#endif
GPT2MI_PRODUCT_KNOB(PP_LGKM_AFTER_BARRIER, 1);
#if PP_LGKM_AFTER_BARRIER
#define PP_LGKM0() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#else
#define PP_LGKM0()
#endif
#define PP_PRIO_HI() __builtin_amdgcn_s_setprio(1);
#define PP_PRIO_LO() __builtin_amdgcn_s_setprio(0);
#define PP_SYNC_MFMA(ACC, NI, VM)                          \
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM) : "memory"); \
  __builtin_amdgcn_sched_barrier(0);                       \
  __builtin_amdgcn_s_barrier();                            \
  PP_LGKM0()                                               \
  __builtin_amdgcn_sched_barrier(0);                       \
  PP_PRIO_HI()                                             \
  mfma_quadrant<NI>(ACC, fr);                              \
  PP_PRIO_LO()                                             \
  __builtin_amdgcn_sched_barrier(0);                       \
  __builtin_amdgcn_s_barrier();                            \
  __builtin_amdgcn_sched_barrier(0);

// the same with the wait chosen at run time: vmcnt(VM + kStores) when FIRST (persistent K-tile 0), else vmcnt(VM)
#define PP_SYNC_MFMA_F(ACC, NI, VM, FIRST)                                             \
  if (FIRST) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(vm_cap((VM) + kStores)) : "memory"); \
  else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VM) : "memory");                       \
  __builtin_amdgcn_sched_barrier(0);                                                  \
  __builtin_amdgcn_s_barrier();                                                       \
  PP_LGKM0()                                                                          \
  __builtin_amdgcn_sched_barrier(0);                                                  \
  PP_PRIO_HI()                                                                        \
  mfma_quadrant<NI>(ACC, fr);                                                         \
  PP_PRIO_LO()                                                                        \
  __builtin_amdgcn_sched_barrier(0);                                                  \
  __builtin_amdgcn_s_barrier();                                                       \
  __builtin_amdgcn_sched_barrier(0);

// workgroup barrier that orders LDS only (the epilogue's global stores stay in flight)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// Timing instrumentation (tools/gemm_timing.py builds a separate library with -DGEMM_PP_TIMING): wave 0
// of every block stamps s_memtime at kernel start (0), first operands landed (1), end of the main loop
// (2) and end of the epilogue (3), plus its HW_ID / XCC_ID, into P.aux (BF16 epilogue only).
#if defined(GEMM_PP_TIMING) && !defined(GPT2MI_AB_BUILD)
#error "GEMM_PP_TIMING writes stamps into P.aux: an A/B build (make timing) only"
#endif
#ifdef GEMM_PP_TIMING
#define PP_STAMP(I)                                                                                  \
  if (EPI == EPI_BF16 && P.aux && threadIdx.x == 0) {                                               \
    uint64_t* ts = reinterpret_cast<uint64_t*>(P.aux) + (size_t)blockIdx.x * 6;                    \
    ts[I] = __builtin_amdgcn_s_memtime();                                                            \
    if (I == 0) {                                                                                    \
      ts[4] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);                                  \
      ts[5] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20);                                 \
    }                                                                                                \
  }
#else
#define PP_STAMP(I)
#endif

// Persistent schedule: the work queue. Items (output tiles) are dealt to the 8 XCD labels (blockIdx % 8) in contiguous
// ranges, as xcd_remap does; the first item of every block is static (blockIdx / 8 within its label), every later one
// is taken from its label's counter (only the label's blocks touch it) by one returning atomic, issued one tile ahead:
// at the end of the previous epilogue (at kernel start for the second item), read back at the end of the main loop
// (whose last waits are vmcnt(0)) and handed to every wave through LDS. One tile ahead keeps a label's in-flight items
// within about one round of 32 consecutive tiles, the static walk's L2 footprint (two ahead spread them over two).
// A block that starts late — its CU held by an RCCL kernel of a data-parallel wrapper, or by any concurrent kernel — so
// takes fewer tiles instead of making the grid end on its last one. Taken (DYN) when the caller says collectives may
// share the CUs (gpt2mi.h GPT2MI_SCHED_SHARED_CUS): alone on the GPU the static walk is 1-3 % faster (the grab's wait
// and LDS hand-off per tile; profiles/r4ab/gemm_dyn.log).
// One slot per launch, rotating over kQueueSlots (at most 4 kernels run at once per process: GPU_MAX_HW_QUEUES); the
// last block out resets its slot to zero for the next launch that takes it.
constexpr int kQueueSlots = 256;
__device__ unsigned g_pp_queue[kQueueSlots][16];  // [slot][XCD label 0..7, 8: blocks out]
// item range of XCD label x over n items (xcd_remap's)
__device__ __forceinline__ void xcd_range(int x, int n, int& base, int& cnt) {
  const int q = n / 8, r = n % 8;
  base = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  cnt = q + (x < r ? 1 : 0);
}

// Output tile of item `pid` (GM M-tiles per group share their B tiles in L2).
#ifndef GPT2MI_PP_GM
#define GPT2MI_PP_GM 4
#endif
GPT2MI_PRODUCT_KNOB(GPT2MI_PP_GM, 4);
__device__ __forceinline__ void tile_of(int pid, int tiles_m, int tiles_n, int& m0, int& n0) {
  constexpr int GM = GPT2MI_PP_GM;
  const int group = pid / (GM * tiles_n);
  const int first_m = group * GM;
  const int gsz = min(tiles_m - first_m, GM);
  m0 = (first_m + (pid % (GM * tiles_n)) % gsz) * BM;
  n0 = ((pid % (GM * tiles_n)) / gsz) * BN;
}

// PERSIST: one block per CU walks the output tiles (item = remap(blockIdx + i * gridDim)); at each tile
// boundary the NEXT tile's first K-tile is staged by LDS-DMA into buffer 0 while this tile's epilogue runs
// through buffer 1 (a 64-row fp32 image, four passes), so the operand latency of a tile start and the
// block launch gap overlap the epilogue instead of following it (the K = 768 shapes spend ~8 us of ~25
// per tile there). Layout-0 shapes without split-K only (host-selected).
// BND: a transposed operand has a partial last tile (M or N not a multiple of 256): its DMA is bounded (dma_half)
// DYN (PERSIST only): tiles from the work queue g_pp_queue (above) instead of the static walk
// GRP: a grouped weight-gradient launch (gpt2mi_gemm_wgrad_grouped): up to kGroupMax problems with the same token count
// and split, each a full-tile (M, N multiples of 256) weight gradient into its own slabs, as ONE launch over the (split,
// problem tile) items, split-major like the single launch (the XCD remap gives each XCD a contiguous item range, so the
// blocks of one split, which read the same token rows of the problems' operands, share an L2). A block finds its problem
// from the tile prefix (wave-uniform, scalar loads of the kernel argument) and runs the single-problem code on it. The
// kernel argument is the problem table then; P below is a reference into it (for GRP = false, to the one problem), so
// the single-problem kernels compile exactly as before (a by-value copy or a device-function parameter made the
// persistent residual kernels spill).
template <bool GRP>
using PPArg = typename std::conditional<GRP, GemmGroup, GemmParams>::type;
template <bool GRP>
__device__ __forceinline__ const GemmParams& pp_problem(const PPArg<GRP>& a, int& item) {
  if constexpr (GRP) {
    const int nsplit = (a.p[0].K + a.p[0].k_per_split - 1) / a.p[0].k_per_split;
    const int it = xcd_remap(blockIdx.x, a.tiles * nsplit);
    const int split = it / a.tiles, t = it - split * a.tiles;
    int g = 0;
#pragma unroll
    for (int k = 1; k < kGroupMax; ++k)
      if (k < a.count && t >= a.prefix[k]) g = k;
    item = split * (a.prefix[g + 1] - a.prefix[g]) + (t - a.prefix[g]);
    return a.p[g];
  } else {
    item = -1;
    return a;
  }
}
template <bool A_T, bool B_T, int EPI, int MAP, bool PERSIST = false, bool BND = false, bool DYN = false,
          bool GRP = false>
__global__ __launch_bounds__(kThreads, 1) void gemm_pp_kernel(PPArg<GRP> KA) {
  PP_STAMP(0)
  int item0;
  const GemmParams& P = pp_problem<GRP>(KA, item0);
  constexpr bool AIL = MAP & 1, BIL = MAP & 2;  // interleaved half-tile maps (A/B experiments)
  static_assert(!PERSIST || MAP == 0, "the persistent epilogue assumes the contiguous half-tile map");
  // phase-4 B reads (see ktile): the persistent schedule and the weight gradients (both operands by buffer DMA); the
  // one-tile-per-block k-contiguous kernels keep the round-2 schedule (their per-lane flat DMA addresses would spill)
  constexpr bool kB0Early = PP_B0_EARLY && (PERSIST || (A_T && B_T));
  __shared__ __attribute__((aligned(1024))) char smem[kLds];
  [[maybe_unused]] __shared__ int s_next;  // PERSIST, DYN: the next tile's item, from the block's grab
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 2, wc = wid & 3;

  // N (and, for the weight gradients, M) may end in a partial tile: a multiple of 64 (GPT-2 1.5B: 1600, 4800)
  const int tiles_m = (P.M + BM - 1) / BM, tiles_n = (P.N + BN - 1) / BN;
  const int ntiles = tiles_m * tiles_n;
  // 1-D grid over (split, tile) items, split-major: the XCD remap gives each XCD a contiguous item range,
  // so the blocks of one K split (which share its A and B token rows) run out of one L2
  const int nsplit = PERSIST ? 1 : (P.K + P.k_per_split - 1) / P.k_per_split;
  int vid = blockIdx.x;  // PERSIST: virtual block id of this tile (blockIdx + i * gridDim, same XCD label)
  const int item = item0 >= 0 ? item0 : xcd_remap(vid, ntiles * nsplit);
  // PERSIST, DYN: the block's XCD label range, the label's block count (its static items) and the item of its NEXT tile
  [[maybe_unused]] int q_base = 0, q_cnt = 0, q_blocks = 0, nxt_item = -1;
  if constexpr (PERSIST && DYN) {
    xcd_range(blockIdx.x % 8, ntiles, q_base, q_cnt);
    q_blocks = (gridDim.x + 7 - blockIdx.x % 8) / 8;
  }
  const int split = item / ntiles;
  int m0, n0;
  tile_of(item - split * ntiles, tiles_m, tiles_n, m0, n0);
  const int kbeg = split * P.k_per_split;
  const int nk = (min(P.K, kbeg + P.k_per_split) - kbeg) / BK;  // even, or odd >= 3 without split-K (host-checked)

  // PERSIST: vector-memory stores each wave issues in an epilogue (one per output row and output array; the
  // column-sum atomic of waves 0-3 only makes the waits below retire more, never less)
  // (bf16 outputs: one 16-B store per lane and row pair, so half as many)
  constexpr bool kWide = !AIL && (EPI == EPI_BF16 || EPI == EPI_GELU || EPI == EPI_GELU_BWD || EPI == EPI_SLAB16);
  constexpr int kStores = (EPI == EPI_GELU ? 64 : 32) / (kWide ? 2 : 1);
  bool after_epi = false;  // the current tile follows an epilogue (wave-uniform)
  f32x4 acc[2][2][4][2];
  auto zero_acc = [&]() {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  zero_acc();

  // An odd K-tile count (K = 1600 / 4800: GPT-2 1.5B; no split-K) runs as nk + 1 tiles whose tile 0 is a ZERO tile
  // (both operands' LDS images zeroed, no DMA): the 4-phase pairs and their counted waits stay as they are (the
  // waits for tile 0's missing DMAs are already satisfied), for one extra K-tile of MFMA work (1/26 at K = 1600).
  const bool odd = !PERSIST && (nk & 1);
  const int nkv = nk + (odd ? 1 : 0);  // virtual K-tile count, even
  const int kbase = kbeg - (odd ? BK : 0);
  auto kofs = [&](int t) { return kbase + t * BK; };
  // PERSIST (k-contiguous A and B): buffer DMA, 2 lane-offset VGPRs for every tile instead of per-tile
  // 64-bit row pointers (the persistent loop keeps its registers under the 256 of 2 waves/SIMD)
  [[maybe_unused]] u32x4 rs_a, rs_b;
  [[maybe_unused]] uint32_t loff_a = 0, loff_b = 0;
  if constexpr (PERSIST) {
    rs_a = buf_desc(P.A);
    rs_b = buf_desc(P.B);
    loff_a = kc_lane_off(P.lda, lane);
    loff_b = kc_lane_off(P.ldb, lane);
  } else {
    loff_a = dma_lane_off<A_T, true, AIL>(P.lda, lane, wid);
    loff_b = dma_lane_off<B_T, false, BIL>(P.ldb, lane, wid);
  }
  auto dma_a_at = [&](int mm0, int t, int h, char* buf) {
    if constexpr (PERSIST)
      dma_half_buf(rs_a, P.lda, mm0 + (h << 7), kofs(t), loff_a, buf + (h ? SA1 : SA0), wid);
    else
      dma_half<A_T, true, AIL, BND>(P.A, P.lda, mm0, h, kofs(t), P.M - 1, buf + (h ? SA1 : SA0), wid, lane, loff_a, P.K);
  };
  auto dma_b_at = [&](int nn0, int t, int h, char* buf) {
    if constexpr (PERSIST)
      dma_half_buf(rs_b, P.ldb, nn0 + (h << 7), kofs(t), loff_b, buf + (h ? SB1 : SB0), wid);
    else
      dma_half<B_T, false, BIL, BND>(P.B, P.ldb, nn0, h, kofs(t), P.N - 1, buf + (h ? SB1 : SB0), wid, lane, loff_b, P.K);
  };
  auto dma_a = [&](int t, int h, char* buf) { dma_a_at(m0, t, h, buf); };
  auto dma_b = [&](int t, int h, char* buf) { dma_b_at(n0, t, h, buf); };
  // tile 0 of the prologue (zero source when odd; the persistent kernel never is)
  auto dma_a0z = [&](int t, int h, char* buf) {
    if constexpr (PERSIST) dma_a_at(m0, t, h, buf);
    else dma_half<A_T, true, AIL, BND>(P.A, P.lda, m0, h, kofs(t), P.M - 1, buf + (h ? SA1 : SA0), wid, lane, loff_a, P.K,
                                   odd);
  };
  auto dma_b0z = [&](int t, int h, char* buf) {
    if constexpr (PERSIST) dma_b_at(n0, t, h, buf);
    else dma_half<B_T, false, BIL, BND>(P.B, P.ldb, n0, h, kofs(t), P.N - 1, buf + (h ? SB1 : SB0), wid, lane, loff_b, P.K,
                                    odd);
  };
  char* buf0 = smem;
  char* buf1 = smem + kBuf;
  // DYN: the queue counter's old value from this block's latest grab (thread 0; written by an asm atomic, so that no
  // compiler-inserted vmcnt(0) drains the DMAs for its return; valid once a wait has retired it: read only at the end of
  // the main loop, after its vmcnt(0) waits). The first grab (for the block's second tile) goes out before the prologue.
  // The compiler cannot see that the return register is written late: tests/test_gemm_grab_hazard.py walks the emitted
  // code of every DYN kernel and checks that no instruction touches that register before a vmcnt(0) retires the atomic.
  // (A compiler-visible __hip_atomic_fetch_add is turned into a wave-reduced atomic followed at once by vmcnt(0),
  // which would drain the epilogue's stores and the next tile's DMAs at every grab.) The labels assume that blocks with
  // equal blockIdx.x % 8 share an XCD: a speed assumption only, each label's counter being private to its blocks.
  [[maybe_unused]] unsigned grab = 0u;
  [[maybe_unused]] auto grab_next = [&]() {
    if (threadIdx.x == 0) {
      unsigned* qa = &g_pp_queue[P.qslot][blockIdx.x % 8];
      asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(grab) : "v"(qa), "v"(1u) : "memory");
    }
  };
  if constexpr (PERSIST && DYN) grab_next();

  // prologue: what phases -6..-1 would have issued (all of tile 0, A_0 / B_0 of tile 1), in order. The zero tile
  // of an odd count: the same DMAs with every lane's source redirected to 16 zero bytes (a select, no branch:
  // a branch here costs the main loop registers)
  dma_a0z(0, 0, buf0);
  dma_b0z(0, 0, buf0);
  dma_b0z(0, 1, buf0);
  dma_a0z(0, 1, buf0);
  if constexpr (kB0Early) {  // phases -2 / -1 of the schedule below issue B_0 then A_0
    dma_b(1, 0, buf1);
    dma_a(1, 0, buf1);
  } else {
    dma_a(1, 0, buf1);
    dma_b(1, 0, buf1);
  }
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // A_0(0), B_0(0) landed
  __builtin_amdgcn_s_barrier();
  PP_STAMP(1)
  if (wr == 1) __builtin_amdgcn_s_barrier();  // group 1 runs one barrier behind group 0
  __builtin_amdgcn_sched_barrier(0);
  for (;;) {  // PERSIST: one iteration per output tile (non-persistent: exactly one)

  Frags fr;
  // kB0Early: B_0 of K-tile 0 into slot 0 ahead of its phase 1 (every later K-tile's B_0 is read in the phase 4 before)
  if constexpr (kB0Early) read_b<B_T, 0>(fr, buf0 + SB0, wc, lane);
  // One K-tile (4 phases): tile tt = t + S, S = 0 / 1 its buffer parity. HN / HN2: tiles tt + 1 / tt + 2 exist. The
  // DMAs for tiles past the end are not issued, and each wait retires what the next phase reads from the real DMAs
  // still outstanding: vmcnt 8,8,8,8 (steady state), 8,8,6,4 (the second-to-last tile), 2,0,0,0 (the last): no
  // re-load traffic, and nothing left in flight for the epilogue to wait for. The counts depend only on (HN, HN2), so
  // an odd number of K-tiles ends ..., (T,T) at parity 0, (T,F) at parity 1, (F,F) at parity 0 (K = 1600 / 4800:
  // GPT-2 1.5B).
  //
  // FIRST (persistent schedule, K-tile 0 of a tile after an epilogue): the waits of phases 1-2 retire half-tiles
  // issued BEFORE the previous tile's epilogue stores. vmcnt counts loads, stores and LDS-DMA together in issue
  // order and waits for all but the N youngest, so those waits count the epilogue's kStores stores among the
  // younger operations instead of draining them: the stores get two more phases to complete in the background.
  auto ktile = [&](int t, auto s_c, auto hn_c, auto hn2_c) {
    constexpr int S = decltype(s_c)::value;
    constexpr bool HN = decltype(hn_c)::value;    // tile tt + 1 exists
    constexpr bool HN2 = decltype(hn2_c)::value;  // tile tt + 2 exists
    // PERSIST, K-tile 0 (t == 0, S == 0) of a tile that follows an epilogue: phases 1-2 wait with the epilogue's
    // stores counted as younger (a wave-uniform branch around the wait alone; nk >= 4 and even, host-checked, so
    // K-tile 0 is always a steady-state tile)
    const bool first = PERSIST && S == 0 && HN2 && t == 0 && after_epi;
    char* cur = S ? buf1 : buf0;
    char* nxt = S ? buf0 : buf1;
    const int tt = t + S;
    if constexpr (kB0Early) {
      // B register slots alternate by parity: B_0 of K-tile tt in slot S, its B_1 in slot 1 - S. Phase 4 reads the NEXT
      // K-tile's B_0 into slot 1 - S (free once phase 3's MFMAs have read B_1), so no phase reads both operands
      // fresh: fragment reads per phase 16 / 8 / 16 / 8 for two transposed operands (was 24 / 8 / 16 / 0). The DMAs of
      // phases 3 / 4 swap (B_0, then A_0 of tile tt + 2) so that phase 3's wait retires B_0 of tt + 1 for phase 4 and
      // phase 4's wait A_0 of tt + 1 for the next phase 1; the counts are unchanged. WAR: B_0 of tt + 1 is read in
      // phase 4 and restaged in phase 3 of tt + 1; A_0 of tt is read in phase 1 and restaged in phase 4.
      // phase 1: quadrant (0,0)
      read_a<A_T>(fr, cur + SA0, wr, lane);
      if constexpr (HN) dma_b(tt + 1, 1, nxt);
      PP_SYNC_MFMA_F(acc[0][0], S, HN ? 8 : 2, first)
      // phase 2: quadrant (0,1)
      read_b<B_T, 1 - S>(fr, cur + SB1, wc, lane);
      if constexpr (HN) dma_a(tt + 1, 1, nxt);
      PP_SYNC_MFMA_F(acc[0][1], 1 - S, HN ? 8 : 0, first)
      // phase 3: quadrant (1,1)
      read_a<A_T>(fr, cur + SA1, wr, lane);
      if constexpr (HN2) dma_b(tt + 2, 0, cur);
      PP_SYNC_MFMA(acc[1][1], 1 - S, HN2 ? 8 : (HN ? 6 : 0))
      // phase 4: quadrant (1,0); B_0 of tt + 1
      if constexpr (HN) read_b<B_T, 1 - S>(fr, nxt + SB0, wc, lane);
      if constexpr (HN2) dma_a(tt + 2, 0, cur);
      PP_SYNC_MFMA(acc[1][0], S, HN2 ? 8 : (HN ? 4 : 0))
    } else {
    // phase 1: quadrant (0,0)
    read_a<A_T>(fr, cur + SA0, wr, lane);
    read_b<B_T, 0>(fr, cur + SB0, wc, lane);
    if constexpr (HN) dma_b(tt + 1, 1, nxt);
    PP_SYNC_MFMA_F(acc[0][0], 0, HN ? 8 : 2, first)
    // phase 2: quadrant (0,1)
    read_b<B_T, 1>(fr, cur + SB1, wc, lane);
    if constexpr (HN) dma_a(tt + 1, 1, nxt);
    PP_SYNC_MFMA_F(acc[0][1], 1, HN ? 8 : 0, first)
    // phase 3: quadrant (1,1)
    read_a<A_T>(fr, cur + SA1, wr, lane);
    if constexpr (HN2) dma_a(tt + 2, 0, cur);
    PP_SYNC_MFMA(acc[1][1], 1, HN2 ? 8 : (HN ? 6 : 0))
    // phase 4: quadrant (1,0) from registers
    if constexpr (HN2) dma_b(tt + 2, 0, cur);
    PP_SYNC_MFMA(acc[1][0], 0, HN2 ? 8 : (HN ? 4 : 0))
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using F = std::false_type;
  using Tr = std::true_type;
  for (int t = 0; t < nkv - 2; t += 2) {
    ktile(t, I0{}, Tr{}, Tr{});
    ktile(t, I1{}, Tr{}, Tr{});
  }
  ktile(nkv - 2, I0{}, Tr{}, F{});
  ktile(nkv - 2, I1{}, F{}, F{});
  if constexpr (PERSIST && DYN) {
    // the item of the tile after this one, from the latest grab: the last K-tile's waits were vmcnt(0), so the atomic
    // has returned (the empty asm keeps the read of `grab` below them)
    asm volatile("" : "+v"(grab));
    if (threadIdx.x == 0) {
      const int idx = (int)grab + q_blocks;
      s_next = idx < q_cnt ? q_base + idx : -1;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();  // re-align the groups (same barrier count)
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (PERSIST && DYN) {
    asm volatile("" ::: "memory");
    nxt_item = __builtin_amdgcn_readfirstlane(s_next);
  }
  PP_STAMP(2)

  // the thread index through an opaque copy: lane constants derived from it are formed here, per tile, instead of
  // being hoisted to kernel entry and spilled across the tile loop (whose reloads would wait vmcnt(0) behind the
  // next tile's DMAs)
  int tid = threadIdx.x;
  if constexpr (PERSIST) {  // wave id (SGPR) * 64 + the lane id recomputed by v_mbcnt (no VGPR kept live for it)
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    tid = wid * 64 + l;
  }
  const int ch = tid & 63;
  const int gn = n0 + 4 * ch;
  // bf16 outputs (kWide): lane (half hl, column group cj) owns columns 8cj..8cj+7 of the even / odd row of a pair
  // (one 16-B store per row pair and output array); otherwise columns 4ch..4ch+3 of one row
  const int cj = tid & 31, hl = (tid >> 5) & 1;
  const int gnb = kWide ? n0 + 8 * cj : gn;  // first bias column of the lane
  // lanes whose columns lie past N (a partial last column tile; N % 64 == 0, so a lane's 4 / 8 columns are all in or
  // all out) load no operands and store nothing
  const bool col_ok = PERSIST || gnb < P.N;  // (the persistent schedule runs full column tiles only)
  // the persistent BF16 epilogue adds its bias in the accumulator layout (bacc below)
  constexpr bool kBf16Acc = EPI == EPI_BF16 && PERSIST;
  const bool has_bias = P.bias && EPI != EPI_GELU_BWD && col_ok && !kBf16Acc;
  const f32x4 bias = has_bias ? *reinterpret_cast<const f32x4*>(P.bias + gnb) : f32x4{0.f, 0.f, 0.f, 0.f};
  [[maybe_unused]] f32x4 bias1 = {0.f, 0.f, 0.f, 0.f};
  if constexpr (kWide) {
    if (has_bias) bias1 = *reinterpret_cast<const f32x4*>(P.bias + gnb + 4);
  }
  // PERSIST: the next tile's K-tile 0 goes into buffer 0 now (last read in this tile's final even K-tile,
  // several barriers ago); the epilogue image lives in buffer 1. The bias is waited for first: hipcc waits
  // vmcnt(0) at the first use of an ordinary load while an LDS-DMA is in flight, which would drain the
  // next tile's DMAs inside the epilogue (the persistent path is only selected for epilogues without
  // other operand loads: BF16, GELU).
  // kBf16Acc: the bias of the lane's accumulator columns n0 + ni*128 + wc*32 + 16j + 4(l >> 4) + 0..3
  [[maybe_unused]] f32x4 bacc[2][2];
  if constexpr (kBf16Acc) {
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        bacc[ni][j] = P.bias ? *reinterpret_cast<const f32x4*>(P.bias + n0 + ni * 128 + wc * 32 + 16 * j + 4 * (lane >> 4))
                             : f32x4{0.f, 0.f, 0.f, 0.f};
        asm volatile("" ::"v"(bacc[ni][j][0]), "v"(bacc[ni][j][1]), "v"(bacc[ni][j][2]), "v"(bacc[ni][j][3]));
      }
  }
  int next_m0 = 0, next_n0 = 0;
  bool has_next = false;
  if constexpr (PERSIST) {
    asm volatile("" ::"v"(bias[0]), "v"(bias[1]), "v"(bias[2]), "v"(bias[3]));
    if constexpr (kWide) asm volatile("" ::"v"(bias1[0]), "v"(bias1[1]), "v"(bias1[2]), "v"(bias1[3]));
    int next_item;
    if constexpr (DYN) {
      next_item = nxt_item;
    } else {
      vid += gridDim.x;
      next_item = vid < ntiles ? xcd_remap(vid, ntiles) : -1;
    }
    has_next = next_item >= 0;
    if (has_next) {
      tile_of(next_item, tiles_m, tiles_n, next_m0, next_n0);
      dma_a_at(next_m0, 0, 0, buf0);
      dma_b_at(next_n0, 0, 0, buf0);
      dma_b_at(next_n0, 0, 1, buf0);
      dma_a_at(next_m0, 0, 1, buf0);
    }
  }

  // ---- epilogue: acc[mi][ni][i][j][r] = C[m0 + mi*128 + wr*64 + 16i + (l&15)][n0 + ni*128 + wc*32 + 16j + 4(l>>4) + r]
  float alpha = P.alpha;
  if (P.alpha_dev) alpha *= P.alpha_dev[0];
  // [128][256] fp32 image (1 KiB rows) over the whole LDS; PERSIST: [64][256] in buffer 1
  float* img = reinterpret_cast<float*>(PERSIST ? buf1 : smem);
  // accumulators of pass mi (tile rows mi*128 + rbase + 16i + (l & 15)) into image rows rbase + 16i + (l & 15); the
  // alpha multiply only when alpha != 1 (one VALU per output element otherwise spent on every GEMM's epilogue)
  auto write_image = [&](int mi, int rbase) {
    auto body = [&](auto sc) {
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int r = rbase + 16 * i + (lane & 15);
            const int c = BIL ? wc * 16 + ni * 8 + 4 * j + (lane >> 4) : ni * 32 + wc * 8 + 4 * j + (lane >> 4);
            f32x4 v = acc[mi][ni][i][j];
            if constexpr (decltype(sc)::value) {
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] *= alpha;
            }
            *reinterpret_cast<f32x4*>(img + r * 256 + 4 * (c ^ (r & 15))) = v;
          }
    };
    if (alpha != 1.f) body(std::true_type{});
    else body(std::false_type{});
  };
  constexpr bool kOpnd = EPI == EPI_RESID || EPI == EPI_GELU_BWD || EPI == EPI_F32;
  // fused bias grad of the stored output (column sums of the rounded stores; reduced per tile below; the
  // persistent schedule has the registers for it only beside the GELU_BWD epilogue, the one that uses it)
  constexpr bool kCsum = PERSIST ? EPI == EPI_GELU_BWD : (EPI == EPI_BF16 || EPI == EPI_GELU_BWD);
  const bool csum_on = kCsum && P.dbias != nullptr;
  f32x4 csum;
  [[maybe_unused]] f32x4 csum1;
  if constexpr (PERSIST) {  // formed per tile (a zero vector hoisted out of the tile loop got spilled)
    float z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    csum = f32x4{z, z, z, z};
    csum1 = csum;
  } else {
    csum = f32x4{0.f, 0.f, 0.f, 0.f};
    csum1 = csum;
  }
  if constexpr (GEMM_STORE_EXP == 3 && PERSIST) {
    // A/B build only: no epilogue at all (the accumulators kept live): the main loop's share of a tile
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(acc[a][b][i][j]));
  } else if constexpr (kBf16Acc) {
    // BF16 output: alpha and the bias applied in the accumulator layout, the tile rounded to bf16 into a [128][256]
    // bf16 image (64 KiB: all of buffer 1, so two 128-row passes of every wave instead of four 64-row fp32 passes; half
    // the LDS bytes). 8-B chunk c of image row r at c ^ 2(r & 15): conflict-free for the 16-row x 8-B writes and the
    // 16-B row reads. Then 16 rows per block-wide step: lane (row tid >> 5, 16-B unit tid & 31) loads 8 columns and
    // stores them with one 16-B store (full 512-B rows per 32 lanes). Bitwise the stores of the fp32-image path.
    char* img16 = buf1;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      if (mi) lds_barrier();  // pass 0's reads are done before pass 1 overwrites the image
      auto put = [&](auto sc) {
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const int r = wr * 64 + 16 * i + (lane & 15);
              const int c = ni * 32 + wc * 8 + 4 * j + (lane >> 4);
              f32x4 v = acc[mi][ni][i][j];
              if constexpr (decltype(sc)::value) v *= alpha;
              v += bacc[ni][j];
              const bf16x4 b = {f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
              *reinterpret_cast<bf16x4*>(img16 + r * 512 + 8 * (c ^ (2 * (r & 15)))) = b;
            }
      };
      if (alpha != 1.f) put(std::true_type{});
      else put(std::false_type{});
      lds_barrier();
      const int cu = tid & 31;
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int r = 16 * it + (tid >> 5);
        const u32x4 v = *reinterpret_cast<const u32x4*>(img16 + r * 512 + 8 * ((2 * cu) ^ (2 * (r & 15))));
        bf16* C = reinterpret_cast<bf16*>(P.C) + out_idx(m0 + mi * 128 + r, P.ldc, n0 + 8 * cu);
        if constexpr (GEMM_STORE_EXP == 1) asm volatile("" ::"v"(v));
        else __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(C));
      }
    }
  } else if constexpr (kWide && PERSIST) {
    // four 64-row passes as below; wave wid, half hl reads rows 16it + 2wid + hl (it = 0..3) of the pass's image,
    // columns 8cj..8cj+7 (two 16-B chunks), and stores each output row pair with one 16-B store per lane
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int mi = q >> 1, g = q & 1;
      [[maybe_unused]] bf16x8 op8[4];
      if constexpr (EPI == EPI_GELU_BWD) {
#pragma unroll
        for (int it = 0; it < 4; ++it)
          op8[it] = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const bf16*>(P.aux) +
                                                     (size_t)(m0 + q * 64 + 16 * it + 2 * wid + hl) * P.ldaux + gnb);
      }
      if (q) lds_barrier();  // the previous pass's reads are done before this pass overwrites the image
      if (wr == g) {
write_image(mi, 0);
      }
      lds_barrier();
      f32x4 va[4], vb[4];
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int r = 16 * it + 2 * wid + hl;
        va[it] = *reinterpret_cast<const f32x4*>(img + r * 256 + 4 * ((2 * cj) ^ (r & 15)));
        vb[it] = *reinterpret_cast<const f32x4*>(img + r * 256 + 4 * ((2 * cj + 1) ^ (r & 15)));
      }
      auto rows = [&](auto vc) {
        constexpr int VC = decltype(vc)::value;
#pragma unroll
        for (int it = 0; it < 4; ++it) {
          const int gm = m0 + q * 64 + 16 * it + 2 * wid + hl;
          f32x4 w0 = va[it], w1 = vb[it];
          w0 += bias;  // vector adds: packed without SLP
          w1 += bias1;
          f32x4 r0, r1;
          bf16x8 op = {};
          if constexpr (EPI == EPI_GELU_BWD) op = op8[it];
          epilogue8<EPI, EPI == EPI_GELU ? VC : 0>(P, gm, gnb, w0, w1, op, r0, r1);
          if constexpr (kCsum && VC == 1) {  // vector adds: packed (v_pk_add_f32) without SLP, see the Makefile
            csum += r0;
            csum1 += r1;
          }
        }
      };
      const bool on = EPI == EPI_GELU ? P.thr != 0u : csum_on;
      if (on) rows(std::integral_constant<int, 1>{});
      else rows(std::integral_constant<int, 0>{});
    }
  } else if constexpr (PERSIST) {
    // four 64-row passes: pass q = 2*mi + g holds rows q*64.. (the 16-row groups of waves with wr == g)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int mi = q >> 1, g = q & 1;
      // the pass's epilogue operands, in flight while the accumulators go through LDS (the bf16 GELU derivative
      // held as loaded: 2 VGPRs a row instead of 4)
      [[maybe_unused]] f32x4 opnd[8];
      [[maybe_unused]] bf16x4 opnd16[8];
      if constexpr (EPI == EPI_GELU_BWD) {
#pragma unroll
        for (int it = 0; it < 8; ++it)
          opnd16[it] = *reinterpret_cast<const bf16x4*>(reinterpret_cast<const bf16*>(P.aux) +
                                                        (size_t)(m0 + q * 64 + it * 8 + wid) * P.ldaux + gn);
      } else if constexpr (kOpnd) {
#pragma unroll
        for (int it = 0; it < 8; ++it) opnd[it] = epilogue_operand<EPI>(P, min(m0 + q * 64 + it * 8 + wid, P.M - 1), gn);
      }
      if (q) lds_barrier();  // the previous pass's reads are done before this pass overwrites the image
      if (wr == g) {
write_image(mi, 0);
      }
      lds_barrier();
      f32x4 v[8];
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int r = it * 8 + wid;
        v[it] = *reinterpret_cast<const f32x4*>(img + r * 256 + 4 * (ch ^ (r & 15)));
      }
      // every row exists (M % 256 == 0, host-checked); the per-tile switch (dropout for RESID / GELU, the fused
      // column sums for BF16 / GELU_BWD) is decided once per pass: straight-line rows
      auto rows = [&](auto vc) {
        constexpr int VC = decltype(vc)::value;
#pragma unroll
        for (int it = 0; it < 8; ++it) {
          const int gm = m0 + q * 64 + it * 8 + wid;
          f32x4 w = v[it];
          w += bias;
          f32x4 op = {0.f, 0.f, 0.f, 0.f};
          if constexpr (EPI == EPI_GELU_BWD) op = f32x4{bf2f(opnd16[it][0]), bf2f(opnd16[it][1]), bf2f(opnd16[it][2]),
                                                         bf2f(opnd16[it][3])};
          else if constexpr (kOpnd) op = opnd[it];
          const f32x4 o = epilogue_apply<EPI, bf16, (EPI == EPI_RESID || EPI == EPI_GELU) ? VC : 0>(P, gm, gn, w, op);
          if constexpr (kCsum && VC == 1) csum += o;
        }
      };
      const bool on = (EPI == EPI_RESID || EPI == EPI_GELU) ? P.thr != 0u : csum_on;
      if (on) rows(std::integral_constant<int, 1>{});
      else rows(std::integral_constant<int, 0>{});
    }
  } else if constexpr (kWide) {
    // one-tile-per-block, bf16 outputs: two 128-row passes; wave wid, half hl takes rows 16it + 2wid + hl
    // (it = 0..7) of the pass, columns 8cj..8cj+7, one 16-B store per row pair and output array
    const bool full = m0 + BM <= P.M && n0 + BN <= P.N;  // block-uniform
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      [[maybe_unused]] bf16x8 op8[8];
      if constexpr (EPI == EPI_GELU_BWD) {
#pragma unroll
        for (int it = 0; it < 8; ++it)
          op8[it] = *reinterpret_cast<const bf16x8*>(
              reinterpret_cast<const bf16*>(P.aux) +
              (size_t)min(m0 + mi * 128 + 16 * it + 2 * wid + hl, P.M - 1) * P.ldaux + min(gnb, P.N - 8));
      }
      if (mi) lds_barrier();  // pass 0's reads are done before pass 1 overwrites the image
write_image(mi, wr * 64);
      lds_barrier();
      // VC: the per-tile switch (dropout for GELU, the fused column sums for BF16 / GELU_BWD); GUARD: partial
      // tile. Two halves of 4 row pairs (their 16 image reads in flight together; 32 VGPRs live, not 64)
      auto rows = [&](auto vc, auto guard_c) {
        constexpr int VC = decltype(vc)::value;
        constexpr bool GUARD = decltype(guard_c)::value;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
        f32x4 va[4], vb[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int r = 16 * (4 * half + k) + 2 * wid + hl;
          va[k] = *reinterpret_cast<const f32x4*>(img + r * 256 + 4 * ((2 * cj) ^ (r & 15)));
          vb[k] = *reinterpret_cast<const f32x4*>(img + r * 256 + 4 * ((2 * cj + 1) ^ (r & 15)));
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int it = 4 * half + k;
          const int gm = m0 + mi * 128 + 16 * it + 2 * wid + hl;
          if (GUARD && (gm >= P.M || !col_ok)) continue;
          f32x4 w0 = va[k], w1 = vb[k];
          w0 += bias;  // vector adds: packed without SLP
          w1 += bias1;
          if constexpr (EPI == EPI_SLAB16) {  // the split's bf16 slab: one 16-B store per lane and row
            bf16* slab = reinterpret_cast<bf16*>(P.C) + (size_t)split * P.M * P.ldc;
            store8_bf16(slab + (size_t)gm * P.ldc + gnb, w0, w1);

          } else {
            f32x4 r0, r1;
            bf16x8 op = {};
            if constexpr (EPI == EPI_GELU_BWD) op = op8[it];
            epilogue8<EPI, EPI == EPI_GELU ? VC : 0>(P, gm, gnb, w0, w1, op, r0, r1);
            if constexpr (kCsum && VC == 1) {  // vector adds: packed (v_pk_add_f32) without SLP, see the Makefile
              csum += r0;
              csum1 += r1;
            }
          }
        }
        }
      };
      const bool on = EPI == EPI_GELU ? P.thr != 0u : csum_on;
      if (full) {
        if (on) rows(std::integral_constant<int, 1>{}, std::false_type{});
        else rows(std::integral_constant<int, 0>{}, std::false_type{});
      } else {
        if (on) rows(std::integral_constant<int, 1>{}, std::true_type{});
        else rows(std::integral_constant<int, 0>{}, std::true_type{});
      }
    }
  } else {
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    // the pass's epilogue operands (residual / pre-activation / old C): all 16 loads in flight
    // while the accumulators go through LDS
    f32x4 opnd[16];
    if constexpr (kOpnd) {
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const int r = it * 8 + wid;
        const int gm = m0 + (AIL ? ((r >> 6) << 7) + mi * 64 + (r & 63) : mi * 128 + r);
        opnd[it] = epilogue_operand<EPI>(P, min(gm, P.M - 1), min(gn, P.N - 4));
      }
    }
    if (mi) lds_barrier();  // pass 0's reads are done before pass 1 overwrites the image
write_image(mi, wr * 64);
    lds_barrier();
    auto row_of = [&](int it) {
      const int r = it * 8 + wid;
      return m0 + (AIL ? ((r >> 6) << 7) + mi * 64 + (r & 63) : mi * 128 + r);
    };
    // VC: the per-tile switch known at compile time in the full-tile path — dropout for RESID / GELU, the fused
    // column sums for BF16 / GELU_BWD (-1: tested per row)
    auto finish = [&](int it, f32x4 v, auto vc) {
      constexpr int VC = decltype(vc)::value;
      const int gm = row_of(it);
      v += bias;
      if constexpr (EPI == EPI_SLAB) {
        float* slab = reinterpret_cast<float*>(P.C) + (size_t)split * P.M * P.ldc;
        // default-policy stores, not the non-temporal ones of the other epilogues: the split-K reduction reads the
        // slabs right after this launch (same-process A/B, same bits: qkv / proj / fc2 wgrad + reduction 1-3.5 %
        // faster, fc1 within noise; profiles/r4fin/slab_store_ab.log)
        if constexpr (GEMM_STORE_EXP == 1) asm volatile("" ::"v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));
        else *reinterpret_cast<f32x4*>(slab + (size_t)gm * P.ldc + gn) = v;
      } else if constexpr (EPI == EPI_SLAB16) {  // 8 B per lane: one 512-B bf16 row per wave-instruction
        bf16* slab = reinterpret_cast<bf16*>(P.C) + (size_t)split * P.M * P.ldc;
        store4<bf16>(slab + (size_t)gm * P.ldc + gn, v);
      } else {
        constexpr int DROPM = (EPI == EPI_RESID || EPI == EPI_GELU) ? VC : -1;
        const f32x4 o = epilogue_apply<EPI, bf16, DROPM>(P, gm, gn, v, kOpnd ? opnd[it] : f32x4{0.f, 0.f, 0.f, 0.f});
        if constexpr (kCsum) {
          if (VC < 0 ? csum_on : VC == 1) csum += o;
        }
      }
    };
    if (m0 + BM <= P.M && n0 + BN <= P.N) {  // full tile (block-uniform): straight-line reads, then the stores
      f32x4 v[16];
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const int r = it * 8 + wid;
        v[it] = *reinterpret_cast<const f32x4*>(img + r * 256 + 4 * (ch ^ (r & 15)));
      }
      auto rows = [&](auto vc) {
#pragma unroll
        for (int it = 0; it < 16; ++it) finish(it, v[it], vc);
      };
      const bool on = (EPI == EPI_RESID || EPI == EPI_GELU) ? P.thr != 0u : csum_on;
      if (on) rows(std::integral_constant<int, 1>{});
      else rows(std::integral_constant<int, 0>{});
    } else {
      for (int it = 0; it < 16; ++it) {
        const int r = it * 8 + wid;
        const f32x4 v = *reinterpret_cast<const f32x4*>(img + r * 256 + 4 * (ch ^ (r & 15)));
        if (row_of(it) < P.M && col_ok) finish(it, v, std::integral_constant<int, -1>{});
      }
    }
  }
  }  // non-persistent epilogue
  if constexpr (kCsum) {
    if (csum_on) {  // the 8 waves hold partial sums of the same 256 columns: reduce in LDS, 1 atomic/column
      lds_barrier();  // every wave has finished reading the staging image
      if constexpr (kWide) {  // lanes l and l ^ 32 hold the same 8 columns (even / odd rows)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          csum[e] += __shfl_xor(csum[e], 32);
          csum1[e] += __shfl_xor(csum1[e], 32);
        }
        if (hl == 0) {
          *reinterpret_cast<f32x4*>(img + wid * 256 + 8 * cj) = csum;
          *reinterpret_cast<f32x4*>(img + wid * 256 + 8 * cj + 4) = csum1;
        }
      } else {
        *reinterpret_cast<f32x4*>(img + (tid >> 6) * 256 + 4 * ch) = csum;
      }
      lds_barrier();
      if (tid < 256 && n0 + tid < P.N) {
        float t = 0.f;
#pragma unroll
        for (int w8 = 0; w8 < 8; ++w8) t += img[w8 * 256 + tid];
        atomicAdd(P.dbias + n0 + tid, t);
      }
    }
  }
  PP_STAMP(3)
  if constexpr (!PERSIST) {
    return;
  } else {
    if (!has_next) {
      if constexpr (DYN) {
        // the last block out (every block's grabs are done before it counts itself out) resets the slot
        if (threadIdx.x == 0) {
          unsigned* q = g_pp_queue[P.qslot];
          if (__hip_atomic_fetch_add(q + 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1)
            for (int x = 0; x < 9; ++x) __hip_atomic_exchange(q + x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      return;
    }
    // DYN: the item of the tile after next (younger than this epilogue's stores, so the FIRST waits below never wait for
    // it; the steady-state waits of the next main loop retire it behind 8 DMAs)
    if constexpr (DYN) grab_next();
    // the next tile's prologue continues: A_0 / B_0 of its K-tile 1 into buffer 1 once every wave is done
    // with the image there, then the same counted wait as the first prologue (epilogue stores issued in
    // between only make it wait longer, never too little: outstanding <= 8 leaves >= 4 DMAs retired)
    lds_barrier();
    m0 = next_m0;
    n0 = next_n0;
    zero_acc();
    if constexpr (kB0Early) {
      dma_b(1, 0, buf1);
      dma_a(1, 0, buf1);
    } else {
      dma_a(1, 0, buf1);
      dma_b(1, 0, buf1);
    }
    // K-tile 0's A_0 / B_0 landed; its B_1 / A_1, the epilogue's kStores stores and K-tile 1's A_0 / B_0 are the
    // younger operations that may stay in flight (see FIRST above)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(vm_cap(8 + kStores)) : "memory");
    __builtin_amdgcn_s_barrier();
    if (wr == 1) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    after_epi = true;
  }
  }  // tile loop
}


// Default half-tile maps: interleaved for m-contiguous (transposed) operands, contiguous otherwise
// (measured, tools/gemm_probe.py: 8192^3 dgrad 1195 vs 1022 TF with B interleaved; no effect on the
// k-contiguous forward operands).
template <bool A_T, bool B_T, int EPI, int MAP = (A_T ? 1 : 0) | (B_T ? 2 : 0)>
int launch(const GemmParams& P, hipStream_t s, int splits) {
  dim3 grid(((P.M + BM - 1) / BM) * ((P.N + BN - 1) / BN) * splits);
  if constexpr (A_T || B_T) {  // a transposed operand with a partial last tile: the bounded DMA
    if ((A_T && P.M % BM != 0) || (B_T && P.N % BN != 0)) {
      gemm_pp_kernel<A_T, B_T, EPI, MAP, false, true><<<grid, kThreads, 0, s>>>(P);
      return gpt2mi::check_launch("gemm_pp");
    }
  }
  gemm_pp_kernel<A_T, B_T, EPI, MAP><<<grid, kThreads, 0, s>>>(P);
  return gpt2mi::check_launch("gemm_pp");
}

}  // namespace
namespace gpt2mi {
int gemm_pp_grouped(const GemmGroup& G, hipStream_t s) {
  const int nsplit = (G.p[0].K + G.p[0].k_per_split - 1) / G.p[0].k_per_split;
  gemm_pp_kernel<true, true, EPI_SLAB, 3, false, false, false, true><<<dim3(G.tiles * nsplit), kThreads, 0, s>>>(G);
  return gpt2mi::check_launch("gemm_pp_grouped");
}
}  // namespace gpt2mi
namespace {

int num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || n <= 0)
      n = 256;
    n = n / 8 * 8;  // a multiple of the 8 XCDs keeps every block's virtual ids on one XCD label
  }
  return n;
}

// persistent variant: one block per CU, grid a multiple of 8
#ifndef GPT2MI_PERSIST_GRID
#define GPT2MI_PERSIST_GRID 0  // A/B builds: a fixed persistent grid (a CU-masked stream's CU count), 0 = every CU
#endif
GPT2MI_PRODUCT_KNOB(GPT2MI_PERSIST_GRID, 0);
template <int EPI>
int launch_persistent(const GemmParams& Pin, hipStream_t s, bool dyn) {
  static std::atomic<unsigned> next_slot{0};
  GemmParams P = Pin;
  P.qslot = (int)(next_slot.fetch_add(1u, std::memory_order_relaxed) % kQueueSlots);
  const int ntiles = ((P.M + BM - 1) / BM) * (P.N / BN);  // N % 256 == 0 (gemm_pp_dispatch)
  dim3 grid(min(ntiles, GPT2MI_PERSIST_GRID > 0 ? GPT2MI_PERSIST_GRID : num_cus()));
  if (dyn) gemm_pp_kernel<false, false, EPI, 0, true, false, true><<<grid, kThreads, 0, s>>>(P);
  else gemm_pp_kernel<false, false, EPI, 0, true><<<grid, kThreads, 0, s>>>(P);
  return gpt2mi::check_launch("gemm_pp_persistent");
}

}  // namespace

namespace gpt2mi {
#ifndef GPT2MI_PERSIST_KMAX
#define GPT2MI_PERSIST_KMAX 4096
#endif
GPT2MI_PRODUCT_KNOB(GPT2MI_PERSIST_KMAX, 4096);
// longest K that takes the persistent schedule by default: the step's K = 768 / 2304 / 3072 shapes (qkv / fc1 dgrad
// and fc2 + residual 2-3 % faster than one tile per block since the persistent kernel reads the next K-tile's B
// fragments in phase 4, tools/gemm_ab.py 0 7); the lm_head dgrad (K = 50 432) stays one tile per block
constexpr int g_persist_kmax = GPT2MI_PERSIST_KMAX;
// Layouts 0 / 1; N % 256 == 0, every split's K range an even number (>= 2) of 64-deep tiles.
// Returns -1 when this kernel does not apply (the caller falls back).
// bf16-slab weight gradients: half-tile map 2 (A contiguous, B interleaved) so that the epilogue takes the wide path
// (8 columns per lane, one 16-B store per row); map 3 (both interleaved, the fp32-slab kernel's) stores 8 B per lane
#ifndef PP_WGRAD16_MAP
#define PP_WGRAD16_MAP 2
#endif
GPT2MI_PRODUCT_KNOB(PP_WGRAD16_MAP, 2);
int gemm_pp_dispatch(int layout, int epilogue, const GemmParams& P, hipStream_t s, int splits, int map,
                     bool persistent_ok, bool shared_cus) {
  // N (and M) multiples of 64; without split-K any K-tile count >= 2 (an odd count ends in a single K-tile); with
  // split-K an even count per split
  if (P.N % 64 != 0 || P.M % 64 != 0 || P.K % BK != 0 || P.K < 2 * BK) return -1;
  if (splits > 1 && (P.k_per_split % (2 * BK) != 0 || P.K % (2 * BK) != 0)) return -1;
  if (splits == 1 && P.k_per_split != P.K) return -1;
  // wgrad (both operands m-contiguous): this kernel since the LDS-DMA went to inline asm (lm_head wgrad 4046 vs
  // 4485 us on the 2-stage gemm256 kernel, qkv 197 vs 230; before, hipcc's vmcnt(0) drains made it the slower
  // one, 698-721 vs 765 TF). map 8 = the same (tools/lib_ab.py impl 8)
  if (layout == 2) {
    if (map != 0 && map != 8) return -1;
    return epilogue == EPI_SLAB     ? launch<true, true, EPI_SLAB>(P, s, splits)
           : epilogue == EPI_SLAB16 ? launch<true, true, EPI_SLAB16, PP_WGRAD16_MAP>(P, s, splits)
           : epilogue == EPI_F32    ? launch<true, true, EPI_F32>(P, s, 1)
                                    : -1;
  }
  // layout 1 split-K slabs: the weight gradient with its X operand transposed (gpt2mi_gemm_wgrad_kt)
  if (layout == 1 && (epilogue == EPI_SLAB || epilogue == EPI_SLAB16)) {
    if (P.N % BN != 0) return -1;
    return epilogue == EPI_SLAB ? launch<false, true, EPI_SLAB>(P, s, splits) : launch<false, true, EPI_SLAB16>(P, s, splits);
  }
  if (map > 0 && epilogue == EPI_BF16 && layout <= 1 && P.N % BN == 0) {  // half-tile maps (tools/gemm_probe.py)
    if (layout == 0) {
      if (map == 1) return launch<false, false, EPI_BF16, 1>(P, s, 1);
      if (map == 2) return launch<false, false, EPI_BF16, 2>(P, s, 1);
      if (map == 3) return launch<false, false, EPI_BF16, 3>(P, s, 1);
    } else {
      if (map == 1) return launch<false, true, EPI_BF16, 1>(P, s, 1);
      if (map == 2) return launch<false, true, EPI_BF16, 2>(P, s, 1);
      if (map == 3) return launch<false, true, EPI_BF16, 3>(P, s, 1);
    }
  }
  // short-K forward-layout shapes: the persistent schedule (map < 0 forces the one-tile-per-block kernel, map 7
  // the persistent one at any K: tools/gemm_ab.py). Epilogue operand loads (residual, GELU derivative) are
  // issued after the next tile's asm DMAs, so the compiler's wait for them retires those DMAs too — early,
  // never late.
  const int ntiles = ((P.M + BM - 1) / BM) * ((P.N + BN - 1) / BN);
  // (full column tiles and an even K-tile count only: the persistent epilogue has no column guard, and its K-tile 0
  // must be a steady-state tile)
  if (layout == 0 && (map == 7 || (map == 0 && persistent_ok && P.K <= g_persist_kmax)) && P.K >= 4 * BK &&
      P.N % BN == 0 && P.K % (2 * BK) == 0 &&
      ntiles >= 2 * num_cus() &&
      ((epilogue == EPI_BF16 && P.dbias == nullptr) || epilogue == EPI_GELU || epilogue == EPI_RESID ||
       epilogue == EPI_GELU_BWD) &&
      P.M % BM == 0 && (size_t)P.M * P.lda * 2 < (1ull << 31) && (size_t)P.N * P.ldb * 2 < (1ull << 31)) {
    switch (epilogue) {
      case EPI_BF16: return launch_persistent<EPI_BF16>(P, s, shared_cus);
      case EPI_GELU: return launch_persistent<EPI_GELU>(P, s, shared_cus);
      case EPI_RESID: return launch_persistent<EPI_RESID>(P, s, shared_cus);
      default: return launch_persistent<EPI_GELU_BWD>(P, s, shared_cus);
    }
  }
  if (map < 0 || map == 7) map = 0;
  switch (layout * 16 + epilogue) {
    case 0 * 16 + EPI_BF16: return launch<false, false, EPI_BF16>(P, s, 1);
    case 0 * 16 + EPI_F32: return launch<false, false, EPI_F32>(P, s, 1);
    case 0 * 16 + EPI_RESID: return launch<false, false, EPI_RESID>(P, s, 1);
    case 0 * 16 + EPI_GELU: return launch<false, false, EPI_GELU>(P, s, 1);
    case 0 * 16 + EPI_GELU_BWD: return launch<false, false, EPI_GELU_BWD>(P, s, 1);
    case 1 * 16 + EPI_BF16: return launch<false, true, EPI_BF16>(P, s, 1);
    case 1 * 16 + EPI_F32: return launch<false, true, EPI_F32>(P, s, 1);
    case 1 * 16 + EPI_GELU_BWD: return launch<false, true, EPI_GELU_BWD>(P, s, 1);
    default: return -1;
  }
}
}  // namespace gpt2mi
