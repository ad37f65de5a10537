// Fused softmax cross-entropy (loss + dlogits in one kernel), flat-arena fused AdamW with the
// clip_grad_norm_(inf) sum of squares folded in and the bf16 weight shadow emitted, and helpers.
//
// Replaces: K13 log_softmax+nll_loss fwd/bwd (model.py:357-359), K15
// clip_grad_norm_ (train_gpt2_distributed.py:419-421), K16 _fused_adamw_ (:356-362,424).
#include "common.h"

namespace {

// --- cross entropy ------------------------------------------------------------------------------
// One 256-thread block per row of logits (bf16, row stride ld, V valid columns).
//   pass 1: online (max, sum exp) per thread over 16-B chunks, block combine -> lse
//   loss_row = lse - logit[label]  (0 and not counted when label == ignore_index)
//   pass 2: dlogits = softmax - onehot (bf16, unscaled; the 1/N and upstream grad are applied as
//           the alpha of the backward GEMMs), zero in the padded columns [V, ld_d).
template <typename TL>
__device__ __forceinline__ void load8(const TL* p, float* f) {
  if constexpr (sizeof(TL) == 2) {
    bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = bf2f(v[j]);
  } else {
    const f32x4 a = reinterpret_cast<const f32x4*>(p)[0], b = reinterpret_cast<const f32x4*>(p)[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f[j] = a[j];
      f[4 + j] = b[j];
    }
  }
}
template <typename TL>
__device__ __forceinline__ void store8(TL* p, const float* f) {
  if constexpr (sizeof(TL) == 2) {
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(f[j]);
    *reinterpret_cast<bf16x8*>(p) = o;
  } else {
    reinterpret_cast<f32x4*>(p)[0] = f32x4{f[0], f[1], f[2], f[3]};
    reinterpret_cast<f32x4*>(p)[1] = f32x4{f[4], f[5], f[6], f[7]};
  }
}

template <typename TL>
__global__ __launch_bounds__(256) void xent_fwd_kernel(const TL* __restrict__ logits, int ld,
                                                       const int64_t* __restrict__ labels, float* __restrict__ loss_rows,
                                                       float* __restrict__ lse_out, TL* __restrict__ dlogits, int ldd,
                                                       int V, int ignore_index) {
  const int row = blockIdx.x;
  const TL* lp = logits + (size_t)row * ld;
  const int tid = threadIdx.x;
  float m = -INFINITY, s = 0.f;
  for (int c = 8 * tid; c < V; c += 8 * 256) {
    float f[8];
    load8<TL>(lp + c, f);
    float cm = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      f[j] = (c + j < V) ? f[j] : -INFINITY;
      cm = fmaxf(cm, f[j]);
    }
    const float nm = fmaxf(m, cm);
    float cs = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) cs += __expf(f[j] - nm);
    s = s * __expf(m - nm) + cs;
    m = nm;
  }
  // wave combine
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    const float nm = fmaxf(m, om);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
  }
  __shared__ float sm[4], ss[4];
  __shared__ float s_lse;
  if ((tid & 63) == 0) {
    sm[tid >> 6] = m;
    ss[tid >> 6] = s;
  }
  __syncthreads();
  if (tid == 0) {
    float M_ = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
    float S_ = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) S_ += (sm[w] == -INFINITY) ? 0.f : ss[w] * __expf(sm[w] - M_);
    const float lse = M_ + __logf(S_);
    s_lse = lse;
    lse_out[row] = lse;
    const int64_t y = labels[row];
    // a label outside [0, V) (other than ignore_index) poisons its row with NaN: F.cross_entropy raises on it
    loss_rows[row] = (y == ignore_index) ? 0.f : (y < 0 || y >= V) ? __builtin_nanf("") : lse - (float)lp[y];
  }
  __syncthreads();
  if (!dlogits) return;
  const int64_t y = labels[row];
  const bool ign = (y == ignore_index);
  const float lse = (!ign && (y < 0 || y >= V)) ? __builtin_nanf("") : s_lse;
  TL* dp = dlogits + (size_t)row * ldd;
  for (int c = 8 * tid; c < ldd; c += 8 * 256) {
    float o[8];
    if (c < V) {
      float v[8];
      load8<TL>(lp + c, v);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        o[j] = (c + j < V && !ign) ? __expf(v[j] - lse) - ((c + j == y) ? 1.f : 0.f) : 0.f;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = 0.f;
    }
    store8<TL>(dp + c, o);
  }
}

// Register-resident variant (the bf16 GPT-2 head: V = 50257): one 1024-thread block per row holds
// the whole row in registers (NCH chunks of 8 logits per thread), so the logits are read from HBM
// ONCE: max -> sum of exp -> lse -> dlogits all from registers (the two-pass kernel above re-reads a
// 100 KB row that no longer sits in L2 when its second pass starts: 3 passes of HBM traffic).
// 60 VGPRs (the row packed, see fence()) = two blocks per CU, so one row's load phase overlaps another's
// store phase (2611 -> 2494 us at cfg 2's head; at 90 VGPRs a CU held one row at a time).
#ifndef XENT_EXP_ONCE
#define XENT_EXP_ONCE 0  // A/B builds: 1 = one exp per logit (the row replaced by its bf16 exp(v - max))
#endif
GPT2MI_PRODUCT_KNOB(XENT_EXP_ONCE, 0);
template <int NCH>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8)))
void xent_row_kernel(const bf16* __restrict__ logits, int ld, const int64_t* __restrict__ labels,
                                                        float* __restrict__ loss_rows, float* __restrict__ lse_out,
                                                        bf16* __restrict__ dlogits, int ldd, int V, int ignore_index) {
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const bf16* lp = logits + (size_t)row * ld;
  __shared__ float red[16];
  __shared__ float s_bcast;
  [[maybe_unused]] __shared__ float s_inv_sum;
  bf16x8 raw[NCH];  // the row, packed (4 VGPRs per chunk of 8)
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = 8 * (tid + 1024 * i);
    raw[i] = c < ld ? *reinterpret_cast<const bf16x8*>(lp + c) : bf16x8{};
    if (c + 8 > V) {  // the padding (and the unread tail) never wins the max and has exp(.) = 0
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (c + j >= V) raw[i][j] = (bf16)(-INFINITY);
    }
  }
  auto val = [&](int i, int j) { return bf2f(raw[i][j]); };
  // the row stays packed between the phases: without these fences the compiler keeps all 56 unpacked fp32 values
  // live across the reductions (90 VGPRs = one 1024-thread block per CU, whose load and store phases never overlap)
  auto fence = [&]() {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      u32x4 t = __builtin_bit_cast(u32x4, raw[i]);
      asm volatile("" : "+v"(t));
      raw[i] = __builtin_bit_cast(bf16x8, t);
    }
  };
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < NCH; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmaxf(m, val(i, j));
  fence();
  m = wave_max(m);
  if (lane == 0) red[w] = m;
  __syncthreads();
  if (tid == 0) {
    float t = red[0];
    for (int k = 1; k < 16; ++k) t = fmaxf(t, red[k]);
    s_bcast = t;
  }
  __syncthreads();
  const float mx = s_bcast;
  float sum = 0.f;
#if XENT_EXP_ONCE
  // (A/B timing build) the row's exp(v - max) replaces it in the packed registers (bf16): dlogits is then one multiply
  // by 1/sum per element instead of a second exp (one more bf16 rounding than the product kernel's)
#pragma unroll
  for (int i = 0; i < NCH; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float e = __expf(val(i, j) - mx);
      sum += e;
      raw[i][j] = f2bf(e);
    }
#else
#pragma unroll
  for (int i = 0; i < NCH; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) sum += __expf(val(i, j) - mx);  // exp(-inf) = 0 for the padding
#endif
  fence();
  sum = wave_sum(sum);
  __syncthreads();  // s_bcast consumed
  if (lane == 0) red[w] = sum;
  __syncthreads();
  if (tid == 0) {
    float t = 0.f;
    for (int k = 0; k < 16; ++k) t += red[k];
    const float lse = mx + __logf(t);
    s_bcast = lse;
#if XENT_EXP_ONCE
    s_inv_sum = 1.f / t;
#endif
    lse_out[row] = lse;
    const int64_t y = labels[row];
    loss_rows[row] = (y == ignore_index) ? 0.f : (y < 0 || y >= V) ? __builtin_nanf("") : lse - bf2f(lp[y]);
  }
  __syncthreads();
  if (!dlogits) return;
  const int64_t y = labels[row];
  const bool ign = (y == ignore_index);
  const float lse = (!ign && (y < 0 || y >= V)) ? __builtin_nanf("") : s_bcast;  // bad label: NaN row
  [[maybe_unused]] const float s_inv = (!ign && (y < 0 || y >= V)) ? __builtin_nanf("") : s_inv_sum;
  bf16* dp = dlogits + (size_t)row * ldd;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = 8 * (tid + 1024 * i);
    if (c >= ldd) continue;
    bf16x8 o;
#pragma unroll
#if XENT_EXP_ONCE
    for (int j = 0; j < 8; ++j) o[j] = f2bf(ign ? 0.f : val(i, j) * s_inv);
#else
    for (int j = 0; j < 8; ++j) o[j] = f2bf(ign ? 0.f : __expf(val(i, j) - lse));
#endif
    if (!ign && (uint32_t)(y - c) < 8u) o[y - c] = f2bf(bf2f(o[y - c]) - 1.f);
    *reinterpret_cast<bf16x8*>(dp + c) = o;
  }
}

// loss = sum(loss_rows)/count(valid); inv_count = 1/count (the dlogits scale for backward).
__global__ __launch_bounds__(1024) void xent_finalize_kernel(const float* __restrict__ loss_rows,
                                                            const int64_t* __restrict__ labels, int M, int ignore_index,
                                                            float* __restrict__ loss, float* __restrict__ inv_count) {
  float s = 0.f, n = 0.f;
  // four rows' loads issued together, then added in row order (the same sums as one row per step: 33 us with one
  // dependent load at a time over cfg 2's 65536 rows)
  int i = threadIdx.x;
  for (; i + 3 * 1024 < M; i += 4 * 1024) {
    float l[4];
    int64_t y[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      l[k] = loss_rows[i + 1024 * k];
      y[k] = labels[i + 1024 * k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      s += l[k];
      n += (y[k] == ignore_index) ? 0.f : 1.f;
    }
  }
  for (; i < M; i += 1024) {
    s += loss_rows[i];
    n += (labels[i] == ignore_index) ? 0.f : 1.f;
  }
  s = wave_sum(s);
  n = wave_sum(n);
  __shared__ float rs[16], rn[16];
  if ((threadIdx.x & 63) == 0) {
    rs[threadIdx.x >> 6] = s;
    rn[threadIdx.x >> 6] = n;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float S = 0.f, N = 0.f;
    for (int w = 0; w < 16; ++w) {
      S += rs[w];
      N += rn[w];
    }
    loss[0] = S / N;  // NaN when every label is ignored, as F.cross_entropy
    inv_count[0] = 1.f / N;
  }
}

// --- AdamW over the flat fp32 arena -------------------------------------------------------------
// torch/optim/adam.py decoupled-decay math (train_gpt2_distributed.py:356-362):
//   g *= grad_scale; p *= 1 - lr*wd; m = m + (1-b1)(g-m); v = b2 v + (1-b2) g^2;
//   p -= step_size * m / (sqrt(v)/bc2_sqrt + eps)       step_size = lr/(1-b1^t), bc2_sqrt = sqrt(1-b2^t)
// Also: partial sums of g^2 (the clip_grad_norm_(inf) total norm, computed from the same read of g
// before the update, as the reference computes it before optim.step()), and the bf16 shadow of p.
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    bf16* __restrict__ pb, size_t n4, float lr, float wd, float b1,
                                                    float b2, float eps, float step_size, float bc2_sqrt,
                                                    float grad_scale, float* __restrict__ partials) {
  float sq = 0.f;
  const float decay = 1.f - lr * wd;
  auto upd = [&](f32x4& pv, f32x4 gv, f32x4& mv, f32x4& vv) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gg = gv[j] * grad_scale;
      sq += gg * gg;
      float pp = pv[j] * decay;
      const float mm = mv[j] + (1.f - b1) * (gg - mv[j]);
      const float vvv = b2 * vv[j] + (1.f - b2) * gg * gg;
      pp -= step_size * mm / (sqrtf(vvv) / bc2_sqrt + eps);
      pv[j] = pp;
      mv[j] = mm;
      vv[j] = vvv;
    }
  };
  // 8 parameters per thread and iteration: the bf16 shadow leaves in one 16-B store (the 8-B form doubles the
  // store instructions of that array), and twice the loads are in flight per wave
  const size_t n8 = n4 / 2;
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n8; i += (size_t)gridDim.x * 256) {
    f32x4 pv0 = reinterpret_cast<f32x4*>(p)[2 * i], pv1 = reinterpret_cast<f32x4*>(p)[2 * i + 1];
    const f32x4 gv0 = reinterpret_cast<const f32x4*>(g)[2 * i], gv1 = reinterpret_cast<const f32x4*>(g)[2 * i + 1];
    f32x4 mv0 = reinterpret_cast<f32x4*>(m)[2 * i], mv1 = reinterpret_cast<f32x4*>(m)[2 * i + 1];
    f32x4 vv0 = reinterpret_cast<f32x4*>(v)[2 * i], vv1 = reinterpret_cast<f32x4*>(v)[2 * i + 1];
    upd(pv0, gv0, mv0, vv0);
    upd(pv1, gv1, mv1, vv1);
    reinterpret_cast<f32x4*>(p)[2 * i] = pv0;
    reinterpret_cast<f32x4*>(p)[2 * i + 1] = pv1;
    reinterpret_cast<f32x4*>(m)[2 * i] = mv0;
    reinterpret_cast<f32x4*>(m)[2 * i + 1] = mv1;
    reinterpret_cast<f32x4*>(v)[2 * i] = vv0;
    reinterpret_cast<f32x4*>(v)[2 * i + 1] = vv1;
    if (pb)
      reinterpret_cast<bf16x8*>(pb)[i] = bf16x8{f2bf(pv0[0]), f2bf(pv0[1]), f2bf(pv0[2]), f2bf(pv0[3]),
                                                f2bf(pv1[0]), f2bf(pv1[1]), f2bf(pv1[2]), f2bf(pv1[3])};
  }
  if (n4 & 1) {  // an odd count of 4-parameter groups: the last one
    const size_t i = n4 - 1;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      f32x4 pv = reinterpret_cast<f32x4*>(p)[i], mv = reinterpret_cast<f32x4*>(m)[i], vv = reinterpret_cast<f32x4*>(v)[i];
      upd(pv, reinterpret_cast<const f32x4*>(g)[i], mv, vv);
      reinterpret_cast<f32x4*>(p)[i] = pv;
      reinterpret_cast<f32x4*>(m)[i] = mv;
      reinterpret_cast<f32x4*>(v)[i] = vv;
      if (pb) reinterpret_cast<bf16x4*>(pb)[i] = bf16x4{f2bf(pv[0]), f2bf(pv[1]), f2bf(pv[2]), f2bf(pv[3])};
    }
  }
  sq = wave_sum(sq);
  __shared__ float r[4];
  if ((threadIdx.x & 63) == 0) r[threadIdx.x >> 6] = sq;
  __syncthreads();
  if (threadIdx.x == 0 && partials) partials[blockIdx.x] = r[0] + r[1] + r[2] + r[3];
}

__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ g, size_t n4, float scale,
                                                    float* __restrict__ partials) {
  float sq = 0.f;
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    f32x4 gv = reinterpret_cast<const f32x4*>(g)[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) sq += gv[j] * gv[j] * scale * scale;
  }
  sq = wave_sum(sq);
  __shared__ float r[4];
  if ((threadIdx.x & 63) == 0) r[threadIdx.x >> 6] = sq;
  __syncthreads();
  if (threadIdx.x == 0) partials[blockIdx.x] = r[0] + r[1] + r[2] + r[3];
}

// Deterministic final reduction of per-block partials: out = sqrt(sum). One 1024-thread block whose threads load 4
// partials per step before adding them (independent loads in flight: FSDP's per-unit optimizer hands it 14 x 2048
// partials, 40 us with one dependent load per step at 256 threads)
__global__ __launch_bounds__(1024) void norm_finalize_kernel(const float* __restrict__ partials, int n,
                                                             float* __restrict__ out) {
  double s = 0.0;
  int i = threadIdx.x;
  for (; i + 3 * 1024 < n; i += 4 * 1024) {
    const float a = partials[i], b = partials[i + 1024], c = partials[i + 2048], d = partials[i + 3072];
    s += a;
    s += b;
    s += c;
    s += d;
  }
  for (; i < n; i += 1024) s += partials[i];
  __shared__ double r[1024];
  r[threadIdx.x] = s;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if (threadIdx.x < o) r[threadIdx.x] += r[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = (float)sqrt(r[0]);
}

__global__ __launch_bounds__(256) void cast_f32_bf16_kernel(const float* __restrict__ x, bf16* __restrict__ y, size_t n) {
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) y[i] = f2bf(x[i]);
}

__global__ void scale_mul_kernel(const float* a, const float* b, float* out) { out[0] = a[0] * b[0]; }

constexpr int kNormBlocks = 2048;

}  // namespace

template <typename TL>
static int xent_fwd_t(const TL* logits, int ld, const int64_t* labels, float* loss_rows, float* lse, TL* dlogits,
                      int ldd, int M, int V, int ignore_index, float* loss, float* inv_count, void* stream) {
  GPT2MI_REQUIRE(ld % 8 == 0 && ld >= V && (dlogits == nullptr || (ldd % 8 == 0 && ldd >= V)),
                 "xent_fwd: row strides must be multiples of 8 and >= V (ld=%d ldd=%d V=%d)", ld, ldd, V);
  hipStream_t s = (hipStream_t)stream;
  const int nch = (max(ld, dlogits ? ldd : 0) + 8 * 1024 - 1) / (8 * 1024);
  if constexpr (sizeof(TL) == 2) {
    if (nch == 7) {  // GPT-2 vocab under autocast: one register-resident pass over the bf16 logits
      xent_row_kernel<7><<<M, 1024, 0, s>>>(logits, ld, labels, loss_rows, lse, dlogits, ldd, V, ignore_index);
      int rc = gpt2mi::check_launch("xent_row");
      if (rc) return rc;
      xent_finalize_kernel<<<1, 1024, 0, s>>>(loss_rows, labels, M, ignore_index, loss, inv_count);
      return gpt2mi::check_launch("xent_finalize");
    }
  }
  xent_fwd_kernel<TL><<<M, 256, 0, s>>>(logits, ld, labels, loss_rows, lse, dlogits, ldd, V, ignore_index);
  int rc = gpt2mi::check_launch("xent_fwd");
  if (rc) return rc;
  xent_finalize_kernel<<<1, 1024, 0, s>>>(loss_rows, labels, M, ignore_index, loss, inv_count);
  return gpt2mi::check_launch("xent_finalize");
}

GPT2MI_EXPORT int gpt2mi_xent_fwd(const uint16_t* logits, int ld, const int64_t* labels, float* loss_rows, float* lse,
                                  uint16_t* dlogits, int ldd, int M, int V, int ignore_index, float* loss,
                                  float* inv_count, void* stream) {
  return xent_fwd_t<bf16>((const bf16*)logits, ld, labels, loss_rows, lse, (bf16*)dlogits, ldd, M, V, ignore_index,
                          loss, inv_count, stream);
}

GPT2MI_EXPORT int gpt2mi_xent_fwd_f32(const float* logits, int ld, const int64_t* labels, float* loss_rows, float* lse,
                                      float* dlogits, int ldd, int M, int V, int ignore_index, float* loss,
                                      float* inv_count, void* stream) {
  return xent_fwd_t<float>(logits, ld, labels, loss_rows, lse, dlogits, ldd, M, V, ignore_index, loss, inv_count,
                           stream);
}

GPT2MI_EXPORT int gpt2mi_adamw(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, size_t n, float lr,
                               float wd, float b1, float b2, float eps, int step, float grad_scale, float* partials,
                               float* grad_norm, void* stream) {
  GPT2MI_REQUIRE(n % 4 == 0, "adamw: n=%zu must be a multiple of 4", n);
  GPT2MI_REQUIRE(step >= 1, "adamw: step must be >= 1");
  hipStream_t s = (hipStream_t)stream;
  const double bc1 = 1.0 - pow((double)b1, step), bc2 = 1.0 - pow((double)b2, step);
  const float step_size = (float)(lr / bc1), bc2_sqrt = (float)sqrt(bc2);
  adamw_kernel<<<kNormBlocks, 256, 0, s>>>(p, g, m, v, (bf16*)p_bf16, n / 4, lr, wd, b1, b2, eps, step_size, bc2_sqrt,
                                           grad_scale, partials);
  int rc = gpt2mi::check_launch("adamw");
  if (rc || !grad_norm) return rc;
  norm_finalize_kernel<<<1, 1024, 0, s>>>(partials, kNormBlocks, grad_norm);
  return gpt2mi::check_launch("adamw_norm");
}

GPT2MI_EXPORT int gpt2mi_grad_norm(const float* g, size_t n, float scale, float* partials, float* out, void* stream) {
  GPT2MI_REQUIRE(n % 4 == 0, "grad_norm: n=%zu must be a multiple of 4", n);
  hipStream_t s = (hipStream_t)stream;
  sumsq_kernel<<<kNormBlocks, 256, 0, s>>>(g, n / 4, scale, partials);
  int rc = gpt2mi::check_launch("grad_norm");
  if (rc) return rc;
  norm_finalize_kernel<<<1, 1024, 0, s>>>(partials, kNormBlocks, out);
  return gpt2mi::check_launch("grad_norm_finalize");
}

GPT2MI_EXPORT int gpt2mi_norm_partials_size(void) { return kNormBlocks; }

GPT2MI_EXPORT int gpt2mi_norm_finalize(const float* partials, int n, float* out, void* stream) {
  GPT2MI_REQUIRE(n > 0, "norm_finalize: n=%d", n);
  norm_finalize_kernel<<<1, 1024, 0, (hipStream_t)stream>>>(partials, n, out);
  return gpt2mi::check_launch("norm_finalize");
}

GPT2MI_EXPORT int gpt2mi_cast_f32_bf16(const float* x, uint16_t* y, size_t n, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  cast_f32_bf16_kernel<<<2048, 256, 0, s>>>(x, (bf16*)y, n);
  return gpt2mi::check_launch("cast_f32_bf16");
}

GPT2MI_EXPORT int gpt2mi_scale_mul(const float* a, const float* b, float* out, void* stream) {
  scale_mul_kernel<<<1, 1, 0, (hipStream_t)stream>>>(a, b, out);
  return gpt2mi::check_launch("scale_mul");
}

// Zero n ranges [off, off+cnt) of a float array in one launch (blockIdx.y = range; ranges = device int64 pairs):
// the grad arena's atomically accumulated slots before a backward whose GEMMs write the weight slots outright.
__global__ __launch_bounds__(256) void zero_ranges_kernel(float* __restrict__ base, const int64_t* __restrict__ ranges) {
  const int64_t off = ranges[2 * blockIdx.y], cnt = ranges[2 * blockIdx.y + 1];
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < cnt; i += (int64_t)gridDim.x * 256) base[off + i] = 0.f;
}

GPT2MI_EXPORT int gpt2mi_zero_ranges(float* base, const int64_t* ranges, int n, void* stream) {
  GPT2MI_REQUIRE(n >= 0 && n <= 65535, "zero_ranges: %d ranges (at most 65535)", n);
  if (n == 0) return 0;
  zero_ranges_kernel<<<dim3(64, n), 256, 0, (hipStream_t)stream>>>(base, ranges);
  return gpt2mi::check_launch("zero_ranges");
}

GPT2MI_EXPORT int gpt2mi_memset_zero(void* ptr, size_t bytes, void* stream) {
  hipError_t e = hipMemsetAsync(ptr, 0, bytes, (hipStream_t)stream);
  if (e != hipSuccess) {
    gpt2mi::set_error("memset_zero: %s", hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}
