/*
 * gpt2mi.h — C ABI of libgpt2mi.so, the MI355X (gfx950) kernels of the GPT-2 training step.
 *
 * The reference (dpickem/gpt_2_distributed) has no native code and no FFI: its hot path is the
 * implicit aten/cuBLAS/NCCL work behind model.py + train_gpt2_distributed.py. Each entry below
 * replaces the aten work of the reference site cited next to it; the
 * Python binding is gpt_2_distributed_amd/_lib.py (ctypes), see INTEGRATION.md.
 *
 * Conventions
 *  - Every pointer is a DEVICE pointer allocated by the caller (PyTorch's caching allocator in
 *    the package). Kernels never allocate or free.
 *  - bf16 tensors are passed as uint16_t* (raw bf16 bits). Shapes are row-major with explicit
 *    leading dimensions (in elements).
 *  - `stream` is a hipStream_t passed as void*; all launches are asynchronous on it.
 *  - Return value: 0 on success; otherwise an errno-style (22 = invalid argument) or hipError_t
 *    code, with a message in gpt2mi_last_error() (thread-local).
 *  - Dropout (p > 0) uses a counter-based hash of (seed, element index) so backward regenerates
 *    the forward mask; p = 0 disables it.
 */
#ifndef GPT2MI_H
#define GPT2MI_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPT2MI_ABI_VERSION 13

const char* gpt2mi_last_error(void);
int gpt2mi_abi_version(void); /* returns GPT2MI_ABI_VERSION of the built library */

/* K1: x[b,t,:] = drop(wte[idx[b,t],:] + wpe[t,:])  — model.py:295-304 (embedding, add, dropout).
 * Rows with t >= T_valid are sequence padding (T rounded up to the attention tile by the engine): x = 0
 * there and neither table is read (wpe may have only T_valid rows). */
int gpt2mi_embed_fwd(const int64_t* idx, const float* wte, const float* wpe, float* x, int B, int T, int T_valid,
                     int C, float p, uint64_t seed, void* stream);
/* embedding_dense_backward of both tables: dwte[idx] += g, dwpe[t] += sum_b g (g = dres masked); rows
 * t >= T_valid are skipped. */
int gpt2mi_embed_bwd(const int64_t* idx, const float* dres, float* dwte, float* dwpe, int B, int T, int T_valid,
                     int C, float p, uint64_t seed, void* stream);

/* K2: nn.LayerNorm forward — model.py:204,210,247 (used :215,218,311). y_bf16 and/or y_f32 may be NULL. */
int gpt2mi_layernorm_fwd(const float* x, const float* w, const float* b, uint16_t* y_bf16, float* y_f32,
                         float* mean, float* rstd, int M, int C, float eps, void* stream);
/* native_layer_norm_backward fused with the residual gradient (dres += dx, or = dx if dres_init),
 * dw/db += ; optionally emits out_bf16 = bf16(dres*keep/(1-p_out)) for the residual branch below and
 * dbias_out += colsum(out_bf16) (that branch's bias grad). */
int gpt2mi_layernorm_bwd(const float* x, const float* w, const float* mean, const float* rstd, const uint16_t* dy,
                         float* dres, float* dw, float* db, uint16_t* out_bf16, float* dbias_out, int M, int C,
                         float p_out, uint64_t seed_out, int dres_init, void* stream);

/* Bias grad of an addmm: db[n] += sum_m g[m,n] (g bf16, row stride ld). */
int gpt2mi_colsum_bf16(const uint16_t* g, float* db, int M, int N, int ld, void* stream);

/* K3/K9/K10/K11/K12/K14 GEMMs — model.py:95-96,174-177,326 (nn.Linear under bf16 autocast) and their
 * autograd backward (train_gpt2_distributed.py:412).
 *   C[m,n] = epi(alpha*(alpha_dev?*alpha_dev:1) * sum_k A(m,k) B(n,k))
 * layout 0: A[M][K], B[N][K]   (x @ W^T)        layout 1: A[M][K], B[K][N]   (dY @ W, dgrad)
 * layout 2: A[K][M], B[K][N]   (dY^T @ X, wgrad)
 * epilogue 0 BF16: C bf16 (+bias)            1 F32: C fp32 (+bias), += when accumulate
 *          2 RESID: C fp32 = resid + drop(acc+bias)
 *          3 GELU: u = acc+bias, C = bf16(drop(gelu(u))), aux = bf16(keep/(1-p) * gelu'(u)) (what backward needs)
 *          4 GELU_BWD: C = bf16(acc * aux) (aux from the GELU forward)   5 ATOMIC: C fp32 += acc (split-K)
 * dbias (may be NULL; BF16 / GELU_BWD epilogues of layouts 0/1): dbias[n] += sum_m C[m][n] of the stored
 * output — the bias gradient of the Linear whose output grad C is (fused into the 256x256 epilogue).
 * Requires M, N multiples of 64 and K a multiple of 64*splits (layout 0: any N multiple of 64 and any K-tile count on
 * the 256x256 kernels; layouts 1 / 2 with N (and M) not multiples of 256 run on the 128x128 kernel).
 * `sched`: GPT2MI_SCHED_* below. */
int gpt2mi_gemm(int layout, int epilogue, int M, int N, int K, const uint16_t* A, int lda, const uint16_t* B, int ldb,
                void* C, int ldc, const float* bias, const float* resid, uint16_t* aux, int ldaux, float alpha,
                const float* alpha_dev, int accumulate, int splits, float p_drop, uint64_t seed, float* dbias,
                int sched, void* stream);

/* GEMM schedule, chosen per call (v8; v7 had process-global switches):
 *  GPT2MI_SCHED_AUTO: the library picks the kernel (ping-pong 256x256; its persistent schedule for the short-K
 *    forward-layout shapes).
 *  GPT2MI_SCHED_NO_PERSISTENT (flag): never the persistent (one block per CU) schedule (one tile per block).
 *  GPT2MI_SCHED_SHARED_CUS (flag, v11): other kernels (the data-parallel wrappers' RCCL collectives) may hold CUs while
 *    this GEMM runs. The persistent schedule then takes its tiles from per-XCD work queues instead of a static walk:
 *    a block whose CU a collective holds takes fewer tiles instead of making the grid end on its latest block.
 *  low byte (A/B experiments and the kernel-equivalence tests only): 1 = 128x128 kernel, 2 = 2-stage 256x256,
 *    3..5 = ping-pong with half-tile map 1..3, 6 = ping-pong one tile per block, 7 = persistent at any K,
 *    8 = weight gradients on the ping-pong kernel (= auto). */
#define GPT2MI_SCHED_AUTO 0
#define GPT2MI_SCHED_NO_PERSISTENT 0x100
#define GPT2MI_SCHED_SHARED_CUS 0x400
/* GPT2MI_SCHED_BF16_SLABS (flag, gpt2mi_gemm_wgrad / gpt2mi_gemm_wgrad_kt only; v10): each split-K partial sum is
 * rounded once to bf16 in its slab, then the slabs are summed in fp32 in split order (still deterministic) — half the
 * slab write and reduce traffic. The reference's autocast weight gradient rounds its whole sum to bf16 once
 * (torch.mm in bf16, cast to the fp32 .grad: train_gpt2_distributed.py:412); this rounds each of `splits` partial
 * sums, an error of the same order. Without the flag the slabs are fp32 (fp32-exact weight gradients). */
#define GPT2MI_SCHED_BF16_SLABS 0x200

/* Weight gradient (train_gpt2_distributed.py:412 autograd wgrad of every nn.Linear):
 * C[M][N] (+)= alpha*(alpha_dev?) * A^T B, A stored [K][M] (dY), B stored [K][N] (X), K = tokens.
 * 256x256 tiles; `splits` K ranges write fp32 (GPT2MI_SCHED_BF16_SLABS: bf16) partial slabs to `workspace`
 * (>= splits*M*N floats), summed into C in a fixed order (deterministic). M, N, K multiples of 64; ldc == N. sched: as gpt2mi_gemm
 * (the low byte 2 selects the 2-stage kernel). When M (N) is not a multiple of 256 (GPT-2 1.5B: 1600, 4800) the
 * partial last tile's reads are bounded by the operand's last element ((K-1)*lda + M, (K-1)*ldb + N; buffer
 * num_records): no slack past the operands is needed (v11; v10 read up to 192 elements past the last row). */
int gpt2mi_gemm_wgrad(int M, int N, int K, const uint16_t* A, int lda, const uint16_t* B, int ldb, float* C, int ldc,
                      int accumulate, float alpha, const float* alpha_dev, float* workspace, size_t workspace_floats,
                      int splits, int sched, void* stream);
/* The same weight gradient with B given transposed, k-contiguous: Bt stored [N][K] (X^T; train_gpt2_distributed.py:412,
 * the tied lm_head's wgrad against the final LayerNorm output transposed once per step). Computes C^T = Bt . A on the
 * ping-pong kernel (one transposed operand instead of two) into split-K slabs (workspace >= splits*M*N floats,
 * required) and sums them, transposed, into C (fixed order: the same bits as gpt2mi_gemm_wgrad). M multiple of 256,
 * N of 64, K of 128; ldc == N. ABI v9. */
int gpt2mi_gemm_wgrad_kt(int M, int N, int K, const uint16_t* A, int lda, const uint16_t* Bt, int ldbt, float* C,
                         int ldc, int accumulate, float alpha, const float* alpha_dev, float* workspace,
                         size_t workspace_floats, int splits, int sched, void* stream);

/* Grouped weight gradients (v13; train_gpt2_distributed.py:412, the autograd wgrads of a GPT2Block's four nn.Linear,
 * model.py:95,96,174,177): for g < count (<= 4), C[g][M[g]][N[g]] (+)= alpha*(alpha_dev?) * A[g]^T B[g] over the same
 * K tokens, as ONE split-K launch and ONE reduction launch. Host arrays of count entries; every M[g], N[g] a multiple of
 * 256, K of 128, ldc == N[g]; workspace >= splits * sum(M[g]*N[g]) floats. Each C[g] gets the bits gpt2mi_gemm_wgrad
 * gives it with the same `splits` and fp32 slabs. sched: GPT2MI_SCHED_AUTO or the CU-sharing flags (no BF16_SLABS). */
int gpt2mi_gemm_wgrad_grouped(int count, const int* M, const int* N, int K, const uint16_t* const* A, const int* lda,
                              const uint16_t* const* B, const int* ldb, float* const* C, int accumulate, float alpha,
                              const float* alpha_dev, float* workspace, size_t workspace_floats, int splits, int sched,
                              void* stream);

/* K4-K8: causal flash attention, head_dim 64 — model.py:124-155. q/k/v read from qkv [B*T, 3C];
 * out [B*T, C] head-merged; lse [B*H, T] (natural log of the 1/sqrt(D)-scaled scores). */
int gpt2mi_attn_fwd(const uint16_t* qkv, uint16_t* out, float* lse, int B, int T, int H, int head_dim, float p_drop,
                    uint64_t seed, void* stream);
/* Backward: delta [B*H, T] workspace (dO.O, formed by the dQ pass); dqkv [B*T, 3C] written in the qkv
 * layout. dqkv_colsum (may be NULL): [B*T/32, 3C] fp32 partial column sums of the stored dqkv, one row
 * per 32 tokens — the qkv bias gradient after gpt2mi_colsum_f32 over its rows (model.py c_attn bias). */
int gpt2mi_attn_bwd(const uint16_t* qkv, const uint16_t* out, const uint16_t* dout, const float* lse, float* delta,
                    uint16_t* dqkv, float* dqkv_colsum, int B, int T, int H, int head_dim, float p_drop,
                    uint64_t seed, void* stream);

/* K13: F.cross_entropy(logits.view(-1,V), labels.view(-1), ignore_index) — model.py:357-359.
 * logits bf16 [M, ld]; writes loss_rows [M], lse [M], loss[0] = mean, inv_count[0] = 1/#valid and, if
 * dlogits != NULL, dlogits = softmax - onehot (bf16 [M, ldd], unscaled, zero in columns >= V). A label
 * outside [0, V) other than ignore_index (F.cross_entropy raises) makes its loss row and dlogits row NaN. */
int gpt2mi_xent_fwd(const uint16_t* logits, int ld, const int64_t* labels, float* loss_rows, float* lse,
                    uint16_t* dlogits, int ldd, int M, int V, int ignore_index, float* loss, float* inv_count,
                    void* stream);

/* K15+K16: fused AdamW over a flat fp32 arena (torch.optim.AdamW(lr, weight_decay, betas, eps), one
 * param group, decoupled decay — train_gpt2_distributed.py:356-362,424) with g *= grad_scale, the
 * clip_grad_norm_(inf) total norm of the scaled grads -> grad_norm[0] (partials: workspace of
 * gpt2mi_norm_partials_size() floats), and the bf16 shadow p_bf16 (may be NULL). */
int gpt2mi_adamw(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, size_t n, float lr, float wd,
                 float b1, float b2, float eps, int step, float grad_scale, float* partials, float* grad_norm,
                 void* stream);
int gpt2mi_grad_norm(const float* g, size_t n, float scale, float* partials, float* out, void* stream);
/* v12: out[0] = sqrt(sum of partials[0..n)) — the norm of several gpt2mi_adamw launches given grad_norm = NULL and
 * consecutive gpt2mi_norm_partials_size()-float slices of one partials buffer (FSDP's AdamW runs once per unit). */
int gpt2mi_norm_finalize(const float* partials, int n, float* out, void* stream);
int gpt2mi_norm_partials_size(void);

/* ---- fp32 mode: the reference model.py run WITHOUT torch.autocast (plain fp32 module; the CPU
 * trajectory goldens and the north star's "fp32 loss within 1e-4" gate). Same contracts as the bf16
 * entries above with every activation / weight operand fp32 (C and aux of the "BF16", GELU and
 * GELU_BWD epilogues are fp32 too). GEMM products are exact fp32 (v_mfma_f32_16x16x4_f32). ---- */
/* K3/K9-K12/K14 in fp32: N % 4 == 0, K % (16*splits) == 0, leading dims % 4 == 0. */
int gpt2mi_gemm_f32(int layout, int epilogue, int M, int N, int K, const float* A, int lda, const float* B, int ldb,
                    void* C, int ldc, const float* bias, const float* resid, float* aux, int ldaux, float alpha,
                    const float* alpha_dev, int accumulate, int splits, float p_drop, uint64_t seed, float* dbias,
                    void* stream);
/* K4-K8 in fp32 (model.py:124-155 without autocast); same dropout mask as gpt2mi_attn_fwd. */
int gpt2mi_attn_fwd_f32(const float* qkv, float* out, float* lse, int B, int T, int H, int head_dim, float p_drop,
                        uint64_t seed, void* stream);
int gpt2mi_attn_bwd_f32(const float* qkv, const float* out, const float* dout, const float* lse, float* delta,
                        float* dqkv, float* dqkv_colsum /* must be NULL */, int B, int T, int H, int head_dim,
                        float p_drop, uint64_t seed, void* stream);
/* LayerNorm backward with fp32 dy and fp32 branch output (see gpt2mi_layernorm_bwd). */
int gpt2mi_layernorm_bwd_f32(const float* x, const float* w, const float* mean, const float* rstd, const float* dy,
                             float* dres, float* dw, float* db, float* out_f32, float* dbias_out, int M, int C,
                             float p_out, uint64_t seed_out, int dres_init, void* stream);
int gpt2mi_colsum_f32(const float* g, float* db, int M, int N, int ld, void* stream);
/* K13 on fp32 logits (the fp32 lm_head output), fp32 dlogits. */
int gpt2mi_xent_fwd_f32(const float* logits, int ld, const int64_t* labels, float* loss_rows, float* lse,
                        float* dlogits, int ldd, int M, int V, int ignore_index, float* loss, float* inv_count,
                        void* stream);

/* dst[c][r] = src[r][c] for a bf16 [R][C] matrix (R, C multiples of 64): the transposed weight shadow
 * the backward dgrad GEMMs read in the forward (k-contiguous) layout. */
int gpt2mi_transpose_bf16(const uint16_t* src, uint16_t* dst, int R, int C, int ld_src, int ld_dst, void* stream);
/* All weights of a shadow arena in one launch: desc (device, int64 [n][4]) = {element offset, R, C, first
 * tile index} with R, C multiples of 64 and first tiles the prefix sums of (R/64)*(C/64); src + offset is a
 * dense [R][C] matrix, dst + offset receives its [C][R] transpose. */
int gpt2mi_transpose_bf16_batched(const uint16_t* src, uint16_t* dst, const int64_t* desc, int n,
                                  int64_t total_tiles, void* stream);
int gpt2mi_cast_f32_bf16(const float* x, uint16_t* y, size_t n, void* stream);
int gpt2mi_cast_bf16_f32(const uint16_t* x, float* y, size_t n, void* stream);

/* ---- v5: the boundary around the fused step (aux_ops.hip) ---- */
/* Gradient entering through the returned logits (model.py:351: logits are returned and differentiable):
 * dl[b*Tp+t][n] = (init ? 0 : alpha_dev[0]*dl) + g[b*Tv+t][n] for t < Tv, n < V; dl columns [V, ldd) = 0;
 * rows t >= Tv (sequence padding) are zeroed when init, else untouched. dl is the lm_head backward's
 * dlogits (bf16 [B*Tp, ldd]); g the caller's grad of the [B, Tv, V] logits (row stride ldg). */
int gpt2mi_dlogits_accum(uint16_t* dl, int ldd, const uint16_t* g, int ldg, int B, int Tp, int Tv, int V,
                         const float* alpha_dev, int init, void* stream);
int gpt2mi_dlogits_accum_f32(float* dl, int ldd, const float* g, int ldg, int B, int Tp, int Tv, int V,
                             const float* alpha_dev, int init, void* stream);
/* Residual-branch output gradient of a stand-alone sub-module backward (model.py:158,191: resid_drop /
 * drop2 then the branch bias): out = dres*keep/(1-p) (bf16 [M,C]; fp32 for _f32), dbias += colsum(out). */
int gpt2mi_branch_bwd(const float* dres, uint16_t* out, float* dbias, int M, int C, float p, uint64_t seed,
                      void* stream);
int gpt2mi_branch_bwd_f32(const float* dres, float* out, float* dbias, int M, int C, float p, uint64_t seed,
                          void* stream);
/* x *= s (n % 4 == 0): DDP's division of a gradient bucket by the world size before a SUM all-reduce
 * (torch/nn/parallel/distributed.py reducer; train_gpt2_distributed.py:163). */
int gpt2mi_scale_f32(float* x, size_t n, float s, void* stream);
/* FSDP flat units (train_gpt2_distributed.py:146-161, MixedPrecision(param=bf16, reduce=bf16)):
 * unpack a gathered unit into the fp32 parameter view and the bf16 GEMM shadow (either may be NULL);
 * pack a unit's fp32 grads into the zero-padded reduce-scatter input (bf16 or fp32);
 * accumulate the reduce-scattered shard into the fp32 grad shard (= when accumulate == 0). */
int gpt2mi_fsdp_unpack(const void* src, int src_f32, float* dst_f32, uint16_t* dst_bf16, size_t n, void* stream);
int gpt2mi_fsdp_pack(const float* src, void* dst, int dst_f32, size_t n, size_t n_pad, void* stream);
int gpt2mi_fsdp_accum(const void* src, int src_f32, float* dst, size_t n, int accumulate, void* stream);
int gpt2mi_scale_mul(const float* a, const float* b, float* out, void* stream);
int gpt2mi_memset_zero(void* ptr, size_t bytes, void* stream);
/* Zero n element ranges of a float array in one launch; ranges = DEVICE int64 pairs (offset, count).
 * Replaces, for the atomically accumulated slots of the grad arena (LayerNorm params, biases, wpe, ln_f),
 * the full-arena zero of optimizer.zero_grad() (torch/optim/optimizer.py zero_grad via
 * train_gpt2_distributed.py:409-425) when the backward's weight-gradient GEMMs write their slots outright. */
int gpt2mi_zero_ranges(float* base, const int64_t* ranges, int n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GPT2MI_H */
