/*
 * prfl_hip.h — C ABI of the MI355X-native (gfx950 / CDNA4) PRFL hot-path kernels.
 *
 * Library: hy-video-prfl_amd/prfl_amd/lib/libprfl_hip.so   (built by `make -C hy-video-prfl_amd`)
 *
 * Conventions (every entry point):
 *   - all tensors are caller-owned device pointers (PyTorch caching allocator or hipMalloc);
 *     kernels never allocate, never synchronise, and are stream-ordered on `stream`
 *     (a hipStream_t passed as void*; NULL = the default stream);
 *   - sizes and leading dimensions are in ELEMENTS; bf16 = IEEE bfloat16 bit pattern (uint16);
 *   - return 0 on success, otherwise a hipError_t code (hipErrorInvalidValue = 1 for bad
 *     shapes/alignment).  The Python layer turns non-zero into RuntimeError.
 *   - stateless and re-entrant except the optional profiling hooks (prfl_prof_*), which are
 *     single-threaded host state.
 *
 * Each function names the reference interface it replaces (paths relative to the
 * Tencent-Hunyuan/HY-Video-PRFL tree).
 */
#ifndef PRFL_HIP_H
#define PRFL_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- GEMM -------------------------------------------------------------------------------
 * Replaces the autocast nn.Linear calls of the DiT block and their autograd backward:
 *   diffusers_lite/wan/modules/model.py:156-159,175-177,200 (self-attn q/k/v/o),
 *   :216-225,257-270 (cross-attn q/k/v/o, k_img/v_img), :313-315 (FFN), :499-505 (embeddings).
 * C[m][n] = sum_k A(m,k) B(n,k) with
 *   A(m,k) = a_kmajor ? A[m*lda+k] : A[k*lda+m];   B(n,k) = b_kmajor ? B[n*ldb+k] : B[k*ldb+n]
 * epilogue: 0 BF16   C = bf16(acc + bias)                              (bias bf16 [N] or NULL)
 *           1 GELU   C = bf16(gelu_tanh(bf16(acc+bias))); aux (opt.) = bf16(acc+bias)
 *           2 RESID  C(f32) = res + bf16(acc+bias) * gate[n]; aux (opt.) = bf16(acc+bias)
 *                    (res fp32 or bf16 per res_bf16, may alias C; gate fp32 [N] or NULL = 1)
 *           3 F32    C(f32) = acc (+ C if accumulate)                  (weight gradients)
 *           4 DGELU  C = bf16(bf16(acc) * gelu_tanh'(aux))              (aux = pre-activation)
 * Requires K % 8 == 0, N % 4 == 0, lda/ldb % 8 == 0, 16-B aligned A/B, and the contiguous
 * extent of an MN-major operand a multiple of 8. */
int prfl_gemm_bf16(const void* A, int64_t lda, int a_kmajor, const void* B, int64_t ldb,
                   int b_kmajor, void* C, int64_t ldc, int64_t M, int64_t N, int64_t K,
                   int epilogue, const void* bias, const float* gate, const void* res,
                   int64_t ldr, int res_bf16, void* aux, int64_t ldaux, int accumulate,
                   void* stream);
/* The same GEMM with the tile chosen by the caller: tile = 0 (by shape, as prfl_gemm_bf16),
 * 128 (128x128 tile, 4 waves), 256 (256x256 tile, four-wave kernel with AGPR accumulators) or
 * 512 (256x256 tile, 8-wave staggered-ring kernel); 256 / 512 need K % 64 == 0 and MN-major
 * extents % 256 == 0, else hipErrorInvalidValue.  All kernels sum every output element in the
 * same k order, so their results are bit-identical. */
int prfl_gemm_bf16_tiled(const void* A, int64_t lda, int a_kmajor, const void* B, int64_t ldb,
                         int b_kmajor, void* C, int64_t ldc, int64_t M, int64_t N, int64_t K,
                         int epilogue, const void* bias, const float* gate, const void* res,
                         int64_t ldr, int res_bf16, void* aux, int64_t ldaux, int accumulate,
                         int tile, void* stream);

/* ---- attention ---------------------------------------------------------------------------
 * Replaces flash_attn.flash_attn_varlen_func at diffusers_lite/wan/modules/attention.py:96-127
 * (called from model.py:188, :221, :262, :264) for head_dim 128, non-causal, no dropout.
 * q/k/v/o are [B][L][H*128] with row stride ld* and batch stride b*; keys >= k_len are masked
 * (the `k_lens=seq_lens` of model.py:191).  lse2 [B][H][Lq] = log2-domain log-sum-exp
 * (max*scale*log2e + log2(sum)), consumed by prfl_attn_bwd. */
int prfl_attn_fwd(const void* q, int64_t ldq, int64_t bq, const void* k, int64_t ldk, int64_t bk,
                  const void* v, int64_t ldv, int64_t bv, void* o, int64_t ldo, int64_t bo,
                  float* lse2, int64_t B, int64_t Lq, int64_t Lk, int64_t H, int64_t k_len,
                  float scale, void* stream);
/* The same with a caller-owned scratch buffer `ws` of prfl_attn_fwd_ws_bytes(B, Lq, Lk, H, k_len)
 * bytes (16-B aligned; null or smaller = prfl_attn_fwd): long-KV launches whose last dispatch
 * round would run only a few workgroups split those units' key tiles over several workgroups
 * and merge the partial softmax states (flash-decoding), so the final round fills the chip. */
int prfl_attn_fwd_ws(const void* q, int64_t ldq, int64_t bq, const void* k, int64_t ldk,
                     int64_t bk, const void* v, int64_t ldv, int64_t bv, void* o, int64_t ldo,
                     int64_t bo, float* lse2, int64_t B, int64_t Lq, int64_t Lk, int64_t H,
                     int64_t k_len, float scale, void* ws, int64_t ws_bytes, void* stream);
/* Scratch bytes prfl_attn_fwd_ws needs on the current device (0 = no split for this shape). */
int64_t prfl_attn_fwd_ws_bytes(int64_t B, int64_t Lq, int64_t Lk, int64_t H, int64_t k_len);
/* prfl_attn_fwd_ws with q in log2 units, q = q_orig * scale * log2(e) (the fused block's
 * RMSNorm+RoPE writes it so, prfl_rms_rope_fwd_scaled out_scale): the S accumulators start at the running
 * row max and P = exp2(S) takes one v_exp per score.  o / lse2 are those of
 * prfl_attn_fwd_ws(q_orig, ..., scale); same scratch. */
int prfl_attn_fwd_l2q_ws(const void* q, int64_t ldq, int64_t bq, const void* k, int64_t ldk,
                         int64_t bk, const void* v, int64_t ldv, int64_t bv, void* o, int64_t ldo,
                         int64_t bo, float* lse2, int64_t B, int64_t Lq, int64_t Lk, int64_t H,
                         int64_t k_len, void* ws, int64_t ws_bytes, void* stream);
/* V in the key-chunked transposed ("VT") layout of the long-KV self-attention forward: per
 * (sample, head) [Lkp/8][128][8] bf16, Lkp = Lk rounded up to 96, the 8 keys of chunk 2j + h
 * being 16j + 4h + {0,1,2,3,8,9,10,11}, zero past Lk.  Same reference interface as
 * prfl_attn_fwd_ws (flash_attn_varlen_func, `wan/modules/attention.py:96-127`); prfl_attn_v_to_vt
 * writes vt (prfl_attn_vt_bytes bytes, 16-B aligned) from v [B][Lk][H*128] (row stride ldv). */
int64_t prfl_attn_vt_bytes(int64_t B, int64_t Lk, int64_t H);
int prfl_attn_v_to_vt(const void* v, int64_t ldv, int64_t bv, void* vt, int64_t B, int64_t Lk,
                      int64_t H, void* stream);
/* prfl_attn_fwd_l2q_ws reading V from its VT image (Lk >= 4096 only, else hipErrorInvalidValue):
 * every V^T fragment is one ds_read_b128; o / lse2 bit-identical to prfl_attn_fwd_l2q_ws. */
int prfl_attn_fwd_l2q_vt_ws(const void* q, int64_t ldq, int64_t bq, const void* k, int64_t ldk,
                            int64_t bk, const void* vt, void* o, int64_t ldo, int64_t bo,
                            float* lse2, int64_t B, int64_t Lq, int64_t Lk, int64_t H,
                            int64_t k_len, void* ws, int64_t ws_bytes, void* stream);
/* Config C5 (fp8): the same forward on the block-scaled e4m3 MFMA.  q, k, v stay bf16 in the
 * layout above and are quantised inside the call (Q per token and head, K per head, V per head
 * and channel, V stored transposed) into the REQUIRED caller-owned scratch `ws` (256-B aligned)
 * of prfl_attn_fwd_fp8_ws_bytes(...) bytes; o and lse2 as prfl_attn_fwd_ws (lse2 is the LSE of
 * the dequantised scores, usable by prfl_attn_bwd).  There is no fp8 flash-attn in the
 * reference, which is bf16 throughout (attention.py:113-127; no fp8 anywhere).  Q.K^T runs on the
 * int8 MFMA, P.V on the e4m3 MFMA. */
int prfl_attn_fwd_fp8(const void* q, int64_t ldq, int64_t bq, const void* k, int64_t ldk,
                      int64_t bk, const void* v, int64_t ldv, int64_t bv, void* o, int64_t ldo,
                      int64_t bo, float* lse2, int64_t B, int64_t Lq, int64_t Lk, int64_t H,
                      int64_t k_len, float scale, void* ws, int64_t ws_bytes, void* stream);
int64_t prfl_attn_fwd_fp8_ws_bytes(int64_t B, int64_t Lq, int64_t Lk, int64_t H, int64_t k_len);
/* prfl_attn_fwd_fp8 with q in log2 units (as prfl_attn_fwd_l2q_ws). */
int prfl_attn_fwd_fp8_l2q(const void* q, int64_t ldq, int64_t bq, const void* k, int64_t ldk,
                          int64_t bk, const void* v, int64_t ldv, int64_t bv, void* o, int64_t ldo,
                          int64_t bo, float* lse2, int64_t B, int64_t Lq, int64_t Lk, int64_t H,
                          int64_t k_len, void* ws, int64_t ws_bytes, void* stream);
/* Backward of the above (flash-attn's _flash_attn_varlen_backward).  delta: [B][H][Lq] fp32
 * caller-owned workspace. */
int prfl_attn_bwd(const void* q, int64_t ldq, int64_t bq, const void* k, int64_t ldk, int64_t bk,
                  const void* v, int64_t ldv, int64_t bv, const void* o, int64_t ldo, int64_t bo,
                  const void* dout, int64_t lddo, int64_t bdo, const float* lse2, float* delta,
                  void* dq, int64_t lddq, int64_t bdq, void* dk, int64_t lddk, int64_t bdk,
                  void* dv, int64_t lddv, int64_t bdv, int64_t B, int64_t Lq, int64_t Lk,
                  int64_t H, int64_t k_len, float scale, void* stream);

/* The same with a caller-owned scratch buffer `ws` of prfl_attn_bwd_ws_bytes(B, Lq, Lk, H, k_len)
 * bytes (16-B aligned; null or smaller = prfl_attn_bwd): long-KV launches split the units of
 * their last, under-filled dispatch round (dK/dV over query tiles, dQ over key tiles) and sum
 * the unscaled fp32 partials. */
int prfl_attn_bwd_ws(const void* q, int64_t ldq, int64_t bq, const void* k, int64_t ldk,
                     int64_t bk, const void* v, int64_t ldv, int64_t bv, const void* o, int64_t ldo,
                     int64_t bo, const void* dout, int64_t lddo, int64_t bdo, const float* lse2,
                     float* delta, void* dq, int64_t lddq, int64_t bdq, void* dk, int64_t lddk,
                     int64_t bdk, void* dv, int64_t lddv, int64_t bdv, int64_t B, int64_t Lq,
                     int64_t Lk, int64_t H, int64_t k_len, float scale, void* ws,
                     int64_t ws_bytes, void* stream);
/* prfl_attn_bwd_l2q_ws with K also given in the VT layout (kt = prfl_attn_v_to_vt of k, the same
 * [B][Lk][H*128] tensor; Lk >= 4096 only): the dQ kernel reads its K^T fragments as one
 * ds_read_b128 each; outputs bit-identical to prfl_attn_bwd_l2q_ws.  Same reference interface
 * (flash_attn's varlen backward). */
int prfl_attn_bwd_l2q_kt_ws(const void* q, int64_t ldq, int64_t bq, const void* k, int64_t ldk,
                            int64_t bk, const void* kt, const void* v, int64_t ldv, int64_t bv,
                            const void* o, int64_t ldo, int64_t bo, const void* dout, int64_t lddo,
                            int64_t bdo, const float* lse2, float* delta, void* dq, int64_t lddq,
                            int64_t bdq, void* dk, int64_t lddk, int64_t bdk, void* dv,
                            int64_t lddv, int64_t bdv, int64_t B, int64_t Lq, int64_t Lk,
                            int64_t H, int64_t k_len, void* ws, int64_t ws_bytes, void* stream);
/* Scratch bytes prfl_attn_bwd_ws needs on the current device (0 = no split for this shape). */
int64_t prfl_attn_bwd_ws_bytes(int64_t B, int64_t Lq, int64_t Lk, int64_t H, int64_t k_len);
/* prfl_attn_bwd_ws for a q in log2 units (prfl_attn_fwd_l2q_ws): dq is the gradient w.r.t. that
 * pre-scaled q (ln 2 * dS.K; the RMSNorm+RoPE backward's out_scale multiplies it back), dk / dv
 * those of the unscaled problem; same scratch. */
int prfl_attn_bwd_l2q_ws(const void* q, int64_t ldq, int64_t bq, const void* k, int64_t ldk,
                         int64_t bk, const void* v, int64_t ldv, int64_t bv, const void* o,
                         int64_t ldo, int64_t bo, const void* dout, int64_t lddo, int64_t bdo,
                         const float* lse2, float* delta, void* dq, int64_t lddq, int64_t bdq,
                         void* dk, int64_t lddk, int64_t bdk, void* dv, int64_t lddv, int64_t bdv,
                         int64_t B, int64_t Lq, int64_t Lk, int64_t H, int64_t k_len, void* ws,
                         int64_t ws_bytes, void* stream);

/* ---- single-query attention pooling (reward head) ----------------------------------------
 * Replaces the core of the 1-query nn.MultiheadAttention of QueryAttention
 * (diffusers_lite/utils/network.py:80; num_queries 1, 8 heads, E = 5120): per sample n and head
 * h, o[n][h*hd:(h+1)*hd] = softmax_l(q_h . k_{l,h} * scale) V_{l,h}, hd = E / H (hd % 8 == 0,
 * hd <= 1024).  q [N][ldq] bf16; kv [N][L][ldkv] bf16 with K in columns [0, E) and V in
 * [E, 2E) (the in-projection output), sample stride bkv.  o32 (optional, [N][E] fp32) receives
 * the output before its bf16 rounding (the backward's D).  Split over L into nsplit parts
 * (prfl_query_pool_splits gives the default); part_m / part_l [N*H*nsplit] and part_o
 * [N*H*nsplit*hd] fp32 are caller-owned workspace.  lse2 [N][H] = log2-domain LSE. */
int prfl_query_pool_splits(int64_t N, int64_t L, int64_t H);
int prfl_query_pool_fwd(const void* q, int64_t ldq, const void* kv, int64_t ldkv, int64_t bkv,
                        int64_t N, int64_t L, int64_t H, int64_t E, float scale, void* o,
                        int64_t ldo, float* lse2, float* o32, float* part_m, float* part_l,
                        float* part_o, int64_t nsplit, void* stream);
/* Backward: dq fp32 [N][lddq] (= scale * sum_l ds k), dkv bf16 [N][L][lddkv] (dK | dV, every
 * row written), part_o [N*H*nsplit*hd] workspace; dout bf16 [N][ldq]; o32 = the forward's fp32
 * output [N][E] (D = rowsum(dout * o32)). */
int prfl_query_pool_bwd(const void* dout, const void* q, int64_t ldq, const void* kv,
                        int64_t ldkv, int64_t bkv, const float* o32, const float* lse2, int64_t N,
                        int64_t L, int64_t H, int64_t E, float scale, float* dq, int64_t lddq,
                        void* dkv, int64_t lddkv, int64_t bdkv, float* part_o, int64_t nsplit,
                        void* stream);

/* ---- normalisation ----------------------------------------------------------------------
 * WanLayerNorm + AdaLN modulation (model.py:125-135, :345, :353):
 *   out = bf16(LN(x) * (1 + scale) + shift)     (w == NULL; LN rounded to bf16 if x_bf16)
 * or the affine norm3 (model.py:304-306, :352):  out = bf16(LN(x) * w + b).
 * x is fp32 or bf16 [L][ldx]; mean/rstd [L] fp32 are saved for the backward.  C <= 5120. */
int prfl_ln_mod_fwd(const void* x, int x_bf16, int64_t ldx, int64_t L, int64_t C,
                    const float* scale, const float* shift, const float* w, const float* b,
                    float eps, void* out, int64_t ldo, float* mean, float* rstd, void* stream);
/* dx (+)= LN backward of dy (bf16); part0/part1 [ceil(L/prfl_norm_rows_per_part())][C] receive
 * partial column sums of dy*xhat (d scale | d w) and dy (d shift | d b). */
int prfl_ln_mod_bwd(const void* dy, int64_t lddy, const void* x, int x_bf16, int64_t ldx,
                    const float* mean, const float* rstd, int64_t L, int64_t C,
                    const float* scale, const float* w, float* dx, int64_t lddx,
                    int dx_accumulate, float* part0, float* part1, void* stream);
int prfl_norm_rows_per_part(void);

/* WanRMSNorm (model.py:106-122) over all C channels + optional 3-D RoPE (rope_apply,
 * model.py:61-103; rope_tab = fp32 (cos,sin) [1024][64] of the complex freqs of model.py:521-526,
 * grid (F,Hg,Wg); rows >= F*Hg*Wg are not rotated; rope_tab == NULL -> no RoPE).
 *   out = bf16(rope(bf16(x * rsqrt(mean(x^2)+eps)) * w) * out_scale)
 * out_scale 1 is the reference's norm_q / norm_k; softmax_scale * log2(e) yields the q operand of
 * the *_l2q attention entries; the backward scales the incoming gradient by out_scale.
 * There is deliberately no unsuffixed prfl_rms_rope_fwd / _bwd: that name carried two different
 * signatures (round 2 without out_scale, round 3 with it), and a float argument dropped from a
 * SysV signature still links, so a stale caller would run with the wrong scale.  Removing the
 * name (round 5) makes such a caller fail to resolve instead (ABI history). */
int prfl_rms_rope_fwd_scaled(const void* x, int64_t ldx, int64_t L, int64_t C, const float* w,
                             float eps, const float* rope_tab, int64_t F, int64_t Hg, int64_t Wg,
                             void* out, int64_t ldo, float* rstd, float out_scale, void* stream);
int prfl_rms_rope_bwd_scaled(const void* dout, int64_t lddo, const void* x, int64_t ldx,
                             const float* rstd, int64_t L, int64_t C, const float* w,
                             const float* rope_tab, int64_t F, int64_t Hg, int64_t Wg, void* dx,
                             int64_t lddx, float* part0, float out_scale, void* stream);
/* The same two with the rows' sequence positions starting at row0 instead of 0: row r of x is
 * token row0 + r of the (F,Hg,Wg) grid, positions >= F*Hg*Wg pass unrotated.  This is the
 * sequence-parallel rope_apply of model.py:89-96 (a rank of an SP group holds tokens
 * [rank * s, (rank + 1) * s) of the padded sequence and rotates them by those positions'
 * frequencies, pad_freqs' unit multipliers past the grid).  The _scaled entries are row0 = 0. */
int prfl_rms_rope_fwd_pos(const void* x, int64_t ldx, int64_t L, int64_t C, const float* w,
                          float eps, const float* rope_tab, int64_t F, int64_t Hg, int64_t Wg,
                          int64_t row0, void* out, int64_t ldo, float* rstd, float out_scale,
                          void* stream);
int prfl_rms_rope_bwd_pos(const void* dout, int64_t lddo, const void* x, int64_t ldx,
                          const float* rstd, int64_t L, int64_t C, const float* w,
                          const float* rope_tab, int64_t F, int64_t Hg, int64_t Wg, int64_t row0,
                          void* dx, int64_t lddx, float* part0, float out_scale, void* stream);

/* ---- element-wise / reductions ------------------------------------------------------------ */
/* autocast weight cast fp32 -> bf16 (the .to(bf16) of every Linear weight under autocast). */
int prfl_cast_f32_bf16(const float* src, void* dst, int64_t n, void* stream);
/* The same cast into the transposed layout: out[k * ldo + n] = bf16(w[n * ldw + k]) for an fp32
 * nn.Linear weight w [N][K] — the forward projection's weight as an MN-major prfl_gemm_bf16
 * operand (b_kmajor = 0, ldb = ldo), bit-identical results to the K-major form.  ldw % 4,
 * ldo % 8 == 0, 16-B aligned pointers. */
int prfl_cast_f32_bf16_t(const float* w, int64_t N, int64_t K, int64_t ldw, void* out, int64_t ldo,
                         void* stream);
/* backward of the gated residual x + y*gate (model.py:348, :355): dy = bf16(dx*gate);
 * partial column sums of dx*y (-> d gate) and of dy (-> d bias of the producing Linear). */
int prfl_gate_bwd(const float* dx, int64_t lddx, const void* y, int64_t ldy, const float* gate,
                  int64_t L, int64_t N, void* dy, int64_t lddy, float* pgate, float* pbias,
                  void* stream);
int prfl_colsum_bf16(const void* x, int64_t ld, int64_t L, int64_t N, float* part, void* stream);
int prfl_colsum_reduce(const float* part, int64_t P, int64_t N, float* out, int accumulate,
                       void* stream);
int prfl_colsum_rows_per_part(void);
/* grad-norm clipping pieces of transformer.clip_grad_norm_ (train_prfl.py:825, :972) */
int prfl_sumsq(const float* x, int64_t n, float* out, void* stream);
int prfl_scale(float* x, int64_t n, const float* factor, void* stream);
/* torch.optim.AdamW step (train_prfl.py:485-491, :827-830) on one fp32 tensor. */
int prfl_adamw(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
               float beta2, float eps, float weight_decay, int64_t step, void* stream);
/* prfl_adamw + optimizer.zero_grad() in the same pass (train_prfl.py:827-830): g is set to 0
 * after it is read, so the gradient buffer stays allocated for the next accumulation. */
int prfl_adamw_zero_grad(float* p, float* g, float* m, float* v, int64_t n, float lr, float beta1,
                         float beta2, float eps, float weight_decay, int64_t step, void* stream);

/* ---- fp8 path (config C5, train_prfl_i2v_720 "fp8 MFMA path"; SURVEY §8c tolerance 5e-2 vs
 * the bf16 path).  The reference itself is bf16-only; these replace the same autocast
 * nn.Linear forwards as prfl_gemm_bf16 when the fp8 path is enabled.
 * prfl_quant_rows_fp8: per-row OCP e4m3 quantisation of x [M][K] (bf16, or fp32 if x_f32):
 *   scale[m] = amax_m / 448, q[m][k] = e4m3(x[m][k] * 448 / amax_m)   (K % 8 == 0, K <= 16384)
 * prfl_gemm_fp8: C = sa[m] * sb[n] * sum_k A(m,k) B(n,k) with A [M][K], B [N][K] e4m3 K-major,
 *   block-scaled MFMA (unit block scales), epilogue 0/1/2 as prfl_gemm_bf16 (bias bf16 [N]);
 *   K % 128 == 0, lda/ldb % 16 == 0, 16-B aligned A/B/sb. */
int prfl_quant_rows_fp8(const void* x, int x_f32, int64_t ldx, int64_t M, int64_t K, void* q,
                        int64_t ldq, float* scale, void* stream);
int prfl_gemm_fp8(const void* A, int64_t lda, const float* sa, const void* B, int64_t ldb,
                  const float* sb, void* C, int64_t ldc, int64_t M, int64_t N, int64_t K,
                  int epilogue, const void* bias, const float* gate, const void* res, int64_t ldr,
                  int res_bf16, void* aux, int64_t ldaux, void* stream);

/* ---- FlowUniPC sampler update (bh2, order <= 2, x0-prediction) ----------------------------
 * Replaces the element-wise body of FlowUniPCMultistepScheduler.step
 * (diffusers_lite/wan/utils/fm_solvers_unipc.py:655-739: convert_model_output :321, UniC
 * corrector :486-626, UniP predictor :350-484), called from train_prfl.py:693 (no-grad rollout)
 * and :734 (the differentiable step the reward gradient flows through).
 * sample / last_sample / sample_c / prev are bf16, model_output / hist1 (= model_outputs[-1]) /
 * hist2 (= model_outputs[-2]) / m_t are fp32, all n contiguous elements.
 * coef[11] (host) = {sigma_i, corrector: sig_t/sig_s0, alpha_t*h_phi_1, rk, rho0, rho_last,
 *                    alpha_t*B_h, predictor: sig_t/sig_s0, alpha_t*h_phi_1, rk, alpha_t*B_h}
 * rho0/rho_last are rounded to bf16 on entry (the reference casts the solved rhos, :612).
 * corr_order 0 = no corrector (then last_sample/hist2 may be NULL, sample_c optional).
 * Bit-identical to the reference's torch chain (fp32 ops in its order, no FMA contraction). */
int prfl_unipc_step(const void* sample, const float* model_output, const void* last_sample,
                    const float* hist1, const float* hist2, float* m_t, void* sample_c,
                    void* prev, int64_t n, const float* coef, int corr_order, int pred_order,
                    void* stream);
/* d prev (bf16) -> d model_output (fp32): the transpose of the map above as torch autograd
 * evaluates it (model_output is the only differentiable input, as in train_prfl.py:734). */
int prfl_unipc_step_bwd(const void* grad_prev, float* grad_model_output, int64_t n,
                        const float* coef, int corr_order, int pred_order, void* stream);

/* ---- profiling (bench.py roofline) -------------------------------------------------------- */
int prfl_prof_enable(int on);
int prfl_prof_collect(int64_t* counts, double* ms, double* work, int nkid);
/* effective shader clock (MHz: launch-time-weighted mean, min, max; n = launches) of the
 * self-attention forwards since the last call, from s_memtime / s_memrealtime in workgroup 0 */
int prfl_prof_clock(double* mean_mhz, double* min_mhz, double* max_mhz, int64_t* n);

#ifdef __cplusplus
}
#endif
#endif /* PRFL_HIP_H */
