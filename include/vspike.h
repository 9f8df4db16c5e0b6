/*
 * vspike.h — C-ABI of the MI355X-native video->spike training hot path (libvspike.so).
 *
 * Plain pointers and sizes only: no torch, no HIP types in the signatures.  Every entry point
 * enqueues work on the caller's HIP stream (`stream` is a hipStream_t, NULL = legacy default
 * stream), never allocates, never synchronises, and is therefore hipGraph-capturable.  Device
 * buffers are owned by the caller (the PyTorch caching allocator on the Python side).
 *
 * Return value: VS_OK (0) on success, VS_EINVAL (-1) for a rejected argument (shape, dtype,
 * alignment, null pointer — nothing was launched), or a positive hipError_t from the launch.
 * `vs_last_error()` returns a static string describing the last rejection.
 *
 * The reference (PPWangyc/video-spike) is pure Python; every op here replaces a torch/cuBLAS/
 * cuDNN kernel that its hot path runs.  Each declaration cites the reference line it replaces
 * (paths relative to the reference repo root; "mv" = src/model/videomae/modeling_videomae.py,
 * the vendored spec of the HF encoder the reference executes).
 */
#ifndef VSPIKE_H
#define VSPIKE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VS_OK 0
#define VS_EINVAL (-1)

/* element types */
#define VS_F32 0
#define VS_BF16 1
#define VS_U8 2   /* raw video frames only (vs_video_preprocess) */
#define VS_FP8 3  /* OCP e4m3 with MX (E8M0 per 32 k) scales: vs_gemm_mxfp8 operands; as vs_vit_layer.dtype:
                     bf16 everywhere + MX-FP8 forward block products (BASELINE C5) */

int vs_version(void);                 /* ABI version (monotonic) */
/* sha256 prefix (16 hex digits) of the sources this library was compiled from: every csrc/ file
 * and this header, hashed by vspike/build.py (source_hash) and baked into the build, so a test or
 * bench can prove which sources the loaded binary was built from */
const char* vs_build_id(void);
const char* vs_last_error(void);      /* static string, last VS_EINVAL reason */
int vs_device_arch(char* buf, int n); /* writes gcnArchName of the current device */
/* sizeof() of the ABI structs, so bindings can verify their mirrors: 0 = vs_gemm_desc,
 * 1 = vs_vit_layer, 2 = vs_vit_layer_grad, 3 = vs_conv3d_desc; -1 for an unknown id */
int vs_struct_size(int which);

/* ------------------------------------------------------------------------------------------
 * GEMM with fused epilogue:  C[M,N] = epilogue( alpha * sum_k A(m,k) * B(k,n) )
 * Replaces every nn.Linear / F.linear on the path and its autograd backward:
 *   mv:233-236 (Q,K,V projections), mv:312-319 (attention output dense), mv:373-383 (fc1+GELU),
 *   mv:390-397 (fc2 + residual), mv:176-181/194-195 (Conv3d patch-embed as im2col GEMM, + the
 *   sinusoid table mv:135 via VS_EPI_POS), src/model/videomae.py:13-14,28-31 (head Linears),
 *   src/model/linear.py:24-32,45-53 (Linear plugin MLP + ReLU), and their dX/dW products
 *   (accelerator.backward, src/trainer/base.py:150).
 * Operand layouts:
 *   a_kcontig=1: A(m,k) = a[m*lda + k]        a_kcontig=0: A(m,k) = a[k*lda + m]
 *   b_kcontig=1: B(k,n) = b[n*ldb + k]  (nn.Linear weight [N,K])   b_kcontig=0: B(k,n) = b[k*ldb + n]
 * Operands are VS_F32 (exact f32 MFMA 16x16x4) or VS_BF16 (MFMA 16x16x32, f32 accumulate).
 * Contiguous extents and leading dims must be multiples of 8 (bf16) / 4 (f32) elements and
 * base pointers 16-byte aligned.
 * ------------------------------------------------------------------------------------------ */
#define VS_EPI_BIAS      0x001u  /* + bias[n] (f32)                                            */
#define VS_EPI_GELU      0x002u  /* aux_out(m,n) = v (pre-activation); v = gelu_erf(v)          */
#define VS_EPI_RELU      0x004u  /* v = max(v, 0)                                              */
#define VS_EPI_RESIDUAL  0x008u  /* + residual[m*ld_residual + n] (f32)                        */
#define VS_EPI_POS       0x010u  /* + pos[(m % pos_rows)*N + n] (f32)                          */
#define VS_EPI_GELU_BWD  0x020u  /* v *= gelu_erf'(aux_in(m,n))                                */
#define VS_EPI_RELU_BWD  0x040u  /* v = aux_in(m,n) > 0 ? v : 0                                */
#define VS_EPI_ATOMIC    0x080u  /* C(m,n) += v (split-K); C must be f32.  With a workspace the  */
                                 /* splits are summed in a fixed order (no atomics); with RELU  */
                                 /* (skinny path only) C = relu(C + v)                          */
#define VS_EPI_ACCUM     0x100u  /* C(m,n) += v (plain read-modify-write); C must be f32      */
#define VS_EPI_GELU_GRAD 0x200u  /* with VS_EPI_GELU: aux_out(m,n) = gelu'(v) instead of v: the  */
                                 /* factor the backward multiplies by (bf16 ViT path: the fc1    */
                                 /* forward stores it, the GELU' dX product uses VS_EPI_MUL_AUX)  */
#define VS_EPI_MUL_AUX   0x400u  /* v *= aux_in(m,n)                                            */

typedef struct vs_gemm_desc {
  int32_t dtype;        /* operand element type, VS_F32 or VS_BF16 */
  int32_t out_dtype;    /* C element type */
  int32_t a_kcontig;
  int32_t b_kcontig;
  int64_t M, N, K;
  const void* a;   int64_t lda;
  const void* b;   int64_t ldb;
  void* c;         int64_t ldc;
  uint32_t epilogue;    /* VS_EPI_* bits */
  float alpha;
  const float* bias;                          /* [N] */
  const float* residual; int64_t ld_residual; /* [M, ld] f32 */
  const float* pos;      int64_t pos_rows;    /* [pos_rows, N] f32 */
  const void* aux_in;    int64_t ld_aux_in;   /* operand dtype */
  void* aux_out;         int64_t ld_aux_out;  /* operand dtype */
  int32_t split_k;      /* 0 = auto; >1 needs VS_EPI_ATOMIC */
  int32_t reserved;
  float* a_rowsum;      /* optional [M] f32: += sum_k A(m,k) (the bias gradient of a dW = dY^T X
                           product, fused: replaces a separate column-sum pass over dY) */
  void* workspace;      /* optional, VS_EPI_ATOMIC split-K only: each split stores its f32 tile   */
  int64_t workspace_bytes; /* here and a second launch adds the splits into C (instead of f32
                              atomics); splits are capped to what fits; NULL/0 keeps atomics */
} vs_gemm_desc;

int vs_gemm(const vs_gemm_desc* d, void* stream);
/* bytes of split-K workspace the automatic split of an ATOMIC GEMM of this shape would use */
size_t vs_gemm_splitk_workspace_bytes(int32_t dtype, int64_t M, int64_t N, int64_t K);

/* ------------------------------------------------------------------------------------------
 * LayerNorm over the last dim, eps = 1e-12 in the reference (mv:416-417, nn.LayerNorm).
 * x is the f32 residual stream; y is written in `y_dtype`; mean/rstd [rows] f32 are saved for
 * the backward.  Backward: dx = dres + LN'(dy); dgamma/dbeta are ACCUMULATED (f32 atomics).
 * dx_lp (optional) receives a bf16 copy of dx for the next bf16 GEMM.
 * ------------------------------------------------------------------------------------------ */
int vs_layernorm_fwd(int32_t y_dtype, int64_t rows, int64_t cols, const float* x, int64_t ldx,
                     const float* gamma, const float* beta, float eps, void* y, int64_t ldy,
                     float* mean, float* rstd, void* stream);
/* workspace (optional, >= vs_layernorm_bwd_workspace_bytes): dgamma/dbeta partial rows per
 * block, summed by a second launch; NULL falls back to one f32 atomic per column per block. */
size_t vs_layernorm_bwd_workspace_bytes(int64_t rows, int64_t cols);
int vs_layernorm_bwd(int64_t rows, int64_t cols, const float* dy, int64_t lddy, const float* x,
                     int64_t ldx, const float* mean, const float* rstd, const float* gamma,
                     const float* dres, int64_t lddres, float* dx, int64_t lddx, void* dx_lp,
                     float* dgamma, float* dbeta, void* workspace, void* stream);
/* The same with a bf16 incoming gradient (dy_dtype VS_BF16, 8-B aligned rows; VS_F32 = the call
 * above): the bf16 ViT block writes its dX products dh1 / dh2 in bf16 and normalises from them. */
int vs_layernorm_bwd_dt(int32_t dy_dtype, int64_t rows, int64_t cols, const void* dy, int64_t lddy,
                        const float* x, int64_t ldx, const float* mean, const float* rstd, const float* gamma,
                        const float* dres, int64_t lddres, float* dx, int64_t lddx, void* dx_lp, float* dgamma,
                        float* dbeta, void* workspace, void* stream);
/* The dX product of a Linear fed straight into the backward of the LayerNorm before it (the ViT
 * block's dh2 = da W1 -> LN2' and dh1 = dqkv Wqkv -> LN1', mv:416-417 + mv:373-383 / mv:233-236):
 *   dh = A B (d: the GEMM, epilogue 0, d->c = an [M, N] f32 scratch used only off the fused path);
 *   dx = dres + LN'(dh; x, mean, rstd, gamma);  dx_lp = bf16(dx) (optional);
 *   dgamma, dbeta += the LN weight gradients (fixed-order partial rows through `workspace`, sized by
 *   vs_layernorm_bwd_workspace_bytes).
 * bf16 with N in {64, 128, 192} and M >= 8192 runs fused (dh never leaves the chip); otherwise it is
 * vs_gemm into d->c followed by vs_layernorm_bwd. */
/* y = A W^T (+ bias) + residual (d: bf16 operands, out f32 = y, epilogue RESIDUAL [| BIAS]) and
 * h = LayerNorm(y; gamma, beta, eps) in bf16 with its row mean / rstd, in ONE launch when the
 * shape allows (the ViT block's proj product + LN2, N = 192: the row-slab kernel owns whole rows),
 * else vs_gemm + vs_layernorm_fwd.  Replaces modeling_videomae.py:434-437 (attention output +
 * residual, layernorm_after). */
int vs_gemm_ln_fwd(const vs_gemm_desc* d, const float* gamma, const float* beta, float eps, void* h, int64_t ldh,
                   float* mean, float* rstd, void* stream);
int vs_gemm_ln_bwd(const vs_gemm_desc* d, const float* x, int64_t ldx, const float* mean, const float* rstd,
                   const float* gamma, const float* dres, int64_t lddres, float* dx, int64_t lddx, void* dx_lp,
                   float* dgamma, float* dbeta, void* workspace, void* stream);

/* The ViT block's whole MLP in one launch (mv:370-399: VideoMAEIntermediate dense + GELU(erf),
 * VideoMAEOutput dense + residual), bf16 operands, f32 accumulation and residual stream:
 *   x_out = y + gelu(h2 W1^T + b1) W2^T + b2,   h2 [M, D] bf16, W1 [F, D] bf16, W2 [D, F] bf16,
 *   y / x_out [M, D] f32.  The [M, F] intermediate never reaches HBM.
 * vs_mlp_bwd_da: its backward's GELU' product with the pre-activation RECOMPUTED from h2 (the same
 *   MFMA chain as the forward):  da = (dy W2) * gelu'(h2 W1^T + b1)  and  a = gelu(h2 W1^T + b1),
 *   dy [M, D] bf16 (dx' of the block), da / a [M, F] bf16 (the operands of dh2 = da W1, dW1 = da^T h2,
 *   dW2 = dy^T a).  GELU: x * sigmoid(x (k1 + k3 x^2 + k5 x^4)), a minimax fit of x Phi(x) with
 *   |error| <= 2.5e-5 (derivative <= 1.1e-4), below the bf16 rounding (2^-9 relative) every stored
 *   value gets; the unfused bf16 path (VSPIKE_MLP_FUSE=0) uses the A&S 7.1.26 erf (<= 1.5e-7), so the
 *   A/B switch changes the GELU's last bits as well as the kernels.
 * Both need vs_mlp_fused_ok(M, D, F): D = 192 (ViT-Tiny), F % 64 == 0, F <= 3072. */
/* ------------------------------------------------------------------------------------------
 * MX-FP8 (BASELINE C5 "fp8 MFMA"): OCP e4m3 elements with one E8M0 power-of-two scale per 32
 * consecutive k (scale = 2^(e - 127), e = 127 + ceil(log2(amax / 448)) over the block: nothing
 * saturates).  vs_quant_mxfp8: x [M, K] (f32 or bf16) -> q [M, K] e4m3 bytes + scales [M, K / 32]
 * bytes.  vs_gemm_mxfp8: the Linear forward of the ViT block on v_mfma_scale_f32_32x32x64_f8f6f4,
 * C = A B^T with A [M, K] and B [N, K] (nn.Linear layout) both VS_FP8, scales as vs_quant_mxfp8
 * writes them, then vs_gemm's epilogue (0, BIAS, BIAS|RESIDUAL or BIAS|GELU|GELU_GRAD); K % 128 == 0,
 * N % 128 == 0.  Replaces the fp32 nn.Linear forwards mv:233-236, 312-319, 373-383, 390-397 at C5.
 * ------------------------------------------------------------------------------------------ */
int vs_quant_mxfp8(int32_t in_dtype, int64_t M, int64_t K, const void* x, int64_t ldx, void* q, int64_t ldq,
                   void* scales, int64_t ld_scales, void* stream);
int vs_gemm_mxfp8(const vs_gemm_desc* d, const void* scale_a, int64_t ld_scale_a, const void* scale_b,
                  int64_t ld_scale_b, void* stream);

int vs_mlp_fused_ok(int64_t M, int64_t D, int64_t F);
int vs_mlp_fwd(int64_t M, int64_t D, int64_t F, const void* h2, int64_t ldh, const void* w1, const float* b1,
               const void* w2, const float* b2, const float* y, int64_t ldy, float* x_out, int64_t ldx, void* stream);
/* vs_mlp_fwd plus the next block's LayerNorm1 on x_out in the epilogue (eps; h_out bf16 [M, D], row
 * mean / rstd): mv:419-445's layernorm_before of block i+1 fused into block i's output (D = 192). */
int vs_mlp_fwd_ln(int64_t M, int64_t D, int64_t F, const void* h2, int64_t ldh, const void* w1, const float* b1,
                  const void* w2, const float* b2, const float* y, int64_t ldy, float* x_out, int64_t ldx,
                  const float* ln_g, const float* ln_b, float eps, void* h_out, int64_t ld_h_out, float* mean_out,
                  float* rstd_out, void* stream);
int vs_mlp_bwd_da(int64_t M, int64_t D, int64_t F, const void* h2, int64_t ldh, const void* w1, const float* b1,
                  const void* w2, const void* dy, int64_t lddy, void* da, int64_t ldda, void* a, int64_t lda,
                  void* stream);

/* ------------------------------------------------------------------------------------------
 * Non-causal multi-head attention, head dim 64 (mv:243-258; SDPA variant mv:286-294):
 *   O = softmax(Q K^T * scale) V per (batch, head), scale = 1/sqrt(64) = 0.125.
 * qkv: [B*N, 3*H*64] rows; Q of head h at column h*64, K at (H+h)*64, V at (2H+h)*64.
 * o: [B*N, H*64]; lse: [B, H, N] f32 natural-log sum-exp of the scaled scores (saved for bwd).
 * Backward writes dQ, dK, dV into dqkv (same layout as qkv); workspace is f32 scratch of
 * vs_attn_bwd_workspace_bytes().  dtype VS_BF16 runs the MFMA flash kernels; VS_F32 runs exact
 * f32 reference-grade kernels (the 1e-4 parity mode).
 * ------------------------------------------------------------------------------------------ */
int vs_attn_fwd(int32_t dtype, int64_t B, int64_t N, int64_t H, int64_t Dh, const void* qkv,
                int64_t ld_qkv, void* o, int64_t ld_o, float* lse, float scale, void* stream);
/* The bf16 forward's fast pass uses no running row maximum: exact while every query's row sum of
 * exp2(scores) stays within [2^-100, 2^96]; a workgroup with a query outside re-runs its tile under the
 * safe online softmax.  vs_attn_redo_count: workgroups that re-ran since the last reset (device-wide,
 * synchronising; reset != 0 zeroes the counter). */
int vs_attn_redo_count(int64_t* out, int32_t reset);
size_t vs_attn_bwd_workspace_bytes(int64_t B, int64_t N, int64_t H, int64_t Dh);
int vs_attn_bwd(int32_t dtype, int64_t B, int64_t N, int64_t H, int64_t Dh, const void* qkv,
                int64_t ld_qkv, const void* o, int64_t ld_o, const void* dout, int64_t ld_do,
                const float* lse, void* dqkv, int64_t ld_dqkv, void* workspace, float scale,
                void* stream);

/* ------------------------------------------------------------------------------------------
 * On-device video preprocessing, the VideoMAE plugin's forward prologue (videomae.py:18-25):
 * frame gather video[:, frame_idx] -> gray repeated to 3 channels -> the HF image processor's
 * resize (shortest edge -> out_size, PIL BILINEAR on uint8 frames, reproduced bit-exactly:
 * 22-bit fixed-point weights, horizontal then vertical pass through a uint8 intermediate) ->
 * centre crop out_size (a no-op for square frames) -> rescale 1/255 -> (x - mean[c]) / std[c].
 * video: (B, T, 1, H, W) contiguous, `in_dtype` VS_F32 (integer-valued 0..255, truncated like
 * numpy astype(uint8)) or VS_U8; H == W, H <= 7 * out_size.  frame_idx: HOST array of n_frames
 * (<= 64) source frame indices.  mean/std: HOST float[3].  out: (B, n_frames, 3, S, S) f32.
 * ------------------------------------------------------------------------------------------ */
int vs_video_preprocess(int32_t in_dtype, int64_t B, int64_t T, int64_t H, int64_t W, const void* video,
                        const int32_t* frame_idx, int32_t n_frames, int64_t out_size, const float* mean,
                        const float* std, float* out, void* stream);

/* ------------------------------------------------------------------------------------------
 * Tubelet patch gather (im2col) for the Conv3d patch embedding (mv:176-181, 194-195):
 * pixels (B, F, C, H, W) f32 -> cols [B*N, C*t*p*p] in `out_dtype`; token n = (f', hp, wp),
 * column = (c, t, i, j) = the Conv3d weight's flatten order.
 * ------------------------------------------------------------------------------------------ */
int vs_patch_im2col(int32_t out_dtype, int64_t B, int64_t F, int64_t C, int64_t H, int64_t W,
                    int64_t tubelet, int64_t patch, const float* pixels, void* cols, void* stream);

/* Patch embedding with the tubelet gather fused into the GEMM's operand load (mv:176-181, 194-195,
 * + bias + the sinusoid table mv:135 in the epilogue): out[m, d] = sum_k X[m, k] W[d, k] + bias[d] +
 * pos[m % n_tok, d], X[m, k] = pixels[b, 2 f' + t, c, 16 hp + i, 16 wp + j] for token m = (b, f', hp, wp)
 * and k = (c, t, i, j) — the Conv3d weight's flatten order; no im2col tensor.  The f32 NCHW pixels
 * are read once, coalesced along image rows, converted to bf16 in registers and staged in LDS.
 * weight: [D, C*2*16*16] bf16; out: [B*n_tok, D] f32; cols (optional, [B*n_tok, C*512] bf16): the
 * gathered rows as a side output (the weight gradient's operand, written only when given).
 * Fused path: tubelet 2, patch 16, D in {64, 128, 192}. */
int vs_patch_embed_fwd(int64_t B, int64_t F, int64_t C, int64_t H, int64_t W, int64_t tubelet, int64_t patch,
                       const float* pixels, const void* weight, const float* bias, const float* pos, int64_t D,
                       float* out, void* cols, void* stream);

/* The patch embedding's weight gradient without the im2col tensor (mv:176-181; replaces
 * vs_patch_im2col + the dW = dx^T cols product of vs_gemm): dweight[d, k] (+)= sum_m dx[m, d] X[m, k],
 * dbias[d] (+)= sum_m dx[m, d] (dbias may be NULL), X the tubelet gather of vs_patch_embed_fwd read
 * straight from the f32 pixels and rounded to bf16 as vs_patch_im2col rounds it.  dx: [B*n_tok, lddx]
 * bf16, D a multiple of 64; dweight: [D, ldw] f32 (k < C*512).  The token reduction is split and the
 * splits are added in a fixed order through `workspace` (>= vs_patch_embed_dw_workspace_bytes):
 * bitwise equal to im2col + vs_gemm's dW product.  Tubelet 2, patch 16, < 2^24 tokens. */
size_t vs_patch_embed_dw_workspace_bytes(int64_t tokens, int64_t D, int64_t K);
int vs_patch_embed_dw(int64_t B, int64_t F, int64_t C, int64_t H, int64_t W, int64_t tubelet, int64_t patch,
                      const float* pixels, const void* dx, int64_t lddx, int64_t D, float* dweight, int64_t ldw,
                      float* dbias, void* workspace, int64_t workspace_bytes, void* stream);

/* Fixed sinusoid position table (mv:101-112), f32 [n_pos, dim] (computed in f64, rounded). */
int vs_sinusoid_table(int64_t n_pos, int64_t dim, float* out, void* stream);

/* out[c] += sum_r x[r*ldx + c] for c < cols (bias gradients); x in `dtype`. */
int vs_colsum(int32_t dtype, int64_t rows, int64_t cols, const void* x, int64_t ldx, float* out,
              void* stream);

/* element-wise cast between VS_F32 and VS_BF16 (round to nearest even) */
int vs_cast(int32_t in_dtype, int32_t out_dtype, int64_t n, const void* in, void* out, void* stream);

/* ------------------------------------------------------------------------------------------
 * Fused PoissonNLLLoss(log_input=True) + mean + gradient (src/train.py:59,
 * src/trainer/base.py:141-143):  loss = mean(exp(x) - y*x);  dx = grad_scale*(exp(x) - y)/n.
 * loss_out: one f32 (deterministic two-stage reduction).  dx may be NULL (forward only).
 * workspace: >= vs_poisson_workspace_bytes(n).
 * ------------------------------------------------------------------------------------------ */
size_t vs_poisson_workspace_bytes(int64_t n);
int vs_poisson_nll(int64_t n, const float* log_rate, const float* target, float* loss_out,
                   float* dx, float grad_scale, void* workspace, void* stream);
/* dx = g[0] * (exp(x) - y) / n with the upstream scalar gradient read from device memory */
int vs_poisson_nll_bwd(int64_t n, const float* log_rate, const float* target,
                       const float* grad_out, float* dx, void* stream);
/* The MSE regression head option (train config `loss: mse`; BASELINE north_star "Poisson/MSE
 * spike-count regression head"), torch.nn.MSELoss(reduction="mean") semantics:
 *   loss = mean((x - y)^2);  dx = grad_scale * 2 (x - y) / n.
 * The reference trains with PoissonNLL only (src/train.py:59) and computes mse as an eval metric
 * (src/utils/utils.py:169-171); same workspace size and determinism as vs_poisson_nll. */
int vs_mse_loss(int64_t n, const float* pred, const float* target, float* loss_out, float* dx,
                float grad_scale, void* workspace, void* stream);
int vs_mse_loss_bwd(int64_t n, const float* pred, const float* target, const float* grad_out, float* dx,
                    void* stream);

/* ------------------------------------------------------------------------------------------
 * Fused AdamW step (torch.optim.AdamW semantics, src/train.py:44-49) over a flat f32 buffer.
 * hyper (device f32[8]): lr, beta1, beta2, eps, weight_decay, step (>=1), grad_scale, unused.
 * param_lp (optional): bf16 shadow of param written in the same pass.
 * ------------------------------------------------------------------------------------------ */
int vs_adamw(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
             void* param_lp, const float* hyper, void* stream);

/* ------------------------------------------------------------------------------------------
 * Evaluation metrics of one session (src/trainer/base.py:180-198 -> src/utils/utils.py:122-175
 * -> src/utils/metric_utils.py:36-102): gt, pred are the concatenated eval tensors
 * [trials, T, N] f32 BEFORE base.py's transposes; log_input = 1 applies base.py:186's exp.
 * bps over neurons 0..n_eval-1 (the reference indexes neurons with its trial loop: pass
 * n_eval = trials, after checking trials <= N), NaN spikes masked, zero rates -> 1e-9;
 * rsquared = sklearn r2_score per trial (neurons = samples, bins = outputs, force_finite),
 * NaN-ignoring mean over trials; mse / mae over all elements (want_r2 computes these three).
 * out (device f64[8]): [0] bps, [1] rsquared, [2] #NaN rates among kept spikes, [3] #negative
 * rates, [4] #NaN/inf rsquared inputs, [5] mse, [6] mae.  The reference raises on [2], [3]
 * (AssertionError) and [4] (ValueError); the host layer does the same.  Optional device outputs:
 * bps_per_neuron f64[n_eval], r2_per_trial f64[trials].  f64 accumulation, fixed order.
 * ------------------------------------------------------------------------------------------ */
size_t vs_spike_metrics_workspace_bytes(int64_t trials, int64_t T, int64_t N);
int vs_spike_metrics(int64_t trials, int64_t T, int64_t N, const float* gt, const float* pred,
                     int32_t log_input, int64_t n_eval, int32_t want_r2, double* out,
                     double* bps_per_neuron, double* r2_per_trial, void* workspace, void* stream);

/* ------------------------------------------------------------------------------------------
 * One pre-LN ViT block (mv:419-445) as a native executor: LN1 -> QKV GEMM -> attention ->
 * out-proj + residual -> LN2 -> fc1+GELU -> fc2 + residual, and its backward.  All tensors are
 * caller-owned; `dtype` is the activation/weight element type (residual stream, LN statistics,
 * softmax statistics and gradients of weights are f32 in both modes).
 * ------------------------------------------------------------------------------------------ */
typedef struct vs_vit_layer {
  int32_t dtype;
  int32_t heads;
  int64_t batch, tokens, hidden, mlp;        /* M = batch*tokens rows */
  float ln_eps;
  float attn_scale;
  /* weights: matrices in `dtype` ([out, in] nn.Linear layout), vectors f32 */
  const float *ln1_g, *ln1_b, *ln2_g, *ln2_b;
  const void* w_qkv;  const float* b_qkv;    /* [3D, D], [3D] (k third == 0) */
  const void* w_proj; const float* b_proj;   /* [D, D] */
  const void* w_fc1;  const float* b_fc1;    /* [F, D] */
  const void* w_fc2;  const float* b_fc2;    /* [D, F] */
  /* activations (saved for the backward) */
  const float* x_in;                         /* [M, D] f32 */
  void* h1;  float* mean1; float* rstd1;     /* [M, D] dtype; [M] */
  void* qkv; void* attn_o; float* lse;       /* [M, 3D]; [M, D]; [B, H, N] */
  float* y;                                  /* [M, D] f32 (after attention residual) */
  void* h2;  float* mean2; float* rstd2;
  void* a_pre; void* a_act;                  /* [M, F] dtype.  bf16 mode (ABI v4): a_pre holds gelu'(pre),
                                                the factor the backward's GELU' product multiplies by
                                                (VS_EPI_GELU_GRAD / VS_EPI_MUL_AUX), not pre itself.
                                                ABI v5: a_pre == NULL selects the FUSED MLP (vs_mlp_fwd /
                                                vs_mlp_bwd_da; bf16 and vs_mlp_fused_ok only): the forward
                                                stores nothing of the intermediate, and a_act is [M, F]
                                                bf16 scratch that the backward writes (gelu(pre) for dW2) —
                                                one buffer may serve every layer of a model */
  float* x_out;                              /* [M, D] f32 */
  /* ABI v6: dtype VS_FP8 (bf16 block with MX-FP8 forward products, BASELINE C5) needs this scratch,
     vs_vit_fp8_workspace_bytes(M, D, F) bytes, 256-B aligned; unused otherwise */
  void* fp8_ws; int64_t fp8_ws_bytes;
  /* ABI v7: the NEXT block's LayerNorm1 produced by this block's fused MLP epilogue (optional; all
     five set or all NULL): next_ln_g/b [D] f32 gamma/beta, next_h1 [M, D] bf16, next_mean1 /
     next_rstd1 [M] f32 (the next block's h1 / mean1 / rstd1).  ln1_ready != 0: this block's h1 /
     mean1 / rstd1 were written that way by the previous block, so its own LayerNorm1 launch is
     skipped (the values are those of LN1(x_in) either way) */
  const float* next_ln_g; const float* next_ln_b;
  void* next_h1; float* next_mean1; float* next_rstd1;
  int32_t ln1_ready; int32_t reserved7;
} vs_vit_layer;
size_t vs_vit_fp8_workspace_bytes(int64_t M, int64_t D, int64_t F);

typedef struct vs_vit_layer_grad {
  /* weight gradients (f32, ACCUMULATED) */
  float *ln1_g, *ln1_b, *ln2_g, *ln2_b;
  float *w_qkv, *b_qkv, *w_proj, *b_proj, *w_fc1, *b_fc1, *w_fc2, *b_fc2;
  /* activation gradients */
  const float* dx_out;  const void* dx_out_lp;   /* [M, D] f32 and a `dtype` copy (bf16 mode) */
  float* dx_in;         void* dx_in_lp;          /* outputs, same shapes */
  /* scratch (caller-owned): */
  void* d_a;            /* [M, F] dtype: d(pre-activation of fc1) */
  float* d_h;           /* [M, D]: grad wrt LN outputs; f32 in fp32 mode, written as bf16 in bf16
                           mode (ABI v4) unless VS_KNOB_DH_F32 or VS_BWD_FUSE_LN is set — size it for f32 */
  float* dy;  void* dy_lp;                       /* [M, D] f32 + dtype copy */
  void* d_o;            /* [M, D] dtype */
  void* d_qkv;          /* [M, 3D] dtype */
  void* attn_ws;        /* vs_attn_bwd_workspace_bytes */
  void* ln_ws;          /* vs_layernorm_bwd_workspace_bytes(M, D) */
  void* gemm_ws;        /* split-K partials of the weight-gradient GEMMs (optional) */
  int64_t gemm_ws_bytes;
  int32_t flags;        /* VS_BWD_* bits */
  int32_t reserved;
  void* chain;          /* vs_bwd_chain of this backward sequence (side stream + join state), or
                           NULL: the weight-gradient products then run on the caller's stream */
} vs_vit_layer_grad;

/* With a chain, the weight-gradient GEMMs of a block run on the chain's side stream.  Default: the
 * caller's stream joins it before vs_vit_layer_bwd returns.  VS_BWD_DEFER_JOIN: no join; instead
 * the NEXT vs_vit_layer_bwd call with the same chain (the next block of the same backward, reusing
 * the same scratch buffers) waits on each product right before overwriting its input.  The weight
 * gradients of a deferred block are therefore complete in the caller's stream order only after
 * the next call; the last block of a backward must not set the flag.  VS_BWD_DEFER_LAST: the
 * caller's stream joins the first three products (dW2, dW1, dWproj) at the end of the block and
 * defers only dWqkv, which the next call waits on before overwriting d_qkv; same last-block rule.
 * Both flags need a chain.  A chain is not thread-safe: one backward sequence uses it at a time
 * (each model / thread creates its own).  Destroying a chain does not wait for its side stream. */
#define VS_BWD_DEFER_JOIN 0x1
#define VS_BWD_DEFER_LAST 0x2
/* VS_BWD_FUSE_LN: run dh2 -> LN2' and dh1 -> LN1' as vs_gemm_ln_bwd (one launch each, dh never
 * leaves the chip).  Off by default: with the side-stream dW products it measured 6.02 vs 5.93
 * ms/step (the fused kernel holds 128 KB of LDS per CU, so the 128-KB dW workgroups cannot share
 * its CUs; serialised, the fusion wins: 6.28 vs 6.36, scripts/r02_run19.sh). */
#define VS_BWD_FUSE_LN    0x4

int vs_vit_layer_fwd(const vs_vit_layer* L, void* stream);
int vs_vit_layer_bwd(const vs_vit_layer* L, const vs_vit_layer_grad* G, void* stream);
int vs_bwd_chain_create(void** chain);   /* on the current device */
int vs_bwd_chain_destroy(void* chain);

/* ------------------------------------------------------------------------------------------
 * Data-parallel gradient exchange over RCCL (xGMI), for hosts that do not run torch.distributed:
 * replaces the implicit DDP all-reduce of accelerate (src/train.py:61-64 `accelerator.prepare`,
 * src/trainer/base.py:150 `accelerator.backward`).  One communicator per process / GPU: rank 0
 * makes an id (vs_comm_unique_id), the host ships its VS_COMM_ID_BYTES to every rank (any
 * channel), each rank calls vs_comm_init on its device.  vs_comm_allreduce_bucket sums one gradient
 * bucket in place across ranks, enqueued on the caller's stream (call it as each bucket's backward
 * products finish: the collective overlaps the rest of the backward); fold 1/world into vs_adamw's
 * grad_scale.  RCCL failures return VS_COMM_ERR_BASE + ncclResult_t.  The Python host uses
 * torch.distributed (backend "nccl" = RCCL) through vspike/dp.py with the same bucketing.
 * ------------------------------------------------------------------------------------------ */
#define VS_COMM_ID_BYTES 128
#define VS_COMM_ERR_BASE 1000
int vs_comm_unique_id(void* id_out /* VS_COMM_ID_BYTES */);
int vs_comm_init(void** comm, const void* id, int32_t world, int32_t rank);
int vs_comm_allreduce_bucket(void* comm, void* buf, int64_t count, int32_t dtype, void* stream);
int vs_comm_finalize(void* comm);

/* ------------------------------------------------------------------------------------------
 * R3D-18 video encoder (BASELINE C4: "ResNet-18 3D-conv encoder, 32x112x112 clips, fp32").  The
 * reference has NO CNN encoder (its registry is src/utils/utils.py:28-34): these
 * entry points replace what torch would run for a torchvision-style r3d_18 behind the plugin surface
 * (nn.Conv3d forward / its autograd dX and dW, nn.BatchNorm3d in training mode, nn.ReLU, the residual
 * add, nn.AdaptiveAvgPool3d(1)), feeding the reference head (src/model/videomae.py:13-14,28-31).
 * Layout: activations channels-last f32 [N][D][H][W][C] with C a power of two >= 4 (the 3-channel
 * input is padded to 4 with zeros); weights [Co][kd][kh][kw][Ci] (torch's [Co][Ci][kd][kh][kw]
 * permuted).  All three conv entry points are implicit GEMMs on v_mfma_f32_16x16x4_f32 (exact f32:
 * a k-ordered fmaf chain per output), no im2col tensor: rows = output voxels, k = (tap, channel) in
 * the [kd][kh][kw][Ci] order, the A operand gathered from the input in the operand load (zero
 * outside the padded volume).  Deterministic: no atomics anywhere (fixed-order partial sums).
 * ------------------------------------------------------------------------------------------ */
typedef struct vs_conv3d_desc {
  int64_t N;                        /* batch */
  int64_t Di, Hi, Wi, Ci;           /* input volume and channels */
  int64_t Do, Ho, Wo, Co;           /* output volume and channels (Do = (Di + 2 pd - kd) / sd + 1, ...) */
  int32_t kd, kh, kw;               /* kernel */
  int32_t sd, sh, sw;               /* stride (1 or 2) */
  int32_t pd, ph, pw;               /* zero padding */
  int32_t reserved;
} vs_conv3d_desc;
/* y = conv(x, w); optional stats [ceil(N Do Ho Wo / 128)][2][Co]: per 128-row tile t (output rows
   [128 t, min(128 t + 128, rows))) the column sum of y and the column sum of (y - the tile's column mean)^2
   (the BatchNorm3d batch statistics, merged by vs_bn3d_stats).  Co % 64 == 0. */
int vs_conv3d_fwd(const vs_conv3d_desc* d, const float* x, const float* w, float* y, float* stats, void* stream);
size_t vs_conv3d_stats_rows(const vs_conv3d_desc* d);
/* dx (=|+=) the input gradient of dy: stride 1 as the flipped-kernel conv of dy, stride 2 as one
   implicit GEMM per parity class of the input positions (only the taps that reach that class), so
   no MFMA runs on a zero.  Weights are regrouped per class into the workspace
   (vs_conv3d_dx_workspace_bytes).  accumulate: 1 adds into dx (a residual branch's gradient),
   0 overwrites every element. Ci % 64 == 0, Co a power of two >= 4. */
size_t vs_conv3d_dx_workspace_bytes(const vs_conv3d_desc* d);
int vs_conv3d_dx(const vs_conv3d_desc* d, const float* dy, const float* w, float* dx, int32_t accumulate,
                 void* workspace, int64_t workspace_bytes, void* stream);
/* dw (=|+=) sum over output voxels of dy^T gather(x): split over the rows into workspace partials,
   summed in split order.  Co % 64 == 0. */
size_t vs_conv3d_dw_workspace_bytes(const vs_conv3d_desc* d);
int vs_conv3d_dw(const vs_conv3d_desc* d, const float* x, const float* dy, float* dw, int32_t accumulate,
                 void* workspace, int64_t workspace_bytes, void* stream);
/* BatchNorm3d (training): from the conv's stats partials (rows = ceil(count / 128) tiles of [2][C] as
   vs_conv3d_fwd writes them) -> mean, rstd over count values per channel (biased variance, eps; the
   tiles merged in f64 with Chan's formula, no E[y^2] - mean^2 cancellation), scale = gamma rstd, shift = beta - mean scale; the
   running buffers (nullable) move by momentum with the unbiased variance (torch semantics). */
size_t vs_bn3d_stats_workspace_bytes(int64_t rows, int64_t C);
int vs_bn3d_stats(int64_t rows, int64_t C, const float* part, int64_t count, const float* gamma,
                  const float* beta, float eps, float momentum, float* mean, float* rstd, float* scale,
                  float* shift, float* running_mean, float* running_var, void* workspace, void* stream);
/* out = [relu](y scale + shift [+ residual]) over M rows x C channels (channels-last). */
int vs_bn3d_apply(int64_t M, int64_t C, const float* y, const float* scale, const float* shift,
                  const float* residual, int32_t relu, float* out, void* stream);
/* Backward of out = [relu](bn(y) [+ residual]): g = dout [* (out > 0)];  dgamma (+)= sum g xhat,
   dbeta (+)= sum g;  dy = gamma rstd (g - mean(g) - xhat mean(g xhat));  dres = g (nullable: the
   shortcut's gradient).  Workspace: vs_bn3d_bwd_workspace_bytes. */
size_t vs_bn3d_bwd_workspace_bytes(int64_t M, int64_t C);
int vs_bn3d_bwd(int64_t M, int64_t C, const float* dout, const float* out, int32_t relu, const float* y,
                const float* mean, const float* rstd, const float* gamma, float* dy, float* dres, float* dgamma,
                float* dbeta, void* workspace, void* stream);
/* The same for an eval-mode (running-statistics) BatchNorm: mean / rstd are the running statistics,
   constants of the forward, so dy = gamma rstd g (no batch-statistics terms); dgamma / dbeta / dres
   as vs_bn3d_bwd (nn.BatchNorm3d.eval() under autograd: frozen-BN fine-tuning). */
int vs_bn3d_bwd_eval(int64_t M, int64_t C, const float* dout, const float* out, int32_t relu, const float* y,
                     const float* mean, const float* rstd, const float* gamma, float* dy, float* dres,
                     float* dgamma, float* dbeta, void* workspace, void* stream);
/* pixels (B, T, C, H, W) f32 -> channels-last (B, T, H, W, Cp) with channels C..Cp-1 zero (Cp = 4 or 8). */
int vs_to_channels_last(int64_t B, int64_t T, int64_t C, int64_t H, int64_t W, int64_t Cp, const float* x,
                        float* out, void* stream);
/* pooled[n][c] = mean over S voxels of x[n][s][c] (nn.AdaptiveAvgPool3d(1)); its backward
   dx[n][s][c] = dpool[n][c] / S. */
int vs_avgpool3d(int64_t N, int64_t S, int64_t C, const float* x, float* pooled, void* stream);
int vs_avgpool3d_bwd(int64_t N, int64_t S, int64_t C, const float* dpool, float* dx, void* stream);

/* ------------------------------------------------------------------------------------------
 * Trial shards (host side of the input path; replaces the per-trial webdataset tars of
 * src/prepare_data.py:210-235 read by src/loader/base.py:21-41).  Fixed-size records: raw uint8
 * frames (T, C, H, W) + f32 spike counts (ap_rows, ap_cols) + a 64-byte "<eid>_<trial>" key.
 * vs_shard_read gathers records into caller (pinned) host buffers with `threads` parallel
 * positional reads.  Host-only: no stream, no device memory.  Errors: VS_EINVAL / NULL with
 * vs_shard_last_error() set.
 * ------------------------------------------------------------------------------------------ */
int vs_shard_write(const char* path, int64_t n, int64_t T, int64_t C, int64_t H, int64_t W,
                   int64_t ap_rows, int64_t ap_cols, const uint8_t* video, const float* ap,
                   const char* keys /* n x 64 bytes */);
void* vs_shard_open(const char* path, int64_t* info /* [8]: n, T, C, H, W, ap_rows, ap_cols, record_bytes */);
int vs_shard_key(void* shard, int64_t i, char* buf, int32_t n /* >= 65 */);
int vs_shard_read(void* shard, const int64_t* idx, int64_t n, uint8_t* video_dst, float* ap_dst,
                  int32_t threads);
void vs_shard_close(void* shard);
const char* vs_shard_last_error(void);

/* ------------------------------------------------------------------------------------------
 * Kernel timing (bench instrumentation).  When enabled, every launch of a tracked entry point is
 * bracketed with hipEvents on its launch stream, and the ALGORITHMIC bytes (or flops) of the call
 * are added to the timer: the bytes a perfect kernel must move (operands read once, outputs
 * written once; split-K partials, re-reads and padding excluded) — the numerator of a roofline
 * fraction.  vs_timing_collect() synchronises on the recorded events and returns the launch
 * count, total milliseconds and total algorithmic bytes of one timer.
 * ------------------------------------------------------------------------------------------ */
#define VS_TIMER_ATTN_FWD 0   /* vs_attn_fwd (bytes: Q,K,V,O,LSE) */
#define VS_TIMER_ATTN_BWD 1   /* vs_attn_bwd incl. the row prep (bytes: Q,K,V,O,dO,LSE,dQKV) */
#define VS_TIMER_GEMM     2   /* vs_gemm, activation products (no VS_EPI_ATOMIC) */
#define VS_TIMER_GEMM_DW  3   /* vs_gemm with VS_EPI_ATOMIC: the token-reduction dW products + reduce */
#define VS_TIMER_LN_FWD   4   /* vs_layernorm_fwd */
#define VS_TIMER_LN_BWD   5   /* vs_layernorm_bwd (+ its partial-sum reduction) */
#define VS_TIMER_ADAMW    6   /* vs_adamw */
#define VS_TIMER_MISC     7   /* vs_cast, vs_colsum, vs_patch_im2col, vs_poisson_nll(_bwd) */
/* per-product tags of the ViT block executor (vs_vit_layer_fwd / _bwd): its vs_gemm calls are
   charged to these instead of VS_TIMER_GEMM / VS_TIMER_GEMM_DW, so every product has its own timer */
#define VS_TIMER_FWD_QKV   8   /* qkv = h1 Wqkv^T + b          (mv:233-236) */
#define VS_TIMER_FWD_PROJ  9   /* y = x + o Wp^T + bp           (mv:312-319) */
#define VS_TIMER_FWD_FC1  10   /* a = gelu(h2 W1^T + b1)        (mv:373-383) */
#define VS_TIMER_FWD_FC2  11   /* x' = y + a W2^T + b2          (mv:390-397) */
#define VS_TIMER_DX_FC2   12   /* da = (dx' W2) * gelu'(pre) */
#define VS_TIMER_DX_FC1   13   /* dh2 = da W1 */
#define VS_TIMER_DX_PROJ  14   /* do = dy Wp */
#define VS_TIMER_DX_QKV   15   /* dh1 = dqkv Wqkv */
#define VS_TIMER_DW_FC2   16   /* dW2 += dx'^T a (+ db2) */
#define VS_TIMER_DW_FC1   17   /* dW1 += da^T h2 (+ db1) */
#define VS_TIMER_DW_PROJ  18   /* dWp += dy^T o (+ dbp) */
#define VS_TIMER_DW_QKV   19   /* dWqkv += dqkv^T h1 (+ dbqkv) */
#define VS_TIMER_FWD_MLP  20   /* the fused MLP forward (vs_mlp_fwd, a_pre == NULL)   (mv:370-399) */
#define VS_TIMER_DX_MLP   21   /* the fused MLP backward's GELU' product (vs_mlp_bwd_da) */
#define VS_TIMER_FP8_QUANT 22  /* the MX-FP8 forward's operand quantisation (vs_quant_mxfp8 of A and W) */
/* the R3D-18 encoder (BASELINE C4): flops are charged for the conv timers (2 M N K of the implicit GEMM,
   valid taps only), bytes for the BatchNorm / elementwise timer */
#define VS_TIMER_CONV_FWD 23   /* vs_conv3d_fwd (+ the fused BatchNorm batch statistics) */
#define VS_TIMER_CONV_DX  24   /* vs_conv3d_dx (every parity class of a strided conv) */
#define VS_TIMER_CONV_DW  25   /* vs_conv3d_dw (+ its split reduce) */
#define VS_TIMER_BN       26   /* vs_bn3d_* and the layout / pooling helpers */
#define VS_TIMER_COUNT    27
int vs_timing_enable(int mask);   /* bit (1 << timer) enables that timer; 0 disables all */
int vs_timing_collect(int timer, int64_t* launches, double* total_ms);
int vs_timing_bytes(int timer, double* algorithmic_bytes);   /* call before vs_timing_collect */

/* ------------------------------------------------------------------------------------------
 * Dispatch counters: every launch of a kernel path adds one to its counter (host-side, relaxed
 * atomics), so a test can assert WHICH kernels an oracle-pinned run reached (e.g. that the
 * benched B=16 step runs the row-slab / W-resident / fused-LN / dW-tile paths).
 * ------------------------------------------------------------------------------------------ */
#define VS_PATH_GEMM_DW       0   /* gemm_dw_kernel: token-reduction weight gradients */
#define VS_PATH_GEMM_SKINNY   1   /* skinny split-K (head) */
#define VS_PATH_GEMM_SLAB     2   /* gemm_bf16_slab: N <= 192 row slabs */
#define VS_PATH_GEMM_BIG      3   /* gemm_bf16_big: 256 x 128 tiles */
#define VS_PATH_GEMM_WRES     4   /* gemm_bf16_wres: W-resident K = 192 */
#define VS_PATH_GEMM_WSLAB    5   /* gemm_bf16_wslab: wide row slabs */
#define VS_PATH_GEMM_PANEL    6
#define VS_PATH_GEMM_FULLK    7
#define VS_PATH_GEMM_RING     8
#define VS_PATH_GEMM_TILE     9   /* generic register-staged tiles */
#define VS_PATH_GEMM_F32     10   /* exact-f32 MFMA kernel */
#define VS_PATH_GEMM_LN_FWD  11   /* vs_gemm_ln_fwd fused (slab + LayerNorm) */
#define VS_PATH_GEMM_LN_BWD  12   /* vs_gemm_ln_bwd fused (slab + LayerNorm') */
#define VS_PATH_ATTN_FWD     13   /* bf16 flash forward */
#define VS_PATH_ATTN_BWD     14   /* bf16 flash backward (row prep + dK/dV + dQ) */
#define VS_PATH_ATTN_F32     15   /* exact-f32 attention, forward or backward */
#define VS_PATH_PATCH_FUSED  16   /* patch embedding GEMM with the tubelet gather in its A-load */
#define VS_PATH_DW_GROUPED   17   /* grouped dW launch (several weight gradients in one launch) */
#define VS_PATH_MLP_FWD      18   /* vs_mlp_fwd: fused fc1 + GELU + fc2 + residual */
#define VS_PATH_MLP_BWD      19   /* vs_mlp_bwd_da: fused recompute + GELU' product */
#define VS_PATH_GEMM_FP8     20   /* vs_gemm_mxfp8: block-scaled fp8 MFMA GEMM */
#define VS_PATH_PATCH_DW     21   /* vs_patch_embed_dw: patch dW with the tubelet gather in its B-load */
#define VS_PATH_CONV_IGEMM   22   /* conv_igemm_kernel: Conv3d forward / dX as an implicit GEMM (f32 MFMA) */
#define VS_PATH_CONV_DW      23   /* conv_dw_kernel: Conv3d weight gradient (implicit-GEMM gather, split over rows) */
#define VS_PATH_GEMM_G256    24   /* gemm_bf16_g256_kernel: 256 x 256 persistent tiles, 64-deep LDS-DMA stages (long-M ViT-Base products) */
#define VS_PATH_GEMM_DW256   25   /* gemm_dw256_kernel: long-K weight gradients on 256 x 256 persistent tiles + fixed-order reduce */
#define VS_PATH_COUNT        26
/* copies min(n, VS_PATH_COUNT) counters into out; returns VS_PATH_COUNT */
int vs_dispatch_counts(int64_t* out, int n);
int vs_dispatch_reset(void);
/* 1 when every compiled instance of the 256 x 256 forward / dX GEMM (VS_PATH_GEMM_G256) has no private
   (scratch) segment: its early-DMA wait counts the epilogue's stores exactly.  An instance that spills
   falls back to vmcnt(0) on its own; this is the test's view of the same check. */
int vs_g256_scratch_free(void);

/* ------------------------------------------------------------------------------------------
 * A/B and test knobs.  Each is read ONCE from the environment (VSPIKE_<NAME>, an integer; unset =
 * the default, which is the benchmarked dispatch) on first use, and can then be overridden by
 * vs_knob_set (tests select a path this way).  No entry point calls getenv on its launch path.
 * ------------------------------------------------------------------------------------------ */
#define VS_KNOB_DW_OLD       0   /* 1: dW products on the generic split-K tiles */
#define VS_KNOB_NO_SKINNY    1
#define VS_KNOB_NO_SLAB      2
#define VS_KNOB_NO_BIG       3
#define VS_KNOB_NO_WRES      4
#define VS_KNOB_WRES_GBWD    5   /* 1: the GELU' dX product on the W-resident kernel */
#define VS_KNOB_NO_WSLAB     6
#define VS_KNOB_WSLAB        7   /* 1: every eligible K <= 192 product on the wide row slabs */
#define VS_KNOB_WSLAB_G      8   /* wide row-slab grid cap (default 512) */
#define VS_KNOB_PANEL        9
#define VS_KNOB_NO_PANEL    10
#define VS_KNOB_PANEL_GRID  11   /* default 512 */
#define VS_KNOB_NO_FULLK    12
#define VS_KNOB_NO_RING     13
#define VS_KNOB_NO_LNF_FUSE 14
#define VS_KNOB_NO_LN_FUSE  15
#define VS_KNOB_DW_BM       16   /* force the dW tile / split / stage choice (0 = planned) */
#define VS_KNOB_DW_BN       17
#define VS_KNOB_DW_SPLITS   18
#define VS_KNOB_DW_STAGES   19
#define VS_KNOB_LN_BLOCKS   20   /* LayerNorm' grid cap (0 = default 512, at most 1024) */
#define VS_KNOB_DH_F32      21   /* 1: the ViT block's dh1 / dh2 stay f32 in bf16 mode */
#define VS_KNOB_NO_PATCH_FUSED 22 /* 1: im2col + GEMM instead of the fused patch embedding */
#define VS_KNOB_NO_DW_GROUP 23   /* 1: one launch per weight gradient instead of the grouped dW launch */
#define VS_KNOB_ATTN_VARIANT 24  /* attention kernel variant (0 = default) */
#define VS_KNOB_SLAB_WV     25   /* row-slab GEMM waves per workgroup: 4 or 8 (0 = by slab length) */
#define VS_KNOB_WRES_WV     26   /* W-resident GEMM waves per workgroup: 8, else 4 */
#define VS_KNOB_WRES_DBG    27   /* VS_DEBUG_KNOBS builds only (ignored otherwise): W-resident GEMM 1 = L2-resident stores, 2 = L2-resident reads (WRONG results) */
#define VS_KNOB_G256        28   /* long-M products on the 256 x 256 persistent kernel: 0 = where measured faster (N or K >= 2304, not the GELU' product), 1 = every eligible product, 2 = never (256 x 128 big tile) */
#define VS_KNOB_G256_GRID   29   /* 256 x 256 persistent GEMM grid cap (0 = 256: one workgroup per CU) */
#define VS_KNOB_G256_DBG    30   /* VS_DEBUG_KNOBS builds only: 256 x 256 GEMM bit 0 = no operand DMA, bit 1 = no epilogue stores (WRONG results) */
#define VS_KNOB_NO_DW256    31   /* 1: the long-K dW products on the split-K dW kernel instead of the 256 x 256 persistent one */
#define VS_KNOB_G256_STAGGER 32  /* 256 x 256 GEMM: odd-slot workgroups start N x s_sleep(127) (~4 us) late */
#define VS_KNOB_CONV_DW128  33   /* 1: Conv3d weight gradient on 128-wide k tiles where K >= 128 (measured slower than the 64-wide default) */
#define VS_KNOB_CONV_MFMA   34   /* Conv3d weight gradient's f32 MFMA shape: 0 = 16x16x4 (default), 1 = 32x32x2 (measured slower) */
#define VS_KNOB_DW256_ALL   36   /* 1: the 768 x 768 projection dW on the 256 x 256 dW kernel too (default: split-K dW tiles) */
#define VS_KNOB_LN_FWD_BLOCKS 37 /* LayerNorm forward (vectorised) grid cap (0 = default 768) */
#define VS_KNOB_G256_A3     35   /* 256 x 256 forward / dX GEMM: the streamed A operand in three LDS slots (DMA two stages ahead, counted stage wait): 0 / 1 = on (default), 2 = off (two slots, round 5) */
#define VS_KNOB_COUNT       40
int vs_knob_get(int knob);               /* VS_EINVAL for an unknown id */
int vs_knob_set(int knob, int value);    /* returns the previous value; VS_EINVAL for an unknown id */
int vs_knob_default(int knob);           /* the built-in default of a knob (before the environment) */
int vs_debug_knobs(void);                /* 1: built with VS_DEBUG_KNOBS (timing-only knobs active) */

#ifdef __cplusplus
}
#endif
#endif /* VSPIKE_H */
