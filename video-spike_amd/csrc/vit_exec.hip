// vit_exec.hip — native executor for one pre-LN ViT block (mv:419-445) and its backward.
//
// Sequencing lives in C++ so a whole block is one host call: 7 launches forward, ~16 backward,
// all on the caller's stream (graph-capturable: no allocation, no synchronisation).
// Forward (dtype T = f32 or bf16; residual stream f32):
//   h1 = LN1(x) [T] -> qkv = h1 Wqkv^T + b [T] -> o = attn(qkv) [T] (+lse)
//   y = x + o Wproj^T + b [f32] -> h2 = LN2(y) [T] -> a = gelu(h2 W1^T + b1) [T] (pre-act saved)
//   x' = y + a W2^T + b2 [f32]
// Backward mirrors it with the weight gradients accumulated in f32 (split-K atomics for the
// token-reduction dW products, whose K is B*N = 25,088 rows at the bench shape).
#include <cstdlib>

#include "common.h"

namespace vs {

static bool dh_f32() { return knob(VS_KNOB_DH_F32) != 0; }

static vs_gemm_desc gdesc(int dtype, int out_dtype, bool akc, bool bkc, int64_t M, int64_t N, int64_t K, const void* a,
                          int64_t lda, const void* b, int64_t ldb, void* c, int64_t ldc, uint32_t epi) {
  vs_gemm_desc d = {};
  d.dtype = dtype;
  d.out_dtype = out_dtype;
  d.a_kcontig = akc;
  d.b_kcontig = bkc;
  d.M = M; d.N = N; d.K = K;
  d.a = a; d.lda = lda;
  d.b = b; d.ldb = ldb;
  d.c = c; d.ldc = ldc;
  d.epilogue = epi;
  d.alpha = 1.0f;
  return d;
}

// Side stream for the weight-gradient products of the backward.  The four dW = dY^T X GEMMs of a
// block (reductions over all B*N tokens, HBM-bound, each ~10-30 us of mostly load/drain latency
// at the bench shape) depend only on tensors the main stream has already produced, and nothing on
// the main stream reads their results within the block, so they run on a second stream: dW2 beside
// da, dW1 beside dh2 + LN2', dWp beside do + the attention backward, dWqkv beside dh1 + LN1'.
// The side stream forks from the caller's stream at each product's input (an event) and joins it
// at the end of the block, so the caller's stream order is unchanged for everything downstream
// (optimizer, gradient exchange) and buffers reused across blocks are never read late.
// Deferred join (VS_BWD_DEFER_JOIN): instead of joining at the end of the block, the side stream
// records one event per weight-gradient product (two parity sets, alternating per call) and the
// NEXT block's main stream waits on each just before it overwrites the buffer that product reads
// (d_a, dy, d_qkv, the dx ping-pong buffer) — by then the product has long finished, so the
// cross-queue wait no longer stalls the main stream (~20 us per block at the bench shape).
// All of that state (side stream, events, parity, pending bits) lives in a caller-owned
// vs_bwd_chain, one per backward sequence: two backwards interleaved on one device (two models,
// or threads) each carry their own chain and never consume each other's events.  Without a chain
// the products run on the caller's stream (no fork, no join, nothing deferred).
struct BwdChain {
  int device = 0;
  hipStream_t side = nullptr;
  hipEvent_t ev[16] = {};
  int parity = 0;
  int pending = 0;  // bit k: the previous block's product k is not joined yet
};

// `to` waits for everything enqueued so far on `from` (event slot k)
static int stream_wait(hipStream_t from, hipStream_t to, hipEvent_t ev) {
  hipError_t e = hipEventRecord(ev, from);
  if (e == hipSuccess) e = hipStreamWaitEvent(to, ev, 0);
  return (int)e;
}

// a_pre == NULL selects the fused MLP (vs_mlp_fwd / vs_mlp_bwd_da): bf16, a shape vs_mlp_fused_ok
// accepts; a_act then points at [M, F] bf16 scratch that the BACKWARD writes (gelu(pre) for dW2)
static bool mlp_fused(const vs_vit_layer* L) { return L->a_pre == nullptr; }

// MX-FP8 scratch of one block forward (the A operand of the product being run, its scales, the
// weight and its scales; reused product by product in stream order)
struct Fp8Ws {
  uint8_t *aq, *as, *wq, *ws;
};
static size_t a256(size_t x) { return (x + 255) / 256 * 256; }
static Fp8Ws fp8_ws(const vs_vit_layer* L) {
  const int64_t M = L->batch * L->tokens, D = L->hidden, F = L->mlp, KM = D > F ? D : F;
  const int64_t WM = 3 * D * D > F * D ? 3 * D * D : F * D;
  Fp8Ws w;
  w.aq = (uint8_t*)L->fp8_ws;
  w.as = w.aq + a256((size_t)(M * KM));
  w.wq = w.as + a256((size_t)(M * KM / 32));
  w.ws = w.wq + a256((size_t)WM);
  return w;
}

// one MX-FP8 forward product: A (bf16 [M, K]) and W (bf16 [N, K]) quantised into the scratch, then
// the block-scaled GEMM with the given epilogue (the epilogue fields of g; g.a / g.b are replaced)
static int fp8_product(const vs_vit_layer* L, vs_gemm_desc g, void* stream) {
  const Fp8Ws w = fp8_ws(L);
  {
    TimerTag tag(VS_TIMER_FP8_QUANT);  // the product's timer then holds the GEMM alone
    VS_CALL(vs_quant_mxfp8(VS_BF16, g.M, g.K, g.a, g.lda, w.aq, g.K, w.as, g.K / 32, stream));
    VS_CALL(vs_quant_mxfp8(VS_BF16, g.N, g.K, g.b, g.ldb, w.wq, g.K, w.ws, g.K / 32, stream));
  }
  g.dtype = VS_FP8;
  g.a = w.aq; g.lda = g.K;
  g.b = w.wq; g.ldb = g.K;
  return vs_gemm_mxfp8(&g, w.as, g.K / 32, w.ws, g.K / 32, stream);
}

static int check_layer(const vs_vit_layer* L) {
  VS_REQUIRE(L, "vs_vit_layer: null");
  VS_REQUIRE(L->dtype == VS_F32 || L->dtype == VS_BF16 || L->dtype == VS_FP8, "vs_vit_layer: bad dtype");
  VS_REQUIRE(L->dtype != VS_FP8 || (L->hidden % 128 == 0 && L->mlp % 128 == 0 && L->fp8_ws &&
                                    (size_t)L->fp8_ws_bytes >= vs_vit_fp8_workspace_bytes(L->batch * L->tokens,
                                                                                           L->hidden, L->mlp)),
             "vs_vit_layer: VS_FP8 needs hidden % 128 == 0, mlp % 128 == 0 and the fp8 workspace");
  VS_REQUIRE(L->hidden == L->heads * 64, "vs_vit_layer: hidden must be heads*64");
  VS_REQUIRE(L->batch > 0 && L->tokens > 0 && L->mlp > 0, "vs_vit_layer: empty");
  VS_REQUIRE(!mlp_fused(L) || (L->dtype == VS_BF16 && vs_mlp_fused_ok(L->batch * L->tokens, L->hidden, L->mlp) &&
                               L->a_act),
             "vs_vit_layer: a_pre == NULL (fused MLP) needs bf16, D = 192, F % 64 == 0 and an a_act scratch");
  VS_REQUIRE(!L->next_ln_g || (mlp_fused(L) && L->next_ln_b && L->next_h1 && L->next_mean1 && L->next_rstd1),
             "vs_vit_layer: next_ln_* (the next block's LayerNorm1) needs the fused MLP and all five pointers");
  return VS_OK;
}

}  // namespace vs

using namespace vs;

extern "C" size_t vs_vit_fp8_workspace_bytes(int64_t M, int64_t D, int64_t F) {
  const int64_t KM = D > F ? D : F, WM = 3 * D * D > F * D ? 3 * D * D : F * D;
  return a256((size_t)(M * KM)) + a256((size_t)(M * KM / 32)) + a256((size_t)WM) + a256((size_t)(WM / 32));
}

extern "C" int vs_vit_layer_fwd(const vs_vit_layer* L, void* stream) {
  VS_CALL(check_layer(L));
  const bool f8 = L->dtype == VS_FP8;  // bf16 block, MX-FP8 forward products
  const int T = f8 ? VS_BF16 : L->dtype;
  auto product = [&](const vs_gemm_desc& g) { return f8 ? fp8_product(L, g, stream) : vs_gemm(&g, stream); };
  const int64_t M = L->batch * L->tokens, D = L->hidden, F = L->mlp;
  if (!L->ln1_ready)  // else the previous block's fused MLP epilogue wrote h1 / mean1 / rstd1
    VS_CALL(vs_layernorm_fwd(T, M, D, L->x_in, D, L->ln1_g, L->ln1_b, L->ln_eps, L->h1, D, L->mean1, L->rstd1, stream));
  {
    vs_gemm_desc g = gdesc(T, T, true, true, M, 3 * D, D, L->h1, D, L->w_qkv, D, L->qkv, 3 * D, VS_EPI_BIAS);
    TimerTag tag(VS_TIMER_FWD_QKV);
    g.bias = L->b_qkv;
    VS_CALL(product(g));
  }
  VS_CALL(vs_attn_fwd(T, L->batch, L->tokens, L->heads, 64, L->qkv, 3 * D, L->attn_o, D, L->lse, L->attn_scale, stream));
  {
    vs_gemm_desc g = gdesc(T, VS_F32, true, true, M, D, D, L->attn_o, D, L->w_proj, D, L->y, D,
                           VS_EPI_BIAS | VS_EPI_RESIDUAL);
    g.bias = L->b_proj;
    TimerTag tag(VS_TIMER_FWD_PROJ);
    g.residual = L->x_in;
    g.ld_residual = D;
    if (f8) {
      VS_CALL(product(g));
    } else if (T == VS_BF16) {  // y and LN2(y) in one launch (the row-slab kernel owns whole rows of y)
      VS_CALL(vs_gemm_ln_fwd(&g, L->ln2_g, L->ln2_b, L->ln_eps, L->h2, D, L->mean2, L->rstd2, stream));
    } else {
      VS_CALL(vs_gemm(&g, stream));
    }
  }
  if (T != VS_BF16 || f8)
    VS_CALL(vs_layernorm_fwd(T, M, D, L->y, D, L->ln2_g, L->ln2_b, L->ln_eps, L->h2, D, L->mean2, L->rstd2, stream));
  if (mlp_fused(L)) {  // the whole MLP in one launch; nothing of the [M, F] intermediate is stored
    TimerTag tag(VS_TIMER_FWD_MLP);
    // with the next block's LayerNorm1 in the epilogue when the caller chained the blocks
    return vs_mlp_fwd_ln(M, D, F, L->h2, D, L->w_fc1, L->b_fc1, L->w_fc2, L->b_fc2, L->y, D, L->x_out, D,
                         L->next_ln_g, L->next_ln_b, L->ln_eps, L->next_h1, D, L->next_mean1, L->next_rstd1, stream);
  }
  {
    // bf16: a_pre holds gelu'(pre) (VS_EPI_GELU_GRAD), so the backward's GELU' product is a plain
    // multiply (VS_EPI_MUL_AUX) instead of an erf/exp evaluation per element; f32 keeps pre.
    const uint32_t epi = VS_EPI_BIAS | VS_EPI_GELU | (T == VS_BF16 ? VS_EPI_GELU_GRAD : 0u);
    vs_gemm_desc g = gdesc(T, T, true, true, M, F, D, L->h2, D, L->w_fc1, D, L->a_act, F, epi);
    TimerTag tag(VS_TIMER_FWD_FC1);
    g.bias = L->b_fc1;
    g.aux_out = L->a_pre;
    g.ld_aux_out = F;
    VS_CALL(product(g));
  }
  {
    vs_gemm_desc g = gdesc(T, VS_F32, true, true, M, D, F, L->a_act, F, L->w_fc2, F, L->x_out, D,
                           VS_EPI_BIAS | VS_EPI_RESIDUAL);
    g.bias = L->b_fc2;
    TimerTag tag(VS_TIMER_FWD_FC2);
    g.residual = L->y;
    g.ld_residual = D;
    VS_CALL(product(g));
  }
  return VS_OK;
}

extern "C" int vs_vit_layer_bwd(const vs_vit_layer* L, const vs_vit_layer_grad* G, void* stream) {
  VS_CALL(check_layer(L));
  VS_REQUIRE(G && G->dx_out && G->dx_in && G->d_a && G->d_h && G->dy && G->d_o && G->d_qkv && G->attn_ws,
             "vs_vit_layer_bwd: null gradient buffer");
  const int T = L->dtype == VS_FP8 ? VS_BF16 : L->dtype;  // the fp8 block's backward runs in bf16
  const bool lp = T == VS_BF16;
  VS_REQUIRE(!lp || (G->dx_out_lp && G->dy_lp), "vs_vit_layer_bwd: bf16 mode needs dx_out_lp and dy_lp");
  const int64_t M = L->batch * L->tokens, D = L->hidden, F = L->mlp;
  const void* gx = lp ? G->dx_out_lp : (const void*)G->dx_out;  // dx' as a GEMM operand
  const void* gy = lp ? G->dy_lp : (const void*)G->dy;
  hipStream_t ms = (hipStream_t)stream;
  BwdChain* ch = (BwdChain*)G->chain;
  VS_REQUIRE(ch || !(G->flags & (VS_BWD_DEFER_JOIN | VS_BWD_DEFER_LAST)),
             "vs_vit_layer_bwd: deferred joins need a vs_bwd_chain");
  if (ch) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return (int)e;
    VS_REQUIRE(dev == ch->device, "vs_vit_layer_bwd: chain belongs to another device");
  }
  hipStream_t ss = ch ? ch->side : ms;
  void* side = (void*)ss;
  hipEvent_t* ev = ch ? ch->ev : nullptr;
  const int par = ch ? ch->parity : 0;
  const int pend = ch ? ch->pending : 0;
  hipEvent_t* pe = ch ? ev + 8 + 4 * (1 - par) : nullptr;  // the previous block's products (deferred join)
  hipEvent_t* ce = ch ? ev + 8 + 4 * par : nullptr;        // this block's
  auto wait_prev = [&](int k) -> int { return (pend >> k) & 1 ? (int)hipStreamWaitEvent(ms, pe[k], 0) : 0; };
  auto mark = [&](int k) -> int { return ch ? (int)hipEventRecord(ce[k], ss) : 0; };
  auto fork = [&](int k) -> int { return ch ? stream_wait(ms, ss, ev[k]) : 0; };

  // ---- MLP: x' = y + a W2^T + b2
  if (mlp_fused(L)) {
    // a (L->a_act) and d_a are rewritten here: the previous block's dW2 / dW1 read them
    VS_CALL(wait_prev(0));
    VS_CALL(wait_prev(1));
    {  // da = (dx' W2) * gelu'(pre), a = gelu(pre), pre recomputed from h2
      TimerTag tag(VS_TIMER_DX_MLP);
      VS_CALL(vs_mlp_bwd_da(M, D, F, L->h2, D, L->w_fc1, L->b_fc1, L->w_fc2, gx, D, G->d_a, F, L->a_act, F, stream));
    }
    VS_CALL(fork(0));  // da, a ready
  } else {
    VS_CALL(fork(0));  // dx' (and the block's saved activations) ready
  }
  {  // [side] dW2[D,F] += dx'^T a;  db2 += colsum(dx') fused
    vs_gemm_desc g = gdesc(T, VS_F32, false, false, D, F, M, gx, D, L->a_act, F, G->w_fc2, F, VS_EPI_ATOMIC);
    TimerTag tag(VS_TIMER_DW_FC2);
    g.a_rowsum = G->b_fc2;
    g.workspace = G->gemm_ws;
    g.workspace_bytes = G->gemm_ws_bytes;
    VS_CALL(vs_gemm(&g, side));
    VS_CALL(mark(0));
  }
  if (!mlp_fused(L)) {
    VS_CALL(wait_prev(1));  // d_a is read by the previous block's dW1
    {  // d(pre-act) = (dx' W2) * gelu'(pre)
      vs_gemm_desc g = gdesc(T, T, true, false, M, F, D, gx, D, L->w_fc2, F, G->d_a, F,
                             lp ? VS_EPI_MUL_AUX : VS_EPI_GELU_BWD);  // bf16: a_pre = gelu'(pre)
      TimerTag tag(VS_TIMER_DX_FC2);
      g.aux_in = L->a_pre;
      g.ld_aux_in = F;
      VS_CALL(vs_gemm(&g, stream));
    }
    VS_CALL(fork(1));  // da ready
  }
  {  // [side] dW1[F,D] += da^T h2;  db1 += colsum(da) fused
    vs_gemm_desc g = gdesc(T, VS_F32, false, false, F, D, M, G->d_a, F, L->h2, D, G->w_fc1, D, VS_EPI_ATOMIC);
    TimerTag tag(VS_TIMER_DW_FC1);
    g.a_rowsum = G->b_fc1;
    g.workspace = G->gemm_ws;
    g.workspace_bytes = G->gemm_ws_bytes;
    VS_CALL(vs_gemm(&g, side));
    VS_CALL(mark(1));
  }
  // dh2 = da W1;  dy = dx' + LN2'(dh2)  (VS_BWD_FUSE_LN: one launch, dh2 stays on the chip)
  VS_CALL(wait_prev(2));  // dy / dy_lp are read by the previous block's dWp
  {
    // bf16: dh2 in bf16 (half the bytes written here and read by LN2'), as every other bf16 operand
    // (VSPIKE_DH_F32=1 keeps it f32, for A/B)
    const int hdt = (G->flags & VS_BWD_FUSE_LN) || dh_f32() ? VS_F32 : T;
    vs_gemm_desc g = gdesc(T, hdt, true, false, M, D, F, G->d_a, F, L->w_fc1, D, G->d_h, D, 0);
    TimerTag tag(VS_TIMER_DX_FC1);
    if (G->flags & VS_BWD_FUSE_LN) {
      VS_CALL(vs_gemm_ln_bwd(&g, L->y, D, L->mean2, L->rstd2, L->ln2_g, G->dx_out, D, G->dy, D,
                             lp ? G->dy_lp : nullptr, G->ln2_g, G->ln2_b, G->ln_ws, stream));
    } else {
      VS_CALL(vs_gemm(&g, stream));
      VS_CALL(vs_layernorm_bwd_dt(hdt, M, D, G->d_h, D, L->y, D, L->mean2, L->rstd2, L->ln2_g, G->dx_out, D, G->dy,
                                  D, lp ? G->dy_lp : nullptr, G->ln2_g, G->ln2_b, G->ln_ws, stream));
    }
  }
  // ---- attention: y = x + o Wp^T + bp
  VS_CALL(fork(2));  // dy ready
  {  // [side] dWp[D,D] += dy^T o;  dbp += colsum(dy) fused
    vs_gemm_desc g = gdesc(T, VS_F32, false, false, D, D, M, gy, D, L->attn_o, D, G->w_proj, D, VS_EPI_ATOMIC);
    TimerTag tag(VS_TIMER_DW_PROJ);
    g.a_rowsum = G->b_proj;
    g.workspace = G->gemm_ws;
    g.workspace_bytes = G->gemm_ws_bytes;
    VS_CALL(vs_gemm(&g, side));
    VS_CALL(mark(2));
  }
  {  // do = dy Wp
    vs_gemm_desc g = gdesc(T, T, true, false, M, D, D, gy, D, L->w_proj, D, G->d_o, D, 0);
    TimerTag tag(VS_TIMER_DX_PROJ);
    VS_CALL(vs_gemm(&g, stream));
  }
  VS_CALL(wait_prev(3));  // d_qkv is read by the previous block's dWqkv
  VS_CALL(vs_attn_bwd(T, L->batch, L->tokens, L->heads, 64, L->qkv, 3 * D, L->attn_o, D, G->d_o, D, L->lse, G->d_qkv,
                      3 * D, G->attn_ws, L->attn_scale, stream));
  VS_CALL(fork(3));  // dqkv ready
  {  // [side] dWqkv[3D,D] += dqkv^T h1;  d(q,k,v bias) += colsum(dqkv) fused
    vs_gemm_desc g = gdesc(T, VS_F32, false, false, 3 * D, D, M, G->d_qkv, 3 * D, L->h1, D, G->w_qkv, D, VS_EPI_ATOMIC);
    TimerTag tag(VS_TIMER_DW_QKV);
    g.a_rowsum = G->b_qkv;
    g.workspace = G->gemm_ws;
    g.workspace_bytes = G->gemm_ws_bytes;
    VS_CALL(vs_gemm(&g, side));
    // the k bias is not a parameter (fixed 0 in the reference, mv:233): its slot stays exactly 0
    hipError_t e = hipMemsetAsync(G->b_qkv + D, 0, D * sizeof(float), ss);
    if (e != hipSuccess) return (int)e;
    VS_CALL(mark(3));
  }
  // dh1 = dqkv Wqkv;  dx = dy + LN1'(dh1)  (one launch, as above)
  VS_CALL(wait_prev(0));  // dx_in is the previous block's dx_out, read by its dW2
  {
    const int hdt = (G->flags & VS_BWD_FUSE_LN) || dh_f32() ? VS_F32 : T;  // bf16 dh1, as dh2 above
    vs_gemm_desc g = gdesc(T, hdt, true, false, M, D, 3 * D, G->d_qkv, 3 * D, L->w_qkv, D, G->d_h, D, 0);
    TimerTag tag(VS_TIMER_DX_QKV);
    if (G->flags & VS_BWD_FUSE_LN) {
      VS_CALL(vs_gemm_ln_bwd(&g, L->x_in, D, L->mean1, L->rstd1, L->ln1_g, G->dy, D, G->dx_in, D,
                             lp ? G->dx_in_lp : nullptr, G->ln1_g, G->ln1_b, G->ln_ws, stream));
    } else {
      VS_CALL(vs_gemm(&g, stream));
      VS_CALL(vs_layernorm_bwd_dt(hdt, M, D, G->d_h, D, L->x_in, D, L->mean1, L->rstd1, L->ln1_g, G->dy, D,
                                  G->dx_in, D, lp ? G->dx_in_lp : nullptr, G->ln1_g, G->ln1_b, G->ln_ws, stream));
    }
  }
  if (!ch) return VS_OK;
  if (G->flags & VS_BWD_DEFER_JOIN) {
    ch->pending = 0xF;  // the next block waits on ce[] before each overwrite
    ch->parity = 1 - par;
  } else if (G->flags & VS_BWD_DEFER_LAST) {
    // join dW2, dW1, dWp (finished during the attention backward, so this wait does not stall);
    // only dWqkv, still running beside dh1 + LN1', is joined by the next block before its
    // attention backward overwrites d_qkv
    VS_CALL((int)hipStreamWaitEvent(ms, ce[2], 0));
    ch->pending = 0x8;
    ch->parity = 1 - par;
  } else {
    VS_CALL(stream_wait(ss, ms, ev[4]));  // join: the block's weight gradients are complete
    ch->pending = 0;
  }
  return VS_OK;
}

extern "C" int vs_bwd_chain_create(void** chain) {
  VS_REQUIRE(chain, "vs_bwd_chain_create: null out pointer");
  *chain = nullptr;
  BwdChain* c = new BwdChain();
  hipError_t e = hipGetDevice(&c->device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking);
  for (int i = 0; i < 16 && e == hipSuccess; ++i) e = hipEventCreateWithFlags(&c->ev[i], hipEventDisableTiming);
  if (e != hipSuccess) {
    vs_bwd_chain_destroy(c);
    return (int)e;
  }
  *chain = c;
  return VS_OK;
}

extern "C" int vs_bwd_chain_destroy(void* chain) {
  BwdChain* c = (BwdChain*)chain;
  if (!c) return VS_OK;
  int dev = -1;
  (void)hipGetDevice(&dev);
  if (dev != c->device) (void)hipSetDevice(c->device);
  // work still queued on the side stream keeps running: destroy returns without waiting, and
  // HIP releases the stream and events once their pending work has completed
  for (auto& x : c->ev)
    if (x) (void)hipEventDestroy(x);
  if (c->side) (void)hipStreamDestroy(c->side);
  if (dev >= 0 && dev != c->device) (void)hipSetDevice(dev);
  delete c;
  return VS_OK;
}
