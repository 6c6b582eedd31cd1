/*
 * cullavo_capi.h — the C-ABI of libcullavo_hip.so, the MI355X (gfx950) kernels behind the
 * CuLLaVO forward/backward hot path.
 *
 * Boundary rules:
 *   - plain pointers, sizes and scalars only; no torch / HIP types in the signatures;
 *   - every function is stream-ordered on the `stream` argument (a hipStream_t passed as void*,
 *     normally torch.cuda.current_stream().cuda_stream) and never allocates, frees or syncs:
 *     scratch is passed in by the caller (sizes from the *_workspace() helpers);
 *   - every function returns 0 on success or a CULLAVO_E* code; cullavo_last_error() returns
 *     the message of the last failure on the calling thread. The Python wrappers raise
 *     RuntimeError / ValueError from these, mirroring the reference's ValueError for a bad
 *     feature-select strategy (reference cullavo/arch_cullavo.py:595-597).
 *
 * Each entry point names the reference computation it replaces (reference = the
 * LTTTDH/Causal-Unified-Language-Vision tree; "tf:" = the HuggingFace transformers modules the
 * reference reaches through cullavo/arch_cullavo.py:582-665).
 * Layout conventions: activations are row-major [rows, cols] with a leading dimension in
 * elements; "tokens" = batch * sequence rows.
 */
#ifndef CULLAVO_CAPI_H
#define CULLAVO_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- dtypes / codes ------------------------------------------------------------------- */
#define CULLAVO_DT_F32 0
#define CULLAVO_DT_BF16 1

#define CULLAVO_OK 0
#define CULLAVO_EINVAL 1       /* bad shape / argument */
#define CULLAVO_EUNSUPPORTED 2 /* dtype or shape the kernels do not implement */
#define CULLAVO_EHIP 3         /* a HIP runtime error (launch failure) */

/* activation codes used by the GEMM epilogue and cullavo_act_bwd */
#define CULLAVO_ACT_NONE 0
#define CULLAVO_ACT_GELU 1       /* erf GELU: LlavaMultiModalProjector act (tf:llava/modeling_llava.py:99) */
#define CULLAVO_ACT_QUICK_GELU 2 /* x*sigmoid(1.702x): CLIPMLP act (tf:activations.py:117-123) */
/* SwiGLU backward fused into the epilogue of the down-projection dX GEMM (LlamaMLP.down_proj
   input gradient, tf:llama/modeling_llama.py:MLP): the product dh [M][N] (rounded to bf16) is not
   stored; with gu = residual [M][2N] (gate | up, ldr >= 2N) C [M][2N] (ldc >= 2N) receives
   dgate | dup exactly as cullavo_swiglu_bwd(dh, gu) writes them. bf16 only, no bias / preact /
   addend / dropout / beta. */
#define CULLAVO_ACT_SWIGLU_BWD 3

/* ABI version: bumped whenever an exported signature changes (2: cullavo_im2col_patches gained
   out_dtype, cullavo_vision_embed_ln dtype, cullavo_gemm_desc f32_operands; 4: the tuning switches
   of the measured-slower GEMM variants removed with them: cullavo_gemm_set_streamk,
   cullavo_gemm_set_prefetch, cullavo_gemm_set_loaders). A consumer built against this header
   checks cullavo_abi_version() == CULLAVO_ABI_VERSION at load. */
#define CULLAVO_ABI_VERSION 4

int cullavo_abi_version(void);
const char* cullavo_last_error(void);

/* ---- GEMM (MFMA bf16, fp32 accumulate) --------------------------------------------------
 * C[M,N] = alpha * sum_k A(m,k) B(k,n)  [+ bias[n]] -> [preact] -> act -> [+ residual] [+ beta*C]
 * a_layout 0: A stored [M,K] (K contiguous, lda >= K)      -- activations
 * a_layout 1: A stored [K,M] (M contiguous, lda >= M)      -- dW = dY^T X
 * b_layout 0: B stored [N,K] (K contiguous, nn.Linear.weight)
 * b_layout 1: B stored [K,N] (N contiguous)                -- dX = dY W
 * N % 8 == 0; K % 8 == 0 unless both layouts are 1; M % 8 == 0 for a_layout 1.
 * Replaces every nn.Linear of CLIP / projector / Llama (tf:clip/modeling_clip.py:280-351,
 * tf:llava/modeling_llava.py:87-107, tf:llama/modeling_llama.py:163-282, lm_head :480) and their
 * autograd backward. A,B,residual,bias,preact are bf16; C is bf16 or f32 (c_dtype).
 * Rounding follows the reference's bf16 module chain: pre = bf16(acc+bias); out = bf16(act(pre));
 * with a residual: out = bf16(out + residual). beta accumulates into C: C = out + beta*C
 * (gradient accumulation into the parameter-gradient arena). */
int cullavo_gemm(int a_layout, int b_layout, int64_t M, int64_t N, int64_t K,
                 const void* A, int64_t lda, const void* B, int64_t ldb,
                 void* C, int64_t ldc, int c_dtype, float alpha,
                 const void* bias, int act, void* preact,
                 const void* residual, int64_t ldr, float beta, void* stream);

/* Extended GEMM for LoRA adapters (peft LoraLayer.forward on a Linear: base(x) +
 * lora_B(lora_A(dropout(x))) * scaling; reference
 * cullavo/load_cullavo.py:94-112). Everything cullavo_gemm takes, plus
 *   addend [M, N] bf16 (ld_addend, multiple of 4, nullable): added after the bias with the
 *           module chain's roundings, v = round(round(alpha*A.B^T + bias) + addend), before
 *           preact / activation / residual;
 *   drop_operand: 0 none; 1 dropout on A (needs a_layout 0, A[m][k] = x[token m][feature k]);
 *           2 on B (needs b_layout 1, B[k][n] = x[token k][feature n]); 3 on the output
 *           (token m, feature n), applied to alpha*A.B^T before bias / beta;
 *   drop_p in [0, 1), drop_seed: one hash(seed, token, feature / 2) per feature pair; element
 *           kept iff its 16-bit half (even feature: low, odd: high) >= round(drop_p * 2^16), kept
 *           values scaled by 1/(1-drop_p) (csrc/common.h drop_row / drop_pair / drop_keep).
 * Operand dropout runs on the register-staged 128x128 kernel. Products whose tile grid cannot
 * fill the GPU but whose K is long (the adapters' r = 64 GEMMs) run split-K when a workspace of
 * cullavo_gemm_workspace(desc) bytes is passed: f32 partials, reduced in a fixed order. */
typedef struct {
  int a_layout, b_layout;
  int64_t M, N, K;
  const void* A;
  int64_t lda;
  const void* B;
  int64_t ldb;
  void* C;
  int64_t ldc;
  int c_dtype;
  float alpha;
  const void* bias;
  int act;
  void* preact;
  const void* residual;
  int64_t ldr;
  float beta;
  const void* addend;
  int64_t ld_addend;
  int drop_operand;
  float drop_p;
  uint64_t drop_seed;
  void* workspace;          /* nullable: split-K f32 partials (size: cullavo_gemm_workspace) */
  int64_t workspace_bytes;
  int f32_operands;         /* 0 (default): A, B, bias, residual, preact, addend bf16;
                               1: every operand and C f32, nothing rounded (the f32 parity
                               mode: an exact f32 MFMA chain, v_mfma_f32_16x16x4_f32) */
  /* ABI 3: the LoRA up-projection fused into the base product (nullable lora_u). For output
   * column n of module m = n / lora_out the kernel adds t = round(lora_scale * u_m . B[n]) with
   * u_m = lora_u[row][m*64 .. m*64+63] (row stride ld_lora_u) and B[n] = lora_b[n][0..63]
   * (the group's lora_B weights stacked, [N, 64]), exactly where `addend` would be added (the
   * same roundings: v = round(round(alpha*A.B^T + bias) + t)); t is never written to memory.
   * Needs a_layout = b_layout = 0, bf16 operands and output, lora_r = 64, lora_out a multiple of
   * 256 dividing N, no addend / dropout / beta, M > 16; otherwise CULLAVO_EUNSUPPORTED. */
  const void* lora_u;
  int64_t ld_lora_u;
  const void* lora_b;
  int64_t lora_out;
  int lora_r;
  float lora_scale;
} cullavo_gemm_desc;
int cullavo_gemm_ex(const cullavo_gemm_desc* desc, void* stream);
/* sizeof(cullavo_gemm_desc) as compiled into the library (binding check) */
size_t cullavo_gemm_desc_size(void);
/* bytes of split-K workspace cullavo_gemm_ex would use for this problem (0: no split) */
size_t cullavo_gemm_workspace(const cullavo_gemm_desc* desc);

/* LoRA adapters' input gradient through their dropout, one launch per adapter group (peft
 * LoraLayer backward, reference cullavo/load_cullavo.py:94-112):
 *   for m = 0 .. n_mod-1 in order: dx = bf16(dx + mask_m / (1 - drop_p) * (du_m A_m))
 * du [M, ld_du] bf16 holds module m's du in columns m*64 .. m*64+63; a_stack [n_mod*64, ld_a] bf16
 * holds lora_A.weight of module m in rows m*64 ..; dx [M, ld_dx] bf16 is accumulated in place;
 * mask_m is the dropout hash of seed_m (csrc/common.h drop_keep, as cullavo_gemm_ex's
 * drop_operand 3). Bitwise the n_mod per-module cullavo_gemm_ex launches (layouts (0,1), K = 64,
 * drop_operand 3, beta 1) it replaces, in one pass over dx. 1 <= n_mod <= 3, N % 8 == 0. */
int cullavo_lora_dx(int n_mod, int64_t M, int64_t N, const void* du, int64_t ld_du, const void* a_stack,
                    int64_t ld_a, void* dx, int64_t ld_dx, float drop_p, uint64_t seed0, uint64_t seed1,
                    uint64_t seed2, void* stream);

/* Kernel-shape selection for cullavo_gemm: -1 = automatic (default), 0 = 128x128 tile /
 * 4 waves (register staged), 2 = 256x256 / 8 waves, 3 = 192x256 / 8 waves, 10 = 288x256 / 8 waves
 * (LDS-DMA staged; 3 and 10 fall back to 2 when A is not K-contiguous; 10 is chosen automatically
 * only for K >= 2048). Other values select automatic. The measured-slower variants of earlier
 * rounds (ping-pong / 8-phase, BK = 32 4-stage, 256x128, other loader waves, the round-5 4-wave
 * 256x256 kernel) are not in the library (ABI 4; tools/lab).
 * Returns the previous mode. For tests and tuning; not thread-safe. */
int cullavo_gemm_set_tile(int mode);
/* Per-tile rate (TFLOP/s) the automatic kernel-shape choice assumes for tile mode 2, 3 or 10
   (its time model: FLOPs / rate x whole rounds of tiles over the CUs); rate <= 0 removes the
   shape from the automatic choice (0 on mode 10 = round-2 behaviour). *previous (nullable)
   receives the old rate. Tuning/A-B switch; not thread-safe. */
int cullavo_gemm_set_tile_rate(int mode, float tflops, float* previous);
/* M-tail split of the automatic plan (tuning/A-B switch, 1 = on, the default): when M is just past
   a multiple of the chosen tile height, the head rows run on that tile in whole rounds and the
   remaining rows as a second, thin product (split over K when cullavo_gemm_workspace sized the
   caller's workspace for it). 2 (the default since round 6) = split wherever the plan's model
   estimates a gain; 1 = only where it estimates >= 5 % (round 5). Returns the previous setting. */
int cullavo_gemm_set_msplit(int on);
/* Tile order of the 8-wave kernels (tuning/A-B switch): > 0 = groups of that many M-tiles
   sweep the N-tiles, < 0 = groups of -group N-tiles sweep the M-tiles (default -4); each XCD
   walks a contiguous run of the order. 0 leaves the setting. Returns the previous setting. */
int cullavo_gemm_set_group(int group);
/* Split-K plan of the small-grid GEMMs (tuning/A-B switch): the number of blocks a split-K
   launch aims for (default 512 = two 4-wave blocks per CU); out-of-range values leave it.
   Returns the previous setting. */
int cullavo_gemm_set_splitk_target(int blocks);
/* Tuning/A-B switch. Bit 0: 1 (default) = the 8-wave kernels stage their epilogue through LDS
   and store 16-B groups of 8 columns; 0 = per-lane 8-B stores straight from the MFMA layout.
   Bit 1: C is written with non-temporal (streaming) stores. Bits 2 / 3 / 4 (round 5, A/B): send
   the LDS epilogue's lean bias/residual, plain-output and activation / SwiGLU-backward paths to
   the general per-option path (same values). Bit 5: no persistent forward kernel. Round 6, A/B
   (same values): bit 6 keeps the SwiGLU-backward dX on the general epilogue path instead of its
   prefetching instantiation; bit 7 keeps the LDS-staged epilogue for the lean cases instead of
   the direct (register, 16-B buffer store) epilogue and its persistent forward kernel; bit 8 opts
   into the persistent 288-row direct forward kernel at K >= 2048 and N > 2048 (elsewhere it is the
   default);
   bit 9 keeps the plan off 288-row tiles at K < 2048 (round 5's plan; the default takes them).
   Returns the previous setting. */
int cullavo_gemm_set_epilogue(int lds_staged);
/* Tuning/A-B switch for the 8-wave 256-row kernels: 1 = per-lane LDS-DMA source offsets
   computed once per tile and the K advance passed as the scalar offset (used when K % 64 == 0
   or the operand is stored [K][rows], layout 1; the default); 0 = offsets recomputed per
   K-tile. Same results either way. Returns the previous setting. */
int cullavo_gemm_set_dma(int precomputed);
/* Tuning/A-B switch for the decode product (plan 14, cullavo_decode_linear): 1 = the weight
   fragments are read with non-temporal loads (each weight byte is read once per token step), 0 =
   default cache policy. Same results either way. Returns the previous setting. */
int cullavo_gemv_set_nt(int on);
/* The kernel shape cullavo_gemm will use for this problem (return value, as above) and its
 * number of workgroups (*grid, nullable) — lets profilers match dispatches to GEMM calls.
 * 9 = the 8-wave 256x256 kernel split over K (a grid of at most half the CUs with >= 32
 * K-tiles, both M and N >= 256): used by cullavo_gemm_ex when the caller passes the workspace
 * cullavo_gemm_workspace() asks for; f32 partials [splits][M][N], reduced in split order
 * (deterministic) with the full epilogue. cullavo_gemm itself (no workspace) never splits.
 * 14 = the weight-streaming decode product (gemv.hip: M <= 16 rows, a_layout = b_layout = 0,
 * automatic tile mode, no dropout): one 8-wave workgroup per 16 rows of B, no workspace.
 * 100 + t = the M-tail split (cullavo_gemm_set_msplit): the first rows in whole rounds of tile
 * mode t (*grid = that launch's workgroups), the remaining rows as a second product, split over
 * K only when the caller passes the workspace cullavo_gemm_workspace() asks for (cullavo_gemm_ex;
 * cullavo_gemm runs them unsplit). */
int cullavo_gemm_plan(int64_t M, int64_t N, int64_t K, int a_layout, int b_layout, int64_t* grid);

/* ---- norms -------------------------------------------------------------------------------
 * LlamaRMSNorm (tf:llama/modeling_llama.py:53-70): fp32 statistics, y = w * bf16(x*rstd).
 * rstd: [rows] f32 saved for backward. cols % 8 == 0, cols <= 8192. */
int cullavo_rmsnorm_fwd(const void* x, const void* w, void* y, float* rstd, int64_t rows,
                        int64_t cols, float eps, int dtype, void* stream);
/* dx (dtype) and optionally dw (w_dtype, nullable; beta accumulates into dw) */
int cullavo_rmsnorm_bwd(const void* dy, const void* x, const void* w, const float* rstd, void* dx,
                        const void* dres, void* dw, int w_dtype, float beta, float* workspace,
                        int64_t rows, int64_t cols, int dtype, void* stream);
/* A/B switch for the bf16/f32 RMSNorm backward with dw at <= 4096 columns: 1 (default) = the
   pipelined one-workgroup-per-CU kernel (next rows' loads in flight under the current rows), 0 = the
   round-1 kernel (two waves per row). Both are deterministic; they add a row's dot-product
   partials and dw's partial rows in different fixed orders. Returns the previous mode. */
int cullavo_rmsnorm_set_bwd(int mode);
/* nn.LayerNorm (CLIP pre_layrnorm / layer_norm1/2, tf:clip/modeling_clip.py:353-384,642).
 * mean/rstd: [rows] f32 saved for backward. The backwards add an optional residual-stream
 * gradient dres (nullable) into dx, fusing the residual branch join. */
int cullavo_layernorm_fwd(const void* x, const void* w, const void* b, void* y, float* mean,
                          float* rstd, int64_t rows, int64_t cols, float eps, int dtype,
                          void* stream);
int cullavo_layernorm_bwd(const void* dy, const void* x, const void* w, const float* mean,
                          const float* rstd, void* dx, const void* dres, void* dw, void* db,
                          int w_dtype, float beta, float* workspace, int64_t rows, int64_t cols,
                          int dtype, void* stream);
/* bytes of f32 workspace the norm backward needs for the weight-gradient partials */
size_t cullavo_norm_bwd_workspace(int64_t rows, int64_t cols);

/* ---- element-wise ------------------------------------------------------------------------ */
/* LlamaMLP act: out = silu(gate) * up  (tf:llama/modeling_llama.py:163-176). gu is the fused
 * gate|up projection output [rows, 2F] (gate in columns [0,F), up in [F,2F)); out [rows, F].
 * The backward writes dgu [rows, 2F] in the same fused layout. */
int cullavo_swiglu_fwd(const void* gu, int64_t rows, int64_t F, void* out, int dtype,
                       void* stream);
int cullavo_swiglu_bwd(const void* dout, const void* gu, int64_t rows, int64_t F, void* dgu,
                       int dtype, void* stream);
/* dst[c, r] = src[r, c] for a 16-bit matrix (bf16/fp16) [rows, cols], leading dims in elements.
 * Keeps a K-major copy of a Linear weight W [N, K] so that the input gradient dx = dy @ W
 * (reference: autograd of F.linear, tf:llama/modeling_llama.py:163-176 / :281-300) runs with
 * both GEMM operands reduction-contiguous. rows, cols, ld_src, ld_dst must be multiples of 8. */
int cullavo_transpose16(const void* src, int64_t ld_src, void* dst, int64_t ld_dst, int64_t rows,
                        int64_t cols, void* stream);
/* dx = dy * act'(preact) for CULLAVO_ACT_GELU / CULLAVO_ACT_QUICK_GELU */
int cullavo_act_bwd(int act, const void* dy, const void* preact, void* dx, int64_t n, int dtype,
                    void* stream);
/* out[c] = beta*out[c] + sum_r x[r,c] (bias gradients); out dtype = out_dtype */
int cullavo_colsum(const void* x, int64_t rows, int64_t cols, void* out, int out_dtype,
                   float beta, float* workspace, int dtype, void* stream);
size_t cullavo_colsum_workspace(int64_t rows, int64_t cols);
/* Llama rotary embedding, rotate_half form (tf:llama/modeling_llama.py:73-160), in place on
 * q [tokens, hq*D] and k [tokens, hk*D] (row strides ldq, ldk). inv_freq = theta^(-2i/D);
 * cos/sin of pos*inv_freq are computed in f32 and rounded to bf16 as the reference does.
 * inverse=1 applies the transpose rotation (the backward). */
int cullavo_rope(void* q, int64_t ldq, void* k, int64_t ldk, const int64_t* position_ids,
                 int64_t tokens, int hq, int hk, int head_dim, float theta, int inverse,
                 int dtype, void* stream);
/* The decode step's RoPE fused with the KV-cache append (reference: the cached branch of
 * tf:llama LlamaAttention.forward, rotary embedding then DynamicCache.update): cullavo_rope's
 * forward rotation on q (in place) and k, the rotated k written to k_cache row start[b] + t % Lnew
 * of sequence b = t / Lnew (token stride ld_tok, batch stride ld_b) instead of back into k, and v
 * copied to v_cache there -- bitwise cullavo_rope followed by cullavo_kv_append. bf16, head_dim a
 * multiple of 16, 16-byte aligned rows. */
int cullavo_rope_kv_append(void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                           const int64_t* position_ids, int64_t tokens, int hq, int hk, int head_dim,
                           float theta, void* k_cache, void* v_cache, int64_t ld_tok, int64_t ld_b,
                           const int32_t* start, int Lnew, int dtype, void* stream);

/* ---- attention (flash-style, MFMA bf16) --------------------------------------------------
 * Replaces tf:llama/modeling_llama.py:191-282 (causal, D=128, FA2 in the reference,
 * cullavo/load_cullavo.py:72) and tf:clip/modeling_clip.py:280-336 (non-causal, D=64).
 * q,k,v,o: [B, L, H, D] with token stride ld* elements (head h at column h*D).
 * lse: [B, H, Lq] f32 natural-log log-sum-exp of the scaled scores (saved for backward).
 * kv_start: nullable int32 [B]: keys < kv_start[b] are masked (left padding).
 * D in {64, 128}; Lq == Lk when causal. */
int cullavo_attn_fwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v,
                     int64_t ldv, void* o, int64_t ldo, float* lse, int B, int H, int Lq, int Lk,
                     int D, float scale, int causal, const int32_t* kv_start, int dtype,
                     void* stream);
/* delta workspace: [B, H, Lq] f32 (= rowsum(dO*O)); dq,dk,dv same layout as q,k,v */
int cullavo_attn_bwd(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v,
                     int64_t ldv, const void* o, int64_t ldo, const void* dout, int64_t lddo,
                     const float* lse, float* delta, void* dq, int64_t lddq, void* dk,
                     int64_t lddk, void* dv, int64_t lddv, int B, int H, int Lq, int Lk, int D,
                     float scale, int causal, const int32_t* kv_start, int dtype, void* stream);
/* cullavo_attn_bwd with a scratch buffer: in mode 7 the dK/dV kernel stores dS^T (bf16,
   [B*H][round_up(Lk,128)][round_up(Lq,128)]) there and dQ is one product over it instead of
   a recompute of S and dP; workspace_bytes below what cullavo_attn_bwd_workspace returns (or
   a null workspace) falls back to mode 4. Caller-owned, stream-ordered like every buffer. */
int cullavo_attn_bwd_ws(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v,
                        int64_t ldv, const void* o, int64_t ldo, const void* dout, int64_t lddo,
                        const float* lse, float* delta, void* dq, int64_t lddq, void* dk,
                        int64_t lddk, void* dv, int64_t lddv, int B, int H, int Lq, int Lk, int D,
                        float scale, int causal, const int32_t* kv_start, int dtype, void* workspace,
                        size_t workspace_bytes, void* stream);
/* bytes of workspace cullavo_attn_bwd_ws uses for this problem in the current mode (0: none) */
size_t cullavo_attn_bwd_workspace(int B, int H, int Lq, int Lk, int D, int dtype);
/* Tuning/A-B switch for cullavo_attn_bwd: 4 = the 8-wave dK/dV kernel (two waves per SIMD;
   waves w and w+4 split each query tile and add their partial sums once, in a fixed order)
   with the 4-wave 32-key dQ kernel; 0-3 = the 4-wave kernels; 7 = mode 4's dK/dV
   kernel storing dS^T + dQ from it (needs the cullavo_attn_bwd_ws workspace); -1 (the default) = 7 for D=128 (4 through cullavo_attn_bwd, which has no workspace), 2 for
   D=64 (measured per head dim).
   In 0-3 with bit 0 = 64 query rows per dK/dV barrier, bit 1 = 64
   keys per dQ barrier (else 32) -- results bitwise identical across 0-3 (same products summed
   in the same order). Modes 5, 6 and 8 (measured slower: both kernels 8-wave, 64 keys per wave,
   the software-pipelined mode-7 pair; profiles/r02/attn/, profiles/r04/attn/) were removed in
   round 5. Other values leave the mode unchanged. Returns the previous mode. */
int cullavo_attn_set_bwd_tiles(int mode);
/* A/B switch for the attention forward's K/V tile staging: 2 = 16-B buffer loads
   through a per-tile scalar descriptor (one loop-invariant lane offset, rows past the sequence
   end zero-filled by the range check), 1 = buffer loads with per-chunk offsets and range selects,
   0 = pointer loads behind a per-chunk bounds branch, 3 = mode 2 with the two MFMA blocks of a
   K/V tile at raised wave priority (s_setprio; A/B experiment), 4 = K/V tiles by
   LDS-DMA (buffer_load ... lds) straight into the swizzled LDS image (no staging registers, no
   ds_write), 5 = mode 4 with the K and V^T fragment reads as inline-asm groups of 4 under
   counted lgkmcnt waits (the next group in flight while the current one's MFMAs issue), 7 = the
   software-pipelined kernel (tile t's softmax in the issue gaps of tile t+1's S MFMAs, K / V in
   rings of their own), -1 (the default) = 7.
   Results are identical. Other
   values leave the setting; returns the previous setting. Not thread-safe. */
int cullavo_attn_set_stage(int buffer_loads);
/* A/B switch for the backward's tile staging, three bits: bit 0 = the 8-wave dK/dV kernel's
   (modes 4, 5, 7) Q / dO tiles, bit 1 = the mode-7 dQ kernel's K / dS^T tiles by LDS-DMA
   straight into the swizzled image (else through registers and ds_write); the default is 1
   (round 5: with LDS-DMA staging the dK/dV kernel's fragment reads are inline asm, one step ahead
   of the MFMAs). Bit 2 (round 6, head dim 128): the mode-7 dQ kernel as a 4-stage LDS-DMA ring,
   one workgroup per CU with three 64-key tiles in flight (takes precedence over bit 1). Bit 3
   (round 6): the dS^T workspace blocked by 128-query column blocks (a dQ tile is one contiguous
   16 KiB run instead of 64 rows of 256 B). Results are identical. Other values leave the setting; returns the previous one. */
int cullavo_attn_set_bwd_stage(int mode);
/* Attention forward's deferred rescale (guide T13): the running row max and the O / l rescale
   move only on K/V tiles where some row's max grew by more than `threshold` (log2 units, in
   [0, 16]; default 8: softmax weights stay <= 2^8 against the stale max, LSE exact). 0 = rescale
   whenever a max grows, bitwise the plain online softmax. Synchronous (device symbol copy);
   *previous (nullable) receives the old threshold. */
int cullavo_attn_set_rescale(float threshold, float* previous);

/* ---- KV-cache decode (generate) --------------------------------------
 * Cache per layer: K, V [B, Lmax, H*D] bf16, token stride ld_tok, batch stride ld_batch.
 * kv_append copies Lnew new rows per batch (k/v: [B*Lnew, hd] with row strides) into cache
 * rows start[b] .. start[b]+Lnew-1. attn_decode: one query row per batch (q [B, H*D], ldq)
 * against cache keys kv_start[b] <= key < kv_len[b] (kv_start nullable); max_len >= every
 * kv_len sizes the split over keys; workspace: cullavo_attn_decode_workspace bytes (f32).
 * A row with no visible key returns zeros (as the training kernel's fully masked rows). */
/* One decode step's RoPE + KV append + attention in one pass (ABI 4, additive): bitwise
 * cullavo_rope_kv_append(q, k, v, position_ids, ..., Lnew = 1) followed by cullavo_attn_decode
 * with kv_len = start + 1, except that q (the unrotated projection row, [B, >=H*D]) is only read:
 * the rotated key and the value of row start[b] are written to the caches, every chunk rotates its
 * query itself. Workspace: cullavo_attn_decode_workspace(B, H, max_len, D) bytes. */
int cullavo_attn_decode_rope(const void* q, int64_t ldq, const void* k, int64_t ldk, const void* v, int64_t ldv,
                             const int64_t* position_ids, float theta, void* k_cache, void* v_cache, int64_t ld_tok,
                             int64_t ld_batch, const int32_t* start, const int32_t* kv_start, void* o, int64_t ldo,
                             int B, int H, int max_len, int D, float scale, float* workspace, void* stream);
int cullavo_kv_append(const void* k, int64_t ldk, const void* v, int64_t ldv, void* k_cache, void* v_cache,
                      int64_t ld_tok, int64_t ld_batch, const int32_t* start, int B, int Lnew, int64_t hd,
                      void* stream);
/* Decode-step Linear over M <= 16 rows (one token per sequence; reference: the cached forward's
 * decoder layer, cullavo/arch_cullavo.py:605-636) with its input transform fused into the weight
 * stream (csrc/gemv.hip): y[M,N] = X W^T (+ residual), W [N,K] bf16 (ldw), where X is
 *   x_transform 0: x [M,K] as given;
 *   1: RMSNorm(x; norm_w, eps) of x [M,K] (the residual stream: replaces cullavo_rmsnorm_fwd
 *      + cullavo_gemm, the values bitwise those of cullavo_rmsnorm_fwd; every workgroup normalises
 *      the rows once into LDS, so M (K + 8) * 2 <= 65536 bytes);
 *   2: SwiGLU of x = gate|up [M,2K] (replaces cullavo_swiglu_fwd + cullavo_gemm, bitwise).
 * x_transform 3 transforms the OUTPUT instead: W holds 2N rows (gate rows, then up rows: the
 *   fused gate|up weight [2N, K]) and y[M,N] = SwiGLU(x W^T), i.e. cullavo_gemm's bf16 gate|up
 *   product followed by cullavo_swiglu_fwd, bitwise, in one launch (no residual);
 *   4 = 1 and 3 together: SwiGLU(RMSNorm(x) W^T).
 * bf16 only; the result is rounded like cullavo_gemm's (residual added after rounding). */
int cullavo_decode_linear(int x_transform, int64_t M, int64_t N, int64_t K, const void* x, int64_t ldx,
                          const void* norm_w, float eps, const void* W, int64_t ldw, void* y, int64_t ldy,
                          const void* residual, int64_t ldr, void* stream);
size_t cullavo_attn_decode_workspace(int B, int H, int max_len, int D);
int cullavo_attn_decode(const void* q, int64_t ldq, const void* k_cache, const void* v_cache, int64_t ld_tok,
                        int64_t ld_batch, const int32_t* kv_len, const int32_t* kv_start, void* o, int64_t ldo,
                        int B, int H, int max_len, int D, float scale, float* workspace, void* stream);

/* ---- image preprocessing (data step) --------------------------------
 * Replaces the CLIPImageProcessor call inside the reference's prompt builders
 * (cullavo/arch_cullavo.py:82,313,516): PIL-bicubic resize of the shortest edge, center crop,
 * rescale, normalise -> pixel_values, bit-identical to the CPU processor.
 * cullavo_resample_coeffs (host only, no GPU): Pillow's precompute_coeffs + 8-bit normalisation
 * for in_size -> out_size; writes bounds[2*out_size] (first source index, tap count) and
 * kk[out_size*ksize] (22-bit fixed point); returns ksize (or the ksize alone when bounds or kk
 * is NULL); bad sizes return CULLAVO_EINVAL (1) like every other entry point.
 * cullavo_clip_image_preprocess: images uint8 [B, C<=3, H, W] at element strides sb/sc/sy/sx,
 * resized size Hr x Wr (tables from cullavo_resample_coeffs(W, Wr) and (H, Hr), device copies),
 * crop window (top, left, crop_h, crop_w); tmp: B*C*H*crop_w bytes; out [B, C, crop_h, crop_w]
 * f32 or bf16. */
int cullavo_resample_coeffs(int in_size, int out_size, int32_t* bounds, int32_t* kk, int ksize_cap);
int cullavo_clip_image_preprocess(const uint8_t* images, int B, int C, int H, int W, int64_t sb, int64_t sc,
                                  int64_t sy, int64_t sx, int Hr, int Wr, const int32_t* h_bounds,
                                  const int32_t* h_kk, int h_ksize, const int32_t* v_bounds,
                                  const int32_t* v_kk, int v_ksize, int top, int left, int crop_h,
                                  int crop_w, double rescale, float mean0, float mean1, float mean2,
                                  float std0, float std1, float std2, uint8_t* tmp, void* out,
                                  int out_dtype, void* stream);

/* ---- box drawing (data step: step-1 prompts and step-2 records with boxes) -----------------
 * Replaces detectron2's Visualizer(img); _default_font_size = 16;
 * overlay_instances(boxes=..., assigned_colors=...).get_image() in the reference's prompt builders
 * (cullavo/arch_cullavo.py:149-153, :441-448): the image as a matplotlib Agg canvas shows it
 * (imshow "nearest" on a (W+0.01) x (H+0.01) figure) with one 4 pt, alpha 0.5 stroked Rectangle
 * per box, pixel-identical to matplotlib 3.10.8 (oracle/boxdraw_oracle.py).
 * cullavo_visimage_geometry (host only, no GPU): rows[H] / cols[W] = source pixel of every canvas
 * pixel; trans4 = matplotlib's transData (sx, tx, sy, ty; display y up) for the boxes.
 * cullavo_draw_boxes: images uint8 [B, 3, H, W] at element strides sb/sc/sy/sx; boxes f32
 * [B, max_boxes, 4] (x0, y0, x1, y1 in image pixels) already in draw order (largest area first,
 * np.argsort(-areas) like overlay_instances), nbox[B] boxes used per image; colors uint8
 * [B, max_boxes, 3]; width_px = max(font_size / 4, 1) pt at 100 dpi; alpha8 = round(alpha * 255);
 * workspace of cullavo_draw_boxes_workspace(B, max_boxes) bytes (its first int32 is set non-zero
 * when a box's outline or cells overflow the kernel's fixed capacity); out uint8 [B, 3, H, W]
 * contiguous. W <= 8192. */
int cullavo_visimage_geometry(int H, int W, int32_t* rows, int32_t* cols, double* trans4);
size_t cullavo_draw_boxes_workspace(int B, int max_boxes);
int cullavo_draw_boxes(const uint8_t* images, int B, int C, int H, int W, int64_t sb, int64_t sc, int64_t sy,
                       int64_t sx, const int32_t* rows, const int32_t* cols, const float* boxes,
                       const int32_t* nbox, const uint8_t* colors, int max_boxes, double td_sx, double td_tx,
                       double td_sy, double td_ty, double width_px, int alpha8, void* workspace, uint8_t* out,
                       void* stream);

/* ---- embeddings / merge ------------------------------------------------------------------ */
/* get_input_embeddings()(input_ids) (reference cullavo/arch_cullavo.py:582) */
int cullavo_embedding_fwd(const int64_t* ids, int64_t n, const void* table, int64_t vocab,
                          int64_t dim, void* out, int dtype, void* stream);
/* dtable[v] = beta*dtable[v] + sum_{i: ids[i]==v} dout[i] for every v that occurs in ids;
 * rows that do not occur are left untouched (caller zeroes for beta=0). Deterministic. */
int cullavo_embedding_bwd(const int64_t* ids, int64_t n, const void* dout, int64_t vocab,
                          int64_t dim, void* dtable, int table_dtype, float beta, int dtype,
                          void* stream);
/* CLIP patch embedding front end (tf:clip/modeling_clip.py:202-218): pixels [B,3,H,W] (f32 or
 * bf16 by pix_dtype) -> patches [B*(1+P), kpad] bf16, row b*(1+P) (the CLS slot) all zeros,
 * column order (c, i, j) like Conv2d.weight.reshape(out, -1), zero pad to kpad. */
int cullavo_im2col_patches(const void* pixels, int pix_dtype, int B, int C, int H, int W,
                           int patch, void* out, int64_t kpad, int out_dtype, void* stream);
/* x[b,t] += (t==0 ? cls : 0) + pos[t] then LayerNorm (pre_layrnorm); x: [B*T, dim] (dtype;
 * bf16 rounds the embedding sum like the reference's bf16 add, f32 keeps it exact) */
int cullavo_vision_embed_ln(const void* x, const void* cls, const void* pos, const void* w,
                            const void* b, void* y, int B, int T, int64_t dim, float eps,
                            int dtype, void* stream);
/* The llava _merge_input_ids_with_image_features index plan (transformers ~4.37, called at
 * reference cullavo/arch_cullavo.py:600-602). ids/mask: [B,S]; per text token its merged
 * row, flattened over the batch (text_dst [B,S] = b*L + position, -1 for image tokens; the
 * backward gathers the text gradient with it), per merged row its source (src [B,L]: text row
 * b*S+s, or B*S + image row, or -1 for zero fill), merged mask [B,L] and position_ids [B,L].
 * n_patches = image feature rows per image. Returns CULLAVO_EINVAL when the image-token count
 * does not match n_images (the reference's ValueError). img_count/left_pad from host. */
int cullavo_merge_plan(const int64_t* ids, const int64_t* mask, int B, int S, int L,
                       int64_t image_token, int64_t n_patches, int left_padding,
                       int64_t* text_dst, int64_t* src, int64_t* merged_mask,
                       int64_t* position_ids, void* stream);
/* out[r] = src[r] < 0 ? 0 : (src[r] < n_a ? a[src[r]] : b[src[r]-n_a]), rows of dim */
int cullavo_row_gather2(const int64_t* src, int64_t rows, const void* a, int64_t n_a,
                        const void* b, int64_t dim, void* out, int dtype, void* stream);

/* ---- loss ---------------------------------------------------------------------------------
 * Shifted, attention-masked CE (reference cullavo/arch_cullavo.py:651-665): target for row
 * (b,t) is labels[b,t+1] when t+1 < L and mask[b,t+1] != 0, else -100 (ignored). */
int cullavo_shift_targets(const int64_t* labels, const int64_t* mask, int B, int L,
                          int64_t ignore_index, int64_t* targets, void* stream);
/* per-row loss (0 for ignored rows) and lse; logits [rows, V] bf16 with row stride ldl */
int cullavo_ce_fwd(const void* logits, int64_t ldl, const int64_t* targets, int64_t rows,
                   int64_t V, int64_t ignore_index, float* row_loss, float* row_lse, int dtype,
                   void* stream);
/* loss_out[0] = sum(row_loss)/count, loss_out[1] = count, loss_out[2] = 1/count */
int cullavo_ce_reduce(const float* row_loss, const int64_t* targets, int64_t rows,
                      int64_t ignore_index, float* loss_out, void* stream);
/* dlogits = (softmax - onehot) * grad_loss[0] * loss_out[2] for non-ignored rows, 0 otherwise */
int cullavo_ce_bwd(const void* logits, int64_t ldl, const int64_t* targets, const float* row_lse,
                   const float* loss_out, const float* grad_loss, int64_t rows, int64_t V,
                   int64_t ignore_index, void* dlogits, int64_t ldd, int dtype, void* stream);

/* ---- optimiser -----------------------------------------------------------------------------
 * torch.optim.AdamW semantics (reference trainer/cullavo_trainer.py:12-14) with an optional
 * device-side gradient scale (the clip_grad_norm_ coefficient, reference
 * pipeline/CuLLaVOPipeline.py:90-91). States have state_dtype, params/grads dtype. */
int cullavo_adamw(void* param, const void* grad, void* exp_avg, void* exp_avg_sq, int64_t n,
                  float lr, float beta1, float beta2, float eps, float weight_decay, int64_t step,
                  const float* grad_scale, int dtype, int state_dtype, void* stream);
/* out[0] += sum(grad^2) (f32, device); run over every grad buffer, then cullavo_clip_coef.
 * Deterministic: CULLAVO_SUMSQ_PARTIALS block sums land in the caller's f32 workspace
 * `partials` and one block adds them to out[0] in a fixed order (no float atomics), so the
 * global norm and the clip coefficient are identical run to run, like torch's
 * clip_grad_norm_ (reference pipeline/CuLLaVOPipeline.py:90). */
#define CULLAVO_SUMSQ_PARTIALS 1024
int cullavo_sumsq(const void* x, int64_t n, float* out, float* partials, int dtype, void* stream);
/* coef[0] = min(1, max_norm / (sqrt(sumsq[0]) + 1e-6)); norm_out[0] = sqrt(sumsq[0]) */
int cullavo_clip_coef(const float* sumsq, float max_norm, float* coef, float* norm_out,
                      void* stream);
/* y = x * scale[0] in place (n elements) */
int cullavo_scale_inplace(void* x, int64_t n, const float* scale, int dtype, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CULLAVO_CAPI_H */
