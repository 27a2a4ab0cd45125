/*
 * cp25.h -- C ABI of the MI355X-native cosmos-predict2.5 sampler kernels (libcp25.so, gfx950).
 *
 * This is the drop-in boundary below the reference's Python operator plug points. Each entry point
 * names the reference interface it replaces (paths relative to the reference repository root,
 * cosmos_predict2/_src/predict2/...). The Python side (cosmos-predict2.5_amd/cosmos_predict2/_native.py)
 * binds these with ctypes; INTEGRATION.md shows the binding a reference maintainer would add.
 *
 * Contract for every function:
 *   - pointers are device pointers (HBM); strides and sizes are in ELEMENTS, int64;
 *   - bf16 tensors are passed as void* holding IEEE bfloat16 bits, fp32 tensors as float*;
 *   - the call is stream-ordered on `stream`, never allocates, never synchronises, is re-entrant
 *     and hipGraph-capturable; the caller owns all memory (PyTorch's caching allocator);
 *   - returns 0 (CP25_OK) or a negative code checked on the host before launching:
 *       -22 bad shape/stride/pointer, -95 unsupported dtype/head-dim/width, -5 launch failure.
 */
#ifndef CP25_H
#define CP25_H

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- tensor descriptors
 * SURVEY.md §8(b)5's descriptor form, for the entry points a reference-side binding most often calls with
 * framework tensors: cp25_attn_fwd_t, cp25_gemm_epi_t, cp25_conv3d_t. A descriptor carries the device pointer, the
 * dtype, the rank and per-dimension sizes and strides (in elements). These entry points check every descriptor on
 * the host and return CP25_ERR_DTYPE (-95) for a wrong dtype, CP25_ERR_INVAL (-22) for a rank / shape / stride /
 * pointer mismatch, before any GPU work; then they run the pointer entry point of the same op. The other entry points
 * keep plain pointers plus sizes (INTEGRATION.md §3 gives the reason). */
#define CP25_MAX_DIMS 6
#define CP25_DT_BF16 1
#define CP25_DT_F32 2
#define CP25_DT_F8E4M3 3
#define CP25_DT_U8 4
typedef struct cp25_tensor {
  void* data;                      /* device pointer */
  int32_t dtype;                   /* CP25_DT_* */
  int32_t ndim;                    /* <= CP25_MAX_DIMS */
  int64_t shape[CP25_MAX_DIMS];
  int64_t strides[CP25_MAX_DIMS];  /* elements */
} cp25_tensor;

/* cp25_attn_fwd over descriptors: q / o [B, Lq, H, D], k / v [B, Lk, H, D], bf16, D = 128, unit head-dim stride. With
 * a workspace of at least cp25_attn_workspace_bytes(B, H, Lq, cp25_attn_plan(B, H, Lq, Lk, D)) bytes the planned
 * key-range split runs (cp25_attn_fwd_split), else the unsplit launch. Replaces: networks/attention.py:90-181. */
int cp25_attn_fwd_t(const cp25_tensor* q, const cp25_tensor* k, const cp25_tensor* v, const cp25_tensor* o,
                    float softmax_scale, void* workspace, size_t ws_bytes, hipStream_t stream);

/* cp25_gemm_epi over descriptors: c [M, N] = epi(a [M, K] w [N, K]^T), bf16, unit inner strides; epilogue
 * CP25_EPI_NONE or CP25_EPI_GELU (the other epilogues take more operands: cp25_gemm_res / _hnorm / _qkv).
 * Replaces: block nn.Linear layers, minimal_v4_dit.py:227-254, 354-363, 401-432. */
int cp25_gemm_epi_t(const cp25_tensor* a, const cp25_tensor* w, const cp25_tensor* c, int epilogue,
                    hipStream_t stream);

/* cp25_conv3d over descriptors: x [T, Hin, Win, Cin] channels-last frames (each contiguous, any frame stride) after
 * pad_front zero frames (the causal padding), weight [Cout, KT, KH, KW, Cin], bias [Cout] or NULL, out contiguous
 * [Tout, Ho, Wo, Cout] whose sizes must match the conv's, all bf16. Replaces: CausalConv3d.forward
 * (tokenizers/wan2pt1.py:44-62). */
int cp25_conv3d_t(const cp25_tensor* x, int pad_front, const cp25_tensor* weight, const cp25_tensor* bias,
                  const cp25_tensor* out, int stride_t, int stride_hw, int pad_top, int pad_left, int pad_bottom,
                  int pad_right, hipStream_t stream);

/* ---------------------------------------------------------------- attention
 * softmax(Q K^T * softmax_scale) V, non-causal, no mask; bf16 in/out, fp32 accumulation.
 * q: [B, Lq, H, D] addressed by q_strides = {batch, token, head} (head dim contiguous), same for
 * k/v ([B, Lk, H, D]) and o ([B, Lq, H, D]). D must be 128. All strides multiples of 8 elements.
 * Replaces: networks/attention.py:90-181 `attention()` as called by MinimalA2AAttnOp
 * (networks/a2a_cp.py:208-219) for self-attention (minimal_v4_dit.py:431) and cross-attention
 * (minimal_v4_dit.py:1216-1226; Lk = 512 text tokens). */
int cp25_attn_fwd(const void* q, const void* k, const void* v, void* o, int B, int H, int Lq, int Lk, int D,
                  const int64_t* q_strides, const int64_t* k_strides, const int64_t* v_strides,
                  const int64_t* o_strides, float softmax_scale, hipStream_t stream);

/* Key-range split ("split-KV") form of cp25_attn_fwd, same arguments and result: each (b, h, 256-query
 * block) is processed by n_split workgroups over consecutive key ranges of ceil(ceil(Lk/64)/n_split)
 * 64-key tiles, which write fp32 partial outputs + log-sum-exp into `workspace`
 * (>= cp25_attn_workspace_bytes(B, H, Lq, n_split) bytes, 16-B aligned), merged into o by a second,
 * stream-ordered launch. Used where B*H*ceil(Lq/256) workgroups would leave the last round of CUs
 * mostly idle (a context-parallel shard's queries against the gathered keys, a head chunk of the
 * K/V all-gather pipeline). n_split = 1 is cp25_attn_fwd. Same reference interface as cp25_attn_fwd;
 * the split is the MI355X work decomposition, the result equals the unsplit softmax up to fp32/bf16
 * rounding. */
int cp25_attn_fwd_split(const void* q, const void* k, const void* v, void* o, int B, int H, int Lq, int Lk, int D,
                        const int64_t* q_strides, const int64_t* k_strides, const int64_t* v_strides,
                        const int64_t* o_strides, float softmax_scale, int n_split, void* workspace,
                        size_t ws_bytes, hipStream_t stream);

/* cp25_attn_fwd_split with caller-supplied upper bounds of the query and key norms:
 * q_norm_bound >= max |q| and k_norm_bound >= max |k| over all rows (0 = unknown). Softmax is shift invariant, so a
 * row's shift only has to keep its terms inside the fp32 / bf16 range. When both bounds are given and
 * b = q_norm_bound * k_norm_bound * softmax_scale * log2(e) <= 98, every score of a row lies in [-b_row, b_row]
 * (Cauchy-Schwarz, b_row from the row's own |q|) and the row uses the fixed shift max(b_row - 96, 0): no max
 * reduction and no output rescale per key tile, the row's largest term >= 2^-100 and every term <= 2^96. Otherwise (or with a 0 bound) the
 * rows run an online max (tile 0 sets the shift to the row max; later tiles move it up, rescaling O and the sum, only
 * when a row max exceeds it by more than 24): any data. Same result as cp25_attn_fwd_split up to rounding. The DiT
 * passes sqrt(D) * max|q_norm.weight| and sqrt(D) * max|k_norm.weight|: the q/k RMSNorm (minimal_v4_dit.py:355-358)
 * bounds every normed row by them and RoPE preserves the norm. */
int cp25_attn_fwd_bounded(const void* q, const void* k, const void* v, void* o, int B, int H, int Lq, int Lk,
                          int D, const int64_t* q_strides, const int64_t* k_strides, const int64_t* v_strides,
                          const int64_t* o_strides, float softmax_scale, float q_norm_bound, float k_norm_bound,
                          int n_split, void* workspace, size_t ws_bytes, hipStream_t stream);

/* cp25_attn_fwd_bounded over a PRE-SCALED q (rows already multiplied by softmax_scale * log2(e), e.g. by
 * cp25_head_rmsnorm_rope_scaled): P = exp2(q k^T - shift) with the row's shift as the initial accumulator of its
 * Q K^T MFMA chains, so no per-score multiply or subtract. Bounds (of the scaled q and of k; 0 = unknown) pick the
 * shift as in cp25_attn_fwd_bounded: product <= 96 no shift, <= 98 a fixed per-row shift, else the online max.
 * Rounds q * scale to bf16 instead of q (the same single bf16 rounding of the query). Replaces the same reference
 * code as cp25_attn_fwd_bounded; the DiT's default form. */
int cp25_attn_fwd_prescaled(const void* q, const void* k, const void* v, void* o, int B, int H, int Lq, int Lk, int D,
                            const int64_t* q_strides, const int64_t* k_strides, const int64_t* v_strides,
                            const int64_t* o_strides, float q_norm_bound, float k_norm_bound, int n_split,
                            void* workspace, size_t ws_bytes, hipStream_t stream);

/* cp25_attn_fwd_prescaled with a data-tight key bound in device memory: the max of k_norm_slots[32 i], i < n_slots
 * (n_slots <= 64; the [64][32] buffer cp25_head_rmsnorm_rope_nmax filled on k) bounds |k| over all keys. Where the host bounds already
 * allow the zero shift (product <= 96) this is cp25_attn_fwd_prescaled. Otherwise the same grid is launched twice
 * (stream-ordered, no host synchronisation): a 256-query block whose own bound max|q_row| max|k| is <= 96 runs the
 * zero-shift loop in the first launch, any other block the online max in the second, so trained q/k norm weights
 * (whose weight-based bounds exceed 96) keep the fast loop wherever the data allows. A row's mode depends on its
 * block, so context-parallel shards must not use this form when they need bit-identical rows. Same reference op as
 * cp25_attn_fwd_bounded. */
int cp25_attn_fwd_prescaled_kslots(const void* q, const void* k, const void* v, void* o, int B, int H, int Lq, int Lk,
                                   int D, const int64_t* q_strides, const int64_t* k_strides, const int64_t* v_strides,
                                   const int64_t* o_strides, float q_norm_bound, float k_norm_bound,
                                   const float* k_norm_slots, int n_slots, int n_split, void* workspace,
                                   size_t ws_bytes, hipStream_t stream);

/* cp25_attn_fwd_prescaled (k_norm_slots NULL) / _kslots with the query normalisation done in the kernel: q holds the
 * raw q projection (the QKV GEMM output) and every workgroup applies cp25_head_rmsnorm_rope's arithmetic to its Q
 * fragments as they load: the per-head RMSNorm over 128 (q_norm_weight [128] bf16, eps), the rotate-half RoPE of
 * the row's token (cos_tab / sin_tab [Lq][64] fp32, indexed by the query row; both NULL: none) and the factor
 * q_scale (the softmax scale * log2 e of the prescaled form), with the same partial-sum order and roundings, so the
 * output equals cp25_head_rmsnorm_rope_scaled followed by cp25_attn_fwd_prescaled bit for bit, without that
 * pass over q in HBM (Attention.compute_qkv's q_norm + apply_rotary_pos_emb, minimal_v4_dit.py:401-419, then
 * attention(), networks/attention.py:90-181). Per-block kernel forms only (a short-key launch that would take the
 * persistent form runs one workgroup per query block instead). */
int cp25_attn_fwd_prescaled_qnorm(const void* q, const void* k, const void* v, void* o, int B, int H, int Lq, int Lk,
                                  int D, const int64_t* q_strides, const int64_t* k_strides, const int64_t* v_strides,
                                  const int64_t* o_strides, float q_norm_bound, float k_norm_bound,
                                  const float* k_norm_slots, int n_slots, const void* q_norm_weight,
                                  const float* cos_tab, const float* sin_tab, float eps, float q_scale, int n_split,
                                  void* workspace, size_t ws_bytes, hipStream_t stream);

/* dst[r, c] = OCP e4m3(bf16 src[r, c] * scale) (saturated to +-448, round to nearest even), row strides in
 * elements; width % 16 == 0. The fixed-scale fp8 copies of q and k for cp25_attn_fwd_prescaled_fp8qk. */
int cp25_cast_fp8_e4m3(const void* src, int64_t src_stride, void* dst, int64_t dst_stride, int64_t n_rows,
                       int64_t width, float scale, hipStream_t stream);

/* The config-5 fp8 option's attention: cp25_attn_fwd_prescaled (zero shift: bound product <= 60) with q and k given
 * as OCP e4m3 (one byte per
 * element; strides in elements = bytes, multiples of 16): q8 = e4m3(q * softmax_scale * log2(e) * 2^s),
 * k8 = e4m3(k * 2^-s) (cp25_cast_fp8_e4m3; the power-of-two scales cancel in q k^T, so no per-score multiply
 * returns). Q K^T runs on v_mfma_f32_32x32x64_f8f6f4; P and V stay bf16, o is bf16. The bounds are those of
 * the scaled bf16 rows, as for cp25_attn_fwd_prescaled. No reference counterpart (the reference has no fp8
 * path); replaces the same attention call. */
int cp25_attn_fwd_prescaled_fp8qk(const void* q8, const void* k8, const void* v, void* o, int B, int H, int Lq, int Lk,
                                  int D, const int64_t* q_strides, const int64_t* k_strides, const int64_t* v_strides,
                                  const int64_t* o_strides, float q_norm_bound, float k_norm_bound, int n_split,
                                  void* workspace, size_t ws_bytes, hipStream_t stream);

/* V for the fp8 P.V of cp25_attn_fwd_prescaled_fp8: v_amax[b * H + h] = max |v| over the head's L rows (float,
 * device memory, B * H entries), then v8t = e4m3(v * 448 / amax) laid out [B][H][ceil(L / 64)][128 d][64 key
 * bytes], the keys of each 64-key tile permuted to the order the kernel's P^T operand holds them (zero keys pad
 * the last tile). v: bf16 [B, L, H, 128] by element strides (e.g. the v columns of the fused qkv buffer). Two
 * HBM passes over v, no host synchronisation. cp25_v_fp8t_bytes gives the v8t size. */
int64_t cp25_v_fp8t_bytes(int B, int H, int L);
int cp25_cast_v_fp8t(const void* v, const int64_t* v_strides, int B, int H, int L, int D, void* v8t, float* v_amax,
                     hipStream_t stream);

/* The config-5 fp8 option's whole attention: cp25_attn_fwd_prescaled_fp8qk's e4m3 Q K^T, then O^T += V^T P^T on
 * v_mfma_f32_32x32x64_f8f6f4 with P = exp2(S - shift) as e5m2 (shift = max(0, 1.13 q_norm_bound k_norm_bound - 15)
 * keeps every P <= 2^15, inside e5m2, whatever the data) and V^T from cp25_cast_v_fp8t's v8t (O rescaled by
 * amax / 448 at the end). The softmax stays fp32 with no per-score multiply and no running max. Requires
 * 1.13 q_norm_bound k_norm_bound <= 30 (the window [2^-15, 2^15] then holds a term of every row unless the row's
 * scores all sit at the bottom of the bound; such a row is written as zeros, never NaN); CP25_ERR_INVAL otherwise.
 * o bf16. No reference counterpart; replaces the same attention call. */
int cp25_attn_fwd_prescaled_fp8(const void* q8, const void* k8, const void* v8t, const float* v_amax, void* o, int B,
                                int H, int Lq, int Lk, int D, const int64_t* q_strides, const int64_t* k_strides,
                                const int64_t* o_strides, float q_norm_bound, float k_norm_bound, int n_split,
                                void* workspace, size_t ws_bytes, hipStream_t stream);

/* Name of the kernel form cp25_attn_fwd_bounded (prescaled = 0, fp8 = 0), _prescaled (prescaled = 1), _prescaled_kslots
 * (prescaled = 2),
 * _prescaled_fp8qk (fp8 = 1) or _prescaled_fp8 (fp8 = 2) launches for these arguments (a static string), e.g.
 * "attn_fwd_m16<self, prescaled, online max>": what a bench or log reports as the kernel that ran. */
const char* cp25_attn_kernel(int Lk, float softmax_scale, float q_norm_bound, float k_norm_bound, int prescaled,
                             int fp8);

/* Bytes of workspace cp25_attn_fwd_split / _bounded need (0 for n_split <= 1). */
size_t cp25_attn_workspace_bytes(int B, int H, int Lq, int n_split);

/* Bytes of workspace with which an unsplit (n_split = 1) bf16 self-attention launch of _split / _bounded / _prescaled
 * (Lk > 4096, no key-norm slots) runs its last, partial round of workgroups as a tail split: the first
 * (nwg - nwg % CUs) query blocks as one launch of whole rounds, the remaining ones as key-range splits merged into o
 * (the split launches' arithmetic). 0 when the shape has no such tail or it would not pay. Passing less (or no
 * workspace) runs the launch whole, as one grid. */
size_t cp25_attn_tail_workspace_bytes(int B, int H, int Lq, int Lk);

/* The key-range split the library picks for this shape on the current device (>= 1; a round model of
 * one workgroup per CU), or a negative error code. */
int cp25_attn_plan(int B, int H, int Lq, int Lk, int D);

/* Kernel form of the short-key (Lk <= 4096: the text cross-attention, minimal_v4_dit.py:1216-1226) launches of
 * cp25_attn_fwd / _bounded / _prescaled: 1 (default) the persistent form (one workgroup per CU walking a run of
 * query blocks as one K/V tile stream, the next block's Q staged through LDS; unsplit launches in the zero-shift or
 * online modes with Lk > 64), 0 one workgroup per query block. Both forms are bit-identical. Returns the previous
 * form, or CP25_ERR_INVAL for another value. */
int cp25_attn_cross_select(int form);

/* ---------------------------------------------------------------- DiT block elementwise
 * Activations are token-major [n_tok, B, D] bf16 (batch inner). Row (tok, b) uses modulation row
 * (b, t) with t = (tok0 + tok) / hw (frame index; tok0 = first global token of this CP shard).
 *
 * cp25_ln_mod: if y != NULL first x' = x + gate * y (two bf16 roundings, stored to x_out [n_tok,B,D]);
 * then h_out = LayerNorm(x', no affine, eps) * (1 + scale) + shift with the reference's bf16
 * rounding after every torch op. x is read as x[tok * x_st + b * x_sb] (x_sb = 0 broadcasts one
 * row to every batch entry). gate/shift/scale: bf16, element (b, t, d) at b*mod_sb + t*mod_st + d.
 * D in {512, 1024, 2048, 4096, 5120}.
 * Replaces: Block.forward _fn + gated residuals, minimal_v4_dit.py:1171-1179, 1204, 1237, 1246. */
int cp25_ln_mod(const void* x, int64_t x_st, int64_t x_sb, const void* y, const void* gate, const void* shift,
                const void* scale, int64_t mod_sb, int64_t mod_st, void* x_out, void* h_out, int64_t n_tok, int B,
                int D, int64_t tok0, int64_t hw, float eps, hipStream_t stream);

/* cp25_ln_mod with h emitted as the fp8 operand of the next GEMM (config 5's fp8 option): h8_out
 * [n_tok * B, D] OCP E4M3 and h_scale [n_tok * B] fp32, exactly cp25_quant_fp8_rows applied to the bf16 h
 * cp25_ln_mod would write (which is not written). Same replaced reference code as cp25_ln_mod. */
int cp25_ln_mod_fp8(const void* x, int64_t x_st, int64_t x_sb, const void* y, const void* gate, const void* shift,
                    const void* scale, int64_t mod_sb, int64_t mod_st, void* x_out, void* h8_out, float* h_scale,
                    int64_t n_tok, int B, int D, int64_t tok0, int64_t hw, float eps, hipStream_t stream);

/* Final layer prologue under the reference's fp32 autocast: [x' = x + gate*y (bf16)], then
 * out = LayerNorm_fp32(x') * (1 + scale) + shift in fp32 (shift/scale fp32).
 * Replaces: FinalLayer.forward, minimal_v4_dit.py:974-991 (and the last block's MLP residual :1246). */
int cp25_final_ln_mod(const void* x, const void* y, const void* gate, int64_t gmod_sb, int64_t gmod_st,
                      const float* shift, const float* scale, int64_t mod_sb, int64_t mod_st, float* out,
                      int64_t n_tok, int B, int D, int64_t tok0, int64_t hw, float eps, hipStream_t stream);

/* Affine LayerNorm of n_rows bf16 rows (row stride x_stride / y_stride elements, multiples of 8; 16-B aligned
 * pointers): y = (x - mean) * rstd * weight + bias in fp32 with fp32 statistics, one bf16 rounding (nn.LayerNorm with
 * elementwise_affine on bf16). D in {512, 1024, 2048, 4096, 5120}.
 * Replaces: MultiViewCrossBlock.layer_norm_cross_view_attn, predict2_multiview/networks/multiview_cross_dit.py:290,
 * :441. */
int cp25_layer_norm(const void* x, int64_t x_stride, const void* weight, const void* bias, void* y, int64_t y_stride,
                    int64_t n_rows, int D, float eps, hipStream_t stream);

/* In-place per-head RMSNorm (weight[128] bf16, eps) of heads [head_off, head_off + H*128) of every
 * row of a bf16 [n_rows, row_stride] buffer, then (if cos_tab != NULL) rotate-half RoPE in fp32
 * with cos/sin tables [n_tok, 64] fp32 indexed by token = row / B, result rounded to bf16.
 * If out2 != NULL the result is also written to out2[row * out2_stride + h*128 + d].
 * Replaces: Attention.compute_qkv norm + TE RoPE + attention() recast, minimal_v4_dit.py:410-420,
 * networks/attention.py:107-109. */
int cp25_head_rmsnorm_rope(void* buf, int64_t row_stride, int64_t n_rows, int B, int H, int head_off,
                           const void* weight, const float* cos_tab, const float* sin_tab, void* out2,
                           int64_t out2_stride, float eps, hipStream_t stream);

/* cp25_head_rmsnorm_rope with the result multiplied by out_scale (fp32) before its bf16 rounding: the
 * fp8 option's q = q * softmax_scale * log2(e), so its attention needs no per-score multiply
 * (cp25_attn_fwd_prescaled). out_scale = 1 is cp25_head_rmsnorm_rope exactly. */
int cp25_head_rmsnorm_rope_scaled(void* buf, int64_t row_stride, int64_t n_rows, int B, int H, int head_off,
                                  const void* weight, const float* cos_tab, const float* sin_tab, void* out2,
                                  int64_t out2_stride, float eps, float out_scale, hipStream_t stream);

/* cp25_head_rmsnorm_rope_scaled that also measures the result: the 64 slots norm_max_slots[32 i] (a float [64][32]
 * buffer in device memory, zeroed by the caller; slots one 128-B line apart so the atomics spread over L2 channels)
 * receive, by atomic max, the largest |row| (L2 norm over a head's 128 bf16 values as written) of the call (the max
 * of the 64 is the max over all rows and heads). For k, that is the data-tight key bound
 * cp25_attn_fwd_prescaled_kslots reads; NULL slots: cp25_head_rmsnorm_rope_scaled. */
int cp25_head_rmsnorm_rope_nmax(void* buf, int64_t row_stride, int64_t n_rows, int B, int H, int head_off,
                                const void* weight, const float* cos_tab, const float* sin_tab, void* out2,
                                int64_t out2_stride, float eps, float out_scale, float* norm_max_slots,
                                hipStream_t stream);

/* dst[r, 0:width] = src[r, 0:width] for bf16 rows (K/V export before the CP all-gather). */
int cp25_copy_rows(const void* src, int64_t src_stride, void* dst, int64_t dst_stride, int64_t n_rows, int64_t width,
                   hipStream_t stream);

/* In-place exact (erf) GELU on n bf16 values (n % 8 == 0).
 * Replaces: GPT2FeedForward activation, minimal_v4_dit.py:249-254. */
int cp25_gelu(void* x, int64_t n, hipStream_t stream);

/* fp32 linear layers: C[b][M, N] = act(A[b][M, K] W[b][N, K]^T + R[b][M, N]) in fp32 on v_mfma_f32_16x16x4_f32 (fp32
 * operands, products and sums). Batch entry b's matrices at a + b * a_batch_stride (etc.); A / W / C row-major with
 * leading dims lda / ldw / ldc (floats; lda, ldw and the A / W batch strides multiples of 4, a / w 16-B aligned). R
 * (NULL: none) at r + b * r_batch_stride + row * ldr + col: ldr = 0 is a bias vector, r_batch_stride = 0 one addend
 * for every entry. act 0: none, 1: SiLU (x * sigmoid(x)) after the addend. K % 32 == 0 (-95 otherwise), any M / N,
 * batch <= 65535. Launches with few tiles (the 62-row conditioning GEMMs) split K over several workgroups when a
 * workspace of cp25_gemm_f32_workspace_floats(M, N, K, batch) floats is given (partial sums, then a second pass adds
 * them in slice order, then R and act); with none, or a smaller one, one slice runs. The slice plan depends only on
 * the shape: a given shape always sums in the same order. Without a workspace an output row's sum does not depend on
 * M (the final linear passes none: a context-parallel shard's rows equal the whole sequence's, bit for bit).
 * Replaces the fp32 F.linear calls of the reference's fp32 conditioning (use_wan_fp32_strategy,
 * minimal_v4_dit.py): TimestepEmbedding linear_1 + SiLU and linear_2 (:727-788), the blocks' AdaLN-LoRA
 * modulation Linear(D, A) / Linear(A, 3D) + the LoRA term (:1136-1154; all 3 x num_blocks sub-layers as one GEMM and
 * one batched GEMM), the final layer's AdaLN (:974-991) and its Linear(D, p p C) (:993-995). */
int cp25_gemm_f32(const float* a, int64_t lda, int64_t a_batch_stride, const float* w, int64_t ldw,
                  int64_t w_batch_stride, const float* r, int64_t ldr, int64_t r_batch_stride, float* c, int64_t ldc,
                  int64_t c_batch_stride, int M, int N, int K, int batch, int act, float* workspace,
                  int64_t workspace_floats, hipStream_t stream);
int64_t cp25_gemm_f32_workspace_floats(int M, int N, int K, int batch);

/* ---------------------------------------------------------------- block projections (GEMM + epilogue)
 * C[M, N] = epi(A[M, K] W[N, K]^T): A, W, C bf16 row-major with leading dims lda / ldw / ldc (elements,
 * multiples of 8, pointers 16-B aligned), fp32 accumulation, one bf16 rounding of the product.
 * epilogue CP25_EPI_NONE: C = bf16(A W^T); CP25_EPI_GELU: C = bf16(gelu_erf(bf16(A W^T))), the same
 * arithmetic as cp25_gelu on the stored product. N must be a multiple of 256 and K of 64 (-95 otherwise:
 * the caller keeps its library GEMM for other shapes); any M.
 * Replaces: the block nn.Linear layers (no bias) of networks/minimal_v4_dit.py -- Attention q/k/v/
 * output projections (:354-363, :401-404, :432; the DiT runs q|k|v as one fused [3D, D] weight) and
 * GPT2FeedForward layer1 + exact GELU (:227-254, CP25_EPI_GELU) and layer2. */
#define CP25_EPI_NONE 0
#define CP25_EPI_GELU 1
#define CP25_EPI_RES 2
#define CP25_EPI_HNORM 3
#define CP25_EPI_QKV 4
int cp25_gemm_epi(const void* a, int64_t lda, const void* w, int64_t ldw, void* c, int64_t ldc, int M, int N, int K,
                  int epilogue, hipStream_t stream);

/* cp25_gemm_epi with the per-head q RMSNorm as the epilogue (CP25_EPI_HNORM): every 128-column head of each output row
 * of bf16(A W^T) normalised over its 128 values (norm_weight [128] bf16, eps) and multiplied by out_scale, with the
 * partial sums, butterfly and roundings of cp25_head_rmsnorm_rope (no RoPE): bit-identical to cp25_gemm_epi followed
 * by cp25_head_rmsnorm_rope_scaled on the output, one HBM pass fewer. Replaces the cross-attention's q_proj + q_norm
 * (minimal_v4_dit.py:401-404, :411-419; the text cross-attention has no RoPE). K / 64 must be even (else
 * CP25_ERR_DTYPE: run the two ops). */
int cp25_gemm_hnorm(const void* a, int64_t lda, const void* w, int64_t ldw, void* c, int64_t ldc, int M, int N, int K,
                    const void* norm_weight, float eps, float out_scale, hipStream_t stream);

/* The fused q|k|v projection with the k columns' per-head RMSNorm + 3D RoPE in the epilogue (CP25_EPI_QKV): output
 * columns [k_col0, k_col0 + k_cols) (multiples of 256) get cp25_head_rmsnorm_rope's arithmetic with k_norm_weight
 * [128] bf16, eps and the rotate-half RoPE of token row / B (cos_tab / sin_tab [M / B][64] fp32; both NULL: none),
 * the other columns are bf16(A W^T): bit-identical to cp25_gemm_epi followed by cp25_head_rmsnorm_rope on the k
 * columns, one HBM pass over k fewer (Attention.compute_qkv's k_proj + k_norm + RoPE, minimal_v4_dit.py:401-419).
 * K / 64 must be even (else CP25_ERR_DTYPE: run the two ops). */
int cp25_gemm_qkv(const void* a, int64_t lda, const void* w, int64_t ldw, void* c, int64_t ldc, int M, int N, int K,
                  int k_col0, int k_cols, const void* k_norm_weight, const float* cos_tab, const float* sin_tab, int B,
                  float eps, hipStream_t stream);

/* cp25_gemm_epi with the block's gated residual as the epilogue: C = bf16(x + bf16(gate * bf16(A W^T))), the two
 * bf16 roundings of the reference's `x + gate * y` (cp25_ln_mod's residual, bit for bit). Output row r is token
 * tok = r / B, batch entry b = r % B of a token-major [n_tok, B, N] activation (B divides 16); x element
 * (tok, b, col) at x + tok * x_st + b * x_sb + col (x_sb = 0 broadcasts one row over the batch), gate element
 * (b, frame, col) at gate + b * g_sb + frame * g_st + col with frame = (tok0 + tok) / hw (tok0 = the CP shard's first
 * token; hw >= 16 / B). All strides multiples of 8 elements, 16-B aligned bases. C may not alias x. The next cp25_ln_mod then
 * runs with y = NULL on C.
 * Replaces: the gated residuals of Block.forward (minimal_v4_dit.py:1204, :1237, :1246) fused into the output
 * projection (:432), the cross-attention output projection and GPT2FeedForward layer2 (:227-254). */
int cp25_gemm_res(const void* a, int64_t lda, const void* w, int64_t ldw, void* c, int64_t ldc, int M, int N, int K,
                  const void* x, int64_t x_st, int64_t x_sb, const void* gate, int64_t g_sb, int64_t g_st, int B,
                  int64_t tok0, int64_t hw, hipStream_t stream);

/* The config-5 fp8 option's block projections on the same hand-written GEMM (no reference counterpart: the reference
 * has no fp8 path): C[M, N] = bf16((A[M, K] W[N, K]^T) * a_scale[m] * w_scale[n]) with A and W OCP e4m3 bytes
 * (row-scaled activations from cp25_ln_mod_fp8 / cp25_quant_fp8_rows / cp25_gelu_quant_fp8; per-output-channel weight
 * scales), fp32 accumulation on v_mfma_scale_f32_16x16x128_f8f6f4 -- torch._scaled_mm's definition with row / column
 * scales. N % 256 == 0, K % 256 == 0 (-95 otherwise), lda / ldw multiples of 16 bytes, any M. cp25_gemm_fp8_res adds
 * cp25_gemm_res's gated-residual epilogue (same x / gate arguments).
 * Replaces: the block nn.Linear layers of minimal_v4_dit.py (:400-432, :227-254) in the fp8 option. */
int cp25_gemm_fp8(const void* a, int64_t lda, const float* a_scale, const void* w, int64_t ldw, const float* w_scale,
                  void* c, int64_t ldc, int M, int N, int K, hipStream_t stream);
int cp25_gemm_fp8_res(const void* a, int64_t lda, const float* a_scale, const void* w, int64_t ldw,
                      const float* w_scale, void* c, int64_t ldc, int M, int N, int K, const void* x, int64_t x_st,
                      int64_t x_sb, const void* gate, int64_t g_sb, int64_t g_st, int B, int64_t tok0, int64_t hw,
                      hipStream_t stream);

/* Latents live in "patch layout" [n_tok, 64] fp32, element (tok, p*16 + c), p = p1*2 + p2 (the
 * final layer's "(p1 p2 t C)" order). cp25_patchify builds the x_embedder input rows [n_tok, 72]
 * bf16 (feature c*4 + p): channels 0..15 = gt*mask + x*(1-mask) (gt may be NULL), channel 16 = the
 * per-frame condition mask, channel 17 = padding mask (pad_mask [n_tok, 4] bf16 or NULL = 0).
 * Replaces: video2world_model_rectified_flow.py:105-107, minimal_v1_lvg_dit.py:46,
 * minimal_v4_dit.py:1547-1554 and PatchEmbed's rearrange (:873-878). */
int cp25_patchify(const float* xs, const float* gt, const float* frame_mask, const void* pad_mask, void* out,
                  int64_t n_tok, int64_t tok0, int64_t hw, hipStream_t stream);

/* cp25_patchify into rows of out_ld elements (out_ld >= 72, a multiple of 8), columns 72 .. out_ld - 1 zeroed: with
 * out_ld = 128 the rows are the K = 128 operand of the own GEMM (cp25_gemm_epi) against the x_embedder weight
 * zero-padded to 128 columns, the same sums as K = 72. */
int cp25_patchify_ld(const float* xs, const float* gt, const float* frame_mask, const void* pad_mask, void* out,
                     int64_t out_ld, int64_t n_tok, int64_t tok0, int64_t hw, hipStream_t stream);

/* v_out[tok, j] from the final-layer output net [n_tok, B, 64] fp32 (B = 1 or 2 = cond, uncond):
 * per branch v_b = (noise - gt) * mask + net_b * (1 - mask) (skipped if gt == NULL), then
 * cfg_mode 0: v = v_c + guidance (v_c - v_u)   (Video2World, video2world_model_rectified_flow.py:209)
 * cfg_mode 1: v = v_u + guidance (v_c - v_u)   (Text2World, text2world_model_rectified_flow.py:511)
 * Replaces: Video2WorldModelRectifiedFlow.denoise :131-136, velocity_fn :206-210, MiniTrainDIT.unpatchify. */
int cp25_cfg_velocity(const float* net, int B, const float* noise, const float* gt, const float* frame_mask,
                      float guidance, int cfg_mode, float* v_out, int64_t n_tok, int64_t tok0, int64_t hw,
                      hipStream_t stream);

/* ---------------------------------------------------------------- UniPC sampler update
 * Host-computed fp32 coefficients of one FlowUniPCMultistepScheduler.step. */
typedef struct cp25_unipc_params {
  float sigma;      /* sigmas[step_index] */
  int use_corr;     /* corrector active */
  int order_c;      /* 1 or 2 */
  float c_a, c_b, c_c, c_inv_rk, c_rho0, c_rho_last;
  int order_p;      /* 1 or 2 */
  float p_a, p_b, p_c, p_inv_rk, p_rho0;
} cp25_unipc_params;

/* One fused, bit-exact UniPC step over n fp32 elements, in place on x (sample), m0/m1 (the two
 * converted model outputs of the history) and last (last_sample); v = the velocity prediction.
 * Replaces: FlowUniPCMultistepScheduler.step elementwise math, models/fm_solvers_unipc.py:266-335,
 * 337-464, 466-601, 630-713. */
int cp25_unipc_step(float* x, const float* v, float* m0, float* m1, float* last, int64_t n,
                    const cp25_unipc_params* params, hipStream_t stream);

/* ---------------------------------------------------------------- Wan2.1 VAE
 * Activations are channels-last frames [H][W][C] bf16.
 *
 * cp25_conv3d: implicit-GEMM convolution out[to] = sum_{kt,kh,kw,ci} W[co][kt][kh][kw][ci] *
 * in(frame to*stride_t + kt)[hi][wi][ci] + bias[co] (fp32 accumulation, bf16 output), then
 * (if residual != NULL) out = out + residual (bf16 add). `frames` is a table of n_frames (<= 24)
 * frame pointers [Hin][Win][Cin]; a NULL entry is a zero frame (causal padding). Spatial: pad_top /
 * pad_left / pad_bottom / pad_right zeros, stride_hw; upsample=1 first nearest-upsamples the input 2x.
 * out: [Tout][Ho][Wo][Cout]; with out_split = c > 0 (Cout == 2c) output channel co >= c goes to frame
 * 2*to + 1, channel co - c (the upsample3d time_conv interleave), out being [2*Tout][Ho][Wo][c].
 * Cin % 16 == 0 (pad channels on the host). Weight layout [Cout][KT][KH][KW][Cin] bf16.
 * Replaces: CausalConv3d.forward (tokenizers/wan2pt1.py:44-62), Resample convs (:96-110, :133-145,
 * :159), ResidualBlock shortcut + residual add (:204, :222), AttentionBlock to_qkv / proj (:236-261),
 * WanVAE_ conv1 / conv2 (:494-495). */
int cp25_conv3d(const void* const* frames, int n_frames, const void* weight, const void* bias, const void* residual,
                void* out, int Hin, int Win, int Cin, int Cout, int Tout, int KT, int KH, int KW, int stride_t,
                int stride_hw, int pad_top, int pad_left, int pad_bottom, int pad_right, int upsample, int out_split,
                hipStream_t stream);

/* Kernel choice of cp25_conv3d for the 3x3 stride-1 convs: 0 (default) the LDS-halo kernel where it applies, 1 the
 * per-tap implicit GEMM everywhere (A/B runs and tests; same arithmetic up to summation order), 2 the round-2 halo
 * kernel with 4 waves per workgroup (one per SIMD; bit-identical to 0, which runs 8). Returns the previous mode. The
 * initial mode is read once at library load from CP25_CONV_KERNEL ("tap" = 1). */
int cp25_conv3d_select(int mode);

/* y = F.normalize(x, dim=C) * sqrt(C) * gamma [then SiLU] per pixel of n_pix channels-last pixels,
 * with the reference's bf16 rounding after each torch op. C % 32 == 0, C/32 in {1,2,3,6,12}.
 * Replaces: RMS_norm.forward (+ nn.SiLU) in ResidualBlock / head / AttentionBlock (wan2pt1.py:65-77,
 * :195-203, :235, :313-315, :413). */
int cp25_rms_norm_silu(const void* x, const void* gamma, void* y, int64_t n_pix, int C, int do_silu,
                       hipStream_t stream);

/* o = softmax(q k^T * scale) v per frame, one head of D = 384 (the Wan VAE AttentionBlock), bf16 in / out, fp32
 * scores and sums, bf16 P. q [T][Lq][D], k / v [T][Lk][D], o [T][Lq][D] given as base pointers with row strides
 * (ld*) and frame strides (f*) in elements (multiples of 8, 16-B aligned bases), so q / k / v can be column
 * slices of the to_qkv output [T][L][3D]. Flash kernel (no score matrix in HBM): one pass over the keys with the
 * softmax shift fixed at the first key tile's row max; a query block whose later scores exceed it by more than 2^24
 * is redone by a second launch with the exact row max of all keys. Replaces F.scaled_dot_product_attention in
 * AttentionBlock.forward (tokenizers/wan2pt1.py:225-261, q, k, v = [b*t, 1, h*w, c]). Returns CP25_ERR_DTYPE for
 * D != 384. `workspace` (cp25_vae_attn_workspace_bytes(T, Lq, Lk, D) bytes, 16-B aligned, required) holds the
 * per-block redo flags and, when the query blocks do not cover the GPU and the keys are split over several
 * workgroups, their partials, merged by a further kernel on the same stream. */
int64_t cp25_vae_attn_workspace_bytes(int T, int Lq, int Lk, int D);
int cp25_vae_attn(const void* q, int64_t ldq, int64_t fq, const void* k, int64_t ldk, int64_t fk, const void* v,
                  int64_t ldv, int64_t fv, void* o, int64_t ldo, int64_t fo, int T, int Lq, int Lk, int D, float scale,
                  void* workspace, int64_t workspace_bytes, hipStream_t stream);

/* p[r, :] = softmax(s[r, :] * scale) for `rows` rows of `cols` fp32 scores (row stride ld_s elements)
 * -> bf16 probabilities (row stride ld_p); vector loads/stores when rows are 16-B / 8-B aligned. The
 * round-1 VAE AttentionBlock ran S = Q K^T (library GEMM, fp32 out), this kernel, and P V (library GEMM);
 * since round 2 it runs cp25_vae_attn and this entry point is kept for the A/B and its tests. */
int cp25_softmax_rows(const float* s, int64_t rows, int cols, int64_t ld_s, float scale, void* p, int64_t ld_p,
                      hipStream_t stream);

/* fp8 activation operand of the DiT's fp8 linear layers (config 5's "fp8 MFMA"; the GEMM is cp25_gemm_fp8 /
 * cp25_gemm_fp8_res, hand-written; torch._scaled_mm is only the tests' reference). Per row m of x [n_rows, k] bf16 (contiguous, k in {512, 1024, 1536,
 * 2048, 3072, 4096, 5120, 6144, 8192, 20480}): scale[m] = max|x[m, :]| / 448 and q[m, :] = fp8_e4m3(x[m, :] * 448 / max|x[m, :]|)
 * (OCP E4M3, round to nearest even, saturated), so x ~= q * scale; an all-zero row gives q = 0, scale 0.
 * cp25_gelu_quant_fp8 quantises GELU(x) rounded to bf16 (Abramowitz-Stegun 7.1.26 erfc: within ~1 bf16 ulp
 * of cp25_gelu's exact-erf value, far below the fp8 rounding).
 * Replaces: the bf16 operand of nn.Linear in Attention (minimal_v4_dit.py:400-432) and GPT2FeedForward
 * (:227-254, whose GELU it fuses); the reference itself has no fp8 inference path. */
int cp25_quant_fp8_rows(const void* x, void* q, float* scale, int64_t n_rows, int64_t k, hipStream_t stream);
int cp25_gelu_quant_fp8(const void* x, void* q, float* scale, int64_t n_rows, int64_t k, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* CP25_H */
