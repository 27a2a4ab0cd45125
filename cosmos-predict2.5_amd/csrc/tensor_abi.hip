// Tensor-descriptor entry points (SURVEY.md §8(b)5's `cp25_tensor` form) for the attention, the block GEMM and the VAE
// conv: each validates dtype, rank, shape agreement and strides on the host, returns CP25_ERR_DTYPE (-95) for a wrong
// dtype and CP25_ERR_INVAL (-22) for a bad shape / stride / pointer before anything touches the GPU, then forwards to
// the pointer entry point of the same op (include/cp25.h). Host code only; no kernel lives here.
#include "cp25_common.h"

#include <algorithm>

namespace {

// dtype first (so a wrong dtype reports -95 whatever else is wrong), then rank / pointer
int check(const cp25_tensor* t, int dtype, int ndim) {
  if (!t) return CP25_ERR_INVAL;
  if (t->dtype != dtype) return CP25_ERR_DTYPE;
  if (t->ndim != ndim || !t->data) return CP25_ERR_INVAL;
  for (int i = 0; i < ndim; ++i)
    if (t->shape[i] <= 0 || t->strides[i] < 0) return CP25_ERR_INVAL;
  return CP25_OK;
}

}  // namespace

extern "C" int cp25_attn_fwd_t(const cp25_tensor* q, const cp25_tensor* k, const cp25_tensor* v, const cp25_tensor* o,
                               float softmax_scale, void* workspace, size_t ws_bytes, hipStream_t stream) {
  for (const cp25_tensor* t : {q, k, v, o}) {
    const int rc = check(t, CP25_DT_BF16, 4);
    if (rc) return rc;
  }
  const int64_t B = q->shape[0], Lq = q->shape[1], H = q->shape[2], D = q->shape[3], Lk = k->shape[1];
  for (const cp25_tensor* t : {k, v})
    if (t->shape[0] != B || t->shape[1] != Lk || t->shape[2] != H || t->shape[3] != D) return CP25_ERR_INVAL;
  if (o->shape[0] != B || o->shape[1] != Lq || o->shape[2] != H || o->shape[3] != D) return CP25_ERR_INVAL;
  for (const cp25_tensor* t : {q, k, v, o})
    if (t->strides[3] != 1) return CP25_ERR_INVAL;
  if (B > INT32_MAX || Lq > INT32_MAX || Lk > INT32_MAX || H > INT32_MAX) return CP25_ERR_INVAL;
  if (D != 128) return CP25_ERR_DTYPE;
  const int64_t qs[3] = {q->strides[0], q->strides[1], q->strides[2]}, ks[3] = {k->strides[0], k->strides[1], k->strides[2]},
                vs[3] = {v->strides[0], v->strides[1], v->strides[2]}, os[3] = {o->strides[0], o->strides[1], o->strides[2]};
  int n_split = cp25_attn_plan((int)B, (int)H, (int)Lq, (int)Lk, (int)D);
  if (n_split < 1 || !workspace || ws_bytes < cp25_attn_workspace_bytes((int)B, (int)H, (int)Lq, n_split)) n_split = 1;
  return cp25_attn_fwd_split(q->data, k->data, v->data, o->data, (int)B, (int)H, (int)Lq, (int)Lk, (int)D, qs, ks, vs, os,
                             softmax_scale, n_split, n_split > 1 ? workspace : nullptr, n_split > 1 ? ws_bytes : 0,
                             stream);
}

extern "C" int cp25_gemm_epi_t(const cp25_tensor* a, const cp25_tensor* w, const cp25_tensor* c, int epilogue,
                               hipStream_t stream) {
  for (const cp25_tensor* t : {a, w, c}) {
    const int rc = check(t, CP25_DT_BF16, 2);
    if (rc) return rc;
  }
  if (epilogue != CP25_EPI_NONE && epilogue != CP25_EPI_GELU) return CP25_ERR_INVAL;  // the others take more operands
  const int64_t M = a->shape[0], K = a->shape[1], N = w->shape[0];
  if (w->shape[1] != K || c->shape[0] != M || c->shape[1] != N) return CP25_ERR_INVAL;
  if (a->strides[1] != 1 || w->strides[1] != 1 || c->strides[1] != 1) return CP25_ERR_INVAL;
  if (M > INT32_MAX || N > INT32_MAX || K > INT32_MAX) return CP25_ERR_INVAL;
  return cp25_gemm_epi(a->data, a->strides[0], w->data, w->strides[0], c->data, c->strides[0], (int)M, (int)N, (int)K,
                       epilogue, stream);
}

extern "C" int cp25_conv3d_t(const cp25_tensor* x, int pad_front, const cp25_tensor* weight, const cp25_tensor* bias,
                             const cp25_tensor* out, int stride_t, int stride_hw, int pad_top, int pad_left,
                             int pad_bottom, int pad_right, hipStream_t stream) {
  int rc = check(x, CP25_DT_BF16, 4);
  if (!rc) rc = check(weight, CP25_DT_BF16, 5);
  if (!rc && bias) rc = check(bias, CP25_DT_BF16, 1);
  if (!rc) rc = check(out, CP25_DT_BF16, 4);
  if (rc) return rc;
  const int64_t T = x->shape[0], Hin = x->shape[1], Win = x->shape[2], Cin = x->shape[3];
  const int64_t Cout = weight->shape[0], KT = weight->shape[1], KH = weight->shape[2], KW = weight->shape[3];
  if (weight->shape[4] != Cin || (bias && bias->shape[0] != Cout) || out->shape[3] != Cout) return CP25_ERR_INVAL;
  // channels-last frames, each contiguous (the kernel addresses a frame as [Hin][Win][Cin]); weight / bias contiguous
  if (x->strides[3] != 1 || x->strides[2] != Cin || x->strides[1] != Win * Cin) return CP25_ERR_INVAL;
  if (weight->strides[4] != 1 || weight->strides[3] != Cin || weight->strides[2] != KW * Cin ||
      weight->strides[1] != KH * KW * Cin || weight->strides[0] != KT * KH * KW * Cin)
    return CP25_ERR_INVAL;
  if (bias && bias->strides[0] != 1) return CP25_ERR_INVAL;
  const int64_t Tout = out->shape[0], Ho = out->shape[1], Wo = out->shape[2];
  if (out->strides[3] != 1 || out->strides[2] != Cout || out->strides[1] != Wo * Cout || out->strides[0] != Ho * Wo * Cout)
    return CP25_ERR_INVAL;
  if (pad_front < 0 || stride_t < 1 || stride_hw < 1) return CP25_ERR_INVAL;
  const int64_t n_frames = pad_front + T;
  if (n_frames > 24 || (Tout - 1) * stride_t + KT > n_frames) return CP25_ERR_INVAL;
  if ((Hin + pad_top + pad_bottom - KH) / stride_hw + 1 != Ho || (Win + pad_left + pad_right - KW) / stride_hw + 1 != Wo)
    return CP25_ERR_INVAL;
  const void* frames[24];
  for (int64_t i = 0; i < n_frames; ++i)
    frames[i] = i < pad_front ? nullptr : (const char*)x->data + (i - pad_front) * x->strides[0] * 2;
  return cp25_conv3d(frames, (int)n_frames, weight->data, bias ? bias->data : nullptr, nullptr, out->data, (int)Hin,
                     (int)Win, (int)Cin, (int)Cout, (int)Tout, (int)KT, (int)KH, (int)KW, stride_t, stride_hw, pad_top,
                     pad_left, pad_bottom, pad_right, 0, 0, stream);
}
