// pybind11 module `_C` exposing the HIP kernel launchers.  Compiled with g++ (no HIP or torch
// headers needed here); the launchers live in the *.hip translation units built by hipcc.
// The Python wrappers in ops/__init__.py validate tensors and pass raw device pointers and the
// current hipStream_t of torch (so every launch is ordered on, and graph-capturable from, the
// caller's stream).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <vector>

#include "ewdml_ops.h"

namespace py = pybind11;

PYBIND11_MODULE(_C, m) {
  m.doc() = "ewdml CDNA4 (gfx950) kernels";
  m.attr("arch") = "gfx950";

  m.def("topk_scratch_bytes", &ew_topk_scratch_bytes);
  m.def("qsgd_scratch_bytes", &ew_qsgd_scratch_bytes);

  m.def("topk_encode",
        [](const std::vector<uintptr_t>& grads, uintptr_t resid, uintptr_t chunks,
           uintptr_t tensors, uintptr_t scratch,
           uintptr_t payload, long long payload_bytes, int T, int C, int scales_off,
           int counts_off, int idx_off, int codes_off, int value_kind, int norm_l2, float levels,
           float inv_levels, uint32_t key, uint32_t bucket_offset, uintptr_t key_ptr,
           uintptr_t stream) {
          TopkEncodeArgs a{grads.data(), (int)grads.size(),
                           resid,      chunks,     tensors,  scratch,   payload,
                           stream,       payload_bytes, T,       C,        scales_off, counts_off,
                           idx_off,      codes_off,  value_kind, norm_l2,  levels,    inv_levels,
                           key,          bucket_offset, key_ptr};
          ew_topk_encode(a);
        });

  m.def("topk_decode_apply",
        [](uintptr_t recv, int nranks, long long stride, uintptr_t chunks, uintptr_t tensors,
           int C, int scales_off, int counts_off, int idx_off, int codes_off, int value_kind,
           float inv_levels, uintptr_t param, uintptr_t mom, uintptr_t grad_out, float lr,
           float momentum, float dampening, float weight_decay, float grad_scale, int nesterov,
           int first, int apply, uintptr_t stream) {
          TopkDecodeArgs a{recv,       chunks,     tensors,    param,       mom,
                           grad_out,   stream,     stride,     nranks,      C,
                           scales_off, counts_off, idx_off,    codes_off,   value_kind,
                           inv_levels, lr,         momentum,   dampening,   weight_decay,
                           grad_scale, nesterov,   first,      apply};
          ew_topk_decode_apply(a);
        });

  m.def("qsgd_encode",
        [](const std::vector<uintptr_t>& grads, uintptr_t resid, uintptr_t chunks,
           uintptr_t tensors, uintptr_t scratch,
           uintptr_t payload, long long payload_bytes, int T, int C, int scales_off, int codes_off,
           int bits, int norm_l2, float levels, float inv_levels, uint32_t key,
           uint32_t bucket_offset, uintptr_t key_ptr, uintptr_t stream) {
          QsgdEncodeArgs a{grads.data(), (int)grads.size(),
                           resid,   chunks,        tensors,   scratch, payload, stream,
                           payload_bytes, T,   C,             scales_off, codes_off, bits, norm_l2,
                           levels,    inv_levels, key,        bucket_offset, key_ptr};
          ew_qsgd_encode(a);
        });

  m.def("qsgd_decode_apply",
        [](uintptr_t recv, int nranks, long long stride, uintptr_t chunks, uintptr_t tensors,
           int C, int scales_off, int codes_off, int bits, float inv_levels, uintptr_t param,
           uintptr_t mom, uintptr_t grad_out, float lr, float momentum, float dampening,
           float weight_decay, float grad_scale, int nesterov, int first, int apply,
           uintptr_t stream) {
          QsgdDecodeArgs a{recv,   chunks,    tensors,   param,        mom,        grad_out,
                           stream, stride,    nranks,    C,            scales_off, codes_off,
                           bits,   inv_levels, lr,       momentum,     dampening,  weight_decay,
                           grad_scale, nesterov, first,  apply};
          ew_qsgd_decode_apply(a);
        });

  m.def("sgd_flat",
        [](uintptr_t param, uintptr_t mom, uintptr_t grad, long long n, int grad_dtype, float lr,
           float momentum, float dampening, float weight_decay, float grad_scale, int nesterov,
           int first, uintptr_t stream) {
          SgdFlatArgs a{param, mom,      grad,      stream,       n,          grad_dtype,
                        lr,    momentum, dampening, weight_decay, grad_scale, nesterov,  first};
          ew_sgd_flat(a);
        });

  m.def("adam_flat",
        [](uintptr_t param, uintptr_t m1, uintptr_t m2, uintptr_t vmax, uintptr_t grad, long long n,
           int grad_dtype, float lr_step, float beta1, float beta2, float eps, float weight_decay,
           float grad_scale, int amsgrad, uintptr_t stream) {
          AdamFlatArgs a{param, m1,    m2,  vmax,  grad,         stream,     n,
                         grad_dtype, lr_step, beta1, beta2, eps, weight_decay, grad_scale,
                         1.0f,  amsgrad};
          ew_adam_flat(a);
        });

  m.def("cast_scale", &ew_cast_scale);
  m.def("pack_grads",
        [](const std::vector<uintptr_t>& grads, int T, uintptr_t chunks, int C, uintptr_t dst,
           int dst_dtype, float scale, uintptr_t stream) {
          ew_pack_grads(grads.data(), (int)grads.size(), T, chunks, C, dst, dst_dtype, scale,
                        stream);
        });
}
