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
using Ptrs = std::vector<uintptr_t>;
using Mask = std::vector<uint32_t>;

PYBIND11_MODULE(_C, m) {
  m.doc() = "ewdml CDNA4 (gfx950) kernels";
  m.attr("arch") = "gfx950";

  m.def("topk_scratch_bytes", &ew_topk_scratch_bytes);
  m.def("topk_lookback_errors", &ew_topk_lookback_errors);
  m.def("topk_stats", &ew_topk_stats);
  m.def("graph_info", &ew_graph_info);
  m.def("qsgd_scratch_bytes", &ew_qsgd_scratch_bytes);

  m.def("topk_encode",
        [](const Ptrs& grads, const Mask& mask, uintptr_t resid, uintptr_t chunks,
           uintptr_t tensors, uintptr_t scratch, uintptr_t payload, long long payload_bytes,
           int T, int C, int scales_off, int counts_off, int idx_off, int codes_off,
           int value_kind, int norm_l2, float levels, float inv_levels, uint32_t key,
           uint32_t bucket_offset, uintptr_t key_ptr, uintptr_t stream, uintptr_t vel,
           uintptr_t param, float dgc_momentum, float dgc_damp1, float dgc_wd,
           int dgc_nesterov, int bitmap_off, int dgc_mask, uintptr_t dgc_lr_ptr,
           long long bucket_len, uintptr_t cblocks, int num_cblocks, int predict,
           int lb_fault, int max_k, uintptr_t apply_param, uintptr_t apply_shadow,
           float apply_lr, uintptr_t apply_lr_ptr, float apply_scale,
           uintptr_t apply_key_state, uint32_t apply_key_seed, uint32_t apply_key_rank,
           int apply_mom_set, uintptr_t apply_mom, float apply_momentum, float apply_dampening,
           float apply_wd, int apply_nesterov, int apply_first, uintptr_t dgc_stamps) {
          TopkEncodeArgs a{};
          a.dgc_stamps = dgc_stamps;
          a.apply_mom_set = apply_mom_set;
          a.apply_mom = apply_mom;
          a.apply_momentum = apply_momentum;
          a.apply_dampening = apply_dampening;
          a.apply_wd = apply_wd;
          a.apply_nesterov = apply_nesterov;
          a.apply_first = apply_first;
          a.apply_param = apply_param;
          a.apply_shadow = apply_shadow;
          a.apply_lr = apply_lr;
          a.apply_lr_ptr = apply_lr_ptr;
          a.apply_scale = apply_scale;
          a.apply_key_state = apply_key_state;
          a.apply_key_seed = apply_key_seed;
          a.apply_key_rank = apply_key_rank;
          a.lb_fault = lb_fault;
          a.max_k = max_k;
          a.bucket_len = bucket_len;
          a.cblocks = cblocks;
          a.num_cblocks = num_cblocks;
          a.predict = predict;
          a.dgc_mask = dgc_mask;
          a.dgc_lr_ptr = dgc_lr_ptr;
          a.bitmap_off = bitmap_off;
          a.vel = vel;
          a.param = param;
          a.dgc_momentum = dgc_momentum;
          a.dgc_damp1 = dgc_damp1;
          a.dgc_wd = dgc_wd;
          a.dgc_nesterov = dgc_nesterov;
          a.grad_ptrs = grads.data();
          a.n_grad_ptrs = (int)grads.size();
          a.bf16_mask = mask.data();
          a.n_bf16_mask = (int)mask.size();
          a.resid = resid;
          a.chunks = chunks;
          a.tensors = tensors;
          a.scratch = scratch;
          a.payload = payload;
          a.stream = stream;
          a.payload_bytes = payload_bytes;
          a.num_tensors = T;
          a.num_chunks = C;
          a.scales_off = scales_off;
          a.counts_off = counts_off;
          a.idx_off = idx_off;
          a.codes_off = codes_off;
          a.value_kind = value_kind;
          a.norm_l2 = norm_l2;
          a.levels = levels;
          a.inv_levels = inv_levels;
          a.key = key;
          a.bucket_offset = bucket_offset;
          a.key_ptr = key_ptr;
          ew_topk_encode(a);
        });

  m.def("topk_decode_apply",
        [](uintptr_t recv, int nranks, long long stride, uintptr_t chunks, uintptr_t tensors,
           int C, int scales_off, int counts_off, int idx_off, int codes_off, int value_kind,
           float inv_levels, uintptr_t param, uintptr_t mom, uintptr_t grad_out, uintptr_t shadow,
           float lr, float momentum, float dampening, float weight_decay, float grad_scale,
           int nesterov, int first, int apply, uintptr_t stream, uintptr_t key_state,
           uint32_t key_seed, uint32_t key_rank, int bitmap_off, uintptr_t lr_ptr) {
          TopkDecodeArgs a{};
          a.lr_ptr = lr_ptr;
          a.bitmap_off = bitmap_off;
          a.key_state = key_state;
          a.key_seed = key_seed;
          a.key_rank = key_rank;
          a.recv = recv;
          a.chunks = chunks;
          a.tensors = tensors;
          a.param = param;
          a.mom = mom;
          a.grad_out = grad_out;
          a.shadow = shadow;
          a.stream = stream;
          a.stride = stride;
          a.nranks = nranks;
          a.num_chunks = C;
          a.scales_off = scales_off;
          a.counts_off = counts_off;
          a.idx_off = idx_off;
          a.codes_off = codes_off;
          a.value_kind = value_kind;
          a.inv_levels = inv_levels;
          a.lr = lr;
          a.momentum = momentum;
          a.dampening = dampening;
          a.weight_decay = weight_decay;
          a.grad_scale = grad_scale;
          a.nesterov = nesterov;
          a.first = first;
          a.apply = apply;
          ew_topk_decode_apply(a);
        });

  m.def("qsgd_encode",
        [](const Ptrs& grads, const Mask& mask, uintptr_t resid, uintptr_t chunks,
           uintptr_t tensors, uintptr_t scratch, uintptr_t payload, long long payload_bytes,
           int T, int C, int scales_off, int codes_off, int bits, int norm_l2, float levels,
           float inv_levels, uint32_t key, uint32_t bucket_offset, uintptr_t key_ptr,
           uintptr_t stream) {
          QsgdEncodeArgs a{};
          a.grad_ptrs = grads.data();
          a.n_grad_ptrs = (int)grads.size();
          a.bf16_mask = mask.data();
          a.n_bf16_mask = (int)mask.size();
          a.resid = resid;
          a.chunks = chunks;
          a.tensors = tensors;
          a.scratch = scratch;
          a.payload = payload;
          a.stream = stream;
          a.payload_bytes = payload_bytes;
          a.num_tensors = T;
          a.num_chunks = C;
          a.scales_off = scales_off;
          a.codes_off = codes_off;
          a.bits = bits;
          a.norm_l2 = norm_l2;
          a.levels = levels;
          a.inv_levels = inv_levels;
          a.key = key;
          a.bucket_offset = bucket_offset;
          a.key_ptr = key_ptr;
          ew_qsgd_encode(a);
        });

  m.def("qsgd_decode_apply",
        [](uintptr_t recv, int nranks, long long stride, uintptr_t chunks, uintptr_t tensors,
           int C, int scales_off, int codes_off, int bits, float inv_levels, uintptr_t param,
           uintptr_t mom, uintptr_t grad_out, uintptr_t shadow, float lr, float momentum,
           float dampening, float weight_decay, float grad_scale, int nesterov, int first,
           int apply, uintptr_t stream, uintptr_t key_state, uint32_t key_seed,
           uint32_t key_rank, uintptr_t lr_ptr) {
          QsgdDecodeArgs a{};
          a.lr_ptr = lr_ptr;
          a.key_state = key_state;
          a.key_seed = key_seed;
          a.key_rank = key_rank;
          a.recv = recv;
          a.chunks = chunks;
          a.tensors = tensors;
          a.param = param;
          a.mom = mom;
          a.grad_out = grad_out;
          a.shadow = shadow;
          a.stream = stream;
          a.stride = stride;
          a.nranks = nranks;
          a.num_chunks = C;
          a.scales_off = scales_off;
          a.codes_off = codes_off;
          a.bits = bits;
          a.inv_levels = inv_levels;
          a.lr = lr;
          a.momentum = momentum;
          a.dampening = dampening;
          a.weight_decay = weight_decay;
          a.grad_scale = grad_scale;
          a.nesterov = nesterov;
          a.first = first;
          a.apply = apply;
          ew_qsgd_decode_apply(a);
        });

  m.def("sgd_flat",
        [](uintptr_t param, uintptr_t mom, uintptr_t grad, uintptr_t shadow, long long n,
           int grad_dtype, float lr, float momentum, float dampening, float weight_decay,
           float grad_scale, int nesterov, int first, uintptr_t stream, uintptr_t lr_ptr) {
          SgdFlatArgs a{};
          a.lr_ptr = lr_ptr;
          a.param = param;
          a.mom = mom;
          a.grad = grad;
          a.shadow = shadow;
          a.stream = stream;
          a.n = n;
          a.grad_dtype = grad_dtype;
          a.lr = lr;
          a.momentum = momentum;
          a.dampening = dampening;
          a.weight_decay = weight_decay;
          a.grad_scale = grad_scale;
          a.nesterov = nesterov;
          a.first = first;
          ew_sgd_flat(a);
        });

  m.def("adam_flat",
        [](uintptr_t param, uintptr_t m1, uintptr_t m2, uintptr_t vmax, uintptr_t grad,
           uintptr_t shadow, long long n, int grad_dtype, float lr_step, float beta1, float beta2,
           float eps, float weight_decay, float grad_scale, int amsgrad, uintptr_t stream,
           uintptr_t step, double lr, uintptr_t lr_ptr) {
          AdamFlatArgs a{};
          a.lr_ptr = lr_ptr;
          a.step = step;
          a.lr = lr;
          a.param = param;
          a.exp_avg = m1;
          a.exp_avg_sq = m2;
          a.max_exp_avg_sq = vmax;
          a.grad = grad;
          a.shadow = shadow;
          a.stream = stream;
          a.n = n;
          a.grad_dtype = grad_dtype;
          a.lr_step = lr_step;
          a.beta1 = beta1;
          a.beta2 = beta2;
          a.eps = eps;
          a.weight_decay = weight_decay;
          a.grad_scale = grad_scale;
          a.bc2_sqrt = 1.0f;
          a.amsgrad = amsgrad;
          ew_adam_flat(a);
        });

  m.def("cast_scale", &ew_cast_scale);

  m.def("pack_grads",
        [](const Ptrs& grads, const Mask& mask, int T, uintptr_t chunks, int C, uintptr_t dst,
           int dst_dtype, float scale, uintptr_t stream) {
          ew_pack_grads(grads.data(), (int)grads.size(), mask.data(), (int)mask.size(), T, chunks,
                        C, dst, dst_dtype, scale, stream);
        });

  m.def("sgd_ptrs",
        [](const Ptrs& grads, const Mask& mask, int T, uintptr_t chunks, int C, uintptr_t param,
           uintptr_t mom, uintptr_t shadow, float lr, float momentum, float dampening,
           float weight_decay, float grad_scale, int nesterov, int first, uintptr_t stream,
           uintptr_t lr_ptr) {
          SgdFlatArgs a{};
          a.param = param;
          a.mom = mom;
          a.shadow = shadow;
          a.stream = stream;
          a.lr = lr;
          a.momentum = momentum;
          a.dampening = dampening;
          a.weight_decay = weight_decay;
          a.grad_scale = grad_scale;
          a.nesterov = nesterov;
          a.first = first;
          a.lr_ptr = lr_ptr;
          ew_sgd_ptrs(grads.data(), (int)grads.size(), mask.data(), (int)mask.size(), T, chunks,
                      C, a);
        });

  m.def("cf_set_glds", &ew_cf_set_glds);
  m.def("cf_set_inred", &ew_cf_set_inred);
  m.def("cf_defer_reduce", &ew_cf_defer_reduce);
  m.def("cf_flush_reduce", &ew_cf_flush_reduce);
  m.def("cf_arm_bn_fin", &ew_cf_arm_bn_fin);
  m.def("cf_flush_bn_fin", &ew_cf_flush_bn_fin);
  m.def("cf_arm_wgout", &ew_cf_arm_wgout);
  m.def("cf_flush_wgout", &ew_cf_flush_wgout);
  m.def("bn_part_floats", &ew_bn_part_floats);
  m.def("bn_relu_fwd",
        [](uintptr_t h, uintptr_t res, uintptr_t y, uintptr_t code, uintptr_t stats,
           uintptr_t part, uintptr_t gamma, uintptr_t beta, uintptr_t cbias, uintptr_t rmean,
           uintptr_t rvar, uintptr_t nbt, long long N, int H, int W, int C, int is_bf16,
           int pool, int mode, int training, float momentum, float eps, int cb_bf16,
           uintptr_t stream, int pre_nblk, int phase) {
          BnFwdArgs a{};
          a.pre_nblk = pre_nblk;
          a.phase = phase;
          a.h = h; a.res = res; a.y = y; a.code = code; a.stats = stats; a.part = part;
          a.gamma = gamma; a.beta = beta; a.cbias = cbias; a.rmean = rmean; a.rvar = rvar;
          a.nbt = nbt; a.N = N; a.H = H; a.W = W; a.C = C;
          a.is_bf16 = is_bf16; a.pool = pool; a.mode = mode; a.training = training;
          a.momentum = momentum; a.eps = eps; a.cb_bf16 = cb_bf16; a.stream = stream;
          ew_bn_relu_fwd(a);
        });
  m.def("bn_relu_bwd",
        [](uintptr_t h, uintptr_t res, uintptr_t dy, uintptr_t code, uintptr_t stats,
           uintptr_t coef, uintptr_t part, uintptr_t dx, uintptr_t dres, uintptr_t dgamma,
           uintptr_t dbeta, uintptr_t dcbias, long long N, int H, int W, int C, int is_bf16,
           int pool, int mode, int cb_bf16, uintptr_t stream, int pre_nblk, int phase) {
          BnBwdArgs a{};
          a.phase = phase;
          a.h = h; a.res = res; a.dy = dy; a.code = code; a.stats = stats; a.coef = coef;
          a.part = part; a.dx = dx; a.dres = dres; a.dgamma = dgamma; a.dbeta = dbeta;
          a.dcbias = dcbias; a.N = N; a.H = H; a.W = W; a.C = C; a.is_bf16 = is_bf16;
          a.pool = pool; a.mode = mode; a.cb_bf16 = cb_bf16; a.stream = stream;
          a.pre_nblk = pre_nblk;
          ew_bn_relu_bwd(a);
        });
  m.def("act_dropout_fwd", &ew_act_dropout_fwd);
  m.def("act_dropout_bwd", &ew_act_dropout_bwd);
  m.def("cross_entropy_fwd", &ew_cross_entropy_fwd);
  m.def("cross_entropy_bwd", &ew_cross_entropy_bwd);
  m.def("conv_ws_floats", &ew_conv_ws_floats);
  m.def("conv_fwd", &ew_conv_fwd);
  m.def("conv_bwd_data", &ew_conv_bwd_data);
  m.def("conv_wgrad", &ew_conv_wgrad);
  m.def("conv_stem_fwd", &ew_conv_stem_fwd);
  m.def("head_fwd", &ew_head_fwd);
  m.def("head_fwd_ce", &ew_head_fwd_ce);
  m.def("head_bwd", &ew_head_bwd);
  m.def("head_bwd_bn", &ew_head_bwd_bn);
  m.def("conv_stem_wgrad", &ew_conv_stem_wgrad);
  m.def("rccl_unique_id", [] { return pybind11::bytes(ew_rccl_unique_id()); });
  m.def("rccl_version", &ew_rccl_version);
  m.def("rccl_init", [](pybind11::bytes uid, int nranks, int rank, int device) {
    return ew_rccl_init(std::string(uid), nranks, rank, device);
  });
  m.def("rccl_destroy", &ew_rccl_destroy);
  m.def("rccl_abort", &ew_rccl_abort);
  m.def("rccl_watchdog_start", &ew_rccl_watchdog_start);
  m.def("rccl_watch", &ew_rccl_watch);
  m.def("rccl_watch_pending", &ew_rccl_watch_pending);
  m.def("rccl_watchdog_stop", &ew_rccl_watchdog_stop,
        pybind11::call_guard<pybind11::gil_scoped_release>());
  m.def("test_flag_alloc", &ew_test_flag_alloc);
  m.def("test_flag_free", &ew_test_flag_free);
  m.def("watchdog_release_flag", &ew_watchdog_release_flag);
  m.def("test_spin", &ew_test_spin);
  m.def("rccl_all_gather", &ew_rccl_all_gather);
  m.def("rccl_all_reduce", &ew_rccl_all_reduce);
  m.def("rccl_reduce_scatter", &ew_rccl_reduce_scatter);
  m.def("rccl_broadcast", &ew_rccl_broadcast);
  m.def("rccl_all_to_all", &ew_rccl_all_to_all);
  m.def("conv_f32_fwd", &ew_conv_f32_fwd);
  m.def("conv_f32_bwd_data", &ew_conv_f32_bwd_data);
  m.def("conv_f32_wgrad", &ew_conv_f32_wgrad);
  m.def("conv_f32_fwd_lz", &ew_conv_f32_fwd_lz);
  m.def("conv_f32_wgrad_lz", &ew_conv_f32_wgrad_lz);
  m.def("conv_f32_fwd_s2", &ew_conv_f32_fwd_s2);
  m.def("conv_f32_bwd_data_s2", &ew_conv_f32_bwd_data_s2);
  m.def("conv_f32_wgrad_s2", &ew_conv_f32_wgrad_s2);
  m.def("conv_f32_stem_fwd", &ew_conv_f32_stem_fwd);
  m.def("conv_f32_stem_wgrad", &ew_conv_f32_stem_wgrad);
  m.def("conv_f32_stem_wgrad_bn", &ew_conv_f32_stem_wgrad_bn);
  m.def("wino_f32_weight", &ew_wino_f32_weight);
  m.def("wino_f32_fwd", &ew_wino_f32_fwd);
  m.def("wino_f32_bwd_data", &ew_wino_f32_bwd_data);
  m.def("wino_f32_wgrad", &ew_wino_f32_wgrad);
  m.def("wino_f32_wgrad_out", &ew_wino_f32_wgrad_out);
  m.def("wino_f32_fwd_bn", &ew_wino_f32_fwd_bn);
  m.def("wino_f32_bwd_data_bn", &ew_wino_f32_bwd_data_bn);
  m.def("sm_f32_ws_floats", &ew_sm_f32_ws_floats);
  m.def("sm_f32_counters", &ew_sm_f32_counters);
  m.def("sm_f32_fwd", &ew_sm_f32_fwd);
  m.def("sm_set_fence", &ew_sm_set_fence);
  m.def("topk_fused_select_max_blocks", &ew_topk_fused_select_max_blocks);
  m.def("topk_one_max_blocks", &ew_topk_one_max_blocks);
  m.def("flag_signal", &ew_flag_signal);
  m.def("flag_wait", &ew_flag_wait);
  m.def("topk_one_stamps", &ew_topk_one_stamps);
  m.def("sm_f32_bwd", &ew_sm_f32_bwd);
  m.def("lenet_ws_floats", &ew_lenet_ws_floats);
  m.def("lenet_counters", &ew_lenet_counters);
  m.def("lenet_set_prof", &ew_lenet_set_prof);
  m.def("lenet_fwd", &ew_lenet_fwd);
  m.def("tail_ws_floats", &ew_tail_ws_floats);
  m.def("tail_counters", &ew_tail_counters);
  m.def("tail_fwd", &ew_tail_fwd);
  m.def("tail_bwd", &ew_tail_bwd);
  m.def("lenet_bwd", &ew_lenet_bwd);
  m.def("maxpool2_nhwc", &ew_maxpool2_nhwc);
  m.def("maxpool3s2_nhwc", &ew_maxpool3s2_nhwc);
  m.def("gap_nhwc", &ew_gap_nhwc);
  m.def("maxpool2_fwd", &ew_maxpool2_fwd);
  m.def("maxpool2_bwd", &ew_maxpool2_bwd);
  m.def("ticket_ints", [] { return EW_TICKET_INTS; });
  m.def("make_batch",
        [](uintptr_t src, uintptr_t labels, uintptr_t perm, long long perm_len, uintptr_t state,
           uintptr_t done, uintptr_t out, uintptr_t out_y, int B, int C, int H, int W, int pad, int augment,
           int out_bf16, int channels_last, uint32_t seed, uint32_t rank,
           const std::vector<float>& mean, const std::vector<float>& inv_std, uintptr_t stream) {
          MakeBatchArgs a{};
          a.src = src; a.labels = labels; a.perm = perm; a.perm_len = perm_len; a.state = state; a.done = done;
          a.out = out; a.out_y = out_y; a.B = B; a.C = C; a.H = H; a.W = W; a.pad = pad;
          a.augment = augment; a.out_bf16 = out_bf16; a.channels_last = channels_last;
          a.seed = seed; a.rank = rank;
          for (int c = 0; c < 4; ++c) {
            a.mean[c] = c < (int)mean.size() ? mean[c] : 0.0f;
            a.inv_std[c] = c < (int)inv_std.size() ? inv_std[c] : 1.0f;
          }
          a.stream = stream;
          ew_make_batch(a);
        });
}
