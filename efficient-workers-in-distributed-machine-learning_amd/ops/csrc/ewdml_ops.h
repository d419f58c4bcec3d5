// Host-side entry points of the ewdml HIP kernels (C++ only, no HIP types), bound to Python in
// bindings.cpp.  Pointers are device addresses passed as integers; `stream` is a hipStream_t.
#pragma once
#include <string>
#include <vector>
#include <stddef.h>
#include <stdint.h>

struct TopkEncodeArgs {
  const uintptr_t* grad_ptrs;  // per-tensor gradient base pointers (host array, n_grad_ptrs)
  int n_grad_ptrs;
  const uint32_t* bf16_mask;   // bit t: tensor t's gradient is bf16
  int n_bf16_mask;
  uintptr_t resid, chunks, tensors, scratch, payload, stream;
  long long payload_bytes;
  int num_tensors, num_chunks;
  int scales_off, counts_off, idx_off, codes_off, bitmap_off;
  int value_kind;  // 0 = int8 QSGD, 1 = int4 QSGD, 2 = fp32 values (plain top-k)
  int norm_l2;     // 0 = max-norm scale, 1 = L2 norm of the selected values
  float levels, inv_levels;
  uint32_t key, bucket_offset;
  uintptr_t key_ptr;  // optional device uint32 overriding `key` (graph replay)
  // error feedback with momentum correction (DGC; compress/oracle.py dgc_accumulate): per-rank
  // velocity (0: plain error feedback) and the bucket's fp32 parameters (read when dgc_wd != 0)
  uintptr_t vel, param;
  float dgc_momentum, dgc_damp1, dgc_wd;  // damp1 = 1 - dampening
  int dgc_nesterov;
  int dgc_mask;          // clear the velocity at sent coordinates (DGC) or keep it (local)
  uintptr_t dgc_lr_ptr;  // nullable device lr: residual accumulates lr-scaled updates
  long long bucket_len;  // elements (sizes the candidate list in the scratch)
  // predictive encode (max-norm scale only): candidate-pass block table (CBlockRow[num_cblocks])
  uintptr_t cblocks;
  int num_cblocks;
  int predict;
  int lb_fault;  // test hook: tensors' first chunks skip their look-back word (lb_err path)
  int max_k;     // largest per-tensor k of the bucket (0: unknown)
  // world of one (the all-gather is this rank's payload): the write pass also applies the update
  // the decode would, p -= lr * scale * sent at each sent coordinate (momentum-corrected error
  // feedback: no receiver momentum); apply_param 0 = off.  apply_key_state: advance the RNG key
  // state {step, key} after every block read the key (the last bucket's decode did it)
  uintptr_t apply_param, apply_shadow, apply_lr_ptr, apply_key_state;
  float apply_lr, apply_scale;
  uint32_t apply_key_seed, apply_key_rank;
  // dense variant (receiver-side momentum SGD over every element; one-launch encodes only)
  uintptr_t dgc_stamps;  // nullable u32[T]: producer-staged tensors (dgc_stage.h)
  int apply_mom_set;
  uintptr_t apply_mom;
  float apply_momentum, apply_dampening, apply_wd;
  int apply_nesterov, apply_first;
};

struct TopkDecodeArgs {
  uintptr_t recv, chunks, tensors, param, mom, grad_out, shadow, stream;
  long long stride;
  int nranks, num_chunks;
  int scales_off, counts_off, idx_off, codes_off, bitmap_off;
  int value_kind;
  float inv_levels;
  float lr, momentum, dampening, weight_decay, grad_scale;
  int nesterov, first, apply;
  uintptr_t key_state;  // nullable int32[2] {step, key}: advanced to the next step (HIP graphs)
  uint32_t key_seed, key_rank;
  uintptr_t lr_ptr;  // nullable device fp32 learning rate (overrides lr)
};

struct QsgdEncodeArgs {
  const uintptr_t* grad_ptrs;
  int n_grad_ptrs;
  const uint32_t* bf16_mask;
  int n_bf16_mask;
  uintptr_t resid, chunks, tensors, scratch, payload, stream;
  long long payload_bytes;
  int num_tensors, num_chunks;
  int scales_off, codes_off, bits, norm_l2;
  float levels, inv_levels;
  uint32_t key, bucket_offset;
  uintptr_t key_ptr;
};

struct QsgdDecodeArgs {
  uintptr_t recv, chunks, tensors, param, mom, grad_out, shadow, stream;
  long long stride;
  int nranks, num_chunks;
  int scales_off, codes_off, bits;
  float inv_levels;
  float lr, momentum, dampening, weight_decay, grad_scale;
  int nesterov, first, apply;
  uintptr_t key_state;  // see TopkDecodeArgs
  uint32_t key_seed, key_rank;
  uintptr_t lr_ptr;
};

struct SgdFlatArgs {
  uintptr_t param, mom, grad, shadow, stream;
  long long n;
  int grad_dtype;  // 0 = fp32, 1 = bf16, 2 = fp16
  float lr, momentum, dampening, weight_decay, grad_scale;
  int nesterov, first;
  uintptr_t lr_ptr;
};

struct AdamFlatArgs {
  uintptr_t param, exp_avg, exp_avg_sq, max_exp_avg_sq, grad, shadow, stream;
  long long n;
  int grad_dtype;
  float lr_step, beta1, beta2, eps, weight_decay, grad_scale, bc2_sqrt;
  int amsgrad;
  uintptr_t step;  // int32 device step counter (nullable: use lr_step as given)
  double lr;       // base lr for the device-side bias correction
  uintptr_t lr_ptr;  // nullable device fp32 base lr (overrides lr)
};

size_t ew_topk_scratch_bytes(int num_tensors, int num_chunks, long long bucket_len,
                             long long total_cap);
std::vector<int> ew_topk_stats(uintptr_t scratch, int num_tensors, int num_chunks);
std::vector<long long> ew_graph_info(uintptr_t graph, const std::string& dot_path);
// largest candidate-block count the fused select kernel takes (0: always three kernels)
int ew_topk_fused_select_max_blocks();
int ew_topk_one_max_blocks();
void ew_flag_signal(uintptr_t flag, uintptr_t stream);
void ew_flag_wait(uintptr_t flag, uintptr_t seen, int need, uintptr_t err, uintptr_t stream);
std::vector<unsigned long long> ew_topk_one_stamps();
int ew_topk_lookback_errors(uintptr_t scratch, int num_tensors, int num_chunks);
void ew_topk_encode(const TopkEncodeArgs& a);
void ew_topk_decode_apply(const TopkDecodeArgs& a);

size_t ew_qsgd_scratch_bytes(int num_tensors, int num_chunks);
void ew_qsgd_encode(const QsgdEncodeArgs& a);
void ew_qsgd_decode_apply(const QsgdDecodeArgs& a);

void ew_sgd_flat(const SgdFlatArgs& a);
void ew_adam_flat(const AdamFlatArgs& a);
// fp32 forward conv GEMMs through LDS-DMA staging (k_cf_gemm_gl) when on (-1: query only);
// returns the previous setting
int ew_cf_set_glds(int on);
int ew_cf_set_inred(int on);
void ew_cf_defer_reduce();
void ew_cf_flush_reduce();
void ew_cf_arm_bn_fin(uintptr_t part, int nblk, int C, long long M, uintptr_t stats, uintptr_t coef,
                      uintptr_t dgamma, uintptr_t dbeta, uintptr_t dcbias, int cb_bf16);
int ew_cf_flush_bn_fin(uintptr_t stream);
void ew_cf_arm_wgout(uintptr_t src, int split, uintptr_t dw, int Nc, int C);
int ew_cf_flush_wgout(uintptr_t stream);
// SGD of one bucket from its per-tensor gradients (pointer table; a.grad / a.n / a.grad_dtype
// unused): param / mom / shadow are the bucket's flat views, chunk rows address them
void ew_sgd_ptrs(const uintptr_t* grad_ptrs, int n_ptrs, const uint32_t* bf16_mask, int n_mask,
                 int num_tensors, uintptr_t chunks, int num_chunks, const SgdFlatArgs& a);
void ew_pack_grads(const uintptr_t* grad_ptrs, int n_ptrs, const uint32_t* bf16_mask, int n_mask,
                   int num_tensors, uintptr_t chunks, int num_chunks, uintptr_t dst,
                   int dst_dtype, float scale, uintptr_t stream);
// dst (bf16 when to_bf16 else fp16) = src * scale
void ew_cast_scale(uintptr_t src, uintptr_t dst, long long n, float scale, int to_bf16,
                   uintptr_t stream);

// ---- model-side kernels (nn.hip) ----
// NHWC BatchNorm + ReLU [+ 2x2 max pool]; h/y/dy/dx bf16 or fp32 ([N,H,W,C] memory), C % 8 == 0
// mode: 0 relu, 2 identity, 3 relu(bn + res) (pool = 1 forces relu + 2x2 pool)
struct BnFwdArgs {
  uintptr_t h, res, y, code, stats, part;        // stats fp32 [4][C]; part: ew_bn_part_floats() floats
  uintptr_t gamma, beta, cbias, rmean, rvar, nbt;  // fp32 [C] (nullable; cbias fp32 or bf16),
  //                                                  nbt int64 (nullable): incremented once
  long long N;
  int H, W, C;
  int is_bf16, pool, training, cb_bf16, mode;
  float momentum, eps;  // momentum < 0: cumulative average over *nbt batches
  uintptr_t stream;
  int pre_nblk;  // > 0: `part` already holds [2][pre_nblk][C] partial sums (skip the stats pass)
  int phase;     // 0: statistics + apply, 1: statistics only (the consumer applies: lazy), 2: apply
};
struct BnBwdArgs {
  uintptr_t h, res, dy, code, stats, coef, part, dx, dres;  // coef fp32 [2][C]
  uintptr_t dgamma, dbeta, dcbias;               // [C] outputs (nullable), dcbias bf16 if cb_bf16
  long long N;
  int H, W, C;  // of h (pre-pool)
  int is_bf16, pool, cb_bf16, mode;
  uintptr_t stream;
  int pre_nblk;  // > 0: `part` already holds [2][pre_nblk][C] sums (sum dz, sum dz*(h-mean))
  int phase;     // 0: statistics + apply, 1: statistics only (coef, dgamma, dbeta), 2: apply
};
// NHWC global average pool: forward x [N, HW, C] -> y [N, C]; backward x = dy [N, C] -> y = dx
// [N, HW, C] (C % 8 == 0)
void ew_gap_nhwc(uintptr_t x, uintptr_t y, long long N, int HW, int C, int is_bf16, int backward,
                 uintptr_t stream);
int ew_bn_part_floats();
void ew_bn_relu_fwd(const BnFwdArgs& a);
void ew_bn_relu_bwd(const BnBwdArgs& a);
void ew_maxpool2_nhwc(uintptr_t x, uintptr_t y, uintptr_t code, long long N, int H, int W, int C,
                      int is_bf16, int backward, uintptr_t stream);
// NHWC 3x3 / stride 2 / pad 1 max pool (C % 8 == 0): forward y + 1-byte tap codes, backward dx
// (x = dy, y = dx) gathered from the windows whose code points at each pixel
void ew_maxpool3s2_nhwc(uintptr_t x, uintptr_t y, uintptr_t code, long long N, int H, int W,
                        int C, int is_bf16, int backward, uintptr_t stream);
// NCHW 2x2 max pool: rows = N*C*H/2
void ew_maxpool2_fwd(uintptr_t x, uintptr_t y, uintptr_t code, long long rows, int W, int is_bf16,
                     uintptr_t stream);
void ew_maxpool2_bwd(uintptr_t dy, uintptr_t code, uintptr_t dx, long long rows, int W,
                     int is_bf16, uintptr_t stream);

// ---- fused input pipeline (data.hip) ----
struct MakeBatchArgs {
  uintptr_t src;     // uint8 [N, C, H, W] dataset
  uintptr_t labels;  // int64 [N]
  uintptr_t perm;    // int64 [>= (pos+1)*B] this rank's sample order for the epoch
  uintptr_t state;   // int64 [2] {pos, epoch}; pos advanced by the kernel
  uintptr_t done;    // uint32 [1] zero-initialised block counter (kernel resets it)
  long long perm_len;
  uintptr_t out, out_y;  // fp32/bf16 [B, C, H, W] (NCHW or channels_last), int64 [B]
  int B, C, H, W, pad, augment, out_bf16, channels_last;
  uint32_t seed, rank;
  float mean[4], inv_std[4];
  uintptr_t stream;
};
void ew_make_batch(const MakeBatchArgs& a);

// ---- 3x3 (pad 1) or 1x1 (pad 0) stride-1 convolution, NHWC bf16, MFMA implicit GEMM (conv.hip) ----
// x [N,H,W,C], w [Nc,k,k,C] (channels_last weight memory), y/dy [N,H,W,Nc]; ws: fp32 split slabs
// (ws_floats of them); ksize 3 or 1
long long ew_conv_ws_floats();
// bnpart (nullable): fp32 [2][rows][Nc] BatchNorm partial sums (sum, sum of squares) of y for the
// BN that follows; returns rows (0 when not written: split-K launch or capacity too small)
int ew_conv_fwd(uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t ws, long long ws_floats,
                long long N, int H, int W, int C, int Nc, int ksize, uintptr_t bnpart,
                long long bnpart_floats, uintptr_t stream);
// bn_h (nullable): also write the BN-backward sums [2][rows][C] (sum dz, sum dz*(h-mean)) of the
// BN(+residual bn_res)(+ReLU)(+pool: bn_code) layer whose output gradient dx is into bnpart;
// returns rows (0: not written).  addend (nullable, [rows][C] bf16): dx = this GEMM + addend.
int ew_conv_bwd_data(uintptr_t dy, uintptr_t w, uintptr_t dx, uintptr_t ws,
                     long long ws_floats, long long N, int H, int W, int C, int Nc, int ksize,
                     uintptr_t bn_h, uintptr_t bn_res, uintptr_t bn_code, uintptr_t bn_stats,
                     int bn_relu, uintptr_t bnpart, long long bnpart_floats, uintptr_t addend,
                     uintptr_t stream);
void ew_conv_wgrad(uintptr_t dy, uintptr_t x, uintptr_t dw, uintptr_t ws, long long ws_floats,
                   long long N, int H, int W, int C, int Nc, int ksize, uintptr_t stream);
// int32 words of a grid arrival ticket (common.h ew_grid_last): 8 sub-counters + 1 top, 128 B apart
#define EW_TICKET_INTS (9 * 32)

// classifier-head Linear (head.hip), bf16 or fp32 (is_f32) tensors: forward z = drop_out(act(drop_in(x) w^T + b)) (+ y = the
// pre-activation), backward dw, db, dx from dz in one launch; dropout = (counter, salt, p)
void ew_head_fwd(uintptr_t x, uintptr_t w, uintptr_t b, uintptr_t z, uintptr_t y, int B, int N,
                 int K, int relu, uintptr_t ctr_in, uint32_t salt_in, float p_in,
                 uintptr_t ctr_out, uint32_t salt_out, float p_out, uintptr_t stream,
                 int is_f32);
void ew_head_fwd_ce(uintptr_t x, uintptr_t w, uintptr_t b, uintptr_t z, int B, int N, int K,
                    uintptr_t yl, uintptr_t lossrow, uintptr_t loss, uintptr_t lse, uintptr_t dlog,
                    uintptr_t tick, uintptr_t stream, int is_f32);
void ew_head_bwd_bn(uintptr_t dz, uintptr_t y, uintptr_t x, uintptr_t w, uintptr_t dx,
                    uintptr_t dw, uintptr_t db, int B, int N, int K, int relu, uintptr_t ctr_out,
                    uint32_t salt_out, float p_out, uintptr_t ctr_in, uint32_t salt_in,
                    float p_in, int advance, uintptr_t bn_h, uintptr_t bn_code,
                    uintptr_t bn_stats, uintptr_t bn_coef, uintptr_t bn_dgamma,
                    uintptr_t bn_dbeta, uintptr_t bn_dcbias, int bn_cb_bf16, uintptr_t bn_tick,
                    uintptr_t stream);
void ew_head_bwd(uintptr_t dz, uintptr_t y, uintptr_t x, uintptr_t w, uintptr_t dx, uintptr_t dw,
                 uintptr_t db, int db_bf16, int B, int N, int K, int relu, uintptr_t ctr_out,
                 uint32_t salt_out, float p_out, uintptr_t ctr_in, uint32_t salt_in, float p_in,
                 int advance, uintptr_t stream, int is_f32);
// stem conv: 3x3 / pad 1 over C = 3 input channels (x [N,H,W,3], w [Nc,3,3,3] channels_last);
// forward returns the BN partial rows written (0: none); wgrad uses ws as its partial slab
int ew_conv_stem_fwd(uintptr_t x, uintptr_t w, uintptr_t y, long long N, int H, int W, int Nc,
                     uintptr_t bnpart, long long bnpart_floats, uintptr_t stream);
void ew_conv_stem_wgrad(uintptr_t dy, uintptr_t x, uintptr_t dw, uintptr_t ws,
                        long long ws_floats, long long N, int H, int W, int Nc, uintptr_t stream);

// ---- the same convolutions in fp32 (conv_f32.hip, v_mfma_f32_16x16x4_f32): fp32 tensors and
// BN operands, same argument meaning as the bf16 entry points above
int ew_conv_f32_fwd(uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t ws, long long ws_floats,
                    long long N, int H, int W, int C, int Nc, int ksize, uintptr_t bnpart,
                    long long bnpart_floats, uintptr_t stream);
int ew_conv_f32_bwd_data(uintptr_t dy, uintptr_t w, uintptr_t dx, uintptr_t ws,
                         long long ws_floats, long long N, int H, int W, int C, int Nc, int ksize,
                         uintptr_t bn_h, uintptr_t bn_res, uintptr_t bn_code, uintptr_t bn_stats,
                         int bn_relu, uintptr_t bnpart, long long bnpart_floats, uintptr_t addend,
                         uintptr_t stream);
void ew_conv_f32_wgrad(uintptr_t dy, uintptr_t x, uintptr_t dw, uintptr_t ws, long long ws_floats,
                       long long N, int H, int W, int C, int Nc, int ksize, uintptr_t stream);
int ew_conv_f32_fwd_lz(uintptr_t h, uintptr_t stats, uintptr_t nbt, uintptr_t w, uintptr_t y,
                       uintptr_t ws, long long ws_floats, long long N, int H, int W, int C, int Nc,
                       uintptr_t bnpart, long long bnpart_floats, uintptr_t stream);
void ew_conv_f32_wgrad_lz(uintptr_t dy, uintptr_t h, uintptr_t stats, uintptr_t dw, uintptr_t ws,
                          long long ws_floats, long long N, int H, int W, int C, int Nc,
                          uintptr_t stream);
// stride-2 3x3 / pad 1 and 1x1 / pad 0 (H, W = the input map, even; y / dy are H/2 x W/2)
int ew_conv_f32_fwd_s2(uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t ws, long long ws_floats,
                       long long N, int H, int W, int C, int Nc, int ksize, uintptr_t bnpart,
                       long long bnpart_floats, uintptr_t stream);
void ew_conv_f32_bwd_data_s2(uintptr_t dy, uintptr_t w, uintptr_t dx, long long N, int H, int W,
                             int C, int Nc, int ksize, uintptr_t addend, uintptr_t stream);
void ew_conv_f32_wgrad_s2(uintptr_t dy, uintptr_t x, uintptr_t dw, uintptr_t ws,
                          long long ws_floats, long long N, int H, int W, int C, int Nc, int ksize,
                          uintptr_t stream);
int ew_conv_f32_stem_fwd(uintptr_t x, uintptr_t w, uintptr_t y, long long N, int H, int W, int Nc,
                         uintptr_t bnpart, long long bnpart_floats, uintptr_t stream);
void ew_conv_f32_stem_wgrad(uintptr_t dy, uintptr_t x, uintptr_t dw, uintptr_t ws,
                            long long ws_floats, long long N, int H, int W, int Nc,
                            uintptr_t stream);
// the same with dy formed from the BatchNorm(+ReLU)(+pool) backward of the stem's output
void ew_conv_f32_stem_wgrad_bn(uintptr_t h, uintptr_t dnext, uintptr_t code, uintptr_t stats,
                               uintptr_t coef, int pool, uintptr_t x, uintptr_t dw, uintptr_t ws,
                               long long ws_floats, long long N, int H, int W, int Nc,
                               uintptr_t stream);
// ---- fp32 3x3 convolutions by Winograd F(m x m, 3x3), m = 2 or 4 (winograd_f32.hip): U[a^2][Nc][C]
// (a = m + 2) from the channels_last weight (standalone, or inside the forward when w != 0);
// forward / backward data over caller-allocated V (a^2 * N*H*W/m^2 * C_in floats) and Mo
// (a^2 * N*H*W/m^2 * C_out floats); return the BN partial rows written (0: none)
void ew_wino_f32_weight(uintptr_t w, uintptr_t U, int Nc, int C, int m, uintptr_t stream);
int ew_wino_f32_fwd(uintptr_t x, uintptr_t w, uintptr_t U, uintptr_t y, uintptr_t V, uintptr_t Mo,
                    long long N, int H, int W, int C, int Nc, int m, uintptr_t bnpart,
                    long long bnpart_floats, uintptr_t stream);
int ew_wino_f32_bwd_data(uintptr_t dy, uintptr_t w, uintptr_t U, uintptr_t dx, uintptr_t V,
                         uintptr_t Mo, long long N, int H, int W, int C, int Nc, int m,
                         uintptr_t bn_h, uintptr_t bn_res, uintptr_t bn_code, uintptr_t bn_stats,
                         int bn_relu, uintptr_t bnpart, long long bnpart_floats,
                         uintptr_t addend, uintptr_t D, uintptr_t wo_src, int wo_split,
                         uintptr_t wo_dw, int wo_Nc, int wo_C, uintptr_t stream);
// the same with the BatchNorm(+ReLU)(+2x2 pool) layer in front applied in the input transform
// (forward; its pool codes written here) / the BatchNorm backward of this conv's output formed
// in the input transform (backward data): winograd_f32.hip WgSrc
int ew_wino_f32_fwd_bn(uintptr_t bn_h, uintptr_t bn_stats, uintptr_t bn_code, uintptr_t nbt,
                       int pool, uintptr_t w, uintptr_t U, uintptr_t y, uintptr_t V,
                       uintptr_t Mo, long long N, int H, int W, int C, int Nc, int m,
                       uintptr_t bnpart, long long bnpart_floats, uintptr_t stream);
int ew_wino_f32_bwd_data_bn(uintptr_t out_h, uintptr_t out_dnext, uintptr_t out_code,
                            uintptr_t out_stats, uintptr_t out_coef, int out_pool, uintptr_t w,
                            uintptr_t U, uintptr_t dx, uintptr_t V, uintptr_t Mo, long long N,
                            int H, int W, int C, int Nc, int m, uintptr_t bn_h, uintptr_t bn_res,
                            uintptr_t bn_code, uintptr_t bn_stats, int bn_relu, uintptr_t bnpart,
                            long long bnpart_floats, uintptr_t addend, uintptr_t D,
                            uintptr_t wo_src, int wo_split, uintptr_t wo_dw, int wo_Nc, int wo_C,
                            uintptr_t stream);
// (wo_*: another layer's deferred weight-gradient output transform riding in the input launch)
int ew_wino_f32_wgrad(uintptr_t dy, uintptr_t V, uintptr_t dw, uintptr_t D, int d_ready,
                      uintptr_t U_scratch, uintptr_t ws, long long ws_floats, long long N, int H,
                      int W, int C, int Nc, int m, int defer_out, uintptr_t stream);
void ew_wino_f32_wgrad_out(uintptr_t src, int split, uintptr_t dw, int Nc, int C, int m,
                           uintptr_t stream);

// ---- fp32 3x3 convolutions over 2x2 maps as dense position GEMMs (smallmap_f32.hip): slab
// workspace floats and ticket ints (zeroed once; the kernels leave them zero) for N, C, Nc
long long ew_sm_f32_ws_floats(long long N, int C, int Nc);
int ew_sm_set_fence(int on);  // split-K hand-off with fences (1) or write-through (0); returns the previous
long long ew_sm_f32_counters(long long N, int C, int Nc);
int ew_sm_f32_fwd(uintptr_t x, uintptr_t bn_h, uintptr_t bn_stats, uintptr_t nbt, uintptr_t w,
                  uintptr_t y, uintptr_t slab, long long slab_floats, uintptr_t cnt,
                  long long cnt_ints, long long N, int C, int Nc, uintptr_t bnpart,
                  long long bnpart_floats, uintptr_t stream);
int ew_sm_f32_bwd(uintptr_t x, uintptr_t bn_h, uintptr_t bn_stats, uintptr_t dy,
                  uintptr_t out_h, uintptr_t out_dnext, uintptr_t out_code, uintptr_t out_stats,
                  uintptr_t out_coef, int out_pool, uintptr_t w, uintptr_t dx, uintptr_t dw,
                  uintptr_t slab, long long slab_floats, uintptr_t cnt, long long cnt_ints,
                  long long N, int C, int Nc, uintptr_t pb_h, uintptr_t pb_res, uintptr_t pb_code,
                  uintptr_t pb_stats, int pb_relu, uintptr_t bnpart, long long bnpart_floats,
                  uintptr_t fin_coef, uintptr_t fin_dgamma, uintptr_t fin_dbeta,
                  uintptr_t fin_dcbias, int fin_cb_bf16, long long fin_M, uintptr_t stream,
                  uintptr_t st_vel = 0, uintptr_t st_resid = 0, uintptr_t st_param = 0,
                  float st_momentum = 0.0f, float st_damp1 = 1.0f, float st_wd = 0.0f,
                  int st_nesterov = 0, uintptr_t st_lr = 0, uintptr_t st_stamp = 0);

// ---- LeNet's fp32 training step in four launches (lenet_f32.hip): persistent workspace floats
// and ticket ints (zeroed once; the kernels leave them zero) for batch B
long long ew_lenet_ws_floats(int B);
int ew_lenet_counters(int B);
void ew_lenet_set_prof(uintptr_t buf);  // probes: phase stamps of the conv backward (0: off)
void ew_lenet_fwd(uintptr_t x, uintptr_t w1, uintptr_t b1, uintptr_t w2, uintptr_t b2,
                  uintptr_t wf1, uintptr_t bf1, uintptr_t wf2, uintptr_t bf2, uintptr_t y, int B,
                  int K, uintptr_t a1, uintptr_t code1, uintptr_t a2, uintptr_t code2,
                  uintptr_t h1, uintptr_t logits, uintptr_t dlogits, uintptr_t dh1,
                  uintptr_t lossrow, uintptr_t loss, uintptr_t ws, long long ws_floats,
                  uintptr_t cnt, int cnt_ints, uintptr_t stream, uintptr_t bsrc = 0,
                  uintptr_t blabels = 0, uintptr_t bperm = 0, long long bperm_len = 0,
                  uintptr_t bstate = 0, uintptr_t bdone = 0, float bmean = 0.0f,
                  float binv_std = 1.0f);
void ew_lenet_bwd(uintptr_t x, uintptr_t w2, uintptr_t wf1, uintptr_t a1, uintptr_t code1,
                  uintptr_t a2, uintptr_t code2, uintptr_t h1, uintptr_t dlogits, uintptr_t dh1,
                  uintptr_t gscale, int B, int K, uintptr_t dp2, uintptr_t dw1, uintptr_t db1,
                  uintptr_t dw2, uintptr_t db2, uintptr_t dwf1, uintptr_t dbf1, uintptr_t dwf2,
                  uintptr_t dbf2, uintptr_t ws, long long ws_floats, uintptr_t cnt, int cnt_ints,
                  uintptr_t stream);

// ---- VGG classifier tail (fc2 + ReLU + fc3 + cross-entropy) and its backward (head_tail.hip)
long long ew_tail_ws_floats(int B, int N2);
int ew_tail_counters(int B);
void ew_tail_fwd(uintptr_t h1, uintptr_t w2, uintptr_t b2, uintptr_t w3, uintptr_t b3, uintptr_t y,
                 int B, int K1, int N2, int K, uintptr_t h2, uintptr_t logits, uintptr_t dlogits,
                 uintptr_t dh2, uintptr_t lossrow, uintptr_t loss, uintptr_t ws,
                 long long ws_floats, uintptr_t cnt, int cnt_ints, uintptr_t stream);
void ew_tail_bwd(uintptr_t h1, uintptr_t h2, uintptr_t dh2, uintptr_t dlogits, uintptr_t w2,
                 uintptr_t gscale, int B, int K1, int N2, int K, uintptr_t dh1, uintptr_t dw2,
                 uintptr_t db2, uintptr_t dw3, uintptr_t db3, uintptr_t stream);

// ---- RCCL communicator issuing collectives on the caller's stream (rccl_comm.hip) ----
// dtype codes: 0 f32, 1 bf16, 2 f16, 3 u8, 4 i32, 5 f64, 6 i64; op: 0 sum, 1 max, 2 min, 3 avg
std::string ew_rccl_unique_id();
int ew_rccl_version();
uintptr_t ew_rccl_init(const std::string& uid, int nranks, int rank, int device);
void ew_rccl_destroy(uintptr_t h);
void ew_rccl_abort(uintptr_t h);
uintptr_t ew_rccl_watchdog_start(uintptr_t comm, int device, double timeout_s, int exit_code);
void ew_rccl_watch(uintptr_t wd, uintptr_t stream);
int ew_rccl_watch_pending(uintptr_t wd);
void ew_rccl_watchdog_stop(uintptr_t wd);
uintptr_t ew_test_flag_alloc();
void ew_test_flag_free(uintptr_t f);
void ew_watchdog_release_flag(uintptr_t wd, uintptr_t f);
void ew_test_spin(uintptr_t flag, double max_s, uintptr_t stream);
void ew_rccl_all_gather(uintptr_t h, uintptr_t send, uintptr_t recv, long long count, int dtype,
                        uintptr_t stream);
void ew_rccl_all_reduce(uintptr_t h, uintptr_t send, uintptr_t recv, long long count, int dtype,
                        int op, uintptr_t stream);
void ew_rccl_reduce_scatter(uintptr_t h, uintptr_t send, uintptr_t recv, long long count,
                            int dtype, int op, uintptr_t stream);
void ew_rccl_broadcast(uintptr_t h, uintptr_t send, uintptr_t recv, long long count, int dtype,
                       int root, uintptr_t stream);
void ew_rccl_all_to_all(uintptr_t h, uintptr_t send, uintptr_t recv, long long count, int dtype,
                        int nranks, uintptr_t stream);

// ---- cross-entropy loss (nn.hip): mean over B rows of [B, K] logits (bf16 or fp32), int64 labels
void ew_cross_entropy_fwd(uintptr_t x, uintptr_t y, int B, int K, int is_bf16, uintptr_t loss,
                          uintptr_t lse, uintptr_t stream, uintptr_t dx);
void ew_cross_entropy_bwd(uintptr_t x, uintptr_t y, uintptr_t lse, uintptr_t grad, int B, int K,
                          int is_bf16, uintptr_t dx, uintptr_t stream);

// ---- classifier-head activation + dropout (nn.hip), bf16 [rows, C]; ctr int32[2] per layer
void ew_act_dropout_fwd(uintptr_t y, uintptr_t z, int n, float p, int relu, uintptr_t ctr,
                        uint32_t salt, uintptr_t stream);
void ew_act_dropout_bwd(uintptr_t dz, uintptr_t y, uintptr_t dy, uintptr_t db, int db_bf16,
                        int rows, int C, float p, int relu, uintptr_t ctr, uint32_t salt,
                        uintptr_t stream);
