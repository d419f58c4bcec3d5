// Multi-tensor optimizers over the flat parameter buffer (one launch for the whole model) and the
// fp32 -> bf16/fp16 cast used by the low-precision all-reduce.  gfx950, wave64, float4 I/O.
//
// Parity: optim/sgd.py:59-91 (SGD with explicit grads: weight decay, momentum buffer initialised
// to the first gradient, dampening, Nesterov) and optim/adam.py:38-94 (Adam / AMSGrad).  The
// reference runs one small launch per parameter tensor; here the 38 (VGG-11) to 161 (ResNet-50)
// tensors are one flat range.
#include "common.h"
#include "ewdml_ops.h"
#include <hip/hip_fp16.h>

namespace {

__device__ __forceinline__ float ew_bf16_to_f32(uint16_t v) { return __uint_as_float((uint32_t)v << 16); }
__device__ __forceinline__ uint16_t ew_f32_to_bf16(float x) { return ew_f2bf(x); }

template <int GT>
__device__ __forceinline__ void ew_load_grad4(const void* g, long long i, float out[4]) {
  if (GT == 0) {
    const float4 v = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(g) + i);
    out[0] = v.x; out[1] = v.y; out[2] = v.z; out[3] = v.w;
  } else if (GT == 1) {
    const uint2 v = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(g) + i);
    out[0] = ew_bf16_to_f32(v.x & 0xffff); out[1] = ew_bf16_to_f32(v.x >> 16);
    out[2] = ew_bf16_to_f32(v.y & 0xffff); out[3] = ew_bf16_to_f32(v.y >> 16);
  } else {
    const __half* h = reinterpret_cast<const __half*>(g) + i;
#pragma unroll
    for (int j = 0; j < 4; ++j) out[j] = __half2float(h[j]);
  }
}

template <int GT>
__global__ __launch_bounds__(EW_BLOCK) void k_sgd_flat(float* __restrict__ p, float* __restrict__ mom,
                                                       const void* __restrict__ g, long long n4,
                                                       uint16_t* __restrict__ shadow, SgdArgs sa) {
  ew_sgd_resolve(sa);
  for (long long v = blockIdx.x * (long long)EW_BLOCK + threadIdx.x; v < n4;
       v += (long long)gridDim.x * EW_BLOCK) {
    float gv[4];
    ew_load_grad4<GT>(g, 4 * v, gv);
    float4 pv = reinterpret_cast<float4*>(p)[v];
    float4 bv = reinterpret_cast<float4*>(mom)[v];
    ew_sgd(pv.x, bv.x, gv[0] * sa.grad_scale, sa);
    ew_sgd(pv.y, bv.y, gv[1] * sa.grad_scale, sa);
    ew_sgd(pv.z, bv.z, gv[2] * sa.grad_scale, sa);
    ew_sgd(pv.w, bv.w, gv[3] * sa.grad_scale, sa);
    reinterpret_cast<float4*>(p)[v] = pv;
    reinterpret_cast<float4*>(mom)[v] = bv;
    if (shadow) {
      const float w[4] = {pv.x, pv.y, pv.z, pv.w};
      ew_st4_bf16(shadow + 4 * v, 4, w);
    }
  }
}

struct AdamArgs {
  float lr_step, beta1, beta2, eps, weight_decay, grad_scale, bc2_sqrt;
  int amsgrad;
  // device step counter (nullable): t = *step + 1 is read at run time and lr_step =
  // lr * sqrt(1 - beta2^t) / (1 - beta1^t) computed from it, so a captured HIP graph replays
  // the bias correction of the current step (the host value is frozen at capture)
  const int* step;
  double lr;
  const float* lr_ptr;  // nullable device base lr
};

__device__ __forceinline__ void ew_adam_resolve(AdamArgs& a) {
  if (a.step) {
    const double t = (double)(*a.step + 1);
    const double lr = a.lr_ptr ? (double)*a.lr_ptr : a.lr;
    a.lr_step = (float)(lr * sqrt(1.0 - pow((double)a.beta2, t)) /
                        (1.0 - pow((double)a.beta1, t)));
  }
}

__device__ __forceinline__ void ew_adam(float& p, float& m, float& v, float& vm, float g,
                                        const AdamArgs& a) {
  if (a.weight_decay != 0.0f) g = g + a.weight_decay * p;
  m = m * a.beta1 + (1.0f - a.beta1) * g;
  v = v * a.beta2 + (1.0f - a.beta2) * (g * g);
  float d;
  if (a.amsgrad) {
    vm = fmaxf(vm, v);
    d = sqrtf(vm) + a.eps;
  } else {
    d = sqrtf(v) + a.eps;
  }
  p = p - a.lr_step * (m / d);
}

template <int GT>
__global__ __launch_bounds__(EW_BLOCK) void k_adam_flat(float* __restrict__ p, float* __restrict__ m,
                                                        float* __restrict__ v, float* __restrict__ vm,
                                                        const void* __restrict__ g, long long n4,
                                                        uint16_t* __restrict__ shadow, AdamArgs a) {
  ew_adam_resolve(a);
  for (long long i = blockIdx.x * (long long)EW_BLOCK + threadIdx.x; i < n4;
       i += (long long)gridDim.x * EW_BLOCK) {
    float gv[4];
    ew_load_grad4<GT>(g, 4 * i, gv);
    float4 pv = reinterpret_cast<float4*>(p)[i];
    float4 mv = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    float4 xv = a.amsgrad ? reinterpret_cast<float4*>(vm)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    ew_adam(pv.x, mv.x, vv.x, xv.x, gv[0] * a.grad_scale, a);
    ew_adam(pv.y, mv.y, vv.y, xv.y, gv[1] * a.grad_scale, a);
    ew_adam(pv.z, mv.z, vv.z, xv.z, gv[2] * a.grad_scale, a);
    ew_adam(pv.w, mv.w, vv.w, xv.w, gv[3] * a.grad_scale, a);
    reinterpret_cast<float4*>(p)[i] = pv;
    reinterpret_cast<float4*>(m)[i] = mv;
    reinterpret_cast<float4*>(v)[i] = vv;
    if (a.amsgrad) reinterpret_cast<float4*>(vm)[i] = xv;
    if (shadow) {
      const float w[4] = {pv.x, pv.y, pv.z, pv.w};
      ew_st4_bf16(shadow + 4 * i, 4, w);
    }
  }
}

__global__ __launch_bounds__(EW_BLOCK) void k_cast_scale(const float* __restrict__ src,
                                                         void* __restrict__ dst, long long n4,
                                                         float scale, int to_bf16) {
  for (long long i = blockIdx.x * (long long)EW_BLOCK + threadIdx.x; i < n4;
       i += (long long)gridDim.x * EW_BLOCK) {
    const float4 x = reinterpret_cast<const float4*>(src)[i];
    const float y[4] = {x.x * scale, x.y * scale, x.z * scale, x.w * scale};
    if (to_bf16) {
      uint2 o;
      o.x = (uint32_t)ew_f32_to_bf16(y[0]) | ((uint32_t)ew_f32_to_bf16(y[1]) << 16);
      o.y = (uint32_t)ew_f32_to_bf16(y[2]) | ((uint32_t)ew_f32_to_bf16(y[3]) << 16);
      reinterpret_cast<uint2*>(dst)[i] = o;
    } else {
      __half* h = reinterpret_cast<__half*>(dst) + 4 * i;
#pragma unroll
      for (int j = 0; j < 4; ++j) h[j] = __float2half(y[j]);
    }
  }
}

// Gather a bucket's per-tensor gradients into the flat (fp32 / bf16 / fp16) all-reduce buffer,
// scaled -- one launch per bucket replaces per-parameter copies (dense codecs).
__global__ __launch_bounds__(EW_BLOCK) void k_pack_grads(GradPtrs gp,
                                                         const ChunkRow* __restrict__ chunks,
                                                         void* __restrict__ dst, int dst_dtype,
                                                         float scale) {
  const ChunkRow c = chunks[blockIdx.x];
  for (int i = 4 * threadIdx.x; i < c.len; i += 4 * EW_BLOCK) {
    float y[4];
    ew_ld4t(gp, nullptr, c, i, y);
#pragma unroll
    for (int j = 0; j < 4; ++j) y[j] = y[j] * scale;
    const long long o = (long long)c.start + i;
    if (dst_dtype == 0) {
      float* d = reinterpret_cast<float*>(dst) + o;
      if (i + 3 < c.len) *reinterpret_cast<float4*>(d) = make_float4(y[0], y[1], y[2], y[3]);
      else for (int j = 0; j < 4 && i + j < c.len; ++j) d[j] = y[j];
    } else if (dst_dtype == 1) {
      uint16_t* d = reinterpret_cast<uint16_t*>(dst) + o;
      for (int j = 0; j < 4 && i + j < c.len; ++j) d[j] = ew_f32_to_bf16(y[j]);
    } else {
      __half* d = reinterpret_cast<__half*>(dst) + o;
      for (int j = 0; j < 4 && i + j < c.len; ++j) d[j] = __float2half(y[j]);
    }
  }
}

// SGD step of one bucket straight from autograd's per-tensor gradients (pointer table): the
// local steps of local SGD (Method 6) read each gradient in place, as the codec passes do -- no
// accumulate-add into a flat gradient buffer, no separate gather.  Block = one chunk row.
__global__ __launch_bounds__(EW_BLOCK) void k_sgd_ptrs(GradPtrs gp,
                                                       const ChunkRow* __restrict__ chunks,
                                                       float* __restrict__ p,
                                                       float* __restrict__ mom,
                                                       uint16_t* __restrict__ shadow, SgdArgs sa) {
  ew_sgd_resolve(sa);
  const ChunkRow c = chunks[blockIdx.x];
  for (int i = 4 * threadIdx.x; i < c.len; i += 4 * EW_BLOCK) {
    float gv[4];
    ew_ld4t(gp, nullptr, c, i, gv);
    const long long o = (long long)c.start + i;
    const int k = c.len - i < 4 ? c.len - i : 4;
    if (k == 4) {
      float4 pv = *reinterpret_cast<float4*>(p + o);
      float4 bv = *reinterpret_cast<float4*>(mom + o);
      ew_sgd(pv.x, bv.x, gv[0] * sa.grad_scale, sa);
      ew_sgd(pv.y, bv.y, gv[1] * sa.grad_scale, sa);
      ew_sgd(pv.z, bv.z, gv[2] * sa.grad_scale, sa);
      ew_sgd(pv.w, bv.w, gv[3] * sa.grad_scale, sa);
      *reinterpret_cast<float4*>(p + o) = pv;
      *reinterpret_cast<float4*>(mom + o) = bv;
      if (shadow) {
        const float w[4] = {pv.x, pv.y, pv.z, pv.w};
        ew_st4_bf16(shadow + o, 4, w);
      }
    } else {
      for (int j = 0; j < k; ++j) {
        ew_sgd(p[o + j], mom[o + j], gv[j] * sa.grad_scale, sa);
        if (shadow) shadow[o + j] = ew_f32_to_bf16(p[o + j]);
      }
    }
  }
}

inline int ew_grid(long long n4) {
  long long b = (n4 + EW_BLOCK - 1) / EW_BLOCK;
  return (int)(b < 2048 ? (b > 0 ? b : 1) : 2048);  // 8 blocks per CU, grid-stride the rest
}

}  // namespace

void ew_sgd_flat(const SgdFlatArgs& a) {
  SgdArgs sa{a.lr, a.momentum, a.dampening, a.weight_decay, a.grad_scale, a.nesterov, a.first};
  sa.lr_ptr = reinterpret_cast<const float*>(a.lr_ptr);
  const long long n4 = a.n / 4;
  auto* p = reinterpret_cast<float*>(a.param);
  auto* m = reinterpret_cast<float*>(a.mom);
  auto* g = reinterpret_cast<const void*>(a.grad);
  auto* sh = reinterpret_cast<uint16_t*>(a.shadow);
  hipStream_t s = (hipStream_t)a.stream;
  if (a.grad_dtype == 0)
    hipLaunchKernelGGL(k_sgd_flat<0>, dim3(ew_grid(n4)), dim3(EW_BLOCK), 0, s, p, m, g, n4, sh, sa);
  else if (a.grad_dtype == 1)
    hipLaunchKernelGGL(k_sgd_flat<1>, dim3(ew_grid(n4)), dim3(EW_BLOCK), 0, s, p, m, g, n4, sh, sa);
  else
    hipLaunchKernelGGL(k_sgd_flat<2>, dim3(ew_grid(n4)), dim3(EW_BLOCK), 0, s, p, m, g, n4, sh, sa);
  EW_CHECK_LAUNCH();
}

void ew_adam_flat(const AdamFlatArgs& a) {
  AdamArgs aa{a.lr_step, a.beta1,      a.beta2,   a.eps,
              a.weight_decay, a.grad_scale, a.bc2_sqrt, a.amsgrad,
              reinterpret_cast<const int*>(a.step), a.lr,
              reinterpret_cast<const float*>(a.lr_ptr)};
  const long long n4 = a.n / 4;
  auto* p = reinterpret_cast<float*>(a.param);
  auto* m = reinterpret_cast<float*>(a.exp_avg);
  auto* v = reinterpret_cast<float*>(a.exp_avg_sq);
  auto* vm = reinterpret_cast<float*>(a.max_exp_avg_sq);
  auto* g = reinterpret_cast<const void*>(a.grad);
  auto* sh = reinterpret_cast<uint16_t*>(a.shadow);
  hipStream_t s = (hipStream_t)a.stream;
  if (a.grad_dtype == 0)
    hipLaunchKernelGGL(k_adam_flat<0>, dim3(ew_grid(n4)), dim3(EW_BLOCK), 0, s, p, m, v, vm, g, n4, sh, aa);
  else if (a.grad_dtype == 1)
    hipLaunchKernelGGL(k_adam_flat<1>, dim3(ew_grid(n4)), dim3(EW_BLOCK), 0, s, p, m, v, vm, g, n4, sh, aa);
  else
    hipLaunchKernelGGL(k_adam_flat<2>, dim3(ew_grid(n4)), dim3(EW_BLOCK), 0, s, p, m, v, vm, g, n4, sh, aa);
  EW_CHECK_LAUNCH();
}

void ew_pack_grads(const uintptr_t* grad_ptrs, int n_ptrs, const uint32_t* bf16_mask, int n_mask,
                   int num_tensors, uintptr_t chunks, int num_chunks, uintptr_t dst,
                   int dst_dtype, float scale, uintptr_t stream) {
  GradPtrs g;
  ew_fill_ptrs(g, grad_ptrs, n_ptrs, num_tensors, bf16_mask, n_mask);
  hipLaunchKernelGGL(k_pack_grads, dim3(num_chunks), dim3(EW_BLOCK), 0, (hipStream_t)stream, g,
                     reinterpret_cast<const ChunkRow*>(chunks), reinterpret_cast<void*>(dst),
                     dst_dtype, scale);
  EW_CHECK_LAUNCH();
}

void ew_sgd_ptrs(const uintptr_t* grad_ptrs, int n_ptrs, const uint32_t* bf16_mask, int n_mask,
                 int num_tensors, uintptr_t chunks, int num_chunks, const SgdFlatArgs& a) {
  GradPtrs g;
  ew_fill_ptrs(g, grad_ptrs, n_ptrs, num_tensors, bf16_mask, n_mask);
  SgdArgs sa{a.lr, a.momentum, a.dampening, a.weight_decay, a.grad_scale, a.nesterov, a.first};
  sa.lr_ptr = reinterpret_cast<const float*>(a.lr_ptr);
  hipLaunchKernelGGL(k_sgd_ptrs, dim3(num_chunks), dim3(EW_BLOCK), 0, (hipStream_t)a.stream, g,
                     reinterpret_cast<const ChunkRow*>(chunks), reinterpret_cast<float*>(a.param),
                     reinterpret_cast<float*>(a.mom), reinterpret_cast<uint16_t*>(a.shadow), sa);
  EW_CHECK_LAUNCH();
}

void ew_cast_scale(uintptr_t src, uintptr_t dst, long long n, float scale, int to_bf16,
                   uintptr_t stream) {
  const long long n4 = n / 4;
  hipLaunchKernelGGL(k_cast_scale, dim3(ew_grid(n4)), dim3(EW_BLOCK), 0, (hipStream_t)stream,
                     reinterpret_cast<const float*>(src), reinterpret_cast<void*>(dst), n4, scale,
                     to_bf16);
  EW_CHECK_LAUNCH();
}
