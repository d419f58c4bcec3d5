// Dense QSGD (reference Method 4, Compresssor/qsgd.py:12-40) of a flat gradient bucket into real
// int8 / int4 codes, and the fused decode -> average -> SGD on the receive side.  gfx950, wave64.
//
// Encode: stats (per-chunk sum of squares + per-tensor max key, one read), scale (one block per
// tensor, fixed-order reduction -> bitwise reproducible), quant (one read, one code write with
// per-element counter RNG).  Each thread owns a group of 4 consecutive elements, so int8 codes are
// one 32-bit store and int4 codes one 16-bit store per group.
#include "common.h"
#include "ewdml_ops.h"

namespace {

template <bool EF>
__global__ __launch_bounds__(EW_BLOCK) void k_qsgd_stats(GradPtrs gp,
                                                         float* __restrict__ resid,
                                                         const ChunkRow* __restrict__ chunks,
                                                         float* __restrict__ chunk_sq,
                                                         uint32_t* __restrict__ maxkey) {
  __shared__ float wsf[EW_WAVES];
  const ChunkRow c = chunks[blockIdx.x];
  float sq = 0.0f;
  uint32_t km = 0;
  for (int i = 4 * threadIdx.x; i < c.len; i += 4 * EW_BLOCK) {
    float xs[4];
    ew_ld4t(gp, nullptr, c, i, xs);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (i + j < c.len) {
        float x = xs[j];
        if (EF) {  // stage e = g + residual in the residual buffer
          x = x + resid[c.start + i + j];
          resid[c.start + i + j] = x;
        }
        sq = sq + x * x;
        km = max(km, ew_key(x));
      }
    }
  }
  km = ew_wave_max_u(km);
  if ((threadIdx.x & 63) == 0) atomicMax(&maxkey[c.tensor], km);
  const float s = ew_block_sum(sq, wsf);
  if (threadIdx.x == 0) chunk_sq[blockIdx.x] = s;
}

__global__ __launch_bounds__(EW_BLOCK) void k_qsgd_scale(const TensorRow* __restrict__ tensors,
                                                         const float* __restrict__ chunk_sq,
                                                         const uint32_t* __restrict__ maxkey,
                                                         float* __restrict__ inv_out,
                                                         uint8_t* __restrict__ payload,
                                                         int scales_off, float levels, int norm_l2) {
  __shared__ float wsf[EW_WAVES];
  const int t = blockIdx.x;
  const TensorRow tr = tensors[t];
  float sq = 0.0f;
  for (int j = threadIdx.x; j < tr.nchunks; j += EW_BLOCK) sq = sq + chunk_sq[tr.chunk0 + j];
  const float total = ew_block_sum(sq, wsf);
  if (threadIdx.x == 0) {
    const float scale = norm_l2 ? sqrtf(total) : __uint_as_float(maxkey[t]);
    reinterpret_cast<float*>(payload + scales_off)[t] = scale;
    inv_out[t] = scale > 0.0f ? levels / scale : 0.0f;
  }
}

template <int BITS, bool EF>
__global__ __launch_bounds__(EW_BLOCK) void k_qsgd_quant(
    GradPtrs gp, float* __restrict__ resid, const ChunkRow* __restrict__ chunks,
    const TensorRow* __restrict__ tensors, const float* __restrict__ inv_arr,
    uint8_t* __restrict__ payload, int scales_off, int codes_off, float levels, float inv_levels,
    uint32_t key_arg, const uint32_t* __restrict__ keyp, uint32_t bucket_offset) {
  const uint32_t key = keyp ? *keyp : key_arg;
  const ChunkRow c = chunks[blockIdx.x];
  const TensorRow tr = tensors[c.tensor];
  const float* flat = EF ? resid : nullptr;
  const float inv = inv_arr[c.tensor];
  const float step = reinterpret_cast<const float*>(payload + scales_off)[c.tensor] * inv_levels;
  const uint32_t gbase = bucket_offset + (uint32_t)c.start;
  const long long cbase = (long long)tr.code0 + (long long)c.local * EW_CHUNK;
  for (int i = 4 * threadIdx.x; i < c.len; i += 4 * EW_BLOCK) {
    float xs[4];
    ew_ld4t(gp, flat, c, i, xs);
    int q[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      q[j] = (i + j < c.len) ? ew_quantize(xs[j], inv, levels, gbase + (uint32_t)(i + j), key) : 0;
      if (EF && i + j < c.len) resid[c.start + i + j] = xs[j] - (float)q[j] * step;
    }
    if (BITS == 8) {
      const uint32_t w = (uint32_t)(q[0] & 0xff) | ((uint32_t)(q[1] & 0xff) << 8) |
                         ((uint32_t)(q[2] & 0xff) << 16) | ((uint32_t)(q[3] & 0xff) << 24);
      *reinterpret_cast<uint32_t*>(payload + codes_off + cbase + i) = w;
    } else {
      const uint16_t w = (uint16_t)((q[0] & 0xf) | ((q[1] & 0xf) << 4) | ((q[2] & 0xf) << 8) |
                                    ((q[3] & 0xf) << 12));
      *reinterpret_cast<uint16_t*>(payload + codes_off + ((cbase + i) >> 1)) = w;
    }
  }
}

__device__ __forceinline__ int ew_nib(uint32_t w, int j) {
  const int q = (int)((w >> (4 * j)) & 0xfu);
  return q >= 8 ? q - 16 : q;
}

template <int BITS>
__global__ __launch_bounds__(EW_BLOCK) void k_qsgd_decode_apply(
    const uint8_t* __restrict__ recv, int nranks, long long stride,
    const ChunkRow* __restrict__ chunks, const TensorRow* __restrict__ tensors, int scales_off,
    int codes_off, float inv_levels, float* __restrict__ param, float* __restrict__ mom,
    float* __restrict__ grad_out, uint16_t* __restrict__ shadow, SgdArgs sa, int apply) {
  const ChunkRow c = chunks[blockIdx.x];
  ew_sgd_resolve(sa);
  const TensorRow tr = tensors[c.tensor];
  ew_key_advance(sa);
  const long long cbase = (long long)tr.code0 + (long long)c.local * EW_CHUNK;
  float* p = param + c.start;
  float* b = mom + c.start;
  float* go = grad_out ? grad_out + c.start : nullptr;
  for (int i = 4 * threadIdx.x; i < c.len; i += 4 * EW_BLOCK) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < nranks; ++r) {
      const uint8_t* pay = recv + r * stride;
      const float step = reinterpret_cast<const float*>(pay + scales_off)[c.tensor] * inv_levels;
      if (BITS == 8) {
        const uint32_t w = *reinterpret_cast<const uint32_t*>(pay + codes_off + cbase + i);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float prod = (float)(int8_t)((w >> (8 * j)) & 0xffu) * step;
          acc[j] = acc[j] + prod;
        }
      } else {
        const uint32_t w = *reinterpret_cast<const uint16_t*>(pay + codes_off + ((cbase + i) >> 1));
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float prod = (float)ew_nib(w, j) * step;
          acc[j] = acc[j] + prod;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (i + j < c.len) {
        const float gv = acc[j] * sa.grad_scale;
        if (go) go[i + j] = gv;
        if (apply) {
          float pv = p[i + j], bv = b[i + j];
          ew_sgd(pv, bv, gv, sa);
          p[i + j] = pv;
          b[i + j] = bv;
          if (shadow) shadow[c.start + i + j] = ew_f2bf(pv);
        }
      }
    }
  }
}

}  // namespace

#define EW_LAUNCH(kern, grid, stream, ...) \
  hipLaunchKernelGGL(kern, dim3(grid), dim3(EW_BLOCK), 0, (hipStream_t)(stream), __VA_ARGS__)

size_t ew_qsgd_scratch_bytes(int T, int C) {
  // maxkey[T] | chunk_sq[C] | inv[T]
  return sizeof(uint32_t) * ((size_t)2 * T + C);
}

void ew_qsgd_encode(const QsgdEncodeArgs& a) {
  auto* chunks = reinterpret_cast<const ChunkRow*>(a.chunks);
  auto* tensors = reinterpret_cast<const TensorRow*>(a.tensors);
  const int T = a.num_tensors, C = a.num_chunks;
  uint32_t* maxkey = reinterpret_cast<uint32_t*>(a.scratch);
  float* chunk_sq = reinterpret_cast<float*>(maxkey + T);
  float* inv = chunk_sq + C;
  hipStream_t s = (hipStream_t)a.stream;
  EW_CHECK(hipMemsetAsync(reinterpret_cast<void*>(a.scratch), 0, ew_qsgd_scratch_bytes(T, C), s));
  GradPtrs g;
  ew_fill_ptrs(g, a.grad_ptrs, a.n_grad_ptrs, T, a.bf16_mask, a.n_bf16_mask);
  float* resid = reinterpret_cast<float*>(a.resid);
  auto* pay = reinterpret_cast<uint8_t*>(a.payload);
  if (resid)
    EW_LAUNCH(k_qsgd_stats<true>, C, s, g, resid, chunks, chunk_sq, maxkey);
  else
    EW_LAUNCH(k_qsgd_stats<false>, C, s, g, resid, chunks, chunk_sq, maxkey);
  EW_LAUNCH(k_qsgd_scale, T, s, tensors, chunk_sq, maxkey, inv, pay, a.scales_off, a.levels,
            a.norm_l2);
#define EW_Q(B, EFV)                                                                             \
  EW_LAUNCH((k_qsgd_quant<B, EFV>), C, s, g, resid, chunks, tensors, inv, pay, a.scales_off,      \
            a.codes_off, a.levels, a.inv_levels, a.key,                                          \
            reinterpret_cast<const uint32_t*>(a.key_ptr), a.bucket_offset)
  if (a.bits == 8) {
    if (resid) EW_Q(8, true); else EW_Q(8, false);
  } else {
    if (resid) EW_Q(4, true); else EW_Q(4, false);
  }
#undef EW_Q
  EW_CHECK_LAUNCH();
}

void ew_qsgd_decode_apply(const QsgdDecodeArgs& a) {
  auto* chunks = reinterpret_cast<const ChunkRow*>(a.chunks);
  auto* tensors = reinterpret_cast<const TensorRow*>(a.tensors);
  SgdArgs sa{a.lr, a.momentum, a.dampening, a.weight_decay, a.grad_scale, a.nesterov, a.first,
             reinterpret_cast<uint32_t*>(a.key_state), a.key_seed, a.key_rank};
  sa.lr_ptr = reinterpret_cast<const float*>(a.lr_ptr);
  auto* recv = reinterpret_cast<const uint8_t*>(a.recv);
  auto* p = reinterpret_cast<float*>(a.param);
  auto* m = reinterpret_cast<float*>(a.mom);
  auto* go = reinterpret_cast<float*>(a.grad_out);
  auto* sh = reinterpret_cast<uint16_t*>(a.shadow);
  if (a.bits == 8)
    EW_LAUNCH(k_qsgd_decode_apply<8>, a.num_chunks, a.stream, recv, a.nranks, a.stride, chunks,
              tensors, a.scales_off, a.codes_off, a.inv_levels, p, m, go, sh, sa, a.apply);
  else
    EW_LAUNCH(k_qsgd_decode_apply<4>, a.num_chunks, a.stream, recv, a.nranks, a.stride, chunks,
              tensors, a.scales_off, a.codes_off, a.inv_levels, p, m, go, sh, sa, a.apply);
  EW_CHECK_LAUNCH();
}
