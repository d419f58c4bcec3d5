// Shared by the fp32 convolution kernels (conv_f32.hip, winograd_f32.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

// Backward-statistics operands of the BN(+ReLU)(+2x2 max pool)(+residual) layer whose output
// gradient a backward-data launch produces (conv.hip CvBnBwd, fp32 tensors): the epilogue sums
// dz = act'(h * scale + shift [+ res]) * dx and dz * (h - mean) per channel (the BN backward then
// skips its statistics pass).
struct CfBnBwd {
  const float* h;       // BN input [rows (pre-pool)][C]; null: not requested
  const float* res;     // residual input (BN + residual + ReLU) or null
  const uint8_t* code;  // pool window codes [rows][C] (null: no pool)
  const float* stats;   // [4][C]: mean, invstd, scale, shift
  int relu;
  int Ho, Wo;           // pooled map dims (pool)
};

__device__ __forceinline__ uint32_t cf_pool_row(uint32_t p, uint32_t HoWo, uint32_t Wo,
                                                uint32_t q) {
  const uint32_t n = p / HoWo, rem = p - n * HoWo;
  const uint32_t ho = rem / Wo, wo = rem - ho * Wo;
  return 4 * n * HoWo + 4 * ho * Wo + 2 * wo + (q >> 1) * (2 * Wo) + (q & 1);
}
