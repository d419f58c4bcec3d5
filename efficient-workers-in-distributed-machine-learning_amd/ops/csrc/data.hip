// Fused input pipeline: one kernel builds a training batch straight from the
// HBM-resident uint8 dataset -- sampler gather, CIFAR augmentation (reflect-pad, random crop,
// random horizontal flip; reference util.py:38-48), /255, per-channel normalisation, layout
// (NCHW or channels_last) and dtype (fp32 or bf16) conversion, label gather.
//
// The batch position comes from a device-resident state {pos, epoch}, so the launch can live
// inside the captured HIP graph: the last block to finish advances pos (grid arrival ticket in
// `done`, EW_TICKET_INTS ints), the host only rewrites the state at an epoch boundary.
// Augmentation draws are a counter hash of (seed, rank, epoch, sample slot): reproducible and
// independent of launch order or graph replay.
#include "common.h"
#include "ewdml_ops.h"

namespace {

struct NormArgs {
  float mean[4];
  float inv_std[4];
};

__device__ __forceinline__ int ew_reflect(int i, int n) {
  i = i < 0 ? -i : i;
  return i >= n ? 2 * n - 2 - i : i;
}

template <typename OUT, bool CL>
__global__ __launch_bounds__(EW_BLOCK) void k_make_batch(
    const uint8_t* __restrict__ src, const long long* __restrict__ labels,
    const long long* __restrict__ perm, long long* __restrict__ state,
    unsigned* __restrict__ done, long long perm_len, int B, int C, int H, int W, int pad,
    int augment, uint32_t seed, uint32_t rank, NormArgs na, OUT* __restrict__ out, long long* __restrict__ out_y) {
  const long long pos = state[0];
  const uint32_t epoch = (uint32_t)state[1];
  const uint32_t HW = (uint32_t)H * W;
  const uint32_t total = (uint32_t)B * HW;
  const uint32_t pix = blockIdx.x * EW_BLOCK + threadIdx.x;
  if (pix < total) {
    const uint32_t b = pix / HW;
    const uint32_t rem = pix - b * HW;
    const int y = (int)(rem / W), x = (int)(rem - (rem / W) * W);
    long long slot = pos * B + b;
    if (slot >= perm_len) slot %= perm_len;  // never read past the permutation
    const long long sample = perm[slot];
    int sy = y, sx = x;
    if (augment) {
      const uint32_t hsh = ew_mix32(ew_mix32(seed * 0x9E3779B9u + rank) ^
                                    ew_mix32(epoch * 0x85EBCA6Bu + (uint32_t)slot));
      const uint32_t span = 2 * pad + 1;
      const int dy = (int)((hsh & 0xffu) % span), dx = (int)(((hsh >> 8) & 0xffu) % span);
      const bool flip = (hsh >> 16) & 1u;
      sy = ew_reflect(y + dy - pad, H);
      sx = ew_reflect((flip ? W - 1 - x : x) + dx - pad, W);
    }
    const uint8_t* s = src + (size_t)sample * C * HW + (size_t)sy * W + sx;
    for (int c = 0; c < C; ++c) {
      const float v = ((float)s[(size_t)c * HW] * (1.0f / 255.0f) - na.mean[c]) * na.inv_std[c];
      const size_t o = CL ? ((size_t)pix * C + c) : (((size_t)b * C + c) * HW + rem);
      if constexpr (sizeof(OUT) == 2) out[o] = ew_f2bf(v);
      else out[o] = v;
    }
    if (rem == 0) out_y[b] = labels[sample];
  }
  // The last block to arrive advances the batch position for the next launch.  No fences: the
  // only cross-block hazard is a block reading state[0] after it was advanced, and every block's
  // read completed before its barrier (the workgroup barrier waits for outstanding loads), hence
  // before its arrival ticket; the next kernel sees the new value at the kernel boundary.  (An
  // agent-scope release fence per block costs an L2 write-back on gfx950.)
  __syncthreads();
  if (threadIdx.x == 0 && ew_grid_last(reinterpret_cast<int*>(done))) state[0] = pos + 1;
}

}  // namespace

void ew_make_batch(const MakeBatchArgs& a) {
  NormArgs na{};
  for (int c = 0; c < 4; ++c) {
    na.mean[c] = a.mean[c];
    na.inv_std[c] = a.inv_std[c];
  }
  const long long total = (long long)a.B * a.H * a.W;
  const int grid = (int)((total + EW_BLOCK - 1) / EW_BLOCK);
  hipStream_t s = (hipStream_t)a.stream;
  const uint8_t* src = reinterpret_cast<const uint8_t*>(a.src);
  const long long* labels = reinterpret_cast<const long long*>(a.labels);
  const long long* perm = reinterpret_cast<const long long*>(a.perm);
  long long* state = reinterpret_cast<long long*>(a.state);
  unsigned* done = reinterpret_cast<unsigned*>(a.done);
  long long* oy = reinterpret_cast<long long*>(a.out_y);
#define EW_MB(OUT, CL)                                                                          \
  hipLaunchKernelGGL((k_make_batch<OUT, CL>), dim3(grid), dim3(EW_BLOCK), 0, s, src, labels,    \
                     perm, state, done, a.perm_len, a.B, a.C, a.H, a.W, a.pad, a.augment, a.seed,  \
                     a.rank, na, reinterpret_cast<OUT*>(a.out), oy)
  if (a.out_bf16) {
    if (a.channels_last) EW_MB(uint16_t, true);
    else EW_MB(uint16_t, false);
  } else {
    if (a.channels_last) EW_MB(float, true);
    else EW_MB(float, false);
  }
#undef EW_MB
  EW_CHECK_LAUNCH();
}
