// Micro-benchmark of the fp32 GEMM k-loop shape (ops/csrc/conv_f32.hip k_cf_gemm<*, 128, 128, 2,
// 4, 32>): 8 waves per block, one block per CU, each wave 2 accumulators of
// v_mfma_f32_32x32x2_f32 (32 MFMAs per 32-deep k-step) fed by 12 ds_read_b128 per step.
// Variants (argv[1]): 0 = MFMAs only (operands in registers), 1 = + LDS fragment reads,
// 2 = + a barrier per step, 3 = + 4 ds_write_b128 per thread per step before the barrier (the
// real loop minus global loads).  Prints TF/s per variant; the fp32 MFMA peak is ~157 TF/s.
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/mfma_loop_probe tools/probes/mfma_loop_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int V, int AHEAD = 2, bool RND = false>
__global__ __launch_bounds__(512) void k_loop(float* out, int steps, const float* __restrict__ src,
                                              long long src_floats) {
  __shared__ __attribute__((aligned(16))) char smem[65536];
  const int t = threadIdx.x, lane = t & 63;
  // RND: pseudo-random operands (switching activity, i.e. power, as with real data); else
  // near-constant ones
  for (int i = t; i < 65536 / 16; i += 512) {
    unsigned h = (unsigned)i * 2654435761u + blockIdx.x * 97u;
    auto r = [&]() { h ^= h << 13; h ^= h >> 17; h ^= h << 5; return (float)(h & 0xffff) * 3e-5f - 1.0f; };
    reinterpret_cast<f32x4*>(smem)[i] = RND ? f32x4{r(), r(), r(), r()} : f32x4{1e-3f, 0, 0, 0};
  }
  __syncthreads();
  f32x16 acc0 = {}, acc1 = {};
  f32x4 a[4][2], b[4];
  for (int r = 0; r < 4; ++r) {
    a[r][0] = a[r][1] = b[r] = f32x4{(float)lane * 1e-6f, 1e-6f, 2e-6f, 3e-6f};
  }
  const int wq = t >> 6;
  const int off = ((wq * 64 + lane) * 16) & 32767;
  // V >= 4: 4 x 16-B global loads per thread per step (a 32 KB block tile), AHEAD steps before
  // their LDS write, register staged (AHEAD sets), from a 256 MB buffer walked per block
  f32x4 g[4][4];
  // 32 KB per step per block: block b, step s reads line group ((b * 7 + s) mod 8192) of the
  // buffer (power-of-two wrap: no 64-bit modulo in the address path)
  // V == 5: the real forward im2col pattern (C = 512 NHWC, 16x16 maps, K = 9 x 512): A rows =
  // 128 pixels of this block, 8 threads per 128-B chunk of a row, rows 2 KB apart, the chunk
  // walking the channels and the tap shifting the pixel; B = weights [128][4608] (18 KB rows)
  auto gload5 = [&](int s, f32x4* d) {
    const int tap = (s >> 4) % 9, cb = s & 15;
    const int shift = (tap / 3 - 1) * 16 + (tap % 3 - 1);
    const long long pix0 = (long long)blockIdx.x * 128 + 1024;  // away from the buffer start
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const long long row = pix0 + (t >> 3) + 64 * i + shift;
      d[i] = *reinterpret_cast<const f32x4*>(src + row * 512 + cb * 32 + (t & 7) * 4);
    }
    const float* wb = src + (60LL << 20);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      d[2 + i] = *reinterpret_cast<const f32x4*>(wb + (long long)((t >> 3) + 64 * i) * 4608 +
                                                  (s % 144) * 32 + (t & 7) * 4);
  };
  auto gload = [&](int s, f32x4* d) {
    if (V == 5) {
      gload5(s, d);
      return;
    }
    const float* p = src + (size_t)(((unsigned)blockIdx.x * 7u + (unsigned)s) & 8191u) * 8192u;
#pragma unroll
    for (int i = 0; i < 4; ++i) d[i] = *reinterpret_cast<const f32x4*>(p + (i * 512 + t) * 4);
  };
  if (V >= 4)
    for (int k = 0; k < AHEAD; ++k) gload(k, g[k]);
  for (int s0 = 0; s0 < steps; s0 += 4) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int s = s0 + u;
    const char* st = smem + (s & 1) * 32768;
    if (V >= 1) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        a[r][0] = *reinterpret_cast<const f32x4*>(st + ((off + r * 2048) & 32767));
        a[r][1] = *reinterpret_cast<const f32x4*>(st + ((off + r * 2048 + 1024) & 32767));
        b[r] = *reinterpret_cast<const f32x4*>(st + ((off + r * 2048 + 16384) & 32767));
      }
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[r][0][jj], b[r][jj], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[r][1][jj], b[r][jj], acc1, 0, 0, 0);
      }
    __builtin_amdgcn_s_setprio(0);
    if (V >= 4) {
      // write the tile loaded AHEAD steps ago, then reload that register set
      f32x4* cur = g[u % AHEAD];  // compile-time register set (the step loop is unrolled by 4)
      char* wst = smem + ((s + 1) & 1) * 32768;
#pragma unroll
      for (int i = 0; i < 4; ++i) *reinterpret_cast<f32x4*>(wst + ((t * 16 + i * 8192) & 32767)) = cur[i];
      gload(s + AHEAD, cur);
    } else if (V >= 3) {
      char* wst = smem + ((s + 1) & 1) * 32768;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *reinterpret_cast<f32x4*>(wst + ((t * 16 + i * 8192) & 32767)) = a[i][0] + b[i];
    }
    if (V >= 2) __syncthreads();
  }
  }
  float v = 0;
  for (int e = 0; e < 16; ++e) v += acc0[e] + acc1[e];
  out[blockIdx.x * 512 + t] = v;
}

template <int V, int AHEAD = 2, bool RND = false>
double run(float* out, int blocks, int steps, const float* src, long long n) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((k_loop<V, AHEAD, RND>), dim3(blocks), dim3(512), 0, 0, out, steps, src, n);
  hipEventRecord(a);
  const int reps = 10;
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((k_loop<V, AHEAD, RND>), dim3(blocks), dim3(512), 0, 0, out, steps, src, n);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  // per step per block: 8 waves x 32 MFMAs x (32 x 32 x 2 x 2) FLOP
  const double flop = (double)blocks * steps * 8 * 32 * 4096 * reps;
  return flop / (ms * 1e-3) / 1e12;
}

int main() {
  const int blocks = 256, steps = 2000;
  float *out, *src;
  const long long n = 64LL << 20;  // 256 MB (8192 groups of 32 KB)
  if (hipMalloc(&out, (size_t)blocks * 512 * 4) != hipSuccess) return 1;
  if (hipMalloc(&src, (size_t)n * 4) != hipSuccess) return 1;
  {
    float* h = (float*)malloc((size_t)n * 4);
    unsigned x = 12345;
    for (long long i = 0; i < n; ++i) {
      x ^= x << 13; x ^= x >> 17; x ^= x << 5;
      h[i] = (float)(x & 0xffff) * 3e-5f - 1.0f;
    }
    hipMemcpy(src, h, (size_t)n * 4, hipMemcpyHostToDevice);
    free(h);
  }
  printf("0 mfma only            %6.1f TF/s\n", run<0>(out, blocks, steps, src, n));
  printf("1 + lds frag reads     %6.1f TF/s\n", run<1>(out, blocks, steps, src, n));
  printf("2 + barrier per step   %6.1f TF/s\n", run<2>(out, blocks, steps, src, n));
  printf("3 + lds writes         %6.1f TF/s\n", run<3>(out, blocks, steps, src, n));
  printf("4 + global loads (2)   %6.1f TF/s\n", run<4, 2>(out, blocks, steps, src, n));
  printf("4 + global loads (4)   %6.1f TF/s\n", run<4, 4>(out, blocks, steps, src, n));
  printf("5 im2col pattern (2)   %6.1f TF/s\n", run<5, 2, true>(out, blocks, steps, src, n));
  printf("5 im2col pattern (4)   %6.1f TF/s\n", run<5, 4, true>(out, blocks, steps, src, n));
  printf("random data: 1         %6.1f TF/s\n", run<1, 2, true>(out, blocks, steps, src, n));
  printf("random data: 4 (2)     %6.1f TF/s\n", run<4, 2, true>(out, blocks, steps, src, n));
  hipFree(src);
  hipFree(out);
  return 0;
}
