// MFMA issue-rate microbenchmark (gfx950): one wave per SIMD (256 threads / WG, one WG per
// CU), 8 independent 16x16x32 bf16 accumulators per step as in cnn_bwd's dgrad loop;
// variants: VGPR accumulators, with per-step VALU address work, AGPR accumulators.
// hipcc --offload-arch=gfx950 -O3 tools/micro/mfma_rate.hip -o /tmp/mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int VARIANT>
__global__ __launch_bounds__(256) void k(float* out, unsigned long long* cyc, int steps) {
  const int lane = threadIdx.x & 63;
  bf16x8 a[4], w[2];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) a[i][j] = (__bf16)(0.001f * (lane + i + j));
  for (int j = 0; j < 8; ++j) { w[0][j] = (__bf16)0.5f; w[1][j] = (__bf16)0.25f; }
  f32x4 acc[4][2];
  for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = f32x4{0, 0, 0, 0};
  int x = lane;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  // unrolled x8: a rolled loop makes hipcc rotate the loop-carried accumulators through
  // accvgpr moves that serialise the MFMAs (measured 44.5 cyc/MFMA)
#pragma unroll 8
  for (int s = 0; s < steps; ++s) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      // inline asm on VGPR accumulators: the builtin in a rolled loop gets its loop-carried
      // accumulators rotated through accvgpr moves that serialise the MFMAs
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[kk][0]) : "v"(a[kk]), "v"(w[0]));
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[kk][1]) : "v"(a[kk]), "v"(w[1]));
    }
    if (VARIANT == 1) {   // ~12 VALU per step, independent of the MFMAs
#pragma unroll
      for (int v = 0; v < 6; ++v) { x = (x + 0x3c0) & 0x7ff0; x ^= 64; }
      asm volatile("" : "+v"(x));
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float sum = 0;
  for (int i = 0; i < 4; ++i) sum += acc[i][0][0] + acc[i][1][1];
  out[blockIdx.x * 256 + threadIdx.x] = sum + x;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float* out; unsigned long long* cyc;
  hipMalloc(&out, 256 * 256 * 4 * 4);
  hipMalloc(&cyc, 256 * 8 * 2);
  unsigned long long h[256];
  const int steps = 4096;
  for (int variant = 0; variant < 2; ++variant) {
    for (int wpb : {64, 128, 256, 512}) {
      for (int rep = 0; rep < 2; ++rep) {
        if (variant == 0) k<0><<<256, wpb>>>(out, cyc, steps); else k<1><<<256, wpb>>>(out, cyc, steps);
      }
      hipDeviceSynchronize();
      hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
      double m = 0; for (int i = 0; i < 256; ++i) m += h[i]; m /= 256;
      printf("variant %d  threads/WG %3d (waves/SIMD %.2f): %.1f cycles per MFMA per wave\n",
             variant, wpb, wpb / 256.0, m / (steps * 8.0));
    }
  }
  // calibrate s_memtime against wall time (events around one long launch)
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const int big = 1 << 18;
  k<0><<<256, 256>>>(out, cyc, big);
  hipEventRecord(e0);
  k<0><<<256, 256>>>(out, cyc, big);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0; hipEventElapsedTime(&ms, e0, e1);
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double m = 0; for (int i = 0; i < 256; ++i) m += h[i]; m /= 256;
  printf("calibration: %.0f memtime ticks in %.3f ms -> %.3f GHz; %.2f TFLOP/s bf16 (16x16x32, 1 wave/SIMD)\n",
         m, ms, m / (ms * 1e6), 256.0 * 4 * big * 8 * 16384.0 / (ms * 1e-3) / 1e12);
  return 0;
}
