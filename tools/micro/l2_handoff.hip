// Does a producer's data stay in its XCD's L2 across a kernel boundary?  Kernel W writes one
// 16 KB region per workgroup (plain stores); the next kernel R reads region (b + shift) % 256
// in workgroup b and sums it.  Blocks b and b + 8 share an XCD (round-robin dispatch), so
// shift 0 / 8 read a region written on the reader's own XCD, shift 1 / 3 one written on
// another XCD.  If the reader's time depends on the shift, L2 lines survive the boundary and
// producer->consumer XCD affinity between the step's kernels is worth having.  The sums are
// checked against the values of the last W (a stale line would show up as a mismatch).
// hipcc --offload-arch=gfx950 -O3 tools/micro/l2_handoff.hip -o tools/micro/l2_handoff
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); std::exit(1); } } while (0)

constexpr int NB = 256, THREADS = 256, REGION_F4 = 1024;   // 16 KB per workgroup

__global__ __launch_bounds__(THREADS) void writer(float4* buf, const int* iter) {
  const float v = (float)(*iter);
  float4* r = buf + (size_t)blockIdx.x * REGION_F4;
  for (int i = threadIdx.x; i < REGION_F4; i += THREADS) r[i] = make_float4(v, v + 1.f, v, blockIdx.x);
}

__global__ __launch_bounds__(THREADS) void reader(const float4* buf, int shift, float* out, int* iter) {
  const int src = (blockIdx.x + shift) % NB;
  const float4* r = buf + (size_t)src * REGION_F4;
  float4 v[REGION_F4 / THREADS];
#pragma unroll
  for (int j = 0; j < REGION_F4 / THREADS; ++j) v[j] = r[threadIdx.x + THREADS * j];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < REGION_F4 / THREADS; ++j) s += v[j].x + v[j].y + v[j].z + v[j].w;
  __shared__ float red[THREADS];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = THREADS / 2; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = red[0];
  if (blockIdx.x == 0 && threadIdx.x == 0) *iter += 1;   // next writer's value
}

int main() {
  float4* buf;
  float* out;
  int* iter;
  CK(hipMalloc(&buf, sizeof(float4) * NB * REGION_F4));
  CK(hipMalloc(&out, sizeof(float) * NB));
  CK(hipMalloc(&iter, sizeof(int)));
  CK(hipMemset(iter, 0, sizeof(int)));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const int iters = 100;
  for (int with_writer = 1; with_writer >= 0; --with_writer) {
    for (int shift : {0, 8, 1, 3, 0, 1}) {
      hipGraph_t g;
      hipGraphExec_t ge;
      writer<<<NB, THREADS, 0, s>>>(buf, iter);
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      for (int i = 0; i < iters; ++i) {
        if (with_writer) writer<<<NB, THREADS, 0, s>>>(buf, iter);
        reader<<<NB, THREADS, 0, s>>>(buf, shift, out, iter);
      }
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      hipEvent_t a, b;
      CK(hipEventCreate(&a));
      CK(hipEventCreate(&b));
      CK(hipEventRecord(a, s));
      for (int r = 0; r < 5; ++r) CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      // check the last reader's sums against the last writer's value
      int it = 0;
      std::vector<float> h(NB);
      CK(hipMemcpy(&it, iter, sizeof(int), hipMemcpyDeviceToHost));
      CK(hipMemcpy(h.data(), out, sizeof(float) * NB, hipMemcpyDeviceToHost));
      int bad = 0;
      if (with_writer) {
        const float v = (float)(it - 1);
        for (int b2 = 0; b2 < NB; ++b2) {
          const int src = (b2 + shift) % NB;
          const float want = (float)REGION_F4 * (3.f * v + 1.f + (float)src);
          if (h[b2] != want) ++bad;
        }
      }
      std::printf("%s shift %d: %.3f us per %s (stale sums: %d)\n",
                  with_writer ? "writer+reader" : "reader only  ", shift,
                  ms * 1e3f / (5 * iters), with_writer ? "W+R pair" : "R", bad);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
      CK(hipEventDestroy(a));
      CK(hipEventDestroy(b));
    }
  }
  CK(hipStreamDestroy(s));
  return 0;
}
