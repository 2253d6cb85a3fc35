// Kernel-boundary cost inside a hipGraph on gfx950: per-launch time of back-to-back
// kernels shaped like the training step's (256 workgroups; 512 threads + 159 KB LDS like
// cnn_bwd, or 256 threads and no LDS like fc1_fwd) that spin a fixed number of shader
// cycles and optionally write a per-workgroup slab (like cnn_bwd's 74 KB gradient slab),
// minus the spin itself.  Answers: how much of a 20 us kernel is the boundary?
// hipcc --offload-arch=gfx950 -O3 tools/micro/launch_overhead.hip -o tools/micro/launch_overhead
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); std::exit(1); } } while (0)

template <int LDS_BYTES>
__global__ void spin_kernel(float* slab, int slab_floats, long long spin, int nt) {
  __shared__ float lds[LDS_BYTES / 4 > 0 ? LDS_BYTES / 4 : 1];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  // every wave spins (bounded: spin is a cycle count, the loop always ends)
  while ((long long)(__builtin_amdgcn_s_memtime() - t0) < spin) __builtin_amdgcn_s_sleep(1);
  if (LDS_BYTES > 0) {
    lds[threadIdx.x] = (float)threadIdx.x;
    __syncthreads();
  }
  if (slab_floats > 0) {
    float* out = slab + (long long)blockIdx.x * slab_floats;
    const float v = LDS_BYTES > 0 ? lds[(threadIdx.x + 1) % blockDim.x] : 1.f;
    for (int i = threadIdx.x; i < slab_floats; i += blockDim.x) {
      if (nt) __builtin_nontemporal_store(v, out + i);
      else out[i] = v;
    }
  }
}

template <int LDS>
static float per_launch_us(int threads, float* slab, int slab_floats, long long spin, int nt) {
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const int iters = 50;
  for (int i = 0; i < 3; ++i) spin_kernel<LDS><<<256, threads, 0, s>>>(slab, slab_floats, spin, nt);
  CK(hipStreamSynchronize(s));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int i = 0; i < iters; ++i) spin_kernel<LDS><<<256, threads, 0, s>>>(slab, slab_floats, spin, nt);
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
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipStreamDestroy(s));
  return ms * 1e3f / (5 * iters);
}

int main() {
  float* slab;
  const int slab_floats = 18816;   // cnn_bwd's per-workgroup slab (75 KB)
  CK(hipMalloc(&slab, sizeof(float) * 256 * slab_floats));
  const double ghz = 2.38;         // s_memtime rate (tools/micro/mfma_rate calibration)
  for (long long spin_us : {0LL, 5LL, 15LL}) {
    const long long cyc = (long long)(spin_us * 1e3 * ghz);
    std::printf("spin %2lld us | 256x256 thr, no LDS: %6.2f us | 256x512 thr, 159 KB LDS: %6.2f us"
                " | + 75 KB slab: %6.2f us | + slab nt: %6.2f us\n",
                spin_us, per_launch_us<0>(256, slab, 0, cyc, 0),
                per_launch_us<162688>(512, slab, 0, cyc, 0),
                per_launch_us<162688>(512, slab, slab_floats, cyc, 0),
                per_launch_us<162688>(512, slab, slab_floats, cyc, 1));
  }
  CK(hipFree(slab));
  return 0;
}
