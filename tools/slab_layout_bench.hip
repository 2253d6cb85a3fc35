// Micro-benchmark: cross-workgroup gradient-slab reduction, slab-major vs tile-major layout.
//
// The bf16 CNN step's conv backward leaves one fp32 slab (18816 floats) per workgroup and the
// optimizer sums them (csrc/kernels/optim.hip, slab segments): a workgroup owns 64 elements
// and reads a 256-B strip from every slab.  This program times that read pattern against a
// tile-major layout ([tile][slab][64]: one workgroup's reads are one contiguous run), each
// read right after a writer kernel that produces the slabs (as cnn_bwd does), and the
// loads in flight per thread (U) / slab groups per workgroup (G) of the reduction.
//
//   hipcc --offload-arch=gfx950 -O3 -o build/slab_layout_bench tools/slab_layout_bench.hip
//   ./build/slab_layout_bench [nslab] [iters]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

constexpr int SLAB = 18816;          // floats per conv slab (dW2 + db2 + dW1 + db1)
constexpr int NT = SLAB / 64;        // 64-element tiles

__device__ __forceinline__ long addr(bool tiled, int nslab, int w, int e) {
  return tiled ? ((long)(e / 64) * nslab + w) * 64 + (e % 64) : (long)w * SLAB + e;
}

__global__ void __launch_bounds__(256) writer(float* s, int nslab, bool tiled, float salt) {
  const int w = blockIdx.x;
  for (int e = threadIdx.x; e < SLAB; e += 256) s[addr(tiled, nslab, w, e)] = salt + w + 1e-3f * e;
}

template <int U, int G>   // U loads in flight per thread, G slab groups (16 lanes each)
__global__ void __launch_bounds__(16 * G) reader(const float* s, float* out, int nslab, bool tiled) {
  __shared__ float4 red[G][16];
  const int t = blockIdx.x, tid = threadIdx.x, c4 = tid & 15, rg = tid >> 4;
  const int e = t * 64 + 4 * c4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int j0 = rg; j0 < nslab; j0 += G * U) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = min(j0 + G * u, nslab - 1);
      v[u] = *reinterpret_cast<const float4*>(s + addr(tiled, nslab, j, e));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool on = j0 + G * u < nslab;
      acc.x += on ? v[u].x : 0.f;
      acc.y += on ? v[u].y : 0.f;
      acc.z += on ? v[u].z : 0.f;
      acc.w += on ? v[u].w : 0.f;
    }
  }
  red[rg][c4] = acc;
  __syncthreads();
  if (tid < 64) {
    const float* rf = reinterpret_cast<const float*>(&red[0][0]);
    float g = 0.f;
    for (int q = 0; q < G; ++q) g += rf[q * 64 + tid];
    out[t * 64 + tid] = g;
  }
}

// the optimizer's slab segment in full (SGD-momentum update of 64 parameters per workgroup,
// parameter / momentum loaded ahead of the reduction, reduced gradient and bf16 copy stored)
__global__ void __launch_bounds__(256) reader_sgd(const float* s, float* out, int nslab, bool tiled,
                                                  float* p, float* m, __bf16* shadow) {
  __shared__ float4 red[16][16];
  const int t = blockIdx.x, tid = threadIdx.x, c4 = tid & 15, rg = tid >> 4;
  const int e = t * 64 + 4 * c4, ep = t * 64 + tid;
  float p0 = 0.f, m0 = 0.f;
  if (tid < 64) { p0 = p[ep]; m0 = m[ep]; }
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int j0 = rg; j0 < nslab; j0 += 128) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      v[u] = *reinterpret_cast<const float4*>(s + addr(tiled, nslab, min(j0 + 16 * u, nslab - 1), e));
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool on = j0 + 16 * u < nslab;
      acc.x += on ? v[u].x : 0.f;
      acc.y += on ? v[u].y : 0.f;
      acc.z += on ? v[u].z : 0.f;
      acc.w += on ? v[u].w : 0.f;
    }
  }
  red[rg][c4] = acc;
  __syncthreads();
  if (tid < 64) {
    const float* rf = reinterpret_cast<const float*>(&red[0][0]);
    float g = 0.f;
    for (int q = 0; q < 16; ++q) g += rf[q * 64 + tid];
    out[ep] = g;
    const float mm = 0.5f * m0 + g;
    const float pp = p0 - 1e-9f * mm;
    m[ep] = mm;
    p[ep] = pp;
    shadow[ep] = (__bf16)pp;
  }
}

int main(int argc, char** argv) {
  const int nslab = argc > 1 ? std::atoi(argv[1]) : 256;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 200;
  float *s, *out;
  CHECK(hipMalloc(&s, (size_t)nslab * SLAB * sizeof(float)));
  CHECK(hipMalloc(&out, (size_t)SLAB * sizeof(float)));
  hipEvent_t ev[3];
  for (auto& e : ev) CHECK(hipEventCreate(&e));
  float* host = (float*)std::malloc(SLAB * sizeof(float));
  struct Variant { const char* name; bool tiled; void (*k)(const float*, float*, int, bool); int threads; };
  const Variant vars[] = {
      {"slab-major U8 G16", false, reader<8, 16>, 256}, {"tile-major U8 G16", true, reader<8, 16>, 256},
      {"slab-major U16 G16", false, reader<16, 16>, 256}, {"slab-major U8 G32", false, reader<8, 32>, 512},
      {"slab-major U4 G64", false, reader<4, 64>, 1024}, {"tile-major U16 G16", true, reader<16, 16>, 256}};
  for (const Variant& vr : vars) {
    double tw = 0, tr = 0;
    for (int i = 0; i < iters + 10; ++i) {
      const float salt = (float)(i & 7);
      CHECK(hipEventRecord(ev[0]));
      writer<<<nslab, 256>>>(s, nslab, vr.tiled, salt);
      CHECK(hipEventRecord(ev[1]));
      vr.k<<<NT, vr.threads>>>(s, out, nslab, vr.tiled);
      CHECK(hipEventRecord(ev[2]));
      CHECK(hipEventSynchronize(ev[2]));
      float a, b;
      CHECK(hipEventElapsedTime(&a, ev[0], ev[1]));
      CHECK(hipEventElapsedTime(&b, ev[1], ev[2]));
      if (i >= 10) { tw += a; tr += b; }
    }
    CHECK(hipMemcpy(host, out, SLAB * sizeof(float), hipMemcpyDeviceToHost));
    // sum over w of (salt + w + 1e-3 e), salt of the last iteration
    const float salt = (float)((iters + 9) & 7);
    double maxerr = 0;
    for (int e = 0; e < SLAB; ++e) {
      const double want = (double)nslab * (salt + 1e-3 * e) + 0.5 * nslab * (nslab - 1);
      const double d = std::abs(host[e] - want) / want;
      if (d > maxerr) maxerr = d;
    }
    const double mb = (double)nslab * SLAB * 4 / 1e6;
    std::printf("{\"variant\": \"%s\", \"nslab\": %d, \"writer_us\": %.2f, \"reader_us\": %.2f, "
                "\"reader_GBps\": %.0f, \"max_rel_err\": %.2e}\n",
                vr.name, nslab, 1e3 * tw / iters, 1e3 * tr / iters, mb / (tr / iters), maxerr);
  }
  {
    float *p, *m;
    __bf16* sh;
    CHECK(hipMalloc(&p, SLAB * sizeof(float)));
    CHECK(hipMalloc(&m, SLAB * sizeof(float)));
    CHECK(hipMalloc(&sh, SLAB * sizeof(__bf16)));
    CHECK(hipMemset(p, 0, SLAB * sizeof(float)));
    CHECK(hipMemset(m, 0, SLAB * sizeof(float)));
    double tr = 0;
    for (int i = 0; i < iters + 10; ++i) {
      writer<<<nslab, 256>>>(s, nslab, false, (float)(i & 7));
      CHECK(hipEventRecord(ev[1]));
      reader_sgd<<<NT, 256>>>(s, out, nslab, false, p, m, sh);
      CHECK(hipEventRecord(ev[2]));
      CHECK(hipEventSynchronize(ev[2]));
      float b;
      CHECK(hipEventElapsedTime(&b, ev[1], ev[2]));
      if (i >= 10) tr += b;
    }
    std::printf("{\"variant\": \"slab-major sgd update\", \"nslab\": %d, \"reader_us\": %.2f}\n",
                nslab, 1e3 * tr / iters);
    CHECK(hipFree(p));
    CHECK(hipFree(m));
    CHECK(hipFree(sh));
  }
  std::free(host);
  CHECK(hipFree(s));
  CHECK(hipFree(out));
  return 0;
}
