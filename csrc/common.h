// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels.
// Wave64 everywhere: lane = threadIdx.x & 63, block sizes are multiples of 64.
#pragma once
#include <type_traits>
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define PDM_WAVE 64

// torchvision ToTensor() + Normalize((0.1307,), (0.3081,)) in fp32, same op order
// (x/255, then (x-mean)/std; HIP's default fp32 division is correctly rounded).
__device__ __forceinline__ float pdm_normalize(uint32_t v) {
  return ((float)v / 255.0f - 0.1307f) / 0.3081f;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Whole-wave sum on the DPP network, no LDS traffic: quad swaps and row rotates leave every
// lane of a 16-lane row with the row's sum, then the four row sums are read as scalars.
// The result is identical in every lane (a different addition order than wave_sum).
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dpp_mov<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_mov<0x124>(v);   // row_ror:4
  v += dpp_mov<0x128>(v);   // row_ror:8
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return (r0 + r1) + (r2 + r3);
}

// v + v[lane ^ 8], v[lane ^ 16], v[lane ^ 32] without LDS traffic: row_ror:8 is the xor-8
// partner inside a 16-lane row; gfx950's permlane16/32 swaps exchange odd and even rows /
// the two wave halves (both results summed in the same order as the shuffle butterfly).
// Full EXEC required.
__device__ __forceinline__ float sum_xor8(float v) { return v + dpp_mov<0x128>(v); }
__device__ __forceinline__ float sum_xor16(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
  return __int_as_float(a[0]) + __int_as_float(a[1]);
}
__device__ __forceinline__ float sum_xor32(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return __int_as_float(a[0]) + __int_as_float(a[1]);
}

// Sum within aligned groups of `width` lanes (width a power of two <= 64).
template <int WIDTH>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = WIDTH / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ bf16 to_bf16(float f) { return (bf16)f; }
__device__ __forceinline__ float from_bf16(bf16 h) { return (float)h; }

// Hand-off stores: bytes a kernel writes for the NEXT launch (gradient slabs, activations,
// partials, the fused fc1 update).  Plain stores leave them dirty in the writer's XCD L2
// until the kernel-end release writes them back, which the dependent launch waits for at the
// boundary (MI355X_MICROARCH.md "boundary": + dirty bytes / 6 TB/s).  Agent-scope
// write-through stores (global_store ... sc1) send them to memory as they are stored,
// beside the kernel's other work; the readers are other workgroups on other XCDs, so no
// L2 locality is given up.  The site groups (G):
//   1 conv gradient slabs (cnn_bwd[_band] -> optimizer / conv_reduce): write-through
//   2 fc1_bwd outputs (dpool, the fc1 gradient, the fused update's weights and copies)
//   4 cnn_fwd[_band] outputs (pool, mask, image, a1 / x hand-offs)
//   8 fc1_fwd split-K partials and cnn_head outputs (dh, dh^T, head slabs)
// Only group 1 is stored write-through: the others were measured neutral or slower that way
// (round 5, profiles/r5/wt/): the next launch reads them on the writer's XCD often enough
// that the L2 copy helps.  (The build-time group mask that measured it was removed in round 6.)
constexpr int PDM_WT_GROUPS = 1;
template <int G, class T>
__device__ __forceinline__ void st_ho(T* p, T v) {
  if constexpr ((PDM_WT_GROUPS & G) == 0) {
    *p = v;
  } else if constexpr (sizeof(T) == 16) {
    unsigned long long w[2];
    __builtin_memcpy(w, &v, 16);
    unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
    __hip_atomic_store(q, w[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 1, w[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    static_assert(sizeof(T) == 1 || sizeof(T) == 2 || sizeof(T) == 4 || sizeof(T) == 8,
                  "hand-off store of 1, 2, 4, 8 or 16 bytes");
    using U = typename std::conditional<sizeof(T) == 1, unsigned char,
              typename std::conditional<sizeof(T) == 2, unsigned short,
              typename std::conditional<sizeof(T) == 4, unsigned int,
                                        unsigned long long>::type>::type>::type;
    U u;
    __builtin_memcpy(&u, &v, sizeof(T));
    __hip_atomic_store(reinterpret_cast<U*>(p), u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Stores / loads of per-workgroup gradient slabs (read once, by the next launch).
// Non-temporal (streaming) forms of both measured slower (round 4, docs/kernels.md).
__device__ __forceinline__ void pdm_slab_store(float* p, float v) { st_ho<1>(p, v); }
__device__ __forceinline__ float4 pdm_slab_load4(const float4* p) { return *p; }
// 16 B of a slab, floats [e, e + 4) of the (workgroup-uniform) slab `base`, e % 4 == 0, in
// one write-through store (sc1, like st_ho<1>): a quarter of the store instructions of four
// pdm_slab_store calls, which a slab tail can be issue-bound on.  A buffer store, not inline
// asm: the compiler must see the store to keep its data registers from being overwritten
// while it is in flight (an asm global_store_dwordx4 measured non-deterministic slabs).
__device__ __forceinline__ void pdm_slab_store4(float* base, int e, f32x4 v) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, e * 4, 0, 16 /* sc1 */);
}

// Bookkeeping done by exactly one thread of a kernel that no other kernel of the
// same step reads concurrently (see runtime/gpu_step.py: the "middle" kernel
// advances the data-step and optimizer-step counters).
#include "pdm_check.h"

// One 256-thread workgroup: metrics[0] += sum_j slab[j][col], metrics[1] += sum_j
// slab[j][col + 1] over the nslab per-workgroup slabs (row stride `stride` floats): the
// fp32 loss / correct partials summed in fp64 in a FIXED order (thread t takes slabs t,
// t + 128, ... of one column, then a fixed tree), so the train metrics are bitwise
// reproducible (fp64 atomics from many workgroups are not: their order varies).
__device__ __forceinline__ void pdm_slab_metrics(const float* __restrict__ slab, int nslab, int col,
                                                 int64_t stride, double* __restrict__ metrics) {
  __shared__ double red[256];
  const int t = threadIdx.x, half = t >> 7, lt = t & 127;
  double s = 0.0;
  for (int j = lt; j < nslab; j += 128) s += (double)slab[(int64_t)j * stride + col + half];
  red[t] = s;
  __syncthreads();
#pragma unroll
  for (int w = 64; w > 0; w >>= 1) {
    if (lt < w) red[t] += red[t + w];
    __syncthreads();
  }
  if (lt == 0) metrics[half] += red[t];
}

__device__ __forceinline__ void pdm_bump_counters(int64_t* c0, int64_t* c1,
                                                  unsigned* c2 = nullptr) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (c0) *c0 += 1;
    if (c1) *c1 += 1;
    if (c2) *c2 += 1;   // xgmi streamed mode: step generation (csrc/xgmi.h)
  }
}
