// Shapes, LDS image layouts and small helpers shared by the CNN kernels.
#pragma once
#include "../common.h"
#include "../kernels.h"

#include <type_traits>
#include <utility>

// Diagnostic build only (PDM_STAMPS=1 python -m pytorch_distributed_mnist_amd.build):
// thread 0 of blocks 0..255 records s_memtime at phase boundaries; never in a timed build.
#ifdef PDM_STAMPS
static __device__ unsigned long long pdm_stamps[256 * 16];
#define PDM_STAMP(slot)                                                              \
  do {                                                                               \
    if (threadIdx.x == 0 && blockIdx.x < 256)                                        \
      pdm_stamps[blockIdx.x * 16 + (slot)] = __builtin_amdgcn_s_memtime();           \
  } while (0)
#define PDM_CLOCK() __builtin_amdgcn_s_memtime()
#define PDM_STAMP_VAL(slot, val)                                                     \
  do {                                                                               \
    if (blockIdx.x < 256) pdm_stamps[blockIdx.x * 16 + (slot)] = (val);              \
  } while (0)
#else
#define PDM_STAMP(slot) \
  do {                  \
  } while (0)
#define PDM_CLOCK() 0ull
#define PDM_STAMP_VAL(slot, val) \
  do {                           \
  } while (0)
#endif

namespace cnn {

// compile-time loop: f(std::integral_constant<int, i>) for i = 0 .. N-1, fully expanded
// (hipcc leaves long `#pragma unroll` loops rolled and keeps the arrays they index in scratch)
template <class F, int... Is>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

constexpr int IMG = 28;               // input 28x28
constexpr int C1 = 32, H1 = 26, P1 = H1 * H1;   // conv1 out 26x26x32
constexpr int C2 = 64, H2 = 24, P2 = H2 * H2;   // conv2 out 24x24x64
constexpr int HP = 12, PP = HP * HP;            // pooled 12x12x64
constexpr int FEAT = CNN_FEAT;        // 9216
constexpr int HID = CNN_HID;          // 128
constexpr int NCLS = CNN_NCLS;        // 10
constexpr int HEAD_ROWS = CNN_HEAD_ROWS;
constexpr int HEAD_SLAB = CNN_HEAD_SLAB;
constexpr int CONV_SLAB = CNN_CONV_SLAB;

// LDS image of a1 (26x26 pixels x 32 bf16 = 64 B/pixel).  The 16-B chunk index is
// XOR-swizzled with (col & 3): with the conv2 A-fragment pattern (4 pooled pixels x
// 2x2 windows, ds_read_b128) every 16-lane group then hits 16 distinct 16-B slots
// (conflict-free; plain layout is 2-way), and the wgrad transposed reads stay <= 2-way.
__device__ __forceinline__ int a1_off(int row, int col, int byte) {
  return (row * H1 + col) * 64 + ((((byte >> 4) ^ (col & 3))) << 4) + (byte & 15);
}

// conv1 epilogue (D[co][pixel] on mfma_f32_16x16x16_bf16): lane (g = lane >> 4, i16) holds
// channels 4g .. 4g + 3 of pixel i16 for both 16-channel halves (o0: co < 16, o1: co >= 16).
// Two 8-B stores per lane at a 64-B pixel stride were 4-way bank conflicts (ds_write_b64:
// 16 contiguous lanes per LDS cycle, one chunk slot per pixel residue mod 4).  Lane pairs
// g, g ^ 1 swap halves on gfx950's v_permlane16_swap (odd rows of the first operand <-> even
// rows of the second), so every lane holds 8 consecutive channels and issues ONE 16-B store:
// even g: channels 4g .. 4g + 7, odd g: 16 + 4(g - 1) .. + 7 -- the 16-B chunk
// conv1_pair_chunk(g) of the pixel (ds_write_b128: 8 contiguous lanes per cycle, 2-way).
// Full EXEC required.
__device__ __forceinline__ uint4 conv1_pair(bf16x4 o0, bf16x4 o1) {
  const uint2 u0 = __builtin_bit_cast(uint2, o0), u1 = __builtin_bit_cast(uint2, o1);
  const auto r0 = __builtin_amdgcn_permlane16_swap(u0.x, u1.x, false, false);
  const auto r1 = __builtin_amdgcn_permlane16_swap(u0.y, u1.y, false, false);
  return make_uint4(r0[0], r1[0], r0[1], r1[1]);
}
__device__ __forceinline__ int conv1_pair_chunk(int g) { return (g >> 1) | ((g & 1) << 1); }

// LDS image of dz2 = dL/d(conv2 pre-activation) (24x24 x 64 bf16 = 128 B/pixel).
// Chunk swizzle (2*row + col) & 7: conflict-free ds_read_b128 for the dgrad A rows,
// 2-way for the wgrad ds_read_b64_tr_b16 column reads (searched, see docs/kernels.md).
__device__ __forceinline__ int dz_off(int row, int col, int byte) {
  return (row * H2 + col) * 128 + ((((byte >> 4) ^ ((2 * row + col) & 7))) << 4) + (byte & 15);
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// ds_read_b64_tr_b16: lane 4q+p of each 16-lane group gives the address of row q,
// columns 4p..4p+3; lane i receives column i of the 4 rows.
// ReLU / max-pool as single integer VALU ops.  hipcc lowers fmaxf (and x > 0 ? x : 0) on a
// value it cannot prove canonical -- every MFMA result -- to two v_max_f32 (a NaN-quieting
// self-max first), and these kernels are VALU-bound where they apply them (64-wide waves
// take 4 cycles per VALU op on CDNA).  On the bit patterns, a signed integer max against 0
// IS relu (negative floats are negative integers, -0.0 becomes +0.0), and among positive
// floats integer order is float order, so the max-pool of relu(x) is relu of the integer
// max.  (Inline-asm v_max_f32 would do it too, but hipcc inserts no MFMA-result wait states
// in front of inline asm.)
__device__ __forceinline__ int fbits(float x) { return __builtin_bit_cast(int, x); }
__device__ __forceinline__ float relu1(float x) {
  return __builtin_bit_cast(float, max(fbits(x), 0));
}

// LDS byte address of a __shared__ pointer (the M0 base of an LDS-DMA load)
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
// Asynchronous 16-B global -> LDS copy (global_load_lds_dwordx4, no VGPR destination): lane l
// of the wave writes LDS bytes [lds + 16 l, +16) (wave-uniform lds) from its own gsrc.  Inline
// asm, so hipcc neither waits for it before every later LDS access (it does for the builtin)
// nor counts it: the caller waits with s_waitcnt vmcnt(0) before a barrier that publishes
// the data, and issues it after its own loads (hipcc's counted waits on those then stay
// correct: they can only over-wait).
__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}

__device__ __forceinline__ s16x4 lds_tr16(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
}

__device__ __forceinline__ bf16x8 cat_tr(s16x4 lo, s16x4 hi) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

template <int N>
__device__ __forceinline__ float row_xent(const float (&lg)[N], int y, float (&p)[N], int& correct) {
  float m = lg[0];
  int am = 0;
#pragma unroll
  for (int n = 1; n < N; ++n)
    if (lg[n] > m) { m = lg[n]; am = n; }
  float s = 0.f;
#pragma unroll
  for (int n = 0; n < N; ++n) { p[n] = expf(lg[n] - m); s += p[n]; }
  const float lse = m + logf(s);
  const float inv = 1.f / s;
#pragma unroll
  for (int n = 0; n < N; ++n) p[n] *= inv;
  correct = (am == y);
  float ly = lg[0];
#pragma unroll
  for (int n = 1; n < N; ++n) ly = (n == y) ? lg[n] : ly;
  return lse - ly;
}

}  // namespace cnn
