// fp32 CNN step on gfx950: the reference's precision (multi_proc_single_gpu.py trains in fp32,
// S:185-191).  fp32 activations, gradients and master weights throughout; the chain and fusions
// of the bf16 kernels.  Two sets of kernels:
//
// Default (`--dtype fp32`): conv2 and fc1 products as SPLIT-BF16 on the bf16 matrix cores,
// v_mfma_f32_16x16x32_bf16 with fp32 accumulation.  Every fp32 operand is carried as
// hi = bf16(x), lo = bf16(x - hi), and a product is hi.hi + hi.lo + lo.hi (4.5e-6 relative
// error per conv output against fp64; TF32 gives 2.9e-4; tests/test_split_bf16.py):
//
//   f32x3_fwd      one image / workgroup: normalise -> conv1 + ReLU on the fp32 MFMA
//                  (16x16x4, exact fp32 products) over the virtual 28-wide pixel grid -> a1
//                  hi / lo planes in LDS -> conv2 (split-bf16, W2 hi / lo planes written by the
//                  optimizer and staged once through LDS) with bias + ReLU + 2x2 max-pool in the
//                  epilogue; training hands a1 and the split W2^T planes to the backward
//   f32x3_fc1_fwd  split-K GEMM pool . W1^T on split operands -> fp32 partials
//   f32x3_fc1_bwd  dW1 tiles (K = batch) | dX tiles (K = 128) on split operands | head-slab
//                  reduction
//   f32x3_conv_bwd (image, row band) units, one round of <= 256 workgroups, one slab each:
//                  dz2 scatter, conv2 dgrad fused with relu'(a1) and the conv1 weight/bias
//                  gradient, conv2 wgrad into persistent accumulators
//
// Exact (`PDM_F32_CONV=exact`): every product on the fp32 MFMA, v_mfma_f32_16x16x4_f32:
//
//   f32_fwd      one image / workgroup: normalise -> conv1 + ReLU (VALU, exact fp32) into an
//                LDS a1 image -> conv2 implicit GEMM (M = 576 pixels ordered (pooled pixel,
//                window position), N = 64, K = 288) with bias + ReLU + 2x2 max-pool fused in
//                the epilogue -> pooled activations + pool mask; training also writes a1 and
//                the normalised x for the backward
//   f32_fc1_fwd  split-K GEMM pool . W1^T -> fp32 partials
//   f32_fc1_bwd  dW1 tiles (K = batch) | dX tiles (K = 128) | head-slab reduction
//   f32_conv_bwd image row band / workgroup: dz2 = maxpool^-1(dpool) -> conv2 dgrad fused with
//                relu'(a1) and the conv1 weight/bias gradient, conv2 wgrad -> one fp32 slab per
//                workgroup
//
// Both sets share the bf16 program's cnn_head (writing dh in fp32) and the optimizer with the
// conv slab reduction fused in at world size 1 (the bf16 kernels' slab layout).
//
// MFMA 16x16x4 f32 operand layout, lane l = 16 g + i: A[m = i][k = g], B[k = g][n = i],
// D[m = 4 g + r][n = i] for r = 0..3.
#include "cnn_common.h"

namespace {

using namespace cnn;

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------------ f32_fwd
constexpr int FT = 512;
constexpr int A1S = 33;                           // a1 pixel stride in floats (bank spread)
constexpr int FX_XS = 0;                          // fp32 x [784]
constexpr int FX_WS = 3136;                       // fp32 w1 [288] | b1 [32] | b2 [64]
constexpr int FX_A1 = FX_WS + 1536;               // fp32 a1 [676][33]
constexpr int FX_W2 = FX_A1 + P1 * A1S * 4;       // fp32 W2 half [288 k][32 co], swizzled
constexpr int FX_TOTAL = FX_W2 + 288 * 32 * 4;
static_assert(FX_TOTAL <= 163840 && FX_A1 % 16 == 0 && FX_W2 % 16 == 0, "f32_fwd LDS");

// W2 half: element (k, c) at k * 32 + (c ^ ((k & 2) << 3)) -- the B reads of a k-step (4
// consecutive k, 16 consecutive c) hit 64 distinct banks
__device__ __forceinline__ int w2h_off(int k, int c) { return k * 32 + (c ^ ((k & 2) << 3)); }

template <bool TRAIN>
__global__ __launch_bounds__(FT, 1) void f32_fwd_kernel(
    const uint8_t* __restrict__ images, const int32_t* __restrict__ labels, int64_t nrow,
    const int64_t* __restrict__ ctr, const StepRows sr, const float* __restrict__ w1,
    const float* __restrict__ b1, const float* __restrict__ w2, const float* __restrict__ b2,
    float* __restrict__ pool, uint8_t* __restrict__ pmask, float* __restrict__ a1g,
    float* __restrict__ xng, int32_t* __restrict__ ylab) {
  __shared__ __attribute__((aligned(16))) char smem[FX_TOTAL];
  float* xs = reinterpret_cast<float*>(smem + FX_XS);
  float* ws = reinterpret_cast<float*>(smem + FX_WS);
  float* a1 = reinterpret_cast<float*>(smem + FX_A1);
  float* w2h = reinterpret_cast<float*>(smem + FX_W2);
  const int img = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15;
  // 0. small weights -> LDS, the image (epoch-buffer row ctr * bfull + img, or row img)
  const int wt = tid - 256;
  if (wt >= 0 && wt < 96) {
    const float4 q = wt < 72 ? reinterpret_cast<const float4*>(w1)[wt]
                     : wt < 80 ? reinterpret_cast<const float4*>(b1)[wt - 72]
                               : reinterpret_cast<const float4*>(b2)[wt - 80];
    reinterpret_cast<float4*>(ws)[wt] = q;
  }
  const int64_t row = min(ctr ? step_row(sr, nrow, *ctr, img) : (int64_t)img, nrow - 1);
  if (tid < 196) {
    const uint32_t v = reinterpret_cast<const uint32_t*>(images + row * 784)[tid];
    const float4 x = make_float4(pdm_normalize(v & 0xff), pdm_normalize((v >> 8) & 0xff),
                                 pdm_normalize((v >> 16) & 0xff), pdm_normalize(v >> 24));
    reinterpret_cast<float4*>(xs)[tid] = x;
    if (TRAIN) reinterpret_cast<float4*>(xng + (int64_t)img * 784)[tid] = x;
  }
  if (tid == 64) ylab[img] = labels[row];
  __syncthreads();
  // 1. conv1 + bias + ReLU: thread = pixel, all 32 channels (weights are LDS broadcasts)
  for (int p = tid; p < P1; p += FT) {
    const int y = p / H1, x = p - y * H1;
    float xv[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) xv[t] = xs[(y + t / 3) * IMG + x + t % 3];
#pragma unroll 2
    for (int c4 = 0; c4 < C1 / 4; ++c4) {
      float o[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int co = 4 * c4 + u;
        float acc = ws[288 + co];
#pragma unroll
        for (int t = 0; t < 9; ++t) acc = fmaf(ws[co * 9 + t], xv[t], acc);
        o[u] = fmaxf(acc, 0.f);
        a1[p * A1S + co] = o[u];
      }
      if (TRAIN)
        reinterpret_cast<float4*>(a1g + ((int64_t)img * P1 + p) * C1)[c4] = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
  // 2. conv2 + bias + ReLU + max-pool, co in two halves (W2 half staged in LDS).  Tile tt =
  // (pooled row py, pooled columns px0 .. px0 + 3): row i16 = 4 q + s is pooled pixel px0 + q,
  // window position s = 2 dy + dx, so a lane's 4 accumulators (rows 4 g + r) are one window.
  const int q = i16 >> 2, s = i16 & 3;
  for (int nh = 0; nh < 2; ++nh) {
    __syncthreads();   // a1 complete (nh = 0) / the previous half's B reads are done
    for (int e = tid; e < 32 * 288; e += FT) {
      const int c = e / 288, k = e - c * 288;
      w2h[w2h_off(k, c)] = w2[(nh * 32 + c) * 288 + k];
    }
    __syncthreads();
    float bias[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) bias[nt] = ws[320 + nh * 32 + nt * 16 + i16];
    // tiles {wave + 8 k} in pairs: four independent accumulator chains, every operand read of
    // a tap (8 A values per tile, 16 B values shared by both tiles) issued before its MFMAs
    for (int tt0 = wave; tt0 < 36; tt0 += 16) {
      const bool two = tt0 + 8 < 36;
      int pb[2];
      f32x4 acc[2][2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int tt = min(tt0 + 8 * u, 35);
        const int py = tt / 3, px0 = 4 * (tt - py * 3);
        pb[u] = (2 * py + (s >> 1)) * H1 + 2 * (px0 + q) + (s & 1);   // a1 pixel, tap 0
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[u][nt] = f32x4{bias[nt], bias[nt], bias[nt], bias[nt]};
      }
#pragma unroll 1
      for (int tap = 0; tap < 9; ++tap) {
        const int toff = (tap / 3) * H1 + tap % 3;
        float av[2][8], bv[2][8];
#pragma unroll
        for (int c8 = 0; c8 < 8; ++c8) {
          const int k = tap * 32 + c8 * 4 + g;
#pragma unroll
          for (int u = 0; u < 2; ++u) av[u][c8] = a1[(pb[u] + toff) * A1S + g + c8 * 4];
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) bv[nt][c8] = w2h[w2h_off(k, nt * 16 + i16)];
        }
#pragma unroll
        for (int c8 = 0; c8 < 8; ++c8)
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) acc[u][nt] = mfma4(av[u][c8], bv[nt][c8], acc[u][nt]);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (u == 1 && !two) break;
        const int tt = tt0 + 8 * u;
        const int py = tt / 3, px0 = 4 * (tt - py * 3);
        const int pp = py * HP + px0 + g;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const int co = nh * 32 + nt * 16 + i16;
          float m = acc[u][nt][0];
          uint32_t oh = 1u;
#pragma unroll
          for (int r = 1; r < 4; ++r) {
            const bool gt = acc[u][nt][r] > m;   // first position holding the max
            m = gt ? acc[u][nt][r] : m;
            oh = gt ? (1u << r) : oh;
          }
          const bool pos = m > 0.f;
          pool[(int64_t)img * FEAT + pp * C2 + co] = pos ? m : 0.f;
          if (TRAIN) pmask[(int64_t)img * FEAT + pp * C2 + co] = (uint8_t)(pos ? 0x80u | oh : 0u);
        }
      }
    }
  }
}

// ------------------------------------------------------------------ f32 conv2 on the bf16 MFMA
// Split-bf16 ("bf16x3") products: an fp32 operand x is carried as hi = bf16(x) and
// lo = bf16(x - hi) (both round-to-nearest-even), |x - hi - lo| <= 2^-16 |x| (a normal x
// whose hi / lo stay normal); a product x.y is taken as hi.hi + hi.lo + lo.hi on
// v_mfma_f32_16x16x32_bf16 (exact bf16 products, fp32 accumulation), dropping lo.lo and the
// operand remainders: relative error <= ~2^-15 per product, below fp32's 2^-24 ULP of a
// partial sum only in the last few bits, far inside TF32's 2^-11 (what cuDNN uses for fp32
// convolutions by default, torch.backends.cudnn.allow_tf32) -- at 3 MFMAs of 16 cycles per
// 16x16x32 block against 8 f32-MFMAs of 32 cycles, 5.3x the fp32-MFMA rate.
__device__ __forceinline__ void split8(const float (&v)[8], bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    hi[j] = to_bf16(v[j]);
    lo[j] = to_bf16(v[j] - from_bf16(hi[j]));
  }
}

__device__ __forceinline__ f32x4 mfma3(bf16x8 ah, bf16x8 al, bf16x8 bh, bf16x8 bl, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);   // small terms first
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
}

// f32x3_fwd: f32_fwd with conv2 on split-bf16 products.  conv1 stays exact fp32 on the VALU;
// its output a1 is stored as hi / lo bf16 planes in the bf16 forward's swizzled LDS layout
// (cnn_common.h a1_off), and conv2 runs cnn_fwd's tiling (16-row tiles = 4 pooled pixels x
// 2x2 window, one tap = one K = 32 step) with the W2 fragments split once into registers.
// Training hands the backward its operands already split, in the backward's LDS layouts
// (plain 16-B copies there instead of strided gathers + splitting per workgroup): the a1
// planes of every image (a1x: [img][hi plane | lo plane], 2 x 43264 B, the fp32 a1g buffer's
// size) and the W2^T planes (w2x: [hi | lo] x [tap][ci][64 co], chunk c at c ^ (ci & 7)),
// the latter written by the first workgroups (grid-stride over its 2304 16-B chunks).
constexpr int A1X_PLANE = P1 * 64;                 // bytes per a1 plane per image
constexpr int W2X_PLANE = 9 * C1 * 128;            // bytes per W2^T plane
constexpr int XF_XS = 0;                          // fp32 x [784]
constexpr int XF_WS = 3136;                       // fp32 w1 [288] | b1 [32] | b2 [64]
constexpr int XF_AH = 4736;                       // bf16 a1 hi plane [676 px][64 B], swizzled
constexpr int XF_AL = XF_AH + P1 * 64;            // bf16 a1 lo plane
constexpr int XF_TOTAL = XF_AL + P1 * 64;         // 91264 B
constexpr int XF_W2RB = 608;                      // W2 hi / lo staging row (bytes): 576 + 32 pad
constexpr int XF_W2PL = C2 * XF_W2RB;             // one staged plane (38912 B)
static_assert(XF_TOTAL <= 163840 && XF_AH % 128 == 0 && XF_AL % 128 == 0, "f32x3_fwd LDS");

template <bool TRAIN>
__global__ __launch_bounds__(FT, 1) void f32x3_fwd_kernel(
    const uint8_t* __restrict__ images, const int32_t* __restrict__ labels, int64_t nrow,
    const int64_t* __restrict__ ctr, const StepRows sr, const float* __restrict__ w1,
    const float* __restrict__ b1, const bf16* __restrict__ w2s, const float* __restrict__ b2,
    float* __restrict__ pool, uint8_t* __restrict__ pmask, char* __restrict__ a1x,
    float* __restrict__ xng, int32_t* __restrict__ ylab, char* __restrict__ w2x) {
  __shared__ __attribute__((aligned(16))) char smem[XF_TOTAL];
  PDM_STAMP(0);
  float* xs = reinterpret_cast<float*>(smem + XF_XS);
  float* ws = reinterpret_cast<float*>(smem + XF_WS);
  const int img = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, i16 = lane & 15;
  // 0. small weights -> LDS, the image (epoch-buffer row ctr * bfull + img, or row img)
  const int wt = tid - 256;
  if (wt >= 0 && wt < 96) {
    const float4 q = wt < 72 ? reinterpret_cast<const float4*>(w1)[wt]
                     : wt < 80 ? reinterpret_cast<const float4*>(b1)[wt - 72]
                               : reinterpret_cast<const float4*>(b2)[wt - 80];
    reinterpret_cast<float4*>(ws)[wt] = q;
  }
  const int64_t row = min(ctr ? step_row(sr, nrow, *ctr, img) : (int64_t)img, nrow - 1);
  if (tid < 196) {
    const uint32_t v = reinterpret_cast<const uint32_t*>(images + row * 784)[tid];
    const float4 x = make_float4(pdm_normalize(v & 0xff), pdm_normalize((v >> 8) & 0xff),
                                 pdm_normalize((v >> 16) & 0xff), pdm_normalize(v >> 24));
    reinterpret_cast<float4*>(xs)[tid] = x;
    if (TRAIN) reinterpret_cast<float4*>(xng + (int64_t)img * 784)[tid] = x;
  }
  if (tid == 64) ylab[img] = labels[row];
  // 1. W2 as split-bf16 hi / lo planes ([co][tap][ci] each; the optimizer writes them with
  // the fp32 update, CnnStepF32.refresh_shadows after any other change), staged once per
  // workgroup through the a1 planes' LDS (608-B rows: conflict-free fragment reads): the
  // waves' own B-fragment loads were 8 x 36.9 KB of L2 reads per CU, 75 MB per launch
  char* w2st = smem + XF_AH;
  static_assert(2 * XF_W2PL <= 2 * P1 * 64, "W2 staging fits the a1 planes");
#pragma unroll
  for (int u = 0; u < 2 * C2 * 576 / 16 / FT; ++u) {
    const int e = tid + u * FT, pl = e / (C2 * 36), k = e - pl * (C2 * 36);
    const int r = k / 36, c16 = k - r * 36;
    *reinterpret_cast<uint4*>(w2st + pl * XF_W2PL + r * XF_W2RB + c16 * 16) =
        reinterpret_cast<const uint4*>(w2s)[e];
  }
  __syncthreads();
  // this wave's conv2 B fragments: co = 32 nh + 16 j + i16, k = ci = 8 g .. 8 g + 7 of tap t
  const int nh = wave & 1;
  bf16x8 bh[9][2], bl[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int o = (nh * 32 + j * 16 + i16) * XF_W2RB + (t * 32 + 8 * g) * 2;
      bh[t][j] = *reinterpret_cast<const bf16x8*>(w2st + o);
      bl[t][j] = *reinterpret_cast<const bf16x8*>(w2st + XF_W2PL + o);
    }
  // pinned here: the compiler would sink the reads below conv1, where the staging area is
  // already overwritten
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(bh[t][j]), "+v"(bl[t][j]));
  if (TRAIN) {
    // W2^T planes for the backward: chunk (tap, c, ci) = co 8 c .. 8 c + 7 of (tap, ci)
    for (int e = img * FT + tid; e < 9 * 8 * C1; e += gridDim.x * FT) {
      const int ci = e & 31, r = e >> 5, tap = r >> 3, c = r & 7;
      bf16x8 h, l;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int o = (8 * c + u) * XF_W2RB + (tap * 32 + ci) * 2;
        h[u] = *reinterpret_cast<const bf16*>(w2st + o);
        l[u] = *reinterpret_cast<const bf16*>(w2st + XF_W2PL + o);
      }
      const int o = (tap * C1 + ci) * 128 + ((c ^ (ci & 7)) << 4);
      *reinterpret_cast<bf16x8*>(w2x + o) = h;
      *reinterpret_cast<bf16x8*>(w2x + W2X_PLANE + o) = l;
    }
  }
  PDM_STAMP(1);
  __syncthreads();   // every wave's staging reads are done: conv1 overwrites the area
  PDM_STAMP(2);
  // 2. conv1 + bias + ReLU, exact fp32 products on the fp32 MFMA (v_mfma_f32_16x16x4_f32,
  // taps 4 s + g in k-step s = 0..2, tap 9.. zero; fp32 accumulation from the bias): conv1's
  // ReLU decisions are the step's first and feed every gradient, so it keeps fp32 products
  // (split-bf16 here flipped ~15 of 1.4 M activations per 64 images and let a 5-step run drift
  // 2e-3 from torch fp32).  A = weights (row = channel 16 nt + i16), B = 16 "virtual pixels"
  // V = 28 y + x of the 28-wide x image (x = 26, 27 and y >= 26 computed and dropped;
  // x & 3 == lane & 3), so the lane's D = 4 consecutive channels 16 nt + 4 g .. + 3 of pixel V:
  // one 8-B store per plane.  It was 12.7k cycles as VALU FMAs (4 issue cycles each).
  {
    float wa[2][3];
    int xo[3];
#pragma unroll
    for (int st = 0; st < 3; ++st) {
      const int tap = 4 * st + g;
      xo[st] = tap < 9 ? (tap / 3) * IMG + tap % 3 : 0;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) wa[nt][st] = tap < 9 ? ws[(16 * nt + i16) * 9 + tap] : 0.f;
    }
    f32x4 bias[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) bias[nt][r] = ws[288 + 16 * nt + 4 * g + r];
    const int a1c = (((g >> 1) ^ (i16 & 3)) << 4) + 8 * (g & 1);   // nt = 0; nt = 1: ^ 32
    for (int tile = wave; tile < (IMG * H1 + 15) / 16; tile += 8) {
      const int V = tile * 16 + i16;
      float xb[3];
#pragma unroll
      for (int st = 0; st < 3; ++st)
        xb[st] = 4 * st + g < 9 ? xs[min(V + xo[st], IMG * IMG - 1)] : 0.f;
      const int y = V / IMG, x = V - y * IMG;
      const bool ok = y < H1 && x < H1;
      const int ab = (V - 2 * y) * 64 + a1c;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        f32x4 acc = bias[nt];
#pragma unroll
        for (int st = 0; st < 3; ++st) acc = mfma4(wa[nt][st], xb[st], acc);
        bf16x4 h, l;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float o = fmaxf(acc[r], 0.f);
          h[r] = to_bf16(o);
          l[r] = to_bf16(o - from_bf16(h[r]));
        }
        if (ok) {
          const int off = ab ^ (32 * nt);
          *reinterpret_cast<bf16x4*>(smem + XF_AH + off) = h;
          *reinterpret_cast<bf16x4*>(smem + XF_AL + off) = l;
          if (TRAIN) {
            char* dst = a1x + (int64_t)img * 2 * A1X_PLANE + off;
            *reinterpret_cast<bf16x4*>(dst) = h;
            *reinterpret_cast<bf16x4*>(dst + A1X_PLANE) = l;
          }
        }
      }
    }
  }
  PDM_STAMP(3);
  __syncthreads();
  PDM_STAMP(4);
  // 3. conv2 implicit GEMM (cnn_fwd's tiling): wave pair pr takes tiles [tt0, tt1), the wave
  // its co half nh; lane (g, i16 = 4 q + s) reads pixel (2 py + (s >> 1) + ky,
  // 2 px0 + 2 q + (s & 1) + kx), channels 8 g .. 8 g + 7 (swizzled chunk, per-lane constant)
  const int q = i16 >> 2, s = i16 & 3;
  const int lp = ((s >> 1) * H1 + 2 * q + (s & 1)) * 64;
  int aoff[9];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
      aoff[ky * 3 + kx] = lp + (ky * H1 + kx) * 64 + ((g ^ ((2 * q + (s & 1) + kx) & 3)) << 4);
  float b2r[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) b2r[j] = ws[320 + nh * 32 + j * 16 + i16];
  const int pr = wave >> 1;
  const int tt0 = pr < 2 ? 10 * pr : 20 + 8 * (pr - 2), tt1 = tt0 + (pr < 2 ? 10 : 8);
  // Software-pipelined over taps: the A hi / lo reads of the next tap (or of the next tile's
  // tap 0) are issued, pinned by a scheduling barrier, before this tap's 6 MFMAs.  Left to the
  // scheduler (the 144 B-fragment registers leave little room) every read waited right in
  // front of its MFMAs, exposing the LDS latency 18 times per tile.
  auto tile_base = [&](int tt) {
    const int py = tt / 3, px0 = 4 * (tt - py * 3);
    return (2 * py * H1 + 2 * px0) * 64;
  };
  bf16x8 ch = *reinterpret_cast<const bf16x8*>(smem + XF_AH + tile_base(tt0) + aoff[0]);
  bf16x8 cl = *reinterpret_cast<const bf16x8*>(smem + XF_AL + tile_base(tt0) + aoff[0]);
  for (int tt = tt0; tt < tt1; ++tt) {
    const int py = tt / 3, px0 = 4 * (tt - py * 3);
    const int tb = tile_base(tt), nb = tile_base(min(tt + 1, tt1 - 1));
    f32x4 acc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[j] = f32x4{b2r[j], b2r[j], b2r[j], b2r[j]};
    static_for<9>([&](auto T) __attribute__((always_inline)) {
      constexpr int t = T;
      const int na = t < 8 ? tb + aoff[t < 8 ? t + 1 : 0] : nb + aoff[0];
      const bf16x8 xh = *reinterpret_cast<const bf16x8*>(smem + XF_AH + na);
      const bf16x8 xl = *reinterpret_cast<const bf16x8*>(smem + XF_AL + na);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[j] = mfma3(ch, cl, bh[t][j], bl[t][j], acc[j]);
      ch = xh;
      cl = xl;
    });
    // epilogue (f32_fwd's): lane's 4 accumulators = the 2x2 window of pooled pixel px0 + g
    const int pp = py * HP + px0 + g;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int co = nh * 32 + j * 16 + i16;
      float m = acc[j][0];
      uint32_t oh = 1u;
#pragma unroll
      for (int r = 1; r < 4; ++r) {
        const bool gt = acc[j][r] > m;   // first position holding the max
        m = gt ? acc[j][r] : m;
        oh = gt ? (1u << r) : oh;
      }
      const bool pos = m > 0.f;
      pool[(int64_t)img * FEAT + pp * C2 + co] = pos ? m : 0.f;
      if (TRAIN) pmask[(int64_t)img * FEAT + pp * C2 + co] = (uint8_t)(pos ? 0x80u | oh : 0u);
    }
  }
  PDM_STAMP(5);
  if (tid == 7 * 64) PDM_STAMP_VAL(6, PDM_CLOCK());
}

// ------------------------------------------------------------------ f32_fc1_fwd
// part[s][row][n] = sum_{k in split s} pool[row][k] W1[n][k]; workgroup = 32 rows x 128 n of
// one split, 4 waves x 32 n; K in LDS-staged chunks of 32 (rows padded to 36 floats: the
// A / B reads of a k-step hit 64 distinct banks)
constexpr int KC = 32, KP = 36;

__global__ __launch_bounds__(256) void f32_fc1_fwd_kernel(const float* __restrict__ pool,
                                                          const float* __restrict__ w1,
                                                          float* __restrict__ part, int B,
                                                          int kchunk) {
  __shared__ __attribute__((aligned(16))) float at[32 * KP];
  __shared__ __attribute__((aligned(16))) float bt[HID * KP];
  const int mtiles = (B + 31) / 32;
  const int sidx = blockIdx.x / mtiles, mtile = blockIdx.x - sidx * mtiles;
  const int b0 = mtile * 32, kbeg = sidx * kchunk;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = kbeg; k0 < kbeg + kchunk; k0 += KC) {
    {
      const int r = tid >> 3, c4 = tid & 7;    // A: 32 rows x 8 float4 (rows past B clamped)
      const float4 v = *reinterpret_cast<const float4*>(pool + (int64_t)min(b0 + r, B - 1) * FEAT + k0 + 4 * c4);
      *reinterpret_cast<float4*>(at + r * KP + 4 * c4) = v;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {              // B: 128 rows x 8 float4
      const int e = tid + 256 * u, n = e >> 3, c4 = e & 7;
      *reinterpret_cast<float4*>(bt + n * KP + 4 * c4) =
          *reinterpret_cast<const float4*>(w1 + (int64_t)n * FEAT + k0 + 4 * c4);
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < KC / 4; ++kk) {
      float a[2], b[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) a[mt] = at[(mt * 16 + i16) * KP + kk * 4 + g];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) b[nt] = bt[(wave * 32 + nt * 16 + i16) * KP + kk * 4 + g];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = mfma4(a[mt], b[nt], acc[mt][nt]);
    }
    __syncthreads();
  }
  float* out = part + (int64_t)sidx * B * HID;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rowi = b0 + mt * 16 + 4 * g + r;
      if (rowi < B) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) out[(int64_t)rowi * HID + wave * 32 + nt * 16 + i16] = acc[mt][nt][r];
      }
    }
}

// f32x3_fc1_fwd: f32_fc1_fwd on split-bf16 products.  Per batch of XK k-steps (96 features)
// the pool rows and W1 rows are split into hi / lo bf16 planes in LDS (row pitch 208 B:
// the 16 rows of a fragment read land on distinct bank quads), then 3 MFMAs per 16x16x32
// block.  XCD-aware grid as the bf16 fc1_fwd: with S % 8 == 0 every XCD owns S / 8 splits for
// all m-tiles, so its L2 serves W1's slice to each m-tile after the first (the fp32 kernel
// re-read all of W1 per m-tile from HBM: 24 MB per step at B = 256, L2 hit 9 %).
constexpr int XK = 3;
constexpr int XKP = XK * 32 * 2 + 16;             // 208 B
constexpr int XF_BH = 2 * 32 * XKP, XF_BL = XF_BH + HID * XKP;
constexpr int XF1_TOTAL = XF_BL + HID * XKP;       // 66560 B

__device__ __forceinline__ void split4_store(char* hi, char* lo, float4 v) {
  const float f[4] = {v.x, v.y, v.z, v.w};
  bf16x4 h, l;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    h[j] = to_bf16(f[j]);
    l[j] = to_bf16(f[j] - from_bf16(h[j]));
  }
  *reinterpret_cast<bf16x4*>(hi) = h;
  *reinterpret_cast<bf16x4*>(lo) = l;
}

__global__ __launch_bounds__(256, 1) void f32x3_fc1_fwd_kernel(const float* __restrict__ pool,
                                                               const float* __restrict__ w1,
                                                               float* __restrict__ part, int B,
                                                               int kchunk) {
  __shared__ __attribute__((aligned(16))) char sm[XF1_TOTAL];
  const int mtiles = (B + 31) / 32, S = FEAT / kchunk;
  const int w = blockIdx.x;
  int mtile, sidx;
  if (S % 8 == 0) {
    const int xcd = w % 8, loc = w / 8, spx = S / 8;
    sidx = xcd * spx + loc % spx;
    mtile = loc / spx;
  } else {
    sidx = w / mtiles;
    mtile = w % mtiles;
  }
  const int b0 = mtile * 32, kbeg = sidx * kchunk;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int C4 = XK * 8;                        // float4 per staged row (24)
  // batch kb + 96's global loads are issued right after batch kb's staging barrier, so they
  // land under its MFMAs (one workgroup per CU at the training split: registers to spare)
  float4 av[3], wv[12];
  auto load = [&](int kb) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 3; ++u) {                   // A: 32 rows x 24 float4 (rows past B clamped)
      const int e = tid + 256 * u, r = e / C4, c4 = e - r * C4;
      av[u] = *reinterpret_cast<const float4*>(pool + (int64_t)min(b0 + r, B - 1) * FEAT + kbeg + kb + 4 * c4);
    }
#pragma unroll
    for (int u = 0; u < 12; ++u) {                  // B: 128 rows x 24 float4
      const int e = tid + 256 * u, r = e / C4, c4 = e - r * C4;
      wv[u] = *reinterpret_cast<const float4*>(w1 + (int64_t)r * FEAT + kbeg + kb + 4 * c4);
    }
  };
  load(0);
  for (int kb = 0; kb < kchunk; kb += 32 * XK) {
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int e = tid + 256 * u, r = e / C4, c4 = e - r * C4;
      split4_store(sm + r * XKP + 8 * c4, sm + (32 + r) * XKP + 8 * c4, av[u]);
    }
#pragma unroll
    for (int u = 0; u < 12; ++u) {
      const int e = tid + 256 * u, r = e / C4, c4 = e - r * C4;
      split4_store(sm + XF_BH + r * XKP + 8 * c4, sm + XF_BL + r * XKP + 8 * c4, wv[u]);
    }
    __syncthreads();
    if (kb + 32 * XK < kchunk) load(kb + 32 * XK);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < XK; ++ks) {
      bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int o = (mt * 16 + i16) * XKP + ks * 64 + g * 16;
        ah[mt] = *reinterpret_cast<const bf16x8*>(sm + o);
        al[mt] = *reinterpret_cast<const bf16x8*>(sm + 32 * XKP + o);
      }
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int o = (wave * 32 + nt * 16 + i16) * XKP + ks * 64 + g * 16;
        bh[nt] = *reinterpret_cast<const bf16x8*>(sm + XF_BH + o);
        bl[nt] = *reinterpret_cast<const bf16x8*>(sm + XF_BL + o);
      }
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = mfma3(ah[mt], al[mt], bh[nt], bl[nt], acc[mt][nt]);
    }
    __syncthreads();   // this batch's reads are done before the next batch's staging
  }
  float* out = part + (int64_t)sidx * B * HID;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rowi = b0 + mt * 16 + 4 * g + r;
      if (rowi < B) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) out[(int64_t)rowi * HID + wave * 32 + nt * 16 + i16] = acc[mt][nt][r];
      }
    }
}

// ------------------------------------------------------------------ f32_fc1_bwd
constexpr int DWF = 64;                 // dW tile: 128 n x 64 features
constexpr int DW_T = FEAT / DWF;        // 144
constexpr int DXF = 256;                // dX tile: 32 rows x 256 features
constexpr int DX_T = FEAT / DXF;        // 36 per 32 rows
constexpr int HRB = (HEAD_SLAB + 63) / 64;   // head-slab reduction workgroups (23)
constexpr int DHP = 144, PTP = 80, DXP = 132, WTP = 272;   // padded LDS row strides (floats)

__device__ __forceinline__ void head_slab_reduce(float* sm, int hb, const float* __restrict__ head_slab,
                                                 int head_blocks, int B, float* __restrict__ gwf2,
                                                 float* __restrict__ gbf2, float* __restrict__ gbf1,
                                                 double* __restrict__ metrics);

__global__ __launch_bounds__(256) void f32_fc1_bwd_kernel(
    const float* __restrict__ dh, int ldt, const float* __restrict__ pool,
    const float* __restrict__ w1, int B, float* __restrict__ gwf1, float* __restrict__ dpool,
    const float* __restrict__ head_slab, int head_blocks, float* __restrict__ gwf2,
    float* __restrict__ gbf2, float* __restrict__ gbf1, double* __restrict__ metrics) {
  __shared__ __attribute__((aligned(16))) float sm[32 * DXP + 32 * WTP];   // 51.7 KB (dX role)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15;
  const int nd = (ldt / 32) * DX_T;
  const int bid = blockIdx.x;
  if (bid < DW_T) {
    // ---- dW1[n][k0 + f] = sum_b dh[b][n] pool[b][k0 + f]: M = n (wave: 32), N = 64 f, K = b
    const int k0 = bid * DWF;
    float* dhs = sm;                  // [32 b][DHP]
    float* pts = sm + 32 * DHP;       // [32 b][PTP]
    f32x4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < ldt; c0 += 32) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {   // dh chunk: 32 rows x 32 float4 (rows >= B are zero)
        const int e = tid + 256 * u, r = e >> 5, c4 = e & 31;
        *reinterpret_cast<float4*>(dhs + r * DHP + 4 * c4) =
            *reinterpret_cast<const float4*>(dh + (int64_t)(c0 + r) * HID + 4 * c4);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {   // pool chunk: 32 rows x 16 float4 (rows >= B -> 0)
        const int e = tid + 256 * u, r = e >> 4, c4 = e & 15;
        const float4 v = *reinterpret_cast<const float4*>(pool + (int64_t)min(c0 + r, B - 1) * FEAT + k0 + 4 * c4);
        *reinterpret_cast<float4*>(pts + r * PTP + 4 * c4) = (c0 + r < B) ? v : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      __syncthreads();
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        float a[2], b[4];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) a[mt] = dhs[(kk * 4 + g) * DHP + wave * 32 + mt * 16 + i16];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) b[nt] = pts[(kk * 4 + g) * PTP + nt * 16 + i16];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = mfma4(a[mt], b[nt], acc[mt][nt]);
      }
      __syncthreads();
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = wave * 32 + mt * 16 + 4 * g + r;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) gwf1[(int64_t)n * FEAT + k0 + nt * 16 + i16] = acc[mt][nt][r];
      }
    return;
  }
  if (bid < DW_T + nd) {
    // ---- dpool[b][f] = sum_n dh[b][n] W1[n][f]: 32 rows x 256 f, K = 128 in 4 LDS chunks of
    // 32 n; wave: 64 f (4 n-tiles) x 32 rows (2 m-tiles)
    const int t = bid - DW_T;
    const int b0 = (t / DX_T) * 32, f0 = (t - (t / DX_T) * DX_T) * DXF;
    float* dhs = sm;                  // [32 rows][DXP]
    float* wts = sm + 32 * DXP;       // [32 n][WTP]
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u, r = e >> 5, c4 = e & 31;
      *reinterpret_cast<float4*>(dhs + r * DXP + 4 * c4) =
          *reinterpret_cast<const float4*>(dh + (int64_t)(b0 + r) * HID + 4 * c4);
    }
    f32x4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int n0 = 0; n0 < HID; n0 += 32) {
      __syncthreads();
#pragma unroll
      for (int u = 0; u < 8; ++u) {   // W1 chunk: 32 n x 64 float4
        const int e = tid + 256 * u, r = e >> 6, c4 = e & 63;
        *reinterpret_cast<float4*>(wts + r * WTP + 4 * c4) =
            *reinterpret_cast<const float4*>(w1 + (int64_t)(n0 + r) * FEAT + f0 + 4 * c4);
      }
      __syncthreads();
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        float a[2], b[4];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) a[mt] = dhs[(mt * 16 + i16) * DXP + n0 + kk * 4 + g];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) b[nt] = wts[(kk * 4 + g) * WTP + wave * 64 + nt * 16 + i16];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = mfma4(a[mt], b[nt], acc[mt][nt]);
      }
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rowi = b0 + mt * 16 + 4 * g + r;
        if (rowi < B) {
#pragma unroll
          for (int nt = 0; nt < 4; ++nt)
            dpool[(int64_t)rowi * FEAT + f0 + wave * 64 + nt * 16 + i16] = acc[mt][nt][r];
        }
      }
    return;
  }
  head_slab_reduce(sm, bid - DW_T - nd, head_slab, head_blocks, B, gwf2, gbf2, gbf1, metrics);
}

// head-slab reduction (fc1_bwd's third role, both product modes): 64 slab columns x 4 groups
// per workgroup, fixed order
__device__ __forceinline__ void head_slab_reduce(float* sm, int hb, const float* __restrict__ head_slab,
                                                 int head_blocks, int B, float* __restrict__ gwf2,
                                                 float* __restrict__ gbf2, float* __restrict__ gbf1,
                                                 double* __restrict__ metrics) {
  const int tid = threadIdx.x;
  {
    float* rs = sm;
    double* rd = reinterpret_cast<double*>(sm + 256);
    const int e = hb * 64 + (tid & 63), grp = tid >> 6;
    const int ec = min(e, HEAD_SLAB - 1);
    float sacc = 0.f;
    double sd = 0.0;
    for (int j0 = grp; j0 < head_blocks; j0 += 4 * 8) {   // 8 loads in flight, fixed order
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = head_slab[(int64_t)min(j0 + 4 * u, head_blocks - 1) * HEAD_SLAB + ec];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float x = (j0 + 4 * u < head_blocks) ? v[u] : 0.f;
        sacc += x;
        sd += (double)x;
      }
    }
    rs[tid] = sacc;
    rd[tid] = sd;
    __syncthreads();
    if (tid < 64 && e < HEAD_SLAB) {
      sacc = ((rs[tid] + rs[64 + tid]) + rs[128 + tid]) + rs[192 + tid];
      sd = ((rd[tid] + rd[64 + tid]) + rd[128 + tid]) + rd[192 + tid];
      if (e < NCLS * HID) gwf2[e] = sacc;
      else if (e < NCLS * HID + NCLS) gbf2[e - NCLS * HID] = sacc;
      else if (e < NCLS * HID + NCLS + HID) gbf1[e - NCLS * HID - NCLS] = sacc;
      else if (e == HEAD_SLAB - 2) { metrics[0] += sd; metrics[2] += (double)B; }
      else metrics[1] += sd;
    }
  }
}

// ------------------------------------------------------------------ f32x3_fc1_bwd
// f32_fc1_bwd's dW and dX roles on split-bf16 products (same grid, same head-slab role).
// Operands are staged as hi / lo bf16 planes in row-major LDS images and the transposed
// operands are read with ds_read_b64_tr_b16 (lane 4q + p of a 16-lane group gives row q,
// columns 4p .. 4p + 3; lane i receives column i); the 32-B column chunk of row r is
// XOR-swizzled so the eight rows {0..3, 8..11} one 32-lane half reads hit distinct banks.
// The next chunk's global operands are loaded into registers under the current chunk's
// MFMAs.
//   dW tile (64 features, all 128 n), K = batch in chunks of 32 rows:
//     A = dh^T  (m = n, k = b): tr reads of the dh planes [32 b][128 n]   (256 B rows)
//     B = pool  (k = b, n = f): tr reads of the pool planes [32 b][64 f]  (128 B rows)
//   dX tile (32 rows x 256 features), K = 128 n in chunks of 32:
//     A = dh    (m = b, k = n): ds_read_b128 of the dh planes [32 b][128 n] (272 B rows)
//     B = W1    (k = n, n = f): tr reads of the W1 planes [32 n][256 f]   (512 B rows)
__device__ __forceinline__ int sw8(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }
__device__ __forceinline__ int sw4(int r) { return ((r >> 1) & 1) | (((r >> 3) & 1) << 1); }
// byte offset of element (row r, col c) in a bf16 plane of 256 B / 512 B rows (32-B chunks
// c / 16 XOR sw8(r)) or of 128 B rows (chunk XOR sw4(r))
__device__ __forceinline__ int pl256(int r, int c) { return r * 256 + (((c >> 4) ^ sw8(r)) << 5) + 2 * (c & 15); }
__device__ __forceinline__ int pl512(int r, int c) { return r * 512 + (((c >> 4) ^ sw8(r)) << 5) + 2 * (c & 15); }
__device__ __forceinline__ int pl128(int r, int c) { return r * 128 + (((c >> 4) ^ sw4(r)) << 5) + 2 * (c & 15); }

constexpr int X1W_DH = 0, X1W_DL = 32 * 256, X1W_PH = 2 * 32 * 256, X1W_PL = X1W_PH + 32 * 128;
constexpr int X1X_DP = 272;                                  // dX: dh plane row pitch
constexpr int X1X_DH = 0, X1X_DL = 32 * X1X_DP, X1X_WH = 2 * 32 * X1X_DP, X1X_WL = X1X_WH + 32 * 512;
constexpr int X1_TOTAL = X1X_WL + 32 * 512;                  // 50176 B (dX; dW uses 24 KB)

__global__ __launch_bounds__(256) void f32x3_fc1_bwd_kernel(
    const float* __restrict__ dh, int ldt, const float* __restrict__ pool,
    const float* __restrict__ w1, int B, float* __restrict__ gwf1, float* __restrict__ dpool,
    const float* __restrict__ head_slab, int head_blocks, float* __restrict__ gwf2,
    float* __restrict__ gbf2, float* __restrict__ gbf1, double* __restrict__ metrics) {
  __shared__ __attribute__((aligned(16))) char smc[X1_TOTAL];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15, q = (lane >> 2) & 3, pq = lane & 3;
  const int nd = (ldt / 32) * DX_T;
  const int bid = blockIdx.x;
  if (bid < DW_T) {
    // ---- dW1[n][k0 + f] = sum_b dh[b][n] pool[b][k0 + f]
    const int k0 = bid * DWF;
    f32x4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // per thread: dh float4 pieces e = tid + 256 u (row e >> 5, cols 4 (e & 31) ..), pool
    // pieces e = tid + 256 u (row e >> 4, cols 4 (e & 15) ..); rows >= B of pool are zero
    float4 dv[4], pv[2];
    auto load = [&](int c0) __attribute__((always_inline)) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = tid + 256 * u, r = e >> 5, c4 = e & 31;
        dv[u] = *reinterpret_cast<const float4*>(dh + (int64_t)(c0 + r) * HID + 4 * c4);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int e = tid + 256 * u, r = e >> 4, c4 = e & 15;
        const float4 v = *reinterpret_cast<const float4*>(pool + (int64_t)min(c0 + r, B - 1) * FEAT + k0 + 4 * c4);
        pv[u] = (c0 + r < B) ? v : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    };
    load(0);
    for (int c0 = 0; c0 < ldt; c0 += 32) {
      __syncthreads();   // the previous chunk's reads are done
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = tid + 256 * u, r = e >> 5, c4 = e & 31;
        const int o = pl256(r, 4 * c4);
        split4_store(smc + X1W_DH + o, smc + X1W_DL + o, dv[u]);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int e = tid + 256 * u, r = e >> 4, c4 = e & 15;
        const int o = pl128(r, 4 * c4);
        split4_store(smc + X1W_PH + o, smc + X1W_PL + o, pv[u]);
      }
      __syncthreads();
      if (c0 + 32 < ldt) load(c0 + 32);   // lands under this chunk's MFMAs
      // A: rows b = 8 g + q (+ 4), columns n = 32 wave + 16 mt + 4 pq; B: rows b, columns
      // f = 16 nt + 4 pq
      bf16x8 ah[2], al[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int c = 32 * wave + 16 * mt + 4 * pq;
        const int o0 = pl256(8 * g + q, c), o1 = pl256(8 * g + 4 + q, c);
        ah[mt] = cat_tr(lds_tr16(smc + X1W_DH + o0), lds_tr16(smc + X1W_DH + o1));
        al[mt] = cat_tr(lds_tr16(smc + X1W_DL + o0), lds_tr16(smc + X1W_DL + o1));
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int c = 16 * nt + 4 * pq;
        const int o0 = pl128(8 * g + q, c), o1 = pl128(8 * g + 4 + q, c);
        const bf16x8 bh = cat_tr(lds_tr16(smc + X1W_PH + o0), lds_tr16(smc + X1W_PH + o1));
        const bf16x8 bl = cat_tr(lds_tr16(smc + X1W_PL + o0), lds_tr16(smc + X1W_PL + o1));
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) acc[mt][nt] = mfma3(ah[mt], al[mt], bh, bl, acc[mt][nt]);
      }
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = wave * 32 + mt * 16 + 4 * g + r;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) gwf1[(int64_t)n * FEAT + k0 + nt * 16 + i16] = acc[mt][nt][r];
      }
    return;
  }
  if (bid < DW_T + nd) {
    // ---- dpool[b][f] = sum_n dh[b][n] W1[n][f]: 32 rows x 256 f; wave: 64 f x 32 rows
    const int t = bid - DW_T;
    const int b0 = (t / DX_T) * 32, f0 = (t - (t / DX_T) * DX_T) * DXF;
    float4 wv[8];
    auto loadw = [&](int n0) __attribute__((always_inline)) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {   // W1 chunk: 32 n x 64 float4
        const int e = tid + 256 * u, r = e >> 6, c4 = e & 63;
        wv[u] = *reinterpret_cast<const float4*>(w1 + (int64_t)(n0 + r) * FEAT + f0 + 4 * c4);
      }
    };
    loadw(0);
#pragma unroll
    for (int u = 0; u < 4; ++u) {     // dh rows b0 .. b0 + 31 (rows >= B are zero)
      const int e = tid + 256 * u, r = e >> 5, c4 = e & 31;
      const float4 v = *reinterpret_cast<const float4*>(dh + (int64_t)(b0 + r) * HID + 4 * c4);
      const int o = r * X1X_DP + 8 * c4;
      split4_store(smc + X1X_DH + o, smc + X1X_DL + o, v);
    }
    f32x4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int n0 = 0; n0 < HID; n0 += 32) {
      __syncthreads();   // the previous chunk's W1 reads are done
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = tid + 256 * u, r = e >> 6, c4 = e & 63;
        const int o = pl512(r, 4 * c4);
        split4_store(smc + X1X_WH + o, smc + X1X_WL + o, wv[u]);
      }
      __syncthreads();
      if (n0 + 32 < HID) loadw(n0 + 32);
      bf16x8 ah[2], al[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int o = (mt * 16 + i16) * X1X_DP + (n0 + 8 * g) * 2;
        ah[mt] = *reinterpret_cast<const bf16x8*>(smc + X1X_DH + o);
        al[mt] = *reinterpret_cast<const bf16x8*>(smc + X1X_DL + o);
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int c = wave * 64 + nt * 16 + 4 * pq;
        const int o0 = pl512(8 * g + q, c), o1 = pl512(8 * g + 4 + q, c);
        const bf16x8 bh = cat_tr(lds_tr16(smc + X1X_WH + o0), lds_tr16(smc + X1X_WH + o1));
        const bf16x8 bl = cat_tr(lds_tr16(smc + X1X_WL + o0), lds_tr16(smc + X1X_WL + o1));
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) acc[mt][nt] = mfma3(ah[mt], al[mt], bh, bl, acc[mt][nt]);
      }
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rowi = b0 + mt * 16 + 4 * g + r;
        if (rowi < B) {
#pragma unroll
          for (int nt = 0; nt < 4; ++nt)
            dpool[(int64_t)rowi * FEAT + f0 + wave * 64 + nt * 16 + i16] = acc[mt][nt][r];
        }
      }
    return;
  }
  head_slab_reduce(reinterpret_cast<float*>(smc), bid - DW_T - nd, head_slab, head_blocks, B, gwf2,
                   gbf2, gbf1, metrics);
}

// ------------------------------------------------------------------ f32_conv_bwd
// Workgroup = (image, row band of R = 4 conv2-output rows): 6 bands per image.  LDS (fp32):
//   x    rows [d0, d0 + 8) of the normalised image                         1 KB
//   a1   rows [d0, d0 + 6), 26 px, stride 33                               20.6 KB
//   dz2  2 zero px + rows [d0 - 2, d0 + 7) x 26 px (cols 24, 25 zero: column -1 / -2 of a row
//        wraps onto them), pixel stride 68 (conflict-free dgrad A reads)   64.2 KB
//   W2^T [tap][co][ci], ci swizzled by (co & 2) << 3                      72 KB
constexpr int CB_R = 4, CB_S = H2 / CB_R;
constexpr int CB_XS = 0;
constexpr int CB_A1 = 1024;
constexpr int CB_DZ = CB_A1 + (CB_R + 2) * H1 * A1S * 4;
constexpr int DZS = 68;
constexpr int CB_ZR = CB_R + 5;
constexpr int CB_W2 = (CB_DZ + (2 + CB_ZR * H1) * DZS * 4 + 15) / 16 * 16;
constexpr int CB_TOTAL = CB_W2 + 9 * C2 * C1 * 4;
static_assert(CB_TOTAL <= 163840, "f32_conv_bwd LDS");
constexpr int SLB_DB2 = CNN_CONV_SLAB_DB2, SLB_DW1 = CNN_CONV_SLAB_DW1, SLB_DB1 = CNN_CONV_SLAB_DB1;

__device__ __forceinline__ int w2t_off(int tap, int co, int ci) {
  return (tap * C2 + co) * C1 + (ci ^ ((co & 2) << 3));
}

__global__ __launch_bounds__(FT, 1) void f32_conv_bwd_kernel(
    const float* __restrict__ a1g, const float* __restrict__ xng, const float* __restrict__ dpool,
    const uint8_t* __restrict__ pmask, const float* __restrict__ w2, int B, int ipb,
    float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) char smem[CB_TOTAL];
  float* xs = reinterpret_cast<float*>(smem + CB_XS);
  float* a1 = reinterpret_cast<float*>(smem + CB_A1);
  float* dz = reinterpret_cast<float*>(smem + CB_DZ);
  float* w2t = reinterpret_cast<float*>(smem + CB_W2);
  const int grp = blockIdx.x / CB_S, band = blockIdx.x - grp * CB_S;
  const int d0 = band * CB_R;
  const int aown = band == CB_S - 1 ? CB_R + 2 : CB_R;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15;
  float* out = slab + (int64_t)blockIdx.x * CNN_CONV_SLAB;
  const int pr0 = band == 0 ? 0 : d0 / 2 - 1;
  const int npr = d0 / 2 + CB_R / 2 - pr0;
  const int npx = aown * H1, nmt = (npx + 15) / 16;
  // W2^T once per workgroup (its images share the band)
  for (int e = tid; e < C2 * 288; e += FT) {
    const int co = e / 288, k = e - co * 288;
    w2t[w2t_off(k >> 5, co, k & 31)] = w2[e];
  }
  // accumulators that persist over the workgroup's images: conv2 wgrad tiles t = wave + 8 j
  // (72 = 4 co tiles x 18 (tap, ci tile)), the conv1 weight/bias partials, db2
  f32x4 wacc[9];
#pragma unroll
  for (int j = 0; j < 9; ++j) wacc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 acc1[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  float db2p = 0.f;
  for (int ii = 0; ii < ipb; ++ii) {
    const int img = grp * ipb + ii;
    if (img >= B) break;                           // workgroup-uniform
    __syncthreads();   // the previous image's reads of dz2 / a1 / x are done
    // ---- staging: zero dz2, x / a1 rows
    for (int i = tid; i < (2 + CB_ZR * H1) * DZS / 4; i += FT)
      reinterpret_cast<float4*>(dz)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i = tid; i < (CB_R + 4) * IMG; i += FT) xs[i] = xng[(int64_t)img * 784 + d0 * IMG + i];
    for (int i = tid; i < (CB_R + 2) * H1 * C1; i += FT) {
      const int p = i >> 5, c = i & 31;
      a1[p * A1S + c] = a1g[((int64_t)img * P1 + d0 * H1) * C1 + i];
    }
    __syncthreads();
    // ---- dz2 scatter of pooled rows [pr0, d0 / 2 + 2) (+ db2 of the band's own rows);
    // thread -> fixed channel co = tid & 63
    for (int it = tid; it < npr * HP * C2; it += FT) {
      const int pl = it >> 6, co = it & 63;
      const int py = pr0 + pl / HP, px = pl - (pl / HP) * HP;
      const int gi = (py * HP + px) * C2 + co;
      const uint8_t mk = pmask[(int64_t)img * FEAT + gi];
      if (mk & 0x80) {
        const float v = dpool[(int64_t)img * FEAT + gi];
        const int sidx = __builtin_ctz((unsigned)mk & 0xf);
        const int lr = 2 * py + (sidx >> 1) - (d0 - 2);
        dz[(2 + lr * H1 + 2 * px + (sidx & 1)) * DZS + co] = v;
        if (py >= d0 / 2) db2p += v;
      }
    }
    __syncthreads();
    // ---- conv2 dgrad over the band's own a1 pixels + relu'(a1) + conv1 weight/bias gradient
    // (see the file comment); per tap every operand read is issued before its 32 MFMAs
    for (int mt = wave; mt < nmt; mt += 8) {
      const int p = min(mt * 16 + i16, npx - 1);
      const int y = p / H1, x = p - y * H1;
      f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll 1
      for (int tap = 0; tap < 9; ++tap) {
        const int ky = tap / 3, kx = tap - 3 * ky;
        const float* ap = dz + (2 + (y + 2 - ky) * H1 + x - kx) * DZS + g;
        float av[16], bv[2][16];
#pragma unroll
        for (int c16 = 0; c16 < 16; ++c16) {
          av[c16] = ap[c16 * 4];
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) bv[nt][c16] = w2t[w2t_off(tap, c16 * 4 + g, nt * 16 + i16)];
        }
#pragma unroll
        for (int c16 = 0; c16 < 16; ++c16)
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) acc[nt] = mfma4(av[c16], bv[nt][c16], acc[nt]);
      }
      float xb[4];
      const int ctap = i16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int pr = mt * 16 + 4 * g + r;
        const int yy = pr / H1, xx = pr - yy * H1;
        const bool valid = pr < npx;
        xb[r] = !valid ? 0.f
                : ctap < 9 ? xs[(yy + ctap / 3) * IMG + xx + ctap % 3]
                : ctap == 9 ? 1.f : 0.f;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const float a1v = valid ? a1[min(pr, npx - 1) * A1S + nt * 16 + i16] : 0.f;
          acc[nt][r] = (valid && a1v > 0.f) ? acc[nt][r] : 0.f;
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc1[nt] = mfma4(acc[nt][r], xb[r], acc1[nt]);
    }
    // ---- conv2 wgrad over the band's own dz2 rows into the persistent tile accumulators:
    // two tiles per pass (independent accumulator chains), operands of 6 k-steps per batch
#pragma unroll
    for (int jp = 0; jp < 9; jp += 2) {
      const int nj = jp + 1 < 9 ? 2 : 1;
      int dzo[2], a1o[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int t = wave + 8 * min(jp + u, 8);
        const int mt = t / 18, nn = t - mt * 18;
        const int tap = nn >> 1, ct = nn & 1;
        const int ky = tap / 3, kx = tap - 3 * ky;
        dzo[u] = (2 + 2 * H1 + g) * DZS + mt * 16 + i16;
        a1o[u] = (ky * H1 + g + kx) * A1S + ct * 16 + i16;
      }
#pragma unroll
      for (int ks0 = 0; ks0 < CB_R * 6; ks0 += 6) {
        float av[2][6], bv[2][6];
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          const int ks = ks0 + k, rr = ks / 6, c0 = (ks - rr * 6) * 4;
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            av[u][k] = dz[dzo[u] + (rr * H1 + c0) * DZS];
            bv[u][k] = a1[a1o[u] + (rr * H1 + c0) * A1S];
          }
        }
#pragma unroll
        for (int k = 0; k < 6; ++k)
#pragma unroll
          for (int u = 0; u < 2; ++u)
            if (u < nj) wacc[jp + u] = mfma4(av[u][k], bv[u][k], wacc[jp + u]);
      }
    }
  }
  __syncthreads();   // dz2 region free: reduction scratch
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const int t = wave + 8 * j;
    const int mt = t / 18, nn = t - mt * 18;
    const int tap = nn >> 1, ct = nn & 1;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      pdm_slab_store(&out[(mt * 16 + 4 * g + r) * 288 + tap * 32 + ct * 16 + i16], wacc[j][r]);
  }
  float* red = dz;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wave * 512 + (nt * 16 + 4 * g + r) * 16 + i16] = acc1[nt][r];
  red[4096 + tid] = db2p;
  __syncthreads();
  if (tid < C2) {
    float sacc = 0.f;
    for (int w = 0; w < 8; ++w) sacc += red[4096 + w * 64 + tid];
    pdm_slab_store(&out[SLB_DB2 + tid], sacc);
  } else if (tid >= 64 && tid < 64 + C1 * 10) {
    const int e = tid - 64, ci = e / 10, tp = e - 10 * ci;
    float sacc = 0.f;
    for (int w = 0; w < 8; ++w) sacc += red[w * 512 + ci * 16 + tp];
    pdm_slab_store(tp < 9 ? &out[SLB_DW1 + ci * 9 + tp] : &out[SLB_DB1 + ci], sacc);
  }
}

// ------------------------------------------------------------------ f32x3_conv_bwd
// f32_conv_bwd with both conv2 GEMMs on split-bf16 products (mfma3).  Workgroup = (image
// group, row band of 4 conv2-output rows), 6 bands per image, as f32_conv_bwd; the operands
// are staged as hi / lo bf16 planes (split once per element at staging):
//   x     fp32 rows [d0, d0 + 8)                                            896 B
//   a1    rows [d0, d0 + 6) x 26 px x 32 ci, a1_off layout (band-local row)  2 x 9984 B
//   dz2   2 zero px + rows [d0 - 2, d0 + 7) x 26 px (cols 24, 25 zero: column -1 / -2 of a
//         row wraps onto them) x 64 co, 128 B per px, 16-B chunk c at c ^ (px & 7)  2 x 30208 B
//   W2^T  [tap][ci] rows of 64 co (128 B), chunk c at c ^ (ci & 7)              2 x 36864 B
// dgrad: D[a1 px][ci] = sum_tap sum_co dz2[px - tap][co] W2[co][tap][ci] (A rows by
// ds_read_b128, K = 64 co per tap = 2 k-steps), fused with relu'(a1) and the conv1
// weight / bias gradient (the exact fp32 MFMA of f32_conv_bwd, A = the dgrad accumulator).
// wgrad: D[co][tap, ci] = sum_px dz2[px][co] a1[px + tap][ci] over the band's 96 output
// pixels (3 k-steps; both operands by ds_read_b64_tr_b16 column reads); wave w owns co tile
// w & 3 and the 9 (tap, ci tile) columns 9 (w >> 2) ..; accumulators persist over the
// workgroup's images.  One fp32 slab per workgroup, f32_conv_bwd's layout.
constexpr int XB_XS = 0;
constexpr int XB_AP = 6 * H1 * 64;                 // a1 plane (9984 B)
constexpr int XB_AH = 1024;
constexpr int XB_AL = XB_AH + XB_AP;
constexpr int XB_DP = (2 + 9 * H1) * 128;          // dz2 plane (30208 B)
constexpr int XB_DH = XB_AL + XB_AP;
constexpr int XB_DL = XB_DH + XB_DP;
constexpr int XB_WP = 9 * C1 * 128;                // W2^T plane (36864 B)
constexpr int XB_WH = XB_DL + XB_DP;
constexpr int XB_WL = XB_WH + XB_WP;
constexpr int XB_TOTAL = XB_WL + XB_WP;            // 155136 B
static_assert(XB_TOTAL <= 163840 && XB_AH % 128 == 0 && XB_DH % 128 == 0 && XB_WH % 128 == 0,
              "f32x3_conv_bwd LDS");
static_assert((8 * 512 + 8 * FT) * 4 <= 2 * XB_DP, "reduction scratch fits the dz2 planes");

__device__ __forceinline__ int xdz_off(int zp, int chunk) { return zp * 128 + ((chunk ^ (zp & 7)) << 4); }
__device__ __forceinline__ int xw_off(int tap, int ci, int chunk) {
  return (tap * C1 + ci) * 128 + ((chunk ^ (ci & 7)) << 4);
}

struct DgFrag {   // one dgrad k-step's operands: dz2 hi / lo rows, W2^T hi / lo of 2 ci tiles
  bf16x8 ah, al, bh[2], bl[2];
};

__global__ __launch_bounds__(FT, 1) void f32x3_conv_bwd_kernel(
    const char* __restrict__ a1x, const float* __restrict__ xng, const float* __restrict__ dpool,
    const uint8_t* __restrict__ pmask, const char* __restrict__ w2x, int B, int upw,
    float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) char smem[XB_TOTAL];
  PDM_STAMP(8);
  float* xs = reinterpret_cast<float*>(smem + XB_XS);
  // units (image, row band), image-major: this workgroup takes [u0, u1)
  const int u0 = blockIdx.x * upw, u1 = min(u0 + upw, B * CB_S);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, i16 = lane & 15;
  float* out = slab + (int64_t)blockIdx.x * CNN_CONV_SLAB;
  // W2^T hi / lo planes once per workgroup: the forward wrote them split in this layout
  for (int i = tid; i < 2 * W2X_PLANE / 16; i += FT)
    reinterpret_cast<uint4*>(smem + XB_WH)[i] = reinterpret_cast<const uint4*>(w2x)[i];
  // wgrad: this wave's co tile and (tap, ci tile) columns; per-lane tr-read pieces, image
  // independent, so computed once: k-step ks covers run v = 4 ks + g = 8 pixels of output
  // row v / 3 from column 8 (v % 3); the lane addresses pixels col0 + q (+ 4), columns
  // 4 pq .. 4 pq + 3.  a1 pixel (r + ky, col0 + q + kx (+ 4)): col0 % 8 == 0, so the a1_off
  // swizzle term depends on (q + kx) & 3 only -> a base per k-step + a constant per tap
  // dgrad W2^T fragment bases (xw_off with ci & 7 == i16 & 7) for k-halves kk = 0, 1
  const int wbase0 = XB_WH + i16 * 128 + ((g ^ (i16 & 7)) << 4);
  const int wbase1 = XB_WH + i16 * 128 + (((4 + g) ^ (i16 & 7)) << 4);
  const int wmt = wave & 3, wn0 = 9 * (wave >> 2);
  const int q = (lane >> 2) & 3, pq = lane & 3;
  int dza[3][2], a1b[3], a1s[3][2];
#pragma unroll
  for (int ks = 0; ks < 3; ++ks) {
    const int v = 4 * ks + g, r = v / 3, col0 = (v - 3 * r) * 8;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int zp = 2 + (r + 2) * H1 + col0 + q + 4 * s2;
      dza[ks][s2] = xdz_off(zp, 2 * wmt + (pq >> 1)) + 8 * (pq & 1);
    }
    a1b[ks] = (r * H1 + col0 + q) * 64 + 8 * (pq & 1);
  }
#pragma unroll
  for (int kx = 0; kx < 3; ++kx)
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) a1s[kx][ct] = ((2 * ct + (pq >> 1)) ^ ((q + kx) & 3)) << 4;
  f32x4 wacc[9];
#pragma unroll
  for (int j = 0; j < 9; ++j) wacc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 acc1[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  float db2p[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // channels 8 (tid & 7) + j
  // A unit's global inputs (scatter mask bytes + dpool values, loaded unconditionally from
  // clamped indices; the x rows; the a1 plane rows) are loaded into registers one unit
  // ahead: the next unit's loads are issued after this unit's staging and land while its
  // dgrad / wgrad run, so the staging after the next barrier only writes LDS.
  static_assert(3 * HP * 8 <= FT, "one whole-window scatter item per thread");
  constexpr int A1Q = (2 * XB_AP / 16 + FT - 1) / FT; // a1 16-B pieces per thread (3)
  // per-thread element offsets of the prefetched a1 pieces (unit independent)
  int aoffq[A1Q];
#pragma unroll
  for (int u = 0; u < A1Q; ++u) {
    const int i = min(tid + u * FT, 2 * XB_AP / 16 - 1);
    const int pl = i >= XB_AP / 16, k = i - pl * (XB_AP / 16);
    aoffq[u] = pl * A1X_PLANE + 16 * k;
  }
  const int xoff = min(tid, (CB_R + 4) * IMG - 1);
  float4 dq0, dq1;                    // the scatter item's 8 pooled gradients
  uint2 mq;                           // and their 8 pool-mask bytes
  float xv = 0.f;
  static_assert(A1Q == 3, "three a1 pieces per thread");
  uint4 a1q0, a1q1, a1q2;             // (named: an array here went to scratch)
  // unit geometry: band b covers a1 rows [d0, d0 + aown) and pooled rows [pr0, pr0 + npr)
#define X3_GEOM(BAND_, D0_, PR0_, NSC_)                                                    \
  const int D0_ = (BAND_) * CB_R;                                                          \
  const int PR0_ = (BAND_) == 0 ? 0 : D0_ / 2 - 1;                                         \
  const int NSC_ = (D0_ / 2 + CB_R / 2 - PR0_) * HP * C2
#define X3_PREFETCH(UNIT_)                                                                 \
  do {                                                                                     \
    const int pimg_ = (UNIT_) / CB_S;                                                      \
    X3_GEOM((UNIT_) - pimg_ * CB_S, pd0_, ppr0_, pnsc_);                                   \
    const int64_t ib_ = (int64_t)pimg_;                                                    \
    const int64_t eo_ = ib_ * FEAT + ppr0_ * HP * C2 + min(tid, pnsc_ / 8 - 1) * 8;         \
    dq0 = *reinterpret_cast<const float4*>(dpool + eo_);                                   \
    dq1 = *reinterpret_cast<const float4*>(dpool + eo_ + 4);                               \
    mq = *reinterpret_cast<const uint2*>(pmask + eo_);                                     \
    xv = xng[ib_ * 784 + pd0_ * IMG + xoff];                                               \
    const char* src_ = a1x + ib_ * 2 * A1X_PLANE + pd0_ * H1 * 64;                         \
    a1q0 = *reinterpret_cast<const uint4*>(src_ + aoffq[0]);                               \
    a1q1 = *reinterpret_cast<const uint4*>(src_ + aoffq[1]);                               \
    a1q2 = *reinterpret_cast<const uint4*>(src_ + aoffq[2]);                               \
  } while (0)
  // the dz2 planes zeroed once: the whole-window scatter rewrites every pixel of its rows
  // (cols 0..23); cols 24, 25, the two pad pixels and local rows 6, 7 are never written
  for (int i = tid; i < 2 * XB_DP / 16; i += FT)
    reinterpret_cast<uint4*>(smem + XB_DH)[i] = make_uint4(0u, 0u, 0u, 0u);
  if (u0 < u1) X3_PREFETCH(u0);
  PDM_STAMP(9);
  for (int un = u0; un < u1; ++un) {
    const int band = un - (un / CB_S) * CB_S;     // workgroup-uniform
    X3_GEOM(band, d0, pr0, nsc);
    const int aown = band == CB_S - 1 ? CB_R + 2 : CB_R;
    const int npx = aown * H1, nmt = (npx + 15) / 16;
    const bool first = un == u0;
    __syncthreads();   // the previous unit's reads of dz2 / a1 / x are done
    // ---- staging: x rows and a1 plane rows from the registers; band 0 re-zeroes local dz2
    // rows 0, 1 (dz2 rows -2, -1; the previous image's last band wrote real rows there)
    if (band == 0) {
      for (int i = tid; i < 2 * 52 * 8; i += FT) {
        const int pl = i >= 52 * 8, k = i - pl * (52 * 8);
        reinterpret_cast<uint4*>(smem + XB_DH + pl * XB_DP + 2 * 128)[k] = make_uint4(0u, 0u, 0u, 0u);
      }
    }
    if (tid < (CB_R + 4) * IMG) xs[tid] = xv;
    {
      const uint4 qv[3] = {a1q0, a1q1, a1q2};
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int i = tid + u * FT;
        if (i < 2 * XB_AP / 16) {
          const int pl = i >= XB_AP / 16, k = i - pl * (XB_AP / 16);
          reinterpret_cast<uint4*>(smem + XB_AH + pl * XB_AP)[k] = qv[u];
        }
      }
    }
    __syncthreads();
    if (first) PDM_STAMP(10);
    if (un == u0 + 1) PDM_STAMP(7);   // the second unit's staging (its inputs prefetched)
    // ---- dz2 scatter of pooled rows [pr0, pr0 + npr) (+ db2 of the band's own rows), whole
    // windows: item (pooled pixel, 8 channels) writes the 16-B chunk of each of its window's
    // 4 pixels in both planes (the pooled gradient at the channel's argmax if it was
    // positive, zero elsewhere): 8 ds_write_b128 per item instead of zeroing 60 KB and
    // 2-byte stores.  Mask byte (f32x3_fwd): 0x80 | 1 << s if the pooled value is > 0, else 0
    if (tid < nsc / 8) {
      const int pl = tid >> 3, c = tid & 7;
      const int py = pr0 + pl / HP, px = pl - (pl / HP) * HP;
      const float v[8] = {dq0.x, dq0.y, dq0.z, dq0.w, dq1.x, dq1.y, dq1.z, dq1.w};
      const uint32_t mw[2] = {mq.x, mq.y};
      uint32_t hp[4], lp[4];             // hi / lo bf16 pairs (channels 2 e, 2 e + 1)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bf16 h0 = to_bf16(v[2 * e]), h1 = to_bf16(v[2 * e + 1]);
        const bf16 l0 = to_bf16(v[2 * e] - from_bf16(h0)), l1 = to_bf16(v[2 * e + 1] - from_bf16(h1));
        hp[e] = __builtin_bit_cast(uint16_t, h0) | (uint32_t)__builtin_bit_cast(uint16_t, h1) << 16;
        lp[e] = __builtin_bit_cast(uint16_t, l0) | (uint32_t)__builtin_bit_cast(uint16_t, l1) << 16;
      }
      const bool own = py >= d0 / 2;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t m = (mw[j >> 2] >> (8 * (j & 3))) & 0xffu;
        db2p[j] += own && (m & 0x80u) ? v[j] : 0.f;
      }
#pragma unroll
      for (int sw = 0; sw < 4; ++sw) {
        const uint32_t need = 0x80u | (1u << sw);
        uint32_t hq[4], lq[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t m0 = (mw[e >> 1] >> (16 * (e & 1))) & 0xffu;
          const uint32_t m1 = (mw[e >> 1] >> (16 * (e & 1) + 8)) & 0xffu;
          const uint32_t keep = ((m0 & need) == need ? 0x0000ffffu : 0u) |
                                ((m1 & need) == need ? 0xffff0000u : 0u);
          hq[e] = hp[e] & keep;
          lq[e] = lp[e] & keep;
        }
        const int lr = 2 * py + (sw >> 1) - (d0 - 2);
        const int zp = 2 + lr * H1 + 2 * px + (sw & 1);
        const int o = xdz_off(zp, c);
        *reinterpret_cast<uint4*>(smem + XB_DH + o) = make_uint4(hq[0], hq[1], hq[2], hq[3]);
        *reinterpret_cast<uint4*>(smem + XB_DL + o) = make_uint4(lq[0], lq[1], lq[2], lq[3]);
      }
    }
    if (un + 1 < u1) X3_PREFETCH(un + 1);   // lands under this unit's compute
    __syncthreads();
    if (first) PDM_STAMP(11);
    // ---- conv2 dgrad over the band's own a1 pixels + relu'(a1) + conv1 weight/bias grad
    for (int mt = wave; mt < nmt; mt += 8) {
      const int p = min(mt * 16 + i16, npx - 1);
      const int y = p / H1, x = p - y * H1;
      f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
      // 18 k-steps (tap, 32-co half kk), software-pipelined: the 6 fragments of step s + 1 are
      // read (pinned by a scheduling barrier) before step s's 6 MFMAs, double-buffered in
      // two named sets (a per-step array index would put them in scratch)
      DgFrag f0, f1;
      const int zp0 = 2 + (y + 2) * H1 + x;
      auto dg_load = [&](auto TAP, auto KK, DgFrag& f) __attribute__((always_inline)) {
        constexpr int tap = decltype(TAP)::value, kk = decltype(KK)::value;
        constexpr int ky = tap / 3, kx = tap - 3 * ky;
        const int zp = zp0 - ky * H1 - kx;
        f.ah = *reinterpret_cast<const bf16x8*>(smem + XB_DH + xdz_off(zp, 4 * kk + g));
        f.al = *reinterpret_cast<const bf16x8*>(smem + XB_DL + xdz_off(zp, 4 * kk + g));
        // W2^T rows ci = 16 nt + i16: xw_off = a per-lane base per kk (ci & 7 == i16 & 7) +
        // a compile-time offset, so no per-(tap, nt) address stays live across the loops
        const char* wb = smem + (kk ? wbase1 : wbase0);
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          f.bh[nt] = *reinterpret_cast<const bf16x8*>(wb + (tap * C1 + nt * 16) * 128);
          f.bl[nt] = *reinterpret_cast<const bf16x8*>(wb + XB_WP + (tap * C1 + nt * 16) * 128);
        }
      };
      dg_load(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, f0);
      static_for<18>([&](auto S) __attribute__((always_inline)) {
        constexpr int st = decltype(S)::value;
        DgFrag& cur = st % 2 == 0 ? f0 : f1;
        DgFrag& nxt = st % 2 == 0 ? f1 : f0;
        if constexpr (st + 1 < 18)
          dg_load(std::integral_constant<int, (st + 1) / 2>{}, std::integral_constant<int, (st + 1) % 2>{}, nxt);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[nt] = mfma3(cur.ah, cur.al, cur.bh[nt], cur.bl[nt], acc[nt]);
      });
      float xb[4];
      const int ctap = i16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int pr = mt * 16 + 4 * g + r;
        const int yy = pr / H1, xx = pr - yy * H1;
        const bool valid = pr < npx;
        xb[r] = !valid ? 0.f
                : ctap < 9 ? xs[(yy + ctap / 3) * IMG + xx + ctap % 3]
                : ctap == 9 ? 1.f : 0.f;
        const int pc = min(pr, npx - 1);
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          // relu'(a1): a1 >= 0, so a1 > 0 iff its hi or lo part is non-zero
          const int o = a1_off(pc / H1, pc % H1, 2 * (nt * 16 + i16));
          const unsigned short hb = *reinterpret_cast<const unsigned short*>(smem + XB_AH + o);
          const unsigned short lb = *reinterpret_cast<const unsigned short*>(smem + XB_AL + o);
          acc[nt][r] = (valid && (hb | lb) != 0) ? acc[nt][r] : 0.f;
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc1[nt] = mfma4(acc[nt][r], xb[r], acc1[nt]);
    }
    if (first) PDM_STAMP(12);
    // ---- conv2 wgrad over the band's 96 own output pixels (3 k-steps of 32): k-run
    // v = 4 ks + g (8 pixels of output row v / 3, columns 8 (v % 3) ..); lane (g, q, pq) gives
    // the addresses of pixels col0 + q and col0 + 4 + q of that run, columns 4 pq .. 4 pq + 3
    {
      // 27 steps (k-step ks, column j), software-pipelined like the dgrad: the B pieces of
      // step s + 1 and (two steps before a k-step starts) its A pieces are read, pinned by a
      // scheduling barrier, before step s's 3 MFMAs; named rotating registers (no arrays; a
      // second step of B lookahead spilled)
      auto ld_a = [&](int ks, bf16x8& ah, bf16x8& al) __attribute__((always_inline)) {
        ah = cat_tr(lds_tr16(smem + XB_DH + dza[ks][0]), lds_tr16(smem + XB_DH + dza[ks][1]));
        al = cat_tr(lds_tr16(smem + XB_DL + dza[ks][0]), lds_tr16(smem + XB_DL + dza[ks][1]));
      };
      auto ld_b = [&](int ks, int j, bf16x8& bh, bf16x8& bl) __attribute__((always_inline)) {
        // (tap, ci tile) of column j: wave-uniform, so ky / kx / ct are per-wave values and
        // the offset below is one add of a per-lane base and a small table entry
        const int nn = wn0 + j, tap = nn >> 1, ct = nn & 1;
        const int ky = tap / 3, kx = tap - 3 * ky;
        const int s0 = ct ? a1s[0][1] : a1s[0][0], s1 = ct ? a1s[1][1] : a1s[1][0];
        const int s2 = ct ? a1s[2][1] : a1s[2][0];
        const int kxs = kx == 0 ? s0 : (kx == 1 ? s1 : s2);   // selects: no indexed registers
        const int o0 = a1b[ks] + (ky * H1 + kx) * 64 + kxs;
        bh = cat_tr(lds_tr16(smem + XB_AH + o0), lds_tr16(smem + XB_AH + o0 + 256));
        bl = cat_tr(lds_tr16(smem + XB_AL + o0), lds_tr16(smem + XB_AL + o0 + 256));
      };
      bf16x8 ah0, al0, ah1, al1, bh0, bl0, bh1, bl1;
      ld_a(0, ah0, al0);
      ld_b(0, 0, bh0, bl0);
      static_for<27>([&](auto S) __attribute__((always_inline)) {
        constexpr int st = decltype(S)::value, ks = st / 9, j = st % 9;
        constexpr int sn = st + 1, ksn = sn / 9, jn = sn % 9;
        bf16x8& bhn = sn % 2 == 0 ? bh0 : bh1;
        bf16x8& bln = sn % 2 == 0 ? bl0 : bl1;
        if constexpr (sn < 27) ld_b(ksn, jn, bhn, bln);
        if constexpr (j == 7 && ks < 2) {
          if constexpr ((ks + 1) % 2 == 0) ld_a(ks + 1, ah0, al0);
          else ld_a(ks + 1, ah1, al1);
        }
        __builtin_amdgcn_sched_barrier(0);
        const bf16x8& ah = ks % 2 == 0 ? ah0 : ah1;
        const bf16x8& al = ks % 2 == 0 ? al0 : al1;
        const bf16x8& bh = st % 2 == 0 ? bh0 : bh1;
        const bf16x8& bl = st % 2 == 0 ? bl0 : bl1;
        wacc[j] = mfma3(ah, al, bh, bl, wacc[j]);
      });
    }
    if (first) PDM_STAMP(13);
  }
  PDM_STAMP(14);
  __syncthreads();   // dz2 planes free: reduction scratch
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const int nn = wn0 + j, tap = nn >> 1, ct = nn & 1;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      pdm_slab_store(&out[(wmt * 16 + 4 * g + r) * 288 + tap * 32 + ct * 16 + i16], wacc[j][r]);
  }
  float* red = reinterpret_cast<float*>(smem + XB_DH);
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wave * 512 + (nt * 16 + 4 * g + r) * 16 + i16] = acc1[nt][r];
  reinterpret_cast<float4*>(red + 4096)[2 * tid] = make_float4(db2p[0], db2p[1], db2p[2], db2p[3]);
  reinterpret_cast<float4*>(red + 4096)[2 * tid + 1] = make_float4(db2p[4], db2p[5], db2p[6], db2p[7]);
  __syncthreads();
  if (tid < C2) {
    // channel tid = 8 c + j: the threads t = c + 8 k held it (fixed order over k)
    float sacc = 0.f;
    for (int k = 0; k < FT / 8; ++k) sacc += red[4096 + ((tid >> 3) + 8 * k) * 8 + (tid & 7)];
    pdm_slab_store(&out[SLB_DB2 + tid], sacc);
  } else if (tid >= 64 && tid < 64 + C1 * 10) {
    const int e = tid - 64, ci = e / 10, tp = e - 10 * ci;
    float sacc = 0.f;
    for (int w = 0; w < 8; ++w) sacc += red[w * 512 + ci * 16 + tp];
    pdm_slab_store(tp < 9 ? &out[SLB_DW1 + ci * 9 + tp] : &out[SLB_DB1 + ci], sacc);
  }
  PDM_STAMP(15);
}

#undef X3_PREFETCH
#undef X3_GEOM

}  // namespace

// f32x3_fwd stamps in slots 0-6, f32x3_conv_bwd in 8-15 (PDM_STAMPS builds; tools/stamps_f32.py)
void read_stamps_f32(unsigned long long* host) {
#ifdef PDM_STAMPS
  hipMemcpyFromSymbol(host, HIP_SYMBOL(pdm_stamps), sizeof(unsigned long long) * 256 * 16);
#else
  for (int i = 0; i < 256 * 16; ++i) host[i] = 0;
#endif
}

void launch_f32_fwd(const uint8_t* images, const int32_t* labels, int64_t nrow, const int64_t* ctr,
                    StepRows sr, int B, const float* w1, const float* b1, const float* w2,
                    const float* b2, float* pool, uint8_t* pmask, float* a1g, float* xng,
                    int32_t* ylab, bool x3, float* w2x, const __bf16* w2s, hipStream_t st) {
  if (x3) {
    // a1g holds the split a1 planes (same bytes as the fp32 a1), w2x the split W2^T planes
    if (a1g != nullptr)
      f32x3_fwd_kernel<true><<<B, FT, 0, st>>>(images, labels, nrow, ctr, sr, w1, b1, w2s, b2, pool,
                                               pmask, reinterpret_cast<char*>(a1g), xng, ylab,
                                               reinterpret_cast<char*>(w2x));
    else
      f32x3_fwd_kernel<false><<<B, FT, 0, st>>>(images, labels, nrow, ctr, sr, w1, b1, w2s, b2,
                                                pool, pmask, nullptr, xng, ylab, nullptr);
    return;
  }
  if (a1g != nullptr)
    f32_fwd_kernel<true><<<B, FT, 0, st>>>(images, labels, nrow, ctr, sr, w1, b1, w2, b2, pool,
                                           pmask, a1g, xng, ylab);
  else
    f32_fwd_kernel<false><<<B, FT, 0, st>>>(images, labels, nrow, ctr, sr, w1, b1, w2, b2, pool,
                                            pmask, a1g, xng, ylab);
}

void launch_f32_fc1_fwd(const float* pool, const float* w1, float* part, int B, int splitk,
                        bool x3, hipStream_t st) {
  if (x3) {
    f32x3_fc1_fwd_kernel<<<((B + 31) / 32) * splitk, 256, 0, st>>>(pool, w1, part, B, FEAT / splitk);
    return;
  }
  f32_fc1_fwd_kernel<<<((B + 31) / 32) * splitk, 256, 0, st>>>(pool, w1, part, B, FEAT / splitk);
}

void launch_f32_fc1_bwd(const float* dh, int ldt, const float* pool, const float* w1, int B,
                        float* gwf1, float* dpool, const float* head_slab, int head_blocks,
                        float* gwf2, float* gbf2, float* gbf1, double* metrics, bool x3,
                        hipStream_t st) {
  const int nblk = DW_T + (ldt / 32) * DX_T + HRB;
  if (x3) {
    f32x3_fc1_bwd_kernel<<<nblk, 256, 0, st>>>(dh, ldt, pool, w1, B, gwf1, dpool, head_slab,
                                               head_blocks, gwf2, gbf2, gbf1, metrics);
    return;
  }
  f32_fc1_bwd_kernel<<<nblk, 256, 0, st>>>(dh, ldt, pool, w1, B, gwf1, dpool, head_slab,
                                           head_blocks, gwf2, gbf2, gbf1, metrics);
}

// exact: (image group of `per` images) x 6 row bands; split-bf16: `per` (image, band) units
int f32_conv_bwd_blocks(int B, int per, bool x3) {
  return x3 ? (B * CB_S + per - 1) / per : ((B + per - 1) / per) * CB_S;
}

void launch_f32_conv_bwd(const float* a1g, const float* xng, const float* dpool,
                         const uint8_t* pmask, const float* w2, int B, int ipb, float* slab,
                         bool x3, const float* w2x, hipStream_t st) {
  // ipb: images per workgroup (exact) or (image, band) units per workgroup (split-bf16)
  if (x3) {
    f32x3_conv_bwd_kernel<<<f32_conv_bwd_blocks(B, ipb, true), FT, 0, st>>>(
        reinterpret_cast<const char*>(a1g), xng, dpool, pmask, reinterpret_cast<const char*>(w2x),
        B, ipb, slab);
    return;
  }
  f32_conv_bwd_kernel<<<f32_conv_bwd_blocks(B, ipb, false), FT, 0, st>>>(a1g, xng, dpool, pmask,
                                                                          w2, B, ipb, slab);
}
