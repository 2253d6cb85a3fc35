// North-star CNN forward on gfx950 (bf16 MFMA, fp32 accumulate).
//
//   cnn_fwd : one workgroup per image — gather the uint8 image by the sampler
//             index, normalise, conv1 (1->32, 3x3) + bias + ReLU on the VALU into an
//             LDS-resident NHWC bf16 image, then conv2 (32->64, 3x3) as an implicit
//             GEMM on mfma_f32_16x16x32_bf16 (one 3x3 tap == one K=32 step == all 32
//             input channels), with bias + ReLU + MaxPool2d(2) fused in-register:
//             the M rows of a 16-row tile are ordered (pooled pixel, window pos), so a
//             lane's 4 accumulator registers ARE one 2x2 window.  Writes the pooled
//             activations (fc1 input), a 1-byte argmax|positive mask per pooled value,
//             and (training) a1 + the gathered bytes for the backward kernel.
//   fc1_fwd : split-K bf16 GEMM  part[s] = pool[:, Ks] . W1[:, Ks]^T  (fp32 slabs),
//             the reduction + bias + ReLU is fused into the head kernel.
//   cnn_head: fc1 split-K reduction + bias + ReLU, fc2, log-softmax/NLL, argmax,
//             and (training) the whole head backward: dlogits, fc2 weight/bias
//             partials, dh = dlogits.W2 * relu'(h) (bf16, + transposed copy for the
//             fc1 weight-gradient GEMM), fc1 bias partials; advances step counters.
#include "cnn_common.h"

namespace {

using namespace cnn;

// ---- cnn_fwd LDS carve (one static array; every offset 16-B aligned) ----
constexpr int F_XS = 0;                       // fp32 [28*28]          3136 B
constexpr int F_A1 = 3136;                    // bf16 a1 image         43264 B
constexpr int F_PS = F_A1 + P1 * 64;          // bf16 pooled [144][64] 18432 B
constexpr int F_MS = F_PS + PP * C2 * 2;      // u8 mask [144][64]     9216 B
constexpr int F_TOTAL = F_MS + PP * C2;       // 74048 B -> 2 workgroups / CU

template <bool TRAIN>
__global__ __launch_bounds__(256, 2) void cnn_fwd_kernel(
    const uint8_t* __restrict__ images, const int32_t* __restrict__ labels,
    const int32_t* __restrict__ idx, const int64_t* __restrict__ ctr, int bfull,
    const float* __restrict__ w1, const float* __restrict__ b1, const bf16* __restrict__ w2,
    const float* __restrict__ b2, bf16* __restrict__ pool, uint8_t* __restrict__ pmask,
    bf16* __restrict__ a1g, uint8_t* __restrict__ xg, int32_t* __restrict__ ylab) {
  __shared__ __attribute__((aligned(16))) char smem[F_TOTAL];
  float* xs = reinterpret_cast<float*>(smem + F_XS);
  char* a1s = smem + F_A1;
  bf16* ps = reinterpret_cast<bf16*>(smem + F_PS);
  uint8_t* ms = reinterpret_cast<uint8_t*>(smem + F_MS);

  const int img = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t src = idx ? (int64_t)idx[(*ctr) * (int64_t)bfull + img] : (int64_t)img;

  // 1. gather + normalise (torchvision ToTensor/Normalize semantics)
  if (tid < 196) {
    const uint32_t w = reinterpret_cast<const uint32_t*>(images + src * 784)[tid];
    float4 v;
    v.x = pdm_normalize(w & 0xff);
    v.y = pdm_normalize((w >> 8) & 0xff);
    v.z = pdm_normalize((w >> 16) & 0xff);
    v.w = pdm_normalize(w >> 24);
    reinterpret_cast<float4*>(xs)[tid] = v;
    if (TRAIN) reinterpret_cast<uint32_t*>(xg + (int64_t)img * 784)[tid] = w;
  }
  if (tid == 0) ylab[img] = labels[src];

  // conv1 weights for this thread's fixed channel group (8 channels)
  const int cg = tid & 3;
  f32x2 w1r[9][4];
  f32x2 b1r[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    b1r[j] = f32x2{b1[cg * 8 + 2 * j], b1[cg * 8 + 2 * j + 1]};
#pragma unroll
    for (int t = 0; t < 9; ++t)
      w1r[t][j] = f32x2{w1[(cg * 8 + 2 * j) * 9 + t], w1[(cg * 8 + 2 * j + 1) * 9 + t]};
  }
  __syncthreads();

  // 2. conv1 + bias + ReLU (packed fp32 FMAs), -> LDS a1 image (+ global a1)
  for (int it = tid; it < P1 * 4; it += 256) {
    const int pix = it >> 2;
    const int row = pix / H1, col = pix - row * H1;
    f32x2 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = b1r[j];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const float xv = xs[(row + ky) * IMG + col + kx];
        const f32x2 xx = {xv, xv};
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __builtin_elementwise_fma(xx, w1r[ky * 3 + kx][j], acc[j]);
      }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[2 * j] = to_bf16(fmaxf(acc[j][0], 0.f));
      o[2 * j + 1] = to_bf16(fmaxf(acc[j][1], 0.f));
    }
    *reinterpret_cast<bf16x8*>(a1s + a1_off(row, col, cg * 16)) = o;
    if (TRAIN) *reinterpret_cast<bf16x8*>(a1g + ((int64_t)img * P1 + pix) * C1 + cg * 8) = o;
  }

  // conv2 B fragments, all 9 taps x 4 n-tiles, held in registers for the whole image:
  // lane l holds B[k = ci = 8(l>>4)+j][n = co = 16nt + (l&15)] = w2[co][tap][ci]
  bf16x8 wb[9][4];
  {
    const int co_l = lane & 15, ci0 = 8 * (lane >> 4);
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        wb[t][nt] = *reinterpret_cast<const bf16x8*>(w2 + ((nt * 16 + co_l) * 9 + t) * 32 + ci0);
  }
  float b2r[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) b2r[nt] = b2[nt * 16 + (lane & 15)];
  __syncthreads();

  // 3. conv2 implicit GEMM: 36 tiles of 16 rows (4 pooled pixels x 2x2 window) x 64 co
  const int m = lane & 15, q = m >> 2, s = m & 3;
  const int chb = (lane >> 4) * 16;
  for (int tt = wave; tt < 36; tt += 4) {
    const int py = tt / 3, px0 = 4 * (tt - py * 3);
    const int oy = 2 * py + (s >> 1), ox = 2 * (px0 + q) + (s & 1);
    f32x4 acc[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(a1s + a1_off(oy + ky, ox + kx, chb));
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wb[ky * 3 + kx][nt], acc[nt], 0, 0, 0);
      }
    // epilogue: lane holds window (4 regs) of pooled pixel pp for channel co
    const int pp = py * HP + px0 + (lane >> 4);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int co = nt * 16 + (lane & 15);
      float best = fmaxf(acc[nt][0] + b2r[nt], 0.f);
      int bi = 0;
#pragma unroll
      for (int r = 1; r < 4; ++r) {
        const float v = fmaxf(acc[nt][r] + b2r[nt], 0.f);
        if (v > best) { best = v; bi = r; }          // first max in (dy, dx) row-major order
      }
      ps[pp * C2 + co] = to_bf16(best);
      ms[pp * C2 + co] = (uint8_t)(bi | (best > 0.f ? 0x80 : 0));
    }
  }
  __syncthreads();

  // 4. coalesced write-out of pooled activations + mask
  uint4* pout = reinterpret_cast<uint4*>(pool + (int64_t)img * FEAT);
  for (int i = tid; i < FEAT * 2 / 16; i += 256) pout[i] = reinterpret_cast<const uint4*>(ps)[i];
  if (TRAIN) {
    uint4* mout = reinterpret_cast<uint4*>(pmask + (int64_t)img * FEAT);
    for (int i = tid; i < FEAT / 16; i += 256) mout[i] = reinterpret_cast<const uint4*>(ms)[i];
  }
}

// ---- fc1 forward: split-K GEMM, 32 rows x 128 cols per block ----
__global__ __launch_bounds__(256) void fc1_fwd_kernel(const bf16* __restrict__ pool,
                                                      const bf16* __restrict__ wf1,
                                                      float* __restrict__ part, int B, int kchunk) {
  const int b0 = blockIdx.x * 32, sidx = blockIdx.y;
  const int kbeg = sidx * kchunk;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int rl = lane & 15, kg = (lane >> 4) * 8;
  const int n0 = wave * 32;
  // rows past B read row B-1 (valid data); their outputs are never stored
  const int r0 = min(b0 + rl, B - 1), r1 = min(b0 + 16 + rl, B - 1);
  const bf16* pa0 = pool + (int64_t)r0 * FEAT + kbeg + kg;
  const bf16* pa1 = pool + (int64_t)r1 * FEAT + kbeg + kg;
  const bf16* pb0 = wf1 + (int64_t)(n0 + rl) * FEAT + kbeg + kg;
  const bf16* pb1 = wf1 + (int64_t)(n0 + 16 + rl) * FEAT + kbeg + kg;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 3
  for (int k = 0; k < kchunk; k += 32) {
    const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(pa0 + k);
    const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(pa1 + k);
    const bf16x8 w0 = *reinterpret_cast<const bf16x8*>(pb0 + k);
    const bf16x8 w1 = *reinterpret_cast<const bf16x8*>(pb1 + k);
    acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, w0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, w1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, w0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, w1, acc[1][1], 0, 0, 0);
  }
  float* out = part + (int64_t)sidx * B * HID;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = b0 + 16 * mt + 4 * (lane >> 4) + r;
      if (row < B) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) out[(int64_t)row * HID + n0 + 16 * nt + rl] = acc[mt][nt][r];
      }
    }
}

// ---- head: fc1 reduce + bias + ReLU, fc2, CE, and (train) the head backward ----
template <bool TRAIN>
__global__ __launch_bounds__(256) void cnn_head_kernel(
    const float* __restrict__ part, int S, int B, const float* __restrict__ bf1,
    const float* __restrict__ wf2, const float* __restrict__ bf2, const int32_t* __restrict__ ylab,
    bf16* __restrict__ dh, bf16* __restrict__ dht, int ldt, float* __restrict__ slab,
    double* __restrict__ metrics, int64_t* c0, int64_t* c1) {
  __shared__ float hs[HEAD_ROWS][HID];
  __shared__ float dhs[HEAD_ROWS][HID];
  __shared__ float dls[HEAD_ROWS][NCLS];
  __shared__ float red[HEAD_ROWS][2];
  const int tid = threadIdx.x, r = tid >> 4, j = tid & 15;
  const int row = blockIdx.x * HEAD_ROWS + r;
  const bool valid = row < B;
  float h[8];
  {
    const float4 ba = reinterpret_cast<const float4*>(bf1 + 8 * j)[0];
    const float4 bb = reinterpret_cast<const float4*>(bf1 + 8 * j)[1];
    h[0] = ba.x; h[1] = ba.y; h[2] = ba.z; h[3] = ba.w;
    h[4] = bb.x; h[5] = bb.y; h[6] = bb.z; h[7] = bb.w;
  }
  if (valid) {
    for (int s = 0; s < S; ++s) {
      const float4* p = reinterpret_cast<const float4*>(part + ((int64_t)s * B + row) * HID + 8 * j);
      const float4 u = p[0], v = p[1];
      h[0] += u.x; h[1] += u.y; h[2] += u.z; h[3] += u.w;
      h[4] += v.x; h[5] += v.y; h[6] += v.z; h[7] += v.w;
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) h[i] = valid ? fmaxf(h[i], 0.f) : 0.f;

  float lg[NCLS];
#pragma unroll
  for (int c = 0; c < NCLS; ++c) {
    const float4 wa = reinterpret_cast<const float4*>(wf2 + c * HID + 8 * j)[0];
    const float4 wb = reinterpret_cast<const float4*>(wf2 + c * HID + 8 * j)[1];
    float p = h[0] * wa.x;
    p = fmaf(h[1], wa.y, p); p = fmaf(h[2], wa.z, p); p = fmaf(h[3], wa.w, p);
    p = fmaf(h[4], wb.x, p); p = fmaf(h[5], wb.y, p); p = fmaf(h[6], wb.z, p);
    p = fmaf(h[7], wb.w, p);
    lg[c] = group_sum<16>(p) + bf2[c];
  }
  const int y = valid ? ylab[row] : 0;
  float prob[NCLS];
  int correct;
  const float loss = row_xent<NCLS>(lg, y, prob, correct);

  if (!TRAIN) {
    if (j == 0) {
      red[r][0] = valid ? loss : 0.f;
      red[r][1] = valid ? (float)correct : 0.f;
    }
    __syncthreads();
    if (tid == 0) {
      double l = 0.0, c = 0.0;
      int n = 0;
      for (int i = 0; i < HEAD_ROWS; ++i) {
        l += red[i][0];
        c += red[i][1];
        n += (blockIdx.x * HEAD_ROWS + i < B);
      }
      atomicAdd(&metrics[0], l);
      atomicAdd(&metrics[1], c);
      atomicAdd(&metrics[2], (double)n);
    }
    return;
  }

  const float invB = 1.f / (float)B;
  float dl[NCLS];
#pragma unroll
  for (int c = 0; c < NCLS; ++c) dl[c] = valid ? (prob[c] - (c == y ? 1.f : 0.f)) * invB : 0.f;
  float dhv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    float a = 0.f;
#pragma unroll
    for (int c = 0; c < NCLS; ++c) a = fmaf(dl[c], wf2[c * HID + 8 * j + i], a);
    dhv[i] = (h[i] > 0.f) ? a : 0.f;
  }
  // row < ldt always (grid = ldt / 16): rows >= B write zeros (GEMM padding)
  bf16x8 o;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    o[i] = to_bf16(dhv[i]);
    dht[(int64_t)(8 * j + i) * ldt + row] = o[i];
    hs[r][8 * j + i] = h[i];
    dhs[r][8 * j + i] = dhv[i];
  }
  *reinterpret_cast<bf16x8*>(dh + (int64_t)row * HID + 8 * j) = o;
  if (j == 0) {
#pragma unroll
    for (int c = 0; c < NCLS; ++c) dls[r][c] = dl[c];
    red[r][0] = valid ? loss : 0.f;
    red[r][1] = valid ? (float)correct : 0.f;
  }
  __syncthreads();
  float* out = slab + (int64_t)blockIdx.x * HEAD_SLAB;
  for (int e = tid; e < NCLS * HID; e += 256) {
    const int c = e / HID, n = e - c * HID;
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < HEAD_ROWS; ++i) a = fmaf(dls[i][c], hs[i][n], a);
    out[e] = a;
  }
  if (tid < NCLS) {
    float a = 0.f;
    for (int i = 0; i < HEAD_ROWS; ++i) a += dls[i][tid];
    out[NCLS * HID + tid] = a;
  } else if (tid >= 16 && tid < 16 + HID) {
    const int n = tid - 16;
    float a = 0.f;
    for (int i = 0; i < HEAD_ROWS; ++i) a += dhs[i][n];
    out[NCLS * HID + NCLS + n] = a;
  } else if (tid == 255) {
    float l = 0.f, c = 0.f;
    for (int i = 0; i < HEAD_ROWS; ++i) { l += red[i][0]; c += red[i][1]; }
    out[HEAD_SLAB - 2] = l;
    out[HEAD_SLAB - 1] = c;
  }
  pdm_bump_counters(c0, c1);
}

}  // namespace

void launch_cnn_fwd(const uint8_t* images, const int32_t* labels, const int32_t* idx,
                    const int64_t* ctr, int bfull, int B, const float* w1, const float* b1,
                    const __bf16* w2, const float* b2, __bf16* pool, uint8_t* pmask, __bf16* a1,
                    uint8_t* xg, int32_t* ylab, hipStream_t st) {
  if (a1 != nullptr)
    cnn_fwd_kernel<true><<<B, 256, 0, st>>>(images, labels, idx, ctr, bfull, w1, b1, w2, b2, pool,
                                            pmask, a1, xg, ylab);
  else
    cnn_fwd_kernel<false><<<B, 256, 0, st>>>(images, labels, idx, ctr, bfull, w1, b1, w2, b2,
                                             pool, pmask, a1, xg, ylab);
}

void launch_fc1_fwd(const __bf16* pool, const __bf16* wf1, float* part, int B, int splitk,
                    hipStream_t st) {
  dim3 grid((B + 31) / 32, splitk);
  fc1_fwd_kernel<<<grid, 256, 0, st>>>(pool, wf1, part, B, FEAT / splitk);
}

void launch_cnn_head(const float* part, int splitk, int B, const float* bf1, const float* wf2,
                     const float* bf2, const int32_t* ylab, bool train, __bf16* dh, __bf16* dht,
                     int ldt, float* slab, double* metrics, int64_t* c0, int64_t* c1,
                     hipStream_t st) {
  if (train) {
    cnn_head_kernel<true><<<ldt / HEAD_ROWS, 256, 0, st>>>(part, splitk, B, bf1, wf2, bf2, ylab, dh,
                                                           dht, ldt, slab, metrics, c0, c1);
  } else {
    const int nblk = (B + HEAD_ROWS - 1) / HEAD_ROWS;
    cnn_head_kernel<false><<<nblk, 256, 0, st>>>(part, splitk, B, bf1, wf2, bf2, ylab, dh, dht,
                                                 ldt, slab, metrics, c0, c1);
  }
}
