// Small-batch CNN forward on gfx950: one image split over S = 24 / R row bands.
//
// cnn_fwd (cnn_fwd.hip) gives every image one 512-thread workgroup; at the per-rank batches
// of the reference's DDP split (S:174: 128 / 64 / 32 images at N = 2 / 4 / 8) most CUs idle
// while each busy CU runs a whole image (7.3 us at B = 32).  Here workgroup (image, band)
// produces the pooled rows [p0, p0 + R / 2) (conv2 rows [d0, d0 + R), d0 = 2 p0): it stages
// x rows [d0, d0 + R + 4), recomputes conv1 + ReLU for a1 rows [d0, d0 + R + 2) (the 2-row
// halo the 3x3 conv2 needs), runs the conv2 implicit GEMM of its 3 R / 2 tiles with bias +
// ReLU + 2x2 max-pool fused (cnn_fwd's tile scheme and swizzles, rows shifted by the band
// offset, which is even) and writes its slice of the pooled activations, the pool mask and
// (training) its rows of the gathered uint8 image.
#include "cnn_common.h"
#include "fc_carry.h"

namespace {

using namespace cnn;

constexpr int FTH = 512;

template <int R>
struct FwdBand {
  static_assert(R == 4 || R == 8 || R == 12, "band rows");
  static constexpr int S = H2 / R;
  static constexpr int RP = R / 2;                  // pooled rows per band
  static constexpr int XR = R + 4;                  // x rows staged
  static constexpr int AR = R + 2;                  // a1 rows computed
  static constexpr int X3 = 0;                      // bf16x4 x3[p] = x[p..p+2], 0
  static constexpr int A1 = (XR * IMG * 8 + 127) / 128 * 128;
  static constexpr int PS = A1 + AR * H1 * 64;      // bf16 pooled [RP * 12][64]
  static constexpr int MS = PS + RP * HP * C2 * 2;  // u8 mask [RP * 12][64]
  static constexpr int LUT = MS + RP * HP * C2;
  static constexpr int W = LUT + 512;               // fp32 w1 [288] | b1 [32] | b2 [64]
  static constexpr int SPARE = W + 1536;            // dropped conv1 stores (64 lanes x 8 B)
  static constexpr int W2 = SPARE + 512;            // conv2 B fragments (fragment-major W2)
  static constexpr int TOTAL = W2 + 36 * 1024;
  static constexpr int NT1 = (AR * IMG + 15) / 16;  // conv1 tiles (16 virtual pixels)
  static constexpr int TPW1 = (NT1 + 7) / 8;
  static constexpr int NT2 = 3 * RP;                // conv2 tiles (4 pooled px x 2x2 window)
  static constexpr int TPW2 = (NT2 + 3) / 4;        // per wave pair
  static_assert(TOTAL <= 81920 && A1 % 128 == 0 && PS % 16 == 0 && MS % 16 == 0 && W2 % 128 == 0,
                "fwd band LDS (two workgroups per CU)");
};

// CARRY: workgroups [nconv, nconv + FCC_WGS) run the previous step's fc1 update
// (fc_carry.h)
template <int R, bool TRAIN, bool CARRY>
__global__ __launch_bounds__(FTH, 2) void cnn_fwd_band_kernel(
    const uint8_t* __restrict__ images, const int32_t* __restrict__ labels,
    const int32_t* __restrict__ idx, int64_t nrow, const int64_t* __restrict__ ctr, const StepRows sr,
    const float* __restrict__ w1, const float* __restrict__ b1, const bf16* __restrict__ w2,
    const float* __restrict__ b2, bf16* __restrict__ pool, uint8_t* __restrict__ pmask,
    bf16* __restrict__ a1g, bf16* __restrict__ xng, uint8_t* __restrict__ xg,
    int32_t* __restrict__ ylab, const FcUpdate fcc, int nconv) {
  using L = FwdBand<R>;
  constexpr int S = L::S;
  __shared__ __attribute__((aligned(16))) char smem[L::TOTAL];
  static_assert(L::TOTAL >= FCC_LDS + 4, "carried fc1 update tiles fit the band's LDS");
  if constexpr (CARRY) {
    if ((int)blockIdx.x >= nconv) {
      fc_carry_role(fcc, blockIdx.x - nconv, gridDim.x - nconv, smem);
      return;
    }
  }
  bf16x4* x3 = reinterpret_cast<bf16x4*>(smem + L::X3);
  char* a1s = smem + L::A1;
  bf16* ps = reinterpret_cast<bf16*>(smem + L::PS);
  uint8_t* ms = reinterpret_cast<uint8_t*>(smem + L::MS);

  const int img = blockIdx.x / S, band = blockIdx.x - img * S;
  const int d0 = band * R, p0 = band * L::RP;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, i16 = lane & 15;
  PDM_STAMP(0);
  // 0. small conv weights through LDS (as cnn_fwd), issued first
  float4 wq = make_float4(0.f, 0.f, 0.f, 0.f);
  const int wt = tid - 256;
  if (wt >= 0 && wt < 96) {
    const float4* srcw = wt < 72 ? reinterpret_cast<const float4*>(w1) + wt
                         : wt < 80 ? reinterpret_cast<const float4*>(b1) + (wt - 72)
                                   : reinterpret_cast<const float4*>(b2) + (wt - 80);
    wq = *srcw;
  }
  __builtin_amdgcn_sched_barrier(0);
  // 1. the dependent chain: counter -> sample row -> this band's x rows
  const int64_t row_u = ctr ? step_row(sr, nrow, *ctr, img) : (int64_t)img;
  PDM_CHECK(row_u < nrow, "cnn_fwd_band sample row past the epoch", row_u, nrow);
  const int64_t row = min(row_u, nrow - 1);
  const int64_t src = idx ? (int64_t)idx[row] : row;
  constexpr int XW = L::XR * 7;                  // 4-pixel words of the staged rows
  uint32_t xw = 0, xn = 0;
  if (tid < XW) {
    const uint32_t* ip = reinterpret_cast<const uint32_t*>(images + src * 784);
    xw = ip[d0 * 7 + tid];
    xn = ip[min(d0 * 7 + tid + 1, 195)];
  }
  int lab = 0;
  if (tid == 64 && band == 0) {
    int vz;
    asm volatile("v_mov_b32 %0, 0" : "=v"(vz));
    lab = labels[src + vz];
  }
  // conv2's B fragments (fragment-major W2, 36 x 1 KB) by LDS-DMA on waves 2, 3, 6, 7, which
  // load nothing else (vmcnt is per wave: the image and weight waves never wait for it);
  // per-wave fragment loads were 18 load instructions in every wave
  if ((wave & 3) >= 2) {
    const int dw = (wave >> 2) * 2 + (wave & 1);  // 0..3
    const unsigned wbase = lds_addr(smem) + L::W2;
#pragma unroll
    for (int m = 0; m < 9; ++m) {
      const int blk = dw + 4 * m;
      glds16(w2 + (blk * 64 + lane) * 8, wbase + blk * 1024);
    }
  }
  bf16* lut = reinterpret_cast<bf16*>(smem + L::LUT);
  if (tid >= 256) lut[tid - 256] = to_bf16(pdm_normalize(tid - 256));
  float* wl = reinterpret_cast<float*>(smem + L::W);
  if (wt >= 0 && wt < 96) reinterpret_cast<float4*>(wl)[wt] = wq;
  __builtin_amdgcn_sched_barrier(0);
  __syncthreads();
  PDM_STAMP(1);

  float w1v[2][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) w1v[mt][j] = wl[(mt * 16 + i16) * 9 + 3 * min(g, 2) + min(j, 2)];
  f32x4 b1v[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) b1v[mt] = reinterpret_cast<const f32x4*>(wl + 288)[mt * 4 + g];
  if (tid < XW) {
    const bf16 v[6] = {lut[xw & 0xff], lut[(xw >> 8) & 0xff], lut[(xw >> 16) & 0xff],
                       lut[xw >> 24], lut[xn & 0xff], lut[(xn >> 8) & 0xff]};
#pragma unroll
    for (int i = 0; i < 4; ++i) x3[4 * tid + i] = bf16x4{v[i], v[i + 1], v[i + 2], bf16{}};
    // training: the band's own rows of the normalised bf16 image (the last band also rows
    // 24-27) for the backward's conv1 weight gradient
    const int own = band == S - 1 ? XW : R * 7;
    if (TRAIN && tid < own) {
      if (xng != nullptr)
        st_ho<4>(reinterpret_cast<bf16x4*>(xng + (int64_t)img * 784) + d0 * 7 + tid, bf16x4{v[0], v[1], v[2], v[3]});
      // the one-image backward (cnn_bwd) reads the gathered uint8 image instead
      if (xg != nullptr) st_ho<4>(reinterpret_cast<uint32_t*>(xg + (int64_t)img * 784) + d0 * 7 + tid, xw);
    }
  }
  __syncthreads();
  PDM_STAMP(2);

  const int nh = wave & 1;
  float b2r[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) b2r[j] = wl[320 + nh * 32 + j * 16 + i16];
  bf16x4 w1f[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int j = 0; j < 4; ++j) w1f[mt][j] = to_bf16(g < 3 && j < 3 ? w1v[mt][j] : 0.f);
  // 2. conv1 + bias + ReLU for a1 rows [d0, d0 + R + 2) (local rows 0 .. AR - 1)
  {
    const int rowg = IMG * (g < 3 ? g : 0);
    const int a1c = (conv1_pair_chunk(g) ^ (i16 & 3)) << 4;   // cnn_common.h conv1_pair
    bf16x4 bx[L::TPW1];
    int vv[L::TPW1];
#pragma unroll
    for (int k = 0; k < L::TPW1; ++k) {
      vv[k] = (wave + 8 * k) * 16 + i16;
      bx[k] = x3[min(vv[k], L::AR * IMG - 1) + rowg];
    }
#pragma unroll
    for (int k = 0; k < L::TPW1; ++k) {
      const int y = vv[k] / IMG, x = vv[k] - y * IMG;
      const bool ok = y < L::AR && x < H1;
      bf16x4 o[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(w1f[mt], bx[k], b1v[mt], 0, 0, 0);
        o[mt] = bf16x4{to_bf16(relu1(acc[0])), to_bf16(relu1(acc[1])),
                       to_bf16(relu1(acc[2])), to_bf16(relu1(acc[3]))};
      }
      // (dropped pixels: lane pairs share a 16-B slot of the 512-B spare area)
      const int dst = ok ? L::A1 + (vv[k] - 2 * y) * 64 + a1c : L::SPARE + (lane & 31) * 16;
      *reinterpret_cast<uint4*>(smem + dst) = conv1_pair(o[0], o[1]);
    }
  }
  if ((wave & 3) >= 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // W2 DMA landed
  __syncthreads();
  PDM_STAMP(3);
  if (TRAIN && a1g != nullptr) {
    // the band's own a1 rows (the last band also 24, 25), in the LDS image's swizzled layout,
    // for the backward (cnn_bwd_band copies them back by LDS-DMA instead of recomputing
    // conv1); a contiguous byte range of the image's [26][26][32] a1
    const int arows = band == S - 1 ? R + 2 : R;
    const uint4* srcv = reinterpret_cast<const uint4*>(a1s);
    uint4* dstv = reinterpret_cast<uint4*>(a1g + (int64_t)img * (P1 * C1) + d0 * H1 * C1);
    for (int i = tid; i < arows * H1 * 4; i += FTH) st_ho<4>(dstv + i, srcv[i]);
  }

  // 3. conv2 implicit GEMM over the band's tiles (local pooled row pyl, px0 % 4 == 0)
  const int q = i16 >> 2, s = i16 & 3;
  const int lp = ((s >> 1) * H1 + 2 * q + (s & 1)) * 64;
  int aoff[9];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
      aoff[ky * 3 + kx] = lp + (ky * H1 + kx) * 64 + ((g ^ ((2 * q + (s & 1) + kx) & 3)) << 4);
  const int pr = wave >> 1;
#pragma unroll 1
  for (int k = 0; k < L::TPW2; ++k) {
    const int tt = pr + 4 * k;
    if (tt >= L::NT2) break;
    const int pyl = tt / 3, px0 = 4 * (tt - pyl * 3);
    const char* tb = a1s + (2 * pyl * H1 + 2 * px0) * 64;
    bf16x8 a[9], wb[9][2];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      a[t] = *reinterpret_cast<const bf16x8*>(tb + aoff[t]);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        wb[t][j] = *reinterpret_cast<const bf16x8*>(smem + L::W2 + (((nh * 2 + j) * 9 + t) * 64 + lane) * 16);
    }
    f32x4 acc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[j] = f32x4{b2r[j], b2r[j], b2r[j], b2r[j]};
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[t], wb[t][j], acc[j], 0, 0, 0);
    const int pp = pyl * HP + px0 + g;           // local pooled pixel
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int co = nh * 32 + j * 16 + i16;
      const int c0 = fbits(acc[j][0]), c1 = fbits(acc[j][1]), c2 = fbits(acc[j][2]);
      const int mb = max(max(max(c0, c1), c2), fbits(acc[j][3]));
      uint32_t oh = c2 == mb ? 4u : 8u;
      oh = c1 == mb ? 2u : oh;
      oh = c0 == mb ? 1u : oh;
      ps[pp * C2 + co] = to_bf16(__builtin_bit_cast(float, max(mb, 0)));
      ms[pp * C2 + co] = (uint8_t)(mb > 0 ? 0x80u | oh : 0u);
    }
  }
  __syncthreads();
  PDM_STAMP(4);
  // 4. coalesced write-out of the band's pooled rows + mask
  constexpr int PB = L::RP * HP * C2;            // pooled values per band
  uint4* pout = reinterpret_cast<uint4*>(pool + (int64_t)img * FEAT + p0 * HP * C2);
  for (int i = tid; i < PB * 2 / 16; i += FTH) st_ho<4>(pout + i, reinterpret_cast<const uint4*>(ps)[i]);
  if (TRAIN) {
    uint4* mout = reinterpret_cast<uint4*>(pmask + (int64_t)img * FEAT + p0 * HP * C2);
    for (int i = tid; i < PB / 16; i += FTH) st_ho<4>(mout + i, reinterpret_cast<const uint4*>(ms)[i]);
  }
  if (tid == 64 && band == 0) st_ho<4>(ylab + img, lab);
  PDM_STAMP(5);
}

template <int R>
void launch_band(const uint8_t* images, const int32_t* labels, const int32_t* idx, int64_t nrow,
                 const int64_t* ctr, StepRows sr, int B, const float* w1, const float* b1,
                 const __bf16* w2, const float* b2, __bf16* pool, uint8_t* pmask, __bf16* a1g,
                 __bf16* xng, uint8_t* xg, int32_t* ylab, const FcUpdate* fcc, hipStream_t st) {
  const int nblk = B * FwdBand<R>::S;
  if (fcc != nullptr) {        // training only (the caller carries an update between steps)
    cnn_fwd_band_kernel<R, true, true><<<nblk + FCC_WGS, FTH, 0, st>>>(
        images, labels, idx, nrow, ctr, sr, w1, b1, w2, b2, pool, pmask, a1g, xng, xg, ylab, *fcc,
        nblk);
    return;
  }
  const FcUpdate none{};
  if (a1g != nullptr || xg != nullptr)
    cnn_fwd_band_kernel<R, true, false><<<nblk, FTH, 0, st>>>(images, labels, idx, nrow, ctr, sr, w1,
                                                              b1, w2, b2, pool, pmask, a1g, xng, xg,
                                                              ylab, none, nblk);
  else
    cnn_fwd_band_kernel<R, false, false><<<nblk, FTH, 0, st>>>(images, labels, idx, nrow, ctr, sr, w1,
                                                               b1, w2, b2, pool, pmask, a1g, xng, xg,
                                                               ylab, none, nblk);
}

}  // namespace

void launch_cnn_fwd_band(const uint8_t* images, const int32_t* labels, const int32_t* idx,
                         int64_t nrow, const int64_t* ctr, StepRows sr, int B, int bands,
                         const float* w1, const float* b1, const __bf16* w2, const float* b2,
                         __bf16* pool, uint8_t* pmask, __bf16* a1g, __bf16* xng, uint8_t* xg,
                         int32_t* ylab, const FcUpdate* fcc, hipStream_t st) {
  switch (bands) {
    case 2:
      launch_band<12>(images, labels, idx, nrow, ctr, sr, B, w1, b1, w2, b2, pool, pmask, a1g, xng,
                      xg, ylab, fcc, st);
      break;
    case 3:
      launch_band<8>(images, labels, idx, nrow, ctr, sr, B, w1, b1, w2, b2, pool, pmask, a1g, xng,
                     xg, ylab, fcc, st);
      break;
    case 6:
      launch_band<4>(images, labels, idx, nrow, ctr, sr, B, w1, b1, w2, b2, pool, pmask, a1g, xng,
                     xg, ylab, fcc, st);
      break;
    default:
      break;   // bind.cpp validates bands
  }
}

#ifdef PDM_STAMPS
void read_stamps_fwd_band(unsigned long long* host) {
  hipMemcpyFromSymbol(host, HIP_SYMBOL(pdm_stamps), sizeof(unsigned long long) * 256 * 16);
}
#else
void read_stamps_fwd_band(unsigned long long* host) {
  for (int i = 0; i < 256 * 16; ++i) host[i] = 0;
}
#endif
