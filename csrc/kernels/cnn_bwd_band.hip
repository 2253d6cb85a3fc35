// Small-batch CNN conv backward on gfx950: one image split over S = 24 / R row bands.
//
// cnn_bwd (cnn_bwd.hip) gives every image one 512-thread workgroup on one CU; at the
// per-rank batches of the reference's DDP split (S:174: 256 / world_size = 128 / 64 / 32
// images at N = 2 / 4 / 8) that leaves 50-88 % of the 256 CUs idle while each busy CU runs
// one image's whole latency chain (15 us at B = 32).  Here workgroup (image, band) owns the
// conv2-output (dz2) rows [d0, d0 + R) and the conv1-output (a1) rows [d0, d0 + R) (the last
// band also rows 24, 25), so an image's work is spread over S CUs:
//
//   staging   x rows [d0, d0 + R + 4) -> normalise -> conv1 recompute of a1 rows
//             [d0, d0 + R + 2) (MFMA 16x16x16 on the 28-wide virtual grid, as cnn_bwd);
//             dz2 = maxpool^-1(dpool) for dz2 rows [d0 - 2, d0 + R + 2) (the 2-row halo above
//             feeds the dgrad of the band's first a1 rows; halo rows outside the image and the
//             band's overflow rows are zero-filled, so no zero-block substitution is needed);
//             W2^T (36 KB) by LDS-DMA
//   waves 0-3 conv2 wgrad over the band's own dz2 rows (K = 24 R pixels = 3R/4 k-steps of
//             32, the cnn_bwd operand addressing shifted by the 2 halo rows)
//   waves 4-7 conv2 dgrad over the band's own a1 rows + relu'(a1) + conv1 wgrad/bias
//   tail      one fp32 slab per workgroup, the cnn_bwd slab layout (conv_reduce / the fused
//             optimizer sum B * S slabs instead of B)
//
// R in {12, 8, 4} (S = 2, 3, 6): the wgrad k-step pattern repeats every 4 dz2 rows, and the
// LDS image swizzles depend on the row only mod 2, which band offsets (even) preserve.
#include "cnn_common.h"
#include "xgmi.h"

namespace {

using namespace cnn;

constexpr int BTH = 512;
constexpr int DSB = 26;   // dz2 row stride in pixels (24 + 2 zero columns)

template <int R>
struct BandLds {
  static_assert(R == 4 || R == 8 || R == 12, "band rows");
  static constexpr int S = H2 / R;              // bands per image
  static constexpr int XR = R + 4;              // x rows staged
  static constexpr int AR = R + 2;              // a1 rows recomputed
  static constexpr int ZR = R + 5;              // dz2 rows staged: global [d0 - 2, d0 + R + 3)
  static constexpr int XS = 0;                  // bf16 [XR * 28 + 16]
  static constexpr int A1 = ((XR * IMG + 16) * 2 + 1023) / 1024 * 1024;   // (DMA pieces of 1 KB)
  static constexpr int Z0 = A1 + AR * H1 * 64;  // 4 zero pixels: column -1, -2 of dz2 row 0
  static constexpr int DZ = Z0 + 512;
  static constexpr int W2 = DZ + ZR * DSB * 128;
  static constexpr int TOTAL = W2 + 9 * C1 * C2 * 2;
  static constexpr int RED = DZ;                // reduction scratch (dz2 is dead by then)
  static constexpr int KS = 3 * R / 4;          // wgrad k-steps
  static constexpr int PR = R / 2 + 1;          // pooled rows staged (own + 1 above)
  static constexpr int SCT = 192;               // scatter threads (waves 5-7)
  static constexpr int NIT = (PR * HP * 8 + SCT - 1) / SCT;   // scatter items per thread
  // dgrad tiles per dgrad wave (waves 4-7 take tiles wd + 4 k, k < MD, in one pass; the wgrad
  // waves take the band's remaining tiles after their wgrad): balances wgrad's 15 R MFMAs
  // per wave against dgrad's 36 per tile
  static constexpr int MD = R == 4 ? 2 : (R == 8 ? 4 : 5);
  static_assert(TOTAL <= 163840, "band LDS carve");
  static_assert(A1 % 128 == 0 && DZ % 128 == 0 && W2 % 128 == 0, "128-B aligned images");
  static_assert((8 * C2 + 4 * C1 * 16) * 4 <= ZR * DSB * 128, "reduction scratch fits dz2");
};

constexpr int RED_DB2 = 0;                     // [8 waves][64]
constexpr int RED_DW1 = RED_DB2 + 8 * C2;      // [4 waves][32 ci][16 taps] (tap 9 = bias)
constexpr int SL_DB2 = CNN_CONV_SLAB_DB2, SL_DW1 = CNN_CONV_SLAB_DW1, SL_DB1 = CNN_CONV_SLAB_DB1;
constexpr int W2_CHUNKS = 9 * C1 * C2 * 2 / 16;   // 2304 16-B chunks of W2^T

// conv2 dgrad of MTP tiles {tile0 + 4k} of 16 virtual pixels V = 28 y + x of the band's
// local a1 grid (y < aown rows are the band's; the rest, and x >= 26, are dropped), fused with
// relu'(a1) and the conv1 weight/bias gradient (acc1).  Same operand scheme as cnn_bwd's
// dgrad_pass; the dz2 halo rows are materialised, so every tap reads the staged image.
template <int R, int MTP, int PFD>
__device__ __forceinline__ void band_dgrad(const char* smem, int tile0, int aown,
                                           const int (&ka1)[4], f32x4 (&acc1)[2]) {
  using L = BandLds<R>;
  const int lane = threadIdx.x & 63, g = lane >> 4, i16 = lane & 15;
  int rb[MTP], gs[MTP];
#pragma unroll
  for (int k = 0; k < MTP; ++k) {
    // clamped: a tile past the band reads staged rows (finite) and its outputs are dropped
    const int v = min((tile0 + 4 * k) * 16 + i16, aown * IMG + 15);
    const int y = v / IMG, x = v - y * IMG;
    rb[k] = L::DZ + (y * DSB + x - 2) * 128;     // dz2 local row y - ky + 2, col x - kx
    gs[k] = (g + 4 * y + x) << 4;
  }
  const int wl0 = L::W2 + i16 * 128 + ((g ^ ((i16 >> 1) & 7)) << 4);
  auto read_step = [&](int tk, bf16x8 (&a)[MTP], bf16x8 (&w)[2]) __attribute__((always_inline)) {
    const int tap = tk >> 1, kh = tk & 1;
    const int ky = tap / 3, kx = tap - 3 * ky;
    const int sk16 = (4 * ky + kx) << 4;
    const int off = ((2 - ky) * DSB + (2 - kx)) * 128;
#pragma unroll
    for (int k = 0; k < MTP; ++k) {
      int ad = ((gs[k] - sk16) & 0x70) | rb[k];
      if (kh) ad ^= 64;
      a[k] = *reinterpret_cast<const bf16x8*>(smem + ad + off);
    }
    const int wl = kh ? (wl0 ^ 64) : wl0;
    w[0] = *reinterpret_cast<const bf16x8*>(smem + wl + tap * 4096);
    w[1] = *reinterpret_cast<const bf16x8*>(smem + wl + tap * 4096 + 2048);
  };
  const int ctap = i16;
  const int cky = ctap / 3, ckx = ctap - 3 * cky;
  const int xoff = (ctap < 9) ? (cky * IMG + ckx) : 0;
  const bf16* xs = reinterpret_cast<const bf16*>(smem + L::XS);
  bf16x4 bx[MTP];
  short av[MTP][4][2];
  bool vhi[MTP];
  auto read_ep = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < MTP; ++k) {
      const int v0 = (tile0 + 4 * k) * 16 + 4 * g;
      const int y = v0 / IMG, x0 = v0 - y * IMG;
      const bool vt = y < aown;
      vhi[k] = vt && x0 < 24;
      const int vc = vt ? v0 : 0;
      const int pb = vt ? L::A1 + (v0 - 2 * y) * 64 : L::Z0;   // zero block: relu' = 0
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        bx[k][r] = xs[vc + r + xoff];
        av[k][r][0] = *reinterpret_cast<const short*>(smem + pb + ka1[r]);
        av[k][r][1] = *reinterpret_cast<const short*>(smem + pb + (ka1[r] ^ 32));
      }
    }
  };
  f32x4 acc[MTP][2];
#pragma unroll
  for (int k = 0; k < MTP; ++k) acc[k][0] = acc[k][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a[PFD + 1][MTP], w[PFD + 1][2];
#pragma unroll
  for (int tk = 0; tk < PFD; ++tk) read_step(tk, a[tk], w[tk]);
#pragma unroll
  for (int tk = 0; tk < 18; ++tk) {
    __builtin_amdgcn_sched_barrier(0);
    if (tk + PFD < 18) read_step(tk + PFD, a[(tk + PFD) % (PFD + 1)], w[(tk + PFD) % (PFD + 1)]);
    else if (tk + PFD == 18) read_ep();
    __builtin_amdgcn_sched_barrier(0);
    const int s = tk % (PFD + 1);
#pragma unroll
    for (int k = 0; k < MTP; ++k) {
      acc[k][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s][k], w[s][0], acc[k][0], 0, 0, 0);
      acc[k][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s][k], w[s][1], acc[k][1], 0, 0, 0);
    }
  }
  const bf16 one = to_bf16(1.f);
#pragma unroll
  for (int k = 0; k < MTP; ++k) {
    const bf16x4 b = (ctap == 9) ? bf16x4{one, one, one, one} : bx[k];
    bf16x4 az[2];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
        az[nt][r] = to_bf16((av[k][r][nt] > 0 && (r < 2 || vhi[k])) ? acc[k][nt][r] : 0.f);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
      acc1[nt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(az[nt], b, acc1[nt], 0, 0, 0);
  }
}

template <int R>
__global__ __launch_bounds__(BTH, 1) void cnn_bwd_band_kernel(
    const bf16* __restrict__ a1g, const bf16* __restrict__ xng, const bf16* __restrict__ dpool,
    const uint8_t* __restrict__ pmask, const bf16* __restrict__ w2t, float* __restrict__ slab,
    unsigned* xg_sync) {
  using L = BandLds<R>;
  constexpr int S = L::S;
  __shared__ __attribute__((aligned(16))) char smem[L::TOTAL];
  // xgmi streamed mode: fc1_bwd has finished, so the fc gradient bucket is complete
  if (xg_sync != nullptr && blockIdx.x == 0 && threadIdx.x == 0) xg_signal_backward(xg_sync);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, i16 = lane & 15;
  const int img = blockIdx.x / S, band = blockIdx.x - img * S;
  const int d0 = band * R;                       // first own dz2 / a1 row (global)
  const int aown = band == S - 1 ? R + 2 : R;    // own a1 rows
  const int pr0 = band == 0 ? 0 : d0 / 2 - 1;    // first staged pooled row
  const int npr = d0 / 2 + R / 2 - pr0;          // staged pooled rows
  const int pown0 = d0 / 2;                      // first own pooled row
  // band geometry: the staged pooled rows fit the scatter's items, and the band's a1 / x rows
  // (incl. halos and the last band's two extra a1 rows) stay inside the image
  PDM_CHECK(npr >= 1 && npr <= L::PR, "cnn_bwd_band staged pooled rows", npr, L::PR);
  PDM_CHECK(d0 + L::AR <= H1 && d0 + L::XR <= IMG, "cnn_bwd_band a1 / x rows past the image",
            d0, band);
  bf16* xs = reinterpret_cast<bf16*>(smem + L::XS);
  float* out = slab + (int64_t)blockIdx.x * CNN_CONV_SLAB;
  PDM_STAMP(0);

  // ---- 1. loads, split by role (vmcnt is per wave: the scatter waves never wait for a DMA)
  //   waves 0-1   a1 rows [d0, d0 + R + 2) as the forward left them (its swizzled LDS image,
  //               cnn_fwd_band) and the normalised x rows [d0, d0 + R + 4), by LDS-DMA
  //   waves 2-4   W2^T (36 KB) by LDS-DMA
  //   waves 5-7   dpool / pmask items of the staged pooled rows
  const int nit = npr * HP * 8;
  uint4 d[L::NIT];
  uint2 mk[L::NIT];
  if (wave < 2) {
    constexpr int AB = L::AR * H1 * 64;          // a1 bytes
    constexpr int NA = (AB + 1023) / 1024;       // 1-KB DMA pieces
    const char* asrc = reinterpret_cast<const char*>(a1g + (int64_t)img * (P1 * C1) + d0 * H1 * C1);
    const unsigned abase = lds_addr(smem) + L::A1;
#pragma unroll
    for (int m = 0; m < (NA + 1) / 2; ++m) {
      const int blk = wave + 2 * m;
      if (blk < NA && blk * 1024 + lane * 16 < AB) glds16(asrc + blk * 1024 + lane * 16, abase + blk * 1024);
    }
    if (wave == 1 && lane * 16 < L::XR * IMG * 2)    // x rows: XR * 56 B <= 1 KB
      glds16(reinterpret_cast<const char*>(xng + (int64_t)img * 784 + d0 * IMG) + lane * 16,
             lds_addr(smem) + L::XS);
  } else if (wave < 5) {
    const unsigned wbase = lds_addr(smem) + L::W2;
#pragma unroll
    for (int m = 0; m < W2_CHUNKS / 64 / 3; ++m) {
      const int blk = (wave - 2) + 3 * m;
      const int row = 8 * blk + (lane >> 3), ch = (lane & 7) ^ ((row >> 1) & 7);
      glds16(w2t + row * 64 + ch * 8, wbase + blk * 1024);
    }
  } else {
    const uint4* dpv = reinterpret_cast<const uint4*>(dpool + (int64_t)img * FEAT) + pr0 * HP * 8;
    const uint2* mkv = reinterpret_cast<const uint2*>(pmask + (int64_t)img * FEAT) + pr0 * HP * 8;
#pragma unroll
    for (int k = 0; k < L::NIT; ++k) {
      const int it = min(tid - 320 + k * L::SCT, nit - 1);
      d[k] = dpv[it];
      mk[k] = mkv[it];
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  PDM_STAMP(1);
  // ---- 2. zero fills: the 2 pad columns of every staged dz2 row, the rows the scatter does
  // not write (halo rows outside the image, overflow rows), the zero block, the x pad
  {
    const int zlo = 2 * pr0 - (d0 - 2);          // first scattered local row (0 or 2)
    const int zhi = zlo + 2 * npr;               // = R + 2
    PDM_CHECK(zlo >= 0 && zhi <= L::ZR, "cnn_bwd_band scattered dz2 rows", zlo, zhi);
    constexpr int NZ = 4 + L::ZR * DSB;          // candidate pixels: zero block + all rows
    for (int i = tid; i < NZ * 8; i += BTH) {
      const int pix = i >> 3, ch = i & 7;
      int off;
      if (pix < 4) {
        off = L::Z0 + pix * 128;
      } else {
        const int p = pix - 4, lr = p / DSB, c = p - lr * DSB;
        if (lr >= zlo && lr < zhi && c < 24) continue;   // written by the scatter
        off = L::DZ + (lr * DSB + c) * 128;
      }
      *reinterpret_cast<uint4*>(smem + off + ch * 16) = make_uint4(0, 0, 0, 0);
    }
    if (tid < 2) reinterpret_cast<uint4*>(xs + L::XR * IMG)[tid] = make_uint4(0, 0, 0, 0);
  }
  PDM_STAMP(2);
  PDM_STAMP(3);
  // ---- 4. the dz2 scatter of pooled rows [pr0, pr0 + npr) (+ the conv2 bias gradient of the
  // band's own pooled rows), whole-window writes as in cnn_bwd
  float db2p[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < L::NIT; ++k) {
    const int it = tid - 320 + k * L::SCT;   // it & 7 == tid & 7: fixed channel chunk
    if (wave >= 5 && it < nit) {
      const int pl = it >> 3, ch = it & 7;
      const int pyl = pl / HP, px = pl - pyl * HP;
      const int py = pr0 + pyl;
      const int lr = 2 * py - (d0 - 2);          // local dz2 row of the window's top row
      // the window's two rows inside the staged halo image [d0 - 2, d0 + R + 3)
      PDM_CHECK(lr >= 0 && lr + 1 < L::ZR, "cnn_bwd_band halo dz2 row", lr, L::ZR);
      const int base = L::DZ + (lr * DSB + 2 * px) * 128;
      const int b0 = 2 * px + ch;                // + 4 (lr + dy) + dx; 4 lr = 0 mod 8
      const uint32_t dw[4] = {d[k].x, d[k].y, d[k].z, d[k].w};
      const uint32_t mw[2] = {mk[k].x, mk[k].y};
      if (py >= pown0) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t sh = mw[h] << 8;
          const uint32_t pos[2] = {__builtin_amdgcn_perm(mw[h], sh, 0x0A0A0808u),
                                   __builtin_amdgcn_perm(mw[h], sh, 0x0B0B0909u)};
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const uint32_t w = dw[2 * h + e] & pos[e];
            db2p[4 * h + 2 * e] += __builtin_bit_cast(float, w << 16);
            db2p[4 * h + 2 * e + 1] += __builtin_bit_cast(float, w & 0xffff0000u);
          }
        }
      }
#pragma unroll
      for (int sw = 0; sw < 4; ++sw) {
        uint4 o;
        uint32_t* ow = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t u = mw[h] << (7 - sw), v = mw[h] << (15 - sw);
          ow[2 * h] = dw[2 * h] & __builtin_amdgcn_perm(u, v, 0x0A0A0808u);
          ow[2 * h + 1] = dw[2 * h + 1] & __builtin_amdgcn_perm(u, v, 0x0B0B0909u);
        }
        const int off = base + (sw >> 1) * (DSB * 128) + (sw & 1) * 128 +
                        (((b0 + 4 * (sw >> 1) + (sw & 1)) & 7) << 4);
        *reinterpret_cast<uint4*>(smem + off) = o;
      }
    }
  }
  PDM_STAMP(4);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMA pieces have landed
  __syncthreads();
  PDM_STAMP(5);

  // relu'(a1) read offsets of channel i16 at pixel x with x & 3 == r (a1_off swizzle)
  int ka1[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) ka1[r] = r * 64 + ((((2 * i16) >> 4) ^ r) << 4) + ((2 * i16) & 15);
  f32x4 acc1[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  if (wave < 4) {
    // ===== conv2 wgrad over the band's own dz2 rows: (tap, ci-tile) pairs {w + 4 pi} =====
    const bool five = wave < 2;
    int abA[3][4], abA2[3][4], abB[3][5];
    {
      int ln;
      asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
      const int gg = ln >> 4, q = (ln >> 2) & 3, pq = ln & 3;
      int cp[5];
#pragma unroll
      for (int pi = 0; pi < 5; ++pi) {
        const int pair = min(wave + 4 * pi, 17);
        const int tap = pair >> 1, nt = pair & 1;
        const int ky = tap / 3, kx = tap - 3 * ky;
        cp[pi] = (ky * H1 + kx) * 64 + (((2 * nt + (pq >> 1)) ^ ((q + kx) & 3)) << 4) + 8 * (pq & 1);
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int v = 4 * j + gg, rj = v / 3, xj = (v - 3 * rj) * 8 + q;
        // own dz2 row rj = local row rj + 2 (4 (rj + 2) = 4 rj mod 8: same rotation)
        const int dbase = L::DZ + ((rj + 2) * DSB + xj) * 128 + 8 * (pq & 1);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
          const int co = (((pq >> 1) + 4 * rj + xj + 2 * mt) & 7) << 4;
          abA[j][mt] = dbase + co;
          abA2[j][mt] = dbase + 512 + (co ^ 64);
        }
#pragma unroll
        for (int pi = 0; pi < 5; ++pi) abB[j][pi] = L::A1 + (rj * H1 + xj) * 64 + cp[pi];
      }
    }
    auto rd_a = [&](int ks, int mt) __attribute__((always_inline)) {
      const int j = ks % 3, m = ks / 3;
      return cat_tr(lds_tr16(smem + abA[j][mt] + m * 4 * DSB * 128),
                    lds_tr16(smem + abA2[j][mt] + m * 4 * DSB * 128));
    };
    auto rd_b = [&](int ks, int pi) __attribute__((always_inline)) {
      const int j = ks % 3, m = ks / 3;
      return cat_tr(lds_tr16(smem + abB[j][pi] + m * 4 * H1 * 64),
                    lds_tr16(smem + abB[j][pi] + m * 4 * H1 * 64 + 256));
    };
    f32x4 acc[5][4];
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 A[2][4], Bv[2][5];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) A[0][mt] = rd_a(0, mt);
#pragma unroll
    for (int pi = 0; pi < 5; ++pi) Bv[0][pi] = rd_b(0, pi);
    static_for<L::KS>([&](auto KS) __attribute__((always_inline)) {
      constexpr int ks = decltype(KS)::value;
      bf16x8 (&Ac)[4] = A[ks & 1];
      bf16x8 (&Bc)[5] = Bv[ks & 1];
      bf16x8 (&An)[4] = A[(ks + 1) & 1];
      bf16x8 (&Bn)[5] = Bv[(ks + 1) & 1];
#pragma unroll
      for (int pi = 0; pi < 5; ++pi) {
        __builtin_amdgcn_sched_barrier(0);
        if (ks + 1 < L::KS) {
          Bn[pi] = rd_b(ks + 1, pi);
          if (pi < 4) An[pi] = rd_a(ks + 1, pi);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          acc[pi][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ac[mt], Bc[pi], acc[pi][mt], 0, 0, 0);
      }
    });
#pragma unroll
    for (int pi = 0; pi < 5; ++pi) {
      if (pi == 4 && !five) break;
      const int pair = wave + 4 * pi;
      const int tap = pair >> 1, nt = pair & 1;
      int o;
      asm volatile("v_mov_b32 %0, %1" : "=v"(o) : "v"(4 * g * 288 + i16));
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          pdm_slab_store(&out[o + (mt * 16 + r) * 288 + tap * 32 + nt * 16], acc[pi][mt][r]);
    }
    PDM_STAMP(6);
    // then the band's dgrad tiles past the dgrad waves' 4 MD (last band / R = 12)
    const int ntile = (aown * IMG + 15) / 16;
#pragma unroll 1
    for (int t = 4 * L::MD + wave; t < ntile; t += 4) band_dgrad<R, 1, 2>(smem, t, aown, ka1, acc1);
  } else {
    // ===== conv2 dgrad over the band's own a1 rows: tiles wd + 4 k, k < MD =====
    band_dgrad<R, L::MD, 2>(smem, wave - 4, aown, ka1, acc1);
    if (tid == 256) PDM_STAMP_VAL(7, PDM_CLOCK());
  }
  __syncthreads();   // every wave is done with the dz2 / a1 images (RED aliases dz2)
  PDM_STAMP(8);
  float* red = reinterpret_cast<float*>(smem + L::RED);
  // conv1 weight/bias partials: waves 4-7 write slot wave & 3, waves 0-3 add theirs
  float* r1 = red + RED_DW1 + (wave & 3) * C1 * 16;
  if (wave >= 4) {
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) r1[(nt * 16 + 4 * g + r) * 16 + i16] = acc1[nt][r];
  }
  __syncthreads();
  if (wave < 4) {
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) r1[(nt * 16 + 4 * g + r) * 16 + i16] += acc1[nt][r];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float v = sum_xor32(sum_xor16(sum_xor8(db2p[j])));
    if (lane < 8) red[RED_DB2 + wave * C2 + lane * 8 + j] = v;
  }
  __syncthreads();
  if (tid < C2) {
    float s = 0.f;
    for (int w = 0; w < 8; ++w) s += red[RED_DB2 + w * C2 + tid];
    pdm_slab_store(&out[SL_DB2 + tid], s);
  } else if (tid >= 64 && tid < 64 + C1 * 10) {
    const int e = tid - 64;
    const int ci = e / 10, t = e - 10 * ci;
    float s = 0.f;
    for (int w = 0; w < 4; ++w) s += red[RED_DW1 + w * C1 * 16 + ci * 16 + t];
    pdm_slab_store(t < 9 ? &out[SL_DW1 + ci * 9 + t] : &out[SL_DB1 + ci], s);
  }
  PDM_STAMP(9);
}

}  // namespace

void launch_cnn_bwd_band(const __bf16* a1g, const __bf16* xng, const __bf16* dpool,
                         const uint8_t* pmask, const __bf16* w2t, int B, int bands, float* slab,
                         unsigned* xg_sync, hipStream_t st) {
  const int nblk = B * bands;
  switch (bands) {
    case 2:
      cnn_bwd_band_kernel<12><<<nblk, BTH, 0, st>>>(a1g, xng, dpool, pmask, w2t, slab, xg_sync);
      break;
    case 3:
      cnn_bwd_band_kernel<8><<<nblk, BTH, 0, st>>>(a1g, xng, dpool, pmask, w2t, slab, xg_sync);
      break;
    case 6:
      cnn_bwd_band_kernel<4><<<nblk, BTH, 0, st>>>(a1g, xng, dpool, pmask, w2t, slab, xg_sync);
      break;
    default:
      break;   // bind.cpp validates bands
  }
}

#ifdef PDM_STAMPS
void read_stamps_bwd_band(unsigned long long* host) {
  hipMemcpyFromSymbol(host, HIP_SYMBOL(pdm_stamps), sizeof(unsigned long long) * 256 * 16);
}
#else
void read_stamps_bwd_band(unsigned long long* host) {
  for (int i = 0; i < 256 * 16; ++i) host[i] = 0;
}
#endif
