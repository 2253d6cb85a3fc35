// North-star CNN forward on gfx950 (bf16 MFMA, fp32 accumulate).
//
//   cnn_fwd : one workgroup per image — gather the uint8 image by the sampler
//             index, normalise, conv1 (1->32, 3x3) + bias + ReLU on the VALU into an
//             LDS-resident NHWC bf16 image, then conv2 (32->64, 3x3) as an implicit
//             GEMM on mfma_f32_16x16x32_bf16 (one 3x3 tap == one K=32 step == all 32
//             input channels), with bias + ReLU + MaxPool2d(2) fused in-register:
//             the M rows of a 16-row tile are ordered (pooled pixel, window pos), so a
//             lane's 4 accumulator registers ARE one 2x2 window.  Writes the pooled
//             activations (fc1 input), a 1-byte mask per pooled value (0x80 | 1 << argmax
//             if positive, else 0),
//             and (training) a1 + the gathered bytes for the backward kernel.
//   fc1_fwd : split-K bf16 GEMM  part[s] = pool[:, Ks] . W1[:, Ks]^T  (fp32 slabs),
//             the reduction + bias + ReLU is fused into the head kernel.
//   cnn_head: fc1 split-K reduction + bias + ReLU, fc2, log-softmax/NLL, argmax,
//             and (training) the whole head backward: dlogits, fc2 weight/bias
//             partials, dh = dlogits.W2 * relu'(h) (bf16, + transposed copy for the
//             fc1 weight-gradient GEMM), fc1 bias partials; advances step counters.
#include "cnn_common.h"
#include "fc_carry.h"

// Translation-unit split: fc1_fwd and the head are compiled from fc1_fwd.hip / cnn_head.hip
// (this file with PDM_FWD_TU = 1 / 2) under their own scheduler flags (build.py
// FILE_FLAGS); this file's own compile holds cnn_fwd.  PDM_STAMPS builds keep everything
// here (one stamp buffer).
#ifndef PDM_FWD_TU
#define PDM_FWD_TU 0
#endif
#if defined(PDM_STAMPS)
#define PDM_WANT_FC1_FWD (PDM_FWD_TU == 0)
#define PDM_WANT_HEAD (PDM_FWD_TU == 0)
#else
#define PDM_WANT_FC1_FWD (PDM_FWD_TU == 1)
#define PDM_WANT_HEAD (PDM_FWD_TU == 2)
#endif
#define PDM_WANT_FWD_REST (PDM_FWD_TU == 0)

namespace {

using namespace cnn;

#if PDM_WANT_FWD_REST
// ---- cnn_fwd LDS carve (one static array; every offset 16-B aligned) ----
constexpr int FWD_THREADS = 512;
constexpr int F_X3 = 0;                       // bf16x4 x3[p] = x[p..p+2], 0  6272 B
constexpr int F_A1 = 6400;                    // bf16 a1 image              43264 B
constexpr int F_PS = F_A1 + P1 * 64;          // bf16 pooled [144][64]      18432 B
constexpr int F_MS = F_PS + PP * C2 * 2;      // u8 mask [144][64]          9216 B
constexpr int F_LUT = F_MS + PP * C2;         // bf16 normalize LUT [256]     512 B
constexpr int F_W = F_LUT + 512;              // fp32 w1 [288] | b1 [32] | b2 [64] 1536 B
constexpr int F_TOTAL = F_W + 1536;           // 79360 B -> 2 workgroups / CU
static_assert(2 * F_TOTAL <= 163840 && F_A1 % 128 == 0, "cnn_fwd LDS carve");

// CARRY: workgroups [B, B + FCC_WGS) run the previous step's fc1 update (fc_carry.h)
template <bool TRAIN, bool CARRY>
__global__ __launch_bounds__(FWD_THREADS, 2) void cnn_fwd_kernel(
    const uint8_t* __restrict__ images, const int32_t* __restrict__ labels,
    const int32_t* __restrict__ idx, int64_t nrow, const int64_t* __restrict__ ctr, const StepRows sr,
    const float* __restrict__ w1, const float* __restrict__ b1, const bf16* __restrict__ w2,
    const float* __restrict__ b2, bf16* __restrict__ pool, uint8_t* __restrict__ pmask,
    uint8_t* __restrict__ xg, int32_t* __restrict__ ylab, const FcUpdate fcc, int nconv) {
  __shared__ __attribute__((aligned(16))) char smem[F_TOTAL];
  static_assert(F_TOTAL >= FCC_LDS + 4, "carried fc1 update tiles fit the forward's LDS");
  if constexpr (CARRY) {
    if ((int)blockIdx.x >= nconv) {
      fc_carry_role(fcc, blockIdx.x - nconv, gridDim.x - nconv, smem);
      return;
    }
  }
  bf16x4* x3 = reinterpret_cast<bf16x4*>(smem + F_X3);
  char* a1s = smem + F_A1;
  bf16* ps = reinterpret_cast<bf16*>(smem + F_PS);
  uint8_t* ms = reinterpret_cast<uint8_t*>(smem + F_MS);

  const int img = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, i16 = lane & 15;
  PDM_STAMP(0);
  // 0. the small conv weights (w1, b1, b2: 384 floats) as 96 16-B loads by waves 4-5, staged
  // through LDS: per-lane gathers were 18 load instructions in every wave (144 per CU) that
  // queued in the texture unit in front of the conv1 phase.  Issued first: they do not
  // depend on the counter, so they land while the image's dependent chain is in flight.
  float4 wq = make_float4(0.f, 0.f, 0.f, 0.f);
  const int wt = tid - 256;
  if (wt >= 0 && wt < 96) {
    const float4* srcw = wt < 72 ? reinterpret_cast<const float4*>(w1) + wt
                         : wt < 80 ? reinterpret_cast<const float4*>(b1) + (wt - 72)
                                   : reinterpret_cast<const float4*>(b2) + (wt - 80);
    wq = *srcw;
  }
  __builtin_amdgcn_sched_barrier(0);
  // 1. gather: the dependent chain (counter -> index -> image row) is issued before
  // anything else so its latency is not queued behind the weight loads.
  // sample row: sampler index (idx), epoch-buffer row (ctr only) or plain row (eval)
  // (clamped to the row space: a counter driven past the epoch reads a valid row)
  const int64_t row_u = ctr ? step_row(sr, nrow, *ctr, img) : (int64_t)img;
  PDM_CHECK(row_u < nrow, "cnn_fwd sample row past the epoch", row_u, nrow);
  const int64_t row = min(row_u, nrow - 1);
  const int64_t src = idx ? (int64_t)idx[row] : row;
  // pixels 4 tid .. 4 tid + 3, and the next word's first two (the x3 entries need x[p + 2])
  uint32_t xw = 0, xn = 0;
  if (tid < 196) {
    xw = reinterpret_cast<const uint32_t*>(images + src * 784)[tid];
    xn = reinterpret_cast<const uint32_t*>(images + src * 784)[min(tid + 1, 195)];
  }
  // the label is a per-lane (vector) load consumed at the very end: a uniform-address
  // scalar load here made wave 0 wait for it (s_waitcnt lgkmcnt(0)) before issuing its
  // weight loads, delaying the first barrier by ~1.7k cycles
  int lab = 0;
  if (tid == 64) {
    int vz;   // a VGPR zero: keeps the load a vector load (a uniform address becomes s_load)
    asm volatile("v_mov_b32 %0, 0" : "=v"(vz));
    lab = labels[src + vz];
  }
  if (tid == 0) PDM_STAMP_VAL(8, PDM_CLOCK());   // image load issued
  // normalize through a 256-entry LUT (exact torchvision arithmetic -- two IEEE divisions --
  // once per byte value, not per pixel), built by the upper waves while the image is in
  // flight and BEFORE they queue their 18 KB of conv2 weight loads (the TA queue would
  // otherwise hold the LUT, and the barrier, back by ~2k cycles)
  bf16* lut = reinterpret_cast<bf16*>(smem + F_LUT);
  if (tid >= 256) lut[tid - 256] = to_bf16(pdm_normalize(tid - 256));
  float* wl = reinterpret_cast<float*>(smem + F_W);
  if (wt >= 0 && wt < 96) reinterpret_cast<float4*>(wl)[wt] = wq;
  __builtin_amdgcn_sched_barrier(0);
  __syncthreads();   // normalize LUT + conv weights ready (the image load keeps flying)

  // conv1 as D[co][pixel] = W1[co][tap] . X[tap][pixel] on mfma_f32_16x16x16_bf16:
  // A = weights (lane row co = i16; k = 4g + j is tap (ky = g, kx = j), zero for g = 3 or
  // j = 3), B = input patches (lane col = pixel): lane group g reads the x3 entry of pixel
  // p + 28 g, i.e. the row-ky triple x[p + 28 ky .. + 2] and a zero, in ONE 8-byte read;
  // bias is the initial accumulator.
  // (the bf16 conversion of the weights happens after the barriers: converting here made
  // every wave wait for its conv1 weight loads before the first barrier)
  float w1v[2][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)   // clamped unconditional load (no branch/wait)
      w1v[mt][j] = wl[(mt * 16 + i16) * 9 + 3 * min(g, 2) + min(j, 2)];
  f32x4 b1v[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) b1v[mt] = reinterpret_cast<const f32x4*>(wl + 288)[mt * 4 + g];
  if (tid < 196) {
    const bf16 v[6] = {lut[xw & 0xff], lut[(xw >> 8) & 0xff], lut[(xw >> 16) & 0xff],
                       lut[xw >> 24], lut[xn & 0xff], lut[(xn >> 8) & 0xff]};
    // (entries 782, 783 take two values past the image: finite, and only ever multiplied
    // into outputs of the virtual columns 26, 27, which are dropped)
#pragma unroll
    for (int i = 0; i < 4; ++i) x3[4 * tid + i] = bf16x4{v[i], v[i + 1], v[i + 2], bf16{}};
    if (TRAIN) st_ho<4>(reinterpret_cast<uint32_t*>(xg + (int64_t)img * 784) + tid, xw);
    if (tid == 0) PDM_STAMP_VAL(9, PDM_CLOCK());   // image landed
  }
  __syncthreads();
  PDM_STAMP(1);

  __builtin_amdgcn_sched_barrier(0);   // (hipcc hoists the conversion above the barrier)
  // conv2 B fragments for this wave's two n-tiles (co = 32*(wave&1) + 16*j + i16):
  // lane l holds B[k = ci = 8g + e][n = co] = w2[co][tap][ci].  Issued only now, once the
  // image has landed: these 18 KB per wave (147 KB per CU, all L2 hits) queued in the L2
  // ahead of the image's HBM request held the image back ~5k cycles; they stream in while
  // conv1 runs.
  const int nh = wave & 1;
  float b2r[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) b2r[j] = wl[320 + nh * 32 + j * 16 + i16];
  bf16x8 wb[9][2];
  // issued 3 per conv1 tile below: all 18 at once filled the CU's TA queue (8 waves x 18 KB)
  // and stalled every wave's conv1 issue behind them for ~2.3k cycles
  auto load_wb = [&](int f) {   // fragments 3f .. 3f+2 of the 18 (tap, n-tile) pairs
#pragma unroll
    for (int e = 3 * f; e < 3 * f + 3; ++e)
      wb[e >> 1][e & 1] = *reinterpret_cast<const bf16x8*>(   // fragment-major W2 (frag_pos)
          w2 + ((int64_t)((nh * 2 + (e & 1)) * 9 + (e >> 1)) * 64 + lane) * 8);
  };

  bf16x4 w1f[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int j = 0; j < 4; ++j) w1f[mt][j] = to_bf16(g < 3 && j < 3 ? w1v[mt][j] : 0.f);
  // 2. conv1 + bias + ReLU -> LDS a1 image; lane holds 4 consecutive channels of one
  // pixel -> one 8-byte LDS store per 16x16 tile.  Tiles of 16 "virtual pixels" V = 28y + x
  // of the 28-wide x image (x = 26, 27 and y >= 26 computed and dropped): V is the pixel's
  // own x index, x & 3 == lane & 3, so the operand reads are V + a per-lane tap offset and
  // the a1 store is (V - 2y) * 64 + a per-lane constant.  46 tiles (48 slots) over 8 waves.
  {
    constexpr int TPW = 6;
    const int rowg = IMG * (g < 3 ? g : 0);   // lane group 3: zero weights, any finite x
    // one 16-B store per lane and tile: lane pairs g, g ^ 1 swap channel halves
    // (cnn_common.h conv1_pair)
    const int a1c = (conv1_pair_chunk(g) ^ (i16 & 3)) << 4;
    // two rounds of 3 tiles: the 72 conv2 B-fragment registers are live here, and 6 tiles'
    // operands at once would push the kernel past 128 VGPRs (2 workgroups / CU)
#pragma unroll
    for (int h = 0; h < TPW; h += 3) {
    bf16x4 bx[TPW];
    int vv[TPW];
#pragma unroll
    for (int k = h; k < h + 3; ++k) {
      vv[k] = (wave + 8 * k) * 16 + i16;
      bx[k] = x3[min(vv[k], IMG * H1 - 1) + rowg];
    }
#pragma unroll
    for (int k = h; k < h + 3; ++k) {
      load_wb(k);
      const int y = vv[k] / IMG, x = vv[k] - y * IMG;
      const bool ok = y < H1 && x < H1;
      bf16x4 o[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(w1f[mt], bx[k], b1v[mt], 0, 0, 0);
        o[mt] = bf16x4{to_bf16(relu1(acc[0])), to_bf16(relu1(acc[1])),
                       to_bf16(relu1(acc[2])), to_bf16(relu1(acc[3]))};
      }
      // dropped pixels store into the (not yet used) pooled-output area: no branch
      const int dst = ok ? F_A1 + (vv[k] - 2 * y) * 64 + a1c : F_PS + lane * 16;
      *reinterpret_cast<uint4*>(smem + dst) = conv1_pair(o[0], o[1]);
    }
    }
  }
  __syncthreads();
  PDM_STAMP(2);

  // 3. conv2 implicit GEMM: 36 tiles of 16 rows (4 pooled pixels x 2x2 window) x 64 co;
  // wave w takes tiles (w>>1) + 4k for its two n-tiles.  Tile (py, px0) is wave-uniform
  // and px0 % 4 == 0, so the A-read swizzle term ((ox + kx) & 3) = ((2q + (s&1) + kx) & 3)
  // is a per-lane constant: the 9 per-tap lane offsets are precomputed.
  const int q = i16 >> 2, s = i16 & 3;
  const int lp = ((s >> 1) * H1 + 2 * q + (s & 1)) * 64;
  int aoff[9];
#pragma unroll
  for (int ky = 0; ky < 3; ++ky)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
      aoff[ky * 3 + kx] = lp + (ky * H1 + kx) * 64 + ((g ^ ((2 * q + (s & 1) + kx) & 3)) << 4);
  // wave pairs (w >> 1) 0, 1 take 10 tiles each, pairs 2, 3 take 8: a SIMD hosts waves w and
  // w + 4, and the issue arbiter favours the older one, so with 9 tiles each waves 4-7
  // finished ~1.3k cycles after waves 0-3, alone on their SIMDs
  const int pr = wave >> 1;
  const int tt0 = pr < 2 ? 10 * pr : 20 + 8 * (pr - 2), tt1 = tt0 + (pr < 2 ? 10 : 8);
  for (int tt = tt0; tt < tt1; ++tt) {
    const int py = tt / 3, px0 = 4 * (tt - py * 3);
    const char* tb = a1s + (2 * py * H1 + 2 * px0) * 64;
    bf16x8 a[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) a[t] = *reinterpret_cast<const bf16x8*>(tb + aoff[t]);
    f32x4 acc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[j] = f32x4{b2r[j], b2r[j], b2r[j], b2r[j]};
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[t], wb[t][j], acc[j], 0, 0, 0);
    // epilogue: lane holds the 2x2 window (4 regs) of pooled pixel pp for channel co
    const int pp = py * HP + px0 + g;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int co = nh * 32 + j * 16 + i16;
      // max-pool of relu = relu of the max, taken on the bit patterns (cnn_common.h relu1);
      // argmax: first window position (dy, dx row-major) holding it (only used when > 0)
      const int b0 = fbits(acc[j][0]), b1 = fbits(acc[j][1]), b2 = fbits(acc[j][2]);
      const int mb = max(max(max(b0, b1), b2), fbits(acc[j][3]));
      uint32_t oh = b2 == mb ? 4u : 8u;   // selects, last to first (no branches)
      oh = b1 == mb ? 2u : oh;
      oh = b0 == mb ? 1u : oh;
      const bool pos = mb > 0;
      ps[pp * C2 + co] = to_bf16(__builtin_bit_cast(float, max(mb, 0)));
      ms[pp * C2 + co] = (uint8_t)(pos ? 0x80u | oh : 0u);   // one-hot argmax
    }
  }
  PDM_STAMP(3);
  // per-wave conv2 end (waves 1-6 -> slots 10-15; blocks >= 64 only: the head overwrites
  // slots 10-15 of blocks 0-63)
  if ((threadIdx.x & 63) == 0 && wave >= 1 && wave <= 6) PDM_STAMP_VAL(9 + wave, PDM_CLOCK());
  __syncthreads();
  PDM_STAMP(4);

  // 4. coalesced write-out of pooled activations + mask
  uint4* pout = reinterpret_cast<uint4*>(pool + (int64_t)img * FEAT);
  for (int i = tid; i < FEAT * 2 / 16; i += FWD_THREADS) st_ho<4>(pout + i, reinterpret_cast<const uint4*>(ps)[i]);
  if (TRAIN) {
    uint4* mout = reinterpret_cast<uint4*>(pmask + (int64_t)img * FEAT);
    for (int i = tid; i < FEAT / 16; i += FWD_THREADS) st_ho<4>(mout + i, reinterpret_cast<const uint4*>(ms)[i]);
  }
  if (tid == 64) st_ho<4>(ylab + img, lab);
  PDM_STAMP(5);
}

#endif  // PDM_WANT_FWD_REST
#if PDM_WANT_FC1_FWD
// ---- fc1 forward: split-K GEMM, 32 MT rows x 128 cols per block ----
// KB = k-steps per load batch: 9 (288 k-steps = 32 batches; split factors dividing 32) or 3
// (96 batches: split factors up to 96, so B <= 64 can put W1 on ~256 CUs instead of 32-64)
// MT = 32-row m-tiles per block: 1, or 4 for large batches (B >= FC1_BIG_B): with 32-row
// tiles every block streams its whole K slice of W1 from L2 for 32 rows only (B = 8192,
// split-K 1: 256 x 2.4 MB = 604 MB of L2 reads, 80 us); 128-row tiles read W1 a quarter as
// often and leave the pool read from HBM as the bound
template <int KB, int MT>
__device__ __forceinline__ void fc1_fwd_body(const int w, const bf16* __restrict__ pool,
                                             const bf16* __restrict__ wf1,
                                             float* __restrict__ part, int B, int kchunk) {
  constexpr int FC1_KB = KB;
  constexpr int FC1_AROW = FC1_KB * 32 * 2 + 32;   // LDS bytes per staged pool row (padded)
  // XCD-aware mapping of the 1-D grid: workgroup w runs on XCD w % 8.  When the split
  // count is a multiple of 8, every XCD owns S/8 splits (1/8 of W1's K range, for all
  // m-tiles), so each XCD's L2 holds only its slice of W1 instead of all of it.
  constexpr int MR = 32 * MT;                      // rows per block
  const int mtiles = (B + MR - 1) / MR, S = FEAT / kchunk;
  int mtile, sidx;
  if (S % 8 == 0) {
    const int xcd = w % 8, loc = w / 8, spx = S / 8;
    sidx = xcd * spx + loc % spx;
    mtile = loc / spx;
  } else {
    sidx = w / mtiles;
    mtile = w % mtiles;
  }
  const int b0 = mtile * MR;
  const int kbeg = sidx * kchunk;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int rl = lane & 15, kg = (lane >> 4) * 8;
  const int n0 = wave * 32;
  // The pool tile (32 rows x 288 k per batch) is staged once per workgroup through LDS by
  // whole-line loads (it was read by each of the 4 waves, as 16 half lines per load);
  // rows are padded by 32 B (608 B / 224 B), so the A-fragment reads (16 rows x 16 B per
  // lane group) are bank-conflict-free (tools/lds_bank_model.py gfx950 ds_read_b128 lane
  // groups: 592 B rows were 2 passes per read, 40 % conflict cycles in the PMC table).  Rows past B read row
  // B-1 (valid data, outputs never stored).
  __shared__ __attribute__((aligned(16))) char at[MR * FC1_AROW];
  // W1 is fragment-major (kernels.h frag_pos): the 16 x 32 fragment (n-tile, k-step) is
  // one 1-KB block and this lane's 16 B sit at lane * 8 in it
  const bf16* pb0 = wf1 + ((int64_t)((n0 >> 4) * (FEAT / 32) + (kbeg >> 5)) * 64 + lane) * 8;
  const bf16* pb1 = pb0 + (int64_t)(FEAT / 32) * 512;
  f32x4 acc[2 * MT][2];
#pragma unroll
  for (int i = 0; i < 2 * MT; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int ACH = MR * FC1_KB * 32 * 2 / 16;   // 16-B chunks of the A tile (1152 at MT 1)
  // K in batches of FC1_KB steps: every operand load of a batch is issued before its
  // MFMAs (kchunk is a multiple of 32 * FC1_KB: the launch picks KB from the split factor)
  for (int kb = 0; kb < kchunk; kb += 32 * FC1_KB) {
    uint4 av[(ACH + 255) / 256];
#pragma unroll
    for (int u = 0; u < (ACH + 255) / 256; ++u) {
      const int c = min((int)threadIdx.x + 256 * u, ACH - 1);   // clamped: rewrites the last
      const int row = c / (FC1_KB * 4), col = c - row * (FC1_KB * 4);
      av[u] = *reinterpret_cast<const uint4*>(pool + (int64_t)min(b0 + row, B - 1) * FEAT + kbeg +
                                              kb + col * 8);
    }
    bf16x8 w0[FC1_KB], w1[FC1_KB];
#pragma unroll
    for (int i = 0; i < FC1_KB; ++i) {
      w0[i] = *reinterpret_cast<const bf16x8*>(pb0 + (kb / 32 + i) * 512);
      w1[i] = *reinterpret_cast<const bf16x8*>(pb1 + (kb / 32 + i) * 512);
    }
    __builtin_amdgcn_sched_barrier(0);   // all loads of the batch before the staging
#pragma unroll
    for (int u = 0; u < (ACH + 255) / 256; ++u) {
      const int c = min((int)threadIdx.x + 256 * u, ACH - 1);
      const int row = c / (FC1_KB * 4), col = c - row * (FC1_KB * 4);
      *reinterpret_cast<uint4*>(at + row * FC1_AROW + col * 16) = av[u];
    }
    __syncthreads();
    if constexpr (MT == 1) {
      bf16x8 a0[FC1_KB], a1[FC1_KB];
#pragma unroll
      for (int i = 0; i < FC1_KB; ++i) {
        a0[i] = *reinterpret_cast<const bf16x8*>(at + rl * FC1_AROW + (32 * i + kg) * 2);
        a1[i] = *reinterpret_cast<const bf16x8*>(at + (16 + rl) * FC1_AROW + (32 * i + kg) * 2);
      }
#pragma unroll
      for (int i = 0; i < FC1_KB; ++i) {
        acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[i], w0[i], acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[i], w1[i], acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[i], w0[i], acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[i], w1[i], acc[1][1], 0, 0, 0);
      }
    } else {
      // one k-step at a time: the 2 MT A fragments of step i, then their 4 MT MFMAs
#pragma unroll
      for (int i = 0; i < FC1_KB; ++i) {
        bf16x8 am[2 * MT];
#pragma unroll
        for (int m = 0; m < 2 * MT; ++m)
          am[m] = *reinterpret_cast<const bf16x8*>(at + (16 * m + rl) * FC1_AROW + (32 * i + kg) * 2);
#pragma unroll
        for (int m = 0; m < 2 * MT; ++m) {
          acc[m][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[m], w0[i], acc[m][0], 0, 0, 0);
          acc[m][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[m], w1[i], acc[m][1], 0, 0, 0);
        }
      }
    }
    __syncthreads();   // this batch's A reads are done before the next batch's staging
  }
  float* out = part + (int64_t)sidx * B * HID;
#pragma unroll
  for (int mt = 0; mt < 2 * MT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = b0 + 16 * mt + 4 * (lane >> 4) + r;
      if (row < B) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          st_ho<8>(&out[(int64_t)row * HID + n0 + 16 * nt + rl], acc[mt][nt][r]);
        }
      }
    }
}

template <int KB, int MT = 1>
__global__ __launch_bounds__(256, 2) void fc1_fwd_kernel(const bf16* __restrict__ pool,
                                                      const bf16* __restrict__ wf1,
                                                      float* __restrict__ part, int B, int kchunk) {
  fc1_fwd_body<KB, MT>(blockIdx.x, pool, wf1, part, B, kchunk);
}

#endif  // PDM_WANT_FC1_FWD
#if PDM_WANT_HEAD
// ---- head: fc1 reduce + bias + ReLU, fc2, CE, and (train) the head backward ----
// One wave per batch row (HEAD_ROWS = 4 rows per workgroup, B/4 workgroups): lane j owns
// hidden units 2j, 2j+1, so the fc2 logits are plain wave reductions and the split-K
// partial loads of a row are spread over a whole wave.

// workgroup blk of nblk (the head's grid)
template <bool TRAIN>
__device__ __forceinline__ void head_body(
    const int blk, const int nblk, const float* __restrict__ part, int S, int B,
    const float* __restrict__ bf1, const float* __restrict__ wf2, const float* __restrict__ bf2,
    const int32_t* __restrict__ ylab, bf16* __restrict__ dh, bf16* __restrict__ dht, int ldt,
    float* __restrict__ slab, double* __restrict__ metrics, int64_t* c0, int64_t* c1, unsigned* c2,
    float* __restrict__ dh32) {
  static_assert(HEAD_ROWS == 4, "one wave per row, 4 waves");
  __shared__ float hs[HEAD_ROWS][HID];
  __shared__ float dhs[HEAD_ROWS][HID];
  __shared__ float dls[HEAD_ROWS][NCLS];
  __shared__ float red[HEAD_ROWS][2];
  const int tid = threadIdx.x, r = tid >> 6, j = tid & 63;
  const int ngroups = (TRAIN ? ldt : B + HEAD_ROWS - 1) / HEAD_ROWS;
  // per-thread slab accumulators across this workgroup's row groups (train)
  float sw[5] = {0.f, 0.f, 0.f, 0.f, 0.f};   // dWfc2 entries tid + 256k
  float sx = 0.f;                             // dbfc2 / dbfc1 / loss / correct entry
  double el = 0.0, ec = 0.0;                  // eval metrics (thread 0)
  int en = 0;
  PDM_STAMP(10);   // head phases in slots 10-15 (cnn_fwd uses 0-9 of the same blocks)
  const float2 bias = reinterpret_cast<const float2*>(bf1)[j];
  // fc2 weights of this lane's two hidden units, loaded once up front and used by both the
  // logits and dh (reloading them for dh was another memory round trip in the chain)
  float2 w2v[NCLS];
#pragma unroll
  for (int c = 0; c < NCLS; ++c) w2v[c] = reinterpret_cast<const float2*>(wf2 + c * HID)[j];
  for (int grp = blk; grp < ngroups; grp += nblk) {
    const int row = grp * HEAD_ROWS + r;
    const bool valid = row < B;
    const int y = valid ? ylab[row] : 0;
    float2 h = bias;
    const int rc = min(row, B - 1);
    if (S == 32) {
      // the training split count at B <= 256: every partial load in flight at once (one
      // memory round trip -- the partials come from other XCDs' writes, ~1.4 us away)
      float2 u[32];
#pragma unroll
      for (int q = 0; q < 32; ++q)
        u[q] = *reinterpret_cast<const float2*>(part + ((int64_t)q * B + rc) * HID + 2 * j);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < 32; ++q) {
        h.x += u[q].x;
        h.y += u[q].y;
      }
    } else {
      // split-K partials in batches of 16 loads in flight (clamped addresses + selects),
      // summed in split order
      for (int s0 = 0; s0 < S; s0 += 16) {
        float2 u[16];
#pragma unroll
        for (int q = 0; q < 16; ++q)
          u[q] = *reinterpret_cast<const float2*>(part + ((int64_t)min(s0 + q, S - 1) * B + rc) * HID +
                                                  2 * j);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const bool on = s0 + q < S;
          h.x += on ? u[q].x : 0.f;
          h.y += on ? u[q].y : 0.f;
        }
      }
    }
    PDM_STAMP(11);
    h.x = valid ? fmaxf(h.x, 0.f) : 0.f;
    h.y = valid ? fmaxf(h.y, 0.f) : 0.f;

    float lg[NCLS];
#pragma unroll
    for (int c = 0; c < NCLS; ++c) lg[c] = wave_sum_dpp(fmaf(h.y, w2v[c].y, h.x * w2v[c].x)) + bf2[c];
    float prob[NCLS];
    int correct;
    const float loss = row_xent<NCLS>(lg, y, prob, correct);
    PDM_STAMP(12);
    if (j == 0) {
      red[r][0] = valid ? loss : 0.f;
      red[r][1] = valid ? (float)correct : 0.f;
    }

    if (TRAIN) {
      const float invB = 1.f / (float)B;
      float dl[NCLS];
#pragma unroll
      for (int c = 0; c < NCLS; ++c) dl[c] = valid ? (prob[c] - (c == y ? 1.f : 0.f)) * invB : 0.f;
      float2 dhv = make_float2(0.f, 0.f);
#pragma unroll
      for (int c = 0; c < NCLS; ++c) {
        dhv.x = fmaf(dl[c], w2v[c].x, dhv.x);
        dhv.y = fmaf(dl[c], w2v[c].y, dhv.y);
      }
      dhv.x = h.x > 0.f ? dhv.x : 0.f;
      dhv.y = h.y > 0.f ? dhv.y : 0.f;
      // row < ldt always: rows >= B write zeros (GEMM padding)
      if (dh32 != nullptr) {
        // fp32 step (cnn_f32.hip): dh row-major in fp32 (rows >= B are zero, GEMM padding)
        st_ho<8>(reinterpret_cast<float2*>(dh32 + (int64_t)row * HID) + j, dhv);
      } else {
        const bf16x2 o = {to_bf16(dhv.x), to_bf16(dhv.y)};
        // both copies fragment-major (kernels.h frag_pos), the layouts fc1_bwd's dW (dh^T: m =
        // hidden unit, k = batch row) and dX (dh: m = batch row, k = hidden unit) tiles load
        st_ho<8>(&dht[frag_pos(2 * j, row, ldt)], o[0]);
        st_ho<8>(&dht[frag_pos(2 * j + 1, row, ldt)], o[1]);
        st_ho<8>(reinterpret_cast<bf16x2*>(dh + frag_pos(row, 2 * j, HID)), o);
      }
      reinterpret_cast<float2*>(hs[r])[j] = h;
      reinterpret_cast<float2*>(dhs[r])[j] = dhv;
      if (j == 0) {
#pragma unroll
        for (int c = 0; c < NCLS; ++c) dls[r][c] = dl[c];
      }
    }
    PDM_STAMP(13);
    __syncthreads();
    if (TRAIN) {
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const int e = tid + 256 * k;
        const int c = e / HID, n = e - c * HID;
        float a = sw[k];
#pragma unroll
        for (int i = 0; i < HEAD_ROWS; ++i) a = fmaf(dls[i][c], hs[i][n], a);
        sw[k] = a;
      }
      if (tid < NCLS) {
        for (int i = 0; i < HEAD_ROWS; ++i) sx += dls[i][tid];
      } else if (tid >= 16 && tid < 16 + HID) {
        for (int i = 0; i < HEAD_ROWS; ++i) sx += dhs[i][tid - 16];
      } else if (tid == 254 || tid == 255) {
        for (int i = 0; i < HEAD_ROWS; ++i) sx += red[i][tid - 254];
      }
    } else if (tid == 0) {
      for (int i = 0; i < HEAD_ROWS; ++i) {
        el += red[i][0];
        ec += red[i][1];
        en += (grp * HEAD_ROWS + i < B);
      }
    }
    PDM_STAMP(14);
    __syncthreads();   // LDS is rewritten by the next row group
  }
  if (!TRAIN) {
    if (tid == 0) {
      atomicAdd(&metrics[0], el);
      atomicAdd(&metrics[1], ec);
      atomicAdd(&metrics[2], (double)en);
    }
    return;
  }
  float* out = slab + (int64_t)blk * HEAD_SLAB;
#pragma unroll
  for (int k = 0; k < 5; ++k) st_ho<8>(&out[tid + 256 * k], sw[k]);
  if (tid < NCLS) st_ho<8>(&out[NCLS * HID + tid], sx);
  else if (tid >= 16 && tid < 16 + HID) st_ho<8>(&out[NCLS * HID + NCLS + tid - 16], sx);
  else if (tid == 254 || tid == 255) st_ho<8>(&out[HEAD_SLAB - 2 + (tid - 254)], sx);
  if (blk == 0 && tid == 0) {          // pdm_bump_counters for the head's first workgroup
    if (c0) *c0 += 1;
    if (c1) *c1 += 1;
    if (c2) *c2 += 1;
  }
  PDM_STAMP(15);
}


template <bool TRAIN>
__global__ __launch_bounds__(256) void cnn_head_kernel(
    const float* __restrict__ part, int S, int B, const float* __restrict__ bf1,
    const float* __restrict__ wf2, const float* __restrict__ bf2, const int32_t* __restrict__ ylab,
    bf16* __restrict__ dh, bf16* __restrict__ dht, int ldt, float* __restrict__ slab,
    double* __restrict__ metrics, int64_t* c0, int64_t* c1, unsigned* c2, float* __restrict__ dh32) {
  head_body<TRAIN>(blockIdx.x, gridDim.x, part, S, B, bf1, wf2, bf2, ylab, dh, dht, ldt, slab,
                   metrics, c0, c1, c2, dh32);
}

#endif  // PDM_WANT_HEAD
}  // namespace

#if PDM_WANT_FWD_REST
void launch_cnn_fwd(const uint8_t* images, const int32_t* labels, const int32_t* idx,
                    int64_t nrow, const int64_t* ctr, StepRows sr, int B, const float* w1, const float* b1,
                    const __bf16* w2, const float* b2, __bf16* pool, uint8_t* pmask, uint8_t* xg,
                    int32_t* ylab, const FcUpdate* fcc, hipStream_t st) {
  if (fcc != nullptr) {        // training only (the caller carries an update between steps)
    cnn_fwd_kernel<true, true><<<B + FCC_WGS, FWD_THREADS, 0, st>>>(
        images, labels, idx, nrow, ctr, sr, w1, b1, w2, b2, pool, pmask, xg, ylab, *fcc, B);
    return;
  }
  const FcUpdate none{};
  if (xg != nullptr)
    cnn_fwd_kernel<true, false><<<B, FWD_THREADS, 0, st>>>(images, labels, idx, nrow, ctr, sr, w1, b1,
                                                           w2, b2, pool, pmask, xg, ylab, none, B);
  else
    cnn_fwd_kernel<false, false><<<B, FWD_THREADS, 0, st>>>(images, labels, idx, nrow, ctr, sr, w1,
                                                            b1, w2, b2, pool, pmask, xg, ylab, none, B);
}

#endif
#if PDM_WANT_FC1_FWD
void launch_fc1_fwd(const __bf16* pool, const __bf16* wf1, float* part, int B, int splitk,
                    hipStream_t st) {
  if (B >= FC1_BIG_B) {                // 128-row blocks, 3-k-step batches (kernels.h)
    dim3 grid(((B + 127) / 128) * splitk);
    fc1_fwd_kernel<3, 4><<<grid, 256, 0, st>>>(pool, wf1, part, B, FEAT / splitk);
    return;
  }
  dim3 grid(((B + 31) / 32) * splitk);
  if (32 % splitk == 0)
    fc1_fwd_kernel<9><<<grid, 256, 0, st>>>(pool, wf1, part, B, FEAT / splitk);
  else
    fc1_fwd_kernel<3><<<grid, 256, 0, st>>>(pool, wf1, part, B, FEAT / splitk);
}

#endif
#if PDM_WANT_HEAD
void launch_cnn_head(const float* part, int splitk, int B, const float* bf1, const float* wf2,
                     const float* bf2, const int32_t* ylab, bool train, __bf16* dh, __bf16* dht,
                     int ldt, float* slab, double* metrics, int64_t* c0, int64_t* c1,
                     unsigned* c2, float* dh32, hipStream_t st) {
  const int groups = (train ? ldt : B + HEAD_ROWS - 1) / HEAD_ROWS;
  const int nblk = cnn_head_blocks(groups);
  if (train)
    cnn_head_kernel<true><<<nblk, 256, 0, st>>>(part, splitk, B, bf1, wf2, bf2, ylab, dh, dht, ldt,
                                                slab, metrics, c0, c1, c2, dh32);
  else
    cnn_head_kernel<false><<<nblk, 256, 0, st>>>(part, splitk, B, bf1, wf2, bf2, ylab, dh, dht,
                                                 ldt, slab, metrics, c0, c1, c2, dh32);
}

int cnn_head_blocks(int groups) { return groups < CNN_HEAD_MAX_BLOCKS ? groups : CNN_HEAD_MAX_BLOCKS; }

#endif  // PDM_WANT_HEAD
#if PDM_WANT_FWD_REST
#ifdef PDM_STAMPS
void read_stamps_fwd(unsigned long long* host) {
  hipMemcpyFromSymbol(host, HIP_SYMBOL(pdm_stamps), sizeof(unsigned long long) * 256 * 16);
}
#else
void read_stamps_fwd(unsigned long long* host) {
  for (int i = 0; i < 256 * 16; ++i) host[i] = 0;
}
#endif
#endif  // PDM_WANT_FWD_REST
