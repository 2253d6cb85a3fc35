// North-star CNN backward on gfx950 (bf16 MFMA, fp32 accumulate).
//
//   fc1_bwd    : three block roles in one launch
//                  dW1 tiles : gW1[n][k] = sum_b dh[b][n] * pool[b][k]   (K = batch; the
//                              pool tile is staged in LDS and read transposed with
//                              ds_read_b64_tr_b16 as the MFMA B operand)
//                  dX tiles  : dpool[b][k] = sum_n dh[b][n] * W1[n][k]   (W1^T bf16 copy
//                              written by the optimizer kernel)
//                  1 block   : fixed-order reduction of the head slabs -> fc2 W/b and fc1
//                              bias gradients + train metrics
//                After this kernel gradient bucket 0 (fc2 + fc1) is complete.
//   cnn_bwd    : 512 threads per image group.  Loads a1 and expands
//                dz2 = maxpool^-1(dpool) * relu'(conv2) into LDS (72 KB), then
//                  waves 0-3 : conv2 weight gradient, dW2[co][tap][ci] += dz2^T . a1(tap)
//                              (both operands read with ds_read_b64_tr_b16), accumulators
//                              persist across the block's images
//                  waves 4-7 : conv2 input gradient da1 = sum_tap dz2(-tap) . W2(tap) with
//                              the 36 W2^T fragments in registers, fused with relu'(a1),
//                              the conv1 weight gradient and the conv1 bias gradient
//                and writes one fp32 slab per block (no atomics, deterministic).
//   conv_reduce: fixed-order slab sum -> conv gradients (bucket 1 complete).
#include "cnn_common.h"
#include "optim_common.h"
#include "xgmi.h"

#include <cstdlib>
#include <type_traits>
#include <utility>

// Translation-unit split: fc1_bwd is compiled from fc1_bwd.hip (this file with
// PDM_FC1_BWD_TU = 1) under its own scheduler flags (build.py FILE_FLAGS); this file's own
// compile holds the rest.  PDM_STAMPS builds keep everything here (one stamp buffer).
#ifndef PDM_FC1_BWD_TU
#define PDM_FC1_BWD_TU 0
#endif
#if defined(PDM_STAMPS)
#define PDM_WANT_FC1_BWD (PDM_FC1_BWD_TU == 0)
#define PDM_WANT_REST (PDM_FC1_BWD_TU == 0)
#else
#define PDM_WANT_FC1_BWD (PDM_FC1_BWD_TU == 1)
#define PDM_WANT_REST (PDM_FC1_BWD_TU == 0)
#endif

namespace {

using namespace cnn;


#if PDM_WANT_FC1_BWD
// ------------------------------------------------------------------ fc1_bwd
// diagnostic stamps (PDM_STAMPS builds; tools/stamps_fc.py): dX tile t -> row t, slots 0-3;
// dW tile b -> row b, slots 8-13 (cnn_bwd overwrites them, so fc1_bwd is stamped alone)
#ifdef PDM_STAMPS
#define FC_STAMP(row, slot)                                                         \
  do {                                                                              \
    if (threadIdx.x == 0 && (row) < 256)                                            \
      pdm_stamps[(row) * 16 + (slot)] = __builtin_amdgcn_s_memtime();              \
  } while (0)
#else
#define FC_STAMP(row, slot) do { } while (0)
#endif
// dW tile: 64 feature columns x 64 * DW_MT hidden rows (each of the 4 waves owns DW_MT 16-row
// m-tiles).  DW_MT = 1 splits the 128 hidden rows over two workgroups (288 tiles): half the
// MFMA work and half the fused update's epilogue per workgroup, twice the workgroups.
#ifndef PDM_DW_MT
#define PDM_DW_MT 1
#endif
constexpr int DW_MT = PDM_DW_MT;
static_assert(DW_MT == 1 || DW_MT == 2, "dW tile: 64 or 128 hidden rows");
constexpr int DW_FT = FEAT / 64;                      // 144 feature tiles
constexpr int DW_TILES = DW_FT * (2 / DW_MT);         // 144 or 288
constexpr int DWC = 128;             // dW1 batch rows staged per LDS round
constexpr int DX_COLS = 384;         // dX tile: 32 batch rows x 384 features per workgroup
constexpr int DX_TILES = FEAT / DX_COLS;   // 24 = 8 XCDs x 3
constexpr int DX_FT = DX_COLS / 64;        // 16-feature sub-tiles per wave (6)
constexpr int NXCD = 8;              // MI355X: workgroups are dealt round-robin to 8 XCDs
static_assert(DX_TILES % NXCD == 0 && DW_TILES % NXCD == 0, "XCD-aware tile mapping");
constexpr int HR_BLOCKS = (HEAD_SLAB + 63) / 64;   // head-slab reduction workgroups (23)

// [rows][128 B] pool tile.  A transposed read's 32-lane half touches rows {0-3, 8-11} (+4)
// of a 16-row block at one 32-B column chunk each: rows of equal parity share banks, so the
// chunk is XORed with row bits 1 and 3 -> the 8 chunks cover all 64 banks once
// (tools/lds_bank_model.py; the bit-3-only swizzle was 2 passes per read)
__device__ __forceinline__ int tile_off(int row, int byte) {
  return row * 128 + (byte ^ ((((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 5));
}

// Two waves per SIMD, i.e. two workgroups per CU (<= 256 registers per lane; 162 VGPRs, no
// spill): the 503 workgroups at B = 256 (288 dW + 192 dX + 23 head-slab) run in one round
// instead of two.  fc1_bwd 10.0 -> 9.6 us, the B = 256 step 54.9 -> 53.9 us (interleaved A/B,
// profiles/r5/fc1bwd_wpe2).
__global__ __launch_bounds__(256, 2) void fc1_bwd_kernel(
    const bf16* __restrict__ dh, const bf16* __restrict__ dht, int ldt,
    const bf16* __restrict__ pool, const bf16* __restrict__ wf1t, int B, float* __restrict__ gwf1,
    bf16* __restrict__ dpool, const float* __restrict__ head_slab, int head_blocks,
    float* __restrict__ gwf2, float* __restrict__ gbf2, float* __restrict__ gbf1,
    double* __restrict__ metrics, int bid_offset, const FcUpdate fcu) {
  // [0, 16 KB): the pool tile, then the fused update's bf16 W1 fragments; [16 KB, 32 KB):
  // the fused update's W1^T fragments (double-buffered W1^T only)
  __shared__ __attribute__((aligned(16))) char tile[2 * DWC * 128];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, pq = i16 & 3;
  const int nd = (ldt / 32) * DX_TILES;
  const int bid = blockIdx.x + bid_offset;

  if (bid < DW_TILES) {
    // ---- dW1 tile: 64 * DW_MT hidden rows (from n0) x 64 feature columns, K = batch ----
    // The batch is consumed in chunks of DWC rows: the whole chunk (pool rows and the
    // dh^T A fragments) is loaded with every load in flight at once, and the next chunk's
    // loads are issued before the current chunk's MFMAs.  The two hidden halves of a
    // feature tile (DW_MT = 1) are DW_FT workgroups apart: the same XCD, one L2 copy of the
    // pool tile they both read.
    const int k0 = (bid % DW_FT) * 64, n0 = (bid / DW_FT) * 64 * DW_MT;
    FC_STAMP(bid, 8);
    f32x4 acc[DW_MT][4];
#pragma unroll
    for (int i = 0; i < DW_MT; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int srow = tid >> 3, sch = tid & 7;
    uint4 pv[DWC / 32];
    bf16x8 a[DW_MT][DWC / 32];
    auto load_chunk = [&](int c0) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < DWC / 32; ++j) {
        const int row = c0 + srow + 32 * j;
        // clamped load + select: rows past B are zero (their dh rows are zero too, but
        // stale pool memory could hold non-finite bit patterns)
        const uint4 v = *reinterpret_cast<const uint4*>(pool + (int64_t)min(row, B - 1) * FEAT +
                                                        k0 + sch * 8);
        pv[j] = row < B ? v : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int mt = 0; mt < DW_MT; ++mt)
#pragma unroll
        for (int kk = 0; kk < DWC / 32; ++kk)
          a[mt][kk] = *reinterpret_cast<const bf16x8*>(   // fragment-major dh^T (frag_pos)
              dht + ((int64_t)((n0 / 16 + wave * DW_MT + mt) * (ldt / 32) +
                               (min(c0 + 32 * kk, ldt - 32) >> 5)) * 64 + lane) * 8);
    };
    load_chunk(0);
    // fused update (fcu.kind >= 0): this tile's fp32 weights and momentum, issued behind the
    // first chunk so they have landed by the epilogue
    // (with the learning rate and step count: loaded in the epilogue they were one more
    // memory round trip on its critical path)
    float fpv[DW_MT][4][4], fmv[DW_MT][4][4];
    double fc_lr = 0.0;
    int64_t fc_t = 0;
    if (fcu.kind >= 0) {
      fc_lr = *fcu.lr;
      fc_t = *fcu.step;
#pragma unroll
      for (int mt = 0; mt < DW_MT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) {
            const int64_t q = (int64_t)(n0 + wave * 16 * DW_MT + mt * 16 + 4 * g + r) * FEAT + k0 +
                              16 * nt + i16;
            fpv[mt][r][nt] = fcu.p[q];
            fmv[mt][r][nt] = fcu.m[q];
          }
    }
    for (int c0 = 0; c0 < ldt; c0 += DWC) {
      __syncthreads();   // previous chunk's tile reads are done
#pragma unroll
      for (int j = 0; j < DWC / 32; ++j)
        *reinterpret_cast<uint4*>(tile + tile_off(srow + 32 * j, sch * 16)) = pv[j];
      bf16x8 ac[DW_MT][DWC / 32];
#pragma unroll
      for (int mt = 0; mt < DW_MT; ++mt)
#pragma unroll
        for (int kk = 0; kk < DWC / 32; ++kk) ac[mt][kk] = a[mt][kk];
      __syncthreads();
      FC_STAMP(bid, c0 == 0 ? 9 : 10);   // chunk landed in LDS
      if (c0 + DWC < ldt) load_chunk(c0 + DWC);
      __builtin_amdgcn_sched_barrier(0);   // next chunk's loads stay ahead of this chunk's MFMAs
      const int nk = min(DWC / 32, (ldt - c0) / 32);
#pragma unroll
      for (int kk = 0; kk < DWC / 32; ++kk) {
        if (kk < nk) {
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) {
            const s16x4 lo = lds_tr16(tile + tile_off(32 * kk + 8 * g + q, 32 * nt + 8 * pq));
            const s16x4 hi = lds_tr16(tile + tile_off(32 * kk + 8 * g + 4 + q, 32 * nt + 8 * pq));
            const bf16x8 bv = cat_tr(lo, hi);
#pragma unroll
            for (int mt = 0; mt < DW_MT; ++mt)
              acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ac[mt][kk], bv, acc[mt][nt], 0, 0, 0);
          }
        }
      }
    }
    FC_STAMP(bid, 11);
    if (fcu.kind < 0 || fcu.store_grad) {
#pragma unroll
      for (int mt = 0; mt < DW_MT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = n0 + wave * 16 * DW_MT + mt * 16 + 4 * g + r;
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) st_ho<2>(&gwf1[(int64_t)n * FEAT + k0 + 16 * nt + i16], acc[mt][nt][r]);
        }
    }
    if (fcu.kind >= 0) {
      // world size 1 (kernels.h FcUpdate): the SGD-momentum update of this tile, from the
      // gradient still in registers; writes the fp32 weight, the momentum and the bf16 [n][k]
      // copy (the transposed copy, which this launch's dX tiles are reading, is re-derived
      // by the optimizer launch).  Same op order as the optimizer kernel: same bits.
      using namespace optim_detail;
      const Hyper h = make_hyper<OPT_SGD>(fcu, fc_lr, fc_t);
      // the bf16 copy is fragment-major (fc1_fwd's B operand, kernels.h frag_pos): this tile
      // is 4 DW_MT n-tiles x 2 k-steps of 1-KB blocks, assembled in LDS and stored as 16-B
      // chunks
      __syncthreads();   // every wave's last reads of the pool tile are done
      bf16* fr = reinterpret_cast<bf16*>(tile);
      // W1^T fragments of this tile (kernels.h shadow_t_pos, m = feature, k = hidden): for
      // each of the 4 16-feature m-frags, the 2 DW_MT 32-row k-frags of this tile, 1 KB each
      // (one contiguous range per m-frag); a lane's 4 rows r are 4 consecutive bf16 (one 8-B
      // store, 512 B contiguous per wave store)
      bf16* frt = reinterpret_cast<bf16*>(tile + DWC * 128);
#pragma unroll
      for (int mt = 0; mt < DW_MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          bf16 pt[4];
          const int nl0 = wave * 16 * DW_MT + mt * 16 + 4 * g;   // tile-local row of r = 0
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int nl = nl0 + r, kl = 16 * nt + i16;
            const int64_t q = (int64_t)(n0 + nl) * FEAT + k0 + kl;
            float m = fmv[mt][r][nt], v = 0.f;
            const float p = update<OPT_SGD>(fpv[mt][r][nt], acc[mt][nt][r], m, v, h, fcu.grad_scale);
            st_ho<2>(&fcu.p[q], p);
            st_ho<2>(&fcu.m[q], m);
            pt[r] = to_bf16(p);
            fr[(((nl >> 4) * 2 + (kl >> 5)) * 64 + ((kl >> 3) & 3) * 16 + (nl & 15)) * 8 + (kl & 7)] = pt[r];
          }
          if (fcu.shadow_t_next != nullptr)
            *reinterpret_cast<bf16x4*>(frt + (((nt * (2 * DW_MT) + (nl0 >> 5)) * 64 +
                                               (((nl0 >> 4) & 1) * 2 + (g >> 1)) * 16 + i16) * 8 +
                                              (g & 1) * 4)) = bf16x4{pt[0], pt[1], pt[2], pt[3]};
        }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < 2 * DW_MT; ++u) {
        const int c = tid + 256 * u, blk = c >> 6;   // blk = local n-tile * 2 + k-step
        st_ho<2>(reinterpret_cast<uint4*>(fcu.shadow + ((int64_t)((n0 / 16 + (blk >> 1)) * (FEAT / 32) +
                                                                   (k0 >> 5) + (blk & 1)) * 64 + (c & 63)) * 8),
                 reinterpret_cast<const uint4*>(fr)[c]);
      }
      if (fcu.shadow_t_next != nullptr) {
        // local block lb = m-frag * 2 DW_MT + local k-frag -> global block
        // (k0 / 16 + m-frag) * (HID / 32) + n0 / 32 + local k-frag, 64 uint4 each
#pragma unroll
        for (int u = 0; u < 2 * DW_MT; ++u) {
          const int c = tid + 256 * u, lb = c >> 6;
          const int64_t gb = (int64_t)(k0 / 16 + lb / (2 * DW_MT)) * (HID / 32) + n0 / 32 +
                             lb % (2 * DW_MT);
          st_ho<2>(reinterpret_cast<uint4*>(fcu.shadow_t_next) + gb * 64 + (c & 63),
                   reinterpret_cast<const uint4*>(frt)[c]);
        }
      }
    }
    FC_STAMP(bid, 13);
    return;
  }

  if (bid < DW_TILES + nd) {
    // ---- dX tile: 32 batch rows x 384 features, K = 128 hidden ----
    // dpool[b][f] = dh[b][:] . W1^T[f][:] (A = dh, B = W1^T fragments): a lane holds 4 rows
    // of one feature, so a wave's store covers 4 rows x 32 B.  (The transposed product with
    // one 8-byte store per lane spread each store over 16 rows: 0.5 us slower.)  Each wave
    // owns 96 features (6 sub-tiles) x 32 rows with every operand load (24 W1^T + 8 dh
    // fragments) issued up front: at B = 256 the 192 tiles are one round of workgroups, each
    // a single load burst (the earlier 576 tiles of 128 features ran ~2.25 latency-bound
    // rounds per CU).  XCD-aware: workgroup t runs on XCD t % 8 (DW_TILES is a multiple of
    // 8), and every XCD owns 1/8 of the feature range, so each XCD's L2 holds only its 1/8
    // of W1^T.
    const int t = bid - DW_TILES;
    FC_STAMP(t, 0);
    constexpr int TPX = DX_TILES / NXCD;                 // feature tiles per XCD
    const int xcd = t % NXCD, loc = t / NXCD;
    const int b0 = (loc / TPX) * 32;
    const int f0 = (xcd * TPX + loc % TPX) * DX_COLS + wave * (16 * DX_FT);
    bf16x8 wa[DX_FT][HID / 32], hb[2][HID / 32];
#pragma unroll
    for (int ks = 0; ks < HID / 32; ++ks) {
#pragma unroll
      for (int bt = 0; bt < 2; ++bt)
        hb[bt][ks] = *reinterpret_cast<const bf16x8*>(
            dh + ((int64_t)(((b0 >> 4) + bt) * (HID / 32) + ks) * 64 + lane) * 8);   // frag_pos
#pragma unroll
      for (int ft = 0; ft < DX_FT; ++ft)
        wa[ft][ks] = *reinterpret_cast<const bf16x8*>(     // fragment-major W1^T (kernels.h)
            wf1t + ((int64_t)(((f0 >> 4) + ft) * (HID / 32) + ks) * 64 + lane) * 8);
    }
    // keep every load above this point: the scheduler would otherwise interleave them
    // with the MFMAs behind per-load waits
    __builtin_amdgcn_sched_barrier(0);
    FC_STAMP(t, 1);
    f32x4 acc[DX_FT][2];
#pragma unroll
    for (int ft = 0; ft < DX_FT; ++ft)
#pragma unroll
      for (int bt = 0; bt < 2; ++bt) acc[ft][bt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < HID / 32; ++ks)
#pragma unroll
      for (int ft = 0; ft < DX_FT; ++ft)
#pragma unroll
        for (int bt = 0; bt < 2; ++bt)
          acc[ft][bt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hb[bt][ks], wa[ft][ks], acc[ft][bt], 0, 0, 0);
    FC_STAMP(t, 2);
    // D[b][f]: lane (g, i16) holds rows b = 4g + r of feature i16: a store covers 4 rows x 32 B
#pragma unroll
    for (int bt = 0; bt < 2; ++bt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = b0 + bt * 16 + 4 * g + r;
        if (row < B) {
#pragma unroll
          for (int ft = 0; ft < DX_FT; ++ft)
            st_ho<2>(&dpool[(int64_t)row * FEAT + f0 + ft * 16 + i16], to_bf16(acc[ft][bt][r]));
        }
      }
    FC_STAMP(t, 3);
    return;
  }

  // ---- head slab reduction: HR_BLOCKS workgroups x 64 slab columns x 4 slab groups ----
  {
    __shared__ float rs[4][64];
    __shared__ double rd[4][64];
    const int e = (bid - DW_TILES - nd) * 64 + (tid & 63), grp = tid >> 6;
    const int ec = min(e, HEAD_SLAB - 1);
    float s = 0.f;
    double sd = 0.0;
    for (int j0 = grp; j0 < head_blocks; j0 += 4 * 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = head_slab[(int64_t)min(j0 + 4 * u, head_blocks - 1) * HEAD_SLAB + ec];
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float x = (j0 + 4 * u < head_blocks) ? v[u] : 0.f;
        s += x;
        sd += (double)x;
      }
    }
    rs[grp][tid & 63] = s;
    rd[grp][tid & 63] = sd;
    __syncthreads();
    if (tid < 64 && e < HEAD_SLAB) {
      s = ((rs[0][tid] + rs[1][tid]) + rs[2][tid]) + rs[3][tid];
      sd = ((rd[0][tid] + rd[1][tid]) + rd[2][tid]) + rd[3][tid];
      if (e < NCLS * HID) gwf2[e] = s;
      else if (e < NCLS * HID + NCLS) gbf2[e - NCLS * HID] = s;
      else if (e < NCLS * HID + NCLS + HID) gbf1[e - NCLS * HID - NCLS] = s;
      else if (e == HEAD_SLAB - 2) { metrics[0] += sd; metrics[2] += (double)B; }
      else metrics[1] += sd;
    }
  }
}

#endif  // PDM_WANT_FC1_BWD
#if PDM_WANT_REST

// ------------------------------------------------------------------ cnn_bwd
// LDS carve (one static array, 163,200 B -> 1 workgroup / CU):
//   x    bf16 [28*28] + zero pad                                     1600
//   a1   26x26 px x 32 ch bf16 (a1_off swizzle)                     43264
//   zero 512 B: target of the dgrad reads whose dz2 row is outside the image
//   dz2  24 rows x 26 px x 64 ch bf16; px 24, 25 of every row are zero, so a dgrad read
//        that runs past either column edge lands on a zero pixel (col -1 of row r is px 25
//        of row r-1; row -1 is the zero block)                        79872
//   W2^T [tap][ci][co] bf16, 16-B chunk c of row (tap, ci) stored at c ^ ((ci >> 1) & 7)
//        (conflict-free B-fragment reads)                             36864
//   lut  bf16 of the normalised pixel value for each byte               512
//   red  fp32 reduction scratch, aliases a1 (only used after the last image)
constexpr int BWD_THREADS = 512;
constexpr int DS = 26;                          // dz2 row stride in pixels (24 + 2 zero)
constexpr int B_XS = 0;
constexpr int B_A1 = 1664;
constexpr int B_Z0 = B_A1 + P1 * 64;            // 44928
constexpr int B_DZ = B_Z0 + 512;                // 45440 (128-B aligned)
constexpr int B_W2 = B_DZ + H2 * DS * 128;      // 125312
constexpr int B_LUT = B_W2 + 9 * C1 * C2 * 2;   // normalize LUT: 256 x bf16    512
constexpr int B_SPARE = B_LUT + 512;           // 512 B target of dropped conv1 stores
constexpr int B_TOTAL = B_SPARE + 512;          // 163200
constexpr int B_RED = B_A1;
constexpr int RED_DB2 = 0;                      // [8 waves][64]
constexpr int RED_DW1 = RED_DB2 + 8 * C2;       // [4 waves][32 ci][16 taps] (tap 9 = bias)
constexpr int RED_N = RED_DW1 + 4 * C1 * 16;    // 2560 floats
static_assert(B_TOTAL <= 163840 && RED_N * 4 <= P1 * 64, "cnn_bwd LDS carve");
static_assert(B_A1 % 128 == 0 && B_Z0 % 128 == 0 && B_DZ % 128 == 0 && B_W2 % 128 == 0,
              "128-B aligned images (the dgrad address ORs a 7-bit swizzle into them)");
constexpr int SL_DB2 = C2 * 9 * C1;             // 18432
constexpr int SL_DW1 = SL_DB2 + C2;             // 18496
constexpr int SL_DB1 = SL_DW1 + C1 * 9;         // 18784
static_assert(SL_DB2 == CNN_CONV_SLAB_DB2 && SL_DW1 == CNN_CONV_SLAB_DW1 &&
              SL_DB1 == CNN_CONV_SLAB_DB1 && SL_DB1 + C1 == CNN_CONV_SLAB, "conv slab layout");

// dz2 image: pixel (r, c), 16-B chunk ch at ((ch + 4r + c) & 7) -- a rotation, so the
// dgrad read address is two VALU ops per (tile, tap) (see dgrad_pass), and one step along
// the dgrad's 28-wide virtual pixel grid (including 27 -> 0 of the next row: 4 - 27 = 1
// mod 8) always advances the rotation by 1.  Conflict-free for the dgrad ds_read_b128 rows
// and the scatter's window writes, 1.67-way for the wgrad ds_read_b64_tr_b16 columns
// (tools/lds_bank_model.py).
constexpr int W2_CHUNKS = 9 * C1 * C2 * 2 / 16;   // 2304 16-B chunks of W2^T
static_assert(W2_CHUNKS % 64 == 0, "W2^T copies in whole 1-KB DMA blocks");

// Stage one image into LDS, ordered so that nothing waits for a load it does not need:
//   1. issue every global load: x and the conv1 weights first, then (the workgroup's first
//      image) W2^T, then dpool / pmask -- vmcnt retires in order;
//   2. first image: build the 256-entry normalize LUT (exact torchvision arithmetic, bf16)
//      and zero the dz2 pad pixels while the loads are in flight, then store W2^T, barrier;
//   3. x -> bf16 through the LUT, barrier, conv1 recompute a1 = relu(conv1(x)) (needs only x
//      and the conv1 weights: it runs while dpool / pmask are still arriving);
//   4. the maxpool-backward scatter of dz2 (+ the conv2 bias gradient).
// The caller's barrier ends the staging.  FIRST is a template flag so no runtime branch
// joins the live W2^T registers (they spill).
template <bool first>
__device__ __forceinline__ void bwd_load_image(char* smem, int img, const uint8_t* __restrict__ xg,
                                               const bf16* __restrict__ dpool,
                                               const uint8_t* __restrict__ pmask,
                                               const float* __restrict__ w1,
                                               const float* __restrict__ b1,
                                               const bf16* __restrict__ w2t, float (&db2p)[8]) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, i16 = lane & 15;
  bf16* xs = reinterpret_cast<bf16*>(smem + B_XS);
  bf16* lut = reinterpret_cast<bf16*>(smem + B_LUT);
  // ---- 1. loads
  uint32_t xw = 0;
  if (tid < 196) xw = reinterpret_cast<const uint32_t*>(xg + (int64_t)img * 784)[tid];
  // conv1 weights and bias: one 16-B load per (mt) each -- lane group g's taps 4g .. 4g + 3
  // of channel 16mt + i16 are 4 consecutive floats (g = 2: tap 8 is the last of taps 5 .. 8;
  // g = 3 has no taps).  (16 dword loads per lane before: every CU of an XCD fetching the
  // same 1.2 KB delayed the dpool / pmask loads behind them by ~2k cycles, stamps.)
  int toff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int tap = 4 * g + j;
    toff[j] = (tap < 9) ? (tap / 3) * IMG + (tap % 3) : IMG * IMG;
  }
  f32x4 w1q[2], b1v[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    __builtin_memcpy(&w1q[mt], w1 + (mt * 16 + i16) * 9 + min(4 * g, 5), 16);   // 4-B aligned
    __builtin_memcpy(&b1v[mt], b1 + mt * 16 + 4 * g, 16);
  }
  const uint4* dpv = reinterpret_cast<const uint4*>(dpool + (int64_t)img * FEAT);
  const uint2* mkv = reinterpret_cast<const uint2*>(pmask + (int64_t)img * FEAT);
  uint4 d[3];
  uint2 mk[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {   // clamped unconditional loads: no divergent branch for the
    const int it = min(tid + k * BWD_THREADS, PP * 8 - 1);   // live W2^T registers to span
    d[k] = dpv[it];
    mk[k] = mkv[it];
  }
  // W2^T (first image): straight into its LDS image by LDS-DMA, behind this thread's own
  // loads; nothing waits for it until the end of the staging, so the normalize barrier and
  // conv1 no longer wait for 36 KB of weights.  Wave w copies 1-KB blocks w + 8m (8 rows of
  // 128 B); lane l fills slot l & 7 of row l >> 3 with chunk (l & 7) ^ ((row >> 1) & 7)
  // (the swizzle goes on the source address: the DMA's LDS side is lane-linear).
  __builtin_amdgcn_sched_barrier(0);
  if (first) {
    const unsigned wbase = lds_addr(smem) + B_W2;
#pragma unroll
    for (int m = 0; m < (W2_CHUNKS / 64 + 7) / 8; ++m) {
      const int blk = wave + 8 * m;
      if (blk < W2_CHUNKS / 64) {
        const int row = 8 * blk + (lane >> 3), ch = (lane & 7) ^ ((row >> 1) & 7);
        glds16(w2t + row * 64 + ch * 8, wbase + blk * 1024);
      }
    }
  }
  // the arithmetic below stays behind the loads (hipcc otherwise hoists it above them and
  // delays the first HBM request)
  __builtin_amdgcn_sched_barrier(0);
  if (threadIdx.x == 0) PDM_STAMP_VAL(11, PDM_CLOCK());
  // ---- 2. LUT + pad zeroing (first image; both persist across the workgroup's images)
  if (first) {
    if (tid >= 256) lut[tid - 256] = to_bf16(pdm_normalize(tid - 256));
    // zero pixels: columns 24, 25 of every dz2 row and the 4-pixel zero block
    for (int i = tid; i < (2 * H2 + 4) * 8; i += BWD_THREADS) {
      const int pix = i >> 3;
      const int off = pix < 2 * H2 ? B_DZ + ((pix >> 1) * DS + 24 + (pix & 1)) * 128
                                   : B_Z0 + (pix - 2 * H2) * 128;
      *reinterpret_cast<uint4*>(smem + off + (i & 7) * 16) = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();   // LUT ready (dpool / pmask / W2^T keep flying)
  }
  // ---- 3. x through the LUT, conv1 recompute
  if (tid < 196) {
    bf16x4 v = {lut[xw & 0xff], lut[(xw >> 8) & 0xff], lut[(xw >> 16) & 0xff], lut[xw >> 24]};
    reinterpret_cast<bf16x4*>(xs)[tid] = v;
  } else if (tid < 200) {
    reinterpret_cast<bf16x4*>(xs)[tid] = bf16x4{};
  }
  bf16x4 w1f[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w1f[mt][j] = to_bf16(4 * g + j < 9 ? (g == 2 ? w1q[mt][3] : w1q[mt][j]) : 0.f);
  __syncthreads();
  if (threadIdx.x == 0) PDM_STAMP_VAL(13, PDM_CLOCK());
  // conv1 recompute: D[co][pixel] on mfma_f32_16x16x16_bf16 (same math as cnn_fwd), over
  // tiles of 16 "virtual pixels" V = 28y + x of the 28-wide x image (x = 26, 27 and y >= 26
  // computed and dropped): V is the pixel's own x-image index, x & 3 == lane & 3, so the
  // operand reads are V + a per-lane tap offset and the a1 store is (V - 2y) * 64 + a
  // per-lane constant.  46 tiles (48 slots) over 8 waves = 6 per wave, every x read of the
  // 6 tiles issued before their MFMAs.
  constexpr int TPW = 6;
  int tb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) tb[j] = toff[j] == IMG * IMG ? 0 : toff[j];   // w = 0 there
  // one 16-B store per lane and tile: lane pairs g, g ^ 1 swap channel halves
  // (cnn_common.h conv1_pair)
  const int a1c = (conv1_pair_chunk(g) ^ (i16 & 3)) << 4;
  bf16x4 bx[TPW];
  int vv[TPW];
#pragma unroll
  for (int k = 0; k < TPW; ++k) {
    vv[k] = (wave + 8 * k) * 16 + i16;
    const int vc = min(vv[k], IMG * H1 - 1);
#pragma unroll
    for (int j = 0; j < 4; ++j) bx[k][j] = xs[vc + tb[j]];
  }
#pragma unroll
  for (int k = 0; k < TPW; ++k) {
    const int y = vv[k] / IMG, x = vv[k] - y * IMG;
    const bool ok = y < H1 && x < H1;
    bf16x4 o[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(w1f[mt], bx[k], b1v[mt], 0, 0, 0);
      o[mt] = bf16x4{to_bf16(relu1(acc[0])), to_bf16(relu1(acc[1])),
                     to_bf16(relu1(acc[2])), to_bf16(relu1(acc[3]))};
    }
    // dropped pixels store into the spare LDS tail (lane pairs share a 16-B slot): no branch
    const int dst = ok ? B_A1 + (vv[k] - 2 * y) * 64 + a1c : B_SPARE + (lane & 31) * 16;
    *reinterpret_cast<uint4*>(smem + dst) = conv1_pair(o[0], o[1]);
  }
  if (threadIdx.x == 0) PDM_STAMP_VAL(14, PDM_CLOCK());
  // ---- 4. the dz2 scatter
  // maxpool backward as whole-window writes: item (pooled pixel pp, 8-channel chunk ch)
  // builds the 16-B chunk of each of the window's 4 pixels (the pooled gradient at the
  // channel's argmax position if it was > 0, zero elsewhere) and stores 4 x 16 B.
  // For window pos s = 2dy + dx the pixel is (2py + dy, 2px + dx), rotation 4(2py + dy) +
  // 2px + dx.  Mask byte (cnn_fwd): 0x80 | 1 << s if the pooled value is > 0, else 0.
  // VALU-lean (this phase is VALU-bound: 8 waves, 2 per SIMD): the keep-mask of a bf16 pair
  // is one v_perm_b32 that replicates two flag bits, moved to bits 15 / 31 of its sources by
  // one shift each, into the two halves of the word.
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int it = tid + k * BWD_THREADS;   // it & 7 == tid & 7: fixed channel chunk
    if (it < PP * 8) {
      const int pp = it >> 3, ch = it & 7;
      const int py = pp / HP, px = pp - py * HP;
      const int base = B_DZ + ((2 * py) * DS + 2 * px) * 128;
      const int b0 = 2 * px + ch;                 // + 4 (2py + dy) + dx: 8py drops mod 8
      const uint32_t dw[4] = {d[k].x, d[k].y, d[k].z, d[k].w};
      const uint32_t mw[2] = {mk[k].x, mk[k].y};
      // conv2 bias gradient: the pooled gradients of positive pooled values
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t sh = mw[h] << 8;           // bit 15 / 31: flag of channel 4h / 4h + 2
        const uint32_t pos[2] = {__builtin_amdgcn_perm(mw[h], sh, 0x0A0A0808u),
                                 __builtin_amdgcn_perm(mw[h], sh, 0x0B0B0909u)};
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const uint32_t w = dw[2 * h + e] & pos[e];
          db2p[4 * h + 2 * e] += __builtin_bit_cast(float, w << 16);
          db2p[4 * h + 2 * e + 1] += __builtin_bit_cast(float, w & 0xffff0000u);
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
        const int off = base + (sw >> 1) * (DS * 128) + (sw & 1) * 128 +
                        (((b0 + 4 * (sw >> 1) + (sw & 1)) & 7) << 4);
        *reinterpret_cast<uint4*>(smem + off) = o;
      }
    }
  }
  if (threadIdx.x == 0) PDM_STAMP_VAL(12, PDM_CLOCK());
  if (threadIdx.x == 448) PDM_STAMP_VAL(15, PDM_CLOCK());
  // the W2^T DMA has landed before the caller's barrier publishes the staging
  if (first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// conv2 input gradient for MTP tiles {tile0 + 4k} of 16 virtual pixels V = 28y + x (the
// 28-wide x-image grid; x = 26, 27 and y >= 26 are computed on garbage and dropped by the
// epilogue), fused with relu'(a1) and the conv1 weight/bias gradient (into acc1).
//   da1[p][ci] = sum_tap sum_co dz2[p - tap][co] * W2[co][tap][ci]
// 18 straight-line (tap, K-half) steps; the dz2 A fragments and the W2^T B fragments (both
// LDS) are read PFD steps ahead.  Address of the A read of tile k at tap (ky, kx), K-half kh:
//   ((gs[k] - 16(4ky + kx)) & 0x70 | rb[k][ky]) ^ 64kh,  immediate ((2-ky)*DS + 2-kx) * 128
// where rb is the tile's row base (or the zero block for a dz2 row outside the image) and
// gs = 16(g + 4y + x) seeds the rotation swizzle.
template <int MTP, int PFD>
__device__ __forceinline__ void dgrad_pass(const char* smem, int tile0, const int (&ka1)[4],
                                           f32x4 (&acc1)[2], unsigned long long& t_mf,
                                           unsigned long long& t_ep) {
  const int lane = threadIdx.x & 63, g = lane >> 4, i16 = lane & 15;
  const unsigned long long c0 = PDM_CLOCK();
  int rb[MTP][3], gs[MTP];
#pragma unroll
  for (int k = 0; k < MTP; ++k) {
    const int v = (tile0 + 4 * k) * 16 + i16;
    const int y = v / IMG, x = v - y * IMG;
    const int a0 = B_DZ + ((y - 2) * DS + x - 2) * 128;
    const int zb = B_Z0 + (x & 1) * 128;       // same bank parity as the real pixel
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
      rb[k][ky] = ((unsigned)(y - ky) < (unsigned)H2) ? a0 : zb - (2 - ky) * DS * 128;
    gs[k] = (g + 4 * y + x) << 4;
  }
  const int wl0 = B_W2 + i16 * 128 + ((g ^ ((i16 >> 1) & 7)) << 4);
  auto read_step = [&](int tk, bf16x8 (&a)[MTP], bf16x8 (&w)[2]) {
    const int tap = tk >> 1, kh = tk & 1;
    const int ky = tap / 3, kx = tap - 3 * ky;
    const int sk16 = (4 * ky + kx) << 4;
    const int off = ((2 - ky) * DS + (2 - kx)) * 128;
#pragma unroll
    for (int k = 0; k < MTP; ++k) {
      int ad = ((gs[k] - sk16) & 0x70) | rb[k][ky];
      if (kh) ad ^= 64;
      a[k] = *reinterpret_cast<const bf16x8*>(smem + ad + off);
    }
    const int wl = kh ? (wl0 ^ 64) : wl0;
    w[0] = *reinterpret_cast<const bf16x8*>(smem + wl + tap * 4096);
    w[1] = *reinterpret_cast<const bf16x8*>(smem + wl + tap * 4096 + 2048);
  };
  // epilogue operands.  Lane (g, ctap = i16) holds the dgrad outputs of pixels V0 + r,
  // V0 = 16 tile + 4g (a run of 4 in one row: 28 = 7 x 4) for channels i16 and 16 + i16.
  // conv1 wgrad B operand: x[V0 + r + tap offset]; relu'(a1) from the a1 image at
  // (V0 - 2y) * 64 + ka1[r] (^ 32 for channel 16 + i16), where x & 3 == r fixes the swizzle.
  const int ctap = i16;
  const int cky = ctap / 3, ckx = ctap - 3 * cky;
  const int xoff = (ctap < 9) ? (cky * IMG + ckx) : 0;   // taps >= 9: any finite value
  const bf16* xs = reinterpret_cast<const bf16*>(smem + B_XS);
  bf16x4 bx[MTP];
  short av[MTP][4][2];
  bool vhi[MTP];
  auto read_ep = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < MTP; ++k) {
      const int v0 = (tile0 + 4 * k) * 16 + 4 * g;
      const int y = v0 / IMG, x0 = v0 - y * IMG;
      const bool vt = y < H1;
      vhi[k] = vt && x0 < 24;                   // pixels x0 + 2, x0 + 3 inside the row
      const int vc = vt ? v0 : 0;
      const int pb = vt ? B_A1 + (v0 - 2 * y) * 64 : B_Z0;   // zero block: relu' = 0
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
    __builtin_amdgcn_sched_barrier(0);   // keep each step's reads where they are issued
    if (tk + PFD < 18) read_step(tk + PFD, a[(tk + PFD) % (PFD + 1)], w[(tk + PFD) % (PFD + 1)]);
    else if (tk + PFD == 18) read_ep();
    // the reads go out before this step's MFMAs (hipcc otherwise sinks them below the
    // MFMAs and the read-ahead shrinks to ~1 step: lgkmcnt(7) instead of lgkmcnt(12))
    __builtin_amdgcn_sched_barrier(0);
    const int s = tk % (PFD + 1);
#pragma unroll
    for (int k = 0; k < MTP; ++k) {
      acc[k][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s][k], w[s][0], acc[k][0], 0, 0, 0);
      acc[k][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s][k], w[s][1], acc[k][1], 0, 0, 0);
    }
  }
  const unsigned long long c1 = PDM_CLOCK();
  t_mf += c1 - c0;
  // epilogue per tile: relu'(a1) -> dz1 (bf16) -> conv1 wgrad on mfma_f32_16x16x16_bf16
  // (M = ci, N = tap 0..8 / 9 = ones -> bias, K = pixels); the dgrad accumulator
  // (lane: ci = 16nt + i16, pixels 4g + r) is already its A operand.  a1 > 0 is tested on
  // the bf16 bits as a signed 16-bit integer.
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
  t_ep += PDM_CLOCK() - c1;
}

// Work split (per image, after the staged load): waves 0-3 run the conv2 wgrad (18 (tap,
// ci-tile) pairs), waves 4-7 the dgrad over 48 tile slots (46 of the 28-wide virtual grid)
// in passes of DG_MTP tiles with operands read DG_PFD steps ahead; with one image per
// workgroup the wgrad waves run the third dgrad pass after their wgrad.
constexpr int DG_MTP = 4;       // tiles per dgrad pass on waves 4-7
constexpr int DG_PFD = 2;       // read-ahead distance in (tap, K-half) steps
static_assert(12 % DG_MTP == 0, "dgrad passes: 12 / DG_MTP passes of DG_MTP tiles per wave (the "
              "wgrad waves take the last pass when a workgroup has one image)");
static_assert(DG_PFD * (DG_MTP + 2) <= 15, "in-flight LDS reads must fit lgkmcnt");

// ONE: one image per workgroup (B <= CUs).  Its own kernel, so that register allocation of the
// straight-line single-image code is not shaped by the multi-image loop (and vice versa).
template <bool ONE>
__global__ __launch_bounds__(BWD_THREADS, 1) void cnn_bwd_kernel(
    const uint8_t* __restrict__ xg, const float* __restrict__ w1, const float* __restrict__ b1,
    const bf16* __restrict__ dpool, const uint8_t* __restrict__ pmask,
    const bf16* __restrict__ w2t, int B, int ipb, float* __restrict__ slab, unsigned* xg_sync) {
  __shared__ __attribute__((aligned(16))) char smem[B_TOTAL];
  // xgmi streamed mode: this kernel starting means fc1_bwd finished, i.e. the fc
  // gradient bucket is complete -> hand it to the persistent collective (csrc/xgmi.h)
  if (xg_sync != nullptr && blockIdx.x == 0 && threadIdx.x == 0) xg_signal_backward(xg_sync);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, pq = i16 & 3;
  float* red = reinterpret_cast<float*>(smem + B_RED);
  const char* a1s = smem + B_A1;
  float* out = slab + (int64_t)blockIdx.x * CONV_SLAB;
  float db2p[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  f32x4 acc1[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  unsigned long long t_mf = 0, t_ep = 0;
  // relu'(a1) read offsets of channel i16 at pixel x with x & 3 == r (a1_off swizzle)
  int ka1[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) ka1[r] = r * 64 + ((((2 * i16) >> 4) ^ r) << 4) + ((2 * i16) & 15);
  PDM_STAMP(0);

  if (wave < 4) {
    // ===== conv2 weight gradient: (tap, ci-tile) pairs {w, w+4, ...} x all 4 co tiles =====
    // K = output pixels in chunks of 8 along a row (24 = 3 chunks): lane group g of k-step
    // ks takes chunk 4ks+g; its lane q reads pixels x = col0+q and x+4 (col0 % 8 == 0).
    f32x4 acc[5][4];   // zeroed after the first image's staging (not live through it)
    const bool five = wave < 2;  // 18 pairs over 4 waves: 5,5,4,4 (+1 discarded on 2,3)
    // Operand addresses of k-step ks = 3m + j: lane group g reads dz2/a1 row 4m + r_j,
    // columns 8c_j + q (and + 4), with 4j + g = 3r_j + c_j.  The dz2 rotation (4 row + x)
    // mod 8 does not depend on m, so every address is a per-lane base of (j, fragment) plus
    // the immediate m * (4 rows): no address arithmetic inside the k loop.
    int abA[3][4], abA2[3][4], abB[3][5];
    // (filled after the first image's loads are issued: 51 VALU-computed registers that
    // would otherwise delay the wgrad waves' share of the staging loads)
    auto setup_addr = [&]() __attribute__((always_inline)) {
    // recomputed per image from a laundered lane id: hoisted out of the image loop, these
    // addresses (or their lane-dependent parts) would stay live through the staging and spill
    int ln;
    asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
    const int g = ln >> 4, q = (ln >> 2) & 3, pq = ln & 3;
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
      const int v = 4 * j + g, rj = v / 3, xj = (v - 3 * rj) * 8 + q;
      const int dbase = B_DZ + (rj * DS + xj) * 128 + 8 * (pq & 1);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        // chunk 2mt + (pq >> 1) rotated by (4 row + x); pixel x + 4 is rotated 4 further,
        // i.e. its chunk offset is this one ^ 64
        const int co = (((pq >> 1) + 4 * rj + xj + 2 * mt) & 7) << 4;
        abA[j][mt] = dbase + co;
        abA2[j][mt] = dbase + 512 + (co ^ 64);
      }
#pragma unroll
      for (int pi = 0; pi < 5; ++pi) abB[j][pi] = B_A1 + (rj * H1 + xj) * 64 + cp[pi];
    }
    };
    auto rd_a = [&](int ks, int mt) __attribute__((always_inline)) {
      const int j = ks % 3, m = ks / 3;
      return cat_tr(lds_tr16(smem + abA[j][mt] + m * 4 * DS * 128),
                    lds_tr16(smem + abA2[j][mt] + m * 4 * DS * 128));
    };
    auto rd_b = [&](int ks, int pi) __attribute__((always_inline)) {
      const int j = ks % 3, m = ks / 3;
      return cat_tr(lds_tr16(smem + abB[j][pi] + m * 4 * H1 * 64),
                    lds_tr16(smem + abB[j][pi] + m * 4 * H1 * 64 + 256));
    };
    // software-pipelined over k-steps: region pi of step ks issues the reads of step ks+1
    // (B fragment pi and A fragment pi) ahead of its 4 MFMAs, so every operand is one whole
    // step (20 MFMAs) old when it is consumed
    auto wgrad_image = [&]() __attribute__((always_inline)) {
      bf16x8 A[2][4], Bv[2][5];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) A[0][mt] = rd_a(0, mt);
#pragma unroll
      for (int pi = 0; pi < 5; ++pi) Bv[0][pi] = rd_b(0, pi);
      // compile-time k loop (hipcc leaves an 18-trip `#pragma unroll` loop rolled and then
      // keeps the register arrays it indexes in scratch)
      static_for<P2 / 32>([&](auto KS) __attribute__((always_inline)) {
        constexpr int ks = decltype(KS)::value;
        bf16x8 (&Ac)[4] = A[ks & 1];
        bf16x8 (&Bc)[5] = Bv[ks & 1];
        bf16x8 (&An)[4] = A[(ks + 1) & 1];
        bf16x8 (&Bn)[5] = Bv[(ks + 1) & 1];
#pragma unroll
        for (int pi = 0; pi < 5; ++pi) {
          __builtin_amdgcn_sched_barrier(0);
          if (ks + 1 < P2 / 32) {
            Bn[pi] = rd_b(ks + 1, pi);
            if (pi < 4) An[pi] = rd_a(ks + 1, pi);
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)   // waves 2,3: pair 4 is a discarded duplicate
            acc[pi][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Bc[pi], Ac[mt], acc[pi][mt], 0, 0, 0);
        }
      });
    };
    // the accumulators persist across the workgroup's images; after the last image they
    // are stored while the dgrad waves are still computing.  The MFMAs compute dW2^T (B and
    // A operands swapped: the same products, summed in the same order), so lane (g, i16)
    // holds co = 16mt + i16, ci = 16nt + 4g + r: 4 consecutive floats of dW2[co][tap][ci],
    // one 16-B store per (pair, co tile) -- 20 instead of 80 store instructions per wave
    // (the tail was store-issue-bound: 4.3k cycles, stamps)
    auto per_image = [&](auto first, auto one, int i, bool last) __attribute__((always_inline)) {
      const int img = blockIdx.x * ipb + i;
      if (img < B) bwd_load_image<decltype(first)::value>(smem, img, xg, dpool, pmask, w1, b1, w2t, db2p);
      setup_addr();
      __syncthreads();
      if constexpr (decltype(first)::value) {
#pragma unroll
        for (int i = 0; i < 5; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      PDM_STAMP(1);
      if (img < B) wgrad_image();
      PDM_STAMP(2);
      if (last) {
#pragma unroll
        for (int pi = 0; pi < 5; ++pi) {
          if (pi == 4 && !five) break;
          const int pair = wave + 4 * pi;
          const int tap = pair >> 1, nt = pair & 1;
          int o;   // laundered: 20 hoisted 64-bit store addresses would be spilled
          asm volatile("v_mov_b32 %0, %1" : "=v"(o) : "v"(i16 * 288 + 4 * g));
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
            pdm_slab_store4(out, o + mt * 16 * 288 + tap * 32 + nt * 16, acc[pi][mt]);
        }
        PDM_STAMP(3);
      }
      // one image per workgroup: with its accumulators stored, this wave also takes the
      // last dgrad pass (tiles 48 - 4 DG_MTP + wave + 4k), which balances the two wave groups (the
      // wgrad's 360 MFMAs vs the dgrad's 432 + epilogues)
      if constexpr (decltype(one)::value) {
        if (img < B)
          dgrad_pass<DG_MTP, DG_PFD>(smem, 48 - 4 * DG_MTP + wave, ka1, acc1, t_mf, t_ep);
      }
      __syncthreads();
    };
    // one image per workgroup (B <= CUs) is its own straight-line instantiation: there the
    // wgrad accumulators are dead once stored, so they are not live (and spilled) through
    // the dgrad pass the same waves run next
    if constexpr (ONE) {
      per_image(std::true_type{}, std::true_type{}, 0, true);
    } else {
      per_image(std::true_type{}, std::false_type{}, 0, false);
      for (int i = 1; i < ipb; ++i) per_image(std::false_type{}, std::false_type{}, i, i == ipb - 1);
    }
  } else {
    // ===== conv2 input gradient + relu'(a1) + conv1 weight/bias gradient =====
    const int wd = wave - 4;
    auto per_image = [&](auto first, int i) __attribute__((always_inline)) {
      const int img = blockIdx.x * ipb + i;
      if (img < B) bwd_load_image<decltype(first)::value>(smem, img, xg, dpool, pmask, w1, b1, w2t, db2p);
      __syncthreads();
      if (img < B) {
        // tiles wd + 4j, j < 12, in passes of DG_MTP tiles; a rolled pass loop keeps one
        // copy of the pass code and stops cross-pass scheduling
        // (one image per workgroup: the wgrad waves take the last pass)
        const int npass = ONE ? 12 / DG_MTP - 1 : 12 / DG_MTP;
#pragma unroll 1
        for (int ps = 0; ps < npass; ++ps)
          dgrad_pass<DG_MTP, DG_PFD>(smem, wd + 4 * DG_MTP * ps, ka1, acc1, t_mf, t_ep);
      }
      __syncthreads();
    };
    per_image(std::true_type{}, 0);
    if constexpr (!ONE)
      for (int i = 1; i < ipb; ++i) per_image(std::false_type{}, i);
    if (tid == 256) {
      PDM_STAMP_VAL(8, t_mf);
      PDM_STAMP_VAL(9, t_ep);
      PDM_STAMP_VAL(10, PDM_CLOCK());
    }
  }
  // conv1 weight/bias partials, acc1[nt]: rows ci = 16nt + 4g + r, col tap = i16.  Waves 4-7
  // write their slot, waves 0-3 then add theirs (slot = wave & 3).  (red aliases a1, which
  // is dead once both wave groups have passed the last image barrier.)
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
  // conv2 bias: lanes sharing (lane & 7) hold the same 8 channels (DPP / permlane swaps:
  // the shuffle butterfly's 24 LDS bpermutes each waited out a full LDS round trip)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float v = sum_xor32(sum_xor16(sum_xor8(db2p[j])));
    if (lane < 8) red[RED_DB2 + wave * C2 + lane * 8 + j] = v;
  }
  __syncthreads();
  PDM_STAMP(4);
  if (tid < C2) {
    float s = 0.f;
    for (int w = 0; w < 8; ++w) s += red[RED_DB2 + w * C2 + tid];
    pdm_slab_store(&out[SL_DB2 + tid], s);
  } else if (tid >= 64 && tid < 64 + C1 * 10) {
    const int e = tid - 64;             // (ci, tap) with tap 0..8 = weight, 9 = bias
    const int ci = e / 10, t = e - 10 * ci;
    float s = 0.f;
    for (int w = 0; w < 4; ++w) s += red[RED_DW1 + w * C1 * 16 + ci * 16 + t];
    pdm_slab_store(t < 9 ? &out[SL_DW1 + ci * 9 + t] : &out[SL_DB1 + ci], s);
  }
}

// ------------------------------------------------------------------ conv_reduce
constexpr int CR_COLS = 64;     // slab columns per conv_reduce workgroup (294 workgroups)
static_assert(CONV_SLAB % CR_COLS == 0, "conv slab must split into whole column tiles");

__global__ __launch_bounds__(256) void conv_reduce_kernel(const float* __restrict__ slab, int nblk,
                                                          float* __restrict__ gw2,
                                                          float* __restrict__ gb2,
                                                          float* __restrict__ gw1,
                                                          float* __restrict__ gb1) {
  // workgroup = 64 slab columns x 16 slab groups: lane c4 = tid & 15 owns 4 columns (float4),
  // group rg = tid >> 4 sums slabs rg, rg + 16, ... in batches of 8 loads in flight; the 16
  // group sums are combined in a fixed order -> deterministic.
  __shared__ float4 red[16][CR_COLS / 4];
  const int tid = threadIdx.x, c4 = tid & 15, rg = tid >> 4;
  const int col = blockIdx.x * CR_COLS + 4 * c4;
  const float4* p = reinterpret_cast<const float4*>(slab + col);
  constexpr int STRIDE4 = CONV_SLAB / 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int j0 = rg; j0 < nblk; j0 += 16 * 8) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[(int64_t)min(j0 + 16 * u, nblk - 1) * STRIDE4];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool on = j0 + 16 * u < nblk;
      acc.x += on ? v[u].x : 0.f;
      acc.y += on ? v[u].y : 0.f;
      acc.z += on ? v[u].z : 0.f;
      acc.w += on ? v[u].w : 0.f;
    }
  }
  red[rg][c4] = acc;
  __syncthreads();
  if (tid < CR_COLS) {
    const float* rf = reinterpret_cast<const float*>(&red[0][0]);
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) t += rf[g * CR_COLS + tid];
    const int e = blockIdx.x * CR_COLS + tid;
    if (e < SL_DB2) gw2[e] = t;
    else if (e < SL_DW1) gb2[e - SL_DB2] = t;
    else if (e < SL_DB1) gw1[e - SL_DW1] = t;
    else gb1[e - SL_DB1] = t;
  }
}

#endif  // PDM_WANT_REST
}  // namespace

#if PDM_WANT_FC1_BWD
void launch_fc1_bwd(const __bf16* dh, const __bf16* dht, int ldt, const __bf16* pool,
                    const __bf16* wf1t, int B, float* gwf1, __bf16* dpool, const float* head_slab,
                    int head_blocks, float* gwf2, float* gbf2, float* gbf1, double* metrics,
                    const FcUpdate& fcu, hipStream_t st) {
  const int nd = (ldt / 32) * DX_TILES;
  const int nblk = DW_TILES + nd + HR_BLOCKS, off = 0;
  fc1_bwd_kernel<<<nblk, 256, 0, st>>>(dh, dht, ldt, pool, wf1t, B, gwf1, dpool, head_slab,
                                       head_blocks, gwf2, gbf2, gbf1, metrics, off, fcu);
}

#endif
#if PDM_WANT_REST
int cnn_bwd_blocks(int B, int ipb) { return (B + ipb - 1) / ipb; }

void launch_cnn_bwd(const uint8_t* xg, const float* w1, const float* b1, const __bf16* dpool,
                    const uint8_t* pmask, const __bf16* w2t, int B, int ipb, float* slab,
                    unsigned* xg_sync, hipStream_t st) {
  if (ipb == 1)
    cnn_bwd_kernel<true><<<cnn_bwd_blocks(B, ipb), BWD_THREADS, 0, st>>>(xg, w1, b1, dpool, pmask,
                                                                       w2t, B, ipb, slab, xg_sync);
  else
    cnn_bwd_kernel<false><<<cnn_bwd_blocks(B, ipb), BWD_THREADS, 0, st>>>(xg, w1, b1, dpool, pmask,
                                                                        w2t, B, ipb, slab, xg_sync);
}

void launch_conv_reduce(const float* slab, int nblk, float* gw2, float* gb2, float* gw1, float* gb1,
                        hipStream_t st) {
  conv_reduce_kernel<<<CONV_SLAB / CR_COLS, 256, 0, st>>>(slab, nblk, gw2, gb2, gw1, gb1);
}

#ifdef PDM_STAMPS
void read_stamps_bwd(unsigned long long* host) {
  hipMemcpyFromSymbol(host, HIP_SYMBOL(pdm_stamps), sizeof(unsigned long long) * 256 * 16);
}
#else
void read_stamps_bwd(unsigned long long* host) {
  for (int i = 0; i < 256 * 16; ++i) host[i] = 0;
}
#endif
#endif  // PDM_WANT_REST
