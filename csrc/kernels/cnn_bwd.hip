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
#include "xgmi.h"

#include <cstdlib>

namespace {

using namespace cnn;

// ------------------------------------------------------------------ fc1_bwd
constexpr int DW_TILES = FEAT / 64;  // 144
constexpr int DWC = 128;             // dW1 batch rows staged per LDS round
constexpr int DX_COLS = 128;         // dX tile: 32 batch rows x 128 features per workgroup
constexpr int DX_TILES = FEAT / DX_COLS;   // 72 = 8 XCDs x 9
constexpr int NXCD = 8;              // MI355X: workgroups are dealt round-robin to 8 XCDs
static_assert(DX_TILES % NXCD == 0 && DW_TILES % NXCD == 0, "XCD-aware tile mapping");
constexpr int HR_BLOCKS = (HEAD_SLAB + 63) / 64;   // head-slab reduction workgroups (23)

__device__ __forceinline__ int tile_off(int row, int byte) {  // [32 rows][128 B], 2-way-free tr reads
  return row * 128 + (byte ^ (((row >> 3) & 1) << 5));
}

__global__ __launch_bounds__(256) void fc1_bwd_kernel(
    const bf16* __restrict__ dh, const bf16* __restrict__ dht, int ldt,
    const bf16* __restrict__ pool, const bf16* __restrict__ wf1t, int B, float* __restrict__ gwf1,
    bf16* __restrict__ dpool, const float* __restrict__ head_slab, int head_blocks,
    float* __restrict__ gwf2, float* __restrict__ gbf2, float* __restrict__ gbf1,
    double* __restrict__ metrics, int bid_offset) {
  __shared__ __attribute__((aligned(16))) char tile[DWC * 128];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, pq = i16 & 3;
  const int nd = (ldt / 32) * DX_TILES;
  const int bid = blockIdx.x + bid_offset;

  if (bid < DW_TILES) {
    // ---- dW1 tile: all 128 hidden rows x 64 feature columns, K = batch ----
    // The batch is consumed in chunks of DWC rows: the whole chunk (pool rows and the
    // dh^T A fragments) is loaded with every load in flight at once, and the next chunk's
    // loads are issued before the current chunk's MFMAs.
    const int k0 = bid * 64;
    f32x4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int srow = tid >> 3, sch = tid & 7;
    uint4 pv[DWC / 32];
    bf16x8 a[2][DWC / 32];
    auto load_chunk = [&](int c0) {
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
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int kk = 0; kk < DWC / 32; ++kk)
          a[mt][kk] = *reinterpret_cast<const bf16x8*>(
              dht + (int64_t)(wave * 32 + mt * 16 + i16) * ldt + min(c0 + 32 * kk, ldt - 32) + 8 * g);
    };
    load_chunk(0);
    for (int c0 = 0; c0 < ldt; c0 += DWC) {
      __syncthreads();   // previous chunk's tile reads are done
#pragma unroll
      for (int j = 0; j < DWC / 32; ++j)
        *reinterpret_cast<uint4*>(tile + tile_off(srow + 32 * j, sch * 16)) = pv[j];
      bf16x8 ac[2][DWC / 32];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int kk = 0; kk < DWC / 32; ++kk) ac[mt][kk] = a[mt][kk];
      __syncthreads();
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
            for (int mt = 0; mt < 2; ++mt)
              acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ac[mt][kk], bv, acc[mt][nt], 0, 0, 0);
          }
        }
      }
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = wave * 32 + mt * 16 + 4 * g + r;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) gwf1[(int64_t)n * FEAT + k0 + 16 * nt + i16] = acc[mt][nt][r];
      }
    return;
  }

  if (bid < DW_TILES + nd) {
    // ---- dX tile: 32 batch rows x 128 features, K = 128 hidden ----
    // Computed transposed, dpool^T[f][b] = W1^T[f][:] . dh^T[:][b]: the MFMA output lane then
    // holds 4 consecutive features of one batch row, stored as one 8-byte bf16x4.  Each wave
    // owns 32 features x 32 rows; all operand loads of the wave are issued up front.
    // XCD-aware: workgroup t runs on XCD t % 8 (DW_TILES is a multiple of 8), and every XCD
    // owns 1/8 of the feature range, so each XCD's L2 holds only its 1/8 of W1^T.
    const int t = bid - DW_TILES;
    constexpr int TPX = DX_TILES / NXCD;                 // feature tiles per XCD
    const int xcd = t % NXCD, loc = t / NXCD;
    const int b0 = (loc / TPX) * 32;
    const int f0 = (xcd * TPX + loc % TPX) * DX_COLS + wave * 32;
    constexpr int FT = 2;
    bf16x8 wa[FT][HID / 32], hb[2][HID / 32];
#pragma unroll
    for (int ks = 0; ks < HID / 32; ++ks) {
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
        wa[ft][ks] = *reinterpret_cast<const bf16x8*>(
            wf1t + (int64_t)(f0 + ft * 16 + i16) * HID + 32 * ks + 8 * g);
#pragma unroll
      for (int bt = 0; bt < 2; ++bt)
        hb[bt][ks] = *reinterpret_cast<const bf16x8*>(
            dh + (int64_t)(b0 + bt * 16 + i16) * HID + 32 * ks + 8 * g);
    }
    // keep every load above this point: the scheduler would otherwise interleave them
    // with the MFMAs behind per-load waits
    __builtin_amdgcn_sched_barrier(0);
    f32x4 acc[FT][2];
#pragma unroll
    for (int ft = 0; ft < FT; ++ft)
#pragma unroll
      for (int bt = 0; bt < 2; ++bt) acc[ft][bt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < HID / 32; ++ks)
#pragma unroll
      for (int ft = 0; ft < FT; ++ft)
#pragma unroll
        for (int bt = 0; bt < 2; ++bt)
          acc[ft][bt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[ft][ks], hb[bt][ks], acc[ft][bt], 0, 0, 0);
#pragma unroll
    for (int bt = 0; bt < 2; ++bt) {
      const int row = b0 + bt * 16 + i16;
      if (row < B) {
#pragma unroll
        for (int ft = 0; ft < FT; ++ft) {
          const bf16x4 o = {to_bf16(acc[ft][bt][0]), to_bf16(acc[ft][bt][1]),
                            to_bf16(acc[ft][bt][2]), to_bf16(acc[ft][bt][3])};
          *reinterpret_cast<bf16x4*>(dpool + (int64_t)row * FEAT + f0 + ft * 16 + 4 * g) = o;
        }
      }
    }
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

// ------------------------------------------------------------------ cnn_bwd
constexpr int BWD_THREADS = 512;
constexpr int DZW = 28;                         // dz2 image padded by 2 on every side
constexpr int B_XS = 0;                         // bf16 x [784] + zero pad 1600
constexpr int B_A1 = 1600;                      // a1 image              43264
constexpr int B_DZ = B_A1 + P1 * 64;            // padded dz2 image      100352
constexpr int B_RED = B_DZ + DZW * DZW * 128;   // fp32 reduction scratch
constexpr int RED_DB2 = 0;                      // [8 waves][64]
constexpr int RED_DW1 = RED_DB2 + 8 * C2;       // [4 waves][32 ci][16 taps] (tap 9 = bias)
constexpr int RED_N = RED_DW1 + 4 * C1 * 16;    // 2560 floats
constexpr int B_MK = B_RED + RED_N * 4;         // relu'(a1) bitmask: u32 [676] (bit = ci)
constexpr int B_TOTAL = B_MK + P1 * 4;           // 158160 B -> 1 workgroup / CU
constexpr int SL_DB2 = C2 * 9 * C1;             // 18432
constexpr int SL_DW1 = SL_DB2 + C2;             // 18496
constexpr int SL_DB1 = SL_DW1 + C1 * 9;         // 18784
static_assert(SL_DB2 == CNN_CONV_SLAB_DB2 && SL_DW1 == CNN_CONV_SLAB_DW1 &&
              SL_DB1 == CNN_CONV_SLAB_DB1 && SL_DB1 + C1 == CNN_CONV_SLAB, "conv slab layout");

// dz2 padded image: pixel (r, c) in [0,28)^2 holds dz2[r-2][c-2] (0 on the border), 128 B,
// 16-B chunk XOR (2r + c) & 7: dgrad row reads conflict-free, wgrad transposed reads 2-way.
__device__ __forceinline__ int dzp_off(int r, int c, int byte) {
  return (r * DZW + c) * 128 + ((((byte >> 4) ^ ((2 * r + c) & 7))) << 4) + (byte & 15);
}

// Stage one image into LDS: x (bf16, zero-padded), dz2 (expanded from the pooled gradient
// and the argmax|positive mask), accumulate the conv2 bias gradient, then recompute
// a1 = relu(conv1(x)) into its LDS image (cheaper than a 43 KB/image HBM round trip).
// Every global load of the image is issued before the first LDS store.
__device__ __forceinline__ void bwd_load_image(char* smem, int img, const uint8_t* __restrict__ xg,
                                               const bf16* __restrict__ dpool,
                                               const uint8_t* __restrict__ pmask,
                                               const float* __restrict__ w1,
                                               const float* __restrict__ b1, bool first,
                                               float (&db2p)[8]) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, i16 = lane & 15;
  bf16* xs = reinterpret_cast<bf16*>(smem + B_XS);
  char* a1s = smem + B_A1;
  char* dzs = smem + B_DZ;
  uint32_t xw = 0;
  if (tid < 196) xw = reinterpret_cast<const uint32_t*>(xg + (int64_t)img * 784)[tid];
  const uint4* dpv = reinterpret_cast<const uint4*>(dpool + (int64_t)img * FEAT);
  const uint2* mkv = reinterpret_cast<const uint2*>(pmask + (int64_t)img * FEAT);
  uint4 d[3];
  uint2 mk[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int it = tid + k * BWD_THREADS;
    if (it < PP * 8) {
      d[k] = dpv[it];
      mk[k] = mkv[it];
    }
  }
  // conv1 operands, issued together with the image loads (unconditional clamped loads
  // + selects: no per-load branch / wait)
  float w1v[2][4];
  int toff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int tap = 4 * g + j;
    toff[j] = (tap < 9) ? (tap / 3) * IMG + (tap % 3) : IMG * IMG;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) w1v[mt][j] = w1[(mt * 16 + i16) * 9 + min(tap, 8)];
  }
  f32x4 b1v[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) b1v[mt][r] = b1[mt * 16 + 4 * g + r];
  if (threadIdx.x == 0) PDM_STAMP_VAL(11, PDM_CLOCK());
  // First image of the workgroup: zero the 2-pixel border of the padded dz2 image (never
  // written afterwards) while the loads are in flight.  The 24x24 interior needs no
  // clearing: the window writes below cover every interior pixel exactly once.
  if (first) {
    for (int i = tid; i < 208 * 8; i += BWD_THREADS) {
      const int pix = i >> 3;
      int r, c;
      if (pix < 112) {                    // rows 0, 1, 26, 27
        r = pix / DZW;
        c = pix - r * DZW;
        r = r < 2 ? r : r + 24;
      } else {                            // columns 0, 1, 26, 27 of rows 2..25
        const int q = pix - 112;
        r = 2 + (q >> 2);
        c = (q & 3) < 2 ? (q & 3) : (q & 3) + 24;
      }
      *reinterpret_cast<uint4*>(dzs + (r * DZW + c) * 128 + (i & 7) * 16) = make_uint4(0, 0, 0, 0);
    }
  }
  if (tid < 196) {
    bf16x4 v = {to_bf16(pdm_normalize(xw & 0xff)), to_bf16(pdm_normalize((xw >> 8) & 0xff)),
                to_bf16(pdm_normalize((xw >> 16) & 0xff)), to_bf16(pdm_normalize(xw >> 24))};
    reinterpret_cast<bf16x4*>(xs)[tid] = v;
  } else if (tid < 200) {
    reinterpret_cast<bf16x4*>(xs)[tid] = bf16x4{};
  }
  // maxpool backward as whole-window writes: item (pooled pixel pp, 8-channel chunk ch)
  // builds the 16-B chunk of each of the window's 4 pixels (the pooled gradient at the
  // channel's argmax position if it was > 0, zero elsewhere) and stores 4 x 16 B.
  // For window pos s = 2dy + dx the padded pixel is base + (dy*28 + dx) and its chunk
  // swizzle (2r + c) & 7 is (b0 + s) & 7.
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int it = tid + k * BWD_THREADS;   // it & 7 == tid & 7: fixed channel chunk
    if (it < PP * 8) {
      const int pp = it >> 3, ch = it & 7;
      const int py = pp / HP, px = pp - py * HP;
      const int base = ((2 * py + 2) * DZW + 2 * px + 2) * 128;
      const int b0 = 4 * py + 2 * px + 6;
      const uint32_t dw[4] = {d[k].x, d[k].y, d[k].z, d[k].w};
      const uint32_t mw[2] = {mk[k].x, mk[k].y};
      uint32_t sel[8];                       // per channel: window position, or 4 if <= 0
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t mb = (mw[j >> 2] >> (8 * (j & 3))) & 0xff;
        const uint32_t dv = (dw[j >> 1] >> (16 * (j & 1))) & 0xffff;
        sel[j] = (mb & 0x80) ? (mb & 3) : 4u;
        db2p[j] += __builtin_bit_cast(float, ((mb & 0x80) ? dv : 0u) << 16);
      }
#pragma unroll
      for (int sw = 0; sw < 4; ++sw) {
        uint4 o;
        uint32_t* ow = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t w = dw[q];
          ow[q] = (sel[2 * q] == (uint32_t)sw ? (w & 0xffffu) : 0u) |
                  (sel[2 * q + 1] == (uint32_t)sw ? (w & 0xffff0000u) : 0u);
        }
        const int off = base + (sw >> 1) * (DZW * 128) + (sw & 1) * 128 + ((ch ^ ((b0 + sw) & 7)) << 4);
        *reinterpret_cast<uint4*>(dzs + off) = o;
      }
    }
  }
  if (threadIdx.x == 0) PDM_STAMP_VAL(12, PDM_CLOCK());
  if (threadIdx.x == 448) PDM_STAMP_VAL(15, PDM_CLOCK());
  bf16x4 w1f[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int j = 0; j < 4; ++j) w1f[mt][j] = to_bf16(4 * g + j < 9 ? w1v[mt][j] : 0.f);
  __syncthreads();
  if (threadIdx.x == 0) PDM_STAMP_VAL(13, PDM_CLOCK());
  // conv1 recompute: D[co][pixel] on mfma_f32_16x16x16_bf16 (same math as cnn_fwd).
  // 43 pixel tiles over 8 waves = 6 per wave (the last round clamps), every x read of
  // the 6 tiles issued before their MFMAs.
  constexpr int NT1 = (P1 + 15) / 16;                      // 43
  constexpr int TPW = (NT1 + BWD_THREADS / 64 - 1) / (BWD_THREADS / 64);   // 6
  bf16x4 bx[TPW];
  int ty[TPW], tx[TPW];
#pragma unroll
  for (int k = 0; k < TPW; ++k) {
    const int nt = min(wave + 8 * k, NT1 - 1);
    const int P = min(nt * 16 + i16, P1 - 1);
    ty[k] = P / H1;
    tx[k] = P - ty[k] * H1;
    const int xb = ty[k] * IMG + tx[k];
#pragma unroll
    for (int j = 0; j < 4; ++j) bx[k][j] = xs[toff[j] == IMG * IMG ? IMG * IMG : xb + toff[j]];
  }
#pragma unroll
  for (int k = 0; k < TPW; ++k) {
    const int nt = wave + 8 * k;
    const bool ok = nt < NT1 && nt * 16 + i16 < P1;
    uint32_t bits = 0;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(w1f[mt], bx[k], b1v[mt], 0, 0, 0);
      bf16x4 o = {to_bf16(fmaxf(acc[0], 0.f)), to_bf16(fmaxf(acc[1], 0.f)),
                  to_bf16(fmaxf(acc[2], 0.f)), to_bf16(fmaxf(acc[3], 0.f))};
#pragma unroll
      for (int r = 0; r < 4; ++r)
        bits |= (from_bf16(o[r]) > 0.f ? 1u : 0u) << (16 * mt + 4 * g + r);
      if (ok) *reinterpret_cast<bf16x4*>(a1s + a1_off(ty[k], tx[k], 32 * mt + 8 * g)) = o;
    }
    // relu' bitmask of the pixel: OR the 4 lane groups' channel bits
    bits |= __shfl_xor(bits, 16, 64);
    bits |= __shfl_xor(bits, 32, 64);
    if (g == 0 && ok) reinterpret_cast<uint32_t*>(smem + B_MK)[nt * 16 + i16] = bits;
  }
  if (threadIdx.x == 0) PDM_STAMP_VAL(14, PDM_CLOCK());
}

// conv2 input gradient for MTP a1 pixel tiles {tile0 + 4k} of the staged image, fused with
// relu'(a1) and the conv1 weight/bias gradient (accumulated into acc1).
//   da1[p][ci] = sum_tap sum_co dz2[p - tap][co] * W2[co][tap][ci]
// 18 straight-line (tap, K-half) steps; each W2^T fragment is loaded 4 steps ahead into its
// own register and the dz2 A fragments one step ahead (double buffer).  Tiles past the
// image (>= 43) compute on clamped pixels and are discarded by the epilogue.
template <int MTP, int PF>
__device__ __forceinline__ void dgrad_pass(const char* dzs, const uint32_t* mks, const bf16* xs,
                                           const bf16* w2t, int tile0, f32x4 (&acc1)[2],
                                           unsigned long long& t_mf, unsigned long long& t_ep) {
  const int lane = threadIdx.x & 63, g = lane >> 4, i16 = lane & 15;
  const unsigned long long c0 = PDM_CLOCK();
  // opaque zero offset per pass: the W2^T loads must not be hoisted out of the pass loop.
  // (Laundering the pointer itself would turn them into flat loads, which also count on
  // lgkmcnt and make every LDS wait drain the in-flight global prefetch.)
  int wz = 0;
  asm volatile("" : "+s"(wz));
  const bf16* w2l = w2t + wz;
  auto wfrag = [&](int t, int kh, int nt) {
    return *reinterpret_cast<const bf16x8*>(w2l + (t * C1 + nt * 16 + i16) * C2 + 32 * kh + 8 * g);
  };
  int dbase[MTP], s0[MTP];
#pragma unroll
  for (int k = 0; k < MTP; ++k) {
    const int P = min((tile0 + 4 * k) * 16 + i16, P1 - 1);
    const int y = P / H1, x = P - y * H1;
    dbase[k] = ((y + 2) * DZW + x + 2) * 128;
    s0[k] = 2 * y + x + 6;
  }
  f32x4 acc[MTP][2];
#pragma unroll
  for (int k = 0; k < MTP; ++k) acc[k][0] = acc[k][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 w[18][2];
#pragma unroll
  for (int tk = 0; tk < PF; ++tk) {
    w[tk][0] = wfrag(tk >> 1, tk & 1, 0);
    w[tk][1] = wfrag(tk >> 1, tk & 1, 1);
  }
  auto read_a = [&](int tk, bf16x8 (&a)[MTP]) {
    const int t = tk >> 1, kh = tk & 1;
    const int ky = t / 3, kx = t - 3 * ky;
    const int toffb = (ky * DZW + kx) * 128;
    const int gk = g + 4 * kh;
    const int sk = 2 * ky + kx;
#pragma unroll
    for (int k = 0; k < MTP; ++k)
      a[k] = *reinterpret_cast<const bf16x8*>(dzs + dbase[k] - toffb +
                                              ((gk ^ ((s0[k] - sk) & 7)) << 4));
  };
  bf16x8 a[2][MTP];
  read_a(0, a[0]);
#pragma unroll
  for (int tk = 0; tk < 18; ++tk) {
    __builtin_amdgcn_sched_barrier(0);   // keep each step's loads where they are issued
    if (tk + PF < 18) {
      w[tk + PF][0] = wfrag((tk + PF) >> 1, (tk + PF) & 1, 0);
      w[tk + PF][1] = wfrag((tk + PF) >> 1, (tk + PF) & 1, 1);
    }
    if (tk + 1 < 18) read_a(tk + 1, a[(tk + 1) & 1]);
#pragma unroll
    for (int k = 0; k < MTP; ++k) {
      acc[k][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[tk & 1][k], w[tk][0], acc[k][0], 0, 0, 0);
      acc[k][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[tk & 1][k], w[tk][1], acc[k][1], 0, 0, 0);
    }
  }
  const unsigned long long c1 = PDM_CLOCK();
  t_mf += c1 - c0;
  // epilogue per tile: relu'(a1) bitmask -> dz1 (bf16) -> conv1 wgrad on
  // mfma_f32_16x16x16_bf16 (M = ci, N = tap 0..8 / 9 = ones -> bias, K = pixels); the
  // dgrad accumulator (lane: ci = 16nt + i16, pixels 4g + r) is already its A operand.
  const int ctap = i16;
  const int cky = ctap / 3, ckx = ctap - 3 * cky;
  const int xoff = (ctap < 9) ? (cky * IMG + ckx) : IMG * IMG;
  const bf16 one = to_bf16(1.f);
#pragma unroll
  for (int k = 0; k < MTP; ++k) {
    const int P0 = (tile0 + 4 * k) * 16 + 4 * g;
    const int y0 = P0 / H1, x0 = P0 - y0 * H1;
    bf16x4 bx;
    uint32_t mw[4];
    bool valid[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool wrap = x0 + r >= H1;
      const int yr = wrap ? y0 + 1 : y0, xr = wrap ? x0 + r - H1 : x0 + r;
      valid[r] = P0 + r < P1;
      const int yc = valid[r] ? yr : 0, xc = valid[r] ? xr : 0;
      const int xi = (ctap < 9) ? yc * IMG + xc + xoff : IMG * IMG;
      bx[r] = xs[xi];
      mw[r] = mks[yc * H1 + xc];
    }
    if (ctap == 9) bx = bf16x4{one, one, one, one};
    bf16x4 az[2];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
        az[nt][r] = to_bf16((valid[r] && ((mw[r] >> (16 * nt + i16)) & 1u)) ? acc[k][nt][r] : 0.f);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
      acc1[nt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(az[nt], bx, acc1[nt], 0, 0, 0);
  }
  t_ep += PDM_CLOCK() - c1;
}

// Work split (per image, after the staged load): waves 0-3 run the conv2 wgrad (18 (tap,
// ci-tile) pairs), waves 4-7 the dgrad over 48 tile slots (43 real) in passes of DG_MTP.
// PDM_DG_SPLIT=16 moves dgrad tiles 0..15 onto the wgrad waves when a workgroup has one
// image.  Measured on MI355X (B=256, tools/kbench.py): split 0 / MTP 6 = 24.8 us, split 16 /
// MTP 8 = 24.8 us, split 16 / MTP 4 = 27.3 us, split 0 / MTP 4 = 27.4 us: the balance does not
// matter, the MFMAs per dgrad step do (the kernel is latency-bound at 2 waves per SIMD).
#ifndef PDM_DG_SPLIT
#define PDM_DG_SPLIT 0
#endif
constexpr int DG_SPLIT = PDM_DG_SPLIT;   // dgrad tiles done by the wgrad waves (0 or 16)
#ifndef PDM_DG_MTP
#define PDM_DG_MTP 6
#endif
constexpr int DG_MTP = PDM_DG_MTP;       // tiles per dgrad pass on waves 4-7

__global__ __launch_bounds__(BWD_THREADS, 1) void cnn_bwd_kernel(
    const uint8_t* __restrict__ xg, const float* __restrict__ w1, const float* __restrict__ b1,
    const bf16* __restrict__ dpool, const uint8_t* __restrict__ pmask,
    const bf16* __restrict__ w2t, int B, int ipb, float* __restrict__ slab, unsigned* xg_sync) {
  __shared__ __attribute__((aligned(16))) char smem[B_TOTAL];
  // xgmi streamed mode: this kernel starting means fc1_bwd finished, i.e. the fc
  // gradient bucket is complete -> hand it to the persistent collective (csrc/xgmi.h)
  if (xg_sync != nullptr && blockIdx.x == 0 && threadIdx.x == 0) xg_signal_ready(xg_sync, 0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, pq = i16 & 3;
  float* red = reinterpret_cast<float*>(smem + B_RED);
  const bf16* xs = reinterpret_cast<const bf16*>(smem + B_XS);
  const char* a1s = smem + B_A1;
  const char* dzs = smem + B_DZ;
  const uint32_t* mks = reinterpret_cast<const uint32_t*>(smem + B_MK);
  float* out = slab + (int64_t)blockIdx.x * CONV_SLAB;
  float db2p[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  f32x4 acc1[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  unsigned long long t_mf = 0, t_ep = 0;
  PDM_STAMP(0);

  if (wave < 4) {
    // ===== conv2 weight gradient: (tap, ci-tile) pairs {w, w+4, ...} x all 4 co tiles =====
    // K = output pixels in chunks of 8 along a row (24 = 3 chunks): lane group g of k-step
    // ks takes chunk 4ks+g; its lane q reads pixels x = col0+q and x+4 (col0 % 8 == 0), so
    // every swizzle term below is a per-lane constant and each read costs one add.
    f32x4 acc[5][4];
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bool five = wave < 2;  // 18 pairs over 4 waves: 5,5,4,4 (+1 discarded on 2,3)
    int cpair[5];
#pragma unroll
    for (int pi = 0; pi < 5; ++pi) {
      const int pair = min(wave + 4 * pi, 17);
      const int tap = pair >> 1, nt = pair & 1;
      const int ky = tap / 3, kx = tap - 3 * ky;
      cpair[pi] = (ky * H1 + kx) * 64 + (((2 * nt + (pq >> 1)) ^ ((q + kx) & 3)) << 4) + 8 * (pq & 1);
    }
    const int u8b = 8 * (pq & 1);
    auto wgrad_image = [&]() {
#pragma unroll 2
      for (int ks = 0; ks < P2 / 32; ++ks) {
        const int c8 = ks * 4 + g;
        const int row = c8 / 3;
        const int x = (c8 - 3 * row) * 8 + q;
        const int abase = (row * H1 + x) * 64;
        const int dbase = ((row + 2) * DZW + x + 2) * 128 + u8b;
        const int t = (((pq >> 1) ^ ((2 * row + x + 6) & 7)) << 4);
        bf16x8 A[4];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
          A[mt] = cat_tr(lds_tr16(dzs + dbase + ((32 * mt) ^ t)),
                         lds_tr16(dzs + dbase + 512 + ((32 * mt) ^ t ^ 64)));
#pragma unroll
        for (int pi = 0; pi < 5; ++pi) {   // waves 2,3: pair 4 is a discarded duplicate
          const bf16x8 Bv = cat_tr(lds_tr16(a1s + abase + cpair[pi]),
                                   lds_tr16(a1s + abase + cpair[pi] + 256));
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
            acc[pi][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[mt], Bv, acc[pi][mt], 0, 0, 0);
        }
      }
    };
    // dW2[co][tap][ci]: rows co = 16mt + 4g + r, col ci = 16nt + i16
    auto store_wgrad = [&]() {
#pragma unroll
      for (int pi = 0; pi < 5; ++pi) {
        if (pi == 4 && !five) break;
        const int pair = wave + 4 * pi;
        const int tap = pair >> 1, nt = pair & 1;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            out[(mt * 16 + 4 * g + r) * 288 + tap * 32 + nt * 16 + i16] = acc[pi][mt][r];
      }
    };
    if (ipb == 1) {
      // one image: wgrad, store it (frees its 80 accumulators), then dgrad tiles 0..15
      const int img = blockIdx.x;
      if (img < B) bwd_load_image(smem, img, xg, dpool, pmask, w1, b1, true, db2p);
      __syncthreads();
      PDM_STAMP(1);
      if (img < B) {
        wgrad_image();
        PDM_STAMP(2);
        store_wgrad();
        if (DG_SPLIT > 0) dgrad_pass<(DG_SPLIT > 0 ? DG_SPLIT / 4 : 1), 4>(dzs, mks, xs, w2t, wave, acc1, t_mf, t_ep);
      } else {
        store_wgrad();
      }
      PDM_STAMP(3);
      __syncthreads();
    } else {
      // several images: the wgrad accumulators persist across them; dgrad is all on 4-7
      for (int i = 0; i < ipb; ++i) {
        const int img = blockIdx.x * ipb + i;
        if (img < B) bwd_load_image(smem, img, xg, dpool, pmask, w1, b1, i == 0, db2p);
        __syncthreads();
        PDM_STAMP(1);
        if (img < B) wgrad_image();
        PDM_STAMP(3);
        __syncthreads();
      }
      store_wgrad();
    }
  } else {
    // ===== conv2 input gradient + relu'(a1) + conv1 weight/bias gradient =====
    const int wd = wave - 4;
    for (int i = 0; i < ipb; ++i) {
      const int img = blockIdx.x * ipb + i;
      if (img < B) bwd_load_image(smem, img, xg, dpool, pmask, w1, b1, i == 0, db2p);
      __syncthreads();
      if (img < B) {
        // tiles T0 + wd + 4j, j < (48 - T0) / 4, in passes of DG_MTP tiles; a rolled pass
        // loop keeps one copy of the pass code and stops cross-pass scheduling
        const int t0 = ipb > 1 ? 0 : DG_SPLIT;
        const int n = (48 - t0) / 4;
#pragma unroll 1
        for (int ps = 0; ps * DG_MTP < n; ++ps)
          dgrad_pass<DG_MTP, 4>(dzs, mks, xs, w2t, t0 + wd + 4 * DG_MTP * ps, acc1, t_mf, t_ep);
      }
      __syncthreads();
    }
    if (tid == 256) {
      PDM_STAMP_VAL(8, t_mf);
      PDM_STAMP_VAL(9, t_ep);
      PDM_STAMP_VAL(10, PDM_CLOCK());
    }
  }
  // conv1 weight/bias partials, acc1[nt]: rows ci = 16nt + 4g + r, col tap = i16.  Waves 4-7
  // write their slot, waves 0-3 then add theirs (slot = wave & 3).
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
  // conv2 bias: lanes sharing (lane & 7) hold the same 8 channels
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float v = db2p[j];
    v += __shfl_xor(v, 8, 64);
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (lane < 8) red[RED_DB2 + wave * C2 + lane * 8 + j] = v;
  }
  __syncthreads();
  PDM_STAMP(4);
  if (tid < C2) {
    float s = 0.f;
    for (int w = 0; w < 8; ++w) s += red[RED_DB2 + w * C2 + tid];
    out[SL_DB2 + tid] = s;
  } else if (tid >= 64 && tid < 64 + C1 * 10) {
    const int e = tid - 64;             // (ci, tap) with tap 0..8 = weight, 9 = bias
    const int ci = e / 10, t = e - 10 * ci;
    float s = 0.f;
    for (int w = 0; w < 4; ++w) s += red[RED_DW1 + w * C1 * 16 + ci * 16 + t];
    if (t < 9) out[SL_DW1 + ci * 9 + t] = s;
    else out[SL_DB1 + ci] = s;
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

}  // namespace

void launch_fc1_bwd(const __bf16* dh, const __bf16* dht, int ldt, const __bf16* pool,
                    const __bf16* wf1t, int B, float* gwf1, __bf16* dpool, const float* head_slab,
                    int head_blocks, float* gwf2, float* gbf2, float* gbf1, double* metrics,
                    hipStream_t st) {
  const int nd = (ldt / 32) * DX_TILES;
  int nblk = DW_TILES + nd + HR_BLOCKS, off = 0;
  // diagnostic only (tools/kbench.py): PDM_FC1BWD_ROLE=dw|dx|hr launches one role alone
  static const char* role = getenv("PDM_FC1BWD_ROLE");
  if (role && role[0] == 'd' && role[1] == 'w') nblk = DW_TILES;
  else if (role && role[0] == 'd' && role[1] == 'x') { nblk = nd; off = DW_TILES; }
  else if (role && role[0] == 'h') { nblk = HR_BLOCKS; off = DW_TILES + nd; }
  fc1_bwd_kernel<<<nblk, 256, 0, st>>>(dh, dht, ldt, pool, wf1t, B, gwf1, dpool, head_slab,
                                       head_blocks, gwf2, gbf2, gbf1, metrics, off);
}

int cnn_bwd_blocks(int B, int ipb) { return (B + ipb - 1) / ipb; }

void launch_cnn_bwd(const uint8_t* xg, const float* w1, const float* b1, const __bf16* dpool,
                    const uint8_t* pmask, const __bf16* w2t, int B, int ipb, float* slab,
                    unsigned* xg_sync, hipStream_t st) {
  cnn_bwd_kernel<<<cnn_bwd_blocks(B, ipb), BWD_THREADS, 0, st>>>(xg, w1, b1, dpool, pmask, w2t, B,
                                                                 ipb, slab, xg_sync);
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
