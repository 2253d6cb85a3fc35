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

namespace {

using namespace cnn;

// ------------------------------------------------------------------ fc1_bwd
constexpr int DW_TILES = FEAT / 64;  // 144

__device__ __forceinline__ int tile_off(int row, int byte) {  // [32 rows][128 B], 2-way-free tr reads
  return row * 128 + (byte ^ (((row >> 3) & 1) << 5));
}

__global__ __launch_bounds__(256) void fc1_bwd_kernel(
    const bf16* __restrict__ dh, const bf16* __restrict__ dht, int ldt,
    const bf16* __restrict__ pool, const bf16* __restrict__ wf1t, int B, float* __restrict__ gwf1,
    bf16* __restrict__ dpool, const float* __restrict__ head_slab, int head_blocks,
    float* __restrict__ gwf2, float* __restrict__ gbf2, float* __restrict__ gbf1,
    double* __restrict__ metrics) {
  __shared__ __attribute__((aligned(16))) char tile[32 * 128];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, pq = i16 & 3;
  const int nd = (ldt / 32) * DW_TILES;
  const int bid = blockIdx.x;

  if (bid < DW_TILES) {
    // ---- dW1 tile: all 128 hidden rows x 64 feature columns, K = batch ----
    const int k0 = bid * 64;
    f32x4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int srow = tid >> 3, sch = tid & 7;
    for (int b0 = 0; b0 < ldt; b0 += 32) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (b0 + srow < B)
        v = *reinterpret_cast<const uint4*>(pool + (int64_t)(b0 + srow) * FEAT + k0 + sch * 8);
      __syncthreads();
      *reinterpret_cast<uint4*>(tile + tile_off(srow, sch * 16)) = v;
      __syncthreads();
      bf16x8 a[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
        a[mt] = *reinterpret_cast<const bf16x8*>(dht + (int64_t)(wave * 32 + mt * 16 + i16) * ldt +
                                                 b0 + 8 * g);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const s16x4 lo = lds_tr16(tile + tile_off(8 * g + q, 32 * nt + 8 * pq));
        const s16x4 hi = lds_tr16(tile + tile_off(8 * g + 4 + q, 32 * nt + 8 * pq));
        const bf16x8 bv = cat_tr(lo, hi);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt], bv, acc[mt][nt], 0, 0, 0);
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
    // ---- dX tile: 32 batch rows x 64 feature columns, K = 128 hidden ----
    const int t = bid - DW_TILES;
    const int b0 = (t / DW_TILES) * 32, k0 = (t % DW_TILES) * 64 + wave * 16;
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int ks = 0; ks < HID / 32; ++ks) {
      const bf16x8 wv =
          *reinterpret_cast<const bf16x8*>(wf1t + (int64_t)(k0 + i16) * HID + 32 * ks + 8 * g);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const bf16x8 av =
            *reinterpret_cast<const bf16x8*>(dh + (int64_t)(b0 + mt * 16 + i16) * HID + 32 * ks + 8 * g);
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, wv, acc[mt], 0, 0, 0);
      }
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = b0 + mt * 16 + 4 * g + r;
        if (row < B) dpool[(int64_t)row * FEAT + k0 + i16] = to_bf16(acc[mt][r]);
      }
    return;
  }

  // ---- head slab reduction (one block) ----
  for (int e = tid; e < HEAD_SLAB; e += 256) {
    float s = 0.f;
    double sd = 0.0;
    for (int j = 0; j < head_blocks; ++j) {
      const float v = head_slab[(int64_t)j * HEAD_SLAB + e];
      s += v;
      sd += (double)v;
    }
    if (e < NCLS * HID) gwf2[e] = s;
    else if (e < NCLS * HID + NCLS) gbf2[e - NCLS * HID] = s;
    else if (e < NCLS * HID + NCLS + HID) gbf1[e - NCLS * HID - NCLS] = s;
    else if (e == HEAD_SLAB - 2) { metrics[0] += sd; metrics[2] += (double)B; }
    else metrics[1] += sd;
  }
}

// ------------------------------------------------------------------ cnn_bwd
constexpr int BWD_THREADS = 512;
constexpr int B_XS = 0;                         // fp32 [784]            3136
constexpr int B_A1 = 3136;                      // a1 image              43264
constexpr int B_DZ = B_A1 + P1 * 64;            // dz2 image             73728
constexpr int B_RED = B_DZ + P2 * 128;          // fp32 reduction scratch
constexpr int RED_DB2 = 0;                      // [8 waves][64]
constexpr int RED_DW1 = RED_DB2 + 8 * C2;       // [4 waves][288]
constexpr int RED_DB1 = RED_DW1 + 4 * C1 * 9;   // [4 waves][32]
constexpr int RED_N = RED_DB1 + 4 * C1;         // 1792 floats
constexpr int B_TOTAL = B_RED + RED_N * 4;      // 127296 B -> 1 workgroup / CU
constexpr int SL_DB2 = C2 * 9 * C1;             // 18432
constexpr int SL_DW1 = SL_DB2 + C2;             // 18496
constexpr int SL_DB1 = SL_DW1 + C1 * 9;         // 18784

// Stage one image into LDS: x (fp32), a1 (swizzled), dz2 (expanded from the pooled
// gradient and the argmax|positive mask), and accumulate the conv2 bias gradient.
__device__ __forceinline__ void bwd_load_image(char* smem, int img, const uint8_t* __restrict__ xg,
                                               const bf16* __restrict__ a1g,
                                               const bf16* __restrict__ dpool,
                                               const uint8_t* __restrict__ pmask, float (&db2p)[8]) {
  const int tid = threadIdx.x;
  float* xs = reinterpret_cast<float*>(smem + B_XS);
  char* a1s = smem + B_A1;
  char* dzs = smem + B_DZ;
  if (tid < 196) {
    const uint32_t w = reinterpret_cast<const uint32_t*>(xg + (int64_t)img * 784)[tid];
    float4 v;
    v.x = pdm_normalize(w & 0xff);
    v.y = pdm_normalize((w >> 8) & 0xff);
    v.z = pdm_normalize((w >> 16) & 0xff);
    v.w = pdm_normalize(w >> 24);
    reinterpret_cast<float4*>(xs)[tid] = v;
  }
  const uint4* a1v = reinterpret_cast<const uint4*>(a1g + (int64_t)img * P1 * C1);
  for (int c = tid; c < P1 * 4; c += BWD_THREADS) {
    const int pix = c >> 2, ch = c & 3;
    const int row = pix / H1, col = pix - row * H1;
    *reinterpret_cast<uint4*>(a1s + a1_off(row, col, ch * 16)) = a1v[c];
  }
  const uint4* dpv = reinterpret_cast<const uint4*>(dpool + (int64_t)img * FEAT);
  const uint2* mkv = reinterpret_cast<const uint2*>(pmask + (int64_t)img * FEAT);
  for (int it = tid; it < PP * 8; it += BWD_THREADS) {  // it & 7 == tid & 7 (fixed channel chunk)
    const int pp = it >> 3, ch = it & 7;
    const int py = pp / HP, px = pp - py * HP;
    const uint4 d = dpv[it];
    const uint2 mk = mkv[it];
    const uint16_t dv[8] = {(uint16_t)(d.x & 0xffff), (uint16_t)(d.x >> 16), (uint16_t)(d.y & 0xffff),
                            (uint16_t)(d.y >> 16),    (uint16_t)(d.z & 0xffff), (uint16_t)(d.z >> 16),
                            (uint16_t)(d.w & 0xffff), (uint16_t)(d.w >> 16)};
    const uint8_t mb[8] = {(uint8_t)(mk.x & 0xff), (uint8_t)((mk.x >> 8) & 0xff),
                           (uint8_t)((mk.x >> 16) & 0xff), (uint8_t)(mk.x >> 24),
                           (uint8_t)(mk.y & 0xff), (uint8_t)((mk.y >> 8) & 0xff),
                           (uint8_t)((mk.y >> 16) & 0xff), (uint8_t)(mk.y >> 24)};
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (mb[j] & 0x80) db2p[j] += __builtin_bit_cast(float, (uint32_t)dv[j] << 16);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      uint32_t w[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t lo = ((mb[2 * j] & 0x83) == (0x80 | s)) ? dv[2 * j] : 0u;
        const uint32_t hi = ((mb[2 * j + 1] & 0x83) == (0x80 | s)) ? dv[2 * j + 1] : 0u;
        w[j] = lo | (hi << 16);
      }
      *reinterpret_cast<uint4*>(dzs + dz_off(2 * py + (s >> 1), 2 * px + (s & 1), ch * 16)) =
          make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

__global__ __launch_bounds__(BWD_THREADS, 1) void cnn_bwd_kernel(
    const uint8_t* __restrict__ xg, const bf16* __restrict__ a1g, const bf16* __restrict__ dpool,
    const uint8_t* __restrict__ pmask, const bf16* __restrict__ w2t, int B, int ipb,
    float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) char smem[B_TOTAL];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, pq = i16 & 3;
  float* red = reinterpret_cast<float*>(smem + B_RED);
  const float* xs = reinterpret_cast<const float*>(smem + B_XS);
  const char* a1s = smem + B_A1;
  const char* dzs = smem + B_DZ;
  float* out = slab + (int64_t)blockIdx.x * CONV_SLAB;
  float db2p[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

  if (wave < 4) {
    // ===== conv2 weight gradient: (tap, ci-tile) pairs {w, w+4, ...} x all 4 co tiles =====
    f32x4 acc[5][4];
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bool five = wave < 2;  // 18 pairs over 4 waves: 5,5,4,4
    for (int i = 0; i < ipb; ++i) {
      const int img = blockIdx.x * ipb + i;
      if (img < B) bwd_load_image(smem, img, xg, a1g, dpool, pmask, db2p);
      __syncthreads();
      if (img < B) {
        for (int ks = 0; ks < P2 / 32; ++ks) {
          const int pa = ks * 32 + 8 * g + q, pb = pa + 4;
          const int ya = pa / H2, xa = pa - ya * H2, yb = pb / H2, xb = pb - yb * H2;
          bf16x8 A[4];
#pragma unroll
          for (int mt = 0; mt < 4; ++mt)
            A[mt] = cat_tr(lds_tr16(dzs + dz_off(ya, xa, mt * 32 + 8 * pq)),
                           lds_tr16(dzs + dz_off(yb, xb, mt * 32 + 8 * pq)));
#pragma unroll
          for (int pi = 0; pi < 5; ++pi) {
            if (pi == 4 && !five) break;
            const int pair = wave + 4 * pi;
            const int tap = pair >> 1, nt = pair & 1;
            const int ky = tap / 3, kx = tap - ky * 3;
            const bf16x8 Bv = cat_tr(lds_tr16(a1s + a1_off(ya + ky, xa + kx, nt * 32 + 8 * pq)),
                                     lds_tr16(a1s + a1_off(yb + ky, xb + kx, nt * 32 + 8 * pq)));
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
              acc[pi][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[mt], Bv, acc[pi][mt], 0, 0, 0);
          }
        }
      }
      __syncthreads();
    }
    // dW2[co][tap][ci]: rows co = 16mt + 4g + r, col ci = 16nt + i16
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
  } else {
    // ===== conv2 input gradient + relu'(a1) + conv1 weight/bias gradient =====
    const int wd = wave - 4;
    bf16x8 wt[9][2][2];  // B[k = co][n = ci] = W2^T[tap][ci][co]
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          wt[t][kh][nt] = *reinterpret_cast<const bf16x8*>(
              w2t + (t * C1 + nt * 16 + i16) * C2 + 32 * kh + 8 * g);
    float dw1p[2][9], db1p[2] = {0.f, 0.f};
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int t = 0; t < 9; ++t) dw1p[nt][t] = 0.f;
    const bf16x8 zero8 = {};
    for (int i = 0; i < ipb; ++i) {
      const int img = blockIdx.x * ipb + i;
      if (img < B) bwd_load_image(smem, img, xg, a1g, dpool, pmask, db2p);
      __syncthreads();
      if (img < B) {
        for (int mt = wd; mt < (P1 + 15) / 16; mt += 4) {
          const int P = mt * 16 + i16;
          const int y = P / H1, x = P - y * H1;
          const bool vP = P < P1;
          f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
          for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
              const int oy = y - ky, ox = x - kx;
              const bool v = vP && oy >= 0 && oy < H2 && ox >= 0 && ox < H2;
              const int oyc = v ? oy : 0, oxc = v ? ox : 0;
#pragma unroll
              for (int kh = 0; kh < 2; ++kh) {
                bf16x8 a = *reinterpret_cast<const bf16x8*>(dzs + dz_off(oyc, oxc, (g + 4 * kh) * 16));
                a = v ? a : zero8;
#pragma unroll
                for (int nt = 0; nt < 2; ++nt)
                  acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wt[ky * 3 + kx][kh][nt],
                                                                    acc[nt], 0, 0, 0);
              }
            }
          // epilogue: lane holds pixels mt*16 + 4g + r, channel ci = 16nt + i16
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int Pr = mt * 16 + 4 * g + r;
            if (Pr < P1) {
              const int yr = Pr / H1, xr = Pr - yr * H1;
              float xv[9];
#pragma unroll
              for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) xv[ky * 3 + kx] = xs[(yr + ky) * IMG + xr + kx];
#pragma unroll
              for (int nt = 0; nt < 2; ++nt) {
                const int ci = nt * 16 + i16;
                const bf16 av = *reinterpret_cast<const bf16*>(a1s + a1_off(yr, xr, ci * 2));
                const float dz1 = (from_bf16(av) > 0.f) ? acc[nt][r] : 0.f;
                db1p[nt] += dz1;
#pragma unroll
                for (int t = 0; t < 9; ++t) dw1p[nt][t] = fmaf(dz1, xv[t], dw1p[nt][t]);
              }
            }
          }
        }
      }
      __syncthreads();
    }
    // reduce over the 4 lanes sharing a channel (g = 0..3), then per-wave scratch
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      float v = db1p[nt];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (g == 0) red[RED_DB1 + wd * C1 + nt * 16 + i16] = v;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        float u = dw1p[nt][t];
        u += __shfl_xor(u, 16, 64);
        u += __shfl_xor(u, 32, 64);
        if (g == 0) red[RED_DW1 + wd * C1 * 9 + (nt * 16 + i16) * 9 + t] = u;
      }
    }
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
  if (tid < C2) {
    float s = 0.f;
    for (int w = 0; w < 8; ++w) s += red[RED_DB2 + w * C2 + tid];
    out[SL_DB2 + tid] = s;
  } else if (tid >= 64 && tid < 64 + C1 * 9) {
    const int e = tid - 64;
    float s = 0.f;
    for (int w = 0; w < 4; ++w) s += red[RED_DW1 + w * C1 * 9 + e];
    out[SL_DW1 + e] = s;
  } else if (tid >= 384 && tid < 384 + C1) {
    const int e = tid - 384;
    float s = 0.f;
    for (int w = 0; w < 4; ++w) s += red[RED_DB1 + w * C1 + e];
    out[SL_DB1 + e] = s;
  }
}

// ------------------------------------------------------------------ conv_reduce
__global__ __launch_bounds__(256) void conv_reduce_kernel(const float* __restrict__ slab, int nblk,
                                                          float* __restrict__ gw2,
                                                          float* __restrict__ gb2,
                                                          float* __restrict__ gw1,
                                                          float* __restrict__ gb1) {
  // block = 256 consecutive slab columns; each thread sums every slab for 1 column with
  // 8 independent accumulators (8 loads in flight), fixed order -> deterministic.
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= CONV_SLAB) return;
  const float* p = slab + e;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int j = 0;
  for (; j + 8 <= nblk; j += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] += p[(int64_t)(j + u) * CONV_SLAB];
  }
  for (; j < nblk; ++j) acc[0] += p[(int64_t)j * CONV_SLAB];
  const float t = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  if (e < SL_DB2) gw2[e] = t;
  else if (e < SL_DW1) gb2[e - SL_DB2] = t;
  else if (e < SL_DB1) gw1[e - SL_DW1] = t;
  else gb1[e - SL_DB1] = t;
}

}  // namespace

void launch_fc1_bwd(const __bf16* dh, const __bf16* dht, int ldt, const __bf16* pool,
                    const __bf16* wf1t, int B, float* gwf1, __bf16* dpool, const float* head_slab,
                    int head_blocks, float* gwf2, float* gbf2, float* gbf1, double* metrics,
                    hipStream_t st) {
  const int nblk = DW_TILES + (ldt / 32) * DW_TILES + 1;
  fc1_bwd_kernel<<<nblk, 256, 0, st>>>(dh, dht, ldt, pool, wf1t, B, gwf1, dpool, head_slab,
                                       head_blocks, gwf2, gbf2, gbf1, metrics);
}

int cnn_bwd_blocks(int B, int ipb) { return (B + ipb - 1) / ipb; }

void launch_cnn_bwd(const uint8_t* xg, const __bf16* a1, const __bf16* dpool, const uint8_t* pmask,
                    const __bf16* w2t, int B, int ipb, float* slab, hipStream_t st) {
  cnn_bwd_kernel<<<cnn_bwd_blocks(B, ipb), BWD_THREADS, 0, st>>>(xg, a1, dpool, pmask, w2t, B, ipb,
                                                                 slab);
}

void launch_conv_reduce(const float* slab, int nblk, float* gw2, float* gb2, float* gw1, float* gb1,
                        hipStream_t st) {
  conv_reduce_kernel<<<(CONV_SLAB + 255) / 256, 256, 0, st>>>(slab, nblk, gw2, gb2, gw1, gb1);
}
