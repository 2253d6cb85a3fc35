// The fc1-weight SGD update of the PREVIOUS step, run by extra workgroups of the forward
// launch (world size > 1, "carried" update; runtime/cnn_step.py CnnStep._fwd_carry_on).
//
// At world size > 1 the fc1 update (4.7 MB of gradients, 28 MB of fp32 weight / momentum /
// bf16-copy traffic) cannot run inside fc1_bwd as it does at world size 1: it needs the
// all-reduced gradient.  In the optimizer launch it is bandwidth-bound work on the step's
// critical path (the B = 32 optimizer: 7.6 us with it, 5.2 without, RCCL nocarry;
// profiles/r5/fc1_carry/).  The next step's first
// kernel, the conv forward, does not read W1, and at the batches the forward is run at it
// fills at most half of the chip's workgroup slots (two 512-thread workgroups per CU), so the
// update's workgroups are appended to its grid and stream beside the conv workgroups; fc1_fwd
// (the first reader of W1) comes after the launch.  Same tile scheme, same op order and same
// bits as the optimizer's transposed-shadow segment (optim.hip): a 512-thread workgroup runs
// two 32 x 64 tiles at a time, one per 256-thread half, and writes W1 (fragment-major, 16-B
// stores) and W1^T (through an LDS transpose, 16-B stores).
#pragma once
#include "cnn_common.h"
#include "optim_common.h"
#include "xgmi.h"

namespace cnn {

constexpr int FCC_TR = 32, FCC_TC = 64;
constexpr int FCC_TILES = (HID / FCC_TR) * (FEAT / FCC_TC);   // 576
// two transpose tiles of [FCC_TC][FCC_TR] bf16 (8 KB); the 16-B chunk k of row c is stored
// at chunk k ^ ((c >> 3) & 3): the column-wise 2-B writes of a wave (8 rows, 8 apart) spread
// over 4 chunk positions instead of one bank group, 2-way instead of 8-way, and the row-wise
// 16-B reads are conflict-free (tools/lds_bank_model.py; the padded layout: 8-way / 3-way)
constexpr int FCC_LDS = 2 * FCC_TC * FCC_TR * 2;
__device__ __forceinline__ int fcc_tpos(int c, int col) {
  return c * FCC_TR + ((((col >> 3) ^ (c >> 3)) & 3) << 3) + (col & 7);
}
// update workgroups, two pairs of tiles each (288 workgroups of one pair were slower at
// B = 32, where they would still fit one round beside the band workgroups:
// profiles/r5/fc1_carry/)
constexpr int FCC_WGS = FCC_TILES / 4;

// workgroup wg of nwg (512 threads); smem: FCC_LDS + 4 bytes of the launch's LDS
__device__ __forceinline__ void fc_carry_role(const FcUpdate& u, int wg, int nwg, char* smem) {
  // xgmi streamed mode: the fc1-weight channel may still be travelling (the optimizer no
  // longer waits for it).  One lane polls its DONE count, the workgroup follows it through a
  // barrier, and the gradient is then read with sc1 loads (past this CU's L1) instead of
  // behind an acquire: every byte of it was stored write-through and drained before the
  // collective's workgroups added to DONE (MI355X_MICROARCH.md, the sc1 hand-off table)
  const bool sc1 = u.wloc != nullptr;
  if (sc1) {
    int* s_ok = reinterpret_cast<int*>(smem + FCC_LDS);
    if (threadIdx.x == 0) *s_ok = xg_wait_done(u.wloc, u.wch, u.wmult, u.wtimeout, /*acquire=*/false);
    __syncthreads();
    if (!*s_ok) return;     // a peer never arrived: error bit set, the host raises
  }
  const __amdgpu_buffer_rsrc_t grs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(u.g), 0, 0x7fffffff, 0x00020000);
  const int half = threadIdx.x >> 8, t = threadIdx.x & 255;
  bf16* tile = reinterpret_cast<bf16*>(smem + half * FCC_TC * FCC_TR * 2);
  const optim_detail::Hyper h = optim_detail::make_hyper<OPT_SGD>(u, *u.lr, *u.step);
  constexpr int tiles_c = FEAT / FCC_TC;
  const int r = t >> 3, c8 = (t & 7) * 8;
  // trip count uniform over the workgroup (both halves pass the same barriers)
  for (int base = 2 * wg; base < FCC_TILES; base += 2 * nwg) {
    const int lb = base + half;
    const int tr0 = (lb / tiles_c) * FCC_TR, tc0 = (lb % tiles_c) * FCC_TC;
    if (lb < FCC_TILES) {
      const int row = tr0 + r, col0 = tc0 + c8;
      PDM_CHECK(row < HID && col0 + 8 <= FEAT, "fc_carry tile position", row, col0);
      PDM_CHECK(fcc_tpos(c8 + 7, r) < FCC_TC * FCC_TR, "fc_carry LDS transpose slot", c8, r);
      const int64_t e = (int64_t)row * FEAT + col0;
      float pv[8], gv[8], mv[8];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const float4 p4 = *reinterpret_cast<const float4*>(u.p + e + 4 * q);
        const float4 g4 =
            sc1 ? __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                      grs, (int)((e + 4 * q) * 4), 0, 16))                   // aux 16: sc1
                : *reinterpret_cast<const float4*>(u.g + e + 4 * q);
        const float4 m4 = *reinterpret_cast<const float4*>(u.m + e + 4 * q);
        pv[4 * q] = p4.x; pv[4 * q + 1] = p4.y; pv[4 * q + 2] = p4.z; pv[4 * q + 3] = p4.w;
        gv[4 * q] = g4.x; gv[4 * q + 1] = g4.y; gv[4 * q + 2] = g4.z; gv[4 * q + 3] = g4.w;
        mv[4 * q] = m4.x; mv[4 * q + 1] = m4.y; mv[4 * q + 2] = m4.z; mv[4 * q + 3] = m4.w;
      }
      bf16x8 hb;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = 0.f;
        pv[j] = optim_detail::update<OPT_SGD>(pv[j], gv[j], mv[j], v, h, u.grad_scale);
        hb[j] = to_bf16(pv[j]);
        tile[fcc_tpos(c8 + j, r)] = hb[j];
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        *reinterpret_cast<float4*>(u.p + e + 4 * q) =
            make_float4(pv[4 * q], pv[4 * q + 1], pv[4 * q + 2], pv[4 * q + 3]);
        *reinterpret_cast<float4*>(u.m + e + 4 * q) =
            make_float4(mv[4 * q], mv[4 * q + 1], mv[4 * q + 2], mv[4 * q + 3]);
      }
      *reinterpret_cast<bf16x8*>(u.shadow + shadow_pos(1, FEAT, row, col0)) = hb;
    }
    __syncthreads();
    if (lb < FCC_TILES) {
      // transposed store: thread -> (col c, 8 consecutive rows) = one 16-B store
      const int c = t >> 2, rr = (t & 3) * 8;
      PDM_CHECK(tr0 + rr + 8 <= HID && tc0 + c < FEAT, "fc_carry transposed tile", tr0 + rr,
                tc0 + c);
      *reinterpret_cast<bf16x8*>(u.shadow_t_next + shadow_t_pos(1, HID, tr0 + rr, tc0 + c)) =
          *reinterpret_cast<const bf16x8*>(&tile[fcc_tpos(c, rr)]);
    }
    __syncthreads();
  }
}

}  // namespace cnn
