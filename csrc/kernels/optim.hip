// Fused flat-arena optimizer step (Adam / SGD-momentum) — one launch per step.
//
// torch runs Adam on GPU as ~7 _foreach_* launches with the bias corrections
// computed on the host.  This kernel sweeps the whole flat
// parameter arena once:
//   * DDP's 1/world_size gradient average is folded in as `grad_scale`,
//   * lr (fp64) and the step count live in device memory (graph-capturable;
//     the step counter was already advanced by an earlier kernel of the step),
//   * the op order matches torch's single-tensor Adam/SGD
//     (lerp / mul+addcmul / sqrt / div / add / addcdiv),
//   * optionally the same pass writes bf16 compute copies of the updated
//     weights: `shadow` (same layout) and `shadow_t` (2-D transposed), which the
//     bf16 forward/backward kernels read as MFMA operands. Transposed segments
//     are processed as 32x64 tiles staged through LDS so both the fp32 sweep and
//     the transposed bf16 store stay coalesced.
#include "common.h"
#include "kernels.h"
#include "optim_common.h"
#include "xgmi.h"

namespace {

using namespace optim_detail;

constexpr int CHUNK = 2048;  // elements per block for plain segments (256 thr x 8)
constexpr int TR = 32, TC = 64;

template <int KIND>
__global__ __launch_bounds__(256) void optim_kernel(OptArgs a) {
  // Every workgroup's prologue is a chain of scalar kernel-argument loads: the control
  // words and every segment's first_block are read up front (one batch, one wait), and the
  // selected segment is copied whole (a second batch) instead of field by field under the
  // branches below, each of which waited out its own load.
  double* const metrics = a.metrics;
  int64_t* const bump = a.bump;
  unsigned* const xgp = a.xg;
  const int nseg = a.nseg;
  int fb[OPT_MAX_SEG];
#pragma unroll
  for (int i = 0; i < OPT_MAX_SEG; ++i) fb[i] = a.seg[i].first_block;
  int si = 0;
#pragma unroll
  for (int i = 1; i < OPT_MAX_SEG; ++i)
    if (i < nseg && (int)blockIdx.x >= fb[i]) si = i;
  // pins the search (and the metrics pointer) ahead of the first branch: otherwise the
  // compiler sinks the first_block loads below the metrics test, a wait apiece
  asm volatile("" ::"s"(si), "s"(metrics));
  if (metrics != nullptr && blockIdx.x == gridDim.x - 1) {
    pdm_slab_metrics(a.mslab, a.mnslab, a.mcol, a.mstride, metrics);
    return;
  }
  const OptSeg s = a.seg[si];
  const int lb = blockIdx.x - s.first_block;
  // segment table: this workgroup lies inside its segment's block range
  PDM_CHECK(si < nseg && lb >= 0 &&
                (int)blockIdx.x < (si + 1 < nseg ? fb[si + 1]
                                                 : (int)gridDim.x - (metrics != nullptr ? 1 : 0)),
            "optim segment table", si, lb);
  if (bump != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *bump += 1;
  if (xgp != nullptr) {
    // xgmi streamed mode: publish the last bucket (every workgroup stores the same value,
    // so none depends on another being dispatched), then wait for this segment's bucket
    __shared__ int s_go;
    if (threadIdx.x == 0) {
      if (a.xg_signal_ch >= 0) xg_signal_ready(a.xg, a.xg_signal_ch);
      // no acquire: a waited segment reads its gradient with sc1 loads (gload below)
      s_go = s.wait_ch < 0 || xg_wait_done(a.xg, s.wait_ch, s.wait_mult, a.xg_timeout,
                                           /*acquire=*/false);
    }
    __syncthreads();
    if (!s_go) return;     // a peer never arrived: error bit set, the host raises
  }
  if (s.tonly) {
    // transpose-only: shadow_t = shadow^T for a TR x TC tile (bf16 in, bf16 out)
    __shared__ __attribute__((aligned(16))) bf16 tt[TC][TR + 8];
    const int tiles_c = (s.cols + TC - 1) / TC;
    const int tr0 = (lb / tiles_c) * TR, tc0 = (lb % tiles_c) * TC;
    // thread -> (row, 8 consecutive cols).  A fragment-major shadow holds this 32 x 64 tile
    // as two runs of 2 KB (n-tile, two k-steps): thread t reads the t-th 16-B chunk of them
    // (its (row, cols) follow from frag_pos), so the wave's loads stay whole-line.
    const int t = threadIdx.x;
    const int r = s.sfrag ? 16 * (t >> 7) + (t & 15) : t >> 3;
    const int c8 = s.sfrag ? 32 * ((t >> 6) & 1) + 8 * ((t >> 4) & 3) : (t & 7) * 8;
    const int row = tr0 + r, col0 = tc0 + c8;
    if (row < s.rows && col0 < s.cols) {
      const int64_t e = shadow_pos(s.sfrag, s.cols, row, col0);
      if (col0 + 8 <= s.cols && (e & 7) == 0) {
        const bf16x8 hb = *reinterpret_cast<const bf16x8*>(s.shadow + e);
#pragma unroll
        for (int j = 0; j < 8; ++j) tt[c8 + j][r] = hb[j];
      } else {
        for (int j = 0; j < 8 && col0 + j < s.cols; ++j)
          tt[c8 + j][r] = s.shadow[shadow_pos(s.sfrag, s.cols, row, col0 + j)];
      }
    }
    __syncthreads();
    const int c = threadIdx.x >> 2, rr = (threadIdx.x & 3) * 8;
    const int col = tc0 + c;
    if (col < s.cols) {
      const int64_t base = shadow_t_pos(s.tfrag, s.rows, tr0 + rr, col);
      if (tr0 + rr + 8 <= s.rows && (base & 7) == 0) {
        *reinterpret_cast<bf16x8*>(s.shadow_t + base) = *reinterpret_cast<const bf16x8*>(&tt[c][rr]);
      } else {
        for (int j = 0; j < 8 && tr0 + rr + j < s.rows; ++j)
          s.shadow_t[shadow_t_pos(s.tfrag, s.rows, tr0 + rr + j, col)] = tt[c][rr + j];
      }
    }
    return;
  }
  float* __restrict__ P = a.p + s.offset;
  const float* __restrict__ G = a.g + s.offset;
  float* __restrict__ M = a.m + s.offset;
  float* __restrict__ V = (KIND == OPT_ADAM) ? a.v + s.offset : nullptr;
  const int64_t numel = (int64_t)s.rows * s.cols;

  if (s.slab != nullptr) {
    // slab-reduced segment: 64 elements per workgroup; lane c4 = tid & 15 owns 4 of them
    // (float4), group rg = tid >> 4 sums slabs rg, rg + 16, ... (8 loads in flight), and
    // the 16 group sums are combined in a fixed order (the conv_reduce order, bit for bit)
    __shared__ float4 red[16][16];
    const int tid = threadIdx.x, c4 = tid & 15, rg = tid >> 4;
    const int e0 = lb * 64;
    // clamped to the segment's last float4 group (the slab row holds the whole group)
    const int col = s.slab_col0 + min(e0 + 4 * c4, (((int)numel + 3) & ~3) - 4);
    PDM_CHECK(col >= 0 && col + 4 <= s.slab_stride, "optim slab column", col, s.slab_stride);
    const float4* sp = reinterpret_cast<const float4*>(s.slab + col);
    const int64_t st4 = s.slab_stride / 4;
    // the update's operands are loaded ahead of the slab reduction (one memory round trip
    // fewer on the launch's critical path)
    const int e = e0 + tid;
    const int ec = min(e, (int)numel - 1);
    // unconditional (clamped) loads: loads under `tid < 64` made the compiler wait for them
    // at the branch join, i.e. before the slab loads below were even issued.  lr and the step
    // count are loaded here too: loaded by make_hyper after the reduction, they were one more
    // memory round trip on every workgroup's critical path.
    const double lr_in = *a.lr;
    const int64_t t_in = *a.step;
    const float p0 = P[ec], m0 = M[ec];
    const float v0 = (KIND == OPT_ADAM) ? V[ec] : 0.f;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int j0 = rg; j0 < s.nslab; j0 += 16 * 8) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = pdm_slab_load4(sp + (int64_t)min(j0 + 16 * u, s.nslab - 1) * st4);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const bool on = j0 + 16 * u < s.nslab;
        acc.x += on ? v[u].x : 0.f;
        acc.y += on ? v[u].y : 0.f;
        acc.z += on ? v[u].z : 0.f;
        acc.w += on ? v[u].w : 0.f;
      }
    }
    red[rg][c4] = acc;
    const Hyper h = make_hyper<KIND>(a, lr_in, t_in);
    __syncthreads();
    float gsum = 0.f;
    if (tid < 64) {
      // a valid element's float4 group is never a clamped one
      const float* rf = reinterpret_cast<const float*>(&red[0][0]);
#pragma unroll
      for (int gq = 0; gq < 16; ++gq) gsum += rf[gq * 64 + tid];
    }
    if (a.xx_on) {
      // world size > 1 over xGMI: this workgroup's 64 sums are all-reduced in-launch (one
      // flag slot per workgroup) before the update -- no conv_reduce launch, no hand-off
      __shared__ int s_xok;
      if (!xg_exchange(a.xx, blockIdx.x, s.offset + e - a.xx.off, tid < 64 && e < numel, gsum,
                       &s_xok))
        return;            // a peer never arrived: error bit set, the host raises
    }
    if (tid < 64 && e < numel) {
      const_cast<float*>(G)[e] = gsum;              // the reduced gradient stays observable
      float m = m0, v = v0;
      const float p = update<KIND>(p0, gsum, m, v, h, a.grad_scale);
      P[e] = p;
      M[e] = m;
      if (KIND == OPT_ADAM) V[e] = v;
      const bf16 hb = to_bf16(p);
      if (s.shadow) s.shadow[shadow_pos(s.sfrag, s.cols, e / s.cols, e % s.cols)] = hb;
      if (s.shadow_lo) s.shadow_lo[e] = to_bf16(p - from_bf16(hb));
      if (s.shadow_t) s.shadow_t[shadow_t_pos(s.tfrag, s.rows, e / s.cols, e % s.cols)] = hb;
    }
    return;
  }

  const Hyper h = make_hyper<KIND>(a);
  // a segment that waited for its bucket (xgmi streamed) reads the gradient with sc1 loads,
  // past this CU's L1, in place of an acquire after the wait: every byte of it was stored
  // write-through and drained before the collective's workgroups added to DONE
  // (MI355X_MICROARCH.md, the sc1 hand-off table)
  const bool gsc1 = xgp != nullptr && s.wait_ch >= 0;
  const __amdgpu_buffer_rsrc_t grs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(G), 0, 0x7fffffff, 0x00020000);
  auto gload4 = [&](int64_t e) __attribute__((always_inline)) {
    return gsc1 ? __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(grs, (int)(e * 4), 0, 16))
                : *reinterpret_cast<const float4*>(G + e);
  };
  auto gload1 = [&](int64_t e) __attribute__((always_inline)) {
    return gsc1 ? __hip_atomic_load(const_cast<float*>(G + e), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                : G[e];
  };
  if (s.shadow_t == nullptr && !s.sfrag) {
    // plain segment: 8 contiguous floats per thread (2 x float4)
    const int64_t e0 = (int64_t)lb * CHUNK + threadIdx.x * 8;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int64_t e = e0 + q * 4;
      if (e + 4 <= numel) {
        float4 p = *reinterpret_cast<float4*>(P + e);
        const float4 g = gload4(e);
        float4 m = *reinterpret_cast<float4*>(M + e);
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (KIND == OPT_ADAM) v = *reinterpret_cast<float4*>(V + e);
        p.x = update<KIND>(p.x, g.x, m.x, v.x, h, a.grad_scale);
        p.y = update<KIND>(p.y, g.y, m.y, v.y, h, a.grad_scale);
        p.z = update<KIND>(p.z, g.z, m.z, v.z, h, a.grad_scale);
        p.w = update<KIND>(p.w, g.w, m.w, v.w, h, a.grad_scale);
        *reinterpret_cast<float4*>(P + e) = p;
        *reinterpret_cast<float4*>(M + e) = m;
        if (KIND == OPT_ADAM) *reinterpret_cast<float4*>(V + e) = v;
        if (s.shadow) {
          bf16x4 hb = {to_bf16(p.x), to_bf16(p.y), to_bf16(p.z), to_bf16(p.w)};
          *reinterpret_cast<bf16x4*>(s.shadow + e) = hb;
          if (s.shadow_lo) {
            bf16x4 lb = {to_bf16(p.x - from_bf16(hb[0])), to_bf16(p.y - from_bf16(hb[1])),
                         to_bf16(p.z - from_bf16(hb[2])), to_bf16(p.w - from_bf16(hb[3]))};
            *reinterpret_cast<bf16x4*>(s.shadow_lo + e) = lb;
          }
        }
      } else {
        for (int64_t j = e; j < numel && j < e + 4; ++j) {
          float m = M[j], v = (KIND == OPT_ADAM) ? V[j] : 0.f;
          const float p = update<KIND>(P[j], gload1(j), m, v, h, a.grad_scale);
          P[j] = p;
          M[j] = m;
          if (KIND == OPT_ADAM) V[j] = v;
          if (s.shadow) s.shadow[j] = to_bf16(p);
          if (s.shadow_lo) s.shadow_lo[j] = to_bf16(p - from_bf16(to_bf16(p)));
        }
      }
    }
    return;
  }

  // transposed-shadow segment: tile of TR rows x TC cols.  Thread -> (row, 8 consecutive
  // cols): every fp32 load/store is a float4 and a row's 64 columns are 256 contiguous
  // bytes; the bf16 values are staged in LDS and written transposed as 16-B stores.
  __shared__ __attribute__((aligned(16))) bf16 tile[TC][TR + 8];
  const int tiles_c = (s.cols + TC - 1) / TC;
  const int tr0 = (lb / tiles_c) * TR, tc0 = (lb % tiles_c) * TC;
  const int r = threadIdx.x >> 3, c8 = (threadIdx.x & 7) * 8;
  const int row = tr0 + r, col0 = tc0 + c8;
  if (row < s.rows && col0 < s.cols) {
    const int64_t e = (int64_t)row * s.cols + col0;
    if (col0 + 8 <= s.cols && (e & 3) == 0) {
      float pv[8], gv[8], mv[8], vv[8];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const float4 p4 = *reinterpret_cast<const float4*>(P + e + 4 * q);
        const float4 g4 = gload4(e + 4 * q);
        const float4 m4 = *reinterpret_cast<const float4*>(M + e + 4 * q);
        pv[4 * q] = p4.x; pv[4 * q + 1] = p4.y; pv[4 * q + 2] = p4.z; pv[4 * q + 3] = p4.w;
        gv[4 * q] = g4.x; gv[4 * q + 1] = g4.y; gv[4 * q + 2] = g4.z; gv[4 * q + 3] = g4.w;
        mv[4 * q] = m4.x; mv[4 * q + 1] = m4.y; mv[4 * q + 2] = m4.z; mv[4 * q + 3] = m4.w;
        if (KIND == OPT_ADAM) {
          const float4 v4 = *reinterpret_cast<const float4*>(V + e + 4 * q);
          vv[4 * q] = v4.x; vv[4 * q + 1] = v4.y; vv[4 * q + 2] = v4.z; vv[4 * q + 3] = v4.w;
        } else {
          vv[4 * q] = vv[4 * q + 1] = vv[4 * q + 2] = vv[4 * q + 3] = 0.f;
        }
      }
      bf16x8 hb;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        pv[j] = update<KIND>(pv[j], gv[j], mv[j], vv[j], h, a.grad_scale);
        hb[j] = to_bf16(pv[j]);
        tile[c8 + j][r] = hb[j];
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        *reinterpret_cast<float4*>(P + e + 4 * q) =
            make_float4(pv[4 * q], pv[4 * q + 1], pv[4 * q + 2], pv[4 * q + 3]);
        *reinterpret_cast<float4*>(M + e + 4 * q) =
            make_float4(mv[4 * q], mv[4 * q + 1], mv[4 * q + 2], mv[4 * q + 3]);
        if (KIND == OPT_ADAM)
          *reinterpret_cast<float4*>(V + e + 4 * q) =
              make_float4(vv[4 * q], vv[4 * q + 1], vv[4 * q + 2], vv[4 * q + 3]);
      }
      if (s.shadow) *reinterpret_cast<bf16x8*>(s.shadow + shadow_pos(s.sfrag, s.cols, row, col0)) = hb;
    } else {
      for (int j = 0; j < 8 && col0 + j < s.cols; ++j) {
        const int64_t ej = e + j;
        float m = M[ej], v = (KIND == OPT_ADAM) ? V[ej] : 0.f;
        const float p = update<KIND>(P[ej], gload1(ej), m, v, h, a.grad_scale);
        P[ej] = p;
        M[ej] = m;
        if (KIND == OPT_ADAM) V[ej] = v;
        const bf16 hb = to_bf16(p);
        if (s.shadow) s.shadow[shadow_pos(s.sfrag, s.cols, row, col0 + j)] = hb;
        tile[c8 + j][r] = hb;
      }
    }
  }
  if (s.shadow_t == nullptr) return;   // fragment-major shadow only (a row shard of W1)
  __syncthreads();
  // transposed store: thread -> (col c, 8 consecutive rows) = one 16-B store
  const int c = threadIdx.x >> 2, rr = (threadIdx.x & 3) * 8;
  const int col = tc0 + c;
  if (col < s.cols) {
    const int64_t base = shadow_t_pos(s.tfrag, s.rows, tr0 + rr, col);
    if (tr0 + rr + 8 <= s.rows && (base & 7) == 0) {
      *reinterpret_cast<bf16x8*>(s.shadow_t + base) = *reinterpret_cast<const bf16x8*>(&tile[c][rr]);
    } else {
      for (int j = 0; j < 8 && tr0 + rr + j < s.rows; ++j)
        s.shadow_t[shadow_t_pos(s.tfrag, s.rows, tr0 + rr + j, col)] = tile[c][rr + j];
    }
  }
}

}  // namespace

int opt_blocks_for(const OptSeg& s) {
  if (s.slab) return (int)(((int64_t)s.rows * s.cols + 63) / 64);
  if (s.shadow_t || s.tonly || s.sfrag) return ((s.rows + TR - 1) / TR) * ((s.cols + TC - 1) / TC);
  const int64_t n = (int64_t)s.rows * s.cols;
  return (int)((n + CHUNK - 1) / CHUNK);
}

void launch_optim(int kind, OptArgs& a, hipStream_t st) {
  int total = 0;
  for (int i = 0; i < a.nseg; ++i) {
    a.seg[i].first_block = total;
    total += opt_blocks_for(a.seg[i]);
  }
  if (total == 0) return;
  if (a.metrics != nullptr) total += 1;   // the metrics workgroup (last)
  if (kind == OPT_ADAM)
    optim_kernel<OPT_ADAM><<<total, 256, 0, st>>>(a);
  else
    optim_kernel<OPT_SGD><<<total, 256, 0, st>>>(a);
}
