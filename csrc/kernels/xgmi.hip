// Direct xGMI all-reduce kernel (protocol: csrc/xgmi.h).
//
// Why not RCCL for the 4.7 MB fc bucket: RCCL's all-reduce kernel needs 19.7 KB
// of LDS and ~280 registers per lane (docs/kernels.md), so it cannot share a CU
// with cnn_bwd and the fc gradients can only travel after the whole backward.
// This kernel uses one LDS word and at most 48 registers per lane (waves_per_eu
// 10), which fits in what cnn_bwd leaves free on every CU, so it runs *beside*
// cnn_bwd; and its push schedule moves the bucket over all N-1 point-to-point
// links at once instead of one link per ring step.
//
// Memory-model recipe (system scope, gfx950):
//   payload  16-B buffer stores with sc0 sc1 (write-through to the owning HBM),
//            each storing wave drains them (s_waitcnt vmcnt(0)), workgroup barrier;
//   signal   one relaxed system-scope store of the call generation per peer flag;
//   consume  one wave polls its peers' flags (relaxed system-scope loads, s_sleep),
//            then a system-scope acquire (buffer_inv sc0 sc1) and a barrier before
//            any wave loads the handed-off bytes.
// All hand-off memory is uncached (hipDeviceMallocUncached), so no L2 on either
// side can hold a stale copy across calls.  Every spin is bounded: past
// `timeout` ticks the workgroup records its cause in `err` (XG_ERR_*; the first
// cause also in XG_LOC_FIRST) and exits, so a dead peer turns into a host-visible
// error instead of a hung GPU.
#include "common.h"
#include "xgmi.h"

namespace {

constexpr int XG_SC0_SC1 = 17;              // aux bits of a system-scope write-through store
constexpr int XG_RSRC_W3 = 0x00020000;      // raw buffer descriptor word 3 (gfx9 family)

__device__ __forceinline__ unsigned flag_load(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void flag_store(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(float* base) {
  return __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, XG_RSRC_W3);
}

__device__ __forceinline__ void store_wt(__amdgpu_buffer_rsrc_t r, int i4, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, i4 * 16, 0, XG_SC0_SC1);
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) {
  return v < lo ? lo : (v > hi ? hi : v);
}

// Every storing wave drains its write-through stores, then one lane publishes the
// generation into each peer's flag block.
__device__ __forceinline__ void signal_peers(const XgmiArgs& a, int ph, int w, unsigned gen) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int d = 0; d < a.nranks; ++d)
      if (d != a.rank) flag_store(a.flags[d] + xg_flag_idx(a.ch, ph, a.rank, w), gen);
  }
}

// Every wave polls this rank's flags from every peer until each reaches `gen` (or the
// deadline passes), then acquires for itself.  No LDS anywhere in these kernels: cnn_bwd
// takes 163,200 of a CU's 163,840 LDS bytes, and a collective workgroup holding even one
// LDS allocation granule on a CU keeps cnn_bwd's workgroup off that CU for the whole
// persistent launch (256 workgroups on the remaining CUs = two rounds: cnn_bwd 17 -> 30 us at
// B = 256, whatever the collective's width; profiles/r5/xgmi_cost).
__device__ __forceinline__ bool wait_peers(const XgmiArgs& a, int ph, int w, unsigned gen,
                                           long long deadline) {
  const int lane = threadIdx.x & (PDM_WAVE - 1);
  const bool mine = lane < a.nranks && lane != a.rank;
  const unsigned* f = a.flags[a.rank] + xg_flag_idx(a.ch, ph, mine ? lane : 0, w);
  unsigned cause = 0;
  for (unsigned it = 0;; ++it) {
    // the error word is read on the first poll and every 64th: a wait that starts after
    // any wait of this rank gave up fails at once, so one missing peer costs one timeout
    const unsigned e = xg_poll_err(it) ? __builtin_amdgcn_readfirstlane(flag_load(a.err)) : 0u;
    const bool arrived = !mine || (int)(flag_load(f) - gen) >= 0;
    if (e != 0) {
      cause = XG_ERR_FAILFAST;
      break;
    }
    if (__all(arrived)) break;
    if ((long long)__builtin_amdgcn_s_memrealtime() > deadline) {
      cause = ph == 0 ? XG_ERR_PEER0 : XG_ERR_PEER1;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  if (a.nranks > 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // buffer_inv sc0 sc1
  if (lane == 0 && cause != 0) xg_record_error(a.err, cause);
  return cause == 0;
}

// One channel's all-reduce for workgroup w of W (its slice of every chunk) at call
// generation `gen`; false when a peer did not arrive before the deadline.
// BATCH: loads kept in flight per lane before their use (the persistent kernel uses 2 to
// stay within the 32 registers per lane that cnn_bwd leaves free on a CU).  Indices are
// 32-bit float4 counts (the host keeps every stage area below 2 GB).

// U: float4 indices per thread per pass (U x BATCH loads in flight before their stores): the
// loops are latency-bound (a 4.7 MB bucket at one load in flight per lane ran at ~0.2 TB/s
// beside cnn_bwd, so the optimizer waited for it; profiles/r5/xgmi_cost).
template <int BATCH, int U>
__device__ __forceinline__ bool xg_channel(const XgmiArgs& a, int w, int W, unsigned gen,
                                           long long deadline) {
  const int tid = threadIdx.x;
  const int N = a.nranks, r = a.rank;
  const f32x4* src = reinterpret_cast<const f32x4*>(a.src);
  const int n4 = (int)(a.n >> 2);
  const bool two = a.mode == XG_TWO_SHOT;
  // two-shot: chunk d of the bucket belongs to rank d; one-shot: one "chunk" = the bucket
  const int c4 = two ? (int)(a.chunk >> 2) : n4;
  const int per = (c4 + W - 1) / W;                     // float4 per workgroup slice
  const int lo = w * per;
  const int par = two ? 0 : (int)(gen & 1u);            // one-shot stage double buffer
  const int row4 = c4;                                  // stage row length (float4)
  // flag slot of this workgroup; the two-shot chunks (one per rank) cover the bucket
  PDM_CHECK(w >= 0 && w < W && W <= XG_MAX_WG, "xgmi channel flag slot", w, W);
  PDM_CHECK(!two || (long long)c4 * 4 * N >= a.n, "xgmi two-shot chunks", c4, a.n);

  // phase 0: push slice w of chunk d (two-shot) / of the bucket (one-shot) into row r
  // of rank d's stage.  Workgroups start at different peers so all N-1 links carry
  // traffic at once; U x BATCH loads are issued before their stores.
  for (int i0 = 0; i0 < N - 1; i0 += BATCH) {
    int dd[BATCH], hid[BATCH];
#pragma unroll
    for (int b = 0; b < BATCH; ++b) {
      const int i = i0 + b < N - 1 ? i0 + b : i0;
      dd[b] = (r + 1 + (i + w) % (N - 1)) % N;
      const int len = two ? clampi(n4 - dd[b] * c4, 0, c4) : n4;
      hid[b] = i0 + b < N - 1 ? (lo + per < len ? lo + per : len) : 0;
    }
    for (int j0 = lo + tid; j0 < lo + per; j0 += XG_THREADS * U) {
      f32x4 v[U][BATCH];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int b = 0; b < BATCH; ++b) {
          const int j = j0 + u * XG_THREADS;
          if (j < hid[b]) v[u][b] = src[(two ? dd[b] * c4 : 0) + j];
        }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int b = 0; b < BATCH; ++b) {
          const int j = j0 + u * XG_THREADS;
          if (j < hid[b]) store_wt(rsrc(a.stage[dd[b]] + (long long)(par * N + r) * row4 * 4), j, v[u][b]);
        }
    }
  }
  signal_peers(a, 0, w, gen);
  if (!wait_peers(a, 0, w, gen, deadline)) return false;

  // fixed rank-order sum of this rank's chunk (two-shot) / of the whole bucket (one-shot)
  {
    const int base = two ? r * c4 : 0;
    const int len = two ? clampi(n4 - base, 0, c4) : n4;
    const int hi = lo + per < len ? lo + per : len;
    const f32x4* own = src + base;
    const f32x4* stage = reinterpret_cast<const f32x4*>(a.stage[r]) + (long long)par * N * row4;
    const long long res = a.off + (long long)base * 4;  // float offset in the result arena
    for (int j0 = lo + tid; j0 < hi; j0 += XG_THREADS * U) {
      f32x4 acc[U];
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int s0 = 0; s0 < N; s0 += BATCH) {
        f32x4 v[U][BATCH];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int b = 0; b < BATCH; ++b) {
            const int s = s0 + b, j = j0 + u * XG_THREADS;
            if (s < N && j < hi) v[u][b] = s == r ? own[j] : stage[s * row4 + j];
          }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int b = 0; b < BATCH; ++b)
            if (s0 + b < N) acc[u] = s0 + b == 0 ? v[u][b] : acc[u] + v[u][b];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = j0 + u * XG_THREADS;
        if (j >= hi) continue;
        if (two) {
          // all-gather push: the sum goes into every rank's result arena
          for (int i = 0; i < N; ++i) store_wt(rsrc(a.result[(r + i + w) % N] + res), j, acc[u]);
        } else {
          store_wt(rsrc(a.result[r] + res), j, acc[u]);
        }
      }
    }
  }
  if (two) {
    signal_peers(a, 1, w, gen);
    if (!wait_peers(a, 1, w, gen, deadline)) return false;
  }
  return true;
}

// One collective call (bucket_ready / all_ready API): grid = the channel's workgroups.
__global__ __launch_bounds__(XG_THREADS) void xgmi_allreduce_kernel(XgmiArgs a) {
  const int w = blockIdx.x;
  const unsigned gen = a.gen[w] + 1;   // this workgroup's call count on this channel
  const long long deadline = (long long)__builtin_amdgcn_s_memrealtime() + a.timeout;
  if (!xg_channel<4, 2>(a, w, gridDim.x, gen, deadline)) return;
  if (threadIdx.x == 0) a.gen[w] = gen;
}

// Streamed mode (csrc/xgmi.h): `nsteps` steps x every channel in one launch, handed
// off with the compute stream through the local READY / DONE words.
// U: float4 per lane per pass (xg_channel).  Two widths: U = 4 (72 registers) fits beside the
// one-image cnn_bwd and every band backward; U = 8 (128 registers, 44.9 vs 47.6 us per step
// at B = 32 N = 1 forced) only beside the band backward of 4- and 8-row bands (B <= 85),
// whose register use leaves room for it (tests/test_kernel_resources.py)
template <int U>
__global__ __launch_bounds__(XG_THREADS) void xgmi_stream_kernel(XgmiStreamArgs s) {
  const int w = blockIdx.x, tid = threadIdx.x;
  unsigned* loc = s.loc;
  unsigned step = loc[XG_LOC_LSTEP + w];
  for (int k = 0; k < s.nsteps; ++k) {
    ++step;
    for (int c = 0; c < s.nch; ++c) {
      const XgmiArgs& a = s.ch[c];
      if (w >= a.nblk) continue;
      const long long deadline = (long long)__builtin_amdgcn_s_memrealtime() + a.timeout;
      // wait for the compute stream to publish this step's bucket c: every wave polls for
      // itself (a wave-uniform verdict, no LDS word to broadcast it, see wait_peers)
      bool ok = true;
      for (unsigned it = 0;; ++it) {
        const unsigned e = xg_poll_err(it) ? __builtin_amdgcn_readfirstlane(__hip_atomic_load(
            loc + XG_LOC_ERR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) : 0u;
        const unsigned ready = __builtin_amdgcn_readfirstlane(__hip_atomic_load(
            loc + XG_LOC_READY + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (e != 0) {                      // this rank already gave up somewhere: fail fast
          ok = false;
          if ((tid & (PDM_WAVE - 1)) == 0) xg_record_error(loc + XG_LOC_ERR, XG_ERR_FAILFAST);
          break;
        }
        if ((int)(ready - step) >= 0) break;
        if ((long long)__builtin_amdgcn_s_memrealtime() > deadline) {
          ok = false;
          if ((tid & (PDM_WAVE - 1)) == 0) xg_record_error(loc + XG_LOC_ERR, XG_ERR_READY);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      if (!ok) return;
      const unsigned gen = a.gen[w] + 1;
      if (!xg_channel<2, U>(a, w, a.nblk, gen, deadline)) return;
      // every byte this workgroup stored for the channel is drained (write-through), and
      // every peer's bytes for its slice have arrived: count the workgroup done
      // (every result byte was stored write-through and is drained, and every peer's
      // bytes arrived behind its flag + our system acquire: no release fence needed)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        a.gen[w] = gen;
        __hip_atomic_fetch_add(loc + XG_LOC_DONE + c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  if (tid == 0) loc[XG_LOC_LSTEP + w] = step;
}

// Streamed mode, compute side: one 64-thread workgroup publishes READY[signal_ch] and
// waits until every listed channel is reduced for this step, so the optimizer after it
// needs no waiting of its own.  A single spinning workgroup (instead of the optimizer's
// whole grid) leaves the GPU to everything else, including other processes' kernels
// when ranks share a device (the one-GPU rehearsal).
__global__ __launch_bounds__(64) void xgmi_wait_kernel(unsigned* loc, int signal_ch, int nwait,
                                                       int4 ch, uint4 mult, long long timeout) {
  if (threadIdx.x != 0) return;
  if (signal_ch >= 0) xg_signal_ready(loc, signal_ch);
  const int c[4] = {ch.x, ch.y, ch.z, ch.w};
  const unsigned m[4] = {mult.x, mult.y, mult.z, mult.w};
  for (int i = 0; i < nwait; ++i)
    if (!xg_wait_done(loc, c[i], m[i], timeout, /*acquire=*/false)) return;
}

// A bounded device stall for fault-injection tests: every wave reaches the exit once the
// deadline passes.
__global__ __launch_bounds__(64) void debug_spin_kernel(long long ticks) {
  const long long end = (long long)__builtin_amdgcn_s_memrealtime() + ticks;
  while ((long long)__builtin_amdgcn_s_memrealtime() < end) __builtin_amdgcn_s_sleep(64);
}

}  // namespace

void launch_debug_spin(long long ticks, hipStream_t st) {
  hipLaunchKernelGGL(debug_spin_kernel, dim3(1), dim3(64), 0, st, ticks);
}

void launch_xgmi_allreduce(const XgmiArgs& a, int nblk, hipStream_t st) {
  hipLaunchKernelGGL(xgmi_allreduce_kernel, dim3(nblk), dim3(XG_THREADS), 0, st, a);
}

void launch_xgmi_wait(unsigned* loc, int signal_ch, int nwait, const int* ch, const unsigned* mult,
                      long long timeout, hipStream_t st) {
  int4 c = {0, 0, 0, 0};
  uint4 m = {0, 0, 0, 0};
  int* cp = &c.x;
  unsigned* mp = &m.x;
  for (int i = 0; i < nwait && i < 4; ++i) {
    cp[i] = ch[i];
    mp[i] = mult[i];
  }
  hipLaunchKernelGGL(xgmi_wait_kernel, dim3(1), dim3(64), 0, st, loc, signal_ch, nwait, c, m,
                     timeout);
}

void launch_xgmi_stream(const XgmiStreamArgs& s, hipStream_t st, bool wide) {
  int grid = 1;
  for (int c = 0; c < s.nch; ++c) grid = s.ch[c].nblk > grid ? s.ch[c].nblk : grid;
  if (wide)
    hipLaunchKernelGGL(xgmi_stream_kernel<8>, dim3(grid), dim3(XG_THREADS), 0, st, s);
  else
    hipLaunchKernelGGL(xgmi_stream_kernel<4>, dim3(grid), dim3(XG_THREADS), 0, st, s);
}
