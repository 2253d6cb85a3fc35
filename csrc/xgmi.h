// Direct xGMI peer-to-peer gradient all-reduce (shared host/device definitions).
//
// Every rank owns one *uncached* device allocation (hipDeviceMallocUncached: no
// L2 copy on either side of an xGMI access) holding
//   flags   [channel][phase][src rank][workgroup]  u32, written by peers
//   result  arena-sized fp32: the all-reduced gradients the optimizer reads
//   stage   per channel: peers' contributions pushed here
// and maps every peer's allocation through hipIpc (dmabuf).  A collective is one
// kernel on the communicator's stream; it only ever STORES to peer memory (posted
// writes over the link) and loads from its own HBM.
//   one-shot: push the whole bucket into every peer's stage (double-buffered by
//             call parity), one flag hand-off, every rank sums all N copies.
//   two-shot: reduce-scatter push (chunk d -> rank d), rank r sums chunk r and
//             pushes the sum into every rank's result, second flag hand-off.
// Sums run in rank order 0..N-1 on exactly one rank per element, so every rank
// ends with bit-identical gradients.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pdm_check.h"

constexpr int XG_MAX_RANKS = 8;
constexpr int XG_MAX_WG = 128;     // workgroups per collective launch
constexpr int XG_MAX_CH = 4;       // channels (one per gradient bucket)
constexpr int XG_THREADS = 256;
constexpr int XG_ONE_SHOT = 0;
constexpr int XG_TWO_SHOT = 1;
constexpr int XG_FLAG_WORDS = XG_MAX_CH * 2 * XG_MAX_RANKS * XG_MAX_WG;
// in-launch exchange slots (XgmiExch): one flag per (source rank, slot) after the channel flags
constexpr int XG_XSLOTS = 512;
constexpr int XG_FLAG_WORDS_ALL = XG_FLAG_WORDS + XG_MAX_RANKS * XG_XSLOTS;

__host__ __device__ constexpr int xg_flag_idx(int ch, int ph, int src, int w) {
  return ((ch * 2 + ph) * XG_MAX_RANKS + src) * XG_MAX_WG + w;
}
__host__ __device__ constexpr int xg_xflag_idx(int src, int slot) {
  return XG_FLAG_WORDS + src * XG_XSLOTS + slot;
}

struct XgmiArgs {
  float* stage[XG_MAX_RANKS];     // this channel's stage area on every rank (peer mappings)
  float* result[XG_MAX_RANKS];    // result arena base on every rank
  unsigned* flags[XG_MAX_RANKS];  // flag block on every rank
  const float* src;               // this rank's gradient bucket (bucket start)
  unsigned* gen;                  // this rank's per-workgroup call counters of the channel
  unsigned* err;                  // this rank's error word (XG_ERR_* bits; XG_LOC_FIRST follows)
  long long off;                  // bucket start in the arena (floats)
  long long n;                    // bucket length (floats, multiple of 64)
  long long chunk;                // two-shot chunk (floats, multiple of 64)
  long long timeout;              // spin limit, s_memrealtime ticks (100 MHz)
  int rank, nranks, ch, mode;
  int nblk;                       // workgroups that carry this channel
};

void launch_xgmi_allreduce(const XgmiArgs& a, int nblk, hipStream_t st);

// ---- streamed mode: one persistent collective launch per captured step sequence.
// A hipGraph edge between two queues costs 5-10 us on MI355X (measured: fork after
// fc1_bwd delayed cnn_bwd by 11 us, each join 6-10 us), more than the transfers
// themselves, so the per-step hand-offs between the compute stream and the
// collective are device-side words in the reducer's local buffer instead:
//   the step's middle kernel (cnn_head / lin_reduce) bumps STEP;
//   the kernel that starts after a bucket is complete (cnn_bwd for the fc bucket,
//   the optimizer for the last bucket) stores READY[c] = STEP;
//   the persistent kernel waits READY[c] >= its own step count, runs the channel,
//   and every workgroup adds 1 to DONE[c];
//   the optimizer's workgroups wait DONE[c] >= nblk_c * STEP before updating.
// Local sync words (uint32) of the reducer's local buffer:
constexpr int XG_LOC_GEN = 0;                        // [XG_MAX_CH][XG_MAX_WG] call counters
constexpr int XG_LOC_ERR = XG_MAX_CH * XG_MAX_WG;    // error bits (XG_ERR_*)
constexpr int XG_LOC_STEP = XG_LOC_ERR + 1;          // step generation
constexpr int XG_LOC_FIRST = XG_LOC_ERR + 2;         // the first error's cause bit (set once)
constexpr int XG_LOC_NPUB = XG_LOC_ERR + 3;          // channels the backward publishes (0: 1)
constexpr int XG_LOC_READY = XG_LOC_ERR + 8;         // [XG_MAX_CH]
constexpr int XG_LOC_DONE = XG_LOC_ERR + 16;         // [XG_MAX_CH]
constexpr int XG_LOC_LSTEP = XG_LOC_ERR + 64;        // [XG_MAX_WG] steps run by the streamed kernel
constexpr int XG_LOC_XGEN = XG_LOC_LSTEP + XG_MAX_WG;  // [XG_XSLOTS] in-launch exchange calls
constexpr int XG_LOC_WORDS = XG_LOC_XGEN + XG_XSLOTS;
// workgroups of the persistent launch (16 / 32 / 64 measured alike beside cnn_bwd once the
// kernel used no LDS, profiles/r5/xgmi_width/)
constexpr int XG_STREAM_WG = 64;
static_assert(XG_STREAM_WG >= 1 && XG_STREAM_WG <= XG_MAX_WG, "persistent launch width");

struct XgmiStreamArgs {
  XgmiArgs ch[XG_MAX_CH];
  unsigned* loc;                  // local sync words
  int nch, nsteps;
};

// wide: the 8-loads-per-lane variant (only beside the 4- / 8-row band backward kernels)
void launch_xgmi_stream(const XgmiStreamArgs& s, hipStream_t st, bool wide = false);

// ---- in-launch exchange: a bucket all-reduced INSIDE the kernel that produces it.
// The optimizer's slab segments (the conv bucket at world size > 1) reduce their 64 slab
// columns, push the 64 sums into every peer's stage row (write-through, system scope),
// signal their slot's flag on every peer, wait for the peers' flags of the same slot and
// sum the N rows in rank order -- a one-shot all-reduce of 256 B per workgroup with no
// conv_reduce launch, no hand-off to the persistent collective and no wait launch in
// between.  Stage rows are double-buffered by call parity, as the one-shot channel's.
struct XgmiExch {
  float* stage[XG_MAX_RANKS];     // the bucket's stage area on every rank (2 x N rows of n)
  unsigned* flags[XG_MAX_RANKS];  // flag block on every rank (slots at xg_xflag_idx)
  unsigned* gen;                  // this rank's per-slot call counters (XG_LOC_XGEN)
  unsigned* err;                  // this rank's error word
  long long off;                  // bucket start in the arena (floats)
  long long n;                    // bucket length (floats): the stage row length
  long long timeout;              // s_memrealtime ticks
  int rank, nranks;
};
// compute side of streamed mode: READY[signal_ch] = STEP, then wait DONE[ch[i]] >= mult[i]*STEP
void launch_xgmi_wait(unsigned* loc, int signal_ch, int nwait, const int* ch, const unsigned* mult,
                      long long timeout, hipStream_t st);
// fault injection (bench.py calibration tests): one wave that sleeps on the device for `ticks`
// of s_memrealtime (100 MHz) and exits -- a bounded stand-in for a stuck kernel
void launch_debug_spin(long long ticks, hipStream_t st);

// Error bits of the rank's error word (XG_LOC_ERR).  A wait that runs past its deadline
// records its own cause; a wait that gives up because the word was already set records
// XG_ERR_FAILFAST only, and the first cause is kept separately in XG_LOC_FIRST, so the
// host can tell the root cause from its consequences.
constexpr unsigned XG_ERR_PEER0 = 1u;      // a collective workgroup's peers missed phase 0
constexpr unsigned XG_ERR_PEER1 = 2u;      // ... phase 1 (two-shot all-gather)
constexpr unsigned XG_ERR_OPTWAIT = 4u;    // the optimizer side waited for a bucket in vain
constexpr unsigned XG_ERR_READY = 8u;      // the persistent collective waited for the compute stream
constexpr unsigned XG_ERR_FAILFAST = 16u;  // a wait gave up because an earlier one had

// Device-side helpers shared by the compute kernels that signal / wait.
#if defined(__HIPCC__)
// `err` points at XG_LOC_ERR of the rank's local words.
__device__ __forceinline__ void xg_record_error(unsigned* err, unsigned bit) {
  atomicOr(err, bit);
  if (bit != XG_ERR_FAILFAST) atomicCAS(err + (XG_LOC_FIRST - XG_LOC_ERR), 0u, bit);
}

// Poll schedule shared by every bounded wait: the error word is read on the first poll
// and every 64th after it, so a wait that starts after this rank's error word was set
// gives up at once (deterministically), and one missing peer costs one timeout.
__device__ __forceinline__ bool xg_poll_err(unsigned it) { return (it & 63u) == 0; }

__device__ __forceinline__ void xg_signal_ready(unsigned* loc, int ch) {
  const unsigned g = __hip_atomic_load(loc + XG_LOC_STEP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(loc + XG_LOC_READY + ch, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The conv backward's first workgroup: the first bucket (the fc bucket, whose gradients
// fc1_bwd finished) is complete -- publish its channels [0, NPUB) (a bucket may be cut into
// several channels: models/specs.py channel_bounds)
__device__ __forceinline__ void xg_signal_backward(unsigned* loc) {
  const unsigned g = __hip_atomic_load(loc + XG_LOC_STEP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned n = __hip_atomic_load(loc + XG_LOC_NPUB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (unsigned c = 0; c < (n ? n : 1u) && c < (unsigned)XG_MAX_CH; ++c)
    __hip_atomic_store(loc + XG_LOC_READY + c, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One lane polls DONE[ch] until it reaches mult * STEP (bounded), then (acquire) an
// agent-scope acquire so this workgroup may read the reduced bytes; false (and
// XG_ERR_OPTWAIT, or XG_ERR_FAILFAST after an earlier error) when it gives up.
// Call from a single lane; the caller barriers its workgroup afterwards.  A kernel that only gates the NEXT kernel needs no acquire: that kernel
// starts behind the boundary's own acquire.
__device__ __forceinline__ bool xg_wait_done(unsigned* loc, int ch, unsigned mult,
                                             long long timeout, bool acquire = true) {
  const unsigned target =
      mult * __hip_atomic_load(loc + XG_LOC_STEP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const long long deadline = (long long)__builtin_amdgcn_s_memrealtime() + timeout;
  for (unsigned it = 0;; ++it) {
    // both loads are issued before either is consumed: the error check adds no latency
    const unsigned e = xg_poll_err(it) ? __hip_atomic_load(loc + XG_LOC_ERR, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT) : 0u;
    const unsigned done = __hip_atomic_load(loc + XG_LOC_DONE + ch, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
    if (e != 0) {                        // an earlier wait of this rank gave up: fail fast
      xg_record_error(loc + XG_LOC_ERR, XG_ERR_FAILFAST);
      return false;
    }
    if ((int)(done - target) >= 0) break;
    if ((long long)__builtin_amdgcn_s_memrealtime() > deadline) {
      xg_record_error(loc + XG_LOC_ERR, XG_ERR_OPTWAIT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  if (acquire) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return true;
}

// In-launch exchange (XgmiExch): called by EVERY thread of a workgroup that owns `slot`;
// threads with `valid` hold one reduced value `v` of the bucket at bucket offset `bl` and
// receive the rank-order sum over all ranks (the one-shot channel's order: same bits as
// conv_reduce followed by the one-shot all-reduce).  False (error bit set) when a peer did
// not arrive before the deadline; the caller must then skip its update.
__device__ __forceinline__ bool xg_exchange(const XgmiExch& x, int slot, long long bl, bool valid,
                                            float& v, int* s_ok) {
  const int N = x.nranks, r = x.rank, tid = threadIdx.x;
  // one flag slot per slab workgroup; the element inside the bucket's stage row
  PDM_CHECK(slot >= 0 && slot < XG_XSLOTS, "xgmi exchange flag slot", slot, XG_XSLOTS);
  PDM_CHECK(!valid || (bl >= 0 && bl < x.n), "xgmi exchange stage offset", bl, x.n);
  if (N == 1) return true;
  const unsigned gen = __hip_atomic_load(x.gen + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const long long par = gen & 1u;
  if (valid) {
    for (int i = 1; i < N; ++i) {
      const int d = r + i < N ? r + i : r + i - N;
      __hip_atomic_store(x.stage[d] + (par * N + r) * x.n + bl, v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // every wave's pushes have landed
  __syncthreads();
  if (tid == 0) {
    for (int d = 0; d < N; ++d)
      if (d != r)
        __hip_atomic_store(x.flags[d] + xg_xflag_idx(r, slot), gen, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (tid < 64) {
    const int lane = tid;
    const bool mine = lane < N && lane != r;
    const unsigned* f = x.flags[r] + xg_xflag_idx(mine ? lane : 0, slot);
    const long long deadline = (long long)__builtin_amdgcn_s_memrealtime() + x.timeout;
    unsigned cause = 0;
    for (unsigned it = 0;; ++it) {
      const unsigned e = xg_poll_err(it) ? __builtin_amdgcn_readfirstlane(
          __hip_atomic_load(x.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) : 0u;
      const bool arrived = !mine || (int)(__hip_atomic_load(f, __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_SYSTEM) - gen) >= 0;
      if (e != 0) {
        cause = XG_ERR_FAILFAST;
        break;
      }
      if (__all(arrived)) break;
      if ((long long)__builtin_amdgcn_s_memrealtime() > deadline) {
        cause = XG_ERR_PEER0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");         // system scope: the peers' rows
    if (lane == 0) {
      *s_ok = cause == 0;
      if (cause != 0) xg_record_error(x.err, cause);
    }
  }
  __syncthreads();
  if (!*s_ok) return false;
  if (valid) {
    const float* st = x.stage[r] + par * N * x.n + bl;
    float acc = 0.f;
    for (int q = 0; q < N; ++q) {
      const float u = q == r ? v : st[(long long)q * x.n];
      acc = q == 0 ? u : acc + u;
    }
    v = acc;
  }
  if (tid == 0) __hip_atomic_store(x.gen + slot, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}
#endif
