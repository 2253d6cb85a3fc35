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

constexpr int XG_MAX_RANKS = 8;
constexpr int XG_MAX_WG = 128;     // workgroups per collective launch
constexpr int XG_MAX_CH = 4;       // channels (one per gradient bucket)
constexpr int XG_THREADS = 256;
constexpr int XG_ONE_SHOT = 0;
constexpr int XG_TWO_SHOT = 1;
constexpr int XG_FLAG_WORDS = XG_MAX_CH * 2 * XG_MAX_RANKS * XG_MAX_WG;

__host__ __device__ constexpr int xg_flag_idx(int ch, int ph, int src, int w) {
  return ((ch * 2 + ph) * XG_MAX_RANKS + src) * XG_MAX_WG + w;
}

struct XgmiArgs {
  float* stage[XG_MAX_RANKS];     // this channel's stage area on every rank (peer mappings)
  float* result[XG_MAX_RANKS];    // result arena base on every rank
  unsigned* flags[XG_MAX_RANKS];  // flag block on every rank
  const float* src;               // this rank's gradient bucket (bucket start)
  unsigned* gen;                  // this rank's per-workgroup call counters of the channel
  unsigned* err;                  // this rank's error word (bit 0: phase-0 timeout, bit 1: phase 1)
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
constexpr int XG_LOC_ERR = XG_MAX_CH * XG_MAX_WG;    // error bits (2: optimizer wait timeout)
constexpr int XG_LOC_STEP = XG_LOC_ERR + 1;          // step generation
constexpr int XG_LOC_READY = XG_LOC_ERR + 8;         // [XG_MAX_CH]
constexpr int XG_LOC_DONE = XG_LOC_ERR + 16;         // [XG_MAX_CH]
constexpr int XG_LOC_LSTEP = XG_LOC_ERR + 64;        // [XG_MAX_WG] steps run by the streamed kernel
constexpr int XG_LOC_WORDS = XG_LOC_LSTEP + XG_MAX_WG;
constexpr int XG_STREAM_WG = 64;                     // workgroups of the persistent launch

struct XgmiStreamArgs {
  XgmiArgs ch[XG_MAX_CH];
  unsigned* loc;                  // local sync words
  int nch, nsteps;
};

void launch_xgmi_stream(const XgmiStreamArgs& s, hipStream_t st);
// compute side of streamed mode: READY[signal_ch] = STEP, then wait DONE[ch[i]] >= mult[i]*STEP
void launch_xgmi_wait(unsigned* loc, int signal_ch, int nwait, const int* ch, const unsigned* mult,
                      long long timeout, hipStream_t st);

// Device-side helpers shared by the compute kernels that signal / wait.
#if defined(__HIPCC__)
__device__ __forceinline__ void xg_signal_ready(unsigned* loc, int ch) {
  const unsigned g = __hip_atomic_load(loc + XG_LOC_STEP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(loc + XG_LOC_READY + ch, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One lane polls DONE[ch] until it reaches mult * STEP (bounded), then (acquire) an
// agent-scope acquire so this workgroup may read the reduced bytes; false (and error
// bit 2) on timeout.  Call from a single lane; the caller barriers its workgroup
// afterwards.  A kernel that only gates the NEXT kernel needs no acquire: that kernel
// starts behind the boundary's own acquire.
__device__ __forceinline__ bool xg_wait_done(unsigned* loc, int ch, unsigned mult,
                                             long long timeout, bool acquire = true) {
  const unsigned target =
      mult * __hip_atomic_load(loc + XG_LOC_STEP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const long long deadline = (long long)__builtin_amdgcn_s_memrealtime() + timeout;
  for (unsigned it = 1; (int)(__hip_atomic_load(loc + XG_LOC_DONE + ch, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT) - target) < 0;
       ++it) {
    // deadline, or (every 64 polls) an earlier give-up of this rank: fail fast
    if ((long long)__builtin_amdgcn_s_memrealtime() > deadline ||
        ((it & 63u) == 0 && __hip_atomic_load(loc + XG_LOC_ERR, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT) != 0)) {
      atomicOr(loc + XG_LOC_ERR, 4u);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  if (acquire) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return true;
}
#endif
