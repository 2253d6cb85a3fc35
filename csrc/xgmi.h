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
};

void launch_xgmi_allreduce(const XgmiArgs& a, int nblk, hipStream_t st);
