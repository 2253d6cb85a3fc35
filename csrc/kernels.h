// Host-side launch API of the gfx950 kernels (raw pointers + stream).
// bind.cpp validates torch tensors (shape / dtype / device / contiguity) before
// calling any of these; the kernels themselves assume the validated shapes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "xgmi.h"


// A training step's rows in the epoch buffer.  The data-step counter c runs on across epochs
// (nothing resets it at an epoch boundary); with spe > 0 steps per epoch the buffer holds two
// epochs, epoch e = c / spe in half e & 1 (rows [(e & 1) * nrow / 2, ...)), so the next
// epoch's samples are gathered into the other half while this one trains and the step graphs
// never change.  spe == 0: one flat buffer, row c * bfull + img.
struct StepRows {
  int bfull;   // full batch: the row stride between consecutive steps
  int spe;     // steps per epoch (0: flat buffer)
};
__host__ __device__ __forceinline__ int64_t step_row(const StepRows g, int64_t nrow, int64_t c,
                                                     int img) {
  if (g.spe <= 0) return c * g.bfull + img;
  const uint32_t e = (uint32_t)c / (uint32_t)g.spe;
  const int64_t s = c - (int64_t)e * g.spe;
  return (int64_t)(e & 1u) * (nrow >> 1) + s * g.bfull + img;
}

// ---------------------------------------------------------------- linear model
constexpr int LIN_K = 784;
constexpr int LIN_N = 10;
// train rows per workgroup (us/step at B = 256, Adam: 1: 17.8, 2: 13.8, 4: 12.4, 8: 13.7, 16: 17.1)
constexpr int LIN_ROWS = 4;
constexpr int LIN_SLAB = 7856;  // 7840 dW + 10 db + loss + correct, padded
constexpr int LIN_EVAL_ROWS = 16;

// idx == nullptr: rows [ctr*bfull, ctr*bfull + B) of `images` (epoch buffer), else the
// sampler gather images[idx[ctr*bfull + i]].  metrics (fp64 [3]) and c1 (optimizer-step
// counter, advanced once) are optional.
void launch_lin_train(const uint8_t* images, const int32_t* labels, const int32_t* idx,
                      int64_t nrow, const int64_t* ctr, StepRows sr, int B, const float* W, const float* b,
                      float* slab, double* metrics, int64_t* c1, hipStream_t st);
// metrics (optional): one extra workgroup sums the loss / correct slab columns into
// metrics[0..1] in a fixed order (lin_train only adds the sample count)
void launch_lin_reduce(const float* slab, int nblk, float* gW, float* gb, int64_t* c0, unsigned* c2,
                       double* metrics, hipStream_t st);
void launch_lin_eval(const uint8_t* images, const int32_t* labels, int n_total, const float* W,
                     const float* b, double* metrics, hipStream_t st);

// ---------------------------------------------------------------- data
void launch_gather_epoch(const uint8_t* images, const int32_t* labels, const int32_t* idx, int n,
                         int nimg, uint8_t* out_images, int32_t* out_labels, int64_t* ctr,
                         int nctr, int64_t* step, int64_t step_value, int max_wgs, hipStream_t st);

// ---------------------------------------------------------------- optimizer
constexpr int OPT_ADAM = 0;
constexpr int OPT_SGD = 1;
constexpr int OPT_MAX_SEG = 8;

struct OptSeg {
  int64_t offset;      // float offset of the segment in the arena
  int32_t rows, cols;  // numel = rows * cols (plain segments: rows = 1)
  int32_t first_block; // filled by launch_optim
  __bf16* shadow;      // optional bf16 copy, same layout
  __bf16* shadow_t;    // optional bf16 copy, transposed [cols][rows]
  __bf16* shadow_lo;   // optional bf16(p - bf16(p)), row-major like shadow: with shadow the
                       // split-bf16 (hi / lo) operand copy of the fp32 program
  // optional: the gradient is the fixed-order sum of `nslab` per-workgroup slabs
  // (row stride `slab_stride` floats, this segment at column `slab_col0`) — the
  // conv_reduce pass fused into the update (world_size 1: no all-reduce in between)
  const float* slab;
  int32_t nslab, slab_col0;
  int64_t slab_stride;
  // optional (xgmi streamed mode): wait until DONE[wait_ch] >= wait_mult * STEP
  int32_t wait_ch;
  uint32_t wait_mult;
  // transpose-only segment: no update; shadow_t is re-derived from shadow (the update ran
  // elsewhere, e.g. fused into cnn_bwd at world size 1)
  int32_t tonly;
  // shadow_t layout: 0 = row-major [cols][rows]; 1 = MFMA-fragment-major (rows % 32 == 0,
  // cols % 16 == 0): the 16 x 32 A fragment (cols 16 fb .., rows 32 ks ..) is one 1-KB block,
  // lane (g, i) holding rows 32 ks + 8 g .. + 7 of col 16 fb + i -- a wave's fragment load
  // is then 8 whole cache lines instead of 16 half lines (fc1_bwd's dX tiles)
  int32_t tfrag;
  int32_t sfrag;       // shadow layout: 0 = row-major, 1 = fragment-major (frag_pos, m = row)
};

// MFMA-fragment-major offset of element (m, k) of an [M][K] bf16 operand (K % 32 == 0,
// M % 16 == 0): the 16 x 32 fragment (m >> 4, k >> 5) is one 512-element block and lane
// ((k >> 3) & 3) * 16 + (m & 15) of a 16x16x32 MFMA operand load holds its 8 k-values --
// a wave's fragment load reads 1 KB contiguous (8 whole cache lines)
__host__ __device__ inline int64_t frag_pos(int64_t m, int64_t k, int32_t K) {
  return (((m >> 4) * (K >> 5) + (k >> 5)) * 64 + ((k >> 3) & 3) * 16 + (m & 15)) * 8 + (k & 7);
}
// offset of element (row, col) of a [rows][cols] matrix in its bf16 copy (sfrag: fragment-
// major with m = row) and in its transposed copy (tfrag: fragment-major with m = col)
__host__ __device__ inline int64_t shadow_pos(int32_t sfrag, int32_t cols, int64_t row, int64_t col) {
  return sfrag ? frag_pos(row, col, cols) : row * cols + col;
}
__host__ __device__ inline int64_t shadow_t_pos(int32_t tfrag, int32_t rows, int64_t row, int64_t col) {
  return tfrag ? frag_pos(col, row, rows) : col * rows + row;
}

struct OptArgs {
  float* p;
  const float* g;
  float* m;   // exp_avg (adam) / momentum_buffer (sgd)
  float* v;   // exp_avg_sq (adam)
  const double* lr;
  const int64_t* step;  // already advanced for this step (t >= 1)
  double beta1_d, beta2_d;
  float beta1, beta2, eps, wd, momentum, dampening;
  int nesterov;
  float grad_scale;
  int nseg;
  OptSeg seg[OPT_MAX_SEG];
  // xgmi streamed mode: local sync words; every workgroup first stores
  // READY[signal_ch] = STEP (signal_ch < 0: none), then waits its segment's channel
  unsigned* xg;
  int xg_signal_ch;
  long long xg_timeout;   // s_memrealtime ticks
  // optional counter advanced once by the launch (world size 1 Linear: the data-step
  // counter, which no optimizer workgroup reads)
  int64_t* bump;
  // optional (world size 1 Linear): one extra workgroup adds the step's train loss / correct
  // partials (slab columns mcol, mcol + 1 of mnslab slabs) to metrics[0..1] in a fixed order
  const float* mslab;
  int32_t mnslab, mcol;
  int64_t mstride;
  double* metrics;
  // optional (xx_on): the slab segments' reduced gradients are all-reduced in-launch over
  // xGMI (XgmiExch, xgmi.h) before their update -- the conv bucket at world size > 1
  int xx_on;
  XgmiExch xx;
};

void launch_optim(int kind, OptArgs& a, hipStream_t st);
// fc1_fwd switches to 128-row blocks from this batch on (runtime.cnn_step.choose_splitk
// sizes the split-K for the same tiles)
constexpr int FC1_BIG_B = 2048;

// World size 1: the fc1-weight update fused into fc1_bwd's weight-gradient tiles (the tile
// is final in registers; nothing else in the step reads the fp32 weights or the bf16 [n][k]
// copy until the next step's fc1_fwd -- the transposed copy that this step's dX tiles read
// is re-derived later by the optimizer launch, or double-buffered: shadow_t_next).  kind < 0:
// off; OPT_SGD only.  Same
// hyper-parameter fields as OptArgs.
struct FcUpdate {
  int kind;
  int64_t numel;        // multiple of 4
  float* p;
  const float* g;
  float* m;
  float* v;
  __bf16* shadow;       // bf16 copy, same layout
  // optional: where the weight tiles write the updated W1^T copy (fragment-major) -- the
  // other half of a double buffer whose current half this launch's dX tiles are reading
  // (the host alternates the halves), so the optimizer launch no longer re-derives W1^T
  __bf16* shadow_t_next;
  const double* lr;
  const int64_t* step;
  double beta1_d, beta2_d;
  float beta1, beta2, eps, wd, momentum, dampening;
  int nesterov;
  float grad_scale;
  // 0: the fused update consumes the gradient in registers and the fp32 fc1-weight gradient
  // is not stored (4.7 MB of writes saved per step; nothing reads it); 1: stored as usual
  int store_grad;
  // carried update (kernels/fc_carry.h), xgmi streamed mode: wait until DONE[wch] >=
  // wmult * STEP in the local sync words `wloc` before reading g (nullptr: no wait)
  unsigned* wloc;
  int wch;
  unsigned wmult;
  long long wtimeout;     // s_memrealtime ticks
};

// ---------------------------------------------------------------- CNN (bf16)
// Layouts (NHWC, see pytorch_distributed_mnist_amd/models/specs.py):
//   x      uint8 [B][28*28]            gathered input bytes (for conv1 wgrad)
//   (a1 = relu(conv1) is never stored: the backward recomputes it from x)
//   pool   bf16  [B][12*12][64]        maxpool(relu(conv2)) == fc1 input
//   pmask  uint8 [B][12*12][64]        argmax in window (0..3) | 0x80 when > 0
//   w2     bf16  [64][9][32]           conv2 weight (co, tap, ci)
//   w2t    bf16  [9][32][64]           conv2 weight (tap, ci, co)   (dgrad)
//   wf1    bf16  [128][9216]           fc1 weight  (n, hwc)
//   wf1t   bf16  [9216][128]           fc1 weight transposed        (dX)
constexpr int CNN_FEAT = 9216;
constexpr int CNN_HID = 128;
constexpr int CNN_NCLS = 10;
constexpr int CNN_HEAD_ROWS = 4;         // rows per head row group (one wave per row)
constexpr int CNN_HEAD_MAX_BLOCKS = 256;  // head workgroups (grid-stride over row groups)
int cnn_head_blocks(int groups);          // head workgroups = head slabs for `groups` row groups
constexpr int CNN_HEAD_SLAB = 1420;   // 1280 dWfc2 + 10 dbfc2 + 128 dbfc1 + loss + correct
constexpr int CNN_CONV_SLAB = 18816;  // 18432 dW2 + 64 db2 + 288 dW1 + 32 db1
constexpr int CNN_CONV_SLAB_DB2 = 18432;   // slab column of db2 ([co][tap][ci] dW2 before it)
constexpr int CNN_CONV_SLAB_DW1 = 18496;   // dW1 [32][9]
constexpr int CNN_CONV_SLAB_DB1 = 18784;   // db1 [32]

void launch_cnn_fwd(const uint8_t* images, const int32_t* labels, const int32_t* idx,
                    int64_t nrow, const int64_t* ctr, StepRows sr, int B, const float* w1, const float* b1,
                    const __bf16* w2, const float* b2, __bf16* pool, uint8_t* pmask, uint8_t* xg,
                    int32_t* ylab, const FcUpdate* fcc, hipStream_t st);
// small batches: each image over `bands` in {2, 3, 6} workgroups of 24 / bands conv2 rows
// (cnn_fwd_band.hip); same pool / pmask / ylab as launch_cnn_fwd; training also writes the a1
// image and the normalised x for cnn_bwd_band (a1g, xng) and / or the gathered uint8 image for
// cnn_bwd (xg)
void launch_cnn_fwd_band(const uint8_t* images, const int32_t* labels, const int32_t* idx,
                         int64_t nrow, const int64_t* ctr, StepRows sr, int B, int bands,
                         const float* w1, const float* b1, const __bf16* w2, const float* b2,
                         __bf16* pool, uint8_t* pmask, __bf16* a1g, __bf16* xng, uint8_t* xg,
                         int32_t* ylab, const FcUpdate* fcc, hipStream_t st);
// fcc (training, world size > 1): the previous step's fc1-weight SGD update, run by extra
// workgroups of the forward launch (kernels/fc_carry.h FCC_WGS); nullptr: none
void launch_fc1_fwd(const __bf16* pool, const __bf16* wf1, float* part, int B, int splitk,
                    hipStream_t st);
void launch_cnn_head(const float* part, int splitk, int B, const float* bf1, const float* wf2,
                     const float* bf2, const int32_t* ylab, bool train, __bf16* dh, __bf16* dht,
                     int ldt, float* slab, double* metrics, int64_t* c0, int64_t* c1,
                     unsigned* c2, float* dh32, hipStream_t st);
void launch_fc1_bwd(const __bf16* dh, const __bf16* dht, int ldt, const __bf16* pool,
                    const __bf16* wf1t, int B, float* gwf1, __bf16* dpool, const float* head_slab,
                    int head_blocks, float* gwf2, float* gbf2, float* gbf1, double* metrics,
                    const FcUpdate& fcu, hipStream_t st);
void launch_cnn_bwd(const uint8_t* xg, const float* w1, const float* b1, const __bf16* dpool,
                    const uint8_t* pmask, const __bf16* w2t, int B, int imgs_per_block, float* slab,
                    unsigned* xg_sync, hipStream_t st);
int cnn_bwd_blocks(int B, int imgs_per_block);
// small batches: each image split over `bands` in {2, 3, 6} workgroups of 24 / bands conv2
// rows (cnn_bwd_band.hip); B * bands workgroups, one slab each (the cnn_bwd slab layout).
// Reads the a1 image (swizzled, [B][26*26*32]) and the normalised x ([B][784] bf16) that
// cnn_fwd_band wrote, instead of recomputing conv1.
void launch_cnn_bwd_band(const __bf16* a1g, const __bf16* xng, const __bf16* dpool,
                         const uint8_t* pmask, const __bf16* w2t, int B, int bands, float* slab,
                         unsigned* xg_sync, hipStream_t st);
void launch_conv_reduce(const float* slab, int nblk, float* gw2, float* gb2, float* gw1, float* gb1,
                        hipStream_t st);

// ---------------------------------------------------------------- CNN (fp32, cnn_f32.hip)
// The reference's precision on the fp32 MFMA (v_mfma_f32_16x16x4_f32).  fp32 layouts as the
// bf16 path (pool [B][12*12][64], pmask, conv2 weight [co][tap][ci], fc1 weight [128][9216]);
// w2s: conv2's weight as split-bf16 hi / lo planes [2][64][288] (split-bf16 path only).
// a1g [B][676][32] and xng [B][784] carry the forward's conv1 activations and normalised
// image to the backward; dh32 [ldt][128] is cnn_head's fp32 dh (launch_cnn_head dh32 != null).
void launch_f32_fwd(const uint8_t* images, const int32_t* labels, int64_t nrow, const int64_t* ctr,
                    StepRows sr, int B, const float* w1, const float* b1, const float* w2,
                    const float* b2, float* pool, uint8_t* pmask, float* a1g, float* xng,
                    int32_t* ylab, bool x3, float* w2x, const __bf16* w2s, hipStream_t st);
void launch_f32_fc1_fwd(const float* pool, const float* w1, float* part, int B, int splitk,
                        bool x3, hipStream_t st);
void launch_f32_fc1_bwd(const float* dh, int ldt, const float* pool, const float* w1, int B,
                        float* gwf1, float* dpool, const float* head_slab, int head_blocks,
                        float* gwf2, float* gbf2, float* gbf1, double* metrics, bool x3, hipStream_t st);
// conv backward: (image group of ipb images, row band) workgroups, one slab each
int f32_conv_bwd_blocks(int B, int per, bool x3);
void launch_f32_conv_bwd(const float* a1g, const float* xng, const float* dpool,
                         const uint8_t* pmask, const float* w2, int B, int ipb, float* slab,
                         bool x3, const float* w2x, hipStream_t st);

// diagnostic timestamps (all zero unless built with PDM_STAMPS=1)
void read_stamps_fwd(unsigned long long* host);
void read_stamps_bwd(unsigned long long* host);
void read_stamps_fwd_band(unsigned long long* host);
void read_stamps_bwd_band(unsigned long long* host);
void read_stamps_f32(unsigned long long* host);
