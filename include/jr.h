/*
 * jr.h — C-ABI of libjr.so, the MI355X (gfx950) compute library behind the
 * jama16-retina-replication hot path: the Inception-v3 training step and
 * ensemble inference of train.py / evaluate.py.
 *
 * The reference has no FFI: every op below replaces a TensorFlow op that the
 * reference graph instantiates.  Each entry point cites the
 * reference call site whose TF op it replaces.
 *
 * Conventions
 *  - Every function returns JR_OK (0) or a negative jr_status; the message of
 *    the last failure on the calling thread is returned by jr_last_error().
 *  - All tensor arguments are caller-owned DEVICE pointers (torch.Tensor
 *    .data_ptr() on the host side).  The library never allocates, except that
 *    multi-kernel ops take a caller-provided workspace sized by the matching
 *    *_workspace_size query.
 *  - Activations are NHWC (channels_last, lib/dataset.py:42-43); conv kernels
 *    are HWIO [kh][kw][cin][cout] (the Keras Conv2D layout).
 *  - A channel slice (c_off, c_stride) addresses channels
 *    [c_off, c_off + c) of a buffer whose pixel rows hold c_stride channels;
 *    this is how Inception-block outputs are written concat-free.
 *  - No host synchronisation inside any call; every call is enqueued on the
 *    given stream (hipStream_t passed as void*; NULL = the null stream), so a
 *    whole training step can be captured into a HIP graph.
 *  - dtype: JR_F32 = IEEE fp32 end to end (the reference's precision);
 *    JR_BF16 = bf16 activations/weights with fp32 accumulation;
 *    JR_F32_X8 (convolution entry points only) = fp32 tensors exactly as
 *    JR_F32, the GEMM products formed on the bf16 matrix cores: every fp32
 *    operand is split exactly into three bf16 terms (x = h + m + l) and eight
 *    bf16 MFMAs accumulate hh+hm+mh+mm+hl+lh+ml+lm in fp32; only l*l
 *    (< 2^-32 |a b|) is dropped, so every product is exact to far below
 *    fp32 rounding and the result differs from JR_F32 only in summation
 *    order (bf16x9-style fp32 emulation).  Non-finite inputs give NaN where
 *    JR_F32 could give +-inf.
 *    JR_F32_X8P (convolution entry points only) = the JR_F32_X8 arithmetic
 *    with the split done once, outside the GEMM: every operand arrives as its
 *    three bf16 planes h, m, l (x = h + m + l exactly; jr_split_x8p,
 *    jr_conv_weights_x8p*), stored back to back, each plane in the JR_BF16
 *    layout of that operand (channel radices padded to 8; fwd filter
 *    W^T [c_out][kh][kw][c8], bwd_data filter HWIO).  The plane stride is the
 *    plane's element count as the descriptor implies: n*h*w*x_c_stride (x),
 *    n*ho*wo*y_c_stride (dy), c_out*kh*kw*c8 (W^T), kh*kw*c_in*c_out (HWIO).
 *    Eight MFMAs per product in the JR_F32_X8 order; outputs (y, dx, dw) are
 *    fp32 exactly as for JR_F32.
 *    JR_F32_X6H (convolution entry points only) = fp32 tensors as JR_F32_X8,
 *    the products on the fp16 matrix cores: each operand is scaled by a
 *    power of two s that puts its largest magnitude (the descriptor's
 *    x/w/dy absmax or bound) in [2^14, 2^15) and split into three fp16 terms
 *    x s = h + m + l (11-bit significands: exact for |x s| >= 2^-1, i.e.
 *    down to 2^-15 of the tensor's max, and down to 2^-24 absolute through
 *    fp16 subnormals); six f16 MFMAs accumulate hh+hm+mh+mm+hl+lh in fp32
 *    (dropped: ml + lm < 2^-32 |a b| and l*l, the JR_F32_X8 class), and the
 *    result is scaled back exactly.  Same tiles, config ids, split-K and
 *    stream-K plans as JR_F32_X8; 3/4 of its MFMAs.  A magnitude above the
 *    stated bound saturates (wrong results): bounds must hold.
 */
#ifndef JR_H_
#define JR_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum jr_status {
  JR_OK = 0,
  JR_ERR_INVALID = -1,     /* bad argument / unsupported geometry          */
  JR_ERR_HIP = -2,         /* a HIP runtime call failed                    */
  JR_ERR_UNSUPPORTED = -3, /* valid request this build does not implement  */
  JR_ERR_WORKSPACE = -4,   /* workspace smaller than *_workspace_size      */
  JR_ERR_DEVICE = -5       /* a kernel reported a device-side failure      */
} jr_status;

typedef enum jr_dtype { JR_F32 = 0, JR_BF16 = 1, JR_F32_X8 = 2, JR_F32_X8P = 3, JR_F32_X6H = 4 } jr_dtype;

typedef enum jr_conv_op { JR_CONV_FWD = 0, JR_CONV_BWD_DATA = 1, JR_CONV_BWD_FILTER = 2 } jr_conv_op;

typedef enum jr_head_mode { JR_HEAD_SIGMOID = 0, JR_HEAD_SOFTMAX = 1 } jr_head_mode;

/* One Conv2D(use_bias=False) layer of keras_applications inception_v3
 * conv2d_bn (instantiated at train.py:129-130).  pad_* are the top/left
 * paddings: 'same' at stride 1 => (k-1)/2, 'valid' => 0. */
typedef struct jr_conv_desc {
  int32_t n, h, w, c_in;          /* input  [n, h, w, c_in] (slice)        */
  int32_t c_out, kh, kw;          /* kernel [kh, kw, c_in, c_out]          */
  int32_t stride_h, stride_w;
  int32_t pad_h, pad_w;
  int32_t ho, wo;                 /* output [n, ho, wo, c_out] (slice)     */
  int32_t x_c_off, x_c_stride;    /* channel slice of the input buffer     */
  int32_t y_c_off, y_c_stride;    /* channel slice of the output buffer    */
  /* JR_F32_X6H only (ignored by every other dtype; zero-initialise): the
   * largest magnitude of x, of the filter block w and of dy, which set each
   * operand's power-of-two scale.  *_absmax: NULL, or 64 device floats whose
   * maximum is (an upper bound of) max |tensor| -- jr_absmax_prep for
   * filters, jr_bn_relu_bwd_multi_absmax / jr_bn_relu_bwd_maxpool_absmax for
   * a data gradient; when NULL, *_bound is a host upper bound (0: 2^14). */
  const float* x_absmax;
  const float* w_absmax;
  const float* dy_absmax;
  float x_bound, w_bound, dy_bound;
} jr_conv_desc;

/* 3x3 pooling window; max: stride 2 'valid', avg: stride 1 'same' with the
 * TF exclude-padding divisor. */
typedef struct jr_pool_desc {
  int32_t n, h, w, c;
  int32_t ho, wo;
  int32_t x_c_off, x_c_stride;
  int32_t y_c_off, y_c_stride;
} jr_pool_desc;

/* ---- library ---------------------------------------------------------- */
int jr_init(int device);
const char* jr_last_error(void);
const char* jr_version(void);
/* Device-side failures of the launches on the CURRENT device since the last
 * check (call it after synchronising the streams that ran them): JR_OK, or
 * JR_ERR_DEVICE when a stream-K hand-off word was not left zero: either a
 * kernel counted a count found past its tile's piece count into the
 * library's device error word, or a hand-off word of a stream with no work
 * in flight is non-zero (a stale count below the piece count, which makes a
 * tile complete early; the words of every idle stream are scanned here).
 * The outputs of the launches since the last check are then invalid.
 * Stream-K blocks never wait for one another, so no timeout exists.  On
 * JR_ERR_DEVICE the call synchronises the device, re-zeroes every stream-K
 * hand-off word and the error word, so the NEXT launches are correct.
 * Host-synchronising (a 4-byte copy plus the used hand-off words of each
 * idle stream; the repair path a device sync). */
int jr_device_check(void);
/* Diagnostics (tests): set every stream-K hand-off word of `stream` (the
 * current device's) to `value`, in stream order -- the next stream-K launch
 * there then miscounts and must be reported by jr_device_check. */
int jr_debug_poison_sk_counts(void* stream, uint32_t value);


/* ---- convolution (train.py:129-130 -> Keras Conv2D -> TF Conv2D,
 *      Conv2DBackpropInput, Conv2DBackpropFilter created by .minimize at
 *      train.py:150-153) ----------------------------------------------- */
/* c_out must be a multiple of 16.  Channel offsets/strides are multiples
 * of q = 4 (JR_F32) or 8 (JR_BF16) elements (one 16 B DMA piece).  c_in % q
 * != 0 (the 3-channel image of conv1) is supported for fwd / bwd_filter by
 * virtual padding to cq = round_up(c_in, q): the input buffer must hold cq
 * channels per pixel (x_c_off + cq <= x_c_stride) and channels [c_in, cq)
 * must be finite (zero).
 * Filter layouts: JR_F32 fwd / bwd_data and JR_BF16 bwd_data take the HWIO
 * kernel [kh][kw][c_in][c_out]; JR_BF16 fwd takes it transposed and padded,
 * [c_out][kh][kw][cq] (jr_conv_weights_bf16 produces both bf16 layouts);
 * bwd_filter writes fp32 HWIO for both dtypes.  JR_BF16 activations,
 * outputs and dx are bf16 (accumulation in fp32 MFMA, rounded once). */
size_t jr_conv2d_workspace_size(const jr_conv_desc* d, int op, int dtype);
/* y[.., y_c_off + co] = sum x * w   (raw conv output, no bias) */
int jr_conv2d_fwd(const jr_conv_desc* d, int dtype, const void* x, const void* w, void* y,
                  void* ws, size_t ws_bytes, void* stream);
/* jr_conv2d_fwd fused with the training-mode BatchNormalization statistics
 * of its output (Keras conv2d_bn: Conv2D -> BatchNormalization, App. C Q1):
 * mean[co] = E[y], invstd[co] = 1/sqrt(biased var + eps) over n*ho*wo rows,
 * of y as stored (bf16-rounded for JR_BF16).  Partial (mean, M2) per group
 * of rows from the GEMM epilogue (or the split-K reduce), combined in fp64
 * in a fixed order: deterministic.  Replaces jr_conv2d_fwd + jr_bn_stats. */
int jr_conv2d_fwd_bn_stats(const jr_conv_desc* d, int dtype, const void* x, const void* w, void* y, float eps,
                           float* mean, float* invstd, void* ws, size_t ws_bytes, void* stream);
/* Grouped jr_conv2d_fwd_bn_stats for the members of an ensemble (evaluate.py
 * -lm: the same layer of `members` models over the same batch, replacing the
 * reference's per-model sess.run of evaluate.py:166-211): ONE launch per GEMM,
 * member i reading x + i*x_member_stride and w + i*w_member_stride and
 * writing y + i*y_member_stride, mean / invstd + i*stats_member_stride
 * (strides in elements of each tensor; w = the filter operand of that dtype:
 * fp32 HWIO, or the bf16 W^T copy for JR_BF16).  dtype JR_F32, JR_BF16,
 * JR_F32_X8 or JR_F32_X6H (member i's magnitude words at x_absmax / w_absmax
 * + 64 i floats).  Each member's plan (tile, split-K) is the per-member plan, so
 * its y, mean and invstd are bitwise those of jr_conv2d_fwd_bn_stats on its
 * own tensors.  Workspace: jr_conv2d_workspace_size_grouped. */
size_t jr_conv2d_workspace_size_grouped(const jr_conv_desc* d, int dtype, int members);
int jr_conv2d_fwd_bn_stats_grouped(const jr_conv_desc* d, int dtype, int members, const void* x,
                                   int64_t x_member_stride, const void* w, int64_t w_member_stride, void* y,
                                   int64_t y_member_stride, float eps, float* mean, float* invstd,
                                   int64_t stats_member_stride, void* ws, size_t ws_bytes, void* stream);
/* The statistics finalize folded into the BN apply (a kernel boundary fewer
 * per conv2d_bn layer): jr_conv2d_bn_partials_layout says where the planned
 * forward GEMM of this geometry leaves its BN-statistics partials in the
 * workspace -- [2][N][P] fp32 (mean, M2) of R rows each (the last group the
 * rest of the M rows) at ws + ws_offset -- and whether they are single-stage;
 * jr_conv2d_fwd_bn_partials is jr_conv2d_fwd_bn_stats without the finalize
 * (JR_ERR_UNSUPPORTED for two-stage partials); jr_bn_relu_apply_stats then
 * combines the partials of its channels (bitwise the statistics
 * jr_conv2d_fwd_bn_stats writes), applies BN + ReLU and writes mean / invstd
 * for the backward.  The partials stay valid until the next call that uses
 * the same workspace. */
typedef struct jr_bn_partials {
  int64_t ws_offset;
  int32_t P, R, M, N;
  int32_t single_stage;
} jr_bn_partials;
int jr_conv2d_bn_partials_layout(const jr_conv_desc* d, int dtype, jr_bn_partials* out);
int jr_conv2d_fwd_bn_partials(const jr_conv_desc* d, int dtype, const void* x, const void* w, void* y, void* ws,
                              size_t ws_bytes, void* stream);
/* dx[.., x_c_off + ci] (+)= sum dy * w ; accumulate != 0 adds into dx */
int jr_conv2d_bwd_data(const jr_conv_desc* d, int dtype, const void* dy, const void* w, void* dx,
                       int accumulate, void* ws, size_t ws_bytes, void* stream);
/* dw[kh][kw][ci][co] = sum x * dy  (fp32 output for both dtypes) */
int jr_conv2d_bwd_filter(const jr_conv_desc* d, int dtype, const void* x, const void* dy, float* dw,
                         void* ws, size_t ws_bytes, void* stream);

/* Deferred filter-gradient reduce (one launch for many layers).  When the
 * planned bwd_filter GEMM of a layer splits K (jr_conv2d_wgrad_seg: splits
 * > 1), jr_conv2d_bwd_filter_slabs writes its fp32 partial slabs
 * [splits][m][n] (splits * m * n * 4 bytes) into caller memory and returns;
 * jr_wgrad_reduce later sums the slabs of every listed layer into its dw in
 * ONE launch, bitwise equal to jr_conv2d_bwd_filter's own reduce.  segs is
 * a DEVICE array; each entry is filled by jr_conv2d_wgrad_seg (geometry,
 * lanes g, blocks) plus the caller's slabs / dw pointers and block0 = the
 * exclusive prefix sum of blocks (total_blocks = the sum).  slab_bytes must
 * EQUAL the segment's splits * m * n * 4: a plan whose split count changed
 * since the segment was filled (another set_config / autotune on the same
 * geometry) fails with JR_ERR_INVALID instead of leaving stale slabs in the
 * reduce. */
typedef struct jr_wgrad_seg {
  const float* slabs;
  float* dw;
  int32_t m, n, splits, c_in, c_pad, g, block0, blocks;
} jr_wgrad_seg;
int jr_conv2d_wgrad_seg(const jr_conv_desc* d, int dtype, jr_wgrad_seg* seg);
int jr_conv2d_bwd_filter_slabs(const jr_conv_desc* d, int dtype, const void* x, const void* dy, float* slabs,
                               size_t slab_bytes, void* stream);
int jr_wgrad_reduce(const jr_wgrad_seg* segs, int32_t nseg, int32_t total_blocks, void* stream);

/* Time every candidate tile configuration of this op on the given buffers
 * (the output buffer is overwritten; host-synchronising) and cache the
 * fastest for later calls with the same geometry in this process.  Call
 * once per layer at plan time, outside graph capture. */
int jr_conv2d_autotune(const jr_conv_desc* d, int op, int dtype, const void* a, const void* b, void* c,
                       void* ws, size_t ws_bytes, void* stream);
/* Tile configuration the next call would use (DGRAD: per stride phase),
 * and an explicit override (reproducibility, tests).  A config id is
 * tile | (splits << 8), splits = 0: planner's split-K factor (at most
 * 1024); set_config
 * with cfg = -1 drops the override (autotuned or set) for that GEMM. */
int jr_conv2d_get_config(const jr_conv_desc* d, int op, int dtype, int phase);
int jr_conv2d_set_config(const jr_conv_desc* d, int op, int dtype, int phase, int cfg);
int jr_conv2d_num_configs(int dtype);   /* tiles of that dtype's table */
/* Process-wide counter, bumped whenever set_config or autotune CHANGES an
 * override (re-setting an equal value does not): a caller that bound plans
 * (e.g. deferred filter-gradient segments) re-applies its own configs when
 * the generation moved since it did. */
unsigned long long jr_conv2d_config_generation(void);

/* ---- BatchNormalization(scale=False, eps) + ReLU, training-mode batch
 *      statistics (Keras conv2d_bn; App. C Q1: always batch stats) ----- */
size_t jr_bn_workspace_size(int64_t m, int32_t c);
/* x: raw conv output [m][c] contiguous.  mean/invstd: [c] fp32 outputs.
 * invstd = 1/sqrt(biased_var + eps). */
int jr_bn_stats(int dtype, const void* x, int64_t m, int32_t c, float eps, float* mean, float* invstd,
                void* ws, size_t ws_bytes, void* stream);
/* y[.., y_c_off + k] = max((x[.., x_c_off + k] - mean) * invstd + beta, 0)
 * (x: a channel slice of the raw conv output, e.g. one member of a fused
 * sibling-conv group) */
int jr_bn_relu_apply(int dtype, const void* x, int32_t x_c_off, int32_t x_c_stride, int64_t m, int32_t c,
                     const float* mean, const float* invstd, const float* beta, void* y, int32_t y_c_off,
                     int32_t y_c_stride, void* stream);
/* BN + ReLU apply of a fused sibling launch's members in ONE launch: x
 * spans the launch's c channels; segment i (channels [sum_{j<i} c_j, ... +
 * c_i), sum c_i = c, each a multiple of 4 fp32 / 8 bf16) writes its own
 * output slice with its own beta.  Per element bitwise jr_bn_relu_apply.
 * 1 <= nseg <= 4. */
typedef struct jr_bn_apply_seg {
  void* y;
  int32_t y_c_off, y_c_stride, c;
  const float* beta;
} jr_bn_apply_seg;
int jr_bn_relu_apply_multi(int dtype, int nseg, const jr_bn_apply_seg* segs, const void* x, int32_t x_c_off,
                           int32_t x_c_stride, int64_t m, int32_t c, const float* mean, const float* invstd,
                           void* stream);
/* jr_bn_relu_apply with the statistics finalize folded in: mean / invstd of
 * the c channels come from the single-stage partials of the producing conv
 * (jr_conv2d_fwd_bn_partials): part = ws + ws_offset, layout [2][n_total][P]
 * of R rows each over m rows, this slice's channels starting at stat_c_off
 * of n_total; mean / invstd [c] are written too (for the backward). */
int jr_bn_relu_apply_stats(int dtype, const void* x, int32_t x_c_off, int32_t x_c_stride, int64_t m, int32_t c,
                           const float* part, int32_t P, int32_t R, int32_t n_total, int32_t stat_c_off, float eps,
                           float* mean, float* invstd, const float* beta, void* y, int32_t y_c_off,
                           int32_t y_c_stride, void* stream);
/* jr_bn_relu_apply for the members of an ensemble in one launch: member i
 * reads x + i*x_member_stride, mean / invstd + i*stats_member_stride, beta +
 * i*beta_member_stride and writes y + i*y_member_stride (elements). */
int jr_bn_relu_apply_grouped(int dtype, int32_t members, const void* x, int32_t x_c_off, int32_t x_c_stride,
                             int64_t x_member_stride, int64_t m, int32_t c, const float* mean, const float* invstd,
                             int64_t stats_member_stride, const float* beta, int64_t beta_member_stride, void* y,
                             int32_t y_c_off, int32_t y_c_stride, int64_t y_member_stride, void* stream);
/* Backward of apply+stats: dy is the gradient w.r.t. y (a channel slice),
 * dx receives the gradient w.r.t. the raw conv output in the same channel
 * slice geometry as x, dbeta [c] receives sum of the ReLU-masked dy. */
int jr_bn_relu_bwd(int dtype, const void* dy, int32_t dy_c_off, int32_t dy_c_stride, const void* x,
                   int32_t x_c_off, int32_t x_c_stride, int64_t m, int32_t c, const float* mean,
                   const float* invstd, const float* beta, void* dx, float* dbeta, void* ws, size_t ws_bytes,
                   void* stream);
/* The same backward for the members of a fused sibling launch in ONE set of
 * launches: x / dx / mean / invstd span the launch's c channels; segment i
 * (channels [sum_{j<i} c_j, ... + c_i), sum c_i = c, each c_i a multiple of
 * 4 fp32 / 8 bf16) brings its own upstream gradient slice and its own beta /
 * dbeta.  1 <= nseg <= 4.  jr_bn_relu_bwd is the one-segment case. */
typedef struct jr_bn_seg {
  const void* dy;
  int32_t dy_c_off, dy_c_stride, c;
  const float* beta;
  float* dbeta;
} jr_bn_seg;
int jr_bn_relu_bwd_multi(int dtype, int nseg, const jr_bn_seg* segs, const void* x, int32_t x_c_off,
                         int32_t x_c_stride, int64_t m, int32_t c, const float* mean, const float* invstd, void* dx,
                         void* ws, size_t ws_bytes, void* stream);
/* jr_bn_relu_bwd_multi that also raises dx_absmax (64 device floats the
 * caller zeroed before the first launch that feeds them) so that their max
 * is max |dx| of every launch that fed them: the dy_absmax of the
 * JR_F32_X6H data- / filter-gradient GEMMs reading dx. */
int jr_bn_relu_bwd_multi_absmax(int dtype, int nseg, const jr_bn_seg* segs, const void* x, int32_t x_c_off,
                                int32_t x_c_stride, int64_t m, int32_t c, const float* mean, const float* invstd,
                                void* dx, void* ws, size_t ws_bytes, float* dx_absmax, void* stream);
/* Up to 8 independent conv2d_bn backwards (the branch-final layers of one
 * Inception block, whose upstream gradients become final together) in ONE
 * set of three launches; layer l is exactly the jr_bn_relu_bwd_multi call
 * with its fields (bitwise the same results), each with at most 512 reduce
 * chunks (the 35^2 / 17^2 / 8^2 shapes at batch 64; larger ones:
 * JR_ERR_UNSUPPORTED).  ws: jr_bn_relu_bwd_batch_workspace_size bytes. */
typedef struct jr_bn_bwd_layer {
  int32_t nseg;
  jr_bn_seg segs[4];
  const void* x;
  int32_t x_c_off, x_c_stride;
  int64_t m;
  int32_t c;
  const float* mean;
  const float* invstd;
  void* dx;
} jr_bn_bwd_layer;
size_t jr_bn_relu_bwd_batch_workspace_size(int32_t n, const jr_bn_bwd_layer* layers);
int jr_bn_relu_bwd_batch(int dtype, int32_t n, const jr_bn_bwd_layer* layers, void* ws, size_t ws_bytes,
                         void* stream);
/* The backward of a conv2d_bn layer whose output only a 3x3/2 max-pool reads
 * (forward: jr_bn_relu_maxpool3x3s2_fwd): the max-pool backward writes dy
 * (d's x slice, from the pooled gradient at d's y slice and the argmax) and
 * adds the BN backward's reduction sums from the same registers, then the
 * finalize and the dx pass run as in jr_bn_relu_bwd -- one read of dy fewer.
 * x: the raw conv output [n*h*w] x x_c_stride (channels 0..d->c), dx: its
 * gradient in that geometry; d->c a multiple of 4, <= 1024.  ws: at least
 * jr_bn_relu_bwd_maxpool_workspace_size(d) bytes. */
size_t jr_bn_relu_bwd_maxpool_workspace_size(const jr_pool_desc* d);
int jr_bn_relu_bwd_maxpool(int dtype, const jr_pool_desc* d, const uint8_t* argmax, const void* pooled_dy, void* dy,
                           const void* x, int32_t x_c_stride, const float* mean, const float* invstd,
                           const float* beta, void* dx, float* dbeta, void* ws, size_t ws_bytes, void* stream);
/* ... raising dx_absmax as jr_bn_relu_bwd_multi_absmax does. */
int jr_bn_relu_bwd_maxpool_absmax(int dtype, const jr_pool_desc* d, const uint8_t* argmax, const void* pooled_dy,
                                  void* dy, const void* x, int32_t x_c_stride, const float* mean, const float* invstd,
                                  const float* beta, void* dx, float* dbeta, void* ws, size_t ws_bytes,
                                  float* dx_absmax, void* stream);

/* ---- pooling (Keras MaxPooling2D((3,3),(2,2)) / AveragePooling2D((3,3),
 *      (1,1),'same') inside InceptionV3, train.py:129-130) ------------ */
/* argmax [n][ho][wo][c] uint8 (window position 0..8, first max in scan
 * order) is written by fwd when non-NULL and routes the gradient in bwd. */
int jr_maxpool3x3s2_fwd(const jr_pool_desc* d, int dtype, const void* x, void* y, uint8_t* argmax,
                        void* stream);
int jr_maxpool3x3s2_bwd(const jr_pool_desc* d, int dtype, const uint8_t* argmax, const void* dy,
                        void* dx, int accumulate, void* stream);
/* The fused forward of a conv2d_bn layer whose only reader is a max-pool
 * (the stem's conv2d_3 / conv2d_5 outputs): raw is the conv output (the
 * descriptor's x slice), each tap is max(bn_pre(raw), 0) in the path dtype
 * (jr_bn_relu_apply's value), then the max-pool as jr_maxpool3x3s2_fwd --
 * y and argmax bitwise the two calls', without the full-resolution
 * activation.  mean / invstd / beta: [c] fp32. */
int jr_bn_relu_maxpool3x3s2_fwd(const jr_pool_desc* d, int dtype, const void* raw, const float* mean,
                                const float* invstd, const float* beta, void* y, uint8_t* argmax, void* stream);
/* The same over the members of an ensemble as one batch of d->n images:
 * image b belongs to member b / images_per_member, whose mean / invstd sit
 * stats_member_stride and beta beta_member_stride floats further. */
int jr_bn_relu_maxpool3x3s2_fwd_grouped(const jr_pool_desc* d, int dtype, int32_t images_per_member,
                                        const void* raw, const float* mean, const float* invstd,
                                        int64_t stats_member_stride, const float* beta, int64_t beta_member_stride,
                                        void* y, uint8_t* argmax, void* stream);
int jr_avgpool3x3s1_fwd(const jr_pool_desc* d, int dtype, const void* x, void* y, void* stream);
int jr_avgpool3x3s1_bwd(const jr_pool_desc* d, int dtype, const void* dy, void* dx, int accumulate,
                        void* stream);

/* ---- GlobalAveragePooling2D (pooling='avg', train.py:130) ------------ */
int jr_gap_fwd(int dtype, const void* x, int32_t n, int32_t hw, int32_t c, float* y, void* stream);
int jr_gap_bwd(int dtype, const float* dy, int32_t n, int32_t hw, int32_t c, void* dx, void* stream);

/* ---- head: tf.layers.dense(units) (train.py:133) + tf.sigmoid
 *      'predictions' (train.py:136) + reduce_mean(sigmoid xent)
 *      (train.py:140-141).  Softmax mode = softmax cross-entropy.
 *      labels may be NULL (inference: loss not computed). ----------- */
int jr_head_fwd(int mode, const float* feat, const float* w, const float* b, const float* labels,
                int32_t n, int32_t c, int32_t units, float* logits, float* probs, float* loss,
                void* stream);
int jr_head_bwd(int mode, const float* feat, const float* w, const float* probs, const float* labels,
                int32_t n, int32_t c, int32_t units, float* dfeat, float* dw, float* db, void* stream);

/* ---- optimizers (train.py:147-153: GradientDescentOptimizer /
 *      MomentumOptimizer(use_nesterov=True) -> TF ApplyMomentum) ------- */
/* accum = accum*momentum + g; w -= g*lr + accum*momentum*lr   (g = grad*grad_scale) */
int jr_nesterov_update(float* w, const float* grad, float* accum, int64_t n, float lr,
                       float momentum, float grad_scale, void* stream);
/* plain momentum (use_nesterov=False): accum = accum*m + g; w -= lr*accum */
int jr_momentum_update(float* w, const float* grad, float* accum, int64_t n, float lr,
                       float momentum, float grad_scale, void* stream);
int jr_sgd_update(float* w, const float* grad, int64_t n, float lr, float grad_scale, void* stream);
/* Adam (north-star extra, not in the reference): TF AdamOptimizer form */
int jr_adam_update(float* w, const float* grad, float* m, float* v, int64_t n, float lr_t,
                   float beta1, float beta2, float eps, float grad_scale, void* stream);

/* ---- bf16 filter copies (the bf16 conv path's weight operands) -------
 * From the fp32 master kernel [kh][kw][c_in][c_out] write
 *   w_hwio: bf16 [kh][kw][c_in][c_out]        (jr_conv2d_bwd_data, JR_BF16)
 *   w_t:    bf16 [c_out][kh][kw][c8], c8 = round_up(c_in, 8), zero padded
 *           (jr_conv2d_fwd, JR_BF16)
 * Either output may be NULL.  The _multi form does every layer of a model
 * in one launch from a DEVICE array of jr_wprep (offsets in elements from
 * the three bases; tile_start = exclusive prefix sum of
 * jr_conv_weights_bf16_tiles over the layers). */
typedef struct jr_wprep {
  int64_t src_off, hwio_off, wt_off;
  int32_t kh, kw, c_in, c_out;
  int32_t tile_start, reserved;
} jr_wprep;
int32_t jr_conv_weights_bf16_tiles(int32_t kh, int32_t kw, int32_t c_in, int32_t c_out);
int jr_conv_weights_bf16(const float* w, int32_t kh, int32_t kw, int32_t c_in, int32_t c_out, void* w_hwio,
                         void* w_t, void* stream);
int jr_conv_weights_bf16_multi(const jr_wprep* layers, int32_t n_layers, int32_t total_tiles, const float* src,
                               void* hwio, void* wt, void* stream);
/* JR_F32_X8P filter operands: the same two layouts as three bf16 planes
 * each (h, m, l of the exact split), plane stride = the layer's element
 * count (kh*kw*c_in*c_out for HWIO, c_out*kh*kw*c8 for W^T); in the _multi
 * form hwio_off / wt_off address each layer's first plane. */
int jr_conv_weights_x8p(const float* w, int32_t kh, int32_t kw, int32_t c_in, int32_t c_out, void* w_hwio,
                        void* w_t, void* stream);
int jr_conv_weights_x8p_multi(const jr_wprep* layers, int32_t n_layers, int32_t total_tiles, const float* src,
                              void* hwio, void* wt, void* stream);
/* Exact three-way bf16 split of an fp32 activation / gradient slice for
 * JR_F32_X8P: h = bf16_rn(x), m = bf16_rn(x - h), l = x - h - m (exact in
 * bf16).  src [rows][src_stride] channels [src_off, src_off + c) ->
 * dst + p * plane_stride (p = 0, 1, 2 for h, m, l), each [rows][dst_stride],
 * channels [dst_off, dst_off + c_pad); channels c..c_pad-1 are written as
 * zeros (the conv1 image: c = 3, c_pad = 8). */
int jr_split_x8p(const float* src, int64_t rows, int32_t c, int32_t src_off, int32_t src_stride, void* dst,
                 int32_t c_pad, int32_t dst_off, int32_t dst_stride, int64_t plane_stride, void* stream);

/* JR_F32_X6H operand magnitudes of parameter blocks (once per step, before
 * the forward): out[0 .. zero_floats) is zeroed (in stream order), then for
 * each segment the 64 floats out[seg.out * 64 ...] are raised so that their
 * max is max |src[off .. off + count)| (a conv launch's filter block: its
 * w_absmax).  limit > 0: a max above it counts a failure into the
 * device error word, which jr_device_check reports (JR_ERR_DEVICE) -- the
 * guard of a host bound that rests on these values (the BN betas bound the
 * activations: |relu(xhat + beta)| <= sqrt(N - 1) + max |beta|). */
typedef struct jr_absmax_seg {
  int64_t off, count;
  int32_t out;
  float limit;
} jr_absmax_seg;
int jr_absmax_prep(const float* src, const jr_absmax_seg* segs, int32_t nseg, float* out, int64_t zero_floats,
                   void* stream);

/* ---- dtype helpers --------------------------------------------------- */
int jr_cast_f32_to_bf16(const float* src, void* dst, int64_t n, void* stream);
int jr_cast_bf16_to_f32(const void* src, float* dst, int64_t n, void* stream);
/* uint8 HWC images -> f32 * f32(1/255) (tf.image.convert_image_dtype,
 * lib/dataset.py:20-21) */
int jr_u8_to_f32_scaled(const uint8_t* src, void* dst, int dtype, int64_t n, void* stream);
/* uint8 [pixels][c] images -> dst [pixels][dst_stride] of f32(x) * f32(1/255),
 * channels [c, dst_stride) set to 0 (the conv1 input is kept 4 channels
 * wide, see jr_conv2d_fwd on c_in % 4 != 0). */
int jr_image_u8_to_nhwc(const uint8_t* src, void* dst, int dtype, int64_t pixels, int32_t c,
                        int32_t dst_stride, void* stream);
/* acc[0] += sum (p - y)^2, acc[1] += n   (tf.metrics.mean_squared_error,
 * train.py:175-177) */
int jr_brier_accumulate(const float* probs, const float* labels, int32_t n, double* acc, void* stream);

/* ---- host (CPU) helpers: TFRecord container and Example records ----- */
uint32_t jr_crc32c(const uint8_t* data, size_t n, uint32_t crc);
/* TFRecord masked CRC32C: ((c >> 15) | (c << 17)) + 0xa282ead8 */
uint32_t jr_masked_crc32c(const uint8_t* data, size_t n);
/* Index the records of one TFRecord file image in memory (replaces the
 * record walk of tf.data.TFRecordDataset behind lib/dataset.py:5-8,44-47).
 * Writes the payload offset/length of each record; stops at the first damaged
 * record (truncated, or CRC mismatch when verify != 0) with *n_records = the
 * good records before it and JR_ERR_INVALID.  offsets == NULL only counts. */
int jr_tfrecord_index(const uint8_t* buf, size_t len, int verify, uint64_t* offsets, uint64_t* lengths,
                      size_t cap, size_t* n_records);
/* Locate the lib/dataset.py:12-16 FixedLenFeatures (image/encoded,
 * image/format, image/class/label, image/height, image/width) in n serialized
 * tf.train.Example records at base + offsets[i] (replaces the
 * tf.parse_single_example of lib/dataset.py:17).  status[i]: 0 ok; > 0 bitmask
 * of keys missing / not exactly one value / wrong list type (bit k = key k in
 * the order above); -1 malformed protobuf.  enc_off is relative to base. */
int jr_example_parse_image(const uint8_t* base, const uint64_t* offsets, const uint64_t* lengths, size_t n,
                           uint64_t* enc_off, uint64_t* enc_len, int64_t* label, int64_t* height,
                           int64_t* width, int32_t* status);

/* ---- collectives: data-parallel gradient exchange over RCCL / xGMI ----
 * Replaces the reference's only multi-GPU path, the external
 * tf_cnn_benchmarks parameter server (benchmarks.yaml.jinja.example:81-90;
 * SURVEY.md §2 row 14, §8b/§8e): one communicator per process (one process
 * per GPU), in-place sum of the flat gradient enqueued on the caller's
 * stream.  The 128-byte unique id comes from rank 0's jr_comm_unique_id and
 * reaches the other ranks through the caller's bootstrap, or through a file
 * (jr_comm_init_file: rank 0 writes it, tagged with run_id, with an atomic
 * rename; the others poll up to timeout_ms, < 0 = forever, for the file of
 * THEIR run_id, so an id an earlier job left at uid_path is never joined;
 * run_id: any non-empty string every rank of one job shares, e.g. the
 * launcher's rendezvous id). */
#define JR_COMM_ID_BYTES 128
typedef struct jr_comm jr_comm;
int jr_comm_unique_id(uint8_t* id);
int jr_comm_init(int rank, int world, const uint8_t* id, int device, jr_comm** comm);
int jr_comm_init_file(int rank, int world, const char* uid_path, const char* run_id, int device, int timeout_ms,
                      jr_comm** comm);
/* buf[0..n) = sum over the ranks of buf[0..n), dtype JR_F32 or JR_BF16 */
int jr_allreduce_sum(jr_comm* comm, void* buf, size_t n, int dtype, void* stream);
int jr_comm_rank(const jr_comm* comm);
int jr_comm_world(const jr_comm* comm);
int jr_comm_destroy(jr_comm* comm);

/* ---- HIP graph capture of a whole step ------------------------------ */
int jr_graph_begin(void* stream);
int jr_graph_end(void* stream, void** graph_exec);
int jr_graph_launch(void* graph_exec, void* stream);
int jr_graph_destroy(void* graph_exec);
/* Device regions the library allocated for a capture (stream-K hand-off
 * flags of captured conv GEMMs) and released by jr_graph_destroy (tests). */
int jr_graph_regions(void* graph_exec);

/* ---- Cross-stream ordering of the branch lanes ---------------------- */
/* Events for device-side ordering between the library's callers' streams
 * (jr.lanes: a consumer on one lane waits for its producer on another):
 * no timing and no system-scope fence -- device memory only, the only
 * thing the lanes order.  (A recorded DisableSystemFence event costs the
 * producer's queue ~1.1 us less than a default one: profiles/r05_sync_probe2.txt.) */
int jr_event_create(void** event);
int jr_event_record(void* event, void* stream);
int jr_stream_wait_event(void* stream, void* event);
int jr_event_destroy(void* event);

#ifdef __cplusplus
}
#endif
#endif /* JR_H_ */
