/*
 * sr_hip.h — C ABI of the MI355X (gfx950) super-resolution engine (libsr_hip.so).
 *
 * This is the drop-in boundary for the hot path named by BASELINE.json:north_star:
 * the SR network forward/backward (EDSR / RCAN / RRDBNet / SwinIR) and the three
 * native ops of basicsr/ops (DCN, fused_act, upfirdn2d).  Every entry point takes
 * plain device pointers, sizes and a hipStream_t (passed as void*), never allocates,
 * never synchronises, and returns 0 on success or a negative sr_status code; the
 * message of the last failure on the calling thread is available from
 * sr_last_error().  The Python host layer (basicsr4rs_amd/_lib.py) binds these with
 * ctypes and raises RuntimeError on a non-zero status, matching the reference's
 * TORCH_CHECK -> RuntimeError behaviour (basicsr/ops/dcn/src/deform_conv_cuda.cpp:511-516).
 *
 * Reference interfaces replaced (file:line in the reference checkout):
 *   sr_conv3x3_*         nn.Conv2d(C, C', 3, 1, 1) as instantiated in
 *                        basicsr/archs/arch_util.py:78-79, edsr_arch.py:44-48,
 *                        rcan_arch.py:40-42, rrdbnet_arch.py:21-25, swinir_arch.py:543
 *                        (cuDNN in the reference; no reference kernel exists)
 *   sr_pixel_shuffle     nn.PixelShuffle (arch_util.py:136,139) and
 *                        pixel_unshuffle (arch_util.py:217-234)
 *   sr_l1_loss           L1Loss (basicsr/losses/basic_loss.py:27-52)
 *   sr_dcn_*             deform_conv_ext.modulated_deform_conv_forward/backward
 *                        (basicsr/ops/dcn/src/deform_conv_ext.cpp:107-147)
 *   sr_fused_bias_act    fused_act_ext.fused_bias_act (basicsr/ops/fused_act/src/fused_bias_act.cpp:14-26)
 *   sr_upfirdn2d         upfirdn2d_ext.upfirdn2d (basicsr/ops/upfirdn2d/src/upfirdn2d.cpp:10-24)
 */
#ifndef SR_HIP_H
#define SR_HIP_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

enum sr_dtype { SR_F32 = 0, SR_BF16 = 1 };
enum sr_status { SR_OK = 0, SR_EINVAL = -1, SR_ELAUNCH = -2, SR_ETOOBIG = -3 };
enum sr_act { SR_ACT_NONE = 0, SR_ACT_RELU = 1, SR_ACT_LRELU = 2 };

/* Library identity / error reporting. */
const char* sr_version(void);
const char* sr_last_error(void);
/* Tuning knobs (A/B switches and split-plan targets, not part of the reference interface).  Each
 * knob is its environment variable of the same name (SR_RING_SPLITS, SR_LWK, SR_DCN_GX_FX, ...), read
 * once per process; sr_set_knob overrides it at run time (value < 0: back to the built-in default)
 * and stores the previous value in *previous when non-NULL.  sr_get_knob returns the current value
 * (-1 unset, -2 unknown name). */
int sr_set_knob(const char* name, int value, int* previous);
int sr_get_knob(const char* name);

/* ---------------------------------------------------------------------------------
 * 3x3 convolution, stride 1, zero padding 1 (implicit GEMM on MFMA).
 *
 * Feature maps are NHWC with an explicit pixel stride (ld*) and channel offset
 * (*coff), element type `dtype`.  Channel counts are the padded GEMM counts
 * (multiples of 8); padded weight rows/columns are zero.
 *
 * Forward:  y = beta*res + alpha * gate_factor * act(conv(x, w) + bias)
 *   in_ps  = r > 0: x is the pixel-shuffled tensor [N, H*r, W*r, Cin/r^2] and GEMM
 *                   input channel k = (i*r + j)*(Cin/r^2) + c is gathered from it
 *                   (dgrad of an Upsample conv reads its pixel-shuffled grad directly).
 *   out_ps = r > 0: output GEMM column n = s*(Cout/r^2) + c is stored pixel-shuffled
 *                   at [n, y*r + s/r, x*r + s%r, c]  (nn.PixelShuffle fused in the store).
 *   out_nchw = 1:   store fp32 NCHW [N, Cout_real, H, W] as v*aff_scale[c] + aff_shift[c]
 *                   (EDSR/RCAN mean un-shift fused into conv_last).
 * w    : [Cout][ldw] GEMM weight rows, K index = tap*Cin + ci (tap = ky*3 + kx).
 * gate : optional, output layout; v *= (gate > 0 ? 1 : gate_slope)  (ReLU/LReLU backward).
 * ------------------------------------------------------------------------------- */
typedef struct sr_conv3x3_desc {
  int dtype;
  int N, H, W;
  int Cin, ldx, xcoff, in_ps;
  int Cout, Cout_real, ldw;
  int ldy, ycoff, out_ps, out_nchw;
  int act;
  float slope, alpha;
  int ldg, gcoff;
  float gate_slope;
  int ldr, rcoff;
  float beta;
  int ldr2, r2coff;
  float beta2;
  int rcols;  /* residuals apply to output columns n < rcols (0 = all) */
  int in_up;  /* x is the [N, H/u, W/u] map read through nearest-neighbour upsampling (0/1 = none) */
  int ksize;  /* 3 (default, 0 = 3) or 1: a 1x1 conv = nn.Linear over the NHWC tokens */
  int gate_mode; /* 0: v *= (gate > 0 ? 1 : gate_slope); 1: v *= gate (gate = the GELU' map a GELU
                  forward stored as its aux: the backward evaluates no erf);
                  2: after the residuals, v *= (gate > 0 ? 1 : gate_slope) on output columns
                  gcol0 <= n < gcol1 only (activation backward of a dense-block slice whose
                  gradient this call completes) */
  int gcol0, gcol1;
  const float* row_scale; /* optional fp32 [N]: alpha of every output pixel of image n is multiplied by
                             row_scale[n] (per-sample stochastic depth, swinir_arch.py:14-40, fused into
                             the proj / fc2 residual epilogues); NULL = 1 */
  const void* dot; /* optional, with colsum: the partial sums are of y * dot (bf16 [M][ldd], channel
                      columns dcoff.. in y's channel order) instead of y -- RCAN's channel-attention
                      backward dot sum_p dy * u (rcan_arch.py:19-27) fused into the conv dgrad that
                      produces dy; band kernel only (bf16, 64 -> 64 channels, W 64 / 128) */
  int ldd, dcoff;
} sr_conv3x3_desc;

/* A SwinIR block's LayerNorm fused into the following linear (norm1 -> attn.qkv, norm2 -> mlp.fc1:
 * basicsr/archs/swinir_arch.py:240, 251, 289-291, 320-323): y = Linear(LayerNorm(x)) on bf16
 * token rows [M][Cin] (dense, ldx == Cin), LayerNorm over the first ln_C channels (fp32 statistics,
 * eps), the normalised rows also written to ln_out [M][Cin] (padded columns zero) with the per-row
 * mean / rstd, as sr_layernorm_fwd would (they feed the weight gradient and the LayerNorm
 * backward).  The linear is sr_conv3x3_fwd's ksize-1 path with a plain (act 0) or GELU +
 * GELU' aux epilogue and Cin <= 192, Cout <= 640. */
int sr_linear_ln_fwd(const sr_conv3x3_desc* d, const void* x, const float* ln_gamma, const float* ln_beta, int ln_C,
                     float eps, void* ln_out, float* ln_mean, float* ln_rstd, const void* w, const float* bias, void* y,
                     void* aux, void* stream);


/* y = beta*res + beta2*res2 + alpha * gate_factor * act(conv(x, w) + bias); res/res2/gate may be NULL.
 * act: SR_ACT_* or 3 = GELU (exact erf).  aux (may be NULL): also store, in y's layout, GELU'(z) for
 * act 3 (z = conv(x, w) + bias; the fc2 dgrad's gate_mode-1 factor, computed with the GELU from one
 * erf) and z itself for the other activations.  colsum (may be NULL): fp32
 * [N * P][Cout] partial channel sums of y as stored, P = sr_conv3x3_fwd_colsum_parts(d) rows per
 * image, sum_p colsum[n*P + p][c] = sum over image n's pixels of y[n, pixel, c] -- RCAN's
 * AdaptiveAvgPool2d(1) (rcan_arch.py:19) fused into the conv that produces its input. */
int sr_conv3x3_fwd(const sr_conv3x3_desc* d, const void* x, const void* w, const float* bias,
                   const void* gate, const void* res, const void* res2, const float* aff_scale,
                   const float* aff_shift, void* y, void* aux, float* colsum, void* stream);
/* Partial rows per image of sr_conv3x3_fwd's colsum for this descriptor (0: not available). */
/* 1 when a call with this descriptor plus a residual, colsum and the dot operand (sr_conv3x3_desc.dot)
 * runs on the band kernel's fused epilogue, else 0 (the caller then computes the dot separately). */
int sr_conv3x3_fwd_dot_ok(const sr_conv3x3_desc* d);
int sr_conv3x3_fwd_colsum_parts(const sr_conv3x3_desc* d);

/* Name of the GPU kernel that sr_conv3x3_fwd / sr_conv3x3_wgrad would launch for a
 * descriptor (static string; for traces and profiler summaries). */
const char* sr_conv3x3_fwd_kernel_name(const sr_conv3x3_desc* d);
const char* sr_conv3x3_wgrad_kernel_name(const struct sr_conv3x3_wgrad_desc* d);
/* Number of kernel launches one sr_conv3x3_fwd call makes for a descriptor (1, or the 64-channel
 * output slices of the sliced band form) -- the per-launch unit of traces and profiler summaries. */
int sr_conv3x3_fwd_launches(const sr_conv3x3_desc* d);

/* Kernel-variant selection for A/B tests: 0 = automatic (default), 1 = never use the
 * 256x256 LDS-DMA kernel (all shapes on the 128-row register-staged kernels). */
int sr_conv3x3_set_variant(int variant);
int sr_conv3x3_get_variant(void); /* the current kernel-variant switch */
/* Diagnostics (not part of the reference interface): per-block clock stamps of the row-band
 * forward kernel into a device buffer of 16 uint64 per block; NULL turns them off. */
int sr_conv3x3_set_stamps(void* buf);

/* Weight gradient: dw[co][ci][ky][kx] = scale * sum_pixels dy[p][co'] * x[p + tap][ci]
 * (param layout, fp32, co = perm(co') undoing out_ps), db[co] = scale * sum_p dy[p][co'].
 * dy is read in GEMM column order (gathered when out_ps > 0).  Needs a workspace of
 * sr_conv3x3_wgrad_workspace(d) bytes (split-K fp32 partial slabs, deterministic). */
typedef struct sr_conv3x3_wgrad_desc {
  int dtype;
  int N, H, W;
  int Cin, Cin_real, ldx, xcoff;
  int Cout, Cout_real, ldy, ycoff, out_ps;
  float scale;
  int in_up;  /* x read through nearest-neighbour upsampling by in_up (0/1 = none) */
  int ksize;  /* 3 (0 = 3) or 1 */
  int accumulate;  /* 1: dw += result, db += result (gradient accumulation in place, e.g. into
                      a flat .grad buffer); 0: overwrite */
} sr_conv3x3_wgrad_desc;

size_t sr_conv3x3_wgrad_workspace(const sr_conv3x3_wgrad_desc* d);
/* co_map[co] / ci_map[ci] (optional, device int arrays over the real param rows / cols) give
 * the GEMM column / input channel of each parameter row / column (padded head layouts). */
int sr_conv3x3_wgrad(const sr_conv3x3_wgrad_desc* d, const void* dy, const void* x,
                     void* workspace, size_t ws_bytes, float* dw, float* db, const int* co_map,
                     const int* ci_map, void* stream);
/* accumulate bit 1 of the descriptor: sr_conv3x3_wgrad writes only the split-K slab into the
 * workspace; sr_conv3x3_wgrad_reduce (same descriptor and workspace, e.g. on another stream)
 * then reduces it into dw / db (bit 0 of accumulate as for sr_conv3x3_wgrad). */
int sr_conv3x3_wgrad_reduce(const sr_conv3x3_wgrad_desc* d, void* workspace, size_t ws_bytes, float* dw, float* db,
                            const int* co_map, const int* ci_map, void* stream);

/* Weight preparation from the nn.Conv2d parameter w[Cout_real][Cin_real][3][3] (fp32):
 *   wf[n][tap*Cin + ci]       forward GEMM rows (n = GEMM column, permuted by out_ps)
 *   wd[ci][tap'*Cout + n]     dgrad GEMM rows (spatially flipped, transposed)
 *   bias_g[n]                 bias in GEMM column order (zero for padded columns)
 * Any of wf / wd / bias_g may be NULL. */
int sr_conv3x3_prep(int dtype, const float* w, const float* bias, int Cout_real, int Cin_real,
                    int Cout, int Cin, int out_ps, void* wf, void* wd, float* bias_g,
                    void* stream);
/* One conv / linear weight of a batched GEMM-image preparation (same meaning as the arguments
 * of sr_conv_prep_mapped; ksize 1 or 3). */
typedef struct {
  const float* w;
  const float* bias;
  int Cout_real, Cin_real, Cout, Cin, out_ps, ksize;
  const int* row_map;
  const int* col_map;
  void* wf;
  void* wd;
  float* bias_g;
} sr_prep_item;
/* Blocks (32 x 32 GEMM-row x channel tiles) item needs (host helper for building block_start). */
int sr_conv_prep_blocks(const sr_prep_item* item);
/* sr_conv_prep_mapped for n items in ONE launch: items and block_start (n + 1 prefix sums of
 * sr_conv_prep_blocks, block_start[n] = total_blocks) in device memory, all items of dtype.
 * Replaces the per-parameter re-preparation after every optimizer step. */
int sr_conv_prep_batch(int dtype, const sr_prep_item* items, const int* block_start, int n, int total_blocks,
                       void* stream);
/* General form: ksize 1 or 3; row_map[n] (n < Cout) = parameter row of GEMM column n or -1
 * (zero row), col_map[k] (k < Cin) = parameter column of GEMM input channel k or -1; NULL maps
 * = identity (+ out_ps permutation).  nn.Linear weights are [out][in] = 1x1 conv weights. */
int sr_conv_prep_mapped(int dtype, int ksize, const float* w, const float* bias, int Cout_real,
                        int Cin_real, int Cout, int Cin, int out_ps, const int* row_map,
                        const int* col_map, void* wf, void* wd, float* bias_g, void* stream);

/* ---------------------------------------------------------------------------------
 * Layout / elementwise ops (HBM-bound).
 * ------------------------------------------------------------------------------- */
/* NCHW fp32 [N,C,H,W] -> NHWC dtype [N,H,W,Cp] (channels >= C zero):
 *   y = (x - shift[c]) * scale[c]   (shift/scale may be NULL -> 0 / 1). */
int sr_nchw_to_nhwc(int dtype, const float* x, int N, int C, int H, int W, int Cp,
                    const float* shift, const float* scale, void* y, void* stream);
/* NHWC dtype [N,H,W,ld] (channel offset coff) -> NCHW fp32 [N,C,H,W], y = x*scale[c]+shift[c]. */
int sr_nhwc_to_nchw(int dtype, const void* x, int N, int H, int W, int ld, int coff, int C,
                    const float* scale, const float* shift, float* y, void* stream);
/* Pixel shuffle (r > 0) / unshuffle (r < 0) on NCHW tensors of dtype, bit-exact index map
 * out[n, c, h*r+i, w*r+j] = in[n, c*r*r + i*r + j, h, w]; C/H/W are of the INPUT. */
int sr_pixel_shuffle_nchw(int dtype, const void* x, int N, int C, int H, int W, int r, void* y,
                          void* stream);
/* L1 loss partial sums + gradient: loss = weight * mean|pred - gt| (reduction 'mean') or
 * weight * sum (reduction 'sum'); grad = weight * sign(pred - gt) / norm.  Writes the loss to
 * *loss (fp32 device scalar) and the gradient to grad (may be NULL).  fp32 tensors. */
int sr_l1_loss(const float* pred, const float* gt, int64_t n, float weight, int mean,
               float* loss, float* grad, void* workspace, size_t ws_bytes, void* stream);
size_t sr_l1_loss_workspace(int64_t n);
/* Activation backward: out = alpha * dy * (y > 0 ? 1 : neg), neg = 0 for SR_ACT_RELU, slope for
 * SR_ACT_LRELU, 1 for SR_ACT_NONE; y is the activation OUTPUT (same sign as its input). */
int sr_act_backward(int dtype, const void* dy, const void* y, int64_t n, int act, float slope, float alpha,
                    void* out, void* stream);
/* out[m][c] = x[m][c] * scale[m / HW] on a dense [M][C] map (C a multiple of 8 bf16 / 4 f32):
 * the per-sample DropPath factor (swinir_arch.py:14-40) on a residual-branch gradient. */
int sr_row_scale(int dtype, const void* x, int64_t M, int C, int HW, const float* scale, void* out, void* stream);
/* Fused Adam (torch.optim.Adam semantics, no amsgrad/weight decay) + EMA of a flat fp32
 * parameter vector: g is scaled by grad_scale (DDP 1/world_size averaging), p, exp_avg,
 * exp_avg_sq updated in place; if ema != NULL, ema = ema*decay + p*(1-decay) after the step
 * (basicsr/models/base_model.py:75-82).  bc1/bc2 = 1 - beta^step. */
int sr_adam_ema(float* p, const float* g, float* m, float* v, float* ema, int64_t n, float lr,
                float beta1, float beta2, float eps, float bc1, float bc2, float ema_decay,
                float grad_scale, void* stream);
/* Graph-capturable form: hyper = device float[3] {step, lr, grad_scale}; the call first
 * increments hyper[0] on the device, then applies the update with bc = 1 - beta^step. */
int sr_adam_ema_dev(float* p, const float* g, float* m, float* v, float* ema, int64_t n, float* hyper,
                    float beta1, float beta2, float eps, float ema_decay, void* stream);

/* ---------------------------------------------------------------------------------
 * Block kernels of MSRResNet / RCAN / RRDBNet (csrc/blocks.hip).
 * ------------------------------------------------------------------------------------- */
/* y = base + bilinear_upsample(x, s) (align_corners=False), fp32 NCHW, x [N,C,H,W]
 * (MSRResNet skip, basicsr/archs/srresnet_arch.py:64-65). */
int sr_bilinear_up_add(const float* x, int N, int C, int H, int W, int s, const float* base, float* y,
                       void* stream);
/* out[n][c] = scale * sum_p a[n,p,c] (* b[n,p,c] if b) over the HW pixels of NHWC maps (channel
 * slices via ld/coff), deterministic; RCAN AdaptiveAvgPool2d(1) (rcan_arch.py:19) and its backward. */
size_t sr_channel_reduce_workspace(int N, int HW, int C);
int sr_channel_reduce(int dtype, const void* a, int lda, int acoff, const void* b, int ldb, int bcoff, int N,
                      int HW, int C, float scale, float* out, void* workspace, size_t ws_bytes, void* stream);
/* First pass of sr_channel_reduce only: parts[n][p][c] partial sums (dots) over pixel chunks,
 * P = sr_channel_partials_count(HW) chunks per image (the consumer sums them). */
int sr_channel_partials_count(int HW);
int sr_channel_partials(int dtype, const void* a, int lda, int acoff, const void* b, int ldb, int bcoff, int N,
                        int HW, int C, float* parts, void* stream);
/* RCAN squeeze MLP (the two 1x1 convs of rcan_arch.py:19-20): pool[n][c] = scale * sum_p
 * parts[n*P + p][c] (P = 1, scale = 1: parts is the pooled vector), h = relu(W1 pool + b1),
 * s = sigmoid(W2 h + b2); W1 [Cr][C], W2 [C][Cr]. */
int sr_ca_mlp_fwd(const float* parts, int P, float scale, const float* w1, const float* b1, const float* w2,
                  const float* b2, int N, int C, int Cr, float* pool, float* h, float* s, void* stream);
/* Its backward for the batch: ds[n][c] = scale * sum_p parts[n*P + p][c] = dL/ds -> dpool, dW1,
 * db1, dW2, db2 (db1/db2 may be NULL); accumulate = 1 adds the parameter gradients into
 * dw1/db1/dw2/db2 (the optimizer's gradient views) instead of storing them. */
int sr_ca_mlp_bwd(const float* parts, int P, float scale, const float* s, const float* h, const float* pool,
                  const float* w1, const float* w2, int N, int C, int Cr, float* dpool, float* dw1, float* db1,
                  float* dw2, float* db2, int accumulate, void* stream);
/* RCAB channel attention fused with its elementwise pass (rcan_arch.py:8-24, :44-46): every block
 * of the pass recomputes its image's squeeze MLP from the partial sums (fixed order, identical in
 * every block), so the MLP is not a dependent single-block launch.
 *   fwd: pool = scale*sum_p parts, h = relu(W1 pool + b1), s = sigmoid(W2 h + b2), y = x + alpha*u*s;
 *        pool / h / s are also stored (for the backward);
 *   bwd: ds = alpha*sum_p parts (parts of dy.u), dz2 = ds*s*(1-s), dz1 = relu'(h)*(W2^T dz2),
 *        du = alpha*dy*s + (W1^T dz1)/HW; dz2 [N][C] and dz1 [N][Cr] are stored for
 *   sr_ca_param_grad: dW2 = dz2^T h, dW1 = dz1^T pool, db2 = sum dz2, db1 = sum dz1 (accumulate = 1
 *        adds into the optimizer's gradient views; db1 / db2 may be NULL).
 * Dense NHWC [N, HW, C], C % 8 == 0, C <= 256, Cr <= 64; W1 [Cr][C], W2 [C][Cr]. */
int sr_ca_fwd_apply(int dtype, const float* parts, int P, float scale, const float* w1, const float* b1,
                    const float* w2, const float* b2, const void* x, const void* u, int N, int HW, int C, int Cr,
                    float alpha, void* y, float* pool, float* h, float* s, void* stream);
int sr_ca_bwd_apply(int dtype, const float* parts, int P, float alpha, const float* s, const float* h, const float* w1,
                    const float* w2, const void* dy, int N, int HW, int C, int Cr, void* du, float* dz2, float* dz1,
                    void* stream);
int sr_ca_param_grad(const float* dz2, const float* dz1, const float* h, const float* pool, int N, int C, int Cr,
                     float* dw1, float* db1, float* dw2, float* db2, int accumulate, void* stream);
/* out = beta*x + alpha*u*s[n,c] + gamma*t[n,c] on dense NHWC [N,HW,C] (x, t may be NULL):
 * RCAB tail x + rs*u*s and its backward rs*dout*s + dpool/HW. */
int sr_nc_affine(int dtype, const void* x, const void* u, const float* s, const float* t, int N, int HW, int C,
                 float beta, float alpha, float gamma, void* out, void* stream);
/* Strided activation backward over channel slices: out = alpha*dy*(y > 0 ? 1 : neg). */
int sr_act_backward_nhwc(int dtype, int64_t P, int C, const void* dy, int ldd, int dcoff, const void* y, int ldy,
                         int ycoff, void* out, int ldo, int ocoff, int act, float slope, float alpha,
                         void* stream);
/* Backward of nearest upsampling by s: out[n,y,x,c] (+)= sum of d over the s x s block
 * (rrdbnet_arch.py:116-117); out has H x W pixels, d has sH x sW. */
int sr_nearest_up_backward(int dtype, const void* d, int ldd, int N, int H, int W, int C, int s, void* out,
                           int ldo, int accumulate, void* stream);
/* The same times the activation derivative of the upsampled map (gate: its H x W LeakyReLU / ReLU output,
 * row stride ldg): out = sum * (gate > 0 ? 1 : slope) -- the conv_up1 / conv_up2 lrelu backward
 * (rrdbnet_arch.py:116-117) fused into the 2x2 sum; gate null = sr_nearest_up_backward. */
int sr_nearest_up_backward_gate(int dtype, const void* d, int ldd, int N, int H, int W, int C, int s,
                                const void* gate, int ldg, float slope, void* out, int ldo, int accumulate,
                                void* stream);
/* Strided channel-slice copy (RRDB dense-block buffers). */
int sr_copy_channels(int dtype, const void* src, int lds, int scoff, void* dst, int ldd, int dcoff, int64_t P,
                     int C, void* stream);

/* ---------------------------------------------------------------------------------
 * SwinIR token kernels (csrc/swin.hip).  Token maps are NHWC rows (= the reference's
 * [B, H*W, C] after PatchEmbed, swinir_arch.py:600-604).
 * ------------------------------------------------------------------------------------- */
/* nn.LayerNorm(C) over rows of [M][ld]: y = (x-mean)*rstd*gamma + beta (channels < C; columns
 * C..Cp-1 of y set to 0); saves per-row mean / rstd (fp32). */
int sr_layernorm_fwd(int dtype, const void* x, int ldx, const float* gamma, const float* beta, int64_t M,
                     int C, int Cp, float eps, void* y, int ldy, float* mean, float* rstd, void* stream);
size_t sr_layernorm_bwd_workspace(int64_t M, int C);
/* dx = LN backward (+ res if not NULL), dgamma / dbeta over all rows (deterministic);
 * accumulate bit 0 adds them to dgamma / dbeta (the optimizer's gradient views); bit 1 leaves
 * the dgamma / dbeta partial rows in the workspace for sr_layernorm_bwd_reduce (when
 * sr_layernorm_bwd_parts > 0), so that reduction can run on another stream. */
int sr_layernorm_bwd(int dtype, const void* dy, int lddy, const void* x, int ldx, const float* mean,
                     const float* rstd, const float* gamma, int64_t M, int C, int Cp, const void* res,
                     int ldr, void* dx, int lddx, float* dgamma, float* dbeta, void* workspace,
                     size_t ws_bytes, int accumulate, void* stream);
/* sr_layernorm_bwd that also writes dx_scaled[m] = dx[m] * row_scale[m / HW] (same layout as dx):
 * the SwinIR proj-branch gradient under stochastic depth (swinir_arch.py:14-40, 320) in the same
 * pass (bf16, Cp <= 256 path only). */
int sr_layernorm_bwd_scaled(int dtype, const void* dy, int lddy, const void* x, int ldx, const float* mean,
                            const float* rstd, const float* gamma, int64_t M, int C, int Cp, const void* res, int ldr,
                            void* dx, int lddx, float* dgamma, float* dbeta, void* workspace, size_t ws_bytes,
                            int accumulate, const float* row_scale, int HW, void* dx_scaled, void* stream);
int sr_layernorm_bwd_parts(int dtype, int64_t M, int Cp, int ldx, int lddx, int lddy, int ldr);
int sr_layernorm_bwd_reduce(const float* workspace, int nparts, int C, float* dgamma, float* dbeta, int accumulate,
                            void* stream);
/* Shifted-window multi-head attention on [N*H*W][ldq] qkv rows laid out [3][nH][hdp]
 * (head_dim hd <= hdp, zero padded): cyclic shift by `shift`, ws x ws windows, scale,
 * relative-position bias table [(2ws-1)^2][nH], -100 shift mask; out rows [nH][hdp];
 * lse = per-query log-sum-exp (for the backward).  ws <= 8, hd <= 32. */
int sr_window_attn_fwd(int dtype, const void* qkv, int ldq, int N, int H, int W, int ws, int shift, int nH,
                       int hd, int hdp, float scale, const float* bias_table, void* out, int ldo, float* lse,
                       void* stream);
/* Fused attention half of a SwinTransformerBlock (basicsr/archs/swinir_arch.py:283-314 with
 * WindowAttention :144-175; round 4): x2 = x + row_scale[n] * proj(WindowAttention(qkv(LN1(x)))) in
 * one launch on bf16 token maps [N][H][W][Cp] (Cp <= 192), window 8, nH heads of dim <= 32 padded
 * to 32 (nH * 32 <= 192), cyclic shift `shift`.  wqkv / wproj are the GEMM images of the qkv
 * (rows [3][nH][32], Cp columns) and proj (Cp rows, nH * 32 columns) linears with their fp32
 * biases; bias_table [(2*8-1)^2][nH]; row_scale [N] (DropPath) or NULL.  Training: qkv != NULL
 * and ln_out / ln_mean / ln_rstd / attn_out / lse receive what sr_linear_ln_fwd and
 * sr_window_attn_fwd write (the backward reads them unchanged); inference: all NULL, only x2 is
 * written.  sr_swin_attn_fused_ok: 1 when a geometry is on this path. */
int sr_swin_attn_fused_ok(int dtype, int N, int H, int W, int ws, int nH, int hd, int hdp, int C, int Cp);
int sr_swin_attn_fused_fwd(const void* x, const float* ln_g, const float* ln_b, int C, float eps, const void* wqkv,
                           const float* bqkv, const float* bias_table, const void* wproj, const float* bproj,
                           const float* row_scale, int N, int H, int W, int shift, int nH, int Cp, float scale, void* x2,
                           void* ln_out, float* ln_mean, float* ln_rstd, void* qkv, void* attn_out, float* lse,
                           void* stream);
/* Fused MLP half of a SwinTransformerBlock (swinir_arch.py:322-323, Mlp :43-60; round 4):
 * out = x + row_scale[n] * fc2(GELU(fc1(LN2(x)))) on bf16 token rows [N * HW][Cp] (Cp <= 192,
 * hidden Hp <= 368, multiples of 8): w1 / w2 the fc1 [Hp][Cp] / fc2 [Cp][Hp] GEMM images with fp32
 * biases.  Training: z != NULL, and ln_out / ln_mean / ln_rstd / z (pre-activation) / h
 * (activation) receive what sr_linear_ln_fwd writes for norm2 -> fc1 (the backward reads them);
 * inference: all NULL. */
int sr_swin_mlp_fused_ok(int dtype, int C, int Cp, int Hp);
int sr_swin_mlp_fused_fwd(const void* x, const float* ln_g, const float* ln_b, int C, float eps, const void* w1,
                          const float* b1, const void* w2, const float* b2, const float* row_scale, int N, int HW,
                          int Cp, int Hp, void* out, void* ln_out, float* ln_mean, float* ln_rstd, void* z, void* h,
                          void* stream);
size_t sr_window_attn_bwd_workspace(int N, int H, int W, int ws, int nH);
int sr_window_attn_bwd(int dtype, const void* qkv, int ldq, const void* out, const void* dout, int ldo,
                       const float* lse, int N, int H, int W, int ws, int shift, int nH, int hd, int hdp,
                       float scale, const float* bias_table, void* dqkv, float* dbias_table, void* workspace,
                       size_t ws_bytes, int accumulate, void* stream);
/* accumulate bit 1 of sr_window_attn_bwd: the relative-bias gradient partial rows (count:
 * sr_window_attn_bwd_parts) stay in the workspace for sr_window_attn_dbias_reduce.  A negative
 * count -P means P per-lane slot rows (the two-wave MFMA backward: 64 lanes x 28 pre-summed bins
 * per row, folded into the (2ws-1)^2 bins by the reduce); pass it through unchanged. */
int sr_window_attn_bwd_parts(int dtype, int N, int H, int W, int ws, int nH, int hd, int hdp, int ldq, int ldo);
int sr_window_attn_dbias_reduce(const float* workspace, int parts, int nH, int ws, float* dbias_table, int accumulate,
                                void* stream);

/* SwinIR absolute position embedding (ape=True, swinir_arch.py:789-791, :879-880) on dense token rows
 * [N][P][Cp]: y = x + pos[p][c] for c < C (pos fp32 [P][C]); its gradient dpos[p][c] (+)= sum_n dy. */
int sr_add_pos_embed(int dtype, const void* x, int N, int P, int C, int Cp, const float* pos, void* y, void* stream);
int sr_pos_embed_grad(int dtype, const void* dy, int N, int P, int C, int Cp, float* dpos, int accumulate,
                      void* stream);

/* ---------------------------------------------------------------------------------
 * basicsr/ops native extensions (replacements of deform_conv_ext, fused_act_ext,
 * upfirdn2d_ext).
 * ------------------------------------------------------------------------------------- */
/* Deformable convolution geometry (csrc/dcn.hip).  x is NHWC [N][H][W][Cp] (dtype);
 * offset [N][DG*2*kh*kw][Ho][Wo] and mask [N][DG*kh*kw][Ho][Wo] are the reference's NCHW
 * fp32 tensors (channel 2*tap = dy, 2*tap+1 = dx, per deformable group).  Columns are
 * pixel-major rows [N*Ho*Wo][groups][kh*kw][cgp] (cgp = padded C/groups), the operand of
 * the 1x1 GEMM (sr_conv3x3_fwd with ksize 1). */
typedef struct sr_dcn_desc {
  int dtype;
  int N, C, H, W, Cp, Ho, Wo;
  int kh, kw, stride_h, stride_w, pad_h, pad_w, dil_h, dil_w;
  int groups, deformable_groups, cgp;
} sr_dcn_desc;
/* columns = mask * bilinear(x, p + tap + offset); mask NULL = DCNv1 (all ones).
 * Replaces modulated_deformable_im2col_cuda / deformable_im2col
 * (deform_conv_cuda_kernel.cu:191-278, :571-634), batched over all images. */
int sr_dcn_im2col(const sr_dcn_desc* d, const void* x, const float* offset, const float* mask, void* cols,
                  void* stream);
/* Fused forward (bf16 only; groups 1, C = Cp = cgp = 64, Cout <= 64, cpg % 8 == 0 -- query with
 * sr_dcn_fwd_fused_ok): y[N][cout][Ho][Wo] fp32 = bf16(W x columns + bias), the columns gathered per
 * tap into LDS and never stored unless cols != NULL (then written as sr_dcn_im2col would, for the
 * backward's weight gradient).  x_blocked: x is [N][8][H][W][8] (channel vectors of 8 as planes; faster
 * gathers) instead of the NHWC [N][H][W][64] of the other entries.  wf: the GEMM weight image [wrows >= cout][ldw >= kh*kw*64] bf16, column
 * tap*64 + ci; bias fp32 [cout] or NULL.  Replaces modulated_deformable_im2col_cuda + the per-image
 * addmm of modulated_deform_conv_cuda_forward (deform_conv_cuda.cpp:560-590). */
int sr_dcn_fwd_fused_ok(const sr_dcn_desc* d, int cout);
int sr_dcn_fwd_fused(const sr_dcn_desc* d, const void* x, int x_blocked, const float* offset, const float* mask,
                     const void* wf, int ldw, int wrows, int cout, const float* bias, float* y, void* cols,
                     void* stream);
/* From dcols (= dy x W, column layout): grad_x += scatter (fp32 NHWC [N][H][W][Cp], caller
 * zeroes it; LDS fixed-point accumulation + fp32 atomics), grad_offset / grad_mask written in
 * full (grad_mask NULL for v1).  Workspace: sr_dcn_col2im_workspace bytes (per-image scale).
 * Replaces the col2im + col2im_coord pair (deform_conv_cuda_kernel.cu:280-466, :636-770). */
size_t sr_dcn_col2im_workspace(const sr_dcn_desc* d);
int sr_dcn_col2im(const sr_dcn_desc* d, const void* dcols, const void* x, const float* offset, const float* mask,
                  float* grad_x, float* grad_offset, float* grad_mask, void* workspace, size_t ws_bytes,
                  void* stream);
/* Fused backward without the column gradient matrix (bf16, groups 1, C = Cp = cgp = 64, cout_p <= 64, a
 * multiple of 8; query sr_dcn_bwd_fused_ok): from dy (bf16 NHWC [N][Ho][Wo][ldy], channels [0, cout_p))
 * and the transposed weight image wd (bf16 [K*64][ldw], row tap*64 + ci, column co -- the GEMM image the
 * dcols path multiplies dy by), each tap's dcols tile is formed on MFMA in registers and consumed at once:
 * grad_offset / grad_mask written in full; grad_x: grad_x_nchw = 0 -> += the bilinear scatter into fp32
 * NHWC [N][H][W][Cp] (caller zeroes it, as sr_dcn_col2im), 1 -> fp32 NCHW [N][C][H][W] written in full.
 * Same results as sr_dcn_col2im on dcols = bf16(dy x wd^T).  Workspace as sr_dcn_col2im.
 * Replaces the addmm into columns + col2im + col2im_coord of deform_conv_cuda.cpp:640-685. */
int sr_dcn_bwd_fused_ok(const sr_dcn_desc* d, int cout_p);
int sr_dcn_bwd_fused(const sr_dcn_desc* d, const void* dy, int ldy, const void* wd, int ldw, int cout_p, const void* x,
                     const float* offset, const float* mask, float* grad_x, int grad_x_nchw, float* grad_offset,
                     float* grad_mask, void* workspace, size_t ws_bytes, void* stream);

/* deform_conv_ext-compatible entries (basicsr/ops/dcn/src/deform_conv_ext.cpp:52-163; argument order
 * of :52-57, :70-76, :89-94, :107-113, :127-134): the reference's tensors in its order as fp32 NCHW
 * contiguous device pointers, then the sizes they carried (input N, C, H, W; Cout = weight.size(0)),
 * then the reference's integer arguments in its order, then a workspace of
 * sr_deform_conv_workspace(...) bytes (the same query serves all five; the modulated entries use
 * im2col_step = N) and the stream.  Buffer semantics as deform_conv_cuda.cpp: output written;
 * gradInput / grad_input += (the reference scatters into it atomically); gradOffset / grad_offset /
 * grad_mask written; gradWeight += scale * dW; grad_weight / grad_bias +=.  columns / ones are
 * accepted and ignored (the reference re-allocates columns itself, deform_conv_cuda.cpp:198, 303, 419,
 * 532, 610; the bias rides in the GEMM epilogue).  with_bias: 0 / 1. */
size_t sr_deform_conv_workspace(int N, int C, int H, int W, int Cout, int kW, int kH, int dW, int dH, int padW,
                                int padH, int dilationW, int dilationH, int group, int deformable_group,
                                int im2col_step);
int sr_deform_conv_forward(const float* input, const float* weight, const float* offset, float* output,
                           float* columns, float* ones, int N, int C, int H, int W, int Cout, int kW, int kH, int dW,
                           int dH, int padW, int padH, int dilationW, int dilationH, int group, int deformable_group,
                           int im2col_step, void* workspace, size_t ws_bytes, void* stream);
int sr_deform_conv_backward_input(const float* input, const float* offset, const float* gradOutput, float* gradInput,
                                  float* gradOffset, const float* weight, float* columns, int N, int C, int H, int W,
                                  int Cout, int kW, int kH, int dW, int dH, int padW, int padH, int dilationW,
                                  int dilationH, int group, int deformable_group, int im2col_step, void* workspace,
                                  size_t ws_bytes, void* stream);
int sr_deform_conv_backward_parameters(const float* input, const float* offset, const float* gradOutput,
                                       float* gradWeight, float* columns, float* ones, int N, int C, int H, int W,
                                       int Cout, int kW, int kH, int dW, int dH, int padW, int padH, int dilationW,
                                       int dilationH, int group, int deformable_group, float scale, int im2col_step,
                                       void* workspace, size_t ws_bytes, void* stream);
int sr_modulated_deform_conv_forward(const float* input, const float* weight, const float* bias, float* ones,
                                     const float* offset, const float* mask, float* output, float* columns, int N,
                                     int C, int H, int W, int Cout, int kernel_h, int kernel_w, int stride_h,
                                     int stride_w, int pad_h, int pad_w, int dilation_h, int dilation_w, int group,
                                     int deformable_group, int with_bias, void* workspace, size_t ws_bytes,
                                     void* stream);
int sr_modulated_deform_conv_backward(const float* input, const float* weight, const float* bias, float* ones,
                                      const float* offset, const float* mask, float* columns, float* grad_input,
                                      float* grad_weight, float* grad_bias, float* grad_offset, float* grad_mask,
                                      const float* grad_output, int N, int C, int H, int W, int Cout, int kernel_h,
                                      int kernel_w, int stride_h, int stride_w, int pad_h, int pad_w, int dilation_h,
                                      int dilation_w, int group, int deformable_group, int with_bias,
                                      void* workspace, size_t ws_bytes, void* stream);

/* fused_bias_act_op (basicsr/ops/fused_act/src/fused_bias_act_kernel.cu): out = scale *
 * act(x + bias[(i / step_b) % size_b]) with act 1 linear / 3 leaky-relu(alpha), grad 0/1/2
 * (grad 1 gates by ref > 0).  bias / ref may be NULL.  size_x < 2^31 (as the reference). */
int sr_fused_bias_act(int dtype, const void* x, const void* bias, const void* ref, void* out, int64_t size_x,
                      int step_b, int size_b, int act, int grad, float alpha, float scale, void* stream);
/* FusedLeakyReLUFunctionBackward.forward (fused_act.py:30-44) on [R][C][S]:
 * dx = dy * scale * (out > 0 ? 1 : alpha); grad_bias[c] = sum of dx over R, S (fp32,
 * deterministic; grad_bias may be NULL). */
size_t sr_fused_lrelu_bwd_workspace(int R, int C, int64_t S);
int sr_fused_lrelu_bwd(int dtype, const void* dy, const void* out, void* dx, float* grad_bias, int R, int C,
                       int64_t S, float alpha, float scale, void* workspace, size_t ws_bytes, void* stream);

/* upfirdn2d (basicsr/ops/upfirdn2d/upfirdn2d.py:97-192): planes [major][in_h][in_w], FIR
 * kernel fp32 [kh][kw]; out [major][out_h][out_w]. */
int sr_upfirdn2d_out_size(int in_h, int in_w, int kh, int kw, int up_x, int up_y, int down_x, int down_y,
                          int pad_x0, int pad_x1, int pad_y0, int pad_y1, int* out_h, int* out_w);
int sr_upfirdn2d(int dtype, const void* x, int major, int in_h, int in_w, const float* kernel, int kh, int kw,
                 int up_x, int up_y, int down_x, int down_y, int pad_x0, int pad_x1, int pad_y0, int pad_y1,
                 void* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif
