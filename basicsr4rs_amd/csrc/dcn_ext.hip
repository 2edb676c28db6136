// deform_conv_ext-compatible entry points (basicsr/ops/dcn/src/deform_conv_ext.cpp:52-163).
//
// The reference binds five functions over at::Tensor; these are their C-ABI forms: the same
// tensors in the same order as plain fp32 pointers (NCHW, contiguous), then the sizes the
// tensors carried (N, C, H, W of input, Cout = weight.size(0)), then the reference's own
// integer arguments in its order, then a caller-provided workspace and the stream.
//
// Buffer semantics follow deform_conv_cuda.cpp exactly:
//   forward            : output written                                           (:196-247, :530-568)
//   backward_input     : gradInput += col2im (the reference atomically adds into it),
//                        gradOffset written                                         (:343-350)
//   backward_parameters: gradWeight += scale * dW                                  (:460-466)
//   modulated_backward : grad_input +=, grad_weight +=, grad_bias +=, grad_offset and
//                        grad_mask written                                          (:623-672)
// ``columns`` and ``ones`` are accepted for binding compatibility and ignored: the reference
// re-allocates ``columns`` internally (at::zeros, :198, :303, :419, :532, :610) and never reads
// the caller's, and ``ones`` only feeds its bias GEMM, which here is an epilogue add.
//
// Execution is the batched HIP path of ops/dcn.py (whole im2col_step chunks per launch instead
// of the reference's per-image loop): NCHW -> NHWC, sr_dcn_im2col, one 1x1 MFMA GEMM per conv
// group (sr_conv3x3_fwd, ksize 1, bias in the epilogue), the split-K wgrad kernel for dW / db
// and sr_dcn_col2im for the input / offset / mask gradients.  fp32 (the reference's float path).
#include <string.h>

#include "sr_common.h"
#include "sr_internal.h"

namespace {

struct Geo {
  int N, C, H, W, Cout, kh, kw, sh, sw, ph, pw, dh, dw, G, DG;
  int Ho, Wo, K, cg, cgp, Cp, cout_g, cout_gp, L, ldy, step;
};

inline int pad8(int c) { return (c + 7) / 8 * 8; }

int make_geo(Geo& g, int N, int C, int H, int W, int Cout, int kh, int kw, int sh, int sw, int ph, int pw, int dh,
             int dw, int G, int DG, int step) {
  g = Geo{N, C, H, W, Cout, kh, kw, sh, sw, ph, pw, dh, dw, G, DG, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  if (N <= 0 || C <= 0 || H <= 0 || W <= 0 || Cout <= 0 || kh <= 0 || kw <= 0 || sh <= 0 || sw <= 0 || dh <= 0 ||
      dw <= 0 || ph < 0 || pw < 0 || G <= 0 || DG <= 0)
    return sr_fail(SR_EINVAL, "deform_conv: non-positive size / stride / dilation or negative padding");
  if (C % G || Cout % G) return sr_fail(SR_EINVAL, "deform_conv: channels not divisible by group");
  if (C % DG) return sr_fail(SR_EINVAL, "deform_conv: channels not divisible by deformable_group");
  g.Ho = (H + 2 * ph - (dh * (kh - 1) + 1)) / sh + 1;
  g.Wo = (W + 2 * pw - (dw * (kw - 1) + 1)) / sw + 1;
  if (g.Ho <= 0 || g.Wo <= 0) return sr_fail(SR_EINVAL, "deform_conv: output size is too small");
  g.K = kh * kw;
  g.cg = C / G;
  g.cgp = pad8(g.cg);
  g.Cp = pad8(C);
  g.cout_g = Cout / G;
  if (G > 1 && g.cout_g % 8) return sr_fail(SR_EINVAL, "deform_conv: grouped conv needs Cout / group % 8 == 0");
  g.cout_gp = pad8(g.cout_g);
  g.L = G * g.K * g.cgp;
  g.ldy = G * g.cout_gp;
  g.step = step > 0 && step < N ? step : N;
  if (N % g.step) return sr_fail(SR_EINVAL, "deform_conv: im2col step must divide batchsize");
  return SR_OK;
}

sr_dcn_desc dcn_desc(const Geo& g, int n) {
  sr_dcn_desc d{};
  d.dtype = SR_F32;
  d.N = n; d.C = g.C; d.H = g.H; d.W = g.W; d.Cp = g.Cp; d.Ho = g.Ho; d.Wo = g.Wo;
  d.kh = g.kh; d.kw = g.kw; d.stride_h = g.sh; d.stride_w = g.sw; d.pad_h = g.ph; d.pad_w = g.pw;
  d.dil_h = g.dh; d.dil_w = g.dw; d.groups = g.G; d.deformable_groups = g.DG; d.cgp = g.cgp;
  return d;
}

sr_conv3x3_desc gemm_desc(int n, int Ho, int Wo, int Cin, int ldx, int xcoff, int Cout, int ldy, int ycoff) {
  sr_conv3x3_desc d{};
  d.dtype = SR_F32;
  d.N = n; d.H = Ho; d.W = Wo;
  d.Cin = Cin; d.ldx = ldx; d.xcoff = xcoff;
  d.Cout = Cout; d.Cout_real = Cout; d.ldw = Cin;
  d.ldy = ldy; d.ycoff = ycoff;
  d.alpha = 1.f; d.beta = 1.f; d.beta2 = 1.f;
  d.ksize = 1;
  return d;
}

sr_conv3x3_wgrad_desc wgrad_desc(const Geo& g, int n, int gi, float scale) {
  sr_conv3x3_wgrad_desc d{};
  d.dtype = SR_F32;
  d.N = n; d.H = g.Ho; d.W = g.Wo;
  d.Cin = g.K * g.cgp; d.Cin_real = g.cg * g.K; d.ldx = g.L; d.xcoff = gi * g.K * g.cgp;
  d.Cout = g.cout_gp; d.Cout_real = g.cout_g; d.ldy = g.ldy; d.ycoff = gi * g.cout_gp;
  d.scale = scale;
  d.ksize = 1;
  d.accumulate = 1;
  return d;
}

// GEMM column k = tap * cgp + ci  <->  parameter column ci * K + tap of weight[co].flatten()
__global__ void dcn_maps_kernel(int K, int cg, int cgp, int* col_map, int* ci_map) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K * cgp) return;
  const int tap = k / cgp, ci = k - tap * cgp;
  col_map[k] = ci < cg ? ci * K + tap : -1;
  if (ci < cg) ci_map[ci * K + tap] = k;
}

// y[n][c][p] += x[n][p][c] (NHWC fp32 [n][P][ld] -> NCHW, first C channels)
__global__ void nhwc_to_nchw_add_kernel(const float* __restrict__ x, int ld, int C, int P, int64_t total,
                                        float* __restrict__ y) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = i / ((int64_t)C * P);
    const int64_t r = i - n * C * P;
    const int c = (int)(r / P), p = (int)(r - (int64_t)c * P);
    y[i] += x[(n * P + p) * ld + c];
  }
}

// Workspace carve-out (256-B aligned pieces).
struct Carver {
  char* base;
  size_t off = 0;
  explicit Carver(void* b) : base((char*)b) {}
  template <typename T> T* take(size_t count) {
    off = (off + 255) / 256 * 256;
    T* p = base ? (T*)(base + off) : nullptr;
    off += count * sizeof(T);
    return p;
  }
};

struct Bufs {
  int* col_map; int* ci_map;
  float *wf, *wd, *bg;                 // per-group GEMM images
  float *xh, *cols, *yh, *dcols, *gx;  // one chunk
  unsigned* cws;                       // col2im workspace
  float* wgws; size_t wgws_bytes;      // wgrad split-K slabs
};

Bufs carve(const Geo& g, void* ws, size_t* total = nullptr) {
  Carver c(ws);
  Bufs b{};
  const size_t kc = (size_t)g.K * g.cgp;
  const size_t rows = (size_t)g.step * g.Ho * g.Wo;
  b.col_map = c.take<int>(kc);
  b.ci_map = c.take<int>((size_t)g.cg * g.K);
  b.wf = c.take<float>((size_t)g.G * g.cout_gp * kc);
  b.wd = c.take<float>((size_t)g.G * kc * g.cout_gp);
  b.bg = c.take<float>((size_t)g.G * g.cout_gp);
  b.xh = c.take<float>((size_t)g.step * g.H * g.W * g.Cp);
  b.cols = c.take<float>(rows * g.L);
  b.yh = c.take<float>(rows * g.ldy);
  b.dcols = c.take<float>(rows * g.L);
  b.gx = c.take<float>((size_t)g.step * g.H * g.W * g.Cp);
  const sr_dcn_desc dd = dcn_desc(g, g.step);
  b.cws = c.take<unsigned>(sr_dcn_col2im_workspace(&dd) / sizeof(unsigned) + 1);
  const sr_conv3x3_wgrad_desc wd = wgrad_desc(g, g.step, 0, 1.f);
  b.wgws_bytes = sr_conv3x3_wgrad_workspace(&wd);
  b.wgws = c.take<float>(b.wgws_bytes / sizeof(float) + 1);
  b.wgws_bytes = (b.wgws_bytes / sizeof(float) + 1) * sizeof(float);
  if (total) *total = c.off + 256;
  return b;
}

size_t workspace_bytes(const Geo& g) {
  size_t total = 0;
  carve(g, nullptr, &total);
  return total;
}

#define SR_TRY(x)                   \
  do {                              \
    const int rc_ = (x);            \
    if (rc_ != SR_OK) return rc_;   \
  } while (0)

// GEMM images of every conv group (+ the column maps).
int prep(const Geo& g, const Bufs& b, const float* weight, const float* bias, hipStream_t s) {
  const int kc = g.K * g.cgp;
  hipLaunchKernelGGL(dcn_maps_kernel, dim3((kc + 255) / 256), dim3(256), 0, s, g.K, g.cg, g.cgp, b.col_map, b.ci_map);
  SR_TRY(sr_check(hipGetLastError(), "deform_conv maps launch"));
  for (int gi = 0; gi < g.G; ++gi)
    SR_TRY(sr_conv_prep_mapped(SR_F32, 1, weight + (size_t)gi * g.cout_g * g.cg * g.K,
                               bias ? bias + (size_t)gi * g.cout_g : nullptr, g.cout_g, g.cg * g.K, g.cout_gp, kc, 0,
                               nullptr, b.col_map, b.wf + (size_t)gi * g.cout_gp * kc, b.wd + (size_t)gi * kc * g.cout_gp,
                               b.bg + (size_t)gi * g.cout_gp, s));
  return SR_OK;
}

// cols of images [n0, n0 + step) (x -> NHWC, deformable im2col)
int chunk_cols(const Geo& g, const Bufs& b, int n0, const float* input, const float* offset, const float* mask,
               hipStream_t s) {
  const sr_dcn_desc d = dcn_desc(g, g.step);
  SR_TRY(sr_nchw_to_nhwc(SR_F32, input + (size_t)n0 * g.C * g.H * g.W, g.step, g.C, g.H, g.W, g.Cp, nullptr, nullptr,
                         b.xh, s));
  return sr_dcn_im2col(&d, b.xh, offset + (size_t)n0 * g.DG * 2 * g.K * g.Ho * g.Wo,
                       mask ? mask + (size_t)n0 * g.DG * g.K * g.Ho * g.Wo : nullptr, b.cols, s);
}

int run_forward(const Geo& g, const Bufs& b, const float* input, const float* offset, const float* mask,
                const float* bias, float* output, hipStream_t s) {
  const int kc = g.K * g.cgp;
  for (int n0 = 0; n0 < g.N; n0 += g.step) {
    SR_TRY(chunk_cols(g, b, n0, input, offset, mask, s));
    for (int gi = 0; gi < g.G; ++gi) {
      const sr_conv3x3_desc d = gemm_desc(g.step, g.Ho, g.Wo, kc, g.L, gi * kc, g.cout_gp, g.ldy, gi * g.cout_gp);
      SR_TRY(sr_conv3x3_fwd(&d, b.cols, b.wf + (size_t)gi * g.cout_gp * kc, bias ? b.bg + (size_t)gi * g.cout_gp : nullptr,
                            nullptr, nullptr, nullptr, nullptr, nullptr, b.yh, nullptr, nullptr, s));
    }
    SR_TRY(sr_nhwc_to_nchw(SR_F32, b.yh, g.step, g.Ho, g.Wo, g.ldy, 0, g.Cout, nullptr, nullptr,
                           output + (size_t)n0 * g.Cout * g.Ho * g.Wo, s));
  }
  return SR_OK;
}

// dy of a chunk as NHWC [step][Ho][Wo][ldy] in b.yh
int chunk_dy(const Geo& g, const Bufs& b, int n0, const float* grad_output, hipStream_t s) {
  return sr_nchw_to_nhwc(SR_F32, grad_output + (size_t)n0 * g.Cout * g.Ho * g.Wo, g.step, g.Cout, g.Ho, g.Wo, g.ldy,
                         nullptr, nullptr, b.yh, s);
}

// gradInput += / gradOffset (gradMask) = for the chunk whose dy is in b.yh and x in b.xh
int chunk_backward_data(const Geo& g, const Bufs& b, int n0, const float* offset, const float* mask,
                        float* grad_input, float* grad_offset, float* grad_mask, hipStream_t s) {
  const int kc = g.K * g.cgp;
  for (int gi = 0; gi < g.G; ++gi) {
    const sr_conv3x3_desc d = gemm_desc(g.step, g.Ho, g.Wo, g.cout_gp, g.ldy, gi * g.cout_gp, kc, g.L, gi * kc);
    SR_TRY(sr_conv3x3_fwd(&d, b.yh, b.wd + (size_t)gi * kc * g.cout_gp, nullptr, nullptr, nullptr, nullptr, nullptr,
                          nullptr, b.dcols, nullptr, nullptr, s));
  }
  const size_t gxn = (size_t)g.step * g.H * g.W * g.Cp;
  SR_TRY(sr_check(hipMemsetAsync(b.gx, 0, gxn * sizeof(float), s), "deform_conv memset"));
  const sr_dcn_desc dd = dcn_desc(g, g.step);
  const size_t offn = (size_t)n0 * g.DG * 2 * g.K * g.Ho * g.Wo, mskn = (size_t)n0 * g.DG * g.K * g.Ho * g.Wo;
  SR_TRY(sr_dcn_col2im(&dd, b.dcols, b.xh, offset + offn, mask ? mask + mskn : nullptr, b.gx, grad_offset + offn,
                       grad_mask ? grad_mask + mskn : nullptr, b.cws, sr_dcn_col2im_workspace(&dd), s));
  const int64_t total = (int64_t)g.step * g.C * g.H * g.W;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(nhwc_to_nchw_add_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const float*)b.gx, g.Cp, g.C,
                     g.H * g.W, total, grad_input + (size_t)n0 * g.C * g.H * g.W);
  return sr_check(hipGetLastError(), "deform_conv grad_input launch");
}

// grad_weight (+ grad_bias) += scale * (dy x cols^T) for the chunk (dy in b.yh, cols in b.cols)
int chunk_backward_params(const Geo& g, const Bufs& b, float* grad_weight, float* grad_bias, float scale,
                          hipStream_t s) {
  for (int gi = 0; gi < g.G; ++gi) {
    const sr_conv3x3_wgrad_desc d = wgrad_desc(g, g.step, gi, scale);
    SR_TRY(sr_conv3x3_wgrad(&d, b.yh, b.cols, b.wgws, b.wgws_bytes, grad_weight + (size_t)gi * g.cout_g * g.cg * g.K,
                            grad_bias ? grad_bias + (size_t)gi * g.cout_g : nullptr, nullptr, b.ci_map, s));
  }
  return SR_OK;
}

int check_ws(const Geo& g, void* ws, size_t ws_bytes) {
  if (!ws || ws_bytes < workspace_bytes(g)) return sr_fail(SR_EINVAL, "deform_conv: workspace too small");
  return SR_OK;
}

}  // namespace

extern "C" {

size_t sr_deform_conv_workspace(int N, int C, int H, int W, int Cout, int kW, int kH, int dW, int dH, int padW,
                                int padH, int dilationW, int dilationH, int group, int deformable_group,
                                int im2col_step) {
  Geo g;
  if (make_geo(g, N, C, H, W, Cout, kH, kW, dH, dW, padH, padW, dilationH, dilationW, group, deformable_group,
               im2col_step) != SR_OK)
    return 0;
  return workspace_bytes(g);
}

int sr_deform_conv_forward(const float* input, const float* weight, const float* offset, float* output,
                           float* columns, float* ones, int N, int C, int H, int W, int Cout, int kW, int kH, int dW,
                           int dH, int padW, int padH, int dilationW, int dilationH, int group, int deformable_group,
                           int im2col_step, void* workspace, size_t ws_bytes, void* stream) {
  (void)columns; (void)ones;
  if (!input || !weight || !offset || !output) return sr_fail(SR_EINVAL, "deform_conv_forward: null pointer");
  Geo g;
  SR_TRY(make_geo(g, N, C, H, W, Cout, kH, kW, dH, dW, padH, padW, dilationH, dilationW, group, deformable_group,
                  im2col_step));
  SR_TRY(check_ws(g, workspace, ws_bytes));
  hipStream_t s = (hipStream_t)stream;
  const Bufs b = carve(g, workspace);
  SR_TRY(prep(g, b, weight, nullptr, s));
  return run_forward(g, b, input, offset, nullptr, nullptr, output, s);
}

int sr_deform_conv_backward_input(const float* input, const float* offset, const float* gradOutput, float* gradInput,
                                  float* gradOffset, const float* weight, float* columns, int N, int C, int H, int W,
                                  int Cout, int kW, int kH, int dW, int dH, int padW, int padH, int dilationW,
                                  int dilationH, int group, int deformable_group, int im2col_step, void* workspace,
                                  size_t ws_bytes, void* stream) {
  (void)columns;
  if (!input || !offset || !gradOutput || !gradInput || !gradOffset || !weight)
    return sr_fail(SR_EINVAL, "deform_conv_backward_input: null pointer");
  Geo g;
  SR_TRY(make_geo(g, N, C, H, W, Cout, kH, kW, dH, dW, padH, padW, dilationH, dilationW, group, deformable_group,
                  im2col_step));
  SR_TRY(check_ws(g, workspace, ws_bytes));
  hipStream_t s = (hipStream_t)stream;
  const Bufs b = carve(g, workspace);
  SR_TRY(prep(g, b, weight, nullptr, s));
  for (int n0 = 0; n0 < g.N; n0 += g.step) {
    SR_TRY(sr_nchw_to_nhwc(SR_F32, input + (size_t)n0 * g.C * g.H * g.W, g.step, g.C, g.H, g.W, g.Cp, nullptr, nullptr,
                           b.xh, s));
    SR_TRY(chunk_dy(g, b, n0, gradOutput, s));
    SR_TRY(chunk_backward_data(g, b, n0, offset, nullptr, gradInput, gradOffset, nullptr, s));
  }
  return SR_OK;
}

int sr_deform_conv_backward_parameters(const float* input, const float* offset, const float* gradOutput,
                                       float* gradWeight, float* columns, float* ones, int N, int C, int H, int W,
                                       int Cout, int kW, int kH, int dW, int dH, int padW, int padH, int dilationW,
                                       int dilationH, int group, int deformable_group, float scale, int im2col_step,
                                       void* workspace, size_t ws_bytes, void* stream) {
  (void)columns; (void)ones;
  if (!input || !offset || !gradOutput || !gradWeight)
    return sr_fail(SR_EINVAL, "deform_conv_backward_parameters: null pointer");
  Geo g;
  SR_TRY(make_geo(g, N, C, H, W, Cout, kH, kW, dH, dW, padH, padW, dilationH, dilationW, group, deformable_group,
                  im2col_step));
  SR_TRY(check_ws(g, workspace, ws_bytes));
  hipStream_t s = (hipStream_t)stream;
  const Bufs b = carve(g, workspace);
  const int kc = g.K * g.cgp;
  hipLaunchKernelGGL(dcn_maps_kernel, dim3((kc + 255) / 256), dim3(256), 0, s, g.K, g.cg, g.cgp, b.col_map, b.ci_map);
  SR_TRY(sr_check(hipGetLastError(), "deform_conv maps launch"));
  for (int n0 = 0; n0 < g.N; n0 += g.step) {
    SR_TRY(chunk_cols(g, b, n0, input, offset, nullptr, s));
    SR_TRY(chunk_dy(g, b, n0, gradOutput, s));
    SR_TRY(chunk_backward_params(g, b, gradWeight, nullptr, scale, s));
  }
  return SR_OK;
}

int sr_modulated_deform_conv_forward(const float* input, const float* weight, const float* bias, float* ones,
                                     const float* offset, const float* mask, float* output, float* columns, int N,
                                     int C, int H, int W, int Cout, int kernel_h, int kernel_w, int stride_h,
                                     int stride_w, int pad_h, int pad_w, int dilation_h, int dilation_w, int group,
                                     int deformable_group, int with_bias, void* workspace, size_t ws_bytes,
                                     void* stream) {
  (void)ones; (void)columns;
  if (!input || !weight || !offset || !mask || !output || (with_bias && !bias))
    return sr_fail(SR_EINVAL, "modulated_deform_conv_forward: null pointer");
  Geo g;
  SR_TRY(make_geo(g, N, C, H, W, Cout, kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w, dilation_h, dilation_w,
                  group, deformable_group, N));
  SR_TRY(check_ws(g, workspace, ws_bytes));
  hipStream_t s = (hipStream_t)stream;
  const Bufs b = carve(g, workspace);
  SR_TRY(prep(g, b, weight, with_bias ? bias : nullptr, s));
  return run_forward(g, b, input, offset, mask, with_bias ? bias : nullptr, output, s);
}

int sr_modulated_deform_conv_backward(const float* input, const float* weight, const float* bias, float* ones,
                                      const float* offset, const float* mask, float* columns, float* grad_input,
                                      float* grad_weight, float* grad_bias, float* grad_offset, float* grad_mask,
                                      const float* grad_output, int N, int C, int H, int W, int Cout, int kernel_h,
                                      int kernel_w, int stride_h, int stride_w, int pad_h, int pad_w, int dilation_h,
                                      int dilation_w, int group, int deformable_group, int with_bias,
                                      void* workspace, size_t ws_bytes, void* stream) {
  (void)ones; (void)columns; (void)bias;
  if (!input || !weight || !offset || !mask || !grad_input || !grad_weight || !grad_offset || !grad_mask ||
      !grad_output || (with_bias && !grad_bias))
    return sr_fail(SR_EINVAL, "modulated_deform_conv_backward: null pointer");
  Geo g;
  SR_TRY(make_geo(g, N, C, H, W, Cout, kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w, dilation_h, dilation_w,
                  group, deformable_group, N));
  SR_TRY(check_ws(g, workspace, ws_bytes));
  hipStream_t s = (hipStream_t)stream;
  const Bufs b = carve(g, workspace);
  SR_TRY(prep(g, b, weight, nullptr, s));
  SR_TRY(chunk_cols(g, b, 0, input, offset, mask, s));
  SR_TRY(chunk_dy(g, b, 0, grad_output, s));
  SR_TRY(chunk_backward_data(g, b, 0, offset, mask, grad_input, grad_offset, grad_mask, s));
  return chunk_backward_params(g, b, grad_weight, with_bias ? grad_bias : nullptr, 1.f, s);
}

}  // extern "C"
