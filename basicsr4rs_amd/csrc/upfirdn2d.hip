// upfirdn2d (StyleGAN2 resampling) for gfx950.
//
// Semantics of basicsr/ops/upfirdn2d/upfirdn2d.py:162-192 (upfirdn2d_native) and the
// reference CUDA op (src/upfirdn2d_kernel.cu): zero-insert upsample by `up`, pad by
// (pad0, pad1) (negative = crop), correlate with the flipped FIR kernel, keep every
// `down`-th sample.  Planes are [major][in_h][in_w] (minor = 1, as the Python wrapper
// reshapes NCHW).  The backward and double-backward of the reference are the same op with
// swapped up/down, flipped kernel and `g_pad` (upfirdn2d.py:121-126), so this one kernel
// serves all three.
//
// Polyphase form: output row oy reads up-space rows Y = oy*down - pad_y0 + t, t in
// [0, kh); only taps with Y = 0 mod up hit an input row (iy = Y / up), so the tap loop
// starts at the first matching phase and steps by `up`.  Each workgroup stages the input
// window of a 2-D output tile (and the kernel) in LDS once; HBM traffic is one read of the
// input and one write of the output (the op is HBM-bound: <= kh*kw/up^2 MACs per output).
// Taps are accumulated in ascending (row, column) order like the reference kernel.
#include "sr_common.h"
#include "sr_internal.h"

namespace {

SR_DEV int floordiv(int a, int b) {
  int q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
  return q;
}
static inline int floordiv_h(int a, int b) {
  int q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
  return q;
}

struct UfdArgs {
  int major, in_h, in_w, out_h, out_w;
  int kh, kw, up_x, up_y, down_x, down_y, px0, py0;
  int TW, TH, IW, IH;  // output tile, staged input window
  int tiles_x, tiles_y;
};

template <typename T>
__global__ void __launch_bounds__(256) upfirdn2d_kernel(UfdArgs a, const T* __restrict__ x,
                                                        const float* __restrict__ kern, T* __restrict__ out) {
  extern __shared__ float s_lds[];
  float* s_k = s_lds;                // [kh][kw]
  float* s_x = s_lds + a.kh * a.kw;  // [IH][IW]
  const int per_plane = a.tiles_x * a.tiles_y;
  const int plane = blockIdx.x / per_plane;
  const int t = blockIdx.x - plane * per_plane;
  const int ty = t / a.tiles_x, tx = t - ty * a.tiles_x;
  const int oy0 = ty * a.TH, ox0 = tx * a.TW;
  const int iy0 = floordiv(oy0 * a.down_y - a.py0, a.up_y);
  const int ix0 = floordiv(ox0 * a.down_x - a.px0, a.up_x);
  for (int i = threadIdx.x; i < a.kh * a.kw; i += blockDim.x) s_k[i] = kern[i];
  const T* xp = x + (int64_t)plane * a.in_h * a.in_w;
  for (int i = threadIdx.x; i < a.IH * a.IW; i += blockDim.x) {
    const int r = i / a.IW, c = i - r * a.IW;
    const int iy = iy0 + r, ix = ix0 + c;
    float v = 0.f;
    if (iy >= 0 && iy < a.in_h && ix >= 0 && ix < a.in_w) v = Elt<T>::to_f(xp[(int64_t)iy * a.in_w + ix]);
    s_x[i] = v;
  }
  __syncthreads();
  T* op = out + (int64_t)plane * a.out_h * a.out_w;
  const int lx = threadIdx.x % a.TW, ly0 = threadIdx.x / a.TW, rows_per_pass = blockDim.x / a.TW;
  const int ox = ox0 + lx;
  if (ox >= a.out_w) return;
  const int X0 = ox * a.down_x - a.px0;
  const int tx0 = ((-X0) % a.up_x + a.up_x) % a.up_x;
  for (int ly = ly0; ly < a.TH; ly += rows_per_pass) {
    const int oy = oy0 + ly;
    if (oy >= a.out_h) break;
    const int Y0 = oy * a.down_y - a.py0;
    const int ty0 = ((-Y0) % a.up_y + a.up_y) % a.up_y;
    float v = 0.f;
    for (int tyy = ty0; tyy < a.kh; tyy += a.up_y) {
      const int r = (Y0 + tyy) / a.up_y - iy0;
      const float* srow = s_x + r * a.IW;
      const float* krow = s_k + (a.kh - 1 - tyy) * a.kw;
      for (int txx = tx0; txx < a.kw; txx += a.up_x) {
        const int c = (X0 + txx) / a.up_x - ix0;
        v += srow[c] * krow[a.kw - 1 - txx];
      }
    }
    op[(int64_t)oy * a.out_w + ox] = Elt<T>::from_f(v);
  }
}

template <typename T>
int launch(UfdArgs a, const void* x, const float* k, void* out, hipStream_t s) {
  // output tile: TW a power of two covering the row (<= 64), 4 outputs per thread
  a.TW = 8;
  while (a.TW < 64 && a.TW < a.out_w) a.TW <<= 1;
  a.TH = 1024 / a.TW;
  size_t lds = 0;
  for (;;) {
    // up-space rows touched by the tile (exact division after the floor of the first)
    a.IH = floordiv_h((a.TH - 1) * a.down_y + a.kh - 1 + a.up_y - 1, a.up_y) + 2;
    a.IW = floordiv_h((a.TW - 1) * a.down_x + a.kw - 1 + a.up_x - 1, a.up_x) + 2;
    lds = ((size_t)a.kh * a.kw + (size_t)a.IH * a.IW) * sizeof(float);
    if (lds <= 65536 || (a.TH <= 4 && a.TW <= 8)) break;
    if (a.TH > 4) a.TH >>= 1;
    else a.TW >>= 1;
  }
  if (lds > 65536) return sr_fail(SR_ETOOBIG, "upfirdn2d: kernel / resampling factors too large for the LDS tile");
  a.tiles_x = (a.out_w + a.TW - 1) / a.TW;
  a.tiles_y = (a.out_h + a.TH - 1) / a.TH;
  const int64_t blocks = (int64_t)a.major * a.tiles_x * a.tiles_y;
  if (blocks >= ((int64_t)1 << 31)) return sr_fail(SR_ETOOBIG, "upfirdn2d: too many tiles");
  hipLaunchKernelGGL((upfirdn2d_kernel<T>), dim3((unsigned)blocks), dim3(256), lds, s, a, (const T*)x, k, (T*)out);
  return sr_check(hipGetLastError(), "upfirdn2d launch");
}

}  // namespace

extern "C" {

int sr_upfirdn2d_out_size(int in_h, int in_w, int kh, int kw, int up_x, int up_y, int down_x, int down_y,
                          int pad_x0, int pad_x1, int pad_y0, int pad_y1, int* out_h, int* out_w) {
  if (up_x <= 0 || up_y <= 0 || down_x <= 0 || down_y <= 0 || kh <= 0 || kw <= 0)
    return sr_fail(SR_EINVAL, "upfirdn2d: non-positive factor or kernel size");
  // upfirdn2d.py:108-109
  *out_h = floordiv_h(in_h * up_y + pad_y0 + pad_y1 - kh, down_y) + 1;
  *out_w = floordiv_h(in_w * up_x + pad_x0 + pad_x1 - kw, down_x) + 1;
  return SR_OK;
}

int sr_upfirdn2d(int dtype, const void* x, int major, int in_h, int in_w, const float* kernel, int kh, int kw,
                 int up_x, int up_y, int down_x, int down_y, int pad_x0, int pad_x1, int pad_y0, int pad_y1,
                 void* out, void* stream) {
  UfdArgs a;
  int rc = sr_upfirdn2d_out_size(in_h, in_w, kh, kw, up_x, up_y, down_x, down_y, pad_x0, pad_x1, pad_y0, pad_y1,
                                 &a.out_h, &a.out_w);
  if (rc) return rc;
  if (!x || !kernel || !out) return sr_fail(SR_EINVAL, "upfirdn2d: null pointer");
  if (major < 0 || in_h <= 0 || in_w <= 0 || a.out_h <= 0 || a.out_w <= 0)
    return sr_fail(SR_EINVAL, "upfirdn2d: empty input or output");
  if (major == 0) return SR_OK;
  a.major = major; a.in_h = in_h; a.in_w = in_w; a.kh = kh; a.kw = kw;
  a.up_x = up_x; a.up_y = up_y; a.down_x = down_x; a.down_y = down_y; a.px0 = pad_x0; a.py0 = pad_y0;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SR_F32) return launch<float>(a, x, kernel, out, s);
  if (dtype == SR_BF16) return launch<bf16_t>(a, x, kernel, out, s);
  return sr_fail(SR_EINVAL, "upfirdn2d: bad dtype");
}

}  // extern "C"
