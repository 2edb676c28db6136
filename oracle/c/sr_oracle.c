/*
 * ORACLE (test infrastructure only) — plain-C restatement of the arithmetic the reference
 * SR nets get from PyTorch, used to pin oracle/nets.py independently of torch:
 *   conv3x3_nchw : nn.Conv2d(Cin, Cout, 3, 1, 1) cross-correlation with zero padding and bias
 *                  (instantiated at basicsr/archs/arch_util.py:78-79), double accumulation;
 *   pixel_shuffle: out[n, c, h*r+i, w*r+j] = in[n, c*r*r + i*r + j, h, w]
 *                  (nn.PixelShuffle, basicsr/archs/arch_util.py:136,139);
 *   pixel_unshuffle: basicsr/archs/arch_util.py:217-234.
 * Only tests/ may load this library (tests/test_oracle.py).
 */
#include <stdint.h>
#include <string.h>

void conv3x3_nchw(const float* x, const float* w, const float* b, float* y, int N, int Cin, int H, int W,
                  int Cout) {
  for (int n = 0; n < N; ++n)
    for (int co = 0; co < Cout; ++co)
      for (int oy = 0; oy < H; ++oy)
        for (int ox = 0; ox < W; ++ox) {
          double s = b ? b[co] : 0.0;
          for (int ci = 0; ci < Cin; ++ci)
            for (int ky = 0; ky < 3; ++ky) {
              const int iy = oy + ky - 1;
              if (iy < 0 || iy >= H) continue;
              for (int kx = 0; kx < 3; ++kx) {
                const int ix = ox + kx - 1;
                if (ix < 0 || ix >= W) continue;
                s += (double)x[(((int64_t)n * Cin + ci) * H + iy) * W + ix] *
                     (double)w[(((int64_t)co * Cin + ci) * 3 + ky) * 3 + kx];
              }
            }
          y[(((int64_t)n * Cout + co) * H + oy) * W + ox] = (float)s;
        }
}

void pixel_shuffle(const float* x, float* y, int N, int C, int H, int W, int r) {
  const int Co = C / (r * r);
  for (int n = 0; n < N; ++n)
    for (int c = 0; c < Co; ++c)
      for (int h = 0; h < H; ++h)
        for (int i = 0; i < r; ++i)
          for (int w = 0; w < W; ++w)
            for (int j = 0; j < r; ++j)
              y[(((int64_t)n * Co + c) * H * r + h * r + i) * W * r + w * r + j] =
                  x[(((int64_t)n * C + c * r * r + i * r + j) * H + h) * W + w];
}

void pixel_unshuffle(const float* x, float* y, int N, int C, int H, int W, int s) {
  const int Ho = H / s, Wo = W / s;
  for (int n = 0; n < N; ++n)
    for (int c = 0; c < C; ++c)
      for (int i = 0; i < s; ++i)
        for (int j = 0; j < s; ++j)
          for (int h = 0; h < Ho; ++h)
            for (int w = 0; w < Wo; ++w)
              y[(((int64_t)n * C * s * s + c * s * s + i * s + j) * Ho + h) * Wo + w] =
                  x[(((int64_t)n * C + c) * H + h * s + i) * W + w * s + j];
}
