// 3x3 average pooling of AmoebaNet-D cells (count_include_pad = False, padding 1, stride 1
// or 2), NCHW fp32, with the node sum (``pool(x) + other``) folded into the forward pass.
//
// The reference builds every pool of the genotype from nn.AvgPool2d (its max_pool_3x3 is an
// average pool too, operations.py:57-59); ATen's generic NCHW frame kernel runs one thread
// per output with integer divisions per tap.  Here one thread computes one output from a
// row-clipped 3x3 window: the divisor is the window's in-image area, the bounds are two
// min/max per axis, and the backward is the matching gather (each input pixel sums the
// gradients of the <= 3x3 outputs whose windows cover it, each divided by that window's
// area) -- no atomics, no zero fill.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace tgpipe {
namespace {

__global__ __launch_bounds__(256) void avgpool3_fwd_kernel(const float* __restrict__ x,
                                                           const float* __restrict__ add,
                                                           float* __restrict__ y, int64_t planes,
                                                           int h, int w, int ho, int wo,
                                                           int stride) {
  const int64_t total = planes * ho * wo;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t pl = i / (ho * wo);
    const int r = static_cast<int>(i - pl * ho * wo);
    const int oy = r / wo, ox = r - oy * wo;
    const int cy = oy * stride, cx = ox * stride;
    const int y0 = max(cy - 1, 0), y1 = min(cy + 1, h - 1);
    const int x0 = max(cx - 1, 0), x1 = min(cx + 1, w - 1);
    const float* p = x + pl * h * w;
    float s = 0.f;
    for (int yy = y0; yy <= y1; ++yy)
      for (int xx = x0; xx <= x1; ++xx) s += p[yy * w + xx];
    float v = s / static_cast<float>((y1 - y0 + 1) * (x1 - x0 + 1));
    if (add != nullptr) v += add[i];
    y[i] = v;
  }
}

__global__ __launch_bounds__(256) void avgpool3_bwd_kernel(const float* __restrict__ dy,
                                                           float* __restrict__ dx, int64_t planes,
                                                           int h, int w, int ho, int wo,
                                                           int stride) {
  const int64_t total = planes * h * w;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t pl = i / (h * w);
    const int r = static_cast<int>(i - pl * h * w);
    const int iy = r / w, ix = r - iy * w;
    // outputs whose window [c-1, c+1] (c = o * stride) contains the input pixel
    const int oy0 = max((iy - 1 + stride - 1) / stride, 0), oy1 = min((iy + 1) / stride, ho - 1);
    const int ox0 = max((ix - 1 + stride - 1) / stride, 0), ox1 = min((ix + 1) / stride, wo - 1);
    const float* g = dy + pl * ho * wo;
    float s = 0.f;
    for (int oy = oy0; oy <= oy1; ++oy) {
      const int cy = oy * stride;
      const int ny = min(cy + 1, h - 1) - max(cy - 1, 0) + 1;
      for (int ox = ox0; ox <= ox1; ++ox) {
        const int cx = ox * stride;
        const int nx = min(cx + 1, w - 1) - max(cx - 1, 0) + 1;
        s += g[oy * wo + ox] / static_cast<float>(ny * nx);
      }
    }
    dx[i] = s;
  }
}

unsigned blocks_for(int64_t work) {
  const int64_t b = (work + 255) / 256;
  return static_cast<unsigned>(b < 16384 ? (b > 0 ? b : 1) : 16384);
}

}  // namespace

void launch_avgpool3_forward(const float* x, const float* add, float* y, int64_t planes, int h,
                             int w, int stride, hipStream_t stream) {
  const int ho = (h - 1) / stride + 1, wo = (w - 1) / stride + 1;
  hipLaunchKernelGGL(avgpool3_fwd_kernel, dim3(blocks_for(planes * ho * wo)), dim3(256), 0,
                     stream, x, add, y, planes, h, w, ho, wo, stride);
}

void launch_avgpool3_backward(const float* dy, float* dx, int64_t planes, int h, int w,
                              int stride, hipStream_t stream) {
  const int ho = (h - 1) / stride + 1, wo = (w - 1) / stride + 1;
  hipLaunchKernelGGL(avgpool3_bwd_kernel, dim3(blocks_for(planes * h * w)), dim3(256), 0, stream,
                     dy, dx, planes, h, w, ho, wo, stride);
}

}  // namespace tgpipe
