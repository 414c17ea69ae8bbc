// U-Net's resolution changes as single passes (models/unet.py):
//
//   up2x_cat:    cat(nearest_upsample_2x(x), skip) along channels -- the decoder's 'up' +
//                'skip' layers (reference: nn.Upsample(scale_factor=2) then torch.cat); one
//                read of x and skip, one write of the concatenation, instead of writing the
//                upsampled tensor and copying it again.
//   up2x_bwd:    dx[n][c][y][x] = sum of the 2x2 block of dy's first C channels; dy may be
//                the channel slice of the concatenation's gradient (read in place).
//   maxpool2x2:  nn.MaxPool2d(2, stride=2) without the int64 index tensor (ATen writes one
//                per output: 3x the output traffic); the backward re-finds the argmax from
//                the input, which the U-Net keeps alive anyway (it is the stashed skip).
//                Ties and NaN follow ATen: the first maximum in row-major window order wins,
//                NaN wins over numbers (the last NaN of a window).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace tgpipe {
namespace {

typedef float floatx2 __attribute__((ext_vector_type(2)));

unsigned grid_for(int64_t work) {
  const int64_t b = (work + 255) / 256;
  return static_cast<unsigned>(b < 16384 ? (b > 0 ? b : 1) : 16384);
}

// One thread per pair of output columns (W even: the pair shares one upsampled source).
__global__ __launch_bounds__(256) void up2x_cat_kernel(const float* __restrict__ x,
                                                       const float* __restrict__ skip,
                                                       float* __restrict__ out, int64_t n,
                                                       int c1, int c2, int h, int w) {
  const int H = 2 * h, W = 2 * w, ct = c1 + c2;
  const int64_t pairs = n * ct * H * w;  // output element pairs
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < pairs;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t plane = i / (static_cast<int64_t>(H) * w);
    const int r = static_cast<int>(i - plane * H * w);
    const int oy = r / w, ox2 = r - oy * w;  // output row, column pair
    const int64_t img = plane / ct;
    const int ch = static_cast<int>(plane - img * ct);
    floatx2 v;
    if (ch < c1) {
      const float s = x[((img * c1 + ch) * h + (oy >> 1)) * w + ox2];
      v = floatx2{s, s};
    } else {
      v = *reinterpret_cast<const floatx2*>(
          skip + ((img * c2 + (ch - c1)) * H + oy) * static_cast<int64_t>(W) + 2 * ox2);
    }
    *reinterpret_cast<floatx2*>(out + (plane * H + oy) * static_cast<int64_t>(W) + 2 * ox2) = v;
  }
}

__global__ __launch_bounds__(256) void up2x_bwd_kernel(const float* __restrict__ dy,
                                                       float* __restrict__ dx, int64_t n, int c,
                                                       int h, int w, int64_t dy_img) {
  const int W = 2 * w;
  const int64_t total = n * c * h * w;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t plane = i / (static_cast<int64_t>(h) * w);
    const int r = static_cast<int>(i - plane * h * w);
    const int y = r / w, xx = r - y * w;
    const int64_t img = plane / c;
    const float* g = dy + img * dy_img + ((plane - img * c) * 2 * h + 2 * y) * W + 2 * xx;
    const floatx2 a = *reinterpret_cast<const floatx2*>(g);
    const floatx2 b = *reinterpret_cast<const floatx2*>(g + W);
    dx[i] = (a[0] + a[1]) + (b[0] + b[1]);
  }
}

// ATen's scan: start from -inf, a later element replaces the maximum when it is strictly
// larger or NaN (so the first of equal maxima and the last NaN win).
__device__ __forceinline__ int argmax4(float v0, float v1, float v2, float v3, float& m) {
  const float v[4] = {v0, v1, v2, v3};
  int k = 0;
  m = -INFINITY;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (v[j] > m || isnan(v[j])) {
      m = v[j];
      k = j;
    }
  }
  return k;
}

__global__ __launch_bounds__(256) void maxpool2x2_fwd_kernel(const float* __restrict__ x,
                                                             const float* __restrict__ add,
                                                             float* __restrict__ y,
                                                             int64_t planes, int h, int w) {
  const int ho = h / 2, wo = w / 2;
  const int64_t total = planes * ho * wo;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t plane = i / (static_cast<int64_t>(ho) * wo);
    const int r = static_cast<int>(i - plane * ho * wo);
    const int oy = r / wo, ox = r - oy * wo;
    const float* p = x + (plane * h + 2 * oy) * static_cast<int64_t>(w) + 2 * ox;
    float m;
    argmax4(p[0], p[1], p[w], p[w + 1], m);
    y[i] = add != nullptr ? m + add[i] : m;  // AmoebaNet's cell-node sum folded in
  }
}

// One thread per 2x2 input block: writes all four input gradients (zeros but the argmax),
// so every input element is written exactly once (odd trailing rows / columns, which no
// window covers, are zeroed by the caller's allocation).  dy may be a channel slice of a
// larger gradient (image stride dy_img, e.g. AmoebaNet's concatenated cell output).
__global__ __launch_bounds__(256) void maxpool2x2_bwd_kernel(const float* __restrict__ x,
                                                             const float* __restrict__ dy,
                                                             float* __restrict__ dx,
                                                             int64_t planes, int channels,
                                                             int h, int w, int64_t dy_img) {
  const int ho = h / 2, wo = w / 2;
  const int64_t total = planes * ho * wo;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t plane = i / (static_cast<int64_t>(ho) * wo);
    const int r = static_cast<int>(i - plane * ho * wo);
    const int oy = r / wo, ox = r - oy * wo;
    const int64_t base = (plane * h + 2 * oy) * static_cast<int64_t>(w) + 2 * ox;
    const float* p = x + base;
    float m;
    const int k = argmax4(p[0], p[1], p[w], p[w + 1], m);
    const int64_t img = plane / channels;
    const float g = dy[img * dy_img + (plane - img * channels) * ho * wo + r];
    float* q = dx + base;
    q[0] = k == 0 ? g : 0.f;
    q[1] = k == 1 ? g : 0.f;
    q[w] = k == 2 ? g : 0.f;
    q[w + 1] = k == 3 ? g : 0.f;
  }
}

typedef float floatx4 __attribute__((ext_vector_type(4)));

// ResNet's residual join: y = relu(x + identity), one pass (the sum and the ReLU were two
// ATen passes over the block output).
__global__ __launch_bounds__(256) void add_relu_kernel(const float* __restrict__ a,
                                                       const float* __restrict__ b,
                                                       float* __restrict__ y, int64_t quads,
                                                       int64_t total) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
  for (int64_t q = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; q < quads; q += stride) {
    const floatx4 v =
        reinterpret_cast<const floatx4*>(a)[q] + reinterpret_cast<const floatx4*>(b)[q];
    floatx4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = v[e] > 0.f ? v[e] : 0.f;
    reinterpret_cast<floatx4*>(y)[q] = o;
  }
  // tail (total % 4), by the first workgroup
  if (blockIdx.x == 0) {
    const int64_t i = quads * 4 + threadIdx.x;
    if (i < total) {
      const float v = a[i] + b[i];
      y[i] = v > 0.f ? v : 0.f;
    }
  }
}

}  // namespace

void launch_add_relu(const float* a, const float* b, float* y, int64_t total,
                     hipStream_t stream) {
  if (total == 0) return;
  const int64_t quads = total / 4;
  int64_t blocks = (quads + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 8192 ? 8192 : blocks);
  hipLaunchKernelGGL(add_relu_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, stream,
                     a, b, y, quads, total);
}

void launch_up2x_cat(const float* x, const float* skip, float* out, int64_t n, int c1, int c2,
                     int h, int w, hipStream_t stream) {
  const int64_t pairs = n * (c1 + c2) * 2 * static_cast<int64_t>(h) * w;
  if (pairs == 0) return;
  hipLaunchKernelGGL(up2x_cat_kernel, dim3(grid_for(pairs)), dim3(256), 0, stream, x, skip, out,
                     n, c1, c2, h, w);
}

void launch_up2x_backward(const float* dy, float* dx, int64_t n, int c, int h, int w,
                          int64_t dy_img, hipStream_t stream) {
  const int64_t total = n * c * static_cast<int64_t>(h) * w;
  if (total == 0) return;
  hipLaunchKernelGGL(up2x_bwd_kernel, dim3(grid_for(total)), dim3(256), 0, stream, dy, dx, n, c,
                     h, w, dy_img);
}

void launch_maxpool2x2_forward(const float* x, const float* add, float* y, int64_t planes, int h,
                               int w, hipStream_t stream) {
  const int64_t total = planes * (h / 2) * static_cast<int64_t>(w / 2);
  if (total == 0) return;
  hipLaunchKernelGGL(maxpool2x2_fwd_kernel, dim3(grid_for(total)), dim3(256), 0, stream, x, add,
                     y, planes, h, w);
}

void launch_maxpool2x2_backward(const float* x, const float* dy, float* dx, int64_t planes,
                                int channels, int h, int w, int64_t dy_img, hipStream_t stream) {
  const int64_t total = planes * (h / 2) * static_cast<int64_t>(w / 2);
  if (total == 0) return;
  hipLaunchKernelGGL(maxpool2x2_bwd_kernel, dim3(grid_for(total)), dim3(256), 0, stream, x, dy,
                     dx, planes, channels, h, w, dy_img);
}

}  // namespace tgpipe
