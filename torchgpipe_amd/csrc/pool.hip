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

// 32-bit index math throughout (the host caps tensors at 2 GiB): 64-bit division by the
// plane size would cost more than the nine loads.
__global__ __launch_bounds__(256) void avgpool3_fwd_kernel(const float* __restrict__ x,
                                                           const float* __restrict__ add,
                                                           float* __restrict__ y, int total,
                                                           int h, int w, int ho, int wo,
                                                           int stride) {
  const int plane_out = ho * wo;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int pl = i / plane_out;
    const int r = i - pl * plane_out;
    const int oy = r / wo, ox = r - oy * wo;
    const int cy = oy * stride, cx = ox * stride;
    const float* p = x + static_cast<int64_t>(pl) * h * w;
    float s = 0.f;
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy) {
      const int yy = cy + dy;
      if (yy < 0 || yy >= h) continue;
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx) {
        const int xx = cx + dx;
        if (xx >= 0 && xx < w) s += p[yy * w + xx];
      }
    }
    const int ny = min(cy + 1, h - 1) - max(cy - 1, 0) + 1;
    const int nx = min(cx + 1, w - 1) - max(cx - 1, 0) + 1;
    float v = s / static_cast<float>(ny * nx);
    if (add != nullptr) v += add[i];
    y[i] = v;
  }
}

__global__ __launch_bounds__(256) void avgpool3_bwd_kernel(const float* __restrict__ dy,
                                                           float* __restrict__ dx, int total,
                                                           int h, int w, int ho, int wo,
                                                           int stride) {
  const int plane_in = h * w;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int pl = i / plane_in;
    const int r = i - pl * plane_in;
    const int iy = r / w, ix = r - iy * w;
    // outputs whose window [c-1, c+1] (c = o * stride) contains the input pixel
    const int oy0 = max((iy - 1 + stride - 1) / stride, 0), oy1 = min((iy + 1) / stride, ho - 1);
    const int ox0 = max((ix - 1 + stride - 1) / stride, 0), ox1 = min((ix + 1) / stride, wo - 1);
    const float* g = dy + static_cast<int64_t>(pl) * ho * wo;
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

// Plane-in-LDS variants (planes up to kPlaneMax floats, i.e. every AmoebaNet pool): one
// workgroup per (image, channel) plane reads the plane once with coalesced loads into LDS,
// then every output gathers its <= 3x3 window from LDS and is stored coalesced.  The
// thread-per-output kernels above re-read each input 9 times through L1/L2 and divide per
// element (~20 us per AmoebaNet pool at 28^2 x 256 x 20 images).
// The LDS is dynamic, sized to the plane (28^2: 3 KiB), and the workgroup to the plane
// (64-256 threads), so small planes keep many workgroups per CU.
constexpr int kPlaneMax = 12544;  // 112 x 112 floats = 49 KiB of LDS

__global__ __launch_bounds__(256) void avgpool3_fwd_plane_kernel(const float* __restrict__ x,
                                                                 const float* __restrict__ add,
                                                                 float* __restrict__ y, int h,
                                                                 int w, int ho, int wo,
                                                                 int stride) {
  extern __shared__ float pl[];
  const int64_t plane = blockIdx.x;
  const int in = h * w, out = ho * wo, nt = blockDim.x;
  const float* src = x + plane * in;
  for (int i = threadIdx.x; i < in; i += nt) pl[i] = src[i];
  __syncthreads();
  float* dst = y + plane * out;
  const float* ad = add ? add + plane * out : nullptr;
  for (int o = threadIdx.x; o < out; o += nt) {
    const int oy = o / wo, ox = o - oy * wo;
    const int cy = oy * stride, cx = ox * stride;
    const int y0 = max(cy - 1, 0), y1 = min(cy + 1, h - 1);
    const int x0 = max(cx - 1, 0), x1 = min(cx + 1, w - 1);
    float sum = 0.f;
    for (int yy = y0; yy <= y1; ++yy)
      for (int xx = x0; xx <= x1; ++xx) sum += pl[yy * w + xx];
    float v = sum / static_cast<float>((y1 - y0 + 1) * (x1 - x0 + 1));
    if (ad) v += ad[o];
    dst[o] = v;
  }
}

__global__ __launch_bounds__(256) void avgpool3_bwd_plane_kernel(const float* __restrict__ dy,
                                                                 float* __restrict__ dx, int h,
                                                                 int w, int ho, int wo,
                                                                 int stride, int channels,
                                                                 int64_t dy_img) {
  extern __shared__ float pl[];  // dy / window area, per output
  const int64_t plane = blockIdx.x;
  const int in = h * w, out = ho * wo, nt = blockDim.x;
  // dy may be a channel slice of a wider gradient (image stride dy_img)
  const int64_t img = plane / channels;
  const float* g = dy + img * dy_img + (plane - img * channels) * out;
  for (int o = threadIdx.x; o < out; o += nt) {
    const int oy = o / wo, ox = o - oy * wo;
    const int cy = oy * stride, cx = ox * stride;
    const int ny = min(cy + 1, h - 1) - max(cy - 1, 0) + 1;
    const int nx = min(cx + 1, w - 1) - max(cx - 1, 0) + 1;
    pl[o] = g[o] / static_cast<float>(ny * nx);
  }
  __syncthreads();
  float* dst = dx + plane * in;
  for (int i = threadIdx.x; i < in; i += nt) {
    const int iy = i / w, ix = i - iy * w;
    const int oy0 = max((iy - 1 + stride - 1) / stride, 0), oy1 = min((iy + 1) / stride, ho - 1);
    const int ox0 = max((ix - 1 + stride - 1) / stride, 0), ox1 = min((ix + 1) / stride, wo - 1);
    float sum = 0.f;
    for (int oy = oy0; oy <= oy1; ++oy)
      for (int ox = ox0; ox <= ox1; ++ox) sum += pl[oy * wo + ox];
    dst[i] = sum;
  }
}

// Planes of <= 64 pixels (AmoebaNet's 7^2 cells): one workgroup per plane left each
// workgroup a single wave with one load, one LDS round trip and one store -- a latency chain
// of a few microseconds, 40 k of them per pool at 40 images x 1024 channels (31 us per
// pool, profiles/r4/rocprof/).  Here each wave takes kSmallPlanes planes, every lane issuing
// its pixel's loads of all of them before using any, and a workgroup holds 4 waves.
constexpr int kSmallPlanes = 4;

__global__ __launch_bounds__(256) void avgpool3_fwd_small_kernel(
    const float* __restrict__ x, const float* __restrict__ add, float* __restrict__ y,
    int64_t planes, int h, int w, int ho, int wo, int stride) {
  __shared__ float pl[4][kSmallPlanes][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int in = h * w, out = ho * wo;
  const int64_t p0 = (static_cast<int64_t>(blockIdx.x) * 4 + wave) * kSmallPlanes;
  float v[kSmallPlanes];
#pragma unroll
  for (int k = 0; k < kSmallPlanes; ++k)
    v[k] = lane < in && p0 + k < planes ? x[(p0 + k) * in + lane] : 0.f;
#pragma unroll
  for (int k = 0; k < kSmallPlanes; ++k) pl[wave][k][lane] = v[k];
  __syncthreads();
  if (lane >= out) return;
  const int oy = lane / wo, ox = lane - oy * wo;
  const int cy = oy * stride, cx = ox * stride;
  const int y0 = max(cy - 1, 0), y1 = min(cy + 1, h - 1);
  const int x0 = max(cx - 1, 0), x1 = min(cx + 1, w - 1);
  const float area = static_cast<float>((y1 - y0 + 1) * (x1 - x0 + 1));
  float a[kSmallPlanes];
#pragma unroll
  for (int k = 0; k < kSmallPlanes; ++k)
    a[k] = add && p0 + k < planes ? add[(p0 + k) * out + lane] : 0.f;
#pragma unroll
  for (int k = 0; k < kSmallPlanes; ++k) {
    if (p0 + k >= planes) break;
    float sum = 0.f;
    for (int yy = y0; yy <= y1; ++yy)
      for (int xx = x0; xx <= x1; ++xx) sum += pl[wave][k][yy * w + xx];
    y[(p0 + k) * out + lane] = sum / area + a[k];  // (the plane kernel's arithmetic)
  }
}

__global__ __launch_bounds__(256) void avgpool3_bwd_small_kernel(
    const float* __restrict__ dy, float* __restrict__ dx, int64_t planes, int h, int w, int ho,
    int wo, int stride, int channels, int64_t dy_img) {
  __shared__ float pl[4][kSmallPlanes][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int in = h * w, out = ho * wo;
  const int64_t p0 = (static_cast<int64_t>(blockIdx.x) * 4 + wave) * kSmallPlanes;
  float g[kSmallPlanes];
  float area = 1.f;
  if (lane < out) {
    const int oy = lane / wo, ox = lane - oy * wo;
    const int cy = oy * stride, cx = ox * stride;
    area = static_cast<float>((min(cy + 1, h - 1) - max(cy - 1, 0) + 1) *
                              (min(cx + 1, w - 1) - max(cx - 1, 0) + 1));
  }
#pragma unroll
  for (int k = 0; k < kSmallPlanes; ++k) {
    const int64_t plane = p0 + k;
    g[k] = 0.f;
    if (lane < out && plane < planes) {
      const int64_t img = plane / channels;
      g[k] = dy[img * dy_img + (plane - img * channels) * out + lane];
    }
  }
#pragma unroll
  for (int k = 0; k < kSmallPlanes; ++k) pl[wave][k][lane] = g[k] / area;
  __syncthreads();
  if (lane >= in) return;
  const int iy = lane / w, ix = lane - iy * w;
  const int oy0 = max((iy - 1 + stride - 1) / stride, 0), oy1 = min((iy + 1) / stride, ho - 1);
  const int ox0 = max((ix - 1 + stride - 1) / stride, 0), ox1 = min((ix + 1) / stride, wo - 1);
#pragma unroll
  for (int k = 0; k < kSmallPlanes; ++k) {
    if (p0 + k >= planes) break;
    float sum = 0.f;
    for (int oy = oy0; oy <= oy1; ++oy)
      for (int ox = ox0; ox <= ox1; ++ox) sum += pl[wave][k][oy * wo + ox];
    dx[(p0 + k) * in + lane] = sum;
  }
}

unsigned plane_threads(int64_t elems) {
  const int64_t t = (elems + 63) / 64 * 64;
  return static_cast<unsigned>(t < 256 ? t : 256);
}

unsigned blocks_for(int64_t work) {
  const int64_t b = (work + 255) / 256;
  return static_cast<unsigned>(b < 16384 ? (b > 0 ? b : 1) : 16384);
}

}  // namespace

void launch_avgpool3_forward(const float* x, const float* add, float* y, int64_t planes, int h,
                             int w, int stride, hipStream_t stream) {
  const int ho = (h - 1) / stride + 1, wo = (w - 1) / stride + 1;
  if (h * w <= 64 && planes < (int64_t{1} << 31)) {
    const int64_t per_block = 4 * kSmallPlanes;
    hipLaunchKernelGGL(avgpool3_fwd_small_kernel,
                       dim3(static_cast<unsigned>((planes + per_block - 1) / per_block)), dim3(256),
                       0, stream, x, add, y, planes, h, w, ho, wo, stride);
    return;
  }
  if (static_cast<int64_t>(h) * w <= kPlaneMax && planes < (int64_t{1} << 31)) {
    hipLaunchKernelGGL(avgpool3_fwd_plane_kernel, dim3(static_cast<unsigned>(planes)),
                       dim3(plane_threads(static_cast<int64_t>(h) * w)),
                       static_cast<unsigned>(h * w * 4), stream, x, add, y, h, w, ho, wo, stride);
    return;
  }
  const int64_t total = planes * ho * wo;  // < 2^31 (2 GiB tensors)
  hipLaunchKernelGGL(avgpool3_fwd_kernel, dim3(blocks_for(total)), dim3(256), 0, stream, x, add,
                     y, static_cast<int>(total), h, w, ho, wo, stride);
}

bool avgpool3_backward_strided_ok(int h, int w) {
  return static_cast<int64_t>(h) * w <= kPlaneMax;
}

void launch_avgpool3_backward(const float* dy, float* dx, int64_t images, int64_t channels,
                              int h, int w, int stride, int64_t dy_img, hipStream_t stream) {
  const int ho = (h - 1) / stride + 1, wo = (w - 1) / stride + 1;
  const int64_t planes = images * channels;
  if (dy_img <= 0) dy_img = channels * ho * wo;
  if (h * w <= 64 && planes < (int64_t{1} << 31)) {
    const int64_t per_block = 4 * kSmallPlanes;
    hipLaunchKernelGGL(avgpool3_bwd_small_kernel,
                       dim3(static_cast<unsigned>((planes + per_block - 1) / per_block)), dim3(256),
                       0, stream, dy, dx, planes, h, w, ho, wo, stride, static_cast<int>(channels),
                       dy_img);
    return;
  }
  if (avgpool3_backward_strided_ok(h, w) && planes < (int64_t{1} << 31)) {
    hipLaunchKernelGGL(avgpool3_bwd_plane_kernel, dim3(static_cast<unsigned>(planes)),
                       dim3(plane_threads(static_cast<int64_t>(h) * w)),
                       static_cast<unsigned>(ho * wo * 4), stream, dy, dx, h, w, ho, wo, stride,
                       static_cast<int>(channels), dy_img);
    return;
  }
  // (dense dy only: the caller makes it contiguous when this path runs)
  const int64_t total = planes * h * w;
  hipLaunchKernelGGL(avgpool3_bwd_kernel, dim3(blocks_for(total)), dim3(256), 0, stream, dy, dx,
                     static_cast<int>(total), h, w, ho, wo, stride);
}

}  // namespace tgpipe
