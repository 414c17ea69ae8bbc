// BatchNorm (training) kernels around the implicit-GEMM convolutions of conv_gemm.hip.
//
// The forward's statistics come from the convolution epilogue as per-(column block,
// channel) (mean, M2) partials; bn_finalize merges them with Chan's parallel formula in
// fp64 (no E[x^2] - E[x]^2 cancellation, whatever the mean), applies the running-stat
// EMA (unbiased variance, like nn.BatchNorm) and writes mean / invstd for bn_apply and
// the backward.  bn_apply normalises and optionally adds the other branch of an
// AmoebaNet node (left + right) in the same pass.  The backward is two passes: per
// channel sums of dy and dy*(z-mean), then dz and the affine gradients -- one launch of
// per-channel workgroups (bn_bwd_channel_kernel) when a channel is small enough.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>
#include <string>

#include "kernels.h"

namespace tgpipe {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

// Chan's parallel merge of (count, mean, M2) triples.
__device__ __forceinline__ void chan_merge(double& na, double& ma, double& m2a, double nb,
                                           double mb, double m2b) {
  const double n = na + nb;
  if (n <= 0.0) return;
  const double d = mb - ma;
  ma += d * nb / n;
  m2a += m2b + d * d * na * nb / n;
  na = n;
}

// 32 lanes per channel merge strided subsets of the column-block partials, then a
// 5-level shuffle tree merges the lanes: ~blocks/32 + 5 dependent fp64 steps instead
// of `blocks` (AmoebaNet's 56^2 planes at 20 images: 980 blocks).
__global__ __launch_bounds__(256) void bn_finalize_kernel(
    const float* __restrict__ pm, const float* __restrict__ pm2, int blocks, int width,
    int64_t total, int64_t c, float eps, double momentum, float* __restrict__ mean,
    float* __restrict__ invstd, float* __restrict__ rm, float* __restrict__ rv,
    int64_t* __restrict__ tracked, double* __restrict__ acc, float* __restrict__ zero2c) {
  const int lane = threadIdx.x & 31;
  const int64_t ch = static_cast<int64_t>(blockIdx.x) * 8 + (threadIdx.x >> 5);
  if (tracked != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *tracked += 1;
  double na = 0.0, ma = 0.0, m2a = 0.0;
  if (ch < c) {
    for (int b = lane; b < blocks; b += 32) {
      const int64_t left = total - static_cast<int64_t>(b) * width;
      chan_merge(na, ma, m2a, static_cast<double>(left < width ? left : width), pm[b * c + ch],
                 pm2[b * c + ch]);
    }
  }
#pragma unroll
  for (int off = 16; off > 0; off >>= 1) {
    const double nb = __shfl_xor(na, off, 32);
    const double mb = __shfl_xor(ma, off, 32);
    const double m2b = __shfl_xor(m2a, off, 32);
    chan_merge(na, ma, m2a, nb, mb, m2b);
  }
  if (ch >= c || lane != 0) return;
  if (zero2c != nullptr) {  // the backward's [2][C] reduction buffer, zeroed here for free
    zero2c[ch] = 0.f;
    zero2c[c + ch] = 0.f;
  }
  const double var = na > 0.0 ? m2a / na : 0.0;
  mean[ch] = static_cast<float>(ma);
  invstd[ch] = static_cast<float>(1.0 / sqrt(var + static_cast<double>(eps)));
  if (acc != nullptr) {
    // DeferredBatchNorm: fold this micro-batch into the mini-batch accumulators
    // (count, mean, M2) -- committed once per mini-batch by dbn_commit64
    double n0 = acc[ch], m0 = acc[c + ch], q0 = acc[2 * c + ch];
    chan_merge(n0, m0, q0, na, ma, m2a);
    acc[ch] = n0;
    acc[c + ch] = m0;
    acc[2 * c + ch] = q0;
  }
  if (rm != nullptr) {
    const double unbiased = na > 1.0 ? m2a / (na - 1.0) : var;
    rm[ch] = static_cast<float>((1.0 - momentum) * rm[ch] + momentum * ma);
    rv[ch] = static_cast<float>((1.0 - momentum) * rv[ch] + momentum * unbiased);
  }
}

// Finalize + apply in one launch.  Workgroup (channel, image range): its 256 threads
// merge the channel's partials (thread-strided Chan merges, a 64-lane shuffle tree, then
// the 4 waves through LDS -- the same fixed order in every workgroup of the channel, so
// all of them hold bit-identical statistics), workgroup (channel, 0) publishes mean /
// invstd / running statistics, and every workgroup normalises its own images.  Saves the
// separate finalize launch per BatchNorm (AmoebaNet: ~17 k launches per training step).
template <bool kVec, bool kAdd, bool kRelu>
__global__ __launch_bounds__(256) void bn_finalize_apply_kernel(
    const float* __restrict__ pm, const float* __restrict__ pm2, int blocks, int width,
    int cols, int n, int c, int s, int n_per, float eps, double momentum,
    float* __restrict__ mean, float* __restrict__ invstd, float* __restrict__ rm,
    float* __restrict__ rv, int64_t* __restrict__ tracked, double* __restrict__ acc,
    float* __restrict__ zero2c, const float* __restrict__ z, const float* __restrict__ gamma,
    const float* __restrict__ beta, const float* __restrict__ add, float* __restrict__ y,
    BnParts parts) {
  const int ch = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // output channel ch of the statistics / z; with parts (a grouped convolution feeding
  // several BatchNorms) its parameters, running statistics and output come from its part
  int yc = c, ych = ch;
  if (parts.count > 0) {
    int pi = 0;
    while (pi + 1 < parts.count && ch >= parts.c_end[pi]) ++pi;
    const int begin = pi == 0 ? 0 : parts.c_end[pi - 1];
    yc = parts.c_end[pi] - begin;
    ych = ch - begin;
    gamma = parts.gamma[pi] ? parts.gamma[pi] - begin : nullptr;
    beta = parts.beta[pi] ? parts.beta[pi] - begin : nullptr;
    rm = parts.rm[pi] ? parts.rm[pi] - begin : nullptr;
    rv = parts.rv[pi] ? parts.rv[pi] - begin : nullptr;
    tracked = ych == 0 ? parts.tracked[pi] : nullptr;
    y = parts.y[pi];
  }
  double na = 0.0, ma = 0.0, m2a = 0.0;
  for (int b = tid; b < blocks; b += 256) {
    const int left = cols - b * width;
    chan_merge(na, ma, m2a, static_cast<double>(left < width ? left : width), pm[b * c + ch],
               pm2[b * c + ch]);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double nb = __shfl_xor(na, off);
    const double mb = __shfl_xor(ma, off);
    const double m2b = __shfl_xor(m2a, off);
    chan_merge(na, ma, m2a, nb, mb, m2b);
  }
  __shared__ double red[3][4];
  __shared__ float kb[3];
  if (lane == 0) {
    red[0][wave] = na;
    red[1][wave] = ma;
    red[2][wave] = m2a;
  }
  __syncthreads();
  if (tid == 0) {
    na = red[0][0];
    ma = red[1][0];
    m2a = red[2][0];
    for (int k = 1; k < 4; ++k) chan_merge(na, ma, m2a, red[0][k], red[1][k], red[2][k]);
    const double var = na > 0.0 ? m2a / na : 0.0;
    const float mu = static_cast<float>(ma);
    const float is = static_cast<float>(1.0 / sqrt(var + static_cast<double>(eps)));
    kb[0] = mu;
    kb[1] = is * (gamma ? gamma[ch] : 1.f);
    kb[2] = beta ? beta[ch] : 0.f;
    if (blockIdx.y == 0) {
      if (tracked != nullptr && (ch == 0 || parts.count > 0)) *tracked += 1;
      if (zero2c != nullptr) {  // the backward's [2][C] reduction buffer
        zero2c[ch] = 0.f;
        zero2c[c + ch] = 0.f;
      }
      mean[ch] = mu;
      invstd[ch] = is;
      if (acc != nullptr) {  // DeferredBatchNorm mini-batch accumulators (dbn_commit64)
        double n0 = acc[ch], m0 = acc[c + ch], q0 = acc[2 * c + ch];
        chan_merge(n0, m0, q0, na, ma, m2a);
        acc[ch] = n0;
        acc[c + ch] = m0;
        acc[2 * c + ch] = q0;
      }
      if (rm != nullptr) {
        const double unbiased = na > 1.0 ? m2a / (na - 1.0) : var;
        rm[ch] = static_cast<float>((1.0 - momentum) * rm[ch] + momentum * ma);
        rv[ch] = static_cast<float>((1.0 - momentum) * rv[ch] + momentum * unbiased);
      }
    }
  }
  __syncthreads();
  const float mu = kb[0], k = kb[1], bb = kb[2];
  const int n0 = blockIdx.y * n_per, n1 = min(n, n0 + n_per);
  if constexpr (kVec) {
    // two quads per thread per round, both loads issued before either is used: one
    // 16-byte load in flight per wave left the pass short of HBM bandwidth
    const int sq = s >> 2, quads = (n1 - n0) * sq;
    for (int q0 = tid; q0 < quads; q0 += 2 * 256) {
      int64_t zo[2], yo[2];
      floatx4 zv[2], av[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int q = q0 + u * 256;
        const int img = n0 + q / sq, p = q - (img - n0) * sq;
        zo[u] = (static_cast<int64_t>(img) * c + ch) * sq + p;
        yo[u] = (static_cast<int64_t>(img) * yc + ych) * sq + p;
        if (q < quads) {
          zv[u] = reinterpret_cast<const floatx4*>(z)[zo[u]];
          if constexpr (kAdd) av[u] = reinterpret_cast<const floatx4*>(add)[zo[u]];
        }
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (q0 + u * 256 >= quads) break;
        // (z - mean) * k, not z * k - mean * k: no cancellation when |mean| >> std; one
        // fma, the same rounding the backward's ReLU mask recomputes (bn_relu_mask)
        floatx4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = __builtin_fmaf(zv[u][e] - mu, k, bb);
        if constexpr (kAdd) v += av[u];
        if constexpr (kRelu) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
        }
        reinterpret_cast<floatx4*>(y)[yo[u]] = v;
      }
    }
  } else {
    // planes of s % 4 != 0 pixels (7^2, 14^2): four elements per thread per round, loads
    // first -- one element per round left one load latency per element exposed
    const int elems = (n1 - n0) * s;
    for (int e0 = tid; e0 < elems; e0 += 4 * 256) {
      int64_t zo[4], yo[4];
      float zv[4], av[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + u * 256;
        const int img = n0 + e / s, p = e - (img - n0) * s;
        zo[u] = (static_cast<int64_t>(img) * c + ch) * s + p;
        yo[u] = (static_cast<int64_t>(img) * yc + ych) * s + p;
        zv[u] = e < elems ? z[zo[u]] : 0.f;
        if constexpr (kAdd) av[u] = e < elems ? add[zo[u]] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (e0 + u * 256 >= elems) break;
        float v = __builtin_fmaf(zv[u] - mu, k, bb);
        if constexpr (kAdd) v += av[u];
        if constexpr (kRelu) v = v > 0.f ? v : 0.f;
        y[yo[u]] = v;
      }
    }
  }
}

// A split-K forward of a small-plane convolution (s <= 64 pixels) and its BatchNorm, after
// the GEMM left its split partials in `ws` ([split][n][c][s]): one workgroup per channel
// sums the partials of every image (z, kept for the backward), takes the channel's
// statistics in fp64 over the values it holds (two passes, mean then M2: no partials to
// merge, no cancellation), finalizes (as bn_finalize_apply: running statistics, counter,
// DeferredBatchNorm accumulators, the backward's zeroed sums) and normalises -- one launch
// instead of split_reduce_stats + bn_finalize_apply, and z read back from registers.
constexpr int kSplitBnPer = 16;  // values per thread: n * s <= 16 * 256

template <bool kAdd, bool kRelu>
__global__ __launch_bounds__(256) void split_bn_small_kernel(
    const float* __restrict__ ws, int splits, int64_t stride, float* __restrict__ z, int n,
    int c, int s, float eps, double momentum, float* __restrict__ mean,
    float* __restrict__ invstd, float* __restrict__ rm, float* __restrict__ rv,
    int64_t* __restrict__ tracked, double* __restrict__ acc, float* __restrict__ zero2c,
    const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ add, float* __restrict__ y, BnParts parts) {
  const int ch = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int yc = c, ych = ch;
  if (parts.count > 0) {  // (as bn_finalize_apply_kernel)
    int pi = 0;
    while (pi + 1 < parts.count && ch >= parts.c_end[pi]) ++pi;
    const int begin = pi == 0 ? 0 : parts.c_end[pi - 1];
    yc = parts.c_end[pi] - begin;
    ych = ch - begin;
    gamma = parts.gamma[pi] ? parts.gamma[pi] - begin : nullptr;
    beta = parts.beta[pi] ? parts.beta[pi] - begin : nullptr;
    rm = parts.rm[pi] ? parts.rm[pi] - begin : nullptr;
    rv = parts.rv[pi] ? parts.rv[pi] - begin : nullptr;
    tracked = ych == 0 ? parts.tracked[pi] : nullptr;
    y = parts.y[pi];
  }
  const int total = n * s;
  float v[kSplitBnPer];
  double sum = 0.0;
#pragma unroll
  for (int r = 0; r < kSplitBnPer; ++r) {
    const int e = tid + 256 * r;
    v[r] = 0.f;
    if (e < total) {
      const int img = e / s, p = e - img * s;
      const int64_t o = (static_cast<int64_t>(img) * c + ch) * s + p;
      float a = 0.f, b = 0.f;
      int k = 0;
      for (; k + 1 < splits; k += 2) {
        a += ws[k * stride + o];
        b += ws[(k + 1) * stride + o];
      }
      if (k < splits) a += ws[k * stride + o];
      v[r] = a + b;
      z[o] = v[r];
      sum += static_cast<double>(v[r]);
    }
  }
  __shared__ double red[4];
  __shared__ float kb[3];
  auto block_sum = [&](double t) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
    __syncthreads();  // (red reused by the second pass)
    if (lane == 0) red[wave] = t;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
  };
  const double na = static_cast<double>(total);
  const double ma = block_sum(sum) / na;
  double sq = 0.0;
#pragma unroll
  for (int r = 0; r < kSplitBnPer; ++r) {
    if (tid + 256 * r < total) {
      const double d = static_cast<double>(v[r]) - ma;
      sq += d * d;
    }
  }
  const double m2a = block_sum(sq);
  if (tid == 0) {
    const double var = m2a / na;
    const float mu = static_cast<float>(ma);
    const float is = static_cast<float>(1.0 / sqrt(var + static_cast<double>(eps)));
    kb[0] = mu;
    kb[1] = is * (gamma ? gamma[ch] : 1.f);  // (part pointers shifted by its first channel)
    kb[2] = beta ? beta[ch] : 0.f;
    if (tracked != nullptr && (ch == 0 || parts.count > 0)) *tracked += 1;
    if (zero2c != nullptr) {
      zero2c[ch] = 0.f;
      zero2c[c + ch] = 0.f;
    }
    mean[ch] = mu;
    invstd[ch] = is;
    if (acc != nullptr) {
      double n0 = acc[ch], m0 = acc[c + ch], q0 = acc[2 * c + ch];
      chan_merge(n0, m0, q0, na, ma, m2a);
      acc[ch] = n0;
      acc[c + ch] = m0;
      acc[2 * c + ch] = q0;
    }
    if (rm != nullptr) {
      const double unbiased = na > 1.0 ? m2a / (na - 1.0) : var;
      rm[ch] = static_cast<float>((1.0 - momentum) * rm[ch] + momentum * ma);
      rv[ch] = static_cast<float>((1.0 - momentum) * rv[ch] + momentum * unbiased);
    }
  }
  __syncthreads();
  const float mu = kb[0], k = kb[1], bb = kb[2];
#pragma unroll
  for (int r = 0; r < kSplitBnPer; ++r) {
    const int e = tid + 256 * r;
    if (e >= total) break;
    const int img = e / s, p = e - img * s;
    float o = __builtin_fmaf(v[r] - mu, k, bb);  // (bn_finalize_apply's rounding)
    if constexpr (kAdd) o += add[(static_cast<int64_t>(img) * c + ch) * s + p];
    if constexpr (kRelu) o = o > 0.f ? o : 0.f;
    y[(static_cast<int64_t>(img) * yc + ych) * s + p] = o;
  }
}

// The ReLU after a BatchNorm (relu_out), re-derived in the backward from the saved
// convolution output: the forward's normalised value > 0, computed with the same fma.
__device__ __forceinline__ bool bn_relu_mask(float z, float mu, float k, float b) {
  return __builtin_fmaf(z - mu, k, b) > 0.f;
}

template <bool kVec, bool kAdd>
__global__ __launch_bounds__(256) void bn_apply_kernel(
    const float* __restrict__ z, const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ gamma, const float* __restrict__ beta, const float* __restrict__ add,
    float* __restrict__ y, int64_t total, int64_t c, int64_t s) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
  if constexpr (kVec) {
    // s % 4 == 0: a quad never straddles two channels
    for (int64_t q = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; q < total / 4;
         q += stride) {
      const int64_t ch = (4 * q / s) % c;
      const float k = invstd[ch] * (gamma ? gamma[ch] : 1.f);
      const float b = beta ? beta[ch] : 0.f;
      const float mu = mean[ch];
      // (z - mean) * k, not z * k - mean * k: no cancellation when |mean| >> std
      floatx4 v = (reinterpret_cast<const floatx4*>(z)[q] - mu) * k + b;
      if constexpr (kAdd) v += reinterpret_cast<const floatx4*>(add)[q];
      reinterpret_cast<floatx4*>(y)[q] = v;
    }
  } else {
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < total;
         i += stride) {
      const int64_t ch = (i / s) % c;
      const float k = invstd[ch] * (gamma ? gamma[ch] : 1.f);
      float v = (z[i] - mean[ch]) * k + (beta ? beta[ch] : 0.f);
      if constexpr (kAdd) v += add[i];
      y[i] = v;
    }
  }
}

// One workgroup per (channel, image range): sums of dy and dy * (z - mean).
// dy may be a channel slice of a wider tensor (the gradient of a concatenated cell
// output): image `img` of dy starts at dy + img * dy_img (z and dz are dense).
// relu_out: dy is the gradient of relu(bn(z)); the ReLU's mask is re-derived from z.
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(
    const float* __restrict__ dy, const float* __restrict__ z, const float* __restrict__ mean,
    float* __restrict__ sums, int64_t n, int64_t c, int64_t s, int64_t n_per, int64_t dy_img,
    int relu_out, const float* __restrict__ invstd, const float* __restrict__ gamma,
    const float* __restrict__ beta) {
  const int64_t ch = blockIdx.x;
  const int64_t n0 = blockIdx.y * n_per, n1 = min(n, n0 + n_per);
  const float mu = mean[ch];
  const float rk = relu_out ? invstd[ch] * (gamma ? gamma[ch] : 1.f) : 0.f;
  const float rb = relu_out && beta ? beta[ch] : 0.f;
  float sd = 0.f, sdz = 0.f;
  for (int64_t img = n0; img < n1; ++img) {
    const int64_t base = (img * c + ch) * s;
    const float* dyp = dy + img * dy_img + ch * s;
    if ((s & 3) == 0) {
      for (int64_t q = threadIdx.x; q < s / 4; q += 256) {
        const floatx4 g = reinterpret_cast<const floatx4*>(dyp)[q];
        const floatx4 v = reinterpret_cast<const floatx4*>(z + base)[q];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float ge = !relu_out || bn_relu_mask(v[e], mu, rk, rb) ? g[e] : 0.f;
          sd += ge;
          sdz += ge * (v[e] - mu);
        }
      }
    } else {
      for (int64_t i = threadIdx.x; i < s; i += 256) {
        const float zv = z[base + i];
        const float g = !relu_out || bn_relu_mask(zv, mu, rk, rb) ? dyp[i] : 0.f;
        sd += g;
        sdz += g * (zv - mu);
      }
    }
  }
  __shared__ float red[2][4];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    sd += __shfl_xor(sd, off);
    sdz += __shfl_xor(sdz, off);
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][wave] = sd;
    red[1][wave] = sdz;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(sums + ch, red[0][0] + red[0][1] + red[0][2] + red[0][3]);
    atomicAdd(sums + c + ch, red[1][0] + red[1][1] + red[1][2] + red[1][3]);
  }
}

template <bool kVec>
__global__ __launch_bounds__(256) void bn_bwd_dz_kernel(
    const float* __restrict__ dy, const float* __restrict__ z, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma,
    const float* __restrict__ sums, float* __restrict__ dz, float* __restrict__ dgamma,
    float* __restrict__ dbeta, int acc_gamma, int acc_beta, int64_t total, int64_t c, int64_t s,
    float inv_m, int64_t dy_img, int relu_out, const float* __restrict__ beta) {
  const int64_t cs = c * s;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
  const int64_t first = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (first < c) {  // parameter gradients, accumulated into .grad across micro-batches
    if (dgamma)
      dgamma[first] = (acc_gamma ? dgamma[first] : 0.f) + sums[c + first] * invstd[first];
    if (dbeta) dbeta[first] = (acc_beta ? dbeta[first] : 0.f) + sums[first];
  }
  if constexpr (kVec) {
    for (int64_t q = first; q < total / 4; q += stride) {
      const int64_t ch = (4 * q / s) % c;
      const float is = invstd[ch];
      const float k1 = (gamma ? gamma[ch] : 1.f) * is;
      const float k2 = sums[ch] * inv_m;
      const float k3 = is * is * sums[c + ch] * inv_m;
      const float mu = mean[ch];
      const int64_t img = 4 * q / cs;
      floatx4 g = *reinterpret_cast<const floatx4*>(dy + img * dy_img + (4 * q - img * cs));
      const floatx4 v = reinterpret_cast<const floatx4*>(z)[q];
      if (relu_out) {
        const float rb = beta ? beta[ch] : 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) g[e] = bn_relu_mask(v[e], mu, k1, rb) ? g[e] : 0.f;
      }
      floatx4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = k1 * (g[e] - k2 - (v[e] - mu) * k3);
      reinterpret_cast<floatx4*>(dz)[q] = o;
    }
  } else {
    for (int64_t i = first; i < total; i += stride) {
      const int64_t ch = (i / s) % c;
      const float is = invstd[ch];
      const float k1 = (gamma ? gamma[ch] : 1.f) * is;
      const int64_t img = i / cs;
      float g = dy[img * dy_img + (i - img * cs)];
      if (relu_out && !bn_relu_mask(z[i], mean[ch], k1, beta ? beta[ch] : 0.f)) g = 0.f;
      dz[i] = k1 * (g - sums[ch] * inv_m - (z[i] - mean[ch]) * is * is * sums[c + ch] * inv_m);
    }
  }
}

// The whole BatchNorm backward of one channel in one workgroup: the (sum dy,
// sum dy * (z - mean)) reduction, then dz and the affine gradients from the workgroup's own
// sums -- one launch instead of bn_bwd_reduce + bn_bwd_dz, no atomics, for channels small
// enough (n * s elements) that the second read of dy / z comes back from L2.  Same
// arithmetic per element as the two-pass kernels.
// kOutMask (ResNet's residual join, relu(bn(z) + identity)): the ReLU mask comes from the
// join's saved output y (same layout as z), the masked gradient -- the identity's gradient
// as well -- is written to gout in the first pass and read back from there in the second,
// instead of a separate threshold_backward pass over dy before this kernel.
template <bool kVec, bool kOutMask>
__global__ __launch_bounds__(256) void bn_bwd_channel_kernel(
    const float* __restrict__ dy, const float* __restrict__ z, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ dz, float* __restrict__ dgamma,
    float* __restrict__ dbeta, int acc_gamma, int acc_beta, int n, int c, int s, float inv_m,
    int64_t dy_img, int relu_out, BnParts parts, const float* __restrict__ ymask,
    float* __restrict__ gout) {
  const int ch = blockIdx.x;
  int dyc = ch;  // dy's channel index (its own part's, with parts)
  if (parts.count > 0) {
    int pi = 0;
    while (pi + 1 < parts.count && ch >= parts.c_end[pi]) ++pi;
    const int begin = pi == 0 ? 0 : parts.c_end[pi - 1];
    dyc = ch - begin;
    dy = parts.dy[pi];
    dy_img = parts.dy_img[pi];
    gamma = parts.gamma[pi] ? parts.gamma[pi] - begin : nullptr;
    beta = parts.beta[pi] ? parts.beta[pi] - begin : nullptr;
    dgamma = parts.dgamma[pi] ? parts.dgamma[pi] - begin : nullptr;
    dbeta = parts.dbeta[pi] ? parts.dbeta[pi] - begin : nullptr;
    acc_gamma = parts.acc_gamma[pi];
    acc_beta = parts.acc_beta[pi];
  }
  const float mu = mean[ch];
  const float is = invstd[ch];
  const float k1 = (gamma ? gamma[ch] : 1.f) * is;
  const float rb = relu_out && beta ? beta[ch] : 0.f;
  float sd = 0.f, sdz = 0.f;
  const int per = kVec ? s / 4 : s;
  const int total = n * per;
  if (dy == nullptr) {  // a part without a gradient: dz = 0, no parameter gradient added
    if (threadIdx.x == 0) {
      if (dgamma && !acc_gamma) dgamma[ch] = 0.f;
      if (dbeta && !acc_beta) dbeta[ch] = 0.f;
    }
    for (int e = threadIdx.x; e < n * s; e += 256) {
      const int img = e / s;
      dz[(static_cast<int64_t>(img) * c + ch) * s + (e - img * s)] = 0.f;
    }
    return;
  }
  if constexpr (kVec) {
    // two quads per thread per round, loads first (summed in the same order as one per
    // round)
    for (int e0 = threadIdx.x; e0 < total; e0 += 2 * 256) {
      floatx4 g[2], v[2], ym[2];
      int64_t zo[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int e = e0 + u * 256;
        if (e >= total) break;
        const int img = e / per, q = e - img * per;
        zo[u] = (static_cast<int64_t>(img) * c + ch) * s + 4 * q;
        g[u] = reinterpret_cast<const floatx4*>(dy + img * dy_img +
                                                static_cast<int64_t>(dyc) * s)[q];
        v[u] = *reinterpret_cast<const floatx4*>(z + zo[u]);
        if constexpr (kOutMask) ym[u] = *reinterpret_cast<const floatx4*>(ymask + zo[u]);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (e0 + u * 256 >= total) break;
        floatx4 gm;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          bool keep;
          if constexpr (kOutMask) keep = ym[u][k] > 0.f;
          else keep = !relu_out || bn_relu_mask(v[u][k], mu, k1, rb);
          const float ge = keep ? g[u][k] : 0.f;
          gm[k] = ge;
          sd += ge;
          sdz += ge * (v[u][k] - mu);
        }
        if constexpr (kOutMask) *reinterpret_cast<floatx4*>(gout + zo[u]) = gm;
      }
    }
  } else {
    // planes of s % 4 != 0 pixels: four elements per thread per round, loads first (one
    // element per round left a load latency per element exposed: 27.6 us per 1024-channel
    // 7^2 BatchNorm at 40 images in the stage-6 trace); summed in the same order
    for (int e0 = threadIdx.x; e0 < total; e0 += 4 * 256) {
      float gv[4], zv[4], yv[4];
      int64_t zo[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + u * 256;
        const int img = e / per, q = e - img * per;
        const bool in = e < total;
        zo[u] = (static_cast<int64_t>(img) * c + ch) * s + q;
        zv[u] = in ? z[zo[u]] : 0.f;
        gv[u] = in ? dy[img * dy_img + static_cast<int64_t>(dyc) * s + q] : 0.f;
        if constexpr (kOutMask) yv[u] = in ? ymask[zo[u]] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (e0 + u * 256 >= total) break;
        bool keep;
        if constexpr (kOutMask) keep = yv[u] > 0.f;
        else keep = !relu_out || bn_relu_mask(zv[u], mu, k1, rb);
        const float g = keep ? gv[u] : 0.f;
        if constexpr (kOutMask) gout[zo[u]] = g;
        sd += g;
        sdz += g * (zv[u] - mu);
      }
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    sd += __shfl_xor(sd, off);
    sdz += __shfl_xor(sdz, off);
  }
  __shared__ float red[2][4];
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][wave] = sd;
    red[1][wave] = sdz;
  }
  __syncthreads();
  sd = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
  sdz = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  if (threadIdx.x == 0) {
    if (dgamma) dgamma[ch] = (acc_gamma ? dgamma[ch] : 0.f) + sdz * is;
    if (dbeta) dbeta[ch] = (acc_beta ? dbeta[ch] : 0.f) + sd;
  }
  const float k2 = sd * inv_m;
  const float k3 = is * is * sdz * inv_m;
  if constexpr (kVec) {
    for (int e0 = threadIdx.x; e0 < total; e0 += 2 * 256) {
      floatx4 g[2], v[2];
      int64_t zo[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int e = e0 + u * 256;
        if (e >= total) break;
        const int img = e / per, q = e - img * per;
        zo[u] = (static_cast<int64_t>(img) * c + ch) * s + 4 * q;
        // (kOutMask: this thread's own first-pass store, masked already)
        if constexpr (kOutMask) g[u] = *reinterpret_cast<const floatx4*>(gout + zo[u]);
        else g[u] = reinterpret_cast<const floatx4*>(dy + img * dy_img +
                                                     static_cast<int64_t>(dyc) * s)[q];
        v[u] = *reinterpret_cast<const floatx4*>(z + zo[u]);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (e0 + u * 256 >= total) break;
        floatx4 o;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float gk =
              !kOutMask && relu_out && !bn_relu_mask(v[u][k], mu, k1, rb) ? 0.f : g[u][k];
          o[k] = k1 * (gk - k2 - (v[u][k] - mu) * k3);
        }
        *reinterpret_cast<floatx4*>(dz + zo[u]) = o;
      }
    }
  } else {
    for (int e0 = threadIdx.x; e0 < total; e0 += 4 * 256) {
      float gv[4], zv[4];
      int64_t zo[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + u * 256;
        const int img = e / per, q = e - img * per;
        const bool in = e < total;
        zo[u] = (static_cast<int64_t>(img) * c + ch) * s + q;
        zv[u] = in ? z[zo[u]] : 0.f;
        if constexpr (kOutMask) gv[u] = in ? gout[zo[u]] : 0.f;
        else gv[u] = in ? dy[img * dy_img + static_cast<int64_t>(dyc) * s + q] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (e0 + u * 256 >= total) break;
        float g = gv[u];
        if (!kOutMask && relu_out && !bn_relu_mask(zv[u], mu, k1, rb)) g = 0.f;
        dz[zo[u]] = k1 * (g - k2 - (zv[u] - mu) * k3);
      }
    }
  }
}

// One wave per (image, channel) plane, four planes per workgroup: mean and centred M2
// of the plane (two passes, the second from L1/L2), 16-byte loads when s % 4 == 0.
// Wave-sized work keeps small planes (7^2..14^2) from leaving 3/4 of a workgroup idle.
template <bool kVec>
__global__ __launch_bounds__(256) void bn_stats_kernel(const float* __restrict__ z,
                                                       float* __restrict__ pm,
                                                       float* __restrict__ pm2, int64_t n,
                                                       int64_t c, int64_t s) {
  const int lane = threadIdx.x & 63;
  const int64_t ch = blockIdx.x, img = static_cast<int64_t>(blockIdx.y) * 4 + (threadIdx.x >> 6);
  if (img >= n) return;
  const float* plane = z + (img * c + ch) * s;
  float acc = 0.f;
  if constexpr (kVec) {
    for (int64_t q = lane; q < s / 4; q += 64) {
      const floatx4 v = reinterpret_cast<const floatx4*>(plane)[q];
      acc += (v[0] + v[1]) + (v[2] + v[3]);
    }
  } else {
    for (int64_t i = lane; i < s; i += 64) acc += plane[i];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  const float mean = acc / static_cast<float>(s);
  float m2 = 0.f;
  if constexpr (kVec) {
    for (int64_t q = lane; q < s / 4; q += 64) {
      const floatx4 v = reinterpret_cast<const floatx4*>(plane)[q];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[e] - mean;
        m2 += d * d;
      }
    }
  } else {
    for (int64_t i = lane; i < s; i += 64) {
      const float d = plane[i] - mean;
      m2 += d * d;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m2 += __shfl_xor(m2, off);
  if (lane == 0) {
    pm[img * c + ch] = mean;
    pm2[img * c + ch] = m2;
  }
}

// DeferredBatchNorm commit: running-stat EMA from the fp64 (count, mean, M2)
// accumulators (unbiased variance), then the accumulators are zeroed.
__global__ __launch_bounds__(256) void dbn_commit64_kernel(double* __restrict__ acc,
                                                           float* __restrict__ rm,
                                                           float* __restrict__ rv, int64_t c,
                                                           double momentum) {
  const int64_t ch = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (ch >= c) return;
  const double n = acc[ch], mean = acc[c + ch], m2 = acc[2 * c + ch];
  if (n > 0.0) {
    const double var = n > 1.0 ? m2 / (n - 1.0) : 0.0;
    rm[ch] = static_cast<float>((1.0 - momentum) * rm[ch] + momentum * mean);
    rv[ch] = static_cast<float>((1.0 - momentum) * rv[ch] + momentum * var);
  }
  acc[ch] = 0.0;
  acc[c + ch] = 0.0;
  acc[2 * c + ch] = 0.0;
}

unsigned grid_for(int64_t work) {
  const int64_t blocks = (work + 255) / 256;
  return static_cast<unsigned>(blocks < 8192 ? (blocks > 0 ? blocks : 1) : 8192);
}

}  // namespace

void launch_bn_finalize(const float* part_mean, const float* part_m2, int blocks, int width,
                        int64_t total, int64_t c, float eps, double momentum, float* mean,
                        float* invstd, float* running_mean, float* running_var, int64_t* tracked,
                        double* acc, float* zero2c, hipStream_t stream) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(static_cast<unsigned>((c + 7) / 8)),
                     dim3(256), 0, stream, part_mean, part_m2, blocks, width, total, c, eps,
                     momentum, mean, invstd, running_mean, running_var, tracked, acc, zero2c);
}

void launch_bn_finalize_apply(const float* part_mean, const float* part_m2, int blocks,
                              int width, int64_t n, int64_t c, int64_t s, float eps,
                              double momentum, float* mean, float* invstd, float* running_mean,
                              float* running_var, int64_t* tracked, double* acc, float* zero2c,
                              const float* z, const float* gamma, const float* beta,
                              const float* add, float* y, hipStream_t stream, bool relu,
                              const BnParts* parts) {
  if (c == 0) return;
  BnParts none{};
  const BnParts& pt = parts != nullptr ? *parts : none;
  // enough (channel, image range) workgroups to cover the chip ~4x
  int64_t splits = (1024 + c - 1) / c;
  if (splits > n) splits = n;
  if (splits < 1) splits = 1;
  const int64_t n_per = (n + splits - 1) / splits;
  splits = n == 0 ? 1 : (n + n_per - 1) / n_per;
  const dim3 grid(static_cast<unsigned>(c), static_cast<unsigned>(splits));
  const int cols = static_cast<int>(n * s);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, stream, part_mean, part_m2, blocks, width, cols,
                       static_cast<int>(n), static_cast<int>(c), static_cast<int>(s),
                       static_cast<int>(n_per), eps, momentum, mean, invstd, running_mean,
                       running_var, tracked, acc, zero2c, z, gamma, beta, add, y, pt);
  };
  const bool vec = (s & 3) == 0;
  if (relu && add) {  // ResNet's residual join relu(bn(z) + identity)
    if (vec) go(bn_finalize_apply_kernel<true, true, true>);
    else go(bn_finalize_apply_kernel<false, true, true>);
  } else if (relu) {  // (ResNet's BatchNorm -> ReLU)
    if (vec) go(bn_finalize_apply_kernel<true, false, true>);
    else go(bn_finalize_apply_kernel<false, false, true>);
  } else if (vec && add) go(bn_finalize_apply_kernel<true, true, false>);
  else if (vec) go(bn_finalize_apply_kernel<true, false, false>);
  else if (add) go(bn_finalize_apply_kernel<false, true, false>);
  else go(bn_finalize_apply_kernel<false, false, false>);
}

bool split_bn_small_ok(int64_t n, int64_t s) {
  static const bool on = env_int("TGPIPE_SPLIT_BN", 1) != 0;
  return on && s <= 64 && n * s <= kSplitBnPer * 256;
}

void launch_split_bn_small(const float* ws, int splits, int64_t stride, float* z, int64_t n,
                           int64_t c, int64_t s, float eps, double momentum, float* mean,
                           float* invstd, float* running_mean, float* running_var,
                           int64_t* tracked, double* acc, float* zero2c, const float* gamma,
                           const float* beta, const float* add, float* y, hipStream_t stream,
                           bool relu, const BnParts* parts) {
  if (c == 0 || n * s == 0) return;
  BnParts none{};
  const BnParts& pt = parts != nullptr ? *parts : none;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(c)), dim3(256), 0, stream, ws, splits,
                       stride, z, static_cast<int>(n), static_cast<int>(c), static_cast<int>(s),
                       eps, momentum, mean, invstd, running_mean, running_var, tracked, acc,
                       zero2c, gamma, beta, add, y, pt);
  };
  if (add != nullptr && relu) go(split_bn_small_kernel<true, true>);
  else if (add != nullptr) go(split_bn_small_kernel<true, false>);
  else if (relu) go(split_bn_small_kernel<false, true>);
  else go(split_bn_small_kernel<false, false>);
}

void launch_dbn_commit64(double* acc, float* running_mean, float* running_var, int64_t c,
                         double momentum, hipStream_t stream) {
  if (c == 0) return;
  hipLaunchKernelGGL(dbn_commit64_kernel, dim3(static_cast<unsigned>((c + 255) / 256)), dim3(256),
                     0, stream, acc, running_mean, running_var, c, momentum);
}

void launch_bn_stats(const float* z, float* part_mean, float* part_m2, int64_t n, int64_t c,
                     int64_t s, hipStream_t stream) {
  if (n == 0 || c == 0) return;
  const dim3 grid(static_cast<unsigned>(c), static_cast<unsigned>((n + 3) / 4));
  if ((s & 3) == 0)
    hipLaunchKernelGGL(bn_stats_kernel<true>, grid, dim3(256), 0, stream, z, part_mean, part_m2,
                       n, c, s);
  else
    hipLaunchKernelGGL(bn_stats_kernel<false>, grid, dim3(256), 0, stream, z, part_mean, part_m2,
                       n, c, s);
}

void launch_bn_apply(const float* z, const float* mean, const float* invstd, const float* gamma,
                     const float* beta, const float* add, float* y, int64_t n, int64_t c,
                     int64_t s, hipStream_t stream) {
  const int64_t total = n * c * s;
  if (total == 0) return;
  const bool vec = (s & 3) == 0;
  const unsigned grid = grid_for(vec ? total / 4 : total);
  if (vec) {
    if (add)
      hipLaunchKernelGGL((bn_apply_kernel<true, true>), dim3(grid), dim3(256), 0, stream, z, mean,
                         invstd, gamma, beta, add, y, total, c, s);
    else
      hipLaunchKernelGGL((bn_apply_kernel<true, false>), dim3(grid), dim3(256), 0, stream, z,
                         mean, invstd, gamma, beta, add, y, total, c, s);
  } else {
    if (add)
      hipLaunchKernelGGL((bn_apply_kernel<false, true>), dim3(grid), dim3(256), 0, stream, z,
                         mean, invstd, gamma, beta, add, y, total, c, s);
    else
      hipLaunchKernelGGL((bn_apply_kernel<false, false>), dim3(grid), dim3(256), 0, stream, z,
                         mean, invstd, gamma, beta, add, y, total, c, s);
  }
}

bool bn_backward_parts_ok(int64_t n, int64_t c, int64_t s) {
  return n * s <= 32768 && n * s * c < (int64_t{1} << 31);
}

void launch_bn_backward_parts(const BnParts& parts, const float* z, const float* mean,
                              const float* invstd, float* dz, int64_t n, int64_t c, int64_t s,
                              hipStream_t stream) {
  if (n * c * s == 0) return;
  bool vec = (s & 3) == 0;
  for (int p = 0; p < parts.count; ++p) vec = vec && (parts.dy_img[p] & 3) == 0;
  const float inv_m1 = 1.f / static_cast<float>(n * s);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(c)), dim3(256), 0, stream,
                       static_cast<const float*>(nullptr), z, mean, invstd,
                       static_cast<const float*>(nullptr), static_cast<const float*>(nullptr),
                       dz, static_cast<float*>(nullptr), static_cast<float*>(nullptr), 0, 0,
                       static_cast<int>(n), static_cast<int>(c), static_cast<int>(s), inv_m1,
                       int64_t{0}, 0, parts, static_cast<const float*>(nullptr),
                       static_cast<float*>(nullptr));
  };
  if (vec) go(bn_bwd_channel_kernel<true, false>);
  else go(bn_bwd_channel_kernel<false, false>);
}

bool bn_backward_one_pass(int64_t n, int64_t c, int64_t s, int64_t dy_img) {
  // Channels of up to 32 k elements: one workgroup per channel does both passes (its dy /
  // z stay in L2 between them).  TGPIPE_BN_BWD_ONEPASS=0: always two passes.
  static const int64_t one_pass_max = [] {
    const char* v = std::getenv("TGPIPE_BN_BWD_ONEPASS");
    return v != nullptr && std::string(v) == "0" ? int64_t{0} : int64_t{32768};
  }();
  if (dy_img <= 0) dy_img = c * s;
  return n * s <= one_pass_max && c >= 64 && n * s * c < (int64_t{1} << 31) &&
         dy_img < (int64_t{1} << 31);
}

void launch_bn_backward(const float* dy, const float* z, const float* mean, const float* invstd,
                        const float* gamma, float* sums, float* dz, float* dgamma, float* dbeta,
                        bool acc_gamma, bool acc_beta, int64_t n, int64_t c, int64_t s,
                        int64_t dy_img, hipStream_t stream, bool relu_out, const float* beta,
                        const float* ymask, float* gout) {
  if (dy_img <= 0) dy_img = c * s;
  const int64_t total = n * c * s;
  if (total == 0) return;
  if (bn_backward_one_pass(n, c, s, dy_img)) {
    const float inv_m1 = 1.f / static_cast<float>(n * s);
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(c)), dim3(256), 0, stream, dy, z, mean,
                         invstd, gamma, beta, dz, dgamma, dbeta, acc_gamma ? 1 : 0,
                         acc_beta ? 1 : 0, static_cast<int>(n), static_cast<int>(c),
                         static_cast<int>(s), inv_m1, dy_img, relu_out ? 1 : 0, BnParts{},
                         ymask, gout);
    };
    const bool vec = (s & 3) == 0 && (dy_img & 3) == 0;
    if (ymask != nullptr) {
      if (vec) go(bn_bwd_channel_kernel<true, true>);
      else go(bn_bwd_channel_kernel<false, true>);
    } else if (vec) {
      go(bn_bwd_channel_kernel<true, false>);
    } else {
      go(bn_bwd_channel_kernel<false, false>);
    }
    return;
  }
  // (ymask / gout only where bn_backward_one_pass holds: convbn_backward masks dy itself
  // elsewhere)
  // enough (channel, image range) workgroups to cover the chip ~4x
  int64_t splits = (1024 + c - 1) / c;
  if (splits > n) splits = n;
  if (splits < 1) splits = 1;
  const int64_t n_per = (n + splits - 1) / splits;
  splits = (n + n_per - 1) / n_per;
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(static_cast<unsigned>(c),
                                                static_cast<unsigned>(splits)),
                     dim3(256), 0, stream, dy, z, mean, sums, n, c, s, n_per, dy_img,
                     relu_out ? 1 : 0, invstd, gamma, beta);
  const bool vec = (s & 3) == 0;
  int64_t work = vec ? total / 4 : total;
  if (work < c) work = c;
  const unsigned grid = grid_for(work);
  const float inv_m = 1.f / static_cast<float>(n * s);
  if (vec)
    hipLaunchKernelGGL((bn_bwd_dz_kernel<true>), dim3(grid), dim3(256), 0, stream, dy, z, mean,
                       invstd, gamma, sums, dz, dgamma, dbeta, acc_gamma ? 1 : 0,
                       acc_beta ? 1 : 0, total, c, s, inv_m, dy_img, relu_out ? 1 : 0, beta);
  else
    hipLaunchKernelGGL((bn_bwd_dz_kernel<false>), dim3(grid), dim3(256), 0, stream, dy, z, mean,
                       invstd, gamma, sums, dz, dgamma, dbeta, acc_gamma ? 1 : 0,
                       acc_beta ? 1 : 0, total, c, s, inv_m, dy_img, relu_out ? 1 : 0, beta);
}

}  // namespace tgpipe
