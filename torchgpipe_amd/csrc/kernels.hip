// HIP kernels of torchgpipe_amd, written for gfx950 (CDNA4, wave64, 256 CUs).
//
//   K3  dna_forward      fused Dropout2d → InstanceNorm2d → LeakyReLU (U-Net cell)
//   K3b dna_backward     its backward (mask regenerated from saved scale)
//   K4  dropout          elementwise inverted dropout, explicit Philox (seed, offset)
//   K5  spin             wall-clock spin (race-provoking tests, cf. torch.cuda._sleep)
//   K6  segments_copy    multi-tensor pack/unpack for inter-stage messages
//
// Design notes (see /opt/skills guides, Appendix B "Reduction" / G13):
// * every streaming access is a 16-byte float4 per lane when the layout allows;
// * reductions: wave64 __shfl_xor tree, then LDS across the waves of a block,
// * K3 keeps the whole H*W plane of one (n, c) pair in VGPRs (up to 36 floats
//   per lane for a 192x192 plane on a 1024-lane group), so the input is read
//   from HBM exactly once in forward (stats + normalise from registers) and
//   twice in backward (x and dy), against 4 reads + 3 writes forward and
//   6 reads + 3 writes backward for the unfused PyTorch sequence.
#include "kernels.h"
#include "philox.h"

#include <hip/hip_runtime.h>
#include <math.h>

namespace tgpipe {

namespace {

constexpr int kWave = 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// Sum over an aligned group of GROUP lanes (GROUP <= 64) inside a wave.
template <int GROUP>
__device__ __forceinline__ float group_sum_in_wave(float v) {
#pragma unroll
  for (int o = GROUP / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

inline int ceil_div(int64_t a, int64_t b) { return static_cast<int>((a + b - 1) / b); }

// ---------------------------------------------------------------------------------------------
// K3: fused Dropout2d -> InstanceNorm2d -> LeakyReLU.
// A group of GROUP lanes owns one plane; lane t holds V slots, a slot being a float4 (VEC) or
// 4 scalars.  Element j of slot k of lane t:
//   VEC:   (k*GROUP + t)*4 + j          (16-byte coalesced)
//   !VEC:  (k*4 + j)*GROUP + t          (4-byte coalesced, any S)
// ---------------------------------------------------------------------------------------------
template <int GROUP>
constexpr int kPlaneBlock = GROUP >= 256 ? GROUP : 256;

template <int GROUP, int V, bool VEC>
struct PlaneTile {
  static constexpr int kBlock = kPlaneBlock<GROUP>;
  static constexpr int kPlanesPerBlock = kBlock / GROUP;
  static constexpr int kCap = GROUP * V * 4;

  __device__ static __forceinline__ int64_t index(int t, int k, int j) {
    return VEC ? static_cast<int64_t>(k * GROUP + t) * 4 + j
               : static_cast<int64_t>(k * 4 + j) * GROUP + t;
  }

  __device__ static __forceinline__ void load(const float* __restrict__ p, int t, int64_t s,
                                              bool active, float (&r)[V * 4]) {
#pragma unroll
    for (int k = 0; k < V; ++k) {
      if (VEC) {
        const int64_t idx = index(t, k, 0);
        float4 v = (active && idx < s) ? *reinterpret_cast<const float4*>(p + idx)
                                       : make_float4(0, 0, 0, 0);
        r[k * 4 + 0] = v.x;
        r[k * 4 + 1] = v.y;
        r[k * 4 + 2] = v.z;
        r[k * 4 + 3] = v.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t idx = index(t, k, j);
          r[k * 4 + j] = (active && idx < s) ? p[idx] : 0.f;
        }
      }
    }
  }

  __device__ static __forceinline__ void store(float* __restrict__ p, int t, int64_t s,
                                               bool active, const float (&r)[V * 4]) {
    if (!active) return;
#pragma unroll
    for (int k = 0; k < V; ++k) {
      if (VEC) {
        const int64_t idx = index(t, k, 0);
        if (idx < s)
          *reinterpret_cast<float4*>(p + idx) =
              make_float4(r[k * 4 + 0], r[k * 4 + 1], r[k * 4 + 2], r[k * 4 + 3]);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t idx = index(t, k, j);
          if (idx < s) p[idx] = r[k * 4 + j];
        }
      }
    }
  }

  __device__ static __forceinline__ bool valid(int t, int k, int j, int64_t s) {
    return index(t, k, j) < s;
  }

  // Sum across the plane's group.  `lds` needs kBlock / 64 floats.
  __device__ static __forceinline__ float reduce(float v, float* lds) {
    if (GROUP <= kWave) return group_sum_in_wave<GROUP>(v);
    v = wave_sum(v);
    const int wave = threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0) lds[wave] = v;
    __syncthreads();
    float total = 0.f;
#pragma unroll
    for (int w = 0; w < GROUP / kWave; ++w) total += lds[w];
    __syncthreads();
    return total;
  }
};

// Device-resident Philox state (captured graphs, parallel/segments.py): when ``rng`` is
// given, the seed is rng[0] and the call's offset is rng[1] + offset (``offset`` is then the
// call's delta inside its cell), so a replayed graph draws a fresh mask every step from
// the values the host wrote into rng before the replay.
__device__ __forceinline__ void philox_resolve(const int64_t* __restrict__ rng, uint64_t& seed,
                                               uint64_t& offset) {
  if (rng != nullptr) {
    seed = static_cast<uint64_t>(rng[0]);
    offset += static_cast<uint64_t>(rng[1]);
  }
}

__device__ __forceinline__ float plane_dropout_scale(int64_t plane, float p, uint64_t seed,
                                                     uint64_t offset, bool dropout) {
  if (!dropout) return 1.f;
  const float u = philox_uniform(philox4x32_10(static_cast<uint64_t>(plane), offset, seed).v[0]);
  return u >= p ? 1.f / (1.f - p) : 0.f;
}

template <int GROUP, int V, bool VEC>
__global__ __launch_bounds__(kPlaneBlock<GROUP>) void dna_forward_kernel(
    const float* __restrict__ x, float* __restrict__ y, float* __restrict__ mean_out,
    float* __restrict__ rstd_out, float* __restrict__ scale_out, int64_t planes, int64_t s,
    float p, float eps, float slope, uint64_t seed, uint64_t offset, bool dropout,
    const int64_t* __restrict__ rng) {
  using T = PlaneTile<GROUP, V, VEC>;
  philox_resolve(rng, seed, offset);
  __shared__ float lds[T::kBlock / kWave];
  const int t = threadIdx.x % GROUP;
  const int64_t plane = static_cast<int64_t>(blockIdx.x) * T::kPlanesPerBlock + threadIdx.x / GROUP;
  const bool active = plane < planes;
  const float* xp = x + (active ? plane : 0) * s;

  float r[V * 4];
  T::load(xp, t, s, active, r);

  float acc = 0.f;
#pragma unroll
  for (int e = 0; e < V * 4; ++e) acc += r[e];
  const float inv_s = 1.f / static_cast<float>(s);
  const float mean = T::reduce(acc, lds) * inv_s;

  float sq = 0.f;
#pragma unroll
  for (int k = 0; k < V; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float d = T::valid(t, k, j, s) ? r[k * 4 + j] - mean : 0.f;
      sq += d * d;
    }
  const float var = T::reduce(sq, lds) * inv_s;

  const float scale = plane_dropout_scale(plane, p, seed, offset, dropout);
  const float rstd = rsqrtf(scale * scale * var + eps);
  const float mul = scale * rstd;
#pragma unroll
  for (int e = 0; e < V * 4; ++e) {
    const float z = (r[e] - mean) * mul;
    r[e] = z > 0.f ? z : z * slope;
  }
  T::store(y + (active ? plane : 0) * s, t, s, active, r);
  if (active && t == 0) {
    mean_out[plane] = mean;
    rstd_out[plane] = rstd;
    scale_out[plane] = scale;
  }
}

template <int GROUP, int V, bool VEC>
__global__ __launch_bounds__(kPlaneBlock<GROUP>) void dna_backward_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, const float* __restrict__ mean_in,
    const float* __restrict__ rstd_in, const float* __restrict__ scale_in, float* __restrict__ dx,
    int64_t planes, int64_t s, float slope) {
  using T = PlaneTile<GROUP, V, VEC>;
  __shared__ float lds[T::kBlock / kWave];
  const int t = threadIdx.x % GROUP;
  const int64_t plane = static_cast<int64_t>(blockIdx.x) * T::kPlanesPerBlock + threadIdx.x / GROUP;
  const bool active = plane < planes;
  const int64_t base = (active ? plane : 0) * s;

  const float mean = active ? mean_in[plane] : 0.f;
  const float rstd = active ? rstd_in[plane] : 0.f;
  const float scale = active ? scale_in[plane] : 0.f;
  const float mul = scale * rstd;

  float z[V * 4];
  float g[V * 4];
  T::load(x + base, t, s, active, z);
  T::load(dy + base, t, s, active, g);

  float sg = 0.f, sgz = 0.f;
#pragma unroll
  for (int e = 0; e < V * 4; ++e) {
    z[e] = (z[e] - mean) * mul;
    g[e] = z[e] > 0.f ? g[e] : g[e] * slope;  // padded lanes carry g = 0
    sg += g[e];
    sgz += g[e] * z[e];
  }
  const float inv_s = 1.f / static_cast<float>(s);
  const float mg = T::reduce(sg, lds) * inv_s;
  const float mgz = T::reduce(sgz, lds) * inv_s;
#pragma unroll
  for (int e = 0; e < V * 4; ++e) g[e] = mul * (g[e] - mg - z[e] * mgz);
  T::store(dx + base, t, s, active, g);
}

// Planes larger than one register tile: three streaming passes per plane.
constexpr int kBigGroup = 1024;

__global__ __launch_bounds__(kBigGroup) void dna_forward_big_kernel(
    const float* __restrict__ x, float* __restrict__ y, float* __restrict__ mean_out,
    float* __restrict__ rstd_out, float* __restrict__ scale_out, int64_t s, float p, float eps,
    float slope, uint64_t seed, uint64_t offset, bool dropout, const int64_t* __restrict__ rng) {
  __shared__ float lds[kBigGroup / kWave];
  philox_resolve(rng, seed, offset);
  using T = PlaneTile<kBigGroup, 1, false>;
  const int64_t plane = blockIdx.x;
  const float* xp = x + plane * s;
  float acc = 0.f;
  for (int64_t i = threadIdx.x; i < s; i += kBigGroup) acc += xp[i];
  const float inv_s = 1.f / static_cast<float>(s);
  const float mean = T::reduce(acc, lds) * inv_s;
  float sq = 0.f;
  for (int64_t i = threadIdx.x; i < s; i += kBigGroup) {
    const float d = xp[i] - mean;
    sq += d * d;
  }
  const float var = T::reduce(sq, lds) * inv_s;
  const float scale = plane_dropout_scale(plane, p, seed, offset, dropout);
  const float rstd = rsqrtf(scale * scale * var + eps);
  const float mul = scale * rstd;
  float* yp = y + plane * s;
  for (int64_t i = threadIdx.x; i < s; i += kBigGroup) {
    const float z = (xp[i] - mean) * mul;
    yp[i] = z > 0.f ? z : z * slope;
  }
  if (threadIdx.x == 0) {
    mean_out[plane] = mean;
    rstd_out[plane] = rstd;
    scale_out[plane] = scale;
  }
}

__global__ __launch_bounds__(kBigGroup) void dna_backward_big_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, const float* __restrict__ mean_in,
    const float* __restrict__ rstd_in, const float* __restrict__ scale_in, float* __restrict__ dx,
    int64_t s, float slope) {
  __shared__ float lds[kBigGroup / kWave];
  using T = PlaneTile<kBigGroup, 1, false>;
  const int64_t plane = blockIdx.x;
  const float mean = mean_in[plane];
  const float mul = scale_in[plane] * rstd_in[plane];
  const float* xp = x + plane * s;
  const float* gp = dy + plane * s;
  float sg = 0.f, sgz = 0.f;
  for (int64_t i = threadIdx.x; i < s; i += kBigGroup) {
    const float z = (xp[i] - mean) * mul;
    const float g = z > 0.f ? gp[i] : gp[i] * slope;
    sg += g;
    sgz += g * z;
  }
  const float inv_s = 1.f / static_cast<float>(s);
  const float mg = T::reduce(sg, lds) * inv_s;
  const float mgz = T::reduce(sgz, lds) * inv_s;
  float* dp = dx + plane * s;
  for (int64_t i = threadIdx.x; i < s; i += kBigGroup) {
    const float z = (xp[i] - mean) * mul;
    const float g = z > 0.f ? gp[i] : gp[i] * slope;
    dp[i] = mul * (g - mg - z * mgz);
  }
}

// ---------------------------------------------------------------------------------------------
// K4: elementwise dropout.  One Philox call yields the 4 draws of 4 consecutive elements.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void dropout_kernel(const float* __restrict__ x,
                                                      float* __restrict__ y, int64_t n, float p,
                                                      uint64_t seed, uint64_t offset, bool vec,
                                                      const int64_t* __restrict__ rng) {
  philox_resolve(rng, seed, offset);
  const float scale = 1.f / (1.f - p);
  const int64_t quads = (n + 3) / 4;
  for (int64_t q = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; q < quads;
       q += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const PhiloxOut r = philox4x32_10(static_cast<uint64_t>(q), offset, seed);
    const int64_t e0 = q * 4;
    if (vec && e0 + 3 < n) {
      float4 v = *reinterpret_cast<const float4*>(x + e0);
      v.x = philox_uniform(r.v[0]) >= p ? v.x * scale : 0.f;
      v.y = philox_uniform(r.v[1]) >= p ? v.y * scale : 0.f;
      v.z = philox_uniform(r.v[2]) >= p ? v.z * scale : 0.f;
      v.w = philox_uniform(r.v[3]) >= p ? v.w * scale : 0.f;
      *reinterpret_cast<float4*>(y + e0) = v;
    } else {
      for (int j = 0; j < 4 && e0 + j < n; ++j)
        y[e0 + j] = philox_uniform(r.v[j]) >= p ? x[e0 + j] * scale : 0.f;
    }
  }
}

__global__ __launch_bounds__(256) void philox_uniform_kernel(float* __restrict__ out, int64_t n,
                                                             uint64_t seed, uint64_t offset,
                                                             const int64_t* __restrict__ rng) {
  philox_resolve(rng, seed, offset);
  const int64_t quads = (n + 3) / 4;
  for (int64_t q = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; q < quads;
       q += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const PhiloxOut r = philox4x32_10(static_cast<uint64_t>(q), offset, seed);
    for (int j = 0; j < 4 && q * 4 + j < n; ++j) out[q * 4 + j] = philox_uniform(r.v[j]);
  }
}

// ---------------------------------------------------------------------------------------------
// K5: spin.  s_memrealtime ticks at a constant 100 MHz; bounded at 60 s.
// ---------------------------------------------------------------------------------------------
__global__ void spin_kernel(uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t limit = ticks < 6000000000ull ? ticks : 6000000000ull;
  while (__builtin_amdgcn_s_memrealtime() - t0 < limit) __builtin_amdgcn_s_sleep(8);
}

// ---------------------------------------------------------------------------------------------
// K6: segment copies (pack/unpack).  blockIdx.y = segment; 16-byte path when aligned.
// ---------------------------------------------------------------------------------------------
struct SegmentTable {
  Segment seg[kMaxSegments];
};

__global__ __launch_bounds__(256) void segments_copy_kernel(SegmentTable table) {
  const Segment sg = table.seg[blockIdx.y];
  const uintptr_t a = reinterpret_cast<uintptr_t>(sg.src) | reinterpret_cast<uintptr_t>(sg.dst);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const int64_t tid = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if ((a & 15) == 0) {
    const int64_t nvec = sg.bytes / 16;
    const uint4* s = reinterpret_cast<const uint4*>(sg.src);
    uint4* d = reinterpret_cast<uint4*>(sg.dst);
    for (int64_t i = tid; i < nvec; i += stride) d[i] = s[i];
    const int64_t tail = nvec * 16;
    const char* sb = reinterpret_cast<const char*>(sg.src);
    char* db = reinterpret_cast<char*>(sg.dst);
    for (int64_t i = tail + tid; i < sg.bytes; i += stride) db[i] = sb[i];
  } else {
    const char* sb = reinterpret_cast<const char*>(sg.src);
    char* db = reinterpret_cast<char*>(sg.dst);
    for (int64_t i = tid; i < sg.bytes; i += stride) db[i] = sb[i];
  }
}

template <int GROUP, int V, bool VEC>
void dna_fwd_launch(const float* x, float* y, float* mean, float* rstd, float* scale,
                    int64_t planes, int64_t s, float p, float eps, float slope, uint64_t seed,
                    uint64_t offset, bool dropout, const int64_t* rng, hipStream_t stream) {
  using T = PlaneTile<GROUP, V, VEC>;
  const int grid = ceil_div(planes, T::kPlanesPerBlock);
  hipLaunchKernelGGL((dna_forward_kernel<GROUP, V, VEC>), dim3(grid), dim3(T::kBlock), 0, stream,
                     x, y, mean, rstd, scale, planes, s, p, eps, slope, seed, offset, dropout,
                     rng);
}

template <int GROUP, int V, bool VEC>
void dna_bwd_launch(const float* dy, const float* x, const float* mean, const float* rstd,
                    const float* scale, float* dx, int64_t planes, int64_t s, float slope,
                    hipStream_t stream) {
  using T = PlaneTile<GROUP, V, VEC>;
  const int grid = ceil_div(planes, T::kPlanesPerBlock);
  hipLaunchKernelGGL((dna_backward_kernel<GROUP, V, VEC>), dim3(grid), dim3(T::kBlock), 0,
                     stream, dy, x, mean, rstd, scale, dx, planes, s, slope);
}

// Tile table: (GROUP, V) with capacity GROUP * V * 4 >= s.  Chosen for U-Net plane sizes
// 36, 144, 576, 2304, 9216, 36864 (192^2 / 4^k) with full slots; anything else rounds up.
#define TGPIPE_DNA_DISPATCH(LAUNCH, VEC, ...)                      \
  if (s <= 16 * 1 * 4) {                                           \
    LAUNCH<16, 1, VEC>(__VA_ARGS__);                               \
  } else if (s <= 64 * 1 * 4) {                                    \
    LAUNCH<64, 1, VEC>(__VA_ARGS__);                               \
  } else if (s <= 64 * 3 * 4) {                                    \
    LAUNCH<64, 3, VEC>(__VA_ARGS__);                               \
  } else if (s <= 64 * 9 * 4) {                                    \
    LAUNCH<64, 9, VEC>(__VA_ARGS__);                               \
  } else if (s <= 256 * 9 * 4) {                                   \
    LAUNCH<256, 9, VEC>(__VA_ARGS__);                              \
  } else {                                                         \
    LAUNCH<1024, 9, VEC>(__VA_ARGS__);                             \
  }

}  // namespace

constexpr int64_t kDnaMaxTile = 1024 * 9 * 4;

void launch_dna_forward(const float* x, float* y, float* mean, float* rstd, float* scale,
                        int64_t planes, int64_t s, float p, float eps, float slope,
                        uint64_t seed, uint64_t offset, bool dropout, const int64_t* rng,
                        hipStream_t stream) {
  if (planes == 0 || s == 0) return;
  if (s > kDnaMaxTile) {
    hipLaunchKernelGGL(dna_forward_big_kernel, dim3(static_cast<unsigned>(planes)),
                       dim3(kBigGroup), 0, stream, x, y, mean, rstd, scale, s, p, eps, slope,
                       seed, offset, dropout, rng);
    return;
  }
  const bool vec = (s % 4 == 0) && (((reinterpret_cast<uintptr_t>(x) |
                                      reinterpret_cast<uintptr_t>(y)) & 15) == 0);
  if (vec) {
    TGPIPE_DNA_DISPATCH(dna_fwd_launch, true, x, y, mean, rstd, scale, planes, s, p, eps, slope,
                        seed, offset, dropout, rng, stream)
  } else {
    TGPIPE_DNA_DISPATCH(dna_fwd_launch, false, x, y, mean, rstd, scale, planes, s, p, eps,
                        slope, seed, offset, dropout, rng, stream)
  }
}

void launch_dna_backward(const float* dy, const float* x, const float* mean, const float* rstd,
                         const float* scale, float* dx, int64_t planes, int64_t s, float slope,
                         hipStream_t stream) {
  if (planes == 0 || s == 0) return;
  if (s > kDnaMaxTile) {
    hipLaunchKernelGGL(dna_backward_big_kernel, dim3(static_cast<unsigned>(planes)),
                       dim3(kBigGroup), 0, stream, dy, x, mean, rstd, scale, dx, s, slope);
    return;
  }
  const bool vec = (s % 4 == 0) && (((reinterpret_cast<uintptr_t>(x) |
                                      reinterpret_cast<uintptr_t>(dy) |
                                      reinterpret_cast<uintptr_t>(dx)) & 15) == 0);
  if (vec) {
    TGPIPE_DNA_DISPATCH(dna_bwd_launch, true, dy, x, mean, rstd, scale, dx, planes, s, slope,
                        stream)
  } else {
    TGPIPE_DNA_DISPATCH(dna_bwd_launch, false, dy, x, mean, rstd, scale, dx, planes, s, slope,
                        stream)
  }
}

void launch_dropout(const float* x, float* y, int64_t n, float p, uint64_t seed, uint64_t offset,
                    const int64_t* rng, hipStream_t stream) {
  if (n == 0) return;
  const int64_t quads = (n + 3) / 4;
  int64_t grid = (quads + 255) / 256;
  if (grid > 2048) grid = 2048;
  const bool vec = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) == 0;
  hipLaunchKernelGGL(dropout_kernel, dim3(static_cast<unsigned>(grid)), dim3(256), 0, stream, x,
                     y, n, p, seed, offset, vec, rng);
}

void launch_philox_uniform(float* out, int64_t n, uint64_t seed, uint64_t offset,
                           const int64_t* rng, hipStream_t stream) {
  if (n == 0) return;
  int64_t grid = ((n + 3) / 4 + 255) / 256;
  if (grid > 2048) grid = 2048;
  hipLaunchKernelGGL(philox_uniform_kernel, dim3(static_cast<unsigned>(grid)), dim3(256), 0,
                     stream, out, n, seed, offset, rng);
}

void launch_spin(uint64_t ns, hipStream_t stream) {
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(1), 0, stream, ns / 10);
}

void launch_segments_copy(const Segment* segs, int count, hipStream_t stream) {
  if (count <= 0) return;
  SegmentTable table{};
  int64_t largest = 0;
  for (int i = 0; i < count && i < kMaxSegments; ++i) {
    table.seg[i] = segs[i];
    if (segs[i].bytes > largest) largest = segs[i].bytes;
  }
  int64_t grid = (largest / 16 + 255) / 256;
  if (grid < 1) grid = 1;
  if (grid > 1024) grid = 1024;
  const int n = count < kMaxSegments ? count : kMaxSegments;
  hipLaunchKernelGGL(segments_copy_kernel, dim3(static_cast<unsigned>(grid), n), dim3(256), 0,
                     stream, table);
}

}  // namespace tgpipe
