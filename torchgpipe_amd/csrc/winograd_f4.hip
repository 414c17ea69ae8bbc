// Winograd F(4x4, 3x3) convolution on the fp32 MFMA pipes of CDNA4 (gfx950).
//
// The F(2x2,3x3) kernels of winograd.hip spend 16 matrix-core multiplies per 4 output
// pixels (4 per pixel, 2.25x fewer than a direct 3x3); F(4x4,3x3) spends 36 per 16
// (2.25 per pixel, 4x fewer), so the same matrix-core time covers 1.78x the output.
// The price is a 6x6 input patch per tile and transforms with coefficients up to 8
// (fp32 rounding at the 1e-6..1e-5 relative level, what cuDNN/MIOpen's F(4x4) fp32
// kernels give as well).
//
//   V[xi][c][t] = (B^T d B)[xi]   6x6 input patch of tile t, channel c       (VALU -> LDS)
//   U[xi][c][o] = (G g G^T)[xi]   pre-transformed weights                     (global -> LDS)
//   M[xi][o][t] = sum_c U[xi][c][o] V[xi][c][t]   36 independent GEMMs        (MFMA 16x16x4)
//   Y[o][t]     = A^T M A                         4x4 output patch            (registers -> HBM)
//
// Workgroup: 8 waves, 64 output channels x 32 tiles (512 output pixels per channel);
// wave (wo, wt) = (wave & 3, wave >> 2) owns 16 channels x 16 tiles for all 36
// positions (36 accumulator tiles, 144 registers), so the output transform runs in
// registers with no exchange.  One pipeline step = 4 reduction channels (the MFMA K):
// 36 MFMAs per wave, operands from a double-buffered LDS image (one barrier per step).
// Staging is split by wave: waves 0-1 load and transform the 128 input patches of the
// step (one per lane), waves 2-7 copy the step's 36 KiB weight slab -- the wave-to-SIMD
// order puts one patch wave and one slab wave on two of the four SIMDs and slab waves
// on the other two, so no SIMD carries two transform streams.
//
// Forward / backward-data variants (host `variant`, ops/conv.py picks):
//    4 / 5   fused, weight slab staged through registers (64 / 32 output channels)
//    6 / 7   fused, weight slab by LDS-DMA (global_load_lds_dwordx4)      <- < 512 channels
//   14 / 15  non-fused: f4_input_transform_kernel writes V in the GEMM's LDS-image order,
//            f4_gemm_kernel copies both operands by LDS-DMA               <- >= 512 channels
//    8-10    timing ablations of the fused patch staging (wrong results)
//   12       6 with 16-byte patch-row loads
// Weight gradient: f4_wgrad_kernel (fused) and f4_wg_vx/_mdy + f4_wgrad_gemm (non-fused).
//
// Padding taps (image borders, tiles past the end) are raw buffer loads with an
// out-of-range offset: the hardware returns 0, so no select sits between a load and
// the transform, and no address ever leaves the tensor.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <string>
#include <type_traits>

#include "kernels.h"

namespace tgpipe {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));

constexpr int kP = 36;                  // Winograd positions of a 6x6 tile
constexpr int kC = 4;                   // reduction channels per step (MFMA K)
constexpr int kOPad = 64;               // output-channel padding of U4
constexpr int kT = 32;                  // output tiles per workgroup
constexpr int kVImg = kC * kT * kP;     // 4608 floats: [4 c][32 t][36]

// Workgroup of OG 16-channel output groups x 2 tile groups = 2*OG waves.
//   OG = 4: 64 channels, 512 threads, 108 KiB LDS -> one workgroup per CU
//   OG = 2: 32 channels, 256 threads,  72 KiB LDS -> two workgroups per CU, whose
//           prologues / epilogues / barriers overlap the other's MFMAs
template <int OG>
struct F4Cfg {
  static constexpr int kO = 16 * OG;
  static constexpr int kThreads = 128 * OG;
  static constexpr int kUImg = kC * kO * kP;            // [OG][4 c][16 o][36]
  static constexpr int kBuf = kUImg + kVImg;            // one LDS buffer; two of them
  static constexpr int kSlabThreads = kThreads - 128;   // waves 2.. copy the weight slab
  static constexpr int kUVec = kUImg / 4 / kSlabThreads;  // float4 per slab thread (6 / 9)
  static_assert(kUVec * 4 * kSlabThreads == kUImg, "slab waves copy the slab evenly");
};
// Buffer offsets of padding taps.  Row, channel (< 2^30) and column terms are added per
// tap; any sum with a bad term is >= 2^30 - 4 >= the tensor's byte size (host-checked:
// < 2^30 - 64), without wrapping past 2^32.  A valid row term of -4 (tap (-1, -1) of the
// first plane) wraps back into range only together with a valid column term >= 4.
constexpr uint32_t kBadRow = 0x80000000u;
constexpr uint32_t kBadCol = 0x40000000u;

// U4[Rp/4][Op/16][4 c][16 o][36] = G g G^T of (output channel o, reduction channel r).
// v = G g G^T (36 values, row-major 6x6) of (output channel o, reduction channel r);
// zeros outside [0, O) x [0, R).
__device__ __forceinline__ void f4_weight_tile(const float* __restrict__ w, int O, int R, int o,
                                               int r, bool flip, float (&v)[kP]) {
  float g[3][3] = {};
  if (r < R && o < O) {
    if (!flip) {  // w = [O][R][3][3]
      const float* src = w + (static_cast<int64_t>(o) * R + r) * 9;
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) g[i][j] = src[i * 3 + j];
    } else {      // w = [R][O][3][3] (forward weights), rotated by 180 degrees
      const float* src = w + (static_cast<int64_t>(r) * O + o) * 9;
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) g[i][j] = src[(2 - i) * 3 + (2 - j)];
    }
  }
  // G: rows (1/4, 0, 0), -(1,1,1)/6, -(1,-1,1)/6, (1/24, 1/12, 1/6), (1/24, -1/12, 1/6), (0,0,1)
  auto lift = [](float a, float b, float c, float (&out)[6]) {
    out[0] = 0.25f * a;
    out[1] = -(a + b + c) / 6.f;
    out[2] = -(a - b + c) / 6.f;
    out[3] = a / 24.f + b / 12.f + c / 6.f;
    out[4] = a / 24.f - b / 12.f + c / 6.f;
    out[5] = c;
  };
  float t[6][3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    float col[6];
    lift(g[0][j], g[1][j], g[2][j], col);
#pragma unroll
    for (int i = 0; i < 6; ++i) t[i][j] = col[i];
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    float row[6];
    lift(t[i][0], t[i][1], t[i][2], row);
#pragma unroll
    for (int j = 0; j < 6; ++j) v[i * 6 + j] = row[j];
  }
}

__global__ void f4_weight_kernel(const float* __restrict__ w, float* __restrict__ u, int O,
                                 int R, int Op, int Rp, bool flip) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= static_cast<int64_t>(Rp) * Op) return;
  const int r = static_cast<int>(idx / Op);
  const int o = static_cast<int>(idx % Op);
  float v[kP];
  f4_weight_tile(w, O, R, o, r, flip, v);
  float* dst = u + (static_cast<int64_t>(r / kC) * (Op / 16) + o / 16) * (kC * 16 * kP) +
               ((r % kC) * 16 + o % 16) * kP;
#pragma unroll
  for (int k = 0; k < kP / 4; ++k)
    *reinterpret_cast<floatx4*>(dst + 4 * k) =
        floatx4{v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]};
}

// B^T of one 6-vector, in place (T = float, or floatx2: two vectors at once on the packed
// fp32 VALU, v_pk_fma_f32 / v_pk_add_f32).
template <typename T>
__device__ __forceinline__ void bt6(T& d0, T& d1, T& d2, T& d3, T& d4, T& d5) {
  const T p = d4 - 4.f * d2, q = d3 - 4.f * d1;
  const T s = d4 - d2, t = 2.f * (d3 - d1);
  const T r0 = 4.f * d0 - 5.f * d2 + d4;
  const T r5 = 4.f * d1 - 5.f * d3 + d5;
  d0 = r0;
  d1 = p + q;
  d2 = p - q;
  d3 = s + t;
  d4 = s - t;
  d5 = r5;
}

// Patch-wave state: raw 6x6 patch (transformed in place) and its tap offsets.
struct F4Patch {
  float d[kP];
  uint32_t row[6];   // byte offset of (row i, column x0) of channel 0, or kBadRow
  uint32_t col[6];   // 4*j, or kBadCol for columns outside the image
};

// kVec (W % 4 == 0): the 4 centre columns of a patch row are one aligned 16-byte load
// (valid whenever the row is), the two halo columns dword loads -- 18 loads, not 36.
template <bool kVec>
__device__ __forceinline__ void f4_load_patch(F4Patch& p, __amdgpu_buffer_rsrc_t xr,
                                              uint32_t chan_bytes) {
  // Opaque per call: otherwise LICM hoists the 36 loop-invariant row+column sums out of
  // the step loop and keeps them live (36 registers -> spills next to 144 accumulators).
#pragma unroll
  for (int i = 0; i < 6; ++i) asm volatile("" : "+v"(p.row[i]), "+v"(p.col[i]));
  // The channel advance goes into the range-checked VGPR offset, not soffset (which the
  // gfx9 raw-buffer range check ignores): padding channels of the last image then read
  // zeros instead of past the tensor.
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const uint32_t rb = p.row[i] + chan_bytes;
    if constexpr (kVec) {
      p.d[i * 6 + 0] =
          __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, rb + p.col[0], 0, 0));
      const auto mid = __builtin_amdgcn_raw_buffer_load_b128(xr, rb + 4, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) p.d[i * 6 + 1 + j] = __uint_as_float(mid[j]);
      p.d[i * 6 + 5] =
          __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, rb + p.col[5], 0, 0));
    } else {
#pragma unroll
      for (int j = 0; j < 6; ++j)
        p.d[i * 6 + j] =
            __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, rb + p.col[j], 0, 0));
    }
  }
}

// V = B^T d B into the lane's 36 contiguous LDS floats.  Both passes run on pairs -- the
// column pass on adjacent column pairs, the row pass on adjacent row pairs -- with the
// packed fp32 VALU: 148 instead of 242 VALU instructions per patch (the patch waves'
// VALU work is what their SIMDs stall on, profiles/pmc_f4_kernels.json valu_per_mfma).
__device__ __forceinline__ void f4_transform(F4Patch& p) {
  float* d = p.d;
#pragma unroll
  for (int jp = 0; jp < 3; ++jp) {
    floatx2 c[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) c[i] = floatx2{d[i * 6 + 2 * jp], d[i * 6 + 2 * jp + 1]};
    bt6(c[0], c[1], c[2], c[3], c[4], c[5]);
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      d[i * 6 + 2 * jp] = c[i][0];
      d[i * 6 + 2 * jp + 1] = c[i][1];
    }
  }
#pragma unroll
  for (int ip = 0; ip < 3; ++ip) {
    floatx2 r[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) r[j] = floatx2{d[2 * ip * 6 + j], d[(2 * ip + 1) * 6 + j]};
    bt6(r[0], r[1], r[2], r[3], r[4], r[5]);
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      d[2 * ip * 6 + j] = r[j][0];
      d[(2 * ip + 1) * 6 + j] = r[j][1];
    }
  }
}

__device__ __forceinline__ void f4_transform_store(F4Patch& p, float* vdst) {
  f4_transform(p);
  const float* d = p.d;
#pragma unroll
  for (int k = 0; k < kP / 4; ++k)
    reinterpret_cast<floatx4*>(vdst)[k] = floatx4{d[4 * k], d[4 * k + 1], d[4 * k + 2], d[4 * k + 3]};
}

template <typename Cfg>
__device__ __forceinline__ void f4_load_slab(floatx4 (&ur)[Cfg::kUVec],
                                             const float* __restrict__ u, int64_t slab, int stid) {
#pragma unroll
  for (int i = 0; i < Cfg::kUVec; ++i)
    ur[i] = *reinterpret_cast<const floatx4*>(u + slab + 4 * (i * Cfg::kSlabThreads + stid));
}

template <typename Cfg>
__device__ __forceinline__ void f4_store_slab(const floatx4 (&ur)[Cfg::kUVec], float* us,
                                              int stid) {
#pragma unroll
  for (int i = 0; i < Cfg::kUVec; ++i)
    *reinterpret_cast<floatx4*>(us + 4 * (i * Cfg::kSlabThreads + stid)) = ur[i];
}

// 36 MFMAs of one step: M[xi] += U[xi]^T V[xi] over the step's 4 channels (U and V images
// at separate LDS addresses).
template <typename Cfg>
__device__ __forceinline__ void f4_mfma_uv(floatx4 (&acc)[kP], const float* ubuf,
                                           const float* vbuf, int lane, int wo, int wt) {
  const floatx4* ua =
      reinterpret_cast<const floatx4*>(ubuf + ((wo * kC + (lane >> 4)) * 16 + (lane & 15)) * kP);
  const floatx4* vb = reinterpret_cast<const floatx4*>(
      vbuf + ((lane >> 4) * kT + wt * 16 + (lane & 15)) * kP);
  // operand quad q+1 is read while quad q's 4 MFMAs issue
  floatx4 a = ua[0], b = vb[0];
#pragma unroll
  for (int q = 0; q < kP / 4; ++q) {
    floatx4 an = a, bn = b;
    if (q + 1 < kP / 4) {
      an = ua[q + 1];
      bn = vb[q + 1];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
      acc[4 * q + e] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e], b[e], acc[4 * q + e], 0, 0, 0);
    a = an;
    b = bn;
  }
  __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
  for (int q = 0; q < kP / 4; ++q) {
    if (q + 1 < kP / 4) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
  }
}

// One LDS buffer = [U image][V image].
template <typename Cfg>
__device__ __forceinline__ void f4_mfma(floatx4 (&acc)[kP], const float* buf, int lane, int wo,
                                        int wt) {
  f4_mfma_uv<Cfg>(acc, buf, buf + Cfg::kUImg, lane, wo, wt);
}

// f4_mfma with the LDS operand quads read kAhead quads before their MFMAs (kAhead = 1 is
// f4_mfma); for the GEMM kernels, whose waves hold no staging registers.  kAhead = 2 ran
// the non-fused GEMMs 1-10 % faster than 1 (3: no further gain; wino_f4_glds_ablation.json).
template <typename Cfg, int kAhead>
__device__ __forceinline__ void f4_mfma_ahead(floatx4 (&acc)[kP], const float* buf, int lane,
                                              int wo, int wt) {
  constexpr int kQ = kP / 4;
  const floatx4* ua =
      reinterpret_cast<const floatx4*>(buf + ((wo * kC + (lane >> 4)) * 16 + (lane & 15)) * kP);
  const floatx4* vb = reinterpret_cast<const floatx4*>(
      buf + Cfg::kUImg + ((lane >> 4) * kT + wt * 16 + (lane & 15)) * kP);
  floatx4 a[kQ], b[kQ];
#pragma unroll
  for (int q = 0; q < kAhead; ++q) {
    a[q] = ua[q];
    b[q] = vb[q];
  }
#pragma unroll
  for (int q = 0; q < kQ; ++q) {
    if (q + kAhead < kQ) {
      a[q + kAhead] = ua[q + kAhead];
      b[q + kAhead] = vb[q + kAhead];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
      acc[4 * q + e] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q][e], b[q][e], acc[4 * q + e], 0, 0, 0);
  }
  __builtin_amdgcn_sched_group_barrier(0x100, 2 * kAhead, 0);
#pragma unroll
  for (int q = 0; q < kQ; ++q) {
    if (q + kAhead < kQ) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
  }
}

// Tap offsets of the 6x6 input patch of output tile t, channel c of the first step.
__device__ __forceinline__ void f4_fwd_offsets(F4Patch& p, int t, int c, int P, int tpi, int TW,
                                               int R, int H, int W) {
  const bool tv = t < P;
  const int tt = tv ? t : 0;
  const int n = tt / tpi;
  const int rem = tt - n * tpi;
  const int ty = rem / TW;
  const int tx = rem - ty * TW;
  const int y0 = 4 * ty - 1, x0 = 4 * tx - 1;
  // element index of (row y0, column x0) of channel c; may be -1 (wraps)
  const int64_t base = (static_cast<int64_t>(n) * R + c) * H * W +
                       static_cast<int64_t>(y0) * W + x0;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const bool ok = tv && y0 + i >= 0 && y0 + i < H;
    p.row[i] = ok ? static_cast<uint32_t>((base + static_cast<int64_t>(i) * W) * 4) : kBadRow;
  }
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const bool ok = x0 + j >= 0 && x0 + j < W;
    p.col[j] = ok ? static_cast<uint32_t>(4 * j) : kBadCol;
  }
}

// Y = A^T M A of one lane's tile tp from its 36 accumulators; register r of each holds
// output channel obase + r.  Writes the 4x4 output patch (+ bias), clipped at the edges.
__device__ __forceinline__ void f4_output_transform(const floatx4 (&acc)[kP],
                                                    float* __restrict__ ydst,
                                                    const float* __restrict__ bias, int tp,
                                                    int tpi, int TW, int H, int W, int O,
                                                    int obase) {
  const int HW = H * W;
  const int pn = tp / tpi;
  const int prem = tp - pn * tpi;
  const int pty = prem / TW;
  const int py = 4 * pty;
  const int px = 4 * (prem - pty * TW);
  const bool full = (W & 3) == 0 && py + 4 <= H;
  // two output channels at a time (adjacent accumulator registers) on the packed fp32 VALU
#pragma unroll
  for (int rp = 0; rp < 2; ++rp) {
    const int o = obase + 2 * rp;
    if (o >= O) continue;
    // A^T along rows (i), for every column j
    floatx2 s[4][6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      floatx2 m[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) m[i] = floatx2{acc[i * 6 + j][2 * rp], acc[i * 6 + j][2 * rp + 1]};
      const floatx2 a = m[1] + m[2], b = m[1] - m[2], c = m[3] + m[4], d = m[3] - m[4];
      s[0][j] = m[0] + a + c;
      s[1][j] = b + 2.f * d;
      s[2][j] = a + 4.f * c;
      s[3][j] = b + 8.f * d + m[5];
    }
    const floatx2 bv{bias ? bias[o] : 0.f, bias && o + 1 < O ? bias[o + 1] : 0.f};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const floatx2 a = s[k][1] + s[k][2], b = s[k][1] - s[k][2];
      const floatx2 c = s[k][3] + s[k][4], d = s[k][3] - s[k][4];
      const floatx2 v0 = s[k][0] + a + c + bv, v1 = b + 2.f * d + bv, v2 = a + 4.f * c + bv;
      const floatx2 v3 = b + 8.f * d + s[k][5] + bv;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        if (o + e >= O) break;
        float* yp = ydst + (static_cast<int64_t>(pn) * O + o + e) * HW +
                    static_cast<int64_t>(py) * W + px;
        const floatx4 out{v0[e], v1[e], v2[e], v3[e]};
        if (full) {
          *reinterpret_cast<floatx4*>(yp + k * W) = out;
        } else if (py + k < H) {
#pragma unroll
          for (int l = 0; l < 4; ++l)
            if (px + l < W) yp[k * W + l] = out[l];
        }
      }
    }
  }
}

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glob_void_t;

// One step's weight slab straight into LDS (global_load_lds_dwordx4, no VGPR staging):
// the slab U4[s][o0/16 .. +OG][4][16][36] is contiguous and so is its LDS image, in
// 1 KiB pieces of one wave-instruction each, dealt round-robin over the slab waves.
template <typename Cfg, int kWaves>
__device__ __forceinline__ void f4_glds_slab(const float* __restrict__ src, float* dst, int sw,
                                             int lane) {
  constexpr int kPieces = Cfg::kUImg / 256;
  static_assert(kPieces % kWaves == 0, "slab waves copy the slab evenly");
#pragma unroll
  for (int i = 0; i < kPieces / kWaves; ++i) {
    const int piece = i * kWaves + sw;
    __builtin_amdgcn_global_load_lds((glob_void_t*)(src + piece * 256 + lane * 4),
                                     (lds_void_t*)(dst + piece * 256), 16, 0, 0);
  }
}

// kAblate (timing ablations only, wrong results; variants 8-10): 1 = no in-loop patch
// loads, 2 = no in-loop B^T d B (raw patch stored), 3 = neither.
template <int OG, bool kVec, bool kGlds = false, int kAblate = 0>
__global__ __launch_bounds__(F4Cfg<OG>::kThreads, 4 / OG) void f4_conv_kernel(
    const float* __restrict__ x, const float* __restrict__ u, const float* __restrict__ bias,
    float* __restrict__ y, int R, int H, int W, int O, int Rp, int Op, int TH, int TW, int P,
    int tblocks, int oblocks, int splits, uint32_t x_bytes) {
  using Cfg = F4Cfg<OG>;
  constexpr int kO = Cfg::kO;
  constexpr int kBuf = Cfg::kBuf;
  __shared__ float lds[2 * kBuf];  // 108 KiB (OG 4) / 72 KiB (OG 2)

  // XCD-aware bijective remap; output-channel blocks of one tile block are adjacent, so
  // they share the block's input patches in one XCD's L2.
  const int nwg = tblocks * oblocks * splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7;
  const int qq = nwg >> 3, rr = nwg & 7;
  const int wgid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int ob = wgid % oblocks;
  const int tb = (wgid / oblocks) % tblocks;
  const int z = wgid / (oblocks * tblocks);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wo = wave % OG;
  const int wt = wave / OG;
  const int t0 = tb * kT;
  const int o0 = ob * kO;
  const int HW = H * W;
  const int tpi = TH * TW;

  const int nsteps = Rp / kC;
  const int s_begin = z * nsteps / splits;
  const int s_end = (z + 1) * nsteps / splits;
  floatx4 acc[kP];
#pragma unroll
  for (int i = 0; i < kP; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};

  if (wave < 2) {
    // -- patch waves: tile t0 + 16*wave + (lane & 15), channel (lane >> 4) of each step --
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), static_cast<short>(0),
                                          static_cast<int>(x_bytes), 0x00020000);
    F4Patch p;
    f4_fwd_offsets(p, t0 + wave * 16 + (lane & 15), lane >> 4, P, tpi, TW, R, H, W);
    float* vmine = lds + Cfg::kUImg + ((lane >> 4) * kT + wave * 16 + (lane & 15)) * kP;
    const uint32_t step_bytes = static_cast<uint32_t>(kC) * HW * 4;
    f4_load_patch<kVec>(p, xr, s_begin * step_bytes);
    f4_transform_store(p, vmine);
    __syncthreads();
    f4_load_patch<kVec>(p, xr, min(s_begin + 1, s_end - 1) * step_bytes);
    // Per step: transform the patch loaded one step ago into the idle buffer, send the
    // loads of the step after next (a whole step of MFMAs hides them), then the MFMAs.
    for (int s = s_begin; s < s_end; ++s) {
      const int buf = (s - s_begin) & 1;
      if constexpr ((kAblate & 2) == 0) {
        f4_transform_store(p, vmine + (buf ^ 1) * kBuf);
      } else {
#pragma unroll
        for (int q = 0; q < kP / 4; ++q)
          reinterpret_cast<floatx4*>(vmine + (buf ^ 1) * kBuf)[q] =
              floatx4{p.d[4 * q], p.d[4 * q + 1], p.d[4 * q + 2], p.d[4 * q + 3]};
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr ((kAblate & 1) == 0)
        f4_load_patch<kVec>(p, xr, min(s + 2, s_end - 1) * step_bytes);
      __builtin_amdgcn_sched_barrier(0);
      f4_mfma<Cfg>(acc, lds + buf * kBuf, lane, wo, wt);
      __syncthreads();
    }
  } else {
    // -- slab waves: the step's [OG o-groups][4 c][16 o][36] weight slab --
    const int stid = tid - 128;
    const int64_t slab_stride = static_cast<int64_t>(Op / 16) * (kC * 16 * kP);
    const float* ubase = u + static_cast<int64_t>(o0 / 16) * (kC * 16 * kP);
    if constexpr (kGlds) {
      constexpr int kGldsWaves = Cfg::kSlabThreads / 64;
      const int sw = stid >> 6;
      {
        // LDS-DMA one step ahead; __syncthreads drains it (vmcnt(0)) before the buffer's use
        f4_glds_slab<Cfg, kGldsWaves>(ubase + s_begin * slab_stride, lds, sw, lane);
        __syncthreads();
        for (int s = s_begin; s < s_end; ++s) {
          const int buf = (s - s_begin) & 1;
          if (s + 1 < s_end)
            f4_glds_slab<Cfg, kGldsWaves>(ubase + (s + 1) * slab_stride, lds + (buf ^ 1) * kBuf,
                                          sw, lane);
          f4_mfma<Cfg>(acc, lds + buf * kBuf, lane, wo, wt);
          __syncthreads();
        }
      }
    } else {
      floatx4 ur[Cfg::kUVec];
      f4_load_slab<Cfg>(ur, ubase, s_begin * slab_stride, stid);
      f4_store_slab<Cfg>(ur, lds, stid);
      __syncthreads();
      f4_load_slab<Cfg>(ur, ubase, min(s_begin + 1, s_end - 1) * slab_stride, stid);
      for (int s = s_begin; s < s_end; ++s) {
        const int buf = (s - s_begin) & 1;
        f4_store_slab<Cfg>(ur, lds + (buf ^ 1) * kBuf, stid);
        __builtin_amdgcn_sched_barrier(0);
        f4_load_slab<Cfg>(ur, ubase, min(s + 2, s_end - 1) * slab_stride, stid);
        __builtin_amdgcn_sched_barrier(0);
        f4_mfma<Cfg>(acc, lds + buf * kBuf, lane, wo, wt);
        __syncthreads();
      }
    }
  }

  // -- output transform Y = A^T M A from the accumulators --------------------------------
  // Lane (wt*16 + j) holds tile t0 + wt*16 + j; register r of accumulator xi holds output
  // channel o0 + wo*16 + 4*(lane >> 4) + r.  Split-K partials go to slab z of y.
  const int tp = t0 + wt * 16 + (lane & 15);
  if (tp >= P) return;
  float* ydst = y + static_cast<int64_t>(z) * (P / tpi) * O * HW;
  f4_output_transform(acc, ydst, bias != nullptr && splits == 1 ? bias : nullptr, tp, tpi, TW,
                      H, W, O, o0 + wo * 16 + 4 * (lane >> 4));
}

// Variant 18: variant 6 with the weight slab two steps ahead.  Variant 6 waits at every
// step's barrier for the slab LDS-DMA issued at the start of that step (__syncthreads
// drains vmcnt to 0; one step of MFMAs, ~0.5 us, does not cover an L2/HBM fetch).  Here
// the U slab has a ring of three LDS images (3 x 36 KiB) next to the two V images
// (2 x 18 KiB): 147 KiB.  The slab waves issue step s+2's DMA, run step s's MFMAs, and
// retire only step s+1's DMA (counted s_waitcnt vmcnt) before a raw s_barrier, so one
// slab stays in flight across every barrier; the patch waves retire their LDS writes
// (lgkmcnt 0) before the same barrier.
template <bool kVec>
__global__ __launch_bounds__(512, 1) void f4_conv_ring_kernel(
    const float* __restrict__ x, const float* __restrict__ u, const float* __restrict__ bias,
    float* __restrict__ y, int R, int H, int W, int O, int Rp, int Op, int TH, int TW, int P,
    int tblocks, int oblocks, int splits, uint32_t x_bytes) {
  using Cfg = F4Cfg<4>;
  constexpr int kO = Cfg::kO;
  constexpr int kSlabWaves = Cfg::kSlabThreads / 64;                   // 6
  constexpr int kDmaPerWave = Cfg::kUImg / 256 / kSlabWaves;           // 6 per step
  static_assert(kDmaPerWave == 6, "the counted vmcnt below assumes 6 DMAs per wave");
  __shared__ float lds[3 * Cfg::kUImg + 2 * kVImg];  // 147 KiB: one workgroup per CU
  float* const uimg = lds;
  float* const vimg = lds + 3 * Cfg::kUImg;

  const int nwg = tblocks * oblocks * splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7;
  const int qq = nwg >> 3, rr = nwg & 7;
  const int wgid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int ob = wgid % oblocks;
  const int tb = (wgid / oblocks) % tblocks;
  const int z = wgid / (oblocks * tblocks);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wo = wave % 4;
  const int wt = wave / 4;
  const int t0 = tb * kT;
  const int o0 = ob * kO;
  const int HW = H * W;
  const int tpi = TH * TW;

  const int nsteps = Rp / kC;
  const int s_begin = z * nsteps / splits;
  const int s_end = (z + 1) * nsteps / splits;
  floatx4 acc[kP];
#pragma unroll
  for (int i = 0; i < kP; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};

  if (wave < 2) {
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), static_cast<short>(0),
                                          static_cast<int>(x_bytes), 0x00020000);
    F4Patch p;
    f4_fwd_offsets(p, t0 + wave * 16 + (lane & 15), lane >> 4, P, tpi, TW, R, H, W);
    float* vmine = vimg + ((lane >> 4) * kT + wave * 16 + (lane & 15)) * kP;
    const uint32_t step_bytes = static_cast<uint32_t>(kC) * HW * 4;
    f4_load_patch<kVec>(p, xr, s_begin * step_bytes);
    f4_transform_store(p, vmine);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    f4_load_patch<kVec>(p, xr, min(s_begin + 1, s_end - 1) * step_bytes);
    int us = 0;
    for (int s = s_begin; s < s_end; ++s) {
      const int vb = (s - s_begin) & 1;
      f4_transform_store(p, vmine + (vb ^ 1) * kVImg);
      __builtin_amdgcn_sched_barrier(0);
      f4_load_patch<kVec>(p, xr, min(s + 2, s_end - 1) * step_bytes);
      __builtin_amdgcn_sched_barrier(0);
      f4_mfma_uv<Cfg>(acc, uimg + us * Cfg::kUImg, vimg + vb * kVImg, lane, wo, wt);
      us = us == 2 ? 0 : us + 1;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  } else {
    const int sw = wave - 2;
    const int64_t slab_stride = static_cast<int64_t>(Op / 16) * (kC * 16 * kP);
    const float* ubase = u + static_cast<int64_t>(o0 / 16) * (kC * 16 * kP);
    f4_glds_slab<Cfg, kSlabWaves>(ubase + s_begin * slab_stride, uimg, sw, lane);
    if (s_begin + 1 < s_end) {
      f4_glds_slab<Cfg, kSlabWaves>(ubase + (s_begin + 1) * slab_stride, uimg + Cfg::kUImg, sw,
                                    lane);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    int us = 0;
    for (int s = s_begin; s < s_end; ++s) {
      const int vb = (s - s_begin) & 1;
      const int un = us == 0 ? 2 : us - 1;  // (us + 2) % 3: the slot step s-1 read
      const bool more = s + 2 < s_end;
      if (more)
        f4_glds_slab<Cfg, kSlabWaves>(ubase + (s + 2) * slab_stride, uimg + un * Cfg::kUImg,
                                      sw, lane);
      f4_mfma_uv<Cfg>(acc, uimg + us * Cfg::kUImg, vimg + vb * kVImg, lane, wo, wt);
      us = us == 2 ? 0 : us + 1;
      // retire step s+1's slab (leave step s+2's in flight), then the barrier
      if (more)
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }

  const int tp = t0 + wt * 16 + (lane & 15);
  if (tp >= P) return;
  float* ydst = y + static_cast<int64_t>(z) * (P / tpi) * O * HW;
  f4_output_transform(acc, ydst, bias != nullptr && splits == 1 ? bias : nullptr, tp, tpi, TW,
                      H, W, O, o0 + wo * 16 + 4 * (lane >> 4));
}

// ---- non-fused variant: input transform pass + two-operand LDS-DMA GEMM ----------------
// Variants 14 / 15 take the input transform out of the GEMM kernel (cuDNN's
// WINOGRAD_NONFUSED split): f4_input_transform_kernel writes V = B^T d B of every (tile,
// channel) once, in the exact LDS image order of the GEMM -- V4[P/32][Rp/4][4 c][32 t][36]
// -- so the GEMM kernel copies both operands per step by LDS-DMA and its eight waves only
// multiply.  The ablation that drove it: without patch staging the fused kernel is 30-37 %
// faster (profiles/wino_f4_glds_ablation.json); the pass costs 2.25x the input in writes.

// One thread per (tile, channel) of the padded grid (tiles to a multiple of 32, channels
// to a multiple of 4; the padding is written as zeros).
__global__ __launch_bounds__(256) void f4_input_transform_kernel(
    const float* __restrict__ x, float* __restrict__ v, int R, int H, int W, int TW, int tpi,
    int P, int Rp, int64_t total, uint32_t x_bytes) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  // idx = ((tb * (Rp/4) + s) * 4 + c4) * 32 + tt  (consecutive threads: consecutive tiles)
  const int tt = static_cast<int>(idx & 31);
  const int64_t rest = idx >> 5;
  const int c4 = static_cast<int>(rest & 3);
  const int64_t sb = rest >> 2;  // tb * (Rp/4) + s
  const int steps = Rp / kC;
  const int s = static_cast<int>(sb % steps);
  const int tb = static_cast<int>(sb / steps);
  const int t = tb * kT + tt;
  const int c = s * kC + c4;
  float* dst = v + idx * kP;
  F4Patch p;
  if (t >= P || c >= R) {
#pragma unroll
    for (int q = 0; q < kP / 4; ++q) reinterpret_cast<floatx4*>(dst)[q] = floatx4{0.f, 0.f, 0.f, 0.f};
    return;
  }
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), static_cast<short>(0),
                                        static_cast<int>(x_bytes), 0x00020000);
  // f4_fwd_offsets with image n's channel c (R channels per image)
  f4_fwd_offsets(p, t, c, P, tpi, TW, R, H, W);
  f4_load_patch<false>(p, xr, 0);
  f4_transform_store(p, dst);
}

// GEMM on the transformed operands: per step both the weight slab and the V slab of the
// tile block arrive by LDS-DMA (1 KiB pieces dealt round-robin over all waves).
template <int OG, int kAhead = 2>
__global__ __launch_bounds__(F4Cfg<OG>::kThreads, 4 / OG) void f4_gemm_kernel(
    const float* __restrict__ v, const float* __restrict__ u, const float* __restrict__ bias,
    float* __restrict__ y, int H, int W, int O, int Rp, int Op, int TH, int TW, int P,
    int tblocks, int oblocks, int splits) {
  using Cfg = F4Cfg<OG>;
  constexpr int kO = Cfg::kO;
  constexpr int kBuf = Cfg::kBuf;
  constexpr int kUPieces = Cfg::kUImg / 256;
  constexpr int kPieces = kBuf / 256;
  constexpr int kWaves = Cfg::kThreads / 64;
  __shared__ float lds[2 * kBuf];

  const int nwg = tblocks * oblocks * splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7;
  const int qq = nwg >> 3, rr = nwg & 7;
  const int wgid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int ob = wgid % oblocks;
  const int tb = (wgid / oblocks) % tblocks;
  const int z = wgid / (oblocks * tblocks);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wo = wave % OG;
  const int wt = wave / OG;
  const int t0 = tb * kT;
  const int o0 = ob * kO;
  const int HW = H * W;
  const int tpi = TH * TW;

  const int nsteps = Rp / kC;
  const int s_begin = z * nsteps / splits;
  const int s_end = (z + 1) * nsteps / splits;
  floatx4 acc[kP];
#pragma unroll
  for (int i = 0; i < kP; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int64_t slab_stride = static_cast<int64_t>(Op / 16) * (kC * 16 * kP);
  const float* ubase = u + static_cast<int64_t>(o0 / 16) * (kC * 16 * kP);
  const float* vbase = v + static_cast<int64_t>(tb) * nsteps * kVImg;
  auto issue = [&](int step, float* dst) {
#pragma unroll
    for (int i = 0; i < (kPieces + kWaves - 1) / kWaves; ++i) {
      const int piece = i * kWaves + wave;
      if (piece < kPieces) {
        const float* src = piece < kUPieces
                               ? ubase + step * slab_stride + piece * 256
                               : vbase + static_cast<int64_t>(step) * kVImg + (piece - kUPieces) * 256;
        __builtin_amdgcn_global_load_lds((glob_void_t*)(src + lane * 4),
                                         (lds_void_t*)(dst + piece * 256), 16, 0, 0);
      }
    }
  };
  issue(s_begin, lds);
  __syncthreads();
  for (int s = s_begin; s < s_end; ++s) {
    const int buf = (s - s_begin) & 1;
    if (s + 1 < s_end) issue(s + 1, lds + (buf ^ 1) * kBuf);
    f4_mfma_ahead<Cfg, kAhead>(acc, lds + buf * kBuf, lane, wo, wt);
    __syncthreads();
  }

  const int tp = t0 + wt * 16 + (lane & 15);
  if (tp >= P) return;
  float* ydst = y + static_cast<int64_t>(z) * (P / tpi) * O * HW;
  f4_output_transform(acc, ydst, bias != nullptr && splits == 1 ? bias : nullptr, tp, tpi,
                          TW, H, W, O, o0 + wo * 16 + 4 * (lane >> 4));
}

// y[i] = sum_z ws[z][i] (+ bias[o]) over the split-K partial slabs.  A 256-thread block
// owns 64 columns (float4 each with kVec) and sums the slabs in 4 interleaved z-lanes,
// combined through LDS: the weight-gradient partials are short rows of up to 512 slabs,
// which one thread per column walked serially (29 us per call in the p1 step).
template <bool kVec>
__global__ __launch_bounds__(256) void f4_split_reduce_kernel(
    const float* __restrict__ ws, const float* __restrict__ bias, float* __restrict__ y,
    int64_t numel, int64_t hw, int O, int splits, bool accum) {
  typedef std::conditional_t<kVec, floatx4, float> T;
  constexpr int kW = kVec ? 4 : 1;
  __shared__ T part[3][64];
  const int col = threadIdx.x & 63;
  const int zl = threadIdx.x >> 6;
  const int64_t i = (static_cast<int64_t>(blockIdx.x) * 64 + col) * kW;  // first element
  const bool ok = i < numel;
  T v{};
  if (ok) {
    const T* src = reinterpret_cast<const T*>(ws + i);
    const int64_t stride = numel / kW;
    int z = zl;
    for (; z + 4 < splits; z += 8) {
      const T a = src[z * stride], b = src[(z + 4) * stride];
      v += a;
      v += b;
    }
    if (z < splits) v += src[z * stride];
  }
  if (zl > 0) part[zl - 1][col] = v;
  __syncthreads();
  if (zl > 0 || !ok) return;
  v += part[0][col];
  v += part[1][col];
  v += part[2][col];
  if constexpr (kVec) {
    if (bias) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] += bias[((i + e) / hw) % O];
    }
    if (accum) v += *reinterpret_cast<const floatx4*>(y + i);
    *reinterpret_cast<floatx4*>(y + i) = v;
  } else {
    if (bias) v += bias[(i / hw) % O];
    y[i] = accum ? y[i] + v : v;
  }
}

void launch_split_reduce(const float* ws, const float* bias, float* y, int64_t numel, int64_t hw,
                         int O, int splits, hipStream_t stream, bool accum = false) {
  const bool vec = (numel & 3) == 0;
  const int64_t cols = vec ? numel / 4 : numel;
  const dim3 grid(static_cast<unsigned>((cols + 63) / 64));
  if (vec)
    hipLaunchKernelGGL(f4_split_reduce_kernel<true>, grid, dim3(256), 0, stream, ws, bias, y,
                       numel, hw, O, splits, accum);
  else
    hipLaunchKernelGGL(f4_split_reduce_kernel<false>, grid, dim3(256), 0, stream, ws, bias, y,
                       numel, hw, O, splits, accum);
}

// ---- weight gradient: dW = G^T [ sum_t (A dY_t A^T) (.) (B^T d_t B) ] G ------------------
//
// The trilinear form of F(4x4,3x3), sum_xi (G g)_xi (B^T d)_xi (A y)_xi = sum y_i g_j d_{i+j},
// read the other way round: the correlation of a 6x6 input patch d with the 4x4 output
// gradient tile dY is the 3x3 weight gradient, G^T [(A dY A^T) (.) (B^T d B)] G.  Summed
// over all tiles t: 36 independent GEMMs dU[xi][k][c] = sum_t M'[xi][k][t] V[xi][c][t]
// with the tiles as the reduction (MFMA K), then one output transform per (k, c).
//
// Workgroup: 8 waves, 64 output channels (k, MFMA rows) x 32 input channels (c, MFMA
// columns), all 36 positions in accumulators (the forward's f4_mfma on the same LDS
// image shapes).  One step = 4 tiles.  Staging by wave: waves 0-1 load and transform the
// step's 128 input patches (4 tiles x 32 channels, one per lane), waves 2, 3, 6, 7 the 256
// gradient tiles (4 tiles x 64 channels) -- SIMDs 0/1 carry one patch wave each, SIMDs
// 2/3 two gradient waves each -- and waves 4-5 only multiply.  Lanes of one channel take 4
// horizontally adjacent tiles, so a load instruction touches 16 channel planes.

// A of one 4-vector: (y0, y0+y1+y2+y3, y0-y1+y2-y3, y0+2y1+4y2+8y3, y0-2y1+4y2-8y3, y3)
// (T = float, or floatx2 for two vectors on the packed fp32 VALU).
template <typename T>
__device__ __forceinline__ void a6(T y0, T y1, T y2, T y3, T (&o)[6]) {
  const T e = y0 + y2, od = y1 + y3;
  const T e2 = y0 + 4.f * y2, o2 = 2.f * y1 + 8.f * y3;
  o[0] = y0;
  o[1] = e + od;
  o[2] = e - od;
  o[3] = e2 + o2;
  o[4] = e2 - o2;
  o[5] = y3;
}

// Running tile position of a staging lane: advanced by 4 tiles per fetched step.
struct F4TileCursor {
  int n, ty, tx;
};

__device__ __forceinline__ void f4_cursor_advance(F4TileCursor& cur, int TH, int TW) {
  cur.tx += 4;
  while (cur.tx >= TW) {
    cur.tx -= TW;
    if (++cur.ty == TH) {
      cur.ty = 0;
      ++cur.n;
    }
  }
}

// 6x6 input patch of (tile at cur, channel ch) -> p.row / p.col; zeros past N or C.
__device__ __forceinline__ void f4_patch_offsets(F4Patch& p, const F4TileCursor& cur, int ch,
                                                 int N, int C, int H, int W) {
  const bool tv = cur.n < N && ch < C;
  const int y0 = 4 * cur.ty - 1, x0 = 4 * cur.tx - 1;
  const int64_t base =
      (static_cast<int64_t>(tv ? cur.n : 0) * C + (tv ? ch : 0)) * H * W +
      static_cast<int64_t>(y0) * W + x0;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const bool ok = tv && y0 + i >= 0 && y0 + i < H;
    p.row[i] = ok ? static_cast<uint32_t>((base + static_cast<int64_t>(i) * W) * 4) : kBadRow;
  }
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const bool ok = x0 + j >= 0 && x0 + j < W;
    p.col[j] = ok ? static_cast<uint32_t>(4 * j) : kBadCol;
  }
}

// 4x4 gradient tile of (tile at cur, channel k): zeros outside; kVec (W % 4 == 0): one
// 16-byte load per row.
template <bool kVec>
__device__ __forceinline__ void f4_load_dy(float (&g)[16], __amdgpu_buffer_rsrc_t dyr,
                                           const F4TileCursor& cur, int k, int N, int K, int H,
                                           int W) {
  const bool tv = cur.n < N && k < K;
  const int y0 = 4 * cur.ty, x0 = 4 * cur.tx;
  const int64_t base =
      (static_cast<int64_t>(tv ? cur.n : 0) * K + (tv ? k : 0)) * H * W +
      static_cast<int64_t>(y0) * W + x0;
  uint32_t col[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) col[j] = x0 + j < W ? static_cast<uint32_t>(4 * j) : kBadCol;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t rb = tv && y0 + i < H
                            ? static_cast<uint32_t>((base + static_cast<int64_t>(i) * W) * 4)
                            : kBadRow;
    if constexpr (kVec) {
      const auto row = __builtin_amdgcn_raw_buffer_load_b128(dyr, rb, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) g[i * 4 + j] = __uint_as_float(row[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        g[i * 4 + j] =
            __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(dyr, rb + col[j], 0, 0));
    }
  }
}

// M' = A g A^T (36 values, row-major 6x6) of one 4x4 gradient tile (both passes on pairs,
// packed fp32 VALU, like f4_transform).
__device__ __forceinline__ void f4_dy_transform(const float (&g)[16], float (&m)[kP]) {
  float t[6][4];
#pragma unroll
  for (int jp = 0; jp < 2; ++jp) {
    floatx2 col[6];
    a6(floatx2{g[0 * 4 + 2 * jp], g[0 * 4 + 2 * jp + 1]},
       floatx2{g[1 * 4 + 2 * jp], g[1 * 4 + 2 * jp + 1]},
       floatx2{g[2 * 4 + 2 * jp], g[2 * 4 + 2 * jp + 1]},
       floatx2{g[3 * 4 + 2 * jp], g[3 * 4 + 2 * jp + 1]}, col);
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      t[i][2 * jp] = col[i][0];
      t[i][2 * jp + 1] = col[i][1];
    }
  }
#pragma unroll
  for (int ip = 0; ip < 3; ++ip) {
    floatx2 row[6];
    a6(floatx2{t[2 * ip][0], t[2 * ip + 1][0]}, floatx2{t[2 * ip][1], t[2 * ip + 1][1]},
       floatx2{t[2 * ip][2], t[2 * ip + 1][2]}, floatx2{t[2 * ip][3], t[2 * ip + 1][3]}, row);
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      m[2 * ip * 6 + j] = row[j][0];
      m[(2 * ip + 1) * 6 + j] = row[j][1];
    }
  }
}

// M' into the lane's 36 contiguous LDS floats.
__device__ __forceinline__ void f4_dy_transform_store(const float (&g)[16], float* mdst) {
  float m[kP];
  f4_dy_transform(g, m);
#pragma unroll
  for (int q = 0; q < kP / 4; ++q)
    reinterpret_cast<floatx4*>(mdst)[q] = floatx4{m[4 * q], m[4 * q + 1], m[4 * q + 2], m[4 * q + 3]};
}

// G^T of one 6-vector: 3 outputs.
__device__ __forceinline__ void gt6(const float (&u)[6], float (&w)[3]) {
  const float a = u[1] + u[2], b = u[3] + u[4];
  w[0] = 0.25f * u[0] - a * (1.f / 6.f) + b * (1.f / 24.f);
  w[1] = (u[2] - u[1]) * (1.f / 6.f) + (u[3] - u[4]) * (1.f / 12.f);
  w[2] = (b - a) * (1.f / 6.f) + u[5];
}

constexpr int kWgThreads = 512;

// dW[k][c] = G^T dU G for the lane's column c and rows kbase + r of its 36 accumulators.
// accum: add into the existing gradient (gradient-accumulation fusion, ops/gradacc.py).
__device__ __forceinline__ void f4_wgrad_epilogue(const floatx4 (&acc)[kP], float* __restrict__ out,
                                                  int c, int kbase, int C, int K, bool accum) {
  if (c >= C) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int k = kbase + r;
    if (k >= K) continue;
    float t[3][6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      float u[6], w3[3];
#pragma unroll
      for (int i = 0; i < 6; ++i) u[i] = acc[i * 6 + j][r];
      gt6(u, w3);
#pragma unroll
      for (int a = 0; a < 3; ++a) t[a][j] = w3[a];
    }
    float* o = out + (static_cast<int64_t>(k) * C + c) * 9;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      float w3[3];
      gt6(t[a], w3);
#pragma unroll
      for (int e = 0; e < 3; ++e) o[a * 3 + e] = accum ? o[a * 3 + e] + w3[e] : w3[e];
    }
  }
}

// ---- non-fused weight gradient (variant 1) ----------------------------------------------
// Both operands transformed by their own passes into the GEMM's per-step LDS images:
//   Vx[P/4][C/32][4 t][32 c][36] = B^T d B     M[P/4][K/64][4 og][4 t][16 k][36] = A dY A^T
// then a GEMM whose eight waves copy 54 KiB per step by LDS-DMA and only multiply.

// One thread per (channel, tile) of the padded grid; consecutive threads: consecutive tiles.
__global__ __launch_bounds__(256) void f4_wg_vx_kernel(const float* __restrict__ x,
                                                      float* __restrict__ vx, int N, int C,
                                                      int H, int W, int TH, int TW, int Ppad,
                                                      int cblocks, int64_t total,
                                                      uint32_t x_bytes) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int t = static_cast<int>(idx % Ppad);
  const int ch = static_cast<int>(idx / Ppad);
  float* dst = vx + ((((static_cast<int64_t>(t >> 2) * cblocks + (ch >> 5)) * 4 + (t & 3)) * 32) +
                     (ch & 31)) * kP;
  F4TileCursor cur;
  const int tpi = TH * TW;
  cur.n = t / tpi;
  const int rem = t - cur.n * tpi;
  cur.ty = rem / TW;
  cur.tx = rem - cur.ty * TW;
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), static_cast<short>(0),
                                        static_cast<int>(x_bytes), 0x00020000);
  F4Patch p;
  f4_patch_offsets(p, cur, ch, N, C, H, W);  // zeros past N or C
  f4_load_patch<false>(p, xr, 0);
  f4_transform_store(p, dst);
}

template <bool kVec>
__global__ __launch_bounds__(256) void f4_wg_mdy_kernel(const float* __restrict__ dy,
                                                       float* __restrict__ m, int N, int K,
                                                       int H, int W, int TH, int TW, int Ppad,
                                                       int kblocks, int64_t total,
                                                       uint32_t dy_bytes) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int t = static_cast<int>(idx % Ppad);
  const int k = static_cast<int>(idx / Ppad);
  // [s][kb][og][t4][k16][36]
  float* dst = m + ((((static_cast<int64_t>(t >> 2) * kblocks + (k >> 6)) * 4 + ((k >> 4) & 3)) * 4 +
                     (t & 3)) * 16 + (k & 15)) * kP;
  F4TileCursor cur;
  const int tpi = TH * TW;
  cur.n = t / tpi;
  const int rem = t - cur.n * tpi;
  cur.ty = rem / TW;
  cur.tx = rem - cur.ty * TW;
  const __amdgpu_buffer_rsrc_t dyr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dy), static_cast<short>(0),
                                        static_cast<int>(dy_bytes), 0x00020000);
  float g[16];
  f4_load_dy<kVec>(g, dyr, cur, k, N, K, H, W);
  f4_dy_transform_store(g, dst);
}

template <int kAhead = 2>
__global__ __launch_bounds__(kWgThreads, 1) void f4_wgrad_gemm_kernel(
    const float* __restrict__ vx, const float* __restrict__ m, float* __restrict__ dw, int C,
    int K, int nsteps, int cblocks, int kblocks, int splits, bool accum) {
  using Cfg = F4Cfg<4>;
  constexpr int kBuf = Cfg::kBuf;
  constexpr int kMPieces = Cfg::kUImg / 256;  // 36
  constexpr int kPieces = kBuf / 256;          // 54
  constexpr int kWaves = kWgThreads / 64;
  __shared__ float lds[2 * kBuf];

  const int nwg = cblocks * kblocks * splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7;
  const int qq = nwg >> 3, rr = nwg & 7;
  const int wgid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int cb = wgid % cblocks;
  const int kb = (wgid / cblocks) % kblocks;
  const int z = wgid / (cblocks * kblocks);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wo = wave & 3;
  const int wt = wave >> 2;
  const int s_begin = static_cast<int>(static_cast<int64_t>(z) * nsteps / splits);
  const int s_end = static_cast<int>(static_cast<int64_t>(z + 1) * nsteps / splits);
  floatx4 acc[kP];
#pragma unroll
  for (int i = 0; i < kP; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int step, float* dst) {
    const float* msrc = m + (static_cast<int64_t>(step) * kblocks + kb) * Cfg::kUImg;
    const float* vsrc = vx + (static_cast<int64_t>(step) * cblocks + cb) * kVImg;
#pragma unroll
    for (int i = 0; i < (kPieces + kWaves - 1) / kWaves; ++i) {
      const int piece = i * kWaves + wave;
      if (piece < kPieces) {
        const float* src = piece < kMPieces ? msrc + piece * 256 : vsrc + (piece - kMPieces) * 256;
        __builtin_amdgcn_global_load_lds((glob_void_t*)(src + lane * 4),
                                         (lds_void_t*)(dst + piece * 256), 16, 0, 0);
      }
    }
  };
  issue(s_begin, lds);
  __syncthreads();
  for (int s = s_begin; s < s_end; ++s) {
    const int buf = (s - s_begin) & 1;
    if (s + 1 < s_end) issue(s + 1, lds + (buf ^ 1) * kBuf);
    f4_mfma_ahead<Cfg, kAhead>(acc, lds + buf * kBuf, lane, wo, wt);
    __syncthreads();
  }
  f4_wgrad_epilogue(acc, dw + static_cast<int64_t>(z) * K * C * 9, cb * 32 + wt * 16 + (lane & 15),
                    kb * 64 + wo * 16 + 4 * (lane >> 4), C, K, accum);
}



template <bool kVec>
__global__ __launch_bounds__(kWgThreads, 1) void f4_wgrad_kernel(
    const float* __restrict__ x, const float* __restrict__ dy, float* __restrict__ dw, int N,
    int C, int K, int H, int W, int TH, int TW, int P, int cblocks, int kblocks, int splits,
    uint32_t x_bytes, uint32_t dy_bytes, bool accum) {
  using Cfg = F4Cfg<4>;
  constexpr int kBuf = Cfg::kBuf;
  __shared__ float lds[2 * kBuf];  // [buffer][M' 64k x 4t x 36 | V 4t x 32c x 36]: 108 KiB

  const int nwg = cblocks * kblocks * splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7;
  const int qq = nwg >> 3, rr = nwg & 7;
  const int wgid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int cb = wgid % cblocks;
  const int kb = (wgid / cblocks) % kblocks;
  const int z = wgid / (cblocks * kblocks);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wo = wave & 3;   // 16 k rows
  const int wt = wave >> 2;  // 16 c columns
  const int c0 = cb * 32;
  const int k0 = kb * 64;

  const int nsteps = (P + 3) / 4;
  const int s_begin = static_cast<int>(static_cast<int64_t>(z) * nsteps / splits);
  const int s_end = static_cast<int>(static_cast<int64_t>(z + 1) * nsteps / splits);
  floatx4 acc[kP];
#pragma unroll
  for (int i = 0; i < kP; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};

  // staging lane's tile cursor: tile 4*s_begin + (lane >> 4)
  F4TileCursor cur;
  {
    const int t = 4 * s_begin + (lane >> 4);
    const int tpi = TH * TW;
    cur.n = t / tpi;
    const int rem = t - cur.n * tpi;
    cur.ty = rem / TW;
    cur.tx = rem - cur.ty * TW;
  }
  const bool dy_wave = (wave & 2) != 0;  // waves 2, 3, 6, 7

  if (wave < 2) {
    // -- input patches: channel c0 + 16*wave + (lane & 15), tile (lane >> 4) of the step --
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), static_cast<short>(0),
                                          static_cast<int>(x_bytes), 0x00020000);
    const int ch = c0 + 16 * wave + (lane & 15);
    float* vmine = lds + Cfg::kUImg + ((lane >> 4) * kT + 16 * wave + (lane & 15)) * kP;
    F4Patch p;
    f4_patch_offsets(p, cur, ch, N, C, H, W);
    f4_load_patch<kVec>(p, xr, 0);
    f4_transform_store(p, vmine);
    __syncthreads();
    f4_cursor_advance(cur, TH, TW);
    f4_patch_offsets(p, cur, ch, N, C, H, W);
    f4_load_patch<kVec>(p, xr, 0);
    for (int s = s_begin; s < s_end; ++s) {
      const int buf = (s - s_begin) & 1;
      f4_transform_store(p, vmine + (buf ^ 1) * kBuf);
      __builtin_amdgcn_sched_barrier(0);
      // the step after next (past the split's end: staged, never read)
      f4_cursor_advance(cur, TH, TW);
      f4_patch_offsets(p, cur, ch, N, C, H, W);
      f4_load_patch<kVec>(p, xr, 0);
      __builtin_amdgcn_sched_barrier(0);
      f4_mfma<Cfg>(acc, lds + buf * kBuf, lane, wo, wt);
      __syncthreads();
    }
  } else if (dy_wave) {
    // -- gradient tiles: channel k0 + 16*d + (lane & 15), tile (lane >> 4) of the step --
    const __amdgpu_buffer_rsrc_t dyr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dy), static_cast<short>(0),
                                          static_cast<int>(dy_bytes), 0x00020000);
    const int d = (wave & 1) | ((wave >> 2) << 1);
    const int k = k0 + 16 * d + (lane & 15);
    float* mmine = lds + ((d * kC + (lane >> 4)) * 16 + (lane & 15)) * kP;
    float g[16];
    f4_load_dy<kVec>(g, dyr, cur, k, N, K, H, W);
    f4_dy_transform_store(g, mmine);
    __syncthreads();
    f4_cursor_advance(cur, TH, TW);
    f4_load_dy<kVec>(g, dyr, cur, k, N, K, H, W);
    for (int s = s_begin; s < s_end; ++s) {
      const int buf = (s - s_begin) & 1;
      f4_dy_transform_store(g, mmine + (buf ^ 1) * kBuf);
      __builtin_amdgcn_sched_barrier(0);
      f4_cursor_advance(cur, TH, TW);
      f4_load_dy<kVec>(g, dyr, cur, k, N, K, H, W);
      __builtin_amdgcn_sched_barrier(0);
      f4_mfma<Cfg>(acc, lds + buf * kBuf, lane, wo, wt);
      __syncthreads();
    }
  } else {
    __syncthreads();
    for (int s = s_begin; s < s_end; ++s) {
      const int buf = (s - s_begin) & 1;
      f4_mfma<Cfg>(acc, lds + buf * kBuf, lane, wo, wt);
      __syncthreads();
    }
  }

  // -- dW = G^T dU G; lane holds c = c0 + wt*16 + (lane & 15), k = k0 + wo*16 + 4(lane>>4) + r
  f4_wgrad_epilogue(acc, dw + static_cast<int64_t>(z) * K * C * 9, c0 + wt * 16 + (lane & 15),
                    k0 + wo * 16 + 4 * (lane >> 4), C, K, accum);
}

// ---- batched-GEMM Winograd: transform passes + 36 independent MFMA GEMMs ----------------
//
// The fused kernels above keep all 36 positions of a 64-channel x 32-tile block in
// registers so the output transform can run in the epilogue; per 4-channel step they
// move 54 KiB through LDS for 0.59 MFLOP (11 FLOP/byte).  On the deep, low-resolution
// U-Net levels (512-2048 channels at 6-24 pixels, 16 images per micro-batch) that made
// f4_gemm_kernel 61 % of a pipeline stage's device time at ~40 % of the matrix peak
// (profiles/r3).  Here the 36 positions are independent GEMMs
//     M[b][o][t] = sum_c U[b][c][o] V[b][c][t]          (b = 0..35)
// run as one batched launch with 128 x BN output tiles (32 FLOP/byte at BN = 128), the
// products written to HBM, and the output transform (A^T M A, + bias) a separate pass that
// also sums split-K slabs.  The weights U are transformed once per step (cached) and the
// input V by its own pass, both straight into the GEMM's per-step LDS image:
//     X[b][step][row][16]   row = output channel (U) or tile (V), 16 reduction values
// with the 16 values of a row permuted (bg_slot) so that the lane of MFMA k-group q reads
// its four k sub-steps as one float4, and the 16 lanes of each ds_read_b128 bank group hit
// 64 distinct banks.  A step's tile is then one contiguous block in memory, copied by
// LDS-DMA (global_load_lds_dwordx4) into a three-stage ring.

// position of reduction index k (0..15 within a step) in the 16 floats of row r
__device__ __forceinline__ int bg_quad(int q, int r) {
  // quad order per 4-row group: [0, 2, 3, 1] (see the bank argument above)
  constexpr int kTbl = 0 | (2 << 2) | (3 << 4) | (1 << 6);
  return q ^ ((kTbl >> (((r >> 2) & 3) * 2)) & 3);
}
__device__ __forceinline__ int bg_slot(int k, int r) { return (bg_quad(k & 3, r) << 2) | (k >> 2); }

// U[b][step][Mp][16] = G g G^T of (output channel m, reduction channel step*16 + k).
__global__ __launch_bounds__(256) void bg_weight_f4_kernel(const float* __restrict__ w,
                                                          float* __restrict__ a, int O, int R,
                                                          int Mp, int ksteps, bool flip) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= static_cast<int64_t>(ksteps) * 16 * Mp) return;
  const int k = static_cast<int>(idx & 15);
  const int64_t rest = idx >> 4;
  const int m = static_cast<int>(rest % Mp);
  const int st = static_cast<int>(rest / Mp);
  float v[kP];
  f4_weight_tile(w, O, R, m, st * 16 + k, flip, v);
  const int64_t plane = static_cast<int64_t>(ksteps) * Mp * 16;
  float* dst = a + (static_cast<int64_t>(st) * Mp + m) * 16 + bg_slot(k, m);
#pragma unroll
  for (int b = 0; b < kP; ++b) dst[b * plane] = v[b];
}

// V[b][step][Np][16] = B^T d B of (tile t, channel step*16 + k); zeros in the padding.
// A thread transforms the four channels k = q, q+4, q+8, q+12 of a step (q = 0..3) for one
// tile: bg_slot puts those four at consecutive floats, so each position is one 16-byte
// store, and a wave (16 tiles x 4 q) writes 1 KiB contiguous per position.  The pass is
// bandwidth-bound (it writes 2.25x the input), so the store width is what matters.
template <bool kVec>
__global__ __launch_bounds__(256) void bg_input_f4_kernel(const float* __restrict__ x,
                                                         float* __restrict__ v, int R, int H,
                                                         int W, int TW, int tpi, int P, int Np,
                                                         int ksteps, uint32_t x_bytes) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= static_cast<int64_t>(ksteps) * 4 * Np) return;
  const int q = static_cast<int>(idx & 3);
  const int64_t rest = idx >> 2;
  const int t = static_cast<int>(rest % Np);
  const int st = static_cast<int>(rest / Np);
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), static_cast<short>(0),
                                        static_cast<int>(x_bytes), 0x00020000);
  const int64_t plane = static_cast<int64_t>(ksteps) * Np * 16;
  float* dst = v + (static_cast<int64_t>(st) * Np + t) * 16 + (bg_quad(q, t) << 2);
  float out[4][kP];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = st * 16 + q + 4 * e;
    F4Patch p;
    if (t < P && c < R) {
      f4_fwd_offsets(p, t, c, P, tpi, TW, R, H, W);
      f4_load_patch<kVec>(p, xr, 0);
      f4_transform(p);
    } else {
#pragma unroll
      for (int b = 0; b < kP; ++b) p.d[b] = 0.f;
    }
#pragma unroll
    for (int b = 0; b < kP; ++b) out[e][b] = p.d[b];
  }
#pragma unroll
  for (int b = 0; b < kP; ++b)
    *reinterpret_cast<floatx4*>(dst + b * plane) = floatx4{out[0][b], out[1][b], out[2][b], out[3][b]};
}

template <int N>
__device__ __forceinline__ void bg_wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 7) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 9) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
  else if constexpr (N == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else if constexpr (N == 11) asm volatile("s_waitcnt vmcnt(11)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (N == 13) asm volatile("s_waitcnt vmcnt(13)" ::: "memory");
  else if constexpr (N == 14) asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
  else if constexpr (N == 15) asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
}

// C[z][b][Mp][Np] = sum over the split's steps of A[b]^T B[b].  Workgroup: kWaves waves, a
// (32 kWaves) x BN tile; wave w owns rows 32w..32w+31 (two 16-row MFMA blocks) and all BN
// columns, i.e. 2 x BN/16 accumulator tiles of v_mfma_f32_16x16x4f32.  A pipeline stage is
// kSub 16-deep steps: per stage and wave kSub (2 + BN/16) ds_read_b128 and 8 kSub BN/16
// MFMAs, one barrier, and the stage's kSub (BM + BN) x 64 B arriving by LDS-DMA into a
// three-slot ring two stages ahead.  The fragments of stage st+1 are read while stage st's
// MFMAs run.  (256-row tiles of 8 waves move fewer bytes per FLOP but ran slower on every
// U-Net shape: profiles/r3/bg_bench.json.)
template <int kWaves, int BN, int kSub>
__global__ __launch_bounds__(64 * kWaves, 512 / (64 * kWaves)) void bg_gemm_kernel(
    const float* __restrict__ a, const float* __restrict__ bmat, float* __restrict__ c, int Mp,
    int Np, int ksteps, int mtiles, int ntiles, int batch, int splits) {
  constexpr int BM = 32 * kWaves;
  constexpr int kA = BM * 16, kB = BN * 16, kSubStage = kA + kB, kStage = kSub * kSubStage;
  constexpr int kSubPieces = kSubStage / 256;  // 1 KiB LDS-DMA pieces per step
  constexpr int kPieces = kSub * kSubPieces;
  constexpr int kAPieces = kA / 256;
  constexpr int kNJ = BN / 16;
  constexpr int kPer = (kPieces + kWaves - 1) / kWaves;
  static_assert(BN % 16 == 0 && kSubStage % 256 == 0 && kPer <= 8, "tile shape");
  __shared__ float lds[3 * kStage];

  const int nwg = ntiles * mtiles * batch * splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7;
  const int qq = nwg >> 3, rr = nwg & 7;
  // consecutive work ids (same A tile, consecutive N tiles) on one XCD: one L2 serves them
  int wid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int nt = wid % ntiles;
  wid /= ntiles;
  const int mt = wid % mtiles;
  wid /= mtiles;
  const int bb = wid % batch;
  const int z = wid / batch;

  const int tid = threadIdx.x;
  // wave-uniform in a scalar register: the DMA issue and counted waits below then branch
  // on SCC instead of running every path under an exec mask
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int64_t astep = static_cast<int64_t>(Mp) * 16, bstep = static_cast<int64_t>(Np) * 16;
  const float* abase = a + static_cast<int64_t>(bb) * ksteps * astep + static_cast<int64_t>(mt) * kA;
  const float* bbase = bmat + static_cast<int64_t>(bb) * ksteps * bstep + static_cast<int64_t>(nt) * kB;
  // stages of kSub steps (ksteps is a multiple of 2: the transforms pad to 32 channels)
  const int nstages = ksteps / kSub;
  const int s0 = static_cast<int>(static_cast<int64_t>(z) * nstages / splits);
  const int s1 = static_cast<int>(static_cast<int64_t>(z + 1) * nstages / splits);

  auto issue = [&](int sg, int buf) {
    float* dst = lds + buf * kStage;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int piece = i * kWaves + wave;
      if (piece < kPieces) {
        const int sub = piece / kSubPieces;
        const int pc = piece - sub * kSubPieces;
        const int st = sg * kSub + sub;
        const float* src = pc < kAPieces ? abase + st * astep + pc * 256
                                         : bbase + st * bstep + (pc - kAPieces) * 256;
        __builtin_amdgcn_global_load_lds((glob_void_t*)(src + lane * 4),
                                         (lds_void_t*)(dst + piece * 256), 16, 0, 0);
      }
    }
  };
  // this wave's pieces per stage: waiting for vmcnt <= k * mine leaves the last k issued
  // stages in flight
  const int mine = (kPieces - wave + kWaves - 1) / kWaves;
  auto wait_stages_in_flight = [&](int k) {
    switch (k * mine) {
      case 0: bg_wait_vm<0>(); break;
      case 1: bg_wait_vm<1>(); break;
      case 2: bg_wait_vm<2>(); break;
      case 3: bg_wait_vm<3>(); break;
      case 4: bg_wait_vm<4>(); break;
      case 5: bg_wait_vm<5>(); break;
      case 6: bg_wait_vm<6>(); break;
      case 7: bg_wait_vm<7>(); break;
      case 8: bg_wait_vm<8>(); break;
      case 9: bg_wait_vm<9>(); break;
      case 10: bg_wait_vm<10>(); break;
      case 11: bg_wait_vm<11>(); break;
      case 12: bg_wait_vm<12>(); break;
      case 13: bg_wait_vm<13>(); break;
      case 14: bg_wait_vm<14>(); break;
      case 15: bg_wait_vm<15>(); break;
      default: bg_wait_vm<16>(); break;
    }
  };

  floatx4 acc[2][kNJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < kNJ; ++jj) acc[i][jj] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int q = lane >> 4, j = lane & 15;
  int aoff[2], boff[kNJ];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = wave * 32 + i * 16 + j;
    aoff[i] = row * 16 + (bg_quad(q, row) << 2);
  }
#pragma unroll
  for (int jj = 0; jj < kNJ; ++jj) {
    const int row = jj * 16 + j;
    boff[jj] = kA + row * 16 + (bg_quad(q, row) << 2);
  }
  floatx4 af[kSub][2], bf[kSub][kNJ];
  auto fetch = [&](int buf) {
    const float* base = lds + buf * kStage;
#pragma unroll
    for (int u = 0; u < kSub; ++u) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[u][i] = *reinterpret_cast<const floatx4*>(base + u * kSubStage + aoff[i]);
#pragma unroll
      for (int jj = 0; jj < kNJ; ++jj)
        bf[u][jj] = *reinterpret_cast<const floatx4*>(base + u * kSubStage + boff[jj]);
    }
  };

  // Software pipeline over the three-slot ring: at stage k the fragments of k are already
  // in registers (read during stage k-1); after one barrier (stage k+1 landed, every wave
  // done reading slot k) the wave issues stage k+3's DMA into slot k, reads stage k+1's
  // fragments and runs stage k's MFMAs while those reads return.
  const int nst = s1 - s0;
  if (nst > 0) {
    issue(s0, 0);
    if (nst > 1) issue(s0 + 1, 1);
    if (nst > 2) issue(s0 + 2, 2);
    wait_stages_in_flight(nst > 2 ? 2 : nst - 1);
    __builtin_amdgcn_s_barrier();
    fetch(0);
  }
  int buf = 0;
  for (int k = 0; k < nst; ++k) {
    floatx4 ac[kSub][2], bc[kSub][kNJ];
#pragma unroll
    for (int u = 0; u < kSub; ++u) {
#pragma unroll
      for (int i = 0; i < 2; ++i) ac[u][i] = af[u][i];
#pragma unroll
      for (int jj = 0; jj < kNJ; ++jj) bc[u][jj] = bf[u][jj];
    }
    const int nb = buf == 2 ? 0 : buf + 1;
    if (k + 1 < nst) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this slot's reads are done
      wait_stages_in_flight(k + 2 < nst ? 1 : 0);          // stage k+1 landed
      __builtin_amdgcn_s_barrier();
      if (k + 3 < nst) issue(s0 + k + 3, buf);
      fetch(nb);
    }
#pragma unroll
    for (int u = 0; u < kSub; ++u)
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
#pragma unroll
        for (int jj = 0; jj < kNJ; ++jj)
#pragma unroll
          for (int i = 0; i < 2; ++i)
            acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[u][i][kk], bc[u][jj][kk],
                                                             acc[i][jj], 0, 0, 0);
    buf = nb;
  }

  float* cz = c + (static_cast<int64_t>(z) * batch + bb) * Mp * Np;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m0 = mt * BM + wave * 32 + i * 16 + 4 * q;
#pragma unroll
    for (int jj = 0; jj < kNJ; ++jj) {
      const int n = nt * BN + jj * 16 + j;
#pragma unroll
      for (int r = 0; r < 4; ++r) cz[static_cast<int64_t>(m0 + r) * Np + n] = acc[i][jj][r];
    }
  }
}

// ---- split-bf16 batched GEMM (EMU) -------------------------------------------------------
// The same 36 / 16 GEMMs on the bf16 matrix pipes, fp32-accurate: every transformed operand
// value v is stored as three bf16 hi + mid + lo == v (exact: round-to-nearest splits, 8
// significant bits each), and a product of two values as the six partial products that
// matter (hi.hi, hi.mid, mid.hi, mid.mid, hi.lo, lo.hi -- the three left out are below
// 2^-24 of it, under one f32 rounding), each exact, accumulated in f32 by
// v_mfma_f32_32x32x16_bf16 at 16x the f32 MFMA's rate: 3/8 of the f32 matrix time.
// (conv_gemm.hip's EMU tile configurations use the same split.)  The transforms write the
// split once per value, so the GEMM moves 1.5x the bytes but does no conversion work.
//
// Operand image (bf16): X[pos][step][plane p][half h][rows][8]: the 16-byte chunk
// (p, h, row) holds plane p of reduction values 8h .. 8h+7 of that row, i.e. exactly the
// fragment lane (row, h) of a 32x32x16 MFMA reads -- 32 consecutive rows are 512 contiguous
// bytes for one ds_read_b128 (conflict-free), and a step's tile is 6 contiguous runs of
// rows in global memory, copied by LDS-DMA.
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void bg_split3(const floatx4& v, bf16x4& hi, bf16x4& mid, bf16x4& lo) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const __bf16 h = static_cast<__bf16>(v[e]);
    const float r = v[e] - static_cast<float>(h);
    const __bf16 m = static_cast<__bf16>(r);
    hi[e] = h;
    mid[e] = m;
    lo[e] = static_cast<__bf16>(r - static_cast<float>(m));
  }
}

// Four consecutive reduction values k = 4g .. 4g+3 of one row at every position: one 8-byte
// store per (position, plane).  `rows` = Mp or Np.
template <int NPOS>
__device__ __forceinline__ void bg_emu_store(float* out, const float (&v)[4][NPOS], int st, int row,
                                             int g, int rows, int ksteps) {
  __bf16* base = reinterpret_cast<__bf16*>(out);
  const int64_t pstride = static_cast<int64_t>(rows) * 8;  // one (plane, half) run
  const int64_t off = (static_cast<int64_t>(st) * 6 + (g >> 1)) * pstride +
                      static_cast<int64_t>(row) * 8 + 4 * (g & 1);
  const int64_t pos_stride = static_cast<int64_t>(ksteps) * 6 * pstride;
#pragma unroll
  for (int b = 0; b < NPOS; ++b) {
    bf16x4 hi, mid, lo;
    bg_split3(floatx4{v[0][b], v[1][b], v[2][b], v[3][b]}, hi, mid, lo);
    __bf16* dst = base + b * pos_stride + off;
    *reinterpret_cast<bf16x4*>(dst) = hi;
    *reinterpret_cast<bf16x4*>(dst + 2 * pstride) = mid;
    *reinterpret_cast<bf16x4*>(dst + 4 * pstride) = lo;
  }
}

// CPT (1 / 2 / 4) consecutive reduction values k = q*CPT .. of one row at every position:
// one 2 / 4 / 8-byte store per (position, plane) -- the input images of small tile counts
// run 2-4x as many threads as the 4-value stores allow (see launch_bg_conv).
template <int NPOS, int CPT>
__device__ __forceinline__ void bg_emu_store_n(float* out, const float (&v)[CPT][NPOS], int st,
                                               int row, int q, int rows, int ksteps) {
  if constexpr (CPT == 4) {
    bg_emu_store<NPOS>(out, v, st, row, q, rows, ksteps);
  } else {
    __bf16* base = reinterpret_cast<__bf16*>(out);
    const int k0 = q * CPT, g = k0 >> 2;
    const int64_t pstride = static_cast<int64_t>(rows) * 8;
    const int64_t off = (static_cast<int64_t>(st) * 6 + (g >> 1)) * pstride +
                        static_cast<int64_t>(row) * 8 + 4 * (g & 1) + (k0 & 3);
    const int64_t pos_stride = static_cast<int64_t>(ksteps) * 6 * pstride;
#pragma unroll
    for (int b = 0; b < NPOS; ++b) {
      __bf16 pl[3][CPT];
#pragma unroll
      for (int e = 0; e < CPT; ++e) {  // bg_split3's arithmetic, element by element
        const __bf16 h = static_cast<__bf16>(v[e][b]);
        const float r = v[e][b] - static_cast<float>(h);
        const __bf16 m = static_cast<__bf16>(r);
        pl[0][e] = h;
        pl[1][e] = m;
        pl[2][e] = static_cast<__bf16>(r - static_cast<float>(m));
      }
      __bf16* dst = base + b * pos_stride + off;
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        if constexpr (CPT == 2) {
          typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
          *reinterpret_cast<bf16x2_t*>(dst + 2 * p * pstride) = bf16x2_t{pl[p][0], pl[p][1]};
        } else {
          dst[2 * p * pstride] = pl[p][0];
        }
      }
    }
  }
}

// U (EMU image) of (output channel m, reduction channels st*16 + 4g .. +3).
__global__ __launch_bounds__(256) void bg_weight_f4_emu_kernel(const float* __restrict__ w,
                                                              float* __restrict__ a, int O, int R,
                                                              int Mp, int ksteps, bool flip) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= static_cast<int64_t>(ksteps) * 4 * Mp) return;
  const int g = static_cast<int>(idx & 3);
  const int64_t rest = idx >> 2;
  const int m = static_cast<int>(rest % Mp);
  const int st = static_cast<int>(rest / Mp);
  float v[4][kP];
#pragma unroll
  for (int e = 0; e < 4; ++e) f4_weight_tile(w, O, R, m, st * 16 + 4 * g + e, flip, v[e]);
  bg_emu_store<kP>(a, v, st, m, g, Mp, ksteps);
}

// V (EMU image) of (tile t, channels st*16 + CPT*q .. +CPT-1); zeros in the padding.
template <bool kVec, int CPT>
__global__ __launch_bounds__(256) void bg_input_f4_emu_kernel(const float* __restrict__ x,
                                                             float* __restrict__ v, int R, int H,
                                                             int W, int TW, int tpi, int P, int Np,
                                                             int ksteps, uint32_t x_bytes) {
  constexpr int kQ = 16 / CPT;  // threads per (tile, step)
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= static_cast<int64_t>(ksteps) * kQ * Np) return;
  const int g = static_cast<int>(idx % kQ);
  const int64_t rest = idx / kQ;
  const int t = static_cast<int>(rest % Np);
  const int st = static_cast<int>(rest / Np);
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), static_cast<short>(0),
                                        static_cast<int>(x_bytes), 0x00020000);
  float out[CPT][kP];
#pragma unroll
  for (int e = 0; e < CPT; ++e) {
    const int c = st * 16 + CPT * g + e;
    F4Patch p;
    if (t < P && c < R) {
      f4_fwd_offsets(p, t, c, P, tpi, TW, R, H, W);
      f4_load_patch<kVec>(p, xr, 0);
      f4_transform(p);
    } else {
#pragma unroll
      for (int b = 0; b < kP; ++b) p.d[b] = 0.f;
    }
#pragma unroll
    for (int b = 0; b < kP; ++b) out[e][b] = p.d[b];
  }
  bg_emu_store_n<kP, CPT>(v, out, st, t, g, Np, ksteps);
}

// C[z][b][Mp][Np] = sum over the split's steps of A[b]^T B[b] on split-bf16 operands.
// Four waves, a 128 x BN tile (BN = 64 / 96 / 128): wave w owns rows 32w .. 32w+31 and all
// BN columns as BN/32 tiles of v_mfma_f32_32x32x16_bf16, six MFMAs per tile and 16-deep
// step.  A step's (128 + BN) x 96 bytes arrive by LDS-DMA (1 KiB pieces) into a three-slot
// ring two steps ahead; the fragments of step k+1 are read while step k's MFMAs run.
template <int BN>
__global__ __launch_bounds__(256, 2) void bg_gemm_emu_kernel(
    const float* __restrict__ a, const float* __restrict__ bmat, float* __restrict__ c, int Mp,
    int Np, int ksteps, int mtiles, int ntiles, int batch, int splits) {
  constexpr int kWaves = 4, BM = 128;
  constexpr int kABytes = 96 * BM, kBBytes = 96 * BN, kStage = kABytes + kBBytes;
  constexpr int kAPieces = kABytes / 1024, kPieces = kStage / 1024;
  constexpr int kPer = (kPieces + kWaves - 1) / kWaves;
  constexpr int kNT = BN / 32;
  static_assert(BN % 32 == 0 && (96 * BN) % 1024 == 0 && kPer <= 8, "tile shape");
  __shared__ __attribute__((aligned(16))) char lds[3 * kStage];

  const int nwg = ntiles * mtiles * batch * splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7;
  const int qq = nwg >> 3, rr = nwg & 7;
  // consecutive work ids (same A tile, consecutive N tiles) on one XCD: one L2 serves them
  int wid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int nt = wid % ntiles;
  wid /= ntiles;
  const int mt = wid % mtiles;
  wid /= mtiles;
  const int bb = wid % batch;
  const int z = wid / batch;

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int64_t astep = static_cast<int64_t>(Mp) * 96, bstep = static_cast<int64_t>(Np) * 96;
  const char* abase = reinterpret_cast<const char*>(a) + static_cast<int64_t>(bb) * ksteps * astep;
  const char* bbase =
      reinterpret_cast<const char*>(bmat) + static_cast<int64_t>(bb) * ksteps * bstep;
  const int s0 = static_cast<int>(static_cast<int64_t>(z) * ksteps / splits);
  const int s1 = static_cast<int>(static_cast<int64_t>(z + 1) * ksteps / splits);

  // this lane's source offset (bytes, within one step) of each of its pieces
  int64_t src_off[kPer];
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int piece = i * kWaves + wave;
    src_off[i] = 0;
    if (piece < kAPieces) {
      const int f = piece * 64 + lane;  // (plane-half, row) of the A image
      const int ph = f / BM, row = f - ph * BM;
      src_off[i] = (static_cast<int64_t>(ph) * Mp + mt * BM + row) * 16;
    } else if (piece < kPieces) {
      const int f = (piece - kAPieces) * 64 + lane;
      const int ph = f / BN, row = f - ph * BN;
      src_off[i] = (static_cast<int64_t>(ph) * Np + static_cast<int64_t>(nt) * BN + row) * 16;
    }
  }
  auto issue = [&](int st, int buf) {
    char* dst = lds + buf * kStage;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int piece = i * kWaves + wave;
      if (piece < kPieces) {
        const char* src = (piece < kAPieces ? abase + st * astep : bbase + st * bstep) +
                          src_off[i];
        __builtin_amdgcn_global_load_lds((glob_void_t*)src, (lds_void_t*)(dst + piece * 1024),
                                         16, 0, 0);
      }
    }
  };
  const int mine = (kPieces - wave + kWaves - 1) / kWaves;
  auto wait_stages_in_flight = [&](int k) {
    switch (k * mine) {
      case 0: bg_wait_vm<0>(); break;
      case 1: bg_wait_vm<1>(); break;
      case 2: bg_wait_vm<2>(); break;
      case 3: bg_wait_vm<3>(); break;
      case 4: bg_wait_vm<4>(); break;
      case 5: bg_wait_vm<5>(); break;
      case 6: bg_wait_vm<6>(); break;
      case 7: bg_wait_vm<7>(); break;
      case 8: bg_wait_vm<8>(); break;
      case 9: bg_wait_vm<9>(); break;
      case 10: bg_wait_vm<10>(); break;
      case 11: bg_wait_vm<11>(); break;
      case 12: bg_wait_vm<12>(); break;
      case 13: bg_wait_vm<13>(); break;
      case 14: bg_wait_vm<14>(); break;
      case 15: bg_wait_vm<15>(); break;
      default: bg_wait_vm<16>(); break;
    }
  };

  floatx16 acc[kNT];
#pragma unroll
  for (int j = 0; j < kNT; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

  const int h = lane >> 5, l32 = lane & 31;
  // byte offsets of this lane's fragments in a slot: plane p at + p * 2 * rows * 16
  const int aoff = (h * BM + wave * 32 + l32) * 16;
  const int boff = kABytes + (h * BN + l32) * 16;
  bf16x8 af[3], bf[3][kNT];
  auto fetch = [&](int buf) {
    const char* base = lds + buf * kStage;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      af[p] = *reinterpret_cast<const bf16x8*>(base + aoff + p * 2 * BM * 16);
#pragma unroll
      for (int j = 0; j < kNT; ++j)
        bf[p][j] = *reinterpret_cast<const bf16x8*>(base + boff + p * 2 * BN * 16 + j * 512);
    }
  };

  const int nst = s1 - s0;
  if (nst > 0) {
    issue(s0, 0);
    if (nst > 1) issue(s0 + 1, 1);
    if (nst > 2) issue(s0 + 2, 2);
    wait_stages_in_flight(nst > 2 ? 2 : nst - 1);
    __builtin_amdgcn_s_barrier();
    fetch(0);
  }
  constexpr int kPairs[6][2] = {{2, 0}, {0, 2}, {1, 1}, {1, 0}, {0, 1}, {0, 0}};
  int buf = 0;
  for (int k = 0; k < nst; ++k) {
    bf16x8 ac[3], bc[3][kNT];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      ac[p] = af[p];
#pragma unroll
      for (int j = 0; j < kNT; ++j) bc[p][j] = bf[p][j];
    }
    const int nb = buf == 2 ? 0 : buf + 1;
    if (k + 1 < nst) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this slot's reads are done
      wait_stages_in_flight(k + 2 < nst ? 1 : 0);          // step k+1 landed
      __builtin_amdgcn_s_barrier();
      if (k + 3 < nst) issue(s0 + k + 3, buf);
      fetch(nb);
    }
#pragma unroll
    for (int t = 0; t < 6; ++t)
#pragma unroll
      for (int j = 0; j < kNT; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ac[kPairs[t][0]], bc[kPairs[t][1]][j],
                                                         acc[j], 0, 0, 0);
    buf = nb;
  }

  float* cz = c + (static_cast<int64_t>(z) * batch + bb) * Mp * Np;
  const int m0 = mt * BM + wave * 32 + 4 * h;
#pragma unroll
  for (int j = 0; j < kNT; ++j) {
    const int64_t n = static_cast<int64_t>(nt) * BN + j * 32 + l32;
#pragma unroll
    for (int r = 0; r < 16; ++r)
      cz[static_cast<int64_t>(m0 + (r & 3) + 8 * (r >> 2)) * Np + n] = acc[j][r];
  }
}

// Y = A^T (sum_z M[z]) A (+ bias): one thread per (output channel, tile), consecutive
// threads on consecutive tiles (coalesced reads of each position's M row).
__global__ __launch_bounds__(256) void bg_output_f4_kernel(
    const float* __restrict__ cbuf, const float* __restrict__ bias, float* __restrict__ y, int O,
    int Mp, int Np, int P, int tpi, int TW, int H, int W, int splits) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= static_cast<int64_t>(O) * P) return;
  const int t = static_cast<int>(idx % P);
  const int o = static_cast<int>(idx / P);
  const int64_t pos = static_cast<int64_t>(Mp) * Np;
  const float* src = cbuf + static_cast<int64_t>(o) * Np + t;
  float m[kP];
#pragma unroll
  for (int b = 0; b < kP; ++b) m[b] = src[b * pos];
  for (int z = 1; z < splits; ++z) {
    const float* sz = src + static_cast<int64_t>(z) * kP * pos;
#pragma unroll
    for (int b = 0; b < kP; ++b) m[b] += sz[b * pos];
  }
  float s[4][6];
#pragma unroll
  for (int jc = 0; jc < 6; ++jc) {
    const float a = m[6 + jc] + m[12 + jc], bq = m[6 + jc] - m[12 + jc];
    const float cc = m[18 + jc] + m[24 + jc], d = m[18 + jc] - m[24 + jc];
    s[0][jc] = m[jc] + a + cc;
    s[1][jc] = bq + 2.f * d;
    s[2][jc] = a + 4.f * cc;
    s[3][jc] = bq + 8.f * d + m[30 + jc];
  }
  const float bv = bias ? bias[o] : 0.f;
  const int n = t / tpi;
  const int rem = t - n * tpi;
  const int ty = rem / TW;
  const int py = 4 * ty, px = 4 * (rem - ty * TW);
  float* yp = y + (static_cast<int64_t>(n) * O + o) * H * W + static_cast<int64_t>(py) * W + px;
  const bool full = (W & 3) == 0 && py + 4 <= H;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float a = s[k][1] + s[k][2], bq = s[k][1] - s[k][2];
    const float cc = s[k][3] + s[k][4], d = s[k][3] - s[k][4];
    const floatx4 out{s[k][0] + a + cc + bv, bq + 2.f * d + bv, a + 4.f * cc + bv,
                      bq + 8.f * d + s[k][5] + bv};
    if (full) {
      *reinterpret_cast<floatx4*>(yp + k * W) = out;
    } else if (py + k < H) {
#pragma unroll
      for (int l = 0; l < 4; ++l)
        if (px + l < W) yp[k * W + l] = out[l];
    }
  }
}

// ---- the same batched GEMM for F(2x2, 3x3): 16 positions, 4x4 patches, 2x2 outputs ------
// On 6x6 planes a 4x4 output tile covers 8x8 (5/9 of its multiplies wasted), so F(2x2)
// does the same matrix-core work with a transformed weight 16/36 the size: the bottom
// U-Net level's 2048 x 2048 layers read 268 MB of U per call instead of 604 MB.
constexpr int kP2 = 16;

// G g G^T of (output channel m, reduction channel r): the 16 F(2x2) positions (0 outside)
__device__ __forceinline__ void f2_weight_tile(const float* __restrict__ w, int O, int R, int m,
                                               int r, bool flip, float (&v)[kP2]) {
  float g[3][3] = {};
  if (r < R && m < O) {
    const float* src = flip ? w + (static_cast<int64_t>(r) * O + m) * 9
                            : w + (static_cast<int64_t>(m) * R + r) * 9;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int jc = 0; jc < 3; ++jc) g[i][jc] = flip ? src[(2 - i) * 3 + (2 - jc)] : src[i * 3 + jc];
  }
  // G = [[1, 0, 0], [1/2, 1/2, 1/2], [1/2, -1/2, 1/2], [0, 0, 1]]
  float t[4][3];
#pragma unroll
  for (int jc = 0; jc < 3; ++jc) {
    t[0][jc] = g[0][jc];
    t[1][jc] = 0.5f * (g[0][jc] + g[1][jc] + g[2][jc]);
    t[2][jc] = 0.5f * (g[0][jc] - g[1][jc] + g[2][jc]);
    t[3][jc] = g[2][jc];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i * 4 + 0] = t[i][0];
    v[i * 4 + 1] = 0.5f * (t[i][0] + t[i][1] + t[i][2]);
    v[i * 4 + 2] = 0.5f * (t[i][0] - t[i][1] + t[i][2]);
    v[i * 4 + 3] = t[i][2];
  }
}

// ---- split-bf16 F(4x4) weight gradient (variant 2) ----------------------------------------
// The non-fused weight gradient as one batched split-bf16 GEMM per position, on the
// batched-GEMM machinery: dU[b][k][c] = sum_t M'[b][k][t] V[b][c][t], the 36 positions b,
// output channels k as GEMM rows (A image, the gradient tiles' M' = A g A^T), input channels
// c as columns (B image, the input patches' V = B^T d B), the tiles t as the reduction in
// 16-deep steps -- the same [b][step][plane, half][rows][8] images bg_gemm_emu_kernel reads,
// with tiles where the forward has channels.  Then dW = G^T (sum of the split partials) G.

// V image of (channel row c, tiles st*16 + 4g .. +3); zeros past the tiles or channels.
template <bool kVec>
__global__ __launch_bounds__(256) void wg_x_emu_kernel(const float* __restrict__ x,
                                                      float* __restrict__ v, int C, int H, int W,
                                                      int TW, int tpi, int P, int Np, int ksteps,
                                                      uint32_t x_bytes) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= static_cast<int64_t>(ksteps) * 4 * Np) return;
  const int g = static_cast<int>(idx & 3);
  const int64_t rest = idx >> 2;
  const int c = static_cast<int>(rest % Np);
  const int st = static_cast<int>(rest / Np);
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), static_cast<short>(0),
                                        static_cast<int>(x_bytes), 0x00020000);
  float out[4][kP];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int t = st * 16 + 4 * g + e;
    F4Patch p;
    if (t < P && c < C) {
      f4_fwd_offsets(p, t, c, P, tpi, TW, C, H, W);
      f4_load_patch<kVec>(p, xr, 0);
      f4_transform(p);
    } else {
#pragma unroll
      for (int b = 0; b < kP; ++b) p.d[b] = 0.f;
    }
#pragma unroll
    for (int b = 0; b < kP; ++b) out[e][b] = p.d[b];
  }
  bg_emu_store<kP>(v, out, st, c, g, Np, ksteps);
}

// M' image of (gradient channel row k, tiles st*16 + 4g .. +3); zeros past the tiles or
// channels.
template <bool kVec>
__global__ __launch_bounds__(256) void wg_dy_emu_kernel(const float* __restrict__ dy,
                                                       float* __restrict__ m, int N, int K,
                                                       int H, int W, int TH, int TW, int Mp,
                                                       int ksteps, uint32_t dy_bytes) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= static_cast<int64_t>(ksteps) * 4 * Mp) return;
  const int g = static_cast<int>(idx & 3);
  const int64_t rest = idx >> 2;
  const int k = static_cast<int>(rest % Mp);
  const int st = static_cast<int>(rest / Mp);
  const __amdgpu_buffer_rsrc_t dyr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dy), static_cast<short>(0),
                                        static_cast<int>(dy_bytes), 0x00020000);
  const int tpi = TH * TW;
  float out[4][kP];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int t = st * 16 + 4 * g + e;
    F4TileCursor cur;
    cur.n = t / tpi;  // t past the last tile: n >= N, f4_load_dy reads zeros
    const int rem = t - cur.n * tpi;
    cur.ty = rem / TW;
    cur.tx = rem - cur.ty * TW;
    float gt[16];
    f4_load_dy<kVec>(gt, dyr, cur, k, N, K, H, W);
    f4_dy_transform(gt, out[e]);
  }
  bg_emu_store<kP>(m, out, st, k, g, Mp, ksteps);
}

// dW[k][c] (+)= G^T (sum_z dU[z][b][k][c] over b as 6x6) G: one thread per (k, c),
// consecutive threads on consecutive c (coalesced reads of each position's row).
__global__ __launch_bounds__(256) void wg_output_emu_kernel(const float* __restrict__ cbuf,
                                                           float* __restrict__ dw, int K, int C,
                                                           int Mp, int Np, int splits,
                                                           bool accum) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= static_cast<int64_t>(K) * C) return;
  const int c = static_cast<int>(idx % C);
  const int k = static_cast<int>(idx / C);
  const int64_t pos = static_cast<int64_t>(Mp) * Np;
  float u[kP];
#pragma unroll
  for (int b = 0; b < kP; ++b) {
    const float* src = cbuf + b * pos + static_cast<int64_t>(k) * Np + c;
    float acc = 0.f;
    for (int z = 0; z < splits; ++z) acc += src[static_cast<int64_t>(z) * kP * pos];
    u[b] = acc;
  }
  float t[3][6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    float col[6], w3[3];
#pragma unroll
    for (int i = 0; i < 6; ++i) col[i] = u[i * 6 + j];
    gt6(col, w3);
#pragma unroll
    for (int a = 0; a < 3; ++a) t[a][j] = w3[a];
  }
  float* o = dw + (static_cast<int64_t>(k) * C + c) * 9;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    float w3[3];
    gt6(t[a], w3);
#pragma unroll
    for (int e = 0; e < 3; ++e) o[a * 3 + e] = accum ? o[a * 3 + e] + w3[e] : w3[e];
  }
}


__global__ __launch_bounds__(256) void bg_weight_f2_kernel(const float* __restrict__ w,
                                                          float* __restrict__ a, int O, int R,
                                                          int Mp, int ksteps, bool flip) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= static_cast<int64_t>(ksteps) * 16 * Mp) return;
  const int k = static_cast<int>(idx & 15);
  const int64_t rest = idx >> 4;
  const int m = static_cast<int>(rest % Mp);
  const int st = static_cast<int>(rest / Mp);
  float v[kP2];
  f2_weight_tile(w, O, R, m, st * 16 + k, flip, v);
  const int64_t plane = static_cast<int64_t>(ksteps) * Mp * 16;
  float* dst = a + (static_cast<int64_t>(st) * Mp + m) * 16 + bg_slot(k, m);
#pragma unroll
  for (int b = 0; b < kP2; ++b) dst[b * plane] = v[b];
}

// B^T d B of (tile t, channel c): the 16 F(2x2) positions (0 in the padding)
__device__ __forceinline__ void f2_input_tile(const float* __restrict__ x, int R, int H, int W,
                                              int TW, int tpi, int P, int t, int c,
                                              float (&vv)[kP2]) {
  float d[4][4] = {};
  if (t < P && c < R) {
    const int n = t / tpi;
    const int rem = t - n * tpi;
    const int ty = rem / TW;
    const int y0 = 2 * ty - 1, x0 = 2 * (rem - ty * TW) - 1;
    const float* src = x + (static_cast<int64_t>(n) * R + c) * H * W;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int yy = y0 + i;
#pragma unroll
      for (int jc = 0; jc < 4; ++jc) {
        const int xx = x0 + jc;
        d[i][jc] = yy >= 0 && yy < H && xx >= 0 && xx < W ? src[yy * W + xx] : 0.f;
      }
    }
  }
  // B^T = [[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]]
  float e[4][4];
#pragma unroll
  for (int jc = 0; jc < 4; ++jc) {
    e[0][jc] = d[0][jc] - d[2][jc];
    e[1][jc] = d[1][jc] + d[2][jc];
    e[2][jc] = d[2][jc] - d[1][jc];
    e[3][jc] = d[1][jc] - d[3][jc];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    vv[i * 4 + 0] = e[i][0] - e[i][2];
    vv[i * 4 + 1] = e[i][1] + e[i][2];
    vv[i * 4 + 2] = e[i][2] - e[i][1];
    vv[i * 4 + 3] = e[i][1] - e[i][3];
  }
}

__global__ __launch_bounds__(256) void bg_input_f2_kernel(const float* __restrict__ x,
                                                         float* __restrict__ v, int R, int H,
                                                         int W, int TW, int tpi, int P, int Np,
                                                         int ksteps) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= static_cast<int64_t>(ksteps) * 16 * Np) return;
  const int k = static_cast<int>(idx & 15);
  const int64_t rest = idx >> 4;
  const int t = static_cast<int>(rest % Np);
  const int st = static_cast<int>(rest / Np);
  float vv[kP2];
  f2_input_tile(x, R, H, W, TW, tpi, P, t, st * 16 + k, vv);
  const int64_t plane = static_cast<int64_t>(ksteps) * Np * 16;
  float* dst = v + (static_cast<int64_t>(st) * Np + t) * 16 + bg_slot(k, t);
#pragma unroll
  for (int b = 0; b < kP2; ++b) dst[b * plane] = vv[b];
}

// F(2x2) EMU images: as bg_weight_f4_emu_kernel / bg_input_f4_emu_kernel, 16 positions.
__global__ __launch_bounds__(256) void bg_weight_f2_emu_kernel(const float* __restrict__ w,
                                                              float* __restrict__ a, int O, int R,
                                                              int Mp, int ksteps, bool flip) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= static_cast<int64_t>(ksteps) * 4 * Mp) return;
  const int g = static_cast<int>(idx & 3);
  const int64_t rest = idx >> 2;
  const int m = static_cast<int>(rest % Mp);
  const int st = static_cast<int>(rest / Mp);
  float v[4][kP2];
#pragma unroll
  for (int e = 0; e < 4; ++e) f2_weight_tile(w, O, R, m, st * 16 + 4 * g + e, flip, v[e]);
  bg_emu_store<kP2>(a, v, st, m, g, Mp, ksteps);
}

template <int CPT>
__global__ __launch_bounds__(256) void bg_input_f2_emu_kernel(const float* __restrict__ x,
                                                             float* __restrict__ v, int R, int H,
                                                             int W, int TW, int tpi, int P, int Np,
                                                             int ksteps) {
  constexpr int kQ = 16 / CPT;
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= static_cast<int64_t>(ksteps) * kQ * Np) return;
  const int g = static_cast<int>(idx % kQ);
  const int64_t rest = idx / kQ;
  const int t = static_cast<int>(rest % Np);
  const int st = static_cast<int>(rest / Np);
  float vv[CPT][kP2];
#pragma unroll
  for (int e = 0; e < CPT; ++e)
    f2_input_tile(x, R, H, W, TW, tpi, P, t, st * 16 + CPT * g + e, vv[e]);
  bg_emu_store_n<kP2, CPT>(v, vv, st, t, g, Np, ksteps);
}

__global__ __launch_bounds__(256) void bg_output_f2_kernel(
    const float* __restrict__ cbuf, const float* __restrict__ bias, float* __restrict__ y, int O,
    int Mp, int Np, int P, int tpi, int TW, int H, int W, int splits) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= static_cast<int64_t>(O) * P) return;
  const int t = static_cast<int>(idx % P);
  const int o = static_cast<int>(idx / P);
  const int64_t pos = static_cast<int64_t>(Mp) * Np;
  const float* src = cbuf + static_cast<int64_t>(o) * Np + t;
  float m[kP2];
#pragma unroll
  for (int b = 0; b < kP2; ++b) m[b] = src[b * pos];
  for (int z = 1; z < splits; ++z) {
    const float* sz = src + static_cast<int64_t>(z) * kP2 * pos;
#pragma unroll
    for (int b = 0; b < kP2; ++b) m[b] += sz[b * pos];
  }
  // A^T = [[1, 1, 1, 0], [0, 1, -1, -1]]
  float s[2][4];
#pragma unroll
  for (int jc = 0; jc < 4; ++jc) {
    s[0][jc] = m[jc] + m[4 + jc] + m[8 + jc];
    s[1][jc] = m[4 + jc] - m[8 + jc] - m[12 + jc];
  }
  const float bv = bias ? bias[o] : 0.f;
  const int n = t / tpi;
  const int rem = t - n * tpi;
  const int ty = rem / TW;
  const int py = 2 * ty, px = 2 * (rem - ty * TW);
  float* yp = y + (static_cast<int64_t>(n) * O + o) * H * W + static_cast<int64_t>(py) * W + px;
#pragma unroll
  for (int kr = 0; kr < 2; ++kr) {
    if (py + kr >= H) break;
    const float v0 = s[kr][0] + s[kr][1] + s[kr][2] + bv;
    const float v1 = s[kr][1] - s[kr][2] - s[kr][3] + bv;
    yp[kr * W] = v0;
    if (px + 1 < W) yp[kr * W + 1] = v1;
  }
}


// The output transform of the batched-GEMM Winograd with the BatchNorm statistics of its
// output in the same pass (a following bn_finalize_apply reads them instead of a
// bn_stats pass re-reading y): wave w of workgroup (x, g) owns output channel 4x + w and the
// tiles of images [g * ipg, (g + 1) * ipg); each lane writes its tiles' outputs exactly as
// bg_output_f4_kernel / bg_output_f2_kernel do, takes each tile's mean and centred M2 over
// its pixels inside the plane, Chan-merges them, and the wave merges its lanes: one
// (mean, M2) partial per (image group, channel), count ipg * H * W (fewer in the last).
__device__ __forceinline__ void chan_merge_f(float& na, float& ma, float& m2a, float nb,
                                             float mb, float m2b) {
  const float nn = na + nb;
  if (nn <= 0.f) return;
  const float d = mb - ma;
  const float f = nb / nn;
  ma += d * f;
  m2a += m2b + d * d * na * f;
  na = nn;
}

template <int TILE>
__global__ __launch_bounds__(256) void bg_output_stats_kernel(
    const float* __restrict__ cbuf, const float* __restrict__ bias, float* __restrict__ y,
    float* __restrict__ pm, float* __restrict__ pm2, int O, int Mp, int Np, int P, int tpi,
    int TW, int H, int W, int splits, int ipg) {
  constexpr int NPOS = TILE == 4 ? kP : kP2;
  const int lane = threadIdx.x & 63;
  const int o = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int g = blockIdx.y;
  if (o >= O) return;  // (whole waves: no barrier below)
  const int t0 = g * ipg * tpi;
  const int t1 = min(P, t0 + ipg * tpi);
  const int64_t pos = static_cast<int64_t>(Mp) * Np;
  const float bv = bias ? bias[o] : 0.f;
  float cnt = 0.f, mean = 0.f, m2 = 0.f;
  for (int t = t0 + lane; t < t1; t += 64) {
    const float* src = cbuf + static_cast<int64_t>(o) * Np + t;
    float m[NPOS];
#pragma unroll
    for (int b = 0; b < NPOS; ++b) m[b] = src[b * pos];
    for (int z = 1; z < splits; ++z) {
      const float* sz = src + static_cast<int64_t>(z) * NPOS * pos;
#pragma unroll
      for (int b = 0; b < NPOS; ++b) m[b] += sz[b * pos];
    }
    float v[TILE][TILE];
    if constexpr (TILE == 4) {  // bg_output_f4_kernel's arithmetic
      float sr[4][6];
#pragma unroll
      for (int jc = 0; jc < 6; ++jc) {
        const float a = m[6 + jc] + m[12 + jc], bq = m[6 + jc] - m[12 + jc];
        const float cc = m[18 + jc] + m[24 + jc], d = m[18 + jc] - m[24 + jc];
        sr[0][jc] = m[jc] + a + cc;
        sr[1][jc] = bq + 2.f * d;
        sr[2][jc] = a + 4.f * cc;
        sr[3][jc] = bq + 8.f * d + m[30 + jc];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float a = sr[k][1] + sr[k][2], bq = sr[k][1] - sr[k][2];
        const float cc = sr[k][3] + sr[k][4], d = sr[k][3] - sr[k][4];
        v[k][0] = sr[k][0] + a + cc + bv;
        v[k][1] = bq + 2.f * d + bv;
        v[k][2] = a + 4.f * cc + bv;
        v[k][3] = bq + 8.f * d + sr[k][5] + bv;
      }
    } else {  // bg_output_f2_kernel's arithmetic
      float sr[2][4];
#pragma unroll
      for (int jc = 0; jc < 4; ++jc) {
        sr[0][jc] = m[jc] + m[4 + jc] + m[8 + jc];
        sr[1][jc] = m[4 + jc] - m[8 + jc] - m[12 + jc];
      }
#pragma unroll
      for (int kr = 0; kr < 2; ++kr) {
        v[kr][0] = sr[kr][0] + sr[kr][1] + sr[kr][2] + bv;
        v[kr][1] = sr[kr][1] - sr[kr][2] - sr[kr][3] + bv;
      }
    }
    const int n = t / tpi;
    const int rem = t - n * tpi;
    const int ty = rem / TW;
    const int py = TILE * ty, px = TILE * (rem - ty * TW);
    float* yp = y + (static_cast<int64_t>(n) * O + o) * H * W + static_cast<int64_t>(py) * W + px;
    const int rows = min(TILE, H - py), cols = min(TILE, W - px);
    float ts = 0.f;
#pragma unroll
    for (int k = 0; k < TILE; ++k) {
      if (k >= rows) break;
      bool stored = false;
      if constexpr (TILE == 4) {
        if (cols == 4 && (W & 3) == 0) {
          *reinterpret_cast<floatx4*>(yp + k * W) = floatx4{v[k][0], v[k][1], v[k][2], v[k][3]};
          stored = true;
        }
      }
      if (!stored) {
#pragma unroll
        for (int l = 0; l < TILE; ++l)
          if (l < cols) yp[k * W + l] = v[k][l];
      }
#pragma unroll
      for (int l = 0; l < TILE; ++l)
        if (l < cols) ts += v[k][l];
    }
    const float tc = static_cast<float>(rows * cols);
    const float tm = ts / tc;
    float tq = 0.f;
#pragma unroll
    for (int k = 0; k < TILE; ++k) {
      if (k >= rows) break;
#pragma unroll
      for (int l = 0; l < TILE; ++l) {
        if (l < cols) {
          const float d = v[k][l] - tm;
          tq += d * d;
        }
      }
    }
    chan_merge_f(cnt, mean, m2, tc, tm, tq);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float nb = __shfl_xor(cnt, off), mb = __shfl_xor(mean, off);
    const float qb = __shfl_xor(m2, off);
    chan_merge_f(cnt, mean, m2, nb, mb, qb);
  }
  if (lane == 0) {
    pm[static_cast<int64_t>(g) * O + o] = mean;
    pm2[static_cast<int64_t>(g) * O + o] = m2;
  }
}

}  // namespace

int64_t wino4_pad_reduction(int64_t r) { return (r + kC - 1) / kC * kC; }
int64_t wino4_pad_output(int64_t o) { return (o + kOPad - 1) / kOPad * kOPad; }

bool wino4_supported(int64_t n, int64_t r, int64_t h, int64_t w, int64_t o) {
  // 32-bit tile / offset arithmetic and the padding-tap encoding need the input below
  // 1 GiB; every split keeps >= 1 step.
  const int64_t x_bytes = n * r * h * w * 4;
  const int64_t tiles = n * ((h + 3) / 4) * ((w + 3) / 4);
  return x_bytes > 0 && x_bytes < (int64_t{1} << 30) - 64 && tiles < (int64_t{1} << 30) &&
         n * o * h * w < (int64_t{1} << 31) && o < (1 << 24);
}

void launch_wino4_weight(const float* w, float* u, int64_t out_channels, int64_t red_channels,
                         bool flip, hipStream_t stream) {
  const int64_t Op = wino4_pad_output(out_channels);
  const int64_t Rp = wino4_pad_reduction(red_channels);
  const int64_t total = Rp * Op;
  hipLaunchKernelGGL(f4_weight_kernel, dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256),
                     0, stream, w, u, static_cast<int>(out_channels),
                     static_cast<int>(red_channels), static_cast<int>(Op), static_cast<int>(Rp),
                     flip);
}

WinoPlan wino4_plan(int64_t n, int64_t red_channels, int64_t h, int64_t w, int64_t out_channels,
                    int variant, int splits) {
  WinoPlan plan;
  plan.variant = (variant >= 4 && variant <= 12 && variant != 11) || variant == 14 ||
                         variant == 15 || variant == 18 ? variant : 5;
  const int og = plan.variant == 5 || plan.variant == 7 || plan.variant == 15 ? 2 : 4;
  const int64_t P = n * ((h + 3) / 4) * ((w + 3) / 4);
  const int64_t blocks = ((P + kT - 1) / kT) * ((out_channels + 16 * og - 1) / (16 * og));
  const int64_t steps = wino4_pad_reduction(red_channels) / kC;
  if (splits > 0) {
    plan.splits = static_cast<int>(std::min<int64_t>(splits, steps));
  } else {
    // Split-K by a cost model fitted to benchmarks/split_sweep.py (profiles/r5/
    // split_sweep.json): ~2.1 us per 4-channel step of a 64-channel workgroup (one per CU;
    // 32-channel workgroups ~1.9 us, two per CU), and per extra split ~0.23 us per MB of
    // output partials plus ~11.6 us for the reduce pass.  (The old ">= 16 steps per split"
    // rule kept ResNet's 28^2 x 128 layers at 22 images on 2 splits: 49 -> 41 us at 3.)
    const int64_t cap = og == 4 ? 256 : 512;
    const double step_us = og == 4 ? 2.1 : 1.9;
    const double mb = static_cast<double>(n) * out_channels * h * w * 4 / 1e6;
    int64_t best = 1;
    double best_cost = 0;
    for (int64_t s = 1; s <= std::min<int64_t>(64, steps); ++s) {
      const int64_t rounds = (blocks * s + cap - 1) / cap;
      const double cost = rounds * ((steps + s - 1) / s) * step_us +
                          (s > 1 ? 11.6 + 0.23 * s * mb : 0.0);
      if (s == 1 || cost < best_cost) {
        best = s;
        best_cost = cost;
      }
    }
    plan.splits = static_cast<int>(best);
  }
  plan.workspace = plan.splits > 1 ? plan.splits * n * out_channels * h * w : 0;
  if (plan.variant >= 14) {  // + the transformed input V4[P/32][Rp/4][4][32][36], first
    plan.workspace += ((P + kT - 1) / kT) * kT * wino4_pad_reduction(red_channels) * kP;
  }
  return plan;
}

void launch_wino4_conv(const float* x, const float* u, const float* bias, float* y, float* ws,
                       int64_t n, int64_t red_channels, int64_t h, int64_t w, int64_t out_channels,
                       const WinoPlan& plan, hipStream_t stream) {
  const int64_t Rp = wino4_pad_reduction(red_channels);
  const int64_t Op = wino4_pad_output(out_channels);
  const int64_t th = (h + 3) / 4, tw = (w + 3) / 4;
  const int64_t P = n * th * tw;
  const int og = plan.variant == 5 || plan.variant == 7 || plan.variant == 15 ? 2 : 4;
  const int tblocks = static_cast<int>((P + kT - 1) / kT);
  if (plan.variant == 18) {
    const int oblocks4 = static_cast<int>((out_channels + 63) / 64);
    const int64_t nwg4 = static_cast<int64_t>(tblocks) * oblocks4 * plan.splits;
    auto kernel = f4_conv_ring_kernel<false>;  // (16-byte centre loads: see variant 12)
    hipLaunchKernelGGL(kernel, dim3(static_cast<unsigned>(nwg4)), dim3(512), 0, stream, x, u,
                       bias, plan.splits > 1 ? ws : y, static_cast<int>(red_channels),
                       static_cast<int>(h), static_cast<int>(w),
                       static_cast<int>(out_channels), static_cast<int>(Rp),
                       static_cast<int>(Op), static_cast<int>(th), static_cast<int>(tw),
                       static_cast<int>(P), tblocks, oblocks4, plan.splits,
                       static_cast<uint32_t>(n * red_channels * h * w * 4));
    if (plan.splits > 1)
      launch_split_reduce(ws, bias, y, n * out_channels * h * w, h * w,
                          static_cast<int>(out_channels), plan.splits, stream);
    return;
  }
  const int oblocks = static_cast<int>((out_channels + 16 * og - 1) / (16 * og));
  const int splits = plan.splits;
  const int64_t nwg = static_cast<int64_t>(tblocks) * oblocks * splits;
  if (plan.variant >= 14) {
    float* vbuf = ws;
    const int64_t vtotal = static_cast<int64_t>(tblocks) * kT * Rp;  // threads
    float* split_ws = ws + vtotal * kP;
    hipLaunchKernelGGL(f4_input_transform_kernel, dim3(static_cast<unsigned>((vtotal + 255) / 256)),
                       dim3(256), 0, stream, x, vbuf, static_cast<int>(red_channels),
                       static_cast<int>(h), static_cast<int>(w), static_cast<int>(tw),
                       static_cast<int>(th * tw), static_cast<int>(P), static_cast<int>(Rp),
                       vtotal, static_cast<uint32_t>(n * red_channels * h * w * 4));
    auto gemm = og == 4 ? f4_gemm_kernel<4> : f4_gemm_kernel<2>;
    hipLaunchKernelGGL(gemm, dim3(static_cast<unsigned>(nwg)), dim3(128 * og), 0, stream, vbuf, u,
                       bias, splits > 1 ? split_ws : y, static_cast<int>(h), static_cast<int>(w),
                       static_cast<int>(out_channels), static_cast<int>(Rp), static_cast<int>(Op),
                       static_cast<int>(th), static_cast<int>(tw), static_cast<int>(P), tblocks,
                       oblocks, splits);
    if (splits > 1)
      launch_split_reduce(split_ws, bias, y, n * out_channels * h * w, h * w,
                          static_cast<int>(out_channels), splits, stream);
    return;
  }
  // 16-byte centre loads (W % 4 == 0) pay off in the 4-wave variant only: the 8-wave one
  // ran 4-16 % slower with them (benchmarks/wino_variants.py, profiles/wino_f4_variants.json)
  const bool vec = (w & 3) == 0;
  auto kernel = og == 4 ? f4_conv_kernel<4, false>
                        : (vec ? f4_conv_kernel<2, true> : f4_conv_kernel<2, false>);
  if (plan.variant == 6) kernel = f4_conv_kernel<4, false, true>;
  if (plan.variant == 8) kernel = f4_conv_kernel<4, false, true, 1>;
  if (plan.variant == 9) kernel = f4_conv_kernel<4, false, true, 2>;
  if (plan.variant == 10) kernel = f4_conv_kernel<4, false, true, 3>;
  if (plan.variant == 12) kernel = vec ? f4_conv_kernel<4, true, true> : f4_conv_kernel<4, false, true>;
  if (plan.variant == 7) kernel = vec ? f4_conv_kernel<2, true, true> : f4_conv_kernel<2, false, true>;
  hipLaunchKernelGGL(kernel, dim3(static_cast<unsigned>(nwg)), dim3(128 * og), 0, stream,
                     x, u, bias, splits > 1 ? ws : y, static_cast<int>(red_channels),
                     static_cast<int>(h), static_cast<int>(w), static_cast<int>(out_channels),
                     static_cast<int>(Rp), static_cast<int>(Op), static_cast<int>(th),
                     static_cast<int>(tw), static_cast<int>(P), tblocks, oblocks, splits,
                     static_cast<uint32_t>(n * red_channels * h * w * 4));
  if (splits > 1) {
    launch_split_reduce(ws, bias, y, n * out_channels * h * w, h * w,
                        static_cast<int>(out_channels), splits, stream);
  }
}

bool wino4_wgrad_supported(int64_t n, int64_t c, int64_t k, int64_t h, int64_t w) {
  const int64_t lim = (int64_t{1} << 30) - 64;
  const int64_t tiles = n * ((h + 3) / 4) * ((w + 3) / 4);
  return n * c * h * w * 4 < lim && n * k * h * w * 4 < lim && n * c * h * w > 0 &&
         n * k * h * w > 0 && tiles + 64 < (int64_t{1} << 30);
}

int wino4_wgrad_splits(int64_t n, int64_t c, int64_t k, int64_t h, int64_t w) {
  // Split-K by a cost model fitted to benchmarks/split_sweep.py (profiles/r5/
  // split_sweep.json): one 8-wave workgroup per CU, ~2.5 us per 4-tile step, and per extra
  // split ~0.8 us per MB of k x c x 36 partials (written, then summed by the reduce pass)
  // plus ~5 us for that pass.  The old ">= 32 steps per split" rule left 3/4 of the CUs
  // idle at ResNet's 15-36-image micro-batches (14^2 x 256 channels at 22 images: 139 ->
  // 57 us).
  const int64_t blocks = ((c + 31) / 32) * ((k + 63) / 64);
  const int64_t steps = (n * ((h + 3) / 4) * ((w + 3) / 4) + 3) / 4;
  const double mb = static_cast<double>(((c + 31) / 32) * 32) * (((k + 63) / 64) * 64) * 9 * 4 /
                    1e6;
  int best = 1;
  double best_cost = 0;
  for (int64_t s = 1; s <= std::min<int64_t>(512, steps); ++s) {
    const int64_t rounds = (blocks * s + 255) / 256;
    const double cost = rounds * ((steps + s - 1) / s) * 2.5 + (s > 1 ? 5.0 + 0.8 * s * mb : 0.0);
    if (s == 1 || cost < best_cost) {
      best = static_cast<int>(s);
      best_cost = cost;
    }
  }
  return best;
}

int64_t wino4_wgrad_workspace(int64_t n, int64_t c, int64_t k, int64_t h, int64_t w, int splits,
                              int variant) {
  if (variant == 2) return wino4_wgrad_emu_workspace(n, c, k, h, w, splits);
  int64_t total = splits > 1 ? splits * k * c * 9 : 0;
  if (variant == 1) {
    const int64_t ppad = ((n * ((h + 3) / 4) * ((w + 3) / 4) + 3) / 4) * 4;
    total += ppad * (((c + 31) / 32) * 32 + ((k + 63) / 64) * 64) * kP;
  }
  return total;
}

void launch_wino4_wgrad(const float* x, const float* dy, float* dw, float* ws, int64_t n,
                        int64_t c, int64_t k, int64_t h, int64_t w, int splits, int variant,
                        bool accum, hipStream_t stream) {
  const int64_t th = (h + 3) / 4, tw = (w + 3) / 4;
  const int64_t P = n * th * tw;
  const int cblocks = static_cast<int>((c + 31) / 32);
  const int kblocks = static_cast<int>((k + 63) / 64);
  const int64_t nwg = static_cast<int64_t>(cblocks) * kblocks * splits;
  const uint32_t x_bytes = static_cast<uint32_t>(n * c * h * w * 4);
  const uint32_t dy_bytes = static_cast<uint32_t>(n * k * h * w * 4);
  if (variant == 2) {
    launch_wino4_wgrad_emu(x, dy, dw, ws, n, c, k, h, w, splits, accum, stream);
    return;
  }
  float* partial = ws;
  if (variant == 1) {
    const int64_t nsteps = (P + 3) / 4;
    const int64_t ppad = nsteps * 4;
    float* vx = ws;
    float* m = vx + ppad * cblocks * 32 * kP;
    partial = m + ppad * kblocks * 64 * kP;
    const int64_t vt = ppad * cblocks * 32, mt = ppad * kblocks * 64;
    hipLaunchKernelGGL(f4_wg_vx_kernel, dim3(static_cast<unsigned>((vt + 255) / 256)), dim3(256), 0,
                       stream, x, vx, static_cast<int>(n), static_cast<int>(c), static_cast<int>(h),
                       static_cast<int>(w), static_cast<int>(th), static_cast<int>(tw),
                       static_cast<int>(ppad), cblocks, vt, x_bytes);
    auto mk = (w & 3) == 0 ? f4_wg_mdy_kernel<true> : f4_wg_mdy_kernel<false>;
    hipLaunchKernelGGL(mk, dim3(static_cast<unsigned>((mt + 255) / 256)), dim3(256), 0, stream, dy,
                       m, static_cast<int>(n), static_cast<int>(k), static_cast<int>(h),
                       static_cast<int>(w), static_cast<int>(th), static_cast<int>(tw),
                       static_cast<int>(ppad), kblocks, mt, dy_bytes);
    hipLaunchKernelGGL(f4_wgrad_gemm_kernel<>, dim3(static_cast<unsigned>(nwg)), dim3(kWgThreads), 0,
                       stream, vx, m, splits > 1 ? partial : dw, static_cast<int>(c),
                       static_cast<int>(k), static_cast<int>(nsteps), cblocks, kblocks, splits,
                       accum && splits == 1);
  } else {
    auto kernel = (w & 3) == 0 ? f4_wgrad_kernel<true> : f4_wgrad_kernel<false>;
    hipLaunchKernelGGL(kernel, dim3(static_cast<unsigned>(nwg)), dim3(kWgThreads), 0,
                       stream, x, dy, splits > 1 ? partial : dw, static_cast<int>(n),
                       static_cast<int>(c), static_cast<int>(k), static_cast<int>(h),
                       static_cast<int>(w), static_cast<int>(th), static_cast<int>(tw),
                       static_cast<int>(P), cblocks, kblocks, splits, x_bytes, dy_bytes,
                       accum && splits == 1);
  }
  if (splits > 1) {
    launch_split_reduce(partial, nullptr, dw, k * c * 9, 9, static_cast<int>(k), splits, stream,
                        accum);
  }
}

// ---- batched-GEMM Winograd host side ---------------------------------------------------

namespace {
constexpr int kBgRowPad = 256;  // weight rows (output channels) padded for either tile height
int64_t bg_round(int64_t v, int64_t m) { return (v + m - 1) / m * m; }
// (waves, BN) instantiations of bg_gemm_kernel
constexpr int kBgTiles[][2] = {{4, 48}, {4, 64}, {4, 96}, {4, 128},
                               {8, 64}, {8, 96}, {8, 128}, {8, 144}};
// 16-deep steps of the transformed operands: the reduction padded to 32 channels, so a
// pipeline stage may hold one or two steps
int64_t bg_ksteps(int64_t red_channels) { return (red_channels + 31) / 32 * 2; }
}  // namespace

bool bg_emu(int emu) {
  static const bool dflt = [] {
    const char* v = std::getenv("TGPIPE_BG_EMU");
    return v == nullptr || *v == 0 || std::string(v) != "0";
  }();
  return emu < 0 ? dflt : emu != 0;
}

int bg_pick_bn(int64_t tiles, int kind, bool emu) {
  // The 128-row tile width that pads the tile count least; ties go to the width measured
  // fastest (benchmarks/bg_bench.py, profiles/r3/bg_bench.json): 48 for F(4x4) (128 on
  // the widest grids), 128 then 96 for F(2x2).  The split-bf16 GEMM's tiles are 32-column
  // multiples.
  static constexpr int kF4[] = {48, 64, 128, 96};
  static constexpr int kF2[] = {128, 96, 48, 64};
  static constexpr int kEmu[] = {128, 64, 96, 128};
  const int* order = emu ? kEmu : (kind == 2 ? kF2 : kF4);
  int best = order[0];
  int64_t best_pad = bg_round(tiles, best);
  for (int i = 1; i < 4; ++i) {
    const int64_t pad = bg_round(tiles, order[i]);
    if (pad < best_pad) {
      best = order[i];
      best_pad = pad;
    }
  }
  if (kind != 2 && tiles >= 4096 && tiles % 128 == 0) best = 128;
  return best;
}

BgPlan bg_plan(int64_t n, int64_t red_channels, int64_t h, int64_t w, int64_t out_channels,
               int bn, int splits, int kind, int waves, int sub, int emu) {
  BgPlan plan;
  plan.kind = kind == 2 ? 2 : 4;
  plan.emu = bg_emu(emu);
  const int tile = plan.kind;
  const int64_t npos = plan.kind == 2 ? kP2 : kP;
  const int64_t P = n * ((h + tile - 1) / tile) * ((w + tile - 1) / tile);
  plan.ksteps = bg_ksteps(red_channels);
  plan.mp = bg_round(out_channels, kBgRowPad);
  bool valid = false;
  for (const auto& t : kBgTiles) valid |= t[0] == waves && t[1] == bn;
  if (plan.emu) {  // 4 waves x bn 64 / 96 / 128, one step per stage
    valid = waves == 4 && (bn == 64 || bn == 96 || bn == 128);
    sub = 1;
    if (!valid) {
      waves = 4;
      bn = bg_pick_bn(P, plan.kind, true);
      valid = true;
    }
  }
  if (!valid) {
    // Auto: 128-row tiles (4 waves), which beat the 256-row ones on every measured U-Net
    // shape once the fragment reads were software-pipelined (profiles/r3/bg_bench.json)
    waves = 4;
    bn = bg_pick_bn(P, plan.kind);
  }
  plan.waves = waves;
  plan.bn = bn;
  // one 16-deep step per stage: two halved the resident workgroups per CU and ran 2-20 %
  // slower on every shape (profiles/r3/bg_bench.json)
  plan.sub = sub == 1 || sub == 2 ? sub : 1;
  plan.np = bg_round(P, plan.bn);
  const int64_t bm = 32 * waves;
  const int64_t tiles = (plan.mp / bm) * (plan.np / plan.bn) * npos;
  if (splits > 0) {
    plan.splits = splits;
  } else {
    // >= 2-3 workgroups per CU, >= 16 steps per split
    const int64_t target = waves == 8 ? 512 : 768;
    int64_t s = 1;
    while (tiles * s < target && plan.ksteps / (s * 2) >= 16) s *= 2;
    plan.splits = static_cast<int>(s);
  }
  // every split owns >= 1 pipeline stage
  plan.splits = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(plan.splits,
                                                                        plan.ksteps / plan.sub)));
  // (split-bf16 V: 24 floats' worth of bytes per row and step instead of 16)
  plan.workspace = npos * plan.ksteps * (plan.emu ? 24 : 16) * plan.np +
                   plan.splits * npos * plan.mp * plan.np;
  return plan;
}

int64_t bg_weight_numel(int64_t out_channels, int64_t red_channels, int kind, int emu) {
  return (kind == 2 ? kP2 : kP) * bg_ksteps(red_channels) * (bg_emu(emu) ? 24 : 16) *
         bg_round(out_channels, kBgRowPad);
}

void launch_bg_weight(const float* w, float* a, int64_t out_channels, int64_t red_channels,
                      bool flip, int kind, hipStream_t stream, int emu) {
  const int64_t mp = bg_round(out_channels, kBgRowPad);
  const int64_t ksteps = bg_ksteps(red_channels);
  if (bg_emu(emu)) {
    const int64_t total = ksteps * 4 * mp;
    hipLaunchKernelGGL(kind == 2 ? bg_weight_f2_emu_kernel : bg_weight_f4_emu_kernel,
                       dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256), 0, stream, w,
                       a, static_cast<int>(out_channels), static_cast<int>(red_channels),
                       static_cast<int>(mp), static_cast<int>(ksteps), flip);
    return;
  }
  const int64_t total = ksteps * 16 * mp;
  hipLaunchKernelGGL(kind == 2 ? bg_weight_f2_kernel : bg_weight_f4_kernel,
                     dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256), 0, stream, w, a,
                     static_cast<int>(out_channels), static_cast<int>(red_channels),
                     static_cast<int>(mp), static_cast<int>(ksteps), flip);
}

int bg_stats_ipg(int64_t n, int64_t h, int64_t w, int kind) {
  // images per statistics group: >= 64 tiles (one per lane of the channel's wave) when the
  // batch allows
  const int64_t tile = kind == 2 ? 2 : 4;
  const int64_t tpi = std::max<int64_t>(1, ((h + tile - 1) / tile) * ((w + tile - 1) / tile));
  return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(n, (64 + tpi - 1) / tpi)));
}

void launch_bg_conv(const float* x, const float* a, const float* bias, float* y, float* ws,
                    int64_t n, int64_t red_channels, int64_t h, int64_t w, int64_t out_channels,
                    const BgPlan& plan, hipStream_t stream, float* pm, float* pm2, int ipg) {
  const int tile = plan.kind;
  const int npos = plan.kind == 2 ? kP2 : kP;
  const int64_t th = (h + tile - 1) / tile, tw = (w + tile - 1) / tile;
  const int64_t P = n * th * tw;
  float* v = ws;
  float* cbuf = ws + npos * plan.ksteps * (plan.emu ? 24 : 16) * plan.np;
  const int64_t vt = plan.ksteps * 16 * plan.np;
  if (plan.emu) {
    // channels per thread: 4 (8-byte stores) while that fills the chip with >= 512
    // workgroups, else 2 or 1 -- ResNet's 14^2 / 7^2 layers at 22-image micro-batches
    // gave 96-workgroup grids at 4
    const int64_t vt4 = plan.ksteps * 4 * plan.np;
    const int cpt = (vt4 + 255) / 256 >= 512 ? 4 : (vt4 * 2 + 255) / 256 >= 512 ? 2 : 1;
    const dim3 grid(static_cast<unsigned>((vt4 * (4 / cpt) + 255) / 256));
    const int ri = static_cast<int>(red_channels), hi = static_cast<int>(h),
              wi = static_cast<int>(w), twi = static_cast<int>(tw), tpi = static_cast<int>(th * tw),
              pi = static_cast<int>(P), npi = static_cast<int>(plan.np),
              ki = static_cast<int>(plan.ksteps);
    if (plan.kind == 2) {
      auto kern = cpt == 4 ? bg_input_f2_emu_kernel<4>
                  : cpt == 2 ? bg_input_f2_emu_kernel<2> : bg_input_f2_emu_kernel<1>;
      hipLaunchKernelGGL(kern, grid, dim3(256), 0, stream, x, v, ri, hi, wi, twi, tpi, pi, npi,
                         ki);
    } else {
      const bool vec = (w & 3) == 0;
      auto kern = vec ? bg_input_f4_emu_kernel<true, 4> : bg_input_f4_emu_kernel<false, 4>;
      if (cpt == 2) kern = vec ? bg_input_f4_emu_kernel<true, 2> : bg_input_f4_emu_kernel<false, 2>;
      if (cpt == 1) kern = vec ? bg_input_f4_emu_kernel<true, 1> : bg_input_f4_emu_kernel<false, 1>;
      hipLaunchKernelGGL(kern, grid, dim3(256), 0, stream, x, v, ri, hi, wi, twi, tpi, pi, npi, ki,
                         static_cast<uint32_t>(n * red_channels * h * w * 4));
    }
  } else if (plan.kind == 2) {
    hipLaunchKernelGGL(bg_input_f2_kernel, dim3(static_cast<unsigned>((vt + 255) / 256)),
                       dim3(256), 0, stream, x, v, static_cast<int>(red_channels),
                       static_cast<int>(h), static_cast<int>(w), static_cast<int>(tw),
                       static_cast<int>(th * tw), static_cast<int>(P),
                       static_cast<int>(plan.np), static_cast<int>(plan.ksteps));
  } else {
    const int64_t vt4 = plan.ksteps * 4 * plan.np;
    hipLaunchKernelGGL((w & 3) == 0 ? bg_input_f4_kernel<true> : bg_input_f4_kernel<false>,
                       dim3(static_cast<unsigned>((vt4 + 255) / 256)), dim3(256), 0, stream, x, v,
                       static_cast<int>(red_channels), static_cast<int>(h), static_cast<int>(w),
                       static_cast<int>(tw), static_cast<int>(th * tw), static_cast<int>(P),
                       static_cast<int>(plan.np), static_cast<int>(plan.ksteps),
                       static_cast<uint32_t>(n * red_channels * h * w * 4));
  }
  const int mtiles = static_cast<int>(plan.mp / (32 * plan.waves));
  const int ntiles = static_cast<int>(plan.np / plan.bn);
  const int64_t nwg = static_cast<int64_t>(mtiles) * ntiles * npos * plan.splits;
  using Gemm = void (*)(const float*, const float*, float*, int, int, int, int, int, int, int);
  Gemm gemm = bg_gemm_kernel<4, 64, 2>;
  if (plan.emu) {
    gemm = plan.bn == 64 ? bg_gemm_emu_kernel<64>
           : plan.bn == 96 ? bg_gemm_emu_kernel<96> : bg_gemm_emu_kernel<128>;
  } else switch (plan.waves * 10000 + plan.bn * 10 + plan.sub) {
    case 40481: gemm = bg_gemm_kernel<4, 48, 1>; break;
    case 40641: gemm = bg_gemm_kernel<4, 64, 1>; break;
    case 40961: gemm = bg_gemm_kernel<4, 96, 1>; break;
    case 41281: gemm = bg_gemm_kernel<4, 128, 1>; break;
    case 40482: gemm = bg_gemm_kernel<4, 48, 2>; break;
    case 40642: gemm = bg_gemm_kernel<4, 64, 2>; break;
    case 40962: gemm = bg_gemm_kernel<4, 96, 2>; break;
    case 41282: gemm = bg_gemm_kernel<4, 128, 2>; break;
    case 80641: gemm = bg_gemm_kernel<8, 64, 1>; break;
    case 80961: gemm = bg_gemm_kernel<8, 96, 1>; break;
    case 81281: gemm = bg_gemm_kernel<8, 128, 1>; break;
    case 81441: gemm = bg_gemm_kernel<8, 144, 1>; break;
    default: break;
  }
  const int block = 64 * plan.waves;
  hipLaunchKernelGGL(gemm, dim3(static_cast<unsigned>(nwg)), dim3(block), 0, stream, a,
                     v, cbuf, static_cast<int>(plan.mp), static_cast<int>(plan.np),
                     static_cast<int>(plan.ksteps), mtiles, ntiles, static_cast<int>(npos),
                     plan.splits);
  if (pm != nullptr) {  // with the BatchNorm statistics of y (bg_output_stats_kernel)
    const int64_t groups = (n + ipg - 1) / ipg;
    const dim3 sgrid(static_cast<unsigned>((out_channels + 3) / 4),
                     static_cast<unsigned>(groups));
    hipLaunchKernelGGL(plan.kind == 2 ? bg_output_stats_kernel<2> : bg_output_stats_kernel<4>,
                       sgrid, dim3(256), 0, stream, cbuf, bias, y, pm, pm2,
                       static_cast<int>(out_channels), static_cast<int>(plan.mp),
                       static_cast<int>(plan.np), static_cast<int>(P),
                       static_cast<int>(th * tw), static_cast<int>(tw), static_cast<int>(h),
                       static_cast<int>(w), plan.splits, ipg);
    return;
  }
  const int64_t ot = out_channels * P;
  hipLaunchKernelGGL(plan.kind == 2 ? bg_output_f2_kernel : bg_output_f4_kernel,
                     dim3(static_cast<unsigned>((ot + 255) / 256)), dim3(256),
                     0, stream, cbuf, bias, y, static_cast<int>(out_channels),
                     static_cast<int>(plan.mp), static_cast<int>(plan.np), static_cast<int>(P),
                     static_cast<int>(th * tw), static_cast<int>(tw), static_cast<int>(h),
                     static_cast<int>(w), plan.splits);
}


// ---- split-bf16 weight gradient host side (variant 2) -------------------------------------

namespace {
struct WgEmuPlan {
  int64_t ksteps, mp, np;
  int bn;
};

WgEmuPlan wg_emu_plan(int64_t n, int64_t c, int64_t k, int64_t h, int64_t w) {
  WgEmuPlan p;
  const int64_t P = n * ((h + 3) / 4) * ((w + 3) / 4);
  p.ksteps = (P + 15) / 16;
  p.bn = bg_pick_bn(c, 4, true);  // columns: the input channels
  p.mp = bg_round(k, 128);        // rows: the gradient channels (128-row tiles)
  p.np = bg_round(c, p.bn);
  return p;
}
}  // namespace

int wino4_wgrad_emu_splits(int64_t n, int64_t c, int64_t k, int64_t h, int64_t w) {
  // two workgroups per CU: >= 2 rounds over the 256 CUs, >= 8 sixteen-tile steps per split
  const WgEmuPlan p = wg_emu_plan(n, c, k, h, w);
  const int64_t tiles = (p.mp / 128) * (p.np / p.bn) * kP;
  int64_t s = 1;
  while (tiles * s < 1024 && p.ksteps / (s * 2) >= 8) s *= 2;
  return static_cast<int>(s);
}

int64_t wino4_wgrad_emu_workspace(int64_t n, int64_t c, int64_t k, int64_t h, int64_t w,
                                  int splits) {
  const WgEmuPlan p = wg_emu_plan(n, c, k, h, w);
  // M' and V images (96 bytes = 24 floats per row and step), then the split partials
  return kP * p.ksteps * 24 * (p.mp + p.np) + static_cast<int64_t>(splits) * kP * p.mp * p.np;
}

void launch_wino4_wgrad_emu(const float* x, const float* dy, float* dw, float* ws, int64_t n,
                            int64_t c, int64_t k, int64_t h, int64_t w, int splits, bool accum,
                            hipStream_t stream) {
  const WgEmuPlan p = wg_emu_plan(n, c, k, h, w);
  const int64_t th = (h + 3) / 4, tw = (w + 3) / 4;
  const int64_t P = n * th * tw;
  float* am = ws;
  float* bv = am + kP * p.ksteps * 24 * p.mp;
  float* cb = bv + kP * p.ksteps * 24 * p.np;
  const bool vec = (w & 3) == 0;
  const int64_t mt = p.ksteps * 4 * p.mp, vt = p.ksteps * 4 * p.np;
  hipLaunchKernelGGL(vec ? wg_dy_emu_kernel<true> : wg_dy_emu_kernel<false>,
                     dim3(static_cast<unsigned>((mt + 255) / 256)), dim3(256), 0, stream, dy, am,
                     static_cast<int>(n), static_cast<int>(k), static_cast<int>(h),
                     static_cast<int>(w), static_cast<int>(th), static_cast<int>(tw),
                     static_cast<int>(p.mp), static_cast<int>(p.ksteps),
                     static_cast<uint32_t>(n * k * h * w * 4));
  hipLaunchKernelGGL(vec ? wg_x_emu_kernel<true> : wg_x_emu_kernel<false>,
                     dim3(static_cast<unsigned>((vt + 255) / 256)), dim3(256), 0, stream, x, bv,
                     static_cast<int>(c), static_cast<int>(h), static_cast<int>(w),
                     static_cast<int>(tw), static_cast<int>(th * tw), static_cast<int>(P),
                     static_cast<int>(p.np), static_cast<int>(p.ksteps),
                     static_cast<uint32_t>(n * c * h * w * 4));
  const int mtiles = static_cast<int>(p.mp / 128);
  const int ntiles = static_cast<int>(p.np / p.bn);
  const int64_t nwg = static_cast<int64_t>(mtiles) * ntiles * kP * splits;
  auto gemm = p.bn == 64 ? bg_gemm_emu_kernel<64>
              : p.bn == 96 ? bg_gemm_emu_kernel<96> : bg_gemm_emu_kernel<128>;
  hipLaunchKernelGGL(gemm, dim3(static_cast<unsigned>(nwg)), dim3(256), 0, stream, am, bv, cb,
                     static_cast<int>(p.mp), static_cast<int>(p.np), static_cast<int>(p.ksteps),
                     mtiles, ntiles, static_cast<int>(kP), splits);
  const int64_t ot = k * c;
  hipLaunchKernelGGL(wg_output_emu_kernel, dim3(static_cast<unsigned>((ot + 255) / 256)),
                     dim3(256), 0, stream, cb, dw, static_cast<int>(k), static_cast<int>(c),
                     static_cast<int>(p.mp), static_cast<int>(p.np), splits, accum);
}

}  // namespace tgpipe
