// Winograd F(2x2, 3x3) convolution on the fp32 MFMA pipes of CDNA4 (gfx950).
//
// The U-Net's 3x3 / stride 1 / pad 1 convolutions are ~60 % of its training
// step.  MIOpen runs them with a VALU Winograd kernel at ~110 TFLOP/s
// (direct-conv FLOP count); here the Winograd-domain products run on
// v_mfma_f32_16x16x4_f32 instead, with the input transform fused in front of
// the matrix core work and the output transform fused behind it:
//
//   for each block of 32 output tiles (2x2 pixels each) x 64 output channels:
//     for each chunk of 8 input channels:
//       V[xi][c][t] = (B^T d B)[xi]   4x4 input patch of tile t, channel c   (VALU -> LDS)
//       U[xi][c][o]                   pre-transformed weights (G g G^T)     (global -> LDS)
//       M[xi][o][t] += sum_c U[xi][c][o] * V[xi][c][t]   16 independent GEMMs (MFMA)
//     Y[o][tile] = A^T M A                                     (registers -> global)
//
// Each wave owns 16 output channels x 32 tiles for ALL 16 Winograd positions
// (32 accumulator tiles of 16x16), so the output transform needs no data
// exchange: lane l holds positions 0..15 of the same (channel, tile) pair.
// Numerics are exact f32 arithmetic (MFMA f32 is an fmaf chain); the Winograd
// transform itself changes rounding relative to a direct convolution at the
// 1e-6 relative level.
//
// Backward-data of a 3x3/s1/p1 convolution is the same convolution of dY with
// the spatially flipped, in/out-transposed kernel: the weight transform takes a
// `flip` flag, and the same main kernel runs it.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "kernels.h"

namespace tgpipe {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kCB = 8;          // reduction channels per main-loop iteration
constexpr int kOBMax = 64;      // output-channel padding granule of U
constexpr int kThreads = 256;   // 4 waves

__device__ float kZeroTap = 0.f;  // load target of zero-padding taps (never written)

// U[r][o][xi] = (G g G^T)[xi] for g = kernel of (output channel o, reduction
// channel r), zero-padded to [Rp][Op][16].
__global__ void wino_weight_kernel(const float* __restrict__ w, float* __restrict__ u, int O,
                                   int R, int Op, int Rp, bool flip) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= static_cast<int64_t>(Rp) * Op) return;
  const int r = static_cast<int>(idx / Op);
  const int o = static_cast<int>(idx % Op);
  float g[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) g[i][j] = 0.f;
  if (r < R && o < O) {
    if (!flip) {  // w = [O][R][3][3]
      const float* src = w + (static_cast<int64_t>(o) * R + r) * 9;
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) g[i][j] = src[i * 3 + j];
    } else {  // w = [R][O][3][3] (forward weights), rotated by 180 degrees
      const float* src = w + (static_cast<int64_t>(r) * O + o) * 9;
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) g[i][j] = src[(2 - i) * 3 + (2 - j)];
    }
  }
  float t[4][3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    t[0][j] = g[0][j];
    t[1][j] = 0.5f * (g[0][j] + g[1][j] + g[2][j]);
    t[2][j] = 0.5f * (g[0][j] - g[1][j] + g[2][j]);
    t[3][j] = g[2][j];
  }
  // xi innermost: one (r, o) pair is 16 contiguous floats (4 x float4 stores).
  float v[16];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i * 4 + 0] = t[i][0];
    v[i * 4 + 1] = 0.5f * (t[i][0] + t[i][1] + t[i][2]);
    v[i * 4 + 2] = 0.5f * (t[i][0] - t[i][1] + t[i][2]);
    v[i * 4 + 3] = t[i][2];
  }
  float4* dst = reinterpret_cast<float4*>(u + idx * 16);
#pragma unroll
  for (int k = 0; k < 4; ++k) dst[k] = make_float4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
}

// Block tile: (16*OW) output channels x (32*TW) output tiles; wave (wo, wt) owns
// 16 channels x 32 tiles for all 16 Winograd positions (32 accumulator tiles).
template <int OW, int TW>
struct Tile {
  static_assert(OW * TW == kThreads / 64, "four waves per block");
  static constexpr int kOB = 16 * OW;
  static constexpr int kTB = 32 * TW;
  // LDS images keep the 16 Winograd positions of one (channel, o) / (channel, tile)
  // pair contiguous, padded to 20 floats: a 16-lane group reading 16 B per lane at
  // a 20-float stride covers all 64 banks once (ds_read_b128 conflict-free).
  static constexpr int kXS = 20;
  static constexpr int kUVec = kCB * kOB * 16 / 4 / kThreads;  // float4 of U per thread
  static constexpr int kPairs = kCB * kTB / kThreads;          // (channel, tile) per thread
};

// Global -> registers staging of one reduction chunk (U slice + raw input patches).
template <typename T>
__device__ __forceinline__ void fetch_chunk(floatx4 (&ur)[T::kUVec], float (&xr)[T::kPairs][16],
                                            const float* __restrict__ u,
                                            const float* __restrict__ x,
                                            const float* const (&xptr)[T::kPairs],
                                            const uint32_t (&vmask)[T::kPairs], int c0, int Op,
                                            int o0, int R, int W, int64_t HW, int tid) {
#pragma unroll
  for (int i = 0; i < T::kUVec; ++i) {
    const int idx = i * kThreads + tid;       // float4 index inside the chunk
    const int c = idx / (T::kOB * 4);
    const int rest = idx - c * (T::kOB * 4);  // (o, xi/4) inside one channel row
    ur[i] = *reinterpret_cast<const floatx4*>(
        u + (static_cast<int64_t>(c0 + c) * Op + o0) * 16 + rest * 4);
  }
#pragma unroll
  for (int k = 0; k < T::kPairs; ++k) {
    const int c = c0 + (k * kThreads + tid) / T::kTB;
    const uint32_t m = c < R ? vmask[k] : 0u;
    const float* xp = xptr[k] + static_cast<int64_t>(c0) * HW;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        // Branch- and select-free: out-of-image taps read a zero word, so nothing
        // consumes the loaded value before the MFMA phase that hides its latency.
        const bool ok = (m >> (i * 4 + j)) & 1u;
        xr[k][i * 4 + j] = *(ok ? xp + i * W + j : &kZeroTap);
      }
  }
}

template <int OW, int TW>
__global__ __launch_bounds__(kThreads, 2) void wino_conv_kernel(
    const float* __restrict__ x, const float* __restrict__ u, const float* __restrict__ bias,
    float* __restrict__ y, int R, int H, int W, int O, int Rp, int Op, int TH, int TW_,
    int64_t P, int tblocks, int oblocks, int splits) {
  using T = Tile<OW, TW>;
  __shared__ float Us[kCB * T::kOB * T::kXS];
  __shared__ float Vs[kCB * T::kTB * T::kXS];

  // XCD-aware bijective remap: consecutive logical blocks (same output-channel
  // block, neighbouring tiles: they share every U chunk) land on one XCD's L2.
  const int nwg = tblocks * oblocks * splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7;
  const int q = nwg >> 3, rr = nwg & 7;
  const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  const int tb = wgid % tblocks;
  const int ob = (wgid / tblocks) % oblocks;
  const int z = wgid / (tblocks * oblocks);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wo = wave % OW;
  const int wt = wave / OW;
  const int64_t t0 = static_cast<int64_t>(tb) * T::kTB;
  const int o0 = ob * T::kOB;
  const int64_t HW = static_cast<int64_t>(H) * W;
  const int tiles_per_image = TH * TW_;

  // Input-transform role: kPairs (channel, tile) pairs per thread and iteration.
  const float* xptr[T::kPairs];
  uint32_t vmask[T::kPairs];  // bit 4i+j: input pixel (i, j) of the patch is inside the image
  int vofs[T::kPairs];        // LDS offset of the pair's 16 positions
#pragma unroll
  for (int k = 0; k < T::kPairs; ++k) {
    const int pq = k * kThreads + tid;
    const int tl = pq % T::kTB;
    const int cl = pq / T::kTB;
    const int64_t t = t0 + tl;
    uint32_t m = 0;
    int64_t n = 0;
    int ty = 0, tx = 0;
    if (t < P) {
      n = t / tiles_per_image;
      const int rem = static_cast<int>(t - n * tiles_per_image);
      ty = rem / TW_;
      tx = rem - ty * TW_;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int yy = 2 * ty - 1 + i, xx = 2 * tx - 1 + j;
          if (yy >= 0 && yy < H && xx >= 0 && xx < W) m |= 1u << (i * 4 + j);
        }
    }
    vmask[k] = m;
    xptr[k] = x + (n * R + cl) * HW + static_cast<int64_t>(2 * ty - 1) * W + (2 * tx - 1);
    vofs[k] = (cl * T::kTB + tl) * T::kXS;
  }

  floatx4 acc[16][2];
#pragma unroll
  for (int xi = 0; xi < 16; ++xi) {
    acc[xi][0] = floatx4{0.f, 0.f, 0.f, 0.f};
    acc[xi][1] = floatx4{0.f, 0.f, 0.f, 0.f};
  }

  const int nchunks = Rp / kCB;
  const int c_begin = (z * nchunks / splits) * kCB;
  const int c_end = ((z + 1) * nchunks / splits) * kCB;

  // Register staging of the NEXT chunk (issued before the MFMA phase of the
  // current one, consumed after it): global latency hides behind the matrix cores.
  floatx4 ur[T::kUVec];
  float xr[T::kPairs][16];
  if (c_begin >= c_end) return;  // (never: every split owns >= 1 chunk)
  fetch_chunk<T>(ur, xr, u, x, xptr, vmask, c_begin, Op, o0, R, W, HW, tid);
  for (int c0 = c_begin; c0 < c_end; c0 += kCB) {
    // -- staged registers -> LDS: U as is, input through V = B^T d B ------------------
#pragma unroll
    for (int i = 0; i < T::kUVec; ++i) {
      const int idx = i * kThreads + tid;
      const int c = idx / (T::kOB * 4);
      const int rest = idx - c * (T::kOB * 4);
      const int o = rest >> 2;
      *reinterpret_cast<floatx4*>(&Us[(c * T::kOB + o) * T::kXS + (rest & 3) * 4]) = ur[i];
    }
#pragma unroll
    for (int k = 0; k < T::kPairs; ++k) {
      const float* d = xr[k];
      float e[4][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        e[0][j] = d[0 * 4 + j] - d[2 * 4 + j];
        e[1][j] = d[1 * 4 + j] + d[2 * 4 + j];
        e[2][j] = d[2 * 4 + j] - d[1 * 4 + j];
        e[3][j] = d[1 * 4 + j] - d[3 * 4 + j];
      }
      float4* vdst = reinterpret_cast<float4*>(&Vs[vofs[k]]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        vdst[i] = make_float4(e[i][0] - e[i][2], e[i][1] + e[i][2], e[i][2] - e[i][1],
                              e[i][1] - e[i][3]);
    }
    __syncthreads();
    // Unconditional (the last iteration re-reads its own chunk): a branch here makes
    // the compiler wait for the loads on the spot instead of behind the MFMAs.
    fetch_chunk<T>(ur, xr, u, x, xptr, vmask, min(c0 + kCB, c_end - kCB), Op, o0, R, W, HW,
                        tid);
    __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead of the MFMA phase
    // -- 16 GEMMs on the matrix cores: M[xi] += U[xi]^T V[xi] ----------------------------
    // 8 operand groups (2 channel quads x 4 position quads), each 3 x ds_read_b128
    // feeding 8 MFMAs; group g+1 is read while group g's MFMAs issue, so the LDS
    // latency hides behind the matrix pipe instead of stalling it.
    {
      const float4* ua0 =
          reinterpret_cast<const float4*>(&Us[((lane >> 4) * T::kOB + wo * 16 + (lane & 15)) *
                                              T::kXS]);
      const float4* vb0 =
          reinterpret_cast<const float4*>(&Vs[((lane >> 4) * T::kTB + wt * 32 + (lane & 15)) *
                                              T::kXS]);
      constexpr int kUQuad = 4 * T::kOB * T::kXS / 4;  // float4 stride of 4 channels in Us
      constexpr int kVQuad = 4 * T::kTB * T::kXS / 4;
      constexpr int kVHalf = 16 * T::kXS / 4;           // second 16-tile half
      floatx4 a_c = *reinterpret_cast<const floatx4*>(ua0);
      floatx4 b0_c = *reinterpret_cast<const floatx4*>(vb0);
      floatx4 b1_c = *reinterpret_cast<const floatx4*>(vb0 + kVHalf);
#pragma unroll
      for (int g = 0; g < (kCB / 4) * 4; ++g) {
        floatx4 a_n = a_c, b0_n = b0_c, b1_n = b1_c;
        if (g + 1 < (kCB / 4) * 4) {
          const int ks = (g + 1) >> 2, k = (g + 1) & 3;
          a_n = *reinterpret_cast<const floatx4*>(ua0 + ks * kUQuad + k);
          b0_n = *reinterpret_cast<const floatx4*>(vb0 + ks * kVQuad + k);
          b1_n = *reinterpret_cast<const floatx4*>(vb0 + ks * kVQuad + kVHalf + k);
        }
        const int k = g & 3;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[4 * k + e][0] =
              __builtin_amdgcn_mfma_f32_16x16x4f32(a_c[e], b0_c[e], acc[4 * k + e][0], 0, 0, 0);
          acc[4 * k + e][1] =
              __builtin_amdgcn_mfma_f32_16x16x4f32(a_c[e], b1_c[e], acc[4 * k + e][1], 0, 0, 0);
        }
        a_c = a_n;
        b0_c = b0_n;
        b1_c = b1_n;
      }
      // Pin the interleave for the machine scheduler: group 0's reads, then per group
      // the next group's 3 LDS reads ahead of this group's 8 MFMAs.
      __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
#pragma unroll
      for (int g = 0; g < (kCB / 4) * 4; ++g) {
        if (g + 1 < (kCB / 4) * 4) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
      }
    }
    __syncthreads();
  }

  // -- output transform Y = A^T M A, straight from the accumulators ---------------------
  // Split-reduction partials go to slab z of the workspace (bias added by the reducer).
  float* ydst = y + static_cast<int64_t>(z) * (P / tiles_per_image) * O * HW;
  const bool add_bias = bias != nullptr && splits == 1;
  const bool even_w = (W & 1) == 0;
#pragma unroll
  for (int ph = 0; ph < 2; ++ph) {
    const int64_t tp = t0 + wt * 32 + ph * 16 + (lane & 15);
    if (tp >= P) continue;
    const int64_t pn = tp / tiles_per_image;
    const int prem = static_cast<int>(tp - pn * tiles_per_image);
    const int pty = prem / TW_;
    const int py = pty * 2;
    const int px = (prem - pty * TW_) * 2;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = o0 + wo * 16 + (lane >> 4) * 4 + r;
      if (o >= O) continue;
      float m[16];
#pragma unroll
      for (int xi = 0; xi < 16; ++xi) m[xi] = acc[xi][ph][r];
      float s[2][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s[0][j] = m[0 * 4 + j] + m[1 * 4 + j] + m[2 * 4 + j];
        s[1][j] = m[1 * 4 + j] - m[2 * 4 + j] - m[3 * 4 + j];
      }
      const float b = add_bias ? bias[o] : 0.f;
      float* yp = ydst + (pn * O + o) * HW + static_cast<int64_t>(py) * W + px;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (py + i >= H) break;
        const float v0 = s[i][0] + s[i][1] + s[i][2] + b;
        const float v1 = s[i][1] - s[i][2] - s[i][3] + b;
        if (even_w) {
          *reinterpret_cast<float2*>(yp + i * W) = make_float2(v0, v1);
        } else {
          yp[i * W] = v0;
          if (px + 1 < W) yp[i * W + 1] = v1;
        }
      }
    }
  }
}

// y[i] = sum_z ws[z][i] (+ bias[o]) over the split-reduction partial slabs.
__global__ void wino_split_reduce_kernel(const float* __restrict__ ws,
                                         const float* __restrict__ bias, float* __restrict__ y,
                                         int64_t numel, int64_t hw, int O, int splits) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= numel) return;
  float v = bias ? bias[(i / hw) % O] : 0.f;
  for (int z = 0; z < splits; ++z) v += ws[z * numel + i];
  y[i] = v;
}

template <int OW, int TW>
void launch_variant(const float* x, const float* u, const float* bias, float* y, float* ws,
                    int64_t n, int64_t R, int64_t H, int64_t W, int64_t O, int splits,
                    hipStream_t stream) {
  using T = Tile<OW, TW>;
  const int64_t Rp = wino_pad_reduction(R);
  const int64_t Op = wino_pad_output(O);
  const int64_t th = (H + 1) / 2, tw = (W + 1) / 2;
  const int64_t P = n * th * tw;
  const int tblocks = static_cast<int>((P + T::kTB - 1) / T::kTB);
  const int oblocks = static_cast<int>((O + T::kOB - 1) / T::kOB);
  const int64_t nwg = static_cast<int64_t>(tblocks) * oblocks * splits;
  hipLaunchKernelGGL((wino_conv_kernel<OW, TW>), dim3(static_cast<unsigned>(nwg)),
                     dim3(kThreads), 0, stream, x, u, bias, splits > 1 ? ws : y,
                     static_cast<int>(R), static_cast<int>(H), static_cast<int>(W),
                     static_cast<int>(O), static_cast<int>(Rp), static_cast<int>(Op),
                     static_cast<int>(th), static_cast<int>(tw), P, tblocks, oblocks, splits);
  if (splits > 1) {
    const int64_t numel = n * O * H * W;
    hipLaunchKernelGGL(wino_split_reduce_kernel, dim3(static_cast<unsigned>((numel + 255) / 256)),
                       dim3(256), 0, stream, ws, bias, y, numel, H * W, static_cast<int>(O),
                       splits);
  }
}


// ---------------------------------------------------------------------------------------
// Variant 2: 64 output channels x 64 tiles per workgroup of 8 waves, ONE workgroup per
// CU (two waves per SIMD), LDS double-buffered so one barrier per channel chunk
// suffices, and the staging of chunk c+1 (global -> registers -> input transform ->
// LDS) cut into small slots that ride between the MFMAs of chunk c.
//
// Why: with two 4-wave workgroups per CU (variants 0/1) both blocks' MFMA phases and
// both blocks' staging phases fall into step through their barriers, so the matrix
// pipe idles during staging (rocprofv3: SQ_VALU_MFMA_BUSY_CYCLES = 41 % of the SIMD
// cycles on 40x64x192^2).  Here staging never has a phase of its own: an f32 MFMA
// holds the SIMD's issue for 8 of its 32 cycles, the rest carries the loads, the LDS
// stores and the transform, and the partner wave on the SIMD fills what is left.
//
// Wave (wo, wt) = (wave & 1, wave >> 1) owns 32 channels x 16 tiles for all 16
// Winograd positions (2 accumulator tiles of 16 x 16 per position, 128 registers).
// Each (channel quad, position quad) operand group is 3 ds_read_b128 feeding 8 MFMAs.
constexpr int kDBT = 64;                      // tiles per workgroup
constexpr int kDBO = 64;                      // output channels per workgroup
constexpr int kDBThreads = 512;
constexpr int kDBImg = kCB * 64 * 20;         // floats per LDS operand image

struct DbStage {
  floatx4 ur[4];   // U of the staged chunk: channel 2i + (tid >> 8), float4 (tid & 255)
  float xr[16];    // raw 4x4 patch: channel tid >> 6, tile tid & 63
};

struct DbCtx {
  float* Us_next;          // LDS images being filled (the other buffer)
  float* Vs_next;
  const float* u_next;     // this thread's U float4 in channel row 0 of the prefetch
  const float* xp_next;    // this thread's (channel, image) plane of the prefetch
  int64_t u_row;           // 2 * Op * 16: float stride between this thread's U rows
  uint32_t vmask;
  int tid;
};

// Staging work of one pipeline step, in slots (slot S runs after MFMA 2S + 1), all on
// the staging registers in place: zero the padding taps (S 0-3), B^T d by columns
// (S 4-7), (B^T d) B rows -> LDS (S 8-11); then the patch registers are free and the
// x prefetch of the chunk after next goes out early (S 12-19, latency-critical: it
// misses to HBM), then the U stores (S 20-23) and the U prefetch (S 24-27, L2-hot).
template <int S>
__device__ __forceinline__ void db_slot(DbStage& s, const DbCtx& c,
                                        const uint32_t (&toff)[16]) {
  float* d = s.xr;
  if constexpr (S < 4) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      d[S * 4 + j] = (c.vmask >> (S * 4 + j)) & 1u ? d[S * 4 + j] : 0.f;
  } else if constexpr (S < 8) {
    constexpr int j = S - 4;
    const float e0 = d[0 * 4 + j] - d[2 * 4 + j];
    const float e1 = d[1 * 4 + j] + d[2 * 4 + j];
    const float e2 = d[2 * 4 + j] - d[1 * 4 + j];
    const float e3 = d[1 * 4 + j] - d[3 * 4 + j];
    d[0 * 4 + j] = e0;
    d[1 * 4 + j] = e1;
    d[2 * 4 + j] = e2;
    d[3 * 4 + j] = e3;
  } else if constexpr (S < 12) {
    constexpr int i = S - 8;
    floatx4* vdst =
        reinterpret_cast<floatx4*>(&c.Vs_next[((c.tid >> 6) * 64 + (c.tid & 63)) * 20]);
    vdst[i] = floatx4{d[i * 4 + 0] - d[i * 4 + 2], d[i * 4 + 1] + d[i * 4 + 2],
                      d[i * 4 + 2] - d[i * 4 + 1], d[i * 4 + 1] - d[i * 4 + 3]};
  } else if constexpr (S < 20) {  // x prefetch, two taps per slot
    constexpr int t = S - 12;
    s.xr[2 * t] = c.xp_next[toff[2 * t]];
    s.xr[2 * t + 1] = c.xp_next[toff[2 * t + 1]];
  } else if constexpr (S < 24) {
    constexpr int i = S - 20;
    *reinterpret_cast<floatx4*>(
        &c.Us_next[((2 * i + (c.tid >> 8)) * 64 + ((c.tid & 255) >> 2)) * 20 +
                   (c.tid & 3) * 4]) = s.ur[i];
  } else if constexpr (S < 28) {  // U prefetch
    s.ur[S - 24] = *reinterpret_cast<const floatx4*>(c.u_next + (S - 24) * c.u_row);
  }
}

// Fake use of the prefetch registers after the loop (see wd_keep).
__device__ __forceinline__ void db_keep(const DbStage& s) {
#pragma unroll
  for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(s.ur[i]));
#pragma unroll
  for (int i = 0; i < 16; ++i) asm volatile("" ::"v"(s.xr[i]));
}

__device__ __forceinline__ void db_fetch(DbStage& s, const float* __restrict__ u,
                                         const float* __restrict__ x,
                                         const uint32_t (&toff)[16], int64_t tile_base, int c0,
                                         int R, int Op, int o0, int64_t HW, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
    s.ur[i] = *reinterpret_cast<const floatx4*>(
        u + (static_cast<int64_t>(c0 + 2 * i + (tid >> 8)) * Op + o0) * 16 + (tid & 255) * 4);
  // Channels >= R (padding of the last chunk) re-read channel R-1: their U rows are
  // zero, any finite value works.
  const float* p =
      x + tile_base + static_cast<int64_t>(min(c0 + (tid >> 6), R - 1)) * HW;
#pragma unroll
  for (int ij = 0; ij < 16; ++ij) s.xr[ij] = p[toff[ij]];
}

__device__ __forceinline__ void db_stage_all(const DbStage& s, float* Us, float* Vs,
                                             uint32_t vmask, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
    *reinterpret_cast<floatx4*>(
        &Us[((2 * i + (tid >> 8)) * 64 + ((tid & 255) >> 2)) * 20 + (tid & 3) * 4]) = s.ur[i];
  float d[16];
#pragma unroll
  for (int ij = 0; ij < 16; ++ij) d[ij] = (vmask >> ij) & 1u ? s.xr[ij] : 0.f;
  float e[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    e[0][j] = d[0 * 4 + j] - d[2 * 4 + j];
    e[1][j] = d[1 * 4 + j] + d[2 * 4 + j];
    e[2][j] = d[2 * 4 + j] - d[1 * 4 + j];
    e[3][j] = d[1 * 4 + j] - d[3 * 4 + j];
  }
  floatx4* vdst = reinterpret_cast<floatx4*>(&Vs[((tid >> 6) * 64 + (tid & 63)) * 20]);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    vdst[i] = floatx4{e[i][0] - e[i][2], e[i][1] + e[i][2], e[i][2] - e[i][1],
                      e[i][1] - e[i][3]};
}

template <int G, int M>
__device__ __forceinline__ void db_group_tail(floatx4 (&acc)[16][2], DbStage& s,
                                              const DbCtx& c, const uint32_t (&toff)[16],
                                              const floatx4& a0, const floatx4& a1,
                                              const floatx4& b0) {
  if constexpr (M < 8) {
    constexpr int ep = M >> 1;
    constexpr int i = M & 1;
    acc[4 * (G & 3) + ep][i] = __builtin_amdgcn_mfma_f32_16x16x4f32(
        (i ? a1 : a0)[ep], b0[ep], acc[4 * (G & 3) + ep][i], 0, 0, 0);
    if constexpr ((M & 1) == 1) db_slot<(G * 8 + M) / 2>(s, c, toff);
    __builtin_amdgcn_sched_barrier(0);
    db_group_tail<G, M + 1>(acc, s, c, toff, a0, a1, b0);
  }
}

template <int G>
__device__ __forceinline__ void db_groups(floatx4 (&acc)[16][2], DbStage& s, const DbCtx& c,
                                          const uint32_t (&toff)[16], const floatx4* ua,
                                          const floatx4* vb, floatx4 a0, floatx4 a1,
                                          floatx4 b0) {
  if constexpr (G < 8) {
    constexpr int kQuad = 4 * 64 * 20 / 4;  // float4 stride of 4 channels
    constexpr int kHalf = 16 * 20 / 4;      // float4 stride of 16 rows (second sub-tile)
    floatx4 na0 = a0, na1 = a1, nb0 = b0;
    if constexpr (G + 1 < 8) {
      constexpr int off = ((G + 1) >> 2) * kQuad + ((G + 1) & 3);
      na0 = ua[off];
      na1 = ua[off + kHalf];
      nb0 = vb[off];
    }
    db_group_tail<G, 0>(acc, s, c, toff, a0, a1, b0);
    db_groups<G + 1>(acc, s, c, toff, ua, vb, na0, na1, nb0);
  }
}

// One pipeline step: the 64 MFMAs of buffer `buf`, with the staging of the prefetched
// chunk into buffer buf^1 and the prefetch of the chunk after it in their issue gaps.
// (A runtime buffer index: the pinned slot order already orders the staging stores and
// the operand reads, and a single-step loop body keeps the accumulators in place.)
__device__ __forceinline__ void db_step(floatx4 (&acc)[16][2], DbStage& s, float* lds, int buf,
                                        const float* __restrict__ u,
                                        const float* __restrict__ x,
                                        const uint32_t (&toff)[16], int64_t tile_base,
                                        uint32_t vmask, int next_c, int R, int Op, int o0,
                                        int64_t HW, int tid, int lane, int wo, int wt) {
  DbCtx c;
  c.Us_next = lds + (buf ^ 1) * 2 * kDBImg;
  c.Vs_next = c.Us_next + kDBImg;
  c.u_row = static_cast<int64_t>(Op) * 32;
  c.u_next = u + (static_cast<int64_t>(next_c + (tid >> 8)) * Op + o0) * 16 + (tid & 255) * 4;
  c.xp_next = x + tile_base + static_cast<int64_t>(min(next_c + (tid >> 6), R - 1)) * HW;
  c.vmask = vmask;
  c.tid = tid;

  const float* Us = lds + buf * 2 * kDBImg;
  const float* Vs = Us + kDBImg;
  const floatx4* ua = reinterpret_cast<const floatx4*>(
      &Us[((lane >> 4) * 64 + wo * 32 + (lane & 15)) * 20]);
  const floatx4* vb = reinterpret_cast<const floatx4*>(
      &Vs[((lane >> 4) * 64 + wt * 16 + (lane & 15)) * 20]);
  constexpr int kHalf = 16 * 20 / 4;
  db_groups<0>(acc, s, c, toff, ua, vb, ua[0], ua[kHalf], vb[0]);
}

__global__ __launch_bounds__(kDBThreads, 1) void wino_conv_db_kernel(
    const float* __restrict__ x, const float* __restrict__ u, const float* __restrict__ bias,
    float* __restrict__ y, int R, int H, int W, int O, int Rp, int Op, int TH, int TW_,
    int64_t P, int tblocks, int oblocks, int splits) {
  __shared__ float lds[2 * 2 * kDBImg];  // [buffer][U | V][8 channels][64][20]: 160 KiB

  const int nwg = tblocks * oblocks * splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7;
  const int qq = nwg >> 3, rr = nwg & 7;
  const int wgid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int tb = wgid % tblocks;
  const int ob = (wgid / tblocks) % oblocks;
  const int z = wgid / (tblocks * oblocks);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wo = wave & 1;
  const int wt = wave >> 1;
  const int64_t t0 = static_cast<int64_t>(tb) * kDBT;
  const int o0 = ob * kDBO;
  const int64_t HW = static_cast<int64_t>(H) * W;
  const int tiles_per_image = TH * TW_;

  // Staging role: tile t0 + (tid & 63), channel tid >> 6 of each chunk.  Padding taps
  // read the tile's always-valid pixel (2ty, 2tx) and are zeroed through `vmask`.
  uint32_t vmask = 0;
  uint32_t toff[16];
  int64_t tile_base = 0;
  {
    const int64_t t = t0 + (tid & 63);
    int ty = 0, tx = 0;
    if (t < P) {
      const int64_t n = t / tiles_per_image;
      const int rem = static_cast<int>(t - n * tiles_per_image);
      ty = rem / TW_;
      tx = rem - ty * TW_;
      tile_base = n * R * HW;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int yy = 2 * ty - 1 + i, xx = 2 * tx - 1 + j;
        const bool ok = t < P && yy >= 0 && yy < H && xx >= 0 && xx < W;
        vmask |= static_cast<uint32_t>(ok) << (i * 4 + j);
        toff[i * 4 + j] = static_cast<uint32_t>(ok ? yy * W + xx : 2 * ty * W + 2 * tx);
      }
  }

  floatx4 acc[16][2];
#pragma unroll
  for (int xi = 0; xi < 16; ++xi) {
    acc[xi][0] = floatx4{0.f, 0.f, 0.f, 0.f};
    acc[xi][1] = floatx4{0.f, 0.f, 0.f, 0.f};
  }

  const int nchunks = Rp / kCB;
  const int c_begin = (z * nchunks / splits) * kCB;
  const int c_end = ((z + 1) * nchunks / splits) * kCB;

  DbStage s;
  db_fetch(s, u, x, toff, tile_base, c_begin, R, Op, o0, HW, tid);
  db_stage_all(s, lds, lds + kDBImg, vmask, tid);
  __syncthreads();
  db_fetch(s, u, x, toff, tile_base, min(c_begin + kCB, c_end - kCB), R, Op, o0, HW, tid);
  // The last step stages a clamped (repeated) chunk into the idle buffer: harmless.
  for (int c0 = c_begin; c0 < c_end; c0 += kCB) {
    db_step(acc, s, lds, ((c0 - c_begin) / kCB) & 1, u, x, toff, tile_base, vmask,
            min(c0 + 2 * kCB, c_end - kCB), R, Op, o0, HW, tid, lane, wo, wt);
    __syncthreads();
  }
  db_keep(s);

  // -- output transform Y = A^T M A from the accumulators ------------------------------
  // Lane (wt*16 + j) holds tile t0 + wt*16 + j: a 2x2 output patch per channel.  When
  // W % 4 == 0 and H is even, tiles 2m and 2m+1 are horizontal neighbours; lanes 2m
  // and 2m+1 trade one patch row (DPP quad_perm [1,0,3,2]) so each stores one 16-byte
  // row segment instead of two 8-byte ones: the epilogue is store-issue bound.
  float* ydst = y + static_cast<int64_t>(z) * (P / tiles_per_image) * O * HW;
  const bool add_bias = bias != nullptr && splits == 1;
  const int64_t tp = t0 + wt * 16 + (lane & 15);
  const bool paired = (W & 3) == 0 && (H & 1) == 0;
  if (tp >= P) return;  // (paired: P is even and tile pairs are valid together)
  const int64_t pn = tp / tiles_per_image;
  const int prem = static_cast<int>(tp - pn * tiles_per_image);
  const int pty = prem / TW_;
  const int py = pty * 2;
  const int px = (prem - pty * TW_) * 2;
  const bool odd = lane & 1;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = o0 + wo * 32 + i * 16 + (lane >> 4) * 4 + r;
      float m[16];
#pragma unroll
      for (int xi = 0; xi < 16; ++xi) m[xi] = acc[xi][i][r];
      float sr[2][4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        sr[0][c] = m[0 * 4 + c] + m[1 * 4 + c] + m[2 * 4 + c];
        sr[1][c] = m[1 * 4 + c] - m[2 * 4 + c] - m[3 * 4 + c];
      }
      const float b = add_bias && o < O ? bias[o] : 0.f;
      float v[2][2];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        v[a][0] = sr[a][0] + sr[a][1] + sr[a][2] + b;
        v[a][1] = sr[a][1] - sr[a][2] - sr[a][3] + b;
      }
      if (paired) {
        // even lane sends row 1, odd lane sends row 0 (all lanes take part in the DPP)
        const float s0 = odd ? v[0][0] : v[1][0];
        const float s1 = odd ? v[0][1] : v[1][1];
        const float r0 = __int_as_float(
            __builtin_amdgcn_mov_dpp(__float_as_int(s0), 0xB1, 0xF, 0xF, false));
        const float r1 = __int_as_float(
            __builtin_amdgcn_mov_dpp(__float_as_int(s1), 0xB1, 0xF, 0xF, false));
        if (o >= O) continue;
        const floatx4 out = odd ? floatx4{r0, r1, v[1][0], v[1][1]}
                                : floatx4{v[0][0], v[0][1], r0, r1};
        float* yp = ydst + (pn * O + o) * HW + static_cast<int64_t>(py + odd) * W +
                    (px - 2 * odd);
        *reinterpret_cast<floatx4*>(yp) = out;
      } else {
        if (o >= O) continue;
        float* yp = ydst + (pn * O + o) * HW + static_cast<int64_t>(py) * W + px;
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          if (py + a >= H) break;
          if ((W & 1) == 0) {
            *reinterpret_cast<float2*>(yp + a * W) = make_float2(v[a][0], v[a][1]);
          } else {
            yp[a * W] = v[a][0];
            if (px + 1 < W) yp[a * W + 1] = v[a][1];
          }
        }
      }
    }
}

void launch_db(const float* x, const float* u, const float* bias, float* y, float* ws,
               int64_t n, int64_t R, int64_t H, int64_t W, int64_t O, int splits,
               hipStream_t stream) {
  const int64_t Rp = wino_pad_reduction(R);
  const int64_t Op = wino_pad_output(O);
  const int64_t th = (H + 1) / 2, tw = (W + 1) / 2;
  const int64_t P = n * th * tw;
  const int tblocks = static_cast<int>((P + kDBT - 1) / kDBT);
  const int oblocks = static_cast<int>((O + kDBO - 1) / kDBO);
  const int64_t nwg = static_cast<int64_t>(tblocks) * oblocks * splits;
  hipLaunchKernelGGL(wino_conv_db_kernel, dim3(static_cast<unsigned>(nwg)), dim3(kDBThreads),
                     0, stream, x, u, bias, splits > 1 ? ws : y, static_cast<int>(R),
                     static_cast<int>(H), static_cast<int>(W), static_cast<int>(O),
                     static_cast<int>(Rp), static_cast<int>(Op), static_cast<int>(th),
                     static_cast<int>(tw), P, tblocks, oblocks, splits);
  if (splits > 1) {
    const int64_t numel = n * O * H * W;
    hipLaunchKernelGGL(wino_split_reduce_kernel, dim3(static_cast<unsigned>((numel + 255) / 256)),
                       dim3(256), 0, stream, ws, bias, y, numel, H * W, static_cast<int>(O),
                       splits);
  }
}


// ---------------------------------------------------------------------------------------
// Weight gradient.  With V_t = B^T d_t B (input patch of tile t) and
// M'_t = A dY_t A^T (output-gradient tile lifted to the 4x4 Winograd domain):
//   dU[xi][c][k] = sum_t V_t[xi][c] * M'_t[xi][k]     16 GEMMs reducing over tiles
//   dW[k][c]     = G^T dU[k][c] G                     (in-register, per lane)
// Block: 64 input channels x 32 output channels; wave w owns channels 16w..16w+15
// for both 16-wide k halves and all 16 positions.  The tile range is split over
// gridDim (deterministic: per-split partial dW slabs, summed by a reduce kernel).
constexpr int kWC = 64;   // input channels per block
constexpr int kWK = 32;   // output channels per block
constexpr int kWT = 8;    // tiles per main-loop iteration
constexpr int kWS = 20;   // padded LDS stride of one (tile, channel) position vector

// Registers <- global for one wgrad iteration: two 4x4 input patches and one 2x2
// output-gradient patch per thread.  Out-of-range taps load from the tensor base
// and are zeroed later through `xmask` / `ymask` (applied in the staging phase, so
// nothing consumes a load before the MFMA phase that hides its latency).
__device__ __forceinline__ void wgrad_fetch(float (&xr)[2][16], float (&yr)[4], uint32_t& xmask,
                                            uint32_t& ymask, const float* __restrict__ x,
                                            const float* __restrict__ dy, int64_t it, int xt,
                                            int xc, int yt, int yk, int c0, int k0, int C, int K,
                                            int H, int W, int TW_, int tiles_per_image,
                                            int64_t P, int64_t HW) {
  xmask = 0;
  ymask = 0;
  {
    // 32-bit tile arithmetic (the host guarantees P < 2^31).
    const int t = static_cast<int>(it) * kWT + xt;
    const bool tv = t < P;
    const int tt = tv ? t : 0;
    const int n = tt / tiles_per_image;
    const int rem = tt - n * tiles_per_image;
    const int ty = rem / TW_;
    const int tx = rem - ty * TW_;
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const int c = c0 + xc + pr * 32;
      const bool cv = tv && c < C;
      const float* xp =
          x + (static_cast<int64_t>(n) * C + c) * HW + static_cast<int64_t>(2 * ty - 1) * W +
          (2 * tx - 1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool rok = cv && 2 * ty - 1 + i >= 0 && 2 * ty - 1 + i < H;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bool ok = rok && 2 * tx - 1 + j >= 0 && 2 * tx - 1 + j < W;
          xmask |= static_cast<uint32_t>(ok) << (pr * 16 + i * 4 + j);
          xr[pr][i * 4 + j] = *(ok ? xp + i * W + j : x);
        }
      }
    }
  }
  {
    const int t = static_cast<int>(it) * kWT + yt;
    const bool tv = t < P;
    const int tt = tv ? t : 0;
    const int n = tt / tiles_per_image;
    const int rem = tt - n * tiles_per_image;
    const int ty = rem / TW_;
    const int tx = rem - ty * TW_;
    const int k = k0 + yk;
    const bool kv = tv && k < K;
    const float* yp =
        dy + (static_cast<int64_t>(n) * K + k) * HW + static_cast<int64_t>(2 * ty) * W + 2 * tx;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bool ok = kv && 2 * ty + i < H && 2 * tx + j < W;
        ymask |= static_cast<uint32_t>(ok) << (i * 2 + j);
        yr[i * 2 + j] = *(ok ? yp + i * W + j : dy);
      }
  }
}

// Weight-gradient store: overwrite, or add into an existing .grad (gradient-accumulation
// fusion, ops/gradacc.py: no separate `grad += new` pass per micro-batch).
__device__ __forceinline__ void wg_store(float* o, float v, bool accum) {
  *o = accum ? *o + v : v;
}

__global__ __launch_bounds__(kThreads, 2) void wino_wgrad_kernel(
    const float* __restrict__ x, const float* __restrict__ dy, float* __restrict__ dw, int C,
    int K, int H, int W, int TH, int TW_, int64_t P, int cblocks, int kblocks, int splits,
    bool accum) {
  __shared__ float Vs[kWT * kWC * kWS];
  __shared__ float Ms[kWT * kWK * kWS];

  const int nwg = cblocks * kblocks * splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7;
  const int q = nwg >> 3, rr = nwg & 7;
  const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  const int cb = wgid % cblocks;
  const int kb = (wgid / cblocks) % kblocks;
  const int z = wgid / (cblocks * kblocks);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int c0 = cb * kWC;
  const int k0 = kb * kWK;
  const int64_t HW = static_cast<int64_t>(H) * W;
  const int tiles_per_image = TH * TW_;
  const int64_t iters_total = (P + kWT - 1) / kWT;
  const int64_t it_begin = z * iters_total / splits;
  const int64_t it_end = (z + 1) * iters_total / splits;

  // roles: two (channel, tile) input pairs and one (k, tile) gradient pair per thread
  const int xt = tid % kWT;          // tile slot of both input pairs
  const int xc = tid / kWT;          // channel of pair 0 (pair 1: + 32)
  const int yt = tid % kWT;
  const int yk = tid / kWT;          // 0..31

  floatx4 acc[16][2];
#pragma unroll
  for (int xi = 0; xi < 16; ++xi) {
    acc[xi][0] = floatx4{0.f, 0.f, 0.f, 0.f};
    acc[xi][1] = floatx4{0.f, 0.f, 0.f, 0.f};
  }

  float xr[2][16];
  float yr[4];
  uint32_t xmask = 0, ymask = 0;
  if (it_begin < it_end)
    wgrad_fetch(xr, yr, xmask, ymask, x, dy, it_begin, xt, xc, yt, yk, c0, k0, C, K, H, W, TW_,
                tiles_per_image, P, HW);
  for (int64_t it = it_begin; it < it_end; ++it) {
    // -- stage: V = B^T d B for both input pairs, M' = A dY A^T for the gradient pair ---
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      float d[16];
#pragma unroll
      for (int b = 0; b < 16; ++b) d[b] = (xmask >> (pr * 16 + b)) & 1u ? xr[pr][b] : 0.f;
      float e[4][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        e[0][j] = d[0 * 4 + j] - d[2 * 4 + j];
        e[1][j] = d[1 * 4 + j] + d[2 * 4 + j];
        e[2][j] = d[2 * 4 + j] - d[1 * 4 + j];
        e[3][j] = d[1 * 4 + j] - d[3 * 4 + j];
      }
      floatx4* vdst = reinterpret_cast<floatx4*>(&Vs[(xt * kWC + xc + pr * 32) * kWS]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        vdst[i] = floatx4{e[i][0] - e[i][2], e[i][1] + e[i][2], e[i][2] - e[i][1],
                          e[i][1] - e[i][3]};
    }
    {
#pragma unroll
      for (int b = 0; b < 4; ++b) yr[b] = (ymask >> b) & 1u ? yr[b] : 0.f;
      float r[4][2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        r[0][j] = yr[0 * 2 + j];
        r[1][j] = yr[0 * 2 + j] + yr[1 * 2 + j];
        r[2][j] = yr[0 * 2 + j] - yr[1 * 2 + j];
        r[3][j] = -yr[1 * 2 + j];
      }
      floatx4* mdst = reinterpret_cast<floatx4*>(&Ms[(yt * kWK + yk) * kWS]);
#pragma unroll
      for (int a = 0; a < 4; ++a)
        mdst[a] = floatx4{r[a][0], r[a][0] + r[a][1], r[a][0] - r[a][1], -r[a][1]};
    }
    __syncthreads();
    wgrad_fetch(xr, yr, xmask, ymask, x, dy, it + 1 < it_end ? it + 1 : it, xt, xc, yt, yk, c0, k0, C, K, H,
                W, TW_, tiles_per_image, P, HW);
    __builtin_amdgcn_sched_barrier(0);
    {
      // same software-pipelined operand groups as the forward kernel
      const floatx4* va0 =
          reinterpret_cast<const floatx4*>(&Vs[((lane >> 4) * kWC + wave * 16 + (lane & 15)) * kWS]);
      const floatx4* mb0 = reinterpret_cast<const floatx4*>(&Ms[((lane >> 4) * kWK + (lane & 15)) * kWS]);
      constexpr int kVQuad = 4 * kWC * kWS / 4;
      constexpr int kMQuad = 4 * kWK * kWS / 4;
      constexpr int kMHalf = 16 * kWS / 4;
      constexpr int kGroups = (kWT / 4) * 4;
      floatx4 a_c = va0[0], b0_c = mb0[0], b1_c = mb0[kMHalf];
#pragma unroll
      for (int g = 0; g < kGroups; ++g) {
        floatx4 a_n = a_c, b0_n = b0_c, b1_n = b1_c;
        if (g + 1 < kGroups) {
          const int ks = (g + 1) >> 2, k = (g + 1) & 3;
          a_n = va0[ks * kVQuad + k];
          b0_n = mb0[ks * kMQuad + k];
          b1_n = mb0[ks * kMQuad + kMHalf + k];
        }
        const int k = g & 3;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[4 * k + e][0] =
              __builtin_amdgcn_mfma_f32_16x16x4f32(a_c[e], b0_c[e], acc[4 * k + e][0], 0, 0, 0);
          acc[4 * k + e][1] =
              __builtin_amdgcn_mfma_f32_16x16x4f32(a_c[e], b1_c[e], acc[4 * k + e][1], 0, 0, 0);
        }
        a_c = a_n;
        b0_c = b0_n;
        b1_c = b1_n;
      }
      __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
#pragma unroll
      for (int g = 0; g < kGroups; ++g) {
        if (g + 1 < kGroups) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
      }
    }
    __syncthreads();
  }

  // -- dW = G^T dU G per (c, k) pair; partial slab z of [splits][K][C][9] --------------
  float* out = dw + static_cast<int64_t>(z) * K * C * 9;
#pragma unroll
  for (int ph = 0; ph < 2; ++ph) {
    const int k = k0 + ph * 16 + (lane & 15);
    if (k >= K) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = c0 + wave * 16 + (lane >> 4) * 4 + r;
      if (c >= C) continue;
      float u[16];
#pragma unroll
      for (int xi = 0; xi < 16; ++xi) u[xi] = acc[xi][ph][r];
      float t[3][4];
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const float s12 = 0.5f * (u[1 * 4 + b] + u[2 * 4 + b]);
        t[0][b] = u[0 * 4 + b] + s12;
        t[1][b] = 0.5f * (u[1 * 4 + b] - u[2 * 4 + b]);
        t[2][b] = s12 + u[3 * 4 + b];
      }
      float* o = out + (static_cast<int64_t>(k) * C + c) * 9;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const float s12 = 0.5f * (t[i][1] + t[i][2]);
        wg_store(o + i * 3 + 0, t[i][0] + s12, accum);
        wg_store(o + i * 3 + 1, 0.5f * (t[i][1] - t[i][2]), accum);
        wg_store(o + i * 3 + 2, s12 + t[i][3], accum);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// Weight gradient, variant 2: the structure of the forward variant 2 applied to
//   dU[xi][c][k] = sum_t V_t[xi][c] * M'_t[xi][k]
// 64 input channels x 64 output channels per 8-wave workgroup (one per CU), 8 tiles per
// pipeline step, LDS double-buffered, staging interleaved into the MFMA stream.  Wave
// (wc, wk) = (wave & 1, wave >> 1) owns 32 channels x 16 output channels for all 16
// positions.  Staging role of a thread: tile slot t = tid & 7 of the step, channel
// (and output channel) tid >> 3.  In LDS, tile row t stores channel c at c ^ t: the
// 8 lanes of one ds_write_b128 group (8 tiles, one channel) then hit 8 different bank
// groups, while the MFMA reads (16 consecutive channels of one tile) stay a conflict-free
// permutation of their 16-channel group.
constexpr int kWDT = 8;                        // tiles per pipeline step
constexpr int kWDImg = kWDT * 64 * 20;         // floats per LDS operand image

struct WdStage {
  float xr[16];      // 4x4 input patch of (tile slot, channel), zero-padded; transformed
                     // in place while it is staged
  float yr[4];       // 2x2 output-gradient patch of (tile slot, output channel)
};

// a / d for 0 <= a < 2^24 through a float reciprocal (exact after one correction).
__device__ __forceinline__ int wd_div(int a, int d, float inv) {
  int q = static_cast<int>(static_cast<float>(a) * inv);
  const int r = a - q * d;
  q += (r >= d) - (r < 0);
  return q;
}

// Per-thread tile geometry of one step: image, top-left input pixel of the 4x4 patch.
struct WdGeo {
  int n, y0, x0;
  bool tv;
};

struct WdShape {
  int C, K, H, W, TW_, tpi;
  float inv_tw, inv_tpi;
  int64_t P, HW;
};

__device__ __forceinline__ WdGeo wd_geo(int64_t t, const WdShape& sh) {
  WdGeo g;
  g.tv = t >= 0 && t < sh.P;
  const int tt = g.tv ? static_cast<int>(t) : 0;
  g.n = wd_div(tt, sh.tpi, sh.inv_tpi);
  const int rem = tt - g.n * sh.tpi;
  const int ty = wd_div(rem, sh.TW_, sh.inv_tw);
  g.y0 = 2 * ty - 1;
  g.x0 = 2 * (rem - ty * sh.TW_) - 1;
  return g;
}

// Global -> registers for one step, in parts: part i < 4 loads input patch row i
// (part 0 also resets the mask), part 4 the 2x2 output-gradient patch.
template <int PART>
__device__ __forceinline__ void wd_fetch_part(WdStage& s, const WdGeo& g,
                                              const float* __restrict__ x,
                                              const float* __restrict__ dy, int c, int k,
                                              const WdShape& sh) {
  // Padding taps, padding tiles and padding channels load the zero word kZeroTap.
  if constexpr (PART < 4) {
    const bool cv = g.tv && c < sh.C;
    const float* xp = x + (static_cast<int64_t>(g.n) * sh.C + (cv ? c : 0)) * sh.HW;
    const int yy = g.y0 + PART;
    const bool rok = cv && yy >= 0 && yy < sh.H;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int xx = g.x0 + j;
      const bool ok = rok && xx >= 0 && xx < sh.W;
      s.xr[PART * 4 + j] = *(ok ? xp + yy * sh.W + xx : &kZeroTap);
    }
  } else {
    const bool kv = g.tv && k < sh.K;
    const float* yp = dy + (static_cast<int64_t>(g.n) * sh.K + (kv ? k : 0)) * sh.HW;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int yy = g.y0 + 1 + i, xx = g.x0 + 1 + j;
        const bool ok = kv && yy < sh.H && xx < sh.W;
        s.yr[i * 2 + j] = *(ok ? yp + yy * sh.W + xx : &kZeroTap);
      }
  }
}

// Fake use of the prefetch registers on a loop exit: otherwise MachineSink moves the
// prefetch loads of a step past the exit branch into the next step (it sees them used
// only there), which serialises them and doubles the live patch registers.
__device__ __forceinline__ void wd_keep(const WdStage& s) {
#pragma unroll
  for (int i = 0; i < 16; ++i) asm volatile("" ::"v"(s.xr[i]));
#pragma unroll
  for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(s.yr[i]));
}

__device__ __forceinline__ void wd_fetch(WdStage& s, int64_t t, const float* __restrict__ x,
                                         const float* __restrict__ dy, int c, int k,
                                         const WdShape& sh) {
  const WdGeo g = wd_geo(t, sh);
  wd_fetch_part<0>(s, g, x, dy, c, k, sh);
  wd_fetch_part<1>(s, g, x, dy, c, k, sh);
  wd_fetch_part<2>(s, g, x, dy, c, k, sh);
  wd_fetch_part<3>(s, g, x, dy, c, k, sh);
  wd_fetch_part<4>(s, g, x, dy, c, k, sh);
}

// V = B^T d B of the staged input patch and M' = A dY A^T of the staged gradient patch
// into LDS image pair (Vs, Ms).
__device__ __forceinline__ void wd_stage_all(const WdStage& s, float* Vs, float* Ms, int tid) {
  const int t = tid & 7, ch = tid >> 3;
  const float* d = s.xr;
  float e[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    e[0][j] = d[0 * 4 + j] - d[2 * 4 + j];
    e[1][j] = d[1 * 4 + j] + d[2 * 4 + j];
    e[2][j] = d[2 * 4 + j] - d[1 * 4 + j];
    e[3][j] = d[1 * 4 + j] - d[3 * 4 + j];
  }
  floatx4* vdst = reinterpret_cast<floatx4*>(&Vs[(t * 64 + (ch ^ t)) * 20]);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    vdst[i] = floatx4{e[i][0] - e[i][2], e[i][1] + e[i][2], e[i][2] - e[i][1],
                      e[i][1] - e[i][3]};
  const float* y = s.yr;
  float r[4][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    r[0][j] = y[0 * 2 + j];
    r[1][j] = y[0 * 2 + j] + y[1 * 2 + j];
    r[2][j] = y[0 * 2 + j] - y[1 * 2 + j];
    r[3][j] = -y[1 * 2 + j];
  }
  floatx4* mdst = reinterpret_cast<floatx4*>(&Ms[(t * 64 + (ch ^ t)) * 20]);
#pragma unroll
  for (int a = 0; a < 4; ++a)
    mdst[a] = floatx4{r[a][0], r[a][0] + r[a][1], r[a][0] - r[a][1], -r[a][1]};
}

struct WdCtx {
  float* Vs_next;
  float* Ms_next;
  const float* x;
  const float* dy;
  int64_t t_next;    // this thread's tile of the step being prefetched
  WdGeo geo;         // its geometry (computed in slot 17)
  int c, k;
  int tid;
};

// Slot S (after MFMA 2S + 1) of one wgrad step: stage the prefetched patches into the
// idle buffer (S 0-11), then fetch the patches of the step after next (S 13-22).
template <int S>
__device__ __forceinline__ void wd_slot(WdStage& s, WdCtx& c, const WdShape& sh) {
  const int t = c.tid & 7, ch = c.tid >> 3;
  float* d = s.xr;
  if constexpr (S < 4) {  // column j = S of B^T d, in place
    constexpr int j = S;
    const float e0 = d[0 * 4 + j] - d[2 * 4 + j];
    const float e1 = d[1 * 4 + j] + d[2 * 4 + j];
    const float e2 = d[2 * 4 + j] - d[1 * 4 + j];
    const float e3 = d[1 * 4 + j] - d[3 * 4 + j];
    d[0 * 4 + j] = e0;
    d[1 * 4 + j] = e1;
    d[2 * 4 + j] = e2;
    d[3 * 4 + j] = e3;
  } else if constexpr (S < 8) {  // row i of (B^T d) B -> LDS
    constexpr int i = S - 4;
    floatx4* vdst = reinterpret_cast<floatx4*>(&c.Vs_next[(t * 64 + (ch ^ t)) * 20]);
    vdst[i] = floatx4{d[i * 4 + 0] - d[i * 4 + 2], d[i * 4 + 1] + d[i * 4 + 2],
                      d[i * 4 + 2] - d[i * 4 + 1], d[i * 4 + 1] - d[i * 4 + 3]};
  } else if constexpr (S < 12) {  // row a of A dY A^T -> LDS
    constexpr int a = S - 8;
    const float* y = s.yr;
    // rows of A dY: [y0, y1], [y0 + y2, y1 + y3], [y0 - y2, y1 - y3], [-y2, -y3]
    const float r0 = a == 0 ? y[0] : a == 1 ? y[0] + y[2] : a == 2 ? y[0] - y[2] : -y[2];
    const float r1 = a == 0 ? y[1] : a == 1 ? y[1] + y[3] : a == 2 ? y[1] - y[3] : -y[3];
    floatx4* mdst = reinterpret_cast<floatx4*>(&c.Ms_next[(t * 64 + (ch ^ t)) * 20]);
    mdst[a] = floatx4{r0, r0 + r1, r0 - r1, -r1};
  } else if constexpr (S == 13) {
    c.geo = wd_geo(c.t_next, sh);
  } else if constexpr (S >= 14 && S < 24 && (S & 1) == 0) {  // prefetch parts 0-4
    wd_fetch_part<(S - 14) / 2>(s, c.geo, c.x, c.dy, c.c, c.k, sh);
  }
}

template <int G, int M>
__device__ __forceinline__ void wd_group_tail(floatx4 (&acc)[16][2], WdStage& s, WdCtx& c,
                                              const WdShape& sh,
                                              const floatx4& a0,
                                              const floatx4& a1, const floatx4& b0) {
  if constexpr (M < 8) {
    constexpr int ep = M >> 1;
    constexpr int i = M & 1;
    acc[4 * (G & 3) + ep][i] = __builtin_amdgcn_mfma_f32_16x16x4f32(
        (i ? a1 : a0)[ep], b0[ep], acc[4 * (G & 3) + ep][i], 0, 0, 0);
    if constexpr ((M & 1) == 1) wd_slot<(G * 8 + M) / 2>(s, c, sh);
    __builtin_amdgcn_sched_barrier(0);
    wd_group_tail<G, M + 1>(acc, s, c, sh, a0, a1, b0);
  }
}

// The A operand of tile quad ks, lane quarter q = lane >> 4: channel (cb + (lane & 15))
// of tile t = 4ks + q sits at position (cb + (lane & 15)) ^ t of row t.
template <int G>
__device__ __forceinline__ void wd_groups(floatx4 (&acc)[16][2], WdStage& s, WdCtx& c,
                                          const WdShape& sh, const float* Vs, const float* Ms,
                                          int lane, int wc,
                                          int wk, floatx4 a0, floatx4 a1, floatx4 b0) {
  if constexpr (G < 8) {
    floatx4 na0 = a0, na1 = a1, nb0 = b0;
    if constexpr (G + 1 < 8) {
      constexpr int ks = (G + 1) >> 2, q4 = (G + 1) & 3;
      const int t = 4 * ks + (lane >> 4);
      const int cA = wc * 32 + (lane & 15);
      const int kB = wk * 16 + (lane & 15);
      na0 = *reinterpret_cast<const floatx4*>(&Vs[(t * 64 + (cA ^ t)) * 20 + q4 * 4]);
      na1 = *reinterpret_cast<const floatx4*>(&Vs[(t * 64 + ((cA + 16) ^ t)) * 20 + q4 * 4]);
      nb0 = *reinterpret_cast<const floatx4*>(&Ms[(t * 64 + (kB ^ t)) * 20 + q4 * 4]);
    }
    wd_group_tail<G, 0>(acc, s, c, sh, a0, a1, b0);
    wd_groups<G + 1>(acc, s, c, sh, Vs, Ms, lane, wc, wk, na0, na1, nb0);
  }
}

// (a runtime buffer index: the pinned slot order already orders the staging stores
// and operand reads, and a single-step loop body keeps the accumulators in place)
__device__ __forceinline__ void wd_step(floatx4 (&acc)[16][2], WdStage& s, float* lds, int buf,
                                        WdCtx& c, const WdShape& sh, int lane, int wc, int wk) {
  c.Vs_next = lds + (buf ^ 1) * 2 * kWDImg;
  c.Ms_next = c.Vs_next + kWDImg;
  const float* Vs = lds + buf * 2 * kWDImg;
  const float* Ms = Vs + kWDImg;
  const int t = lane >> 4;
  const int cA = wc * 32 + (lane & 15);
  const int kB = wk * 16 + (lane & 15);
  const floatx4 a0 = *reinterpret_cast<const floatx4*>(&Vs[(t * 64 + (cA ^ t)) * 20]);
  const floatx4 a1 = *reinterpret_cast<const floatx4*>(&Vs[(t * 64 + ((cA + 16) ^ t)) * 20]);
  const floatx4 b0 = *reinterpret_cast<const floatx4*>(&Ms[(t * 64 + (kB ^ t)) * 20]);
  wd_groups<0>(acc, s, c, sh, Vs, Ms, lane, wc, wk, a0, a1, b0);
}

__global__ __launch_bounds__(kDBThreads, 1) void wino_wgrad_db_kernel(
    const float* __restrict__ x, const float* __restrict__ dy, float* __restrict__ dw, int C,
    int K, int H, int W, int TH, int TW_, int64_t P, int cblocks, int kblocks, int splits,
    bool accum) {
  __shared__ float lds[2 * 2 * kWDImg];  // [buffer][V | M'][8 tiles][64][20]: 160 KiB

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
  const int wc = wave & 1;
  const int wk = wave >> 1;
  const int64_t HW = static_cast<int64_t>(H) * W;
  const int64_t steps_total = (P + kWDT - 1) / kWDT;
  const int64_t st_begin = z * steps_total / splits;
  const int64_t st_end = (z + 1) * steps_total / splits;

  floatx4 acc[16][2];
#pragma unroll
  for (int xi = 0; xi < 16; ++xi) {
    acc[xi][0] = floatx4{0.f, 0.f, 0.f, 0.f};
    acc[xi][1] = floatx4{0.f, 0.f, 0.f, 0.f};
  }

  // (every split owns >= 1 step: the host caps splits at the step count)
  WdShape sh;
  sh.C = C;
  sh.K = K;
  sh.H = H;
  sh.W = W;
  sh.TW_ = TW_;
  sh.tpi = TH * TW_;
  sh.inv_tw = 1.f / static_cast<float>(TW_);
  sh.inv_tpi = 1.f / static_cast<float>(sh.tpi);
  sh.P = P;
  sh.HW = HW;
  WdCtx c;
  c.x = x;
  c.dy = dy;
  c.c = cb * 64 + (tid >> 3);
  c.k = kb * 64 + (tid >> 3);
  c.tid = tid;
  const int slot = tid & 7;
  WdStage s;
  wd_fetch(s, st_begin * kWDT + slot, x, dy, c.c, c.k, sh);
  wd_stage_all(s, lds, lds + kWDImg, tid);
  __syncthreads();
  // Prefetches past the split's last step re-read its last step (staged, never read).
  wd_fetch(s, min(st_begin + 1, st_end - 1) * kWDT + slot, x, dy, c.c, c.k, sh);
  for (int64_t st = st_begin; st < st_end; ++st) {
    c.t_next = min(st + 2, st_end - 1) * kWDT + slot;
    wd_step(acc, s, lds, static_cast<int>((st - st_begin) & 1), c, sh, lane, wc, wk);
    __syncthreads();
  }
  wd_keep(s);

  // -- dW = G^T dU G per (c, k) pair; partial slab z of [splits][K][C][9] --------------
  float* out = dw + static_cast<int64_t>(z) * K * C * 9;
  const int k = kb * 64 + wk * 16 + (lane & 15);
  if (k >= K) return;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ch = cb * 64 + wc * 32 + i * 16 + (lane >> 4) * 4 + r;
      if (ch >= C) continue;
      float u[16];
#pragma unroll
      for (int xi = 0; xi < 16; ++xi) u[xi] = acc[xi][i][r];
      float t[3][4];
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const float s12 = 0.5f * (u[1 * 4 + b] + u[2 * 4 + b]);
        t[0][b] = u[0 * 4 + b] + s12;
        t[1][b] = 0.5f * (u[1 * 4 + b] - u[2 * 4 + b]);
        t[2][b] = s12 + u[3 * 4 + b];
      }
      float* o = out + (static_cast<int64_t>(k) * C + ch) * 9;
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const float s12 = 0.5f * (t[a][1] + t[a][2]);
        wg_store(o + a * 3 + 0, t[a][0] + s12, accum);
        wg_store(o + a * 3 + 1, 0.5f * (t[a][1] - t[a][2]), accum);
        wg_store(o + a * 3 + 2, s12 + t[a][3], accum);
      }
    }
}

__global__ void wino_wgrad_reduce_kernel(const float* __restrict__ ws, float* __restrict__ dw,
                                         int64_t numel, int splits, bool accum) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= numel) return;
  float v = 0.f;
  for (int z = 0; z < splits; ++z) v += ws[z * numel + i];
  wg_store(dw + i, v, accum);
}

}  // namespace

int64_t wino_pad_reduction(int64_t r) { return (r + kCB - 1) / kCB * kCB; }
int64_t wino_pad_output(int64_t o) { return (o + kOBMax - 1) / kOBMax * kOBMax; }

void launch_wino_weight(const float* w, float* u, int64_t out_channels, int64_t red_channels,
                        bool flip, hipStream_t stream) {
  const int64_t Op = wino_pad_output(out_channels);
  const int64_t Rp = wino_pad_reduction(red_channels);
  const int64_t total = Rp * Op;
  const int blocks = static_cast<int>((total + 255) / 256);
  hipLaunchKernelGGL(wino_weight_kernel, dim3(blocks), dim3(256), 0, stream, w, u,
                     static_cast<int>(out_channels), static_cast<int>(red_channels),
                     static_cast<int>(Op), static_cast<int>(Rp), flip);
}

WinoPlan wino_plan(int64_t n, int64_t red_channels, int64_t h, int64_t w, int64_t out_channels,
                   int variant, int splits) {
  WinoPlan plan;
  plan.variant = variant >= 0 ? variant : (out_channels <= 32 ? 1 : 2);
  const int ob = plan.variant == 1 ? 32 : 64;
  const int tbk = plan.variant == 0 ? 32 : 64;
  const int64_t P = n * ((h + 1) / 2) * ((w + 1) / 2);
  const int64_t blocks = ((P + tbk - 1) / tbk) * ((out_channels + ob - 1) / ob);
  const int64_t chunks = wino_pad_reduction(red_channels) / kCB;
  if (splits > 0) {
    plan.splits = static_cast<int>(std::min<int64_t>(splits, chunks));
  } else {
    // Fill the chip: >= 2 rounds of workgroups over the CUs (variant 2 runs one per CU,
    // variants 0/1 two), keeping enough channel chunks per split to amortise the
    // pipeline prologue.
    const int64_t target = plan.variant == 2 ? 512 : 1024;
    const int64_t min_chunks = plan.variant == 2 ? 8 : 16;
    int64_t s = 1;
    while (blocks * s < target && chunks / (s * 2) >= min_chunks) s *= 2;
    plan.splits = static_cast<int>(s);
  }
  plan.workspace = plan.splits > 1 ? plan.splits * n * out_channels * h * w : 0;
  return plan;
}

void launch_wino_conv(const float* x, const float* u, const float* bias, float* y, float* ws,
                      int64_t n, int64_t red_channels, int64_t h, int64_t w, int64_t out_channels,
                      const WinoPlan& plan, hipStream_t stream) {
  if (plan.variant == 2) {
    launch_db(x, u, bias, y, ws, n, red_channels, h, w, out_channels, plan.splits, stream);
  } else if (plan.variant == 1) {
    launch_variant<2, 2>(x, u, bias, y, ws, n, red_channels, h, w, out_channels, plan.splits,
                         stream);
  } else {
    launch_variant<4, 1>(x, u, bias, y, ws, n, red_channels, h, w, out_channels, plan.splits,
                         stream);
  }
}

int wino_wgrad_splits(int64_t n, int64_t c, int64_t k, int64_t h, int64_t w, int variant) {
  const int64_t P = n * ((h + 1) / 2) * ((w + 1) / 2);
  if (variant == 2) {
    // one workgroup per CU: >= 2 rounds of 256, >= 8 steps of 8 tiles per split
    const int64_t tiles_blocks = ((c + 63) / 64) * ((k + 63) / 64);
    const int64_t steps = (P + kWDT - 1) / kWDT;
    int64_t s = (512 + tiles_blocks - 1) / tiles_blocks;
    s = std::min<int64_t>(s, std::max<int64_t>(1, steps / 8));
    s = std::min<int64_t>(s, 256);
    return static_cast<int>(std::max<int64_t>(s, 1));
  }
  const int64_t tiles_blocks = ((c + kWC - 1) / kWC) * ((k + kWK - 1) / kWK);
  const int64_t iters = (P + kWT - 1) / kWT;
  int64_t s = (1024 + tiles_blocks - 1) / tiles_blocks;
  s = std::min<int64_t>(s, std::max<int64_t>(1, iters / 16));  // >= 16 iterations per split
  s = std::min<int64_t>(s, 256);
  return static_cast<int>(std::max<int64_t>(s, 1));
}

void launch_wino_wgrad(const float* x, const float* dy, float* dw, float* ws, int64_t n,
                       int64_t c, int64_t k, int64_t h, int64_t w, int splits, int variant,
                       bool accum, hipStream_t stream) {
  const int64_t th = (h + 1) / 2, tw = (w + 1) / 2;
  const int64_t P = n * th * tw;
  if (variant == 2) {
    const int cblocks = static_cast<int>((c + 63) / 64);
    const int kblocks = static_cast<int>((k + 63) / 64);
    const int64_t nwg = static_cast<int64_t>(cblocks) * kblocks * splits;
    hipLaunchKernelGGL(wino_wgrad_db_kernel, dim3(static_cast<unsigned>(nwg)),
                       dim3(kDBThreads), 0, stream, x, dy, splits > 1 ? ws : dw,
                       static_cast<int>(c), static_cast<int>(k), static_cast<int>(h),
                       static_cast<int>(w), static_cast<int>(th), static_cast<int>(tw), P,
                       cblocks, kblocks, splits, accum && splits == 1);
  } else {
    const int cblocks = static_cast<int>((c + kWC - 1) / kWC);
    const int kblocks = static_cast<int>((k + kWK - 1) / kWK);
    const int64_t nwg = static_cast<int64_t>(cblocks) * kblocks * splits;
    hipLaunchKernelGGL(wino_wgrad_kernel, dim3(static_cast<unsigned>(nwg)), dim3(kThreads), 0,
                       stream, x, dy, splits > 1 ? ws : dw, static_cast<int>(c),
                       static_cast<int>(k), static_cast<int>(h), static_cast<int>(w),
                       static_cast<int>(th), static_cast<int>(tw), P, cblocks, kblocks,
                       splits, accum && splits == 1);
  }
  if (splits > 1) {
    const int64_t numel = k * c * 9;
    hipLaunchKernelGGL(wino_wgrad_reduce_kernel,
                       dim3(static_cast<unsigned>((numel + 255) / 256)), dim3(256), 0, stream,
                       ws, dw, numel, splits, accum);
  }
}

}  // namespace tgpipe
