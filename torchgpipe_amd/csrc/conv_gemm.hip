// Implicit-GEMM convolution on the fp32 MFMA pipes of CDNA4 (gfx950) for the
// AmoebaNet-D cell operations: 1x1 (stride 1 / 2, input offset for FactorizedReduce)
// and 1xk / kx1 convolutions, NCHW fp32, fused with the ReLU that precedes every
// convolution of the model and with the statistics of the BatchNorm that follows it.
// Any kh x kw kernel at any stride (U-Net's 3-channel input convolution, AmoebaNet's stem
// and the stride-2 3x3 of its reduction cells); strided kernels larger than 1x1 run the
// backward-data over every input pixel, the taps that fall into stride holes reading 0.
//
//   forward      Z[n][co][p]    = sum_{ci,t} W[co][ci][t] * relu(X[n][ci][tap(p,t)])
//                M = Co, N = images x output pixels, K = Ci x taps
//                epilogue: Z tile -> LDS -> coalesced stores + per-(channel, column block)
//                (mean, M2) partials for the BatchNorm (merged with Chan's formula later)
//   backward-data dX[n][ci][q]  = relu'(X) * sum_{co,t} W[co][ci][t] * dZ[n][co][tap^-1(q,t)]
//                M = Ci, N = images x input pixels, K = Co x taps  (A = W transposed)
//                strided 1x1 ("scatter"): N = output pixels, each result scattered to
//                its input pixel (the stride holes are zero; 4x less work than a
//                dense pass that reads zeros for them)
//                strided k x k ("phase", conv_gemm_phases): one GEMM per residue of the
//                input pixel modulo the stride, over exactly the taps that reach it --
//                N = that phase's pixels, K = Co x its taps, results scattered likewise
//   weight-grad  dW[co][ci][t]  = sum_{n,p} dZ[n][co][p] * relu(X[n][ci][tap(p,t)])
//                M = Co, N = Ci x taps, K = images x output pixels
//
// Workgroups (Cfg): 128 x 128 blocks of 8 waves (2 x 4, each 64 x 32 = two
// v_mfma_f32_32x32x2_f32 tiles) or 64 x 64 blocks of 4 waves (one tile each), BK = 32
// reduction steps per double-buffered LDS stage: one barrier and 32 / 16 MFMAs per wave
// per stage, with the next stage's global loads in flight meanwhile (a two-stage-ahead
// variant with two register sets measured 3 % slower: profiles/convbn_bench.json notes).
// Grids that would not fill the 256 CUs split the reduction (grid.y): each split stores
// its partial tile into a workspace slice and split_reduce sums them (no atomics); the
// forward then leaves the BatchNorm statistics to a separate pass (bn_stats).
//
// Element-gathered N-major operands (planes whose pixel count is not a multiple of 4, e.g.
// AmoebaNet's 7x7; every kernel with taps) give each lane columns BN/4 apart, so one load
// instruction reads a contiguous run of pixels across the lanes (store_nmajor `spread`).
//
// LDS images:
//   K-major operand (k contiguous in HBM: weights, dZ in weight-grad, X in weight-grad)
//     [BK/4][2][rows][2]: k quad g split into the pairs (k0, k2) / (k1, k3) that lane half
//     h of a 32x32x2 MFMA pair (k-steps 2g, 2g+1) reads as one conflict-free ds_read_b64.
//   N-major operand (pixels contiguous: X in forward, dZ in backward-data)
//     [BK][cols + 32]: the two lane halves read rows k and k+1, 32 banks apart.
// Out-of-range taps (padding, stride holes, tails) are raw buffer loads at an offset
// past the buffer: the hardware returns 0, so padding needs no select.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>
#include <vector>

#include "kernels.h"

namespace tgpipe {

int env_int(const char* name, int fallback);

namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kBK = 32;
constexpr int kConvGemmCfgs = 12;  // tile configurations (Cfg<0..11>; 7..11 split-bf16)
constexpr int kFirstEmuCfg = 7;
// mfma_stage: all of a stage's LDS fragment reads ahead of its MFMAs (see there)
constexpr bool kMfmaReadsFirst = true;
constexpr uint32_t kOOB = 0x7ffffff0u;  // buffer offset past every tensor (< 2 GiB)

enum Mode : int { kFwd = 0, kBwdData = 1, kWgrad = 2 };

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), static_cast<short>(0),
                                           static_cast<int>(bytes), 0x00020000);
}

__device__ __forceinline__ float bload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}

__device__ __forceinline__ floatx4 bload4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return floatx4{__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]),
                 __uint_as_float(v[3])};
}

__device__ __forceinline__ float relu(float v) { return v > 0.f ? v : 0.f; }

// Division by a per-launch constant without the ~20-instruction integer divide: the
// implicit-GEMM gathers split flat indices into (channel, tap) / (image, pixel) / (row,
// column) in their inner loops.  n / d = umulhi(n, mul) >> shr for 0 <= n < 2^31, with
// shr = ceil(log2 d) - 1 and mul = ceil(2^(31 + ceil(log2 d)) / d) (d = 1: n itself).
struct FastDiv {
  uint32_t mul, shr;
  int d;
  __device__ __forceinline__ int div(int n) const {
    return d == 1 ? n : static_cast<int>(__umulhi(static_cast<uint32_t>(n), mul) >> shr);
  }
};

FastDiv make_fastdiv(int d) {
  FastDiv f{0u, 0u, d};
  if (d > 1) {
    int l = 0;
    while ((1ll << l) < d) ++l;  // ceil(log2 d)
    f.mul = static_cast<uint32_t>(((1ull << (31 + l)) + static_cast<uint64_t>(d) - 1) /
                                  static_cast<uint64_t>(d));
    f.shr = static_cast<uint32_t>(l - 1);
  }
  return f;
}

// Geometry of one convolution (all byte offsets fit in 31 bits: checked on the host).
struct Geo {
  int n, ci, h, w;       // input
  int co, ho, wo;        // output (co = channels of this convolution)
  int co_total, co_off;  // channel count / offset of its output inside Z (concat outputs)
  int kh, kw, taps;      // kernel, taps = kh * kw (tap t = (t / kw, t % kw))
  int sh, sw, ph, pw;    // stride, padding
  int oh, ow;            // extra input offset (FactorizedReduce's shifted branch: 1)
  int relu;              // ReLU on the input (forward / weight-grad) / its mask (bwd-data)
  int scatter;           // bwd-data over output pixels, results scattered (strided 1x1)
  int a_t;               // bwd-data: A is the transposed weight [ci][co*T] (row-major)
  int spread;            // element-gathered N-major columns spread over the lanes
  FastDiv fd_taps, fd_kw, fd_hwo, fd_wo, fd_hwi;  // / taps, / kw, / (ho*wo), / wo, / (h*w)
  // bwd-data of one stride phase (scatter set too): ho x wo = the phase grid, zh x zw =
  // the dZ plane, tap (th, tw) of column (y, x) reads dZ[y + dy0 - th][x + dx0 - tw]
  int phase, zh, zw, dy0, dx0;
  int fill;  // strided 1x1 bwd-data: zeros into the 2x2 blocks' other pixels (ConvGemmGeo)
};

// All stride phases of one backward-data in one launch (grid.z = phase): what differs
// between them (conv_gemm_phases), and each phase's slice of the concatenated weights.
constexpr int kMaxPhases = 4;
struct PhaseSet {
  int count;  // 0: an ordinary launch
  int kh[kMaxPhases], kw[kMaxPhases], ho[kMaxPhases], wo[kMaxPhases];
  int dy0[kMaxPhases], dx0[kMaxPhases], oh[kMaxPhases], ow[kMaxPhases];
  int64_t a_off[kMaxPhases], a_bytes[kMaxPhases];
  FastDiv fd_taps[kMaxPhases], fd_kw[kMaxPhases], fd_hwo[kMaxPhases], fd_wo[kMaxPhases];
};

// Tile configurations.  CFG 0: 64 x 64 block, 4 waves (2 x 2) of one 32 x 32 MFMA tile;
// CFG 1: 128 x 128 block, 8 waves (2 x 4) of 64 x 32 (two tiles) -- two waves per SIMD
// from one workgroup, so one wave's MFMAs cover the other's LDS reads and barrier;
// CFG 2: 128 x 128 block, 4 waves (2 x 2) of 64 x 64 (2 x 2 tiles): each A / B fragment
// read from LDS feeds two MFMAs, half the LDS traffic per MFMA of CFG 1.
// CFG 3 / 4 / 5 / 6: CFG 0 / 1 / 2 / 0 with SUB = 4 / 2 / 2 / 2 BK-deep sub-stages per barrier and
// per prefetch: a small grid (one workgroup per CU) then keeps SUB x more loads in flight
// per wave -- each stage's MFMAs cover one global-load latency instead of a fraction.
//
// CFG 7 / 8 / 9: the tiles of CFG 0 / 2 / 1 on the bf16 matrix pipes (EMU, see
// "split-bf16 products" below): 64 x 64 (3 x 48 KiB per CU), 128 x 128 / 4 waves and
// 128 x 128 / 8 waves (96 KiB).
// CFG 10: CFG 9 with ONE operand buffer (48 KiB; the epilogue's 68 KiB C tile sets the
// footprint): two workgroups per CU, four waves per SIMD.  CFG 9's double buffer holds one
// workgroup per CU, and its waves sat in waits for 35-47 % of their cycles (PMC,
// profiles/KERNELS.md "Pre-split weights"): here the stage's loads still go to registers
// during its MFMAs, the store into the one buffer waits for a barrier behind the last
// reader, and the other workgroup's waves fill that barrier and the waits.  Fragments are
// read per 16-deep step (a 128-register budget) rather than a whole stage ahead.
// CFG 11: CFG 7 (64 x 64, 4 waves) single-buffered the same way: 24 KiB of operands, four
// workgroups per CU at four waves per SIMD (CFG 7: three).
template <int CFG>
struct Cfg {
  static constexpr bool EMU = CFG >= kFirstEmuCfg;
  static constexpr bool SINGLE = CFG == 10 || CFG == 11;  // one operand buffer (see above)
  static constexpr int TILE =
      !EMU ? CFG % 3 : (CFG == 7 || CFG == 11 ? 0 : (CFG == 8 ? 2 : 1));
  static constexpr int SUB = EMU || CFG < 3 ? 1 : (CFG == 3 ? 4 : 2);  // (CFG 6: 2 x 80 KiB)
  static constexpr int WVM = 2;
  static constexpr int WVN = TILE == 1 ? 4 : 2;
  static constexpr int TM = TILE == 0 ? 1 : 2;   // 32 x 32 MFMA tiles per wave (rows)
  static constexpr int TN = TILE == 2 ? 2 : 1;   // (columns)
  static constexpr int kThreads = 64 * WVM * WVN;
  // waves per SIMD when the LDS footprint's workgroups per CU are resident (4 x 40 KiB /
  // 2 x 72 KiB / 1 x 147-160 KiB): the register budget __launch_bounds__ holds them to
  static constexpr int kWavesPerSimd =
      CFG == 0 || CFG == 1 || CFG == 10 || CFG == 11 ? 4
      : CFG == 7                        ? 3
      : (CFG == 2 || CFG == 4 || CFG == 6 || CFG == 9 ? 2 : 1);
  static constexpr int BM = WVM * 32 * TM;
  static constexpr int BN = WVN * 32 * TN;
  // K-major images (one sub-stage): f32 [BK][rows], or EMU three bf16 planes of
  // [BK/8][rows][8] (emu_off)
  static constexpr int kAImg = EMU ? 3 * kBK * BM / 2 : kBK * BM;
  static constexpr int kBImgK = EMU ? 3 * kBK * BN / 2 : kBK * BN;
  static constexpr int kBStrideN = BN + 32;       // N-major row stride
  static constexpr int kBImgN = kBK * kBStrideN;  // N-major image (f32 only)
  // epilogue C tile row stride: rows 4 apart (the two halves of an MFMA result
  // register) land 32 banks apart
  static constexpr int kCStride = BN + 8;
  static constexpr int kOpFloats(bool k_major) {
    return (SINGLE ? 1 : 2) * SUB * (kAImg + (k_major || EMU ? kBImgK : kBImgN));
  }
  // operand images (double-buffered), reused by the epilogue's C tile (forward /
  // bwd-data); 128 x 128: 72 KiB -> two workgroups per CU
  static constexpr int kLdsFloats(int mode) {
    return mode == 2 ? kOpFloats(true)
                     : (kOpFloats(false) > BM * kCStride ? kOpFloats(false) : BM * kCStride);
  }
  static constexpr int kAQuads = kBK * BM / 4 / kThreads;   // per thread per stage
  static constexpr int kBQuadsN = kBK * BN / 4 / kThreads;
  static constexpr int kBQuadsK = kBK * BN / 4 / kThreads;
};

// ---- operand staging -----------------------------------------------------------------------
// K-major operand: quad index i of thread t -> row r = (t >> 3) + (THREADS / 8) * i,
// k quad q = t & 7 (k = 4q .. 4q+3).  The quad is split into the two k pairs the two lane
// halves of a 32x32x2 MFMA pair consume -- half 0 = (k0, k2), half 1 = (k1, k3) -- each
// stored as 8 bytes at slot [q][half][r ^ 2q]:
//   * an MFMA fragment read (ds_read_b64, lane groups 0-31 / 32-63) is 32 consecutive
//     rows of one half: 256 contiguous bytes, all 64 banks, no conflict (a [q][r][4]
//     image puts rows r and r + 16 of a 16-byte-slot layout on the same banks: 2-way);
//   * the two ds_write_b64 per quad (16-lane groups: 8 quads x 2 rows) land on 16
//     distinct 8-byte bank pairs thanks to the r ^ 2q swizzle, which keeps every aligned
//     32-row block a permutation of itself.
__device__ __forceinline__ int kswz(int row, int q) { return row ^ (2 * q); }

template <int ROWS, int Q, int THREADS>
__device__ __forceinline__ void store_kmajor(float* img, const floatx4 (&v)[Q], int tid) {
  const int q = tid & 7;
#pragma unroll
  for (int i = 0; i < Q; ++i) {
    const int row = (tid >> 3) + (THREADS / 8) * i;
    float* base = img + ((2 * q) * ROWS + kswz(row, q)) * 2;
    *reinterpret_cast<floatx2*>(base) = floatx2{v[i][0], v[i][2]};
    *reinterpret_cast<floatx2*>(base + 2 * ROWS) = floatx2{v[i][1], v[i][3]};
  }
}

// N-major operand: quad index i of thread t -> row k = t / (BN/4) + (THREADS / (BN/4)) * i,
// column quad t % (BN/4) -- or, when the operand is gathered element by element
// (`spread`: columns whose pixels are not 16-byte quads), columns t % (BN/4) + (BN/4) e
// for e = 0..3, so the lanes of one load instruction read consecutive pixels (one
// contiguous run per row) instead of every fourth one.
template <int BN, int Q, int THREADS>
__device__ __forceinline__ void store_nmajor(float* img, const floatx4 (&v)[Q], int tid,
                                             bool spread) {
  constexpr int QPR = BN / 4;
  constexpr int RPP = THREADS / QPR;
#pragma unroll
  for (int i = 0; i < Q; ++i) {
    const int k = tid / QPR + RPP * i;
    float* row = img + k * (BN + 32);
    if (spread) {
#pragma unroll
      for (int e = 0; e < 4; ++e) row[tid % QPR + QPR * e] = v[i][e];
    } else {
      *reinterpret_cast<floatx4*>(row + (tid % QPR) * 4) = v[i];
    }
  }
}

// ---- split-bf16 products (EMU configurations) -------------------------------------------------
// An f32 x is exactly hi + mid + lo with three bf16 (8-bit significands, round to nearest
// each: x - hi has at most 16 significant bits, x - hi - mid at most 8).  A product a * b
// is then the nine partial products of the parts, each exact in f32; the six kept here
// (hi.hi, hi.mid, mid.hi, mid.mid, hi.lo, lo.hi) leave out terms below 2^-24 |a b| -- less
// than the rounding of one f32 product -- and run on v_mfma_f32_32x32x16_bf16, 16x the f32
// MFMA's rate per product: six of them cost 3/8 of the f32 MFMA time of the same tile.
// Accumulation stays f32 in the MFMA accumulators; the fp64 tests hold these
// configurations to the same error bounds as the f32 ones (tests/ops/test_convbn_gpu.py).
__device__ __forceinline__ void split1(float v, __bf16& hi, __bf16& mid, __bf16& lo) {
  const __bf16 h = static_cast<__bf16>(v);
  const float r = v - static_cast<float>(h);
  const __bf16 m = static_cast<__bf16>(r);
  hi = h;
  mid = m;
  lo = static_cast<__bf16>(r - static_cast<float>(m));
}

__device__ __forceinline__ void split3(const floatx4& v, bf16x4& hi, bf16x4& mid, bf16x4& lo) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    __bf16 h, m, l;
    split1(v[e], h, m, l);
    hi[e] = h;
    mid[e] = m;
    lo[e] = l;
  }
}

// EMU image of one K-major operand plane: [slot j = k / 8][row ^ 2j][8 k], 16 bytes per
// (slot, row), three planes (hi, mid, lo) of BK x ROWS bf16 each.  Lane half h of a
// 32x32x16 MFMA at k step s reads slot j = 2s + h of 32 consecutive rows with one
// ds_read_b128 (512 contiguous bytes: conflict-free); a k quad q (k = 4q .. 4q+3) of a row
// is the 8-byte half (q & 1) of slot q >> 1, and the row ^ 2j swizzle puts the 16 lanes of
// a ds_write_b64 (8 quads x 2 rows) on 16 distinct 8-byte bank pairs.
template <int ROWS>
__device__ __forceinline__ int emu_off(int j, int row) {  // in bf16 elements
  return (j * ROWS + (row ^ (2 * j))) * 8;
}

template <int ROWS>
__device__ __forceinline__ void store_emu_quad(float* img, const floatx4& v, int row, int q) {
  bf16x4 hi, mid, lo;
  split3(v, hi, mid, lo);
  __bf16* p = reinterpret_cast<__bf16*>(img) + emu_off<ROWS>(q >> 1, row) + 4 * (q & 1);
  constexpr int kPlane = kBK * ROWS;
  *reinterpret_cast<bf16x4*>(p) = hi;
  *reinterpret_cast<bf16x4*>(p + kPlane) = mid;
  *reinterpret_cast<bf16x4*>(p + 2 * kPlane) = lo;
}

// ---- the GEMM core ------------------------------------------------------------------------

// EMU stage: two k steps of 16; per 32 x 32 tile and step six MFMAs (small parts first).
// All fragments of the stage are read ahead of its MFMAs; `between(0..3)` carries the next
// stage's loads (after the first four MFMA groups: the stage is 3/8 as long as an f32 one).
template <int CFG, typename Between>
__device__ __forceinline__ void mfma_stage_emu(floatx16 (&acc)[Cfg<CFG>::TM][Cfg<CFG>::TN],
                                               const float* aimg, const float* bimg, int lane,
                                               int wm, int wn, Between&& between) {
  using C = Cfg<CFG>;
  constexpr int WM = C::TM, WN = C::TN, S = kBK / 16;
  const int h = lane >> 5, l32 = lane & 31;
  const __bf16* ab = reinterpret_cast<const __bf16*>(aimg);
  const __bf16* bb = reinterpret_cast<const __bf16*>(bimg);
  constexpr int kPairs[6][2] = {{2, 0}, {0, 2}, {1, 1}, {1, 0}, {0, 1}, {0, 0}};
  if constexpr (C::SINGLE) {
    // per 16-deep step: its fragments, then its MFMAs (the other workgroup's waves cover
    // the read latency; a whole stage of fragments would not fit 128 registers)
#pragma unroll
    for (int s = 0; s < S; ++s) {
      bf16x8 a[3][WM], b[3][WN];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
#pragma unroll
        for (int i = 0; i < WM; ++i)
          a[p][i] = *reinterpret_cast<const bf16x8*>(
              ab + p * kBK * C::BM + emu_off<C::BM>(2 * s + h, wm * 32 * WM + i * 32 + l32));
#pragma unroll
        for (int j = 0; j < WN; ++j)
          b[p][j] = *reinterpret_cast<const bf16x8*>(
              bb + p * kBK * C::BN + emu_off<C::BN>(2 * s + h, wn * 32 * WN + j * 32 + l32));
      }
#pragma unroll
      for (int t = 0; t < 6; ++t) {
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                a[kPairs[t][0]][i], b[kPairs[t][1]][j], acc[i][j], 0, 0, 0);
        if (s == 0 && t < 4) between(t);
      }
    }
    return;
  }
  bf16x8 a[S][3][WM], b[S][3][WN];
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int p = 0; p < 3; ++p) {
#pragma unroll
      for (int i = 0; i < WM; ++i)
        a[s][p][i] = *reinterpret_cast<const bf16x8*>(
            ab + p * kBK * C::BM + emu_off<C::BM>(2 * s + h, wm * 32 * WM + i * 32 + l32));
#pragma unroll
      for (int j = 0; j < WN; ++j)
        b[s][p][j] = *reinterpret_cast<const bf16x8*>(
            bb + p * kBK * C::BN + emu_off<C::BN>(2 * s + h, wn * 32 * WN + j * 32 + l32));
    }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int s = 0; s < S; ++s) {
#pragma unroll
    for (int t = 0; t < 6; ++t) {
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              a[s][kPairs[t][0]][i], b[s][kPairs[t][1]][j], acc[i][j], 0, 0, 0);
      if (s == 0 && t < 4) between(t);  // the loads within the stage's first third
    }
  }
}

// `between(g)` runs after MFMA group g (the two k-steps of k quad g): the main loop issues the
// next stage's loads from it, pinned there by scheduling barriers.
template <int CFG, bool kBKMajor, typename Between>
__device__ __forceinline__ void mfma_stage(floatx16 (&acc)[Cfg<CFG>::TM][Cfg<CFG>::TN],
                                           const float* aimg, const float* bimg, int lane, int wm,
                                           int wn, Between&& between) {
  using C = Cfg<CFG>;
  constexpr int WM = C::TM, WN = C::TN, G = kBK / 4;
  const int h = lane >> 5, l32 = lane & 31;
  auto read_a = [&](int g, int i) {
    return *reinterpret_cast<const floatx2*>(
        aimg + ((2 * g + h) * C::BM + kswz(wm * 32 * WM + i * 32 + l32, g)) * 2);
  };
  auto read_b = [&](int g, int j) -> floatx2 {
    if constexpr (kBKMajor) {
      return *reinterpret_cast<const floatx2*>(
          bimg + ((2 * g + h) * C::BN + kswz(wn * 32 * WN + j * 32 + l32, g)) * 2);
    } else {
      const int col = wn * 32 * WN + j * 32 + l32;
      return floatx2{bimg[(4 * g + h) * C::kBStrideN + col],
                     bimg[(4 * g + 2 + h) * C::kBStrideN + col]};
    }
  };
  // Every fragment of the stage read before the first MFMA: read next to its MFMA pair (as
  // the compiler schedules a per-group loop), each group's LDS latency sat exposed in front
  // of the dependent accumulator chain -- 6 waits per 16 MFMAs in the ISA, 0.41 MFMA busy
  // on 1024 x 7^2 x 1024 at micro-batch 40 (profiles/r4/pmc).  One wait per stage instead.
  // (Not for the 8-wave 128 x 128 tile: the extra fragment registers would pass the 128
  // that its two workgroups per CU allow.)
  constexpr bool kFirst = kMfmaReadsFirst && CFG != 1;
  if constexpr (kFirst) {
    floatx2 a[G][WM], b[G][WN];
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
      for (int i = 0; i < WM; ++i) a[g][i] = read_a(g, i);
#pragma unroll
      for (int j = 0; j < WN; ++j) b[g][j] = read_b(g, j);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[g][i][s], b[g][j][s], acc[i][j],
                                                             0, 0, 0);
      between(g);
    }
  } else {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      floatx2 a[WM], b[WN];
#pragma unroll
      for (int i = 0; i < WM; ++i) a[i] = read_a(g, i);
#pragma unroll
      for (int j = 0; j < WN; ++j) b[j] = read_b(g, j);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j)
            acc[i][j] =
                __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][s], b[j][s], acc[i][j], 0, 0, 0);
      between(g);
    }
  }
}

// Per-column constants of an N-major operand column (fixed for the whole K loop).
struct Col {
  int base;  // element offset of the column's image / channel-0 plane (+ pixel if plain)
  int y, x;  // pixel coordinates (tap-independent part of the source position)
  bool ok;
};

// kPlain: 1x1 / stride 1 / no padding / no offset: column pixel == source pixel.
template <int MODE, bool kPlain>
__device__ __forceinline__ Col make_col(const Geo& g, int j, int N) {
  Col c;
  c.ok = j < N;
  const int jj = c.ok ? j : 0;
  const bool out_space = MODE == kFwd || g.scatter;  // columns are output pixels
  const int hw = out_space ? g.ho * g.wo : g.h * g.w;
  const int wdt = out_space ? g.wo : g.w;
  const int n = jj / hw, p = jj - n * hw;
  if constexpr (MODE == kFwd) {
    if (kPlain) {
      c.base = n * g.ci * hw + p;
      c.y = c.x = 0;
    } else {
      const int y = p / wdt;
      c.base = n * g.ci * g.h * g.w;
      c.y = y * g.sh - g.ph + g.oh;
      c.x = (p - y * wdt) * g.sw - g.pw + g.ow;
    }
  } else {  // bwd-data: dZ source
    if (g.phase) {
      const int y = p / wdt;
      c.base = (n * g.co_total + g.co_off) * g.zh * g.zw;
      c.y = y + g.dy0;
      c.x = (p - y * wdt) + g.dx0;
    } else if (kPlain || g.scatter) {
      c.base = (n * g.co_total + g.co_off) * g.ho * g.wo + p;
      c.y = c.x = 0;
      if (g.scatter) {  // destination input pixel, for the epilogue
        const int y = p / wdt;
        c.y = y * g.sh - g.ph + g.oh;
        c.x = (p - y * wdt) * g.sw - g.pw + g.ow;
      }
    } else {
      const int y = p / wdt;
      c.base = (n * g.co_total + g.co_off) * g.ho * g.wo;
      c.y = y + g.ph - g.oh;
      c.x = (p - y * wdt) + g.pw - g.ow;
    }
  }
  return c;
}

// kPreA (EMU forward / backward-data): A arrives pre-split ([M][ceil(K/8)][hi, mid, lo][8]
// bf16, conv_gemm_presplit_kernel) -- the weights, split once per step instead of by every
// column block of every micro-batch; each thread stages whole k octets of it (three 16-byte
// loads and three ds_write_b128 per octet, no split arithmetic).
template <int MODE, int CFG, bool kPlain, bool kPreA>
__global__ __launch_bounds__(Cfg<CFG>::kThreads, Cfg<CFG>::kWavesPerSimd) void conv_gemm_kernel(
    const float* __restrict__ a_src, const float* __restrict__ b_src,
    const float* __restrict__ x_mask, float* __restrict__ out, float* __restrict__ part_mean,
    float* __restrict__ part_m2, Geo g, int M, int N, int K, int k_chunk, int64_t split_stride,
    int accumulate, int64_t a_bytes, int64_t b_bytes, PhaseSet ps) {
  using C = Cfg<CFG>;
  if constexpr (MODE == kBwdData) {
    // this workgroup's stride phase (grid.z: one phase's grid after the other -- phases
    // as the fastest block index, the tiles of one pixel block together on one XCD, ran
    // the 3x3 stride-2 shapes 15-55 % slower, profiles/r4/phase_order/)
    if (ps.count > 0) {
      const int z = blockIdx.z;
      g.kh = ps.kh[z];
      g.kw = ps.kw[z];
      g.taps = g.kh * g.kw;
      g.ho = ps.ho[z];
      g.wo = ps.wo[z];
      g.dy0 = ps.dy0[z];
      g.dx0 = ps.dx0[z];
      g.oh = ps.oh[z];
      g.ow = ps.ow[z];
      g.fd_taps = ps.fd_taps[z];
      g.fd_kw = ps.fd_kw[z];
      g.fd_hwo = ps.fd_hwo[z];
      g.fd_wo = ps.fd_wo[z];
      a_src += ps.a_off[z];
      a_bytes = ps.a_bytes[z];
      K = g.co * g.taps;
      N = g.n * g.ho * g.wo;
    }
  }
  constexpr int WM = C::TM, WN = C::TN, kThreads = C::kThreads;
  constexpr bool kBK_major = MODE == kWgrad;
  constexpr bool kEmu = C::EMU;
  constexpr int kBImg = kBK_major || kEmu ? C::kBImgK : C::kBImgN;
  constexpr int SUB = C::SUB;
  __shared__ __attribute__((aligned(16))) float lds[C::kLdsFloats(MODE)];
  // buffer b, sub-stage u
  constexpr int kBufs = C::SINGLE ? 1 : 2;
  auto aimg = [&](int b, int u) { return lds + ((C::SINGLE ? 0 : b) * SUB + u) * C::kAImg; };
  auto bimg = [&](int b, int u) {
    return lds + kBufs * SUB * C::kAImg + ((C::SINGLE ? 0 : b) * SUB + u) * kBImg;
  };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % C::WVM, wn = wave / C::WVM;

  // XCD-aware block order: the 8 XCDs take consecutive blocks round-robin; remap so
  // each XCD owns a contiguous run of (m fastest) blocks, i.e. the m-blocks sharing a
  // column block (one B tile) run on one XCD's L2.
  const int mb_count = (M + C::BM - 1) / C::BM;
  int bid = blockIdx.x;
  const int nblk = gridDim.x;
  if ((nblk & 7) == 0) bid = (bid & 7) * (nblk >> 3) + (bid >> 3);
  const int mblk = bid % mb_count, nb_i = bid / mb_count;
  const int m0 = mblk * C::BM, n0 = nb_i * C::BN;
  if (n0 >= N) return;  // (a stride phase smaller than the grid's largest: whole workgroup)
  const int k_begin = blockIdx.y * k_chunk;
  const int k_end = min(K, k_begin + k_chunk);

  const __amdgpu_buffer_rsrc_t ar = rsrc(a_src, a_bytes);
  const __amdgpu_buffer_rsrc_t br = rsrc(b_src, b_bytes);
  const int hw_out = g.ho * g.wo, hw_in = g.h * g.w;
  const bool quads = kPlain && (hw_out & 3) == 0;

  constexpr int kRB = kBK_major ? C::kBQuadsK : C::kBQuadsN;
  static_assert(!kPreA || (kEmu && MODE != kWgrad), "pre-split A: EMU forward / bwd-data");
  constexpr int kAOct = kBK * C::BM / 8 / kThreads;  // pre-split A octets per thread
  constexpr int kAU = kPreA ? kAOct : C::kAQuads;    // A load units
  floatx4 ra[SUB][C::kAQuads], rb[SUB][kRB];
  floatx4 rs[SUB][kPreA ? kAOct : 1][3];  // pre-split A: the three planes of one octet

  // N-major B columns of this thread (forward / bwd-data): a quad of adjacent columns when
  // the operand is read as 16-byte quads (1x1, planes of 4k pixels), else columns BN/4
  // apart (store_nmajor's `spread`)
  constexpr int QPR = C::BN / 4;
  const bool spread = !kBK_major && g.spread &&
                      !(((MODE == kFwd && kPlain) ||
                         (MODE == kBwdData && (kPlain || (g.scatter && !g.phase)))) &&
                        (hw_out & 3) == 0);
  Col col[4];
  if constexpr (!kBK_major && kEmu) {
    // EMU: one column per thread, gathered as k quads of that column (the EMU image is
    // K-major for both operands)
    col[0] = make_col<MODE, kPlain>(g, n0 + tid % C::BN, N);
  } else if constexpr (!kBK_major) {
    const int jq = n0 + (tid % QPR) * (spread ? 1 : 4);
    const int cstep = spread ? QPR : 1;
#pragma unroll
    for (int e = 0; e < 4; ++e) col[e] = make_col<MODE, kPlain>(g, jq + cstep * e, N);
  }

  // Operand loads, one 16-byte quad per call (unit i of this thread's kAQuads / kRB), so the
  // main loop can spread a stage's loads between the MFMAs of the previous stage.  Tail
  // handling is by buffer offsets past the end (kOOB reads 0) selected per quad wherever the
  // quad layout allows it (K a multiple of 4; planes of 4k pixels), not by divergent
  // branches: those split the unit into basic blocks with exec-mask juggling around every
  // quad.
  const bool k4 = (K & 3) == 0;  // (then k_end is too: k quads never straddle it)
  // A: K-major rows (tid >> 3) + (threads / 8) i, k quad (tid & 7)
  auto load_a = [&](int k0, int i) -> floatx4 {
    const int k = k0 + 4 * (tid & 7);
    const int row = m0 + (tid >> 3) + (kThreads / 8) * i;
    floatx4 v;
    if constexpr (MODE == kFwd || MODE == kBwdData) {
      // forward W[co][ci*T + t] / transposed weight [ci][co*T]: K-contiguous rows
      if (MODE == kFwd || g.a_t) {
        if (k4) {
          v = bload4(ar, row < M && k < k_end ? static_cast<uint32_t>((row * K + k) * 4)
                                              : kOOB);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v[e] = bload(ar, row < M && k + e < k_end
                                 ? static_cast<uint32_t>((row * K + k + e) * 4) : kOOB);
        }
        return v;
      }
      // A[ci][co*T + t] = W[co][ci][t]: gathered from the untransposed weight (L2)
      const int T = g.taps;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        uint32_t off = kOOB;
        if (row < M && k + e < k_end) {
          const int co = T == 1 ? k + e : (k + e) / T;
          const int t = k + e - co * T;
          off = static_cast<uint32_t>(((co * g.ci + row) * T + t) * 4);
        }
        v[e] = bload(ar, off);
      }
      return v;
    } else {
      // dZ rows: A[co][k = (n, p)]
      if (quads) {  // K = n * hw_out, 4 | hw_out: a k quad is one image's 4 pixels
        const int n = g.fd_hwo.div(k), p = k - n * hw_out;
        v = bload4(ar, row < M && k < k_end
                           ? static_cast<uint32_t>(
                                 ((n * g.co_total + g.co_off + row) * hw_out + p) * 4)
                           : kOOB);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          uint32_t off = kOOB;
          if (row < M && k + e < k_end) {
            const int n = g.fd_hwo.div(k + e), p = k + e - n * hw_out;
            off = static_cast<uint32_t>(((n * g.co_total + g.co_off + row) * hw_out + p) * 4);
          }
          v[e] = bload(ar, off);
        }
      }
      return v;
    }
  };

  // pre-split A: row (tid >> 2) + (threads / 4) i, k octet (tid & 3) -- 48 bytes at
  // (row * ceil(K/8) + k/8) * 48 (k0 and k_end are multiples of 8 within K; the octet past
  // a K that is not is zero-padded)
  auto load_a_split = [&](int k0, int i, floatx4 (&v)[3]) {
    const int k = k0 + 8 * (tid & 3);
    const int row = m0 + (tid >> 2) + (kThreads / 4) * i;
    const uint32_t off = row < M && k < k_end
                             ? static_cast<uint32_t>((row * ((K + 7) >> 3) + (k >> 3)) * 48)
                             : kOOB;
#pragma unroll
    for (int p = 0; p < 3; ++p) v[p] = bload4(ar, off + 16 * p);
  };

  auto load_b = [&](int k0, int i) -> floatx4 {
    floatx4 v;
    if constexpr (MODE == kFwd) {
      // relu(X) taps: B[k = (ci, t)][j = output pixel]  (ReLU at store time: using the value
      // here would wait for the load)
      const int k = k0 + tid / QPR + (kThreads / QPR) * i;
      const bool kin = k < k_end;
      if constexpr (kPlain) {
        const int coff = k * hw_in;
        if (quads) {  // 4 | N: a column quad is valid or not as a whole
          v = bload4(br, col[0].ok && kin ? static_cast<uint32_t>((col[0].base + coff) * 4)
                                          : kOOB);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v[e] = bload(br, col[e].ok && kin
                                 ? static_cast<uint32_t>((col[e].base + coff) * 4) : kOOB);
        }
      } else {
        const int ci = g.fd_taps.div(k), t = k - ci * g.taps;
        const int th = g.fd_kw.div(t), tw = t - th * g.kw;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int yi = col[e].y + th, xi = col[e].x + tw;
          const bool ok = col[e].ok && kin && yi >= 0 && yi < g.h && xi >= 0 && xi < g.w;
          v[e] = bload(br, ok ? static_cast<uint32_t>(
                                    (col[e].base + (ci * g.h + yi) * g.w + xi) * 4) : kOOB);
        }
      }
    } else if constexpr (MODE == kBwdData) {
      // dZ taps: B[k = (co, t)][j = pixel]
      const int k = k0 + tid / QPR + (kThreads / QPR) * i;
      const bool kin = k < k_end;
      if (g.phase) {
        // dZ taps of this phase: dense, stride 1 (the decomposition removed the holes)
        const int co = g.fd_taps.div(k), t = k - co * g.taps;
        const int th = g.fd_kw.div(t), tw = t - th * g.kw;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int y = col[e].y - th, x = col[e].x - tw;
          const bool ok = col[e].ok && kin && y >= 0 && y < g.zh && x >= 0 && x < g.zw;
          v[e] = bload(br, ok ? static_cast<uint32_t>(
                                    (col[e].base + (co * g.zh + y) * g.zw + x) * 4) : kOOB);
        }
      } else if (kPlain || g.scatter) {
        const int coff = k * hw_out;
        if ((hw_out & 3) == 0) {  // adjacent column quads (no spread), valid as a whole
          v = bload4(br, col[0].ok && kin ? static_cast<uint32_t>((col[0].base + coff) * 4)
                                          : kOOB);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v[e] = bload(br, col[e].ok && kin
                                 ? static_cast<uint32_t>((col[e].base + coff) * 4) : kOOB);
        }
      } else {
        // output pixel * stride = input pixel + pad - tap - offset (stride holes: none)
        const int co = g.fd_taps.div(k), t = k - co * g.taps;
        const int th = g.fd_kw.div(t), tw = t - th * g.kw;
        if (g.sh == 1 && g.sw == 1) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int y = col[e].y - th, x = col[e].x - tw;
            const bool ok = col[e].ok && kin && y >= 0 && y < g.ho && x >= 0 && x < g.wo;
            v[e] = bload(br, ok ? static_cast<uint32_t>(
                                      (col[e].base + co * hw_out + y * g.wo + x) * 4) : kOOB);
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int ys = col[e].y - th, xs = col[e].x - tw;
            const int y = ys / g.sh, x = xs / g.sw;
            const bool ok = col[e].ok && kin && ys >= 0 && xs >= 0 && y * g.sh == ys &&
                            x * g.sw == xs && y < g.ho && x < g.wo;
            v[e] = bload(br, ok ? static_cast<uint32_t>(
                                      (col[e].base + co * hw_out + y * g.wo + x) * 4) : kOOB);
          }
        }
      }
    } else {
      // relu(X) taps: B[k = output pixel (n, p)][j = (ci, t)]  (ReLU at store time)
      const int k = k0 + 4 * (tid & 7);
      const int j = n0 + (tid >> 3) + (kThreads / 8) * i;
      const int ci = g.fd_taps.div(j), t = j - ci * g.taps;
      if (quads) {  // 1x1 stride 1 over planes of 4k pixels: a k quad is 4 adjacent pixels
        const int n = g.fd_hwo.div(k), p = k - n * hw_out;
        v = bload4(br, j < N && k < k_end
                           ? static_cast<uint32_t>(((n * g.ci + ci) * hw_in + p) * 4) : kOOB);
      } else {
        const int th = g.fd_kw.div(t), tw = t - th * g.kw;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          uint32_t off = kOOB;
          if (j < N && k + e < k_end) {
            const int n = g.fd_hwo.div(k + e), p = k + e - n * hw_out;
            const int y = g.fd_wo.div(p), x = p - y * g.wo;
            const int yi = y * g.sh - g.ph + th + g.oh, xi = x * g.sw - g.pw + tw + g.ow;
            if (yi >= 0 && yi < g.h && xi >= 0 && xi < g.w)
              off = static_cast<uint32_t>((((n * g.ci + ci) * g.h + yi) * g.w + xi) * 4);
          }
          v[e] = bload(br, off);
        }
      }
    }
    return v;
  };

  // EMU forward / backward-data B: k quad kq_of(i) of this thread's column col[0], one
  // element load per k (the lanes of a load read consecutive columns)
  auto kq_of = [&](int i) { return tid / C::BN + (kThreads / C::BN) * i; };
  auto load_b_emu = [&](int k0, int i) -> floatx4 {
    floatx4 v;
    const Col& c = col[0];
    const int kb = k0 + 4 * kq_of(i);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = kb + e;
      const bool kin = c.ok && k < k_end;
      uint32_t off = kOOB;
      if constexpr (MODE == kFwd) {
        if constexpr (kPlain) {
          if (kin) off = static_cast<uint32_t>((c.base + k * hw_in) * 4);
        } else {
          const int ci = g.fd_taps.div(k), t = k - ci * g.taps;
          const int th = g.fd_kw.div(t), tw = t - th * g.kw;
          const int yi = c.y + th, xi = c.x + tw;
          if (kin && yi >= 0 && yi < g.h && xi >= 0 && xi < g.w)
            off = static_cast<uint32_t>((c.base + (ci * g.h + yi) * g.w + xi) * 4);
        }
      } else {
        if (g.phase) {
          const int co = g.fd_taps.div(k), t = k - co * g.taps;
          const int th = g.fd_kw.div(t), tw = t - th * g.kw;
          const int y = c.y - th, x = c.x - tw;
          if (kin && y >= 0 && y < g.zh && x >= 0 && x < g.zw)
            off = static_cast<uint32_t>((c.base + (co * g.zh + y) * g.zw + x) * 4);
        } else if (kPlain || g.scatter) {
          if (kin) off = static_cast<uint32_t>((c.base + k * hw_out) * 4);
        } else {
          const int co = g.fd_taps.div(k), t = k - co * g.taps;
          const int th = g.fd_kw.div(t), tw = t - th * g.kw;
          const int ys = c.y - th, xs = c.x - tw;
          if (g.sh == 1 && g.sw == 1) {
            if (kin && ys >= 0 && ys < g.ho && xs >= 0 && xs < g.wo)
              off = static_cast<uint32_t>((c.base + co * hw_out + ys * g.wo + xs) * 4);
          } else {
            const int y = ys / g.sh, x = xs / g.sw;
            if (kin && ys >= 0 && xs >= 0 && y * g.sh == ys && x * g.sw == xs && y < g.ho &&
                x < g.wo)
              off = static_cast<uint32_t>((c.base + co * hw_out + y * g.wo + x) * 4);
          }
        }
      }
      v[e] = bload(br, off);
    }
    return v;
  };

  // load unit q of sub-stage u (A quads first, then B quads) for the stage at k0
  constexpr int kUnits = kAU + kRB;
  auto load_unit = [&](int k0, int u, int q) {
    if (q < kAU) {
      if constexpr (kPreA)
        load_a_split(k0 + u * kBK, q, rs[u][q]);
      else
        ra[u][q] = load_a(k0 + u * kBK, q);
    } else if constexpr (kEmu && !kBK_major) {
      rb[u][q - kAU] = load_b_emu(k0 + u * kBK, q - kAU);
    } else {
      rb[u][q - kAU] = load_b(k0 + u * kBK, q - kAU);
    }
  };
  // The forward / weight-gradient ReLU of X is applied here, after the stage's MFMAs:
  // applied in load_b it made every prefetch wait for its own loads (vmcnt(0) right
  // after issue), leaving the global-load latency exposed once per stage.
  auto store_stage = [&](int buf) {
    if constexpr (MODE != kBwdData) {
      if (g.relu) {
#pragma unroll
        for (int u = 0; u < SUB; ++u)
#pragma unroll
          for (int i = 0; i < kRB; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) rb[u][i][e] = relu(rb[u][i][e]);
      }
    }
    if constexpr (kEmu) {
#pragma unroll
      for (int u = 0; u < SUB; ++u) {
        if constexpr (kPreA) {
#pragma unroll
          for (int i = 0; i < kAOct; ++i) {
            __bf16* p = reinterpret_cast<__bf16*>(aimg(buf, u)) +
                        emu_off<C::BM>(tid & 3, (tid >> 2) + (kThreads / 4) * i);
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
              *reinterpret_cast<floatx4*>(p + pl * kBK * C::BM) = rs[u][i][pl];
          }
        } else {
#pragma unroll
          for (int i = 0; i < C::kAQuads; ++i)
            store_emu_quad<C::BM>(aimg(buf, u), ra[u][i], (tid >> 3) + (kThreads / 8) * i,
                                  tid & 7);
        }
#pragma unroll
        for (int i = 0; i < kRB; ++i) {
          if constexpr (kBK_major)
            store_emu_quad<C::BN>(bimg(buf, u), rb[u][i], (tid >> 3) + (kThreads / 8) * i,
                                  tid & 7);
          else
            store_emu_quad<C::BN>(bimg(buf, u), rb[u][i], tid % C::BN, kq_of(i));
        }
      }
      return;
    }
#pragma unroll
    for (int u = 0; u < SUB; ++u) {
      store_kmajor<C::BM, C::kAQuads, kThreads>(aimg(buf, u), ra[u], tid);
      if constexpr (kBK_major)
        store_kmajor<C::BN, C::kBQuadsK, kThreads>(bimg(buf, u), rb[u], tid);
      else
        store_nmajor<C::BN, C::kBQuadsN, kThreads>(bimg(buf, u), rb[u], tid, spread);
    }
  };

  floatx16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto run_stage = [&](const float* ai, const float* bi, auto&& between) {
    if constexpr (kEmu)
      mfma_stage_emu<CFG>(acc, ai, bi, lane, wm, wn, between);
    else
      mfma_stage<CFG, kBK_major>(acc, ai, bi, lane, wm, wn, between);
  };
  constexpr int kStageK = kBK * SUB;
  const int stages = (k_end - k_begin + kStageK - 1) / kStageK;
  if (stages > 0) {
#pragma unroll
    for (int u = 0; u < SUB; ++u)
#pragma unroll
      for (int q = 0; q < kUnits; ++q) load_unit(k_begin, u, q);
    store_stage(0);
    __syncthreads();
    // (the last stage is peeled off: with a `more` test inside the loop the compiler's
    // path-insensitive wait analysis assumed loads still in flight at the loop head and
    // put a vmcnt(0) in front of the interleaved loads)
    for (int s = 0; s + 1 < stages; ++s) {
      const int buf = s & 1;
      const int k_next = k_begin + (s + 1) * kStageK;
      // The MFMA groups carry the next stage's loads, so the address arithmetic, exec masks
      // and load issue of a unit run while the matrix core works through the dependent MFMA
      // chain instead of in front of it (~200 instructions per stage serialised with 1024 MFMA cycles:
      // 0.41-0.47 MFMA busy on the AmoebaNet 7^2 / 14^2 shapes, profiles/r4/pmc).
      // (The 8-wave 128 x 128 tile keeps its loads in front for the gathered forward and
      // the backward-data: interleaved, their unit temporaries pass the 128 registers of two
      // workgroups per CU and spill.)
      constexpr bool kInterleave = CFG != 1 || MODE == kWgrad || (MODE == kFwd && kPlain);
      if constexpr (!kInterleave) {
#pragma unroll
        for (int u = 0; u < SUB; ++u)
#pragma unroll
          for (int q = 0; q < kUnits; ++q) load_unit(k_next, u, q);
      }
      // sub-stage u's MFMA groups carry the next stage's sub-stage u loads, spread over the
      // first half of the groups: each unit then keeps half a sub-stage of MFMAs to cover
      // its latency before store_stage waits for it
#pragma unroll
      for (int u = 0; u < SUB; ++u)
        run_stage(aimg(buf, u), bimg(buf, u), [&](int grp) {
                                     if constexpr (kInterleave) {
#pragma unroll
                                       for (int q = 0; q < kUnits; ++q)
                                         if (q * (kBK / 8) / kUnits == grp) {
                                           load_unit(k_next, u, q);
                                           __builtin_amdgcn_sched_barrier(0);
                                         }
                                     }
                                   });
      if constexpr (C::SINGLE) {
        __syncthreads();  // every wave is done reading the one buffer
        store_stage(0);
      } else {
        store_stage(buf ^ 1);
      }
      __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < SUB; ++u)
      run_stage(aimg((stages - 1) & 1, u), bimg((stages - 1) & 1, u), [](int) {});
    __syncthreads();
  }

  // ---- epilogues ----
  // split reductions: each split writes its own slice of a workspace (reduced by
  // split_reduce_kernel), plain stores, no atomics
  out += blockIdx.y * split_stride;
  const int h = lane >> 5, l32 = lane & 31;
  if constexpr (MODE == kWgrad) {
    // dW[co][ci*T + t] (or this split's workspace slice)
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        const int cj = n0 + wn * 32 * WN + j * 32 + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm * 32 * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (row < M && cj < N) {
            // (one split: this is the gradient itself, accumulated into .grad when asked)
            float* o = out + static_cast<int64_t>(row) * N + cj;
            *o = accumulate ? *o + acc[i][j][r] : acc[i][j][r];
          }
        }
      }
    return;
  }

  // C tile through LDS (reusing the operand images): coalesced row stores.
  float* ct = lds;
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * 32 * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int cc = wn * 32 * WN + j * 32 + l32;
        ct[row * C::kCStride + cc] = acc[i][j][r];
      }
  __syncthreads();

  constexpr int kQuads = C::BN / 4;
  const bool scatter = MODE == kBwdData && g.scatter;
  const int hw = (MODE == kFwd || scatter) ? hw_out : hw_in;
  const FastDiv& fdh = (MODE == kFwd || scatter) ? g.fd_hwo : g.fd_hwi;
  const int ch_total = MODE == kFwd ? g.co_total : g.ci;
  const int ch_off = MODE == kFwd ? g.co_off : 0;
  const __amdgpu_buffer_rsrc_t mr = rsrc(x_mask, x_mask ? static_cast<int64_t>(g.n) * g.ci *
                                                              hw_in * 4 : 0);
  for (int idx = tid; idx < C::BM * kQuads; idx += kThreads) {
    const int row = idx / kQuads, q = idx - row * kQuads;
    const int m = m0 + row, j = n0 + 4 * q;
    if (m >= M || j >= N) continue;
    floatx4 v = *reinterpret_cast<const floatx4*>(ct + row * C::kCStride + 4 * q);
    if (scatter) {
      // strided 1x1 backward-data: output pixel (y, x) -> input (y*sh+oh, x*sw+ow)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int je = j + e;
        if (je >= N) break;
        const int n = g.fd_hwo.div(je), p = je - n * hw_out;
        const int y = g.fd_wo.div(p), x = p - y * g.wo;
        const int yi = y * g.sh - g.ph + g.oh, xi = x * g.sw - g.pw + g.ow;
        if (yi < 0 || yi >= g.h || xi < 0 || xi >= g.w) continue;
        const int64_t off = ((static_cast<int64_t>(n) * g.ci + m) * g.h + yi) * g.w + xi;
        float val = v[e];
        if (g.relu && !(bload(mr, static_cast<uint32_t>(off * 4)) > 0.f)) val = 0.f;
        if (g.fill) {  // (host-checked: stride 2, even width, no padding, offset or accumulate)
          *reinterpret_cast<floatx2*>(out + off) = floatx2{val, 0.f};
          if (yi + 1 < g.h) *reinterpret_cast<floatx2*>(out + off + g.w) = floatx2{0.f, 0.f};
          continue;
        }
        out[off] = accumulate ? out[off] + val : val;
      }
      continue;
    }
    const int n = fdh.div(j), p = j - n * hw;
    const int64_t base = (static_cast<int64_t>(n) * ch_total + ch_off + m) * hw + p;
    if ((hw & 3) == 0 && j + 3 < N) {
      if constexpr (MODE == kBwdData) {
        if (g.relu) {
          const floatx4 xv = bload4(mr, static_cast<uint32_t>(base * 4));
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = xv[e] > 0.f ? v[e] : 0.f;
        }
      }
      if (MODE == kBwdData && accumulate) v += *reinterpret_cast<const floatx4*>(out + base);
      *reinterpret_cast<floatx4*>(out + base) = v;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int je = j + e;
        if (je >= N) break;
        const int ne = fdh.div(je), pe = je - ne * hw;
        const int64_t off = (static_cast<int64_t>(ne) * ch_total + ch_off + m) * hw + pe;
        float val = v[e];
        if constexpr (MODE == kBwdData) {
          if (g.relu && !(bload(mr, static_cast<uint32_t>(off * 4)) > 0.f)) val = 0.f;
        }
        out[off] = (MODE == kBwdData && accumulate) ? out[off] + val : val;
      }
    }
  }

  if constexpr (MODE == kFwd) {
    if (part_mean == nullptr) return;
    // BatchNorm statistics of this block's columns: one wave per row at a time, lanes
    // across columns (conflict-free LDS reads), shuffle-reduced mean then centred M2.
    const int cols = min(C::BN, N - n0);
    constexpr int kWaves = kThreads / 64;
    for (int row = wave; row < C::BM; row += kWaves) {
      const float* r = ct + row * C::kCStride;
      float s = 0.f;
      for (int c = lane; c < cols; c += 64) s += r[c];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
      const float mean = s / static_cast<float>(cols);
      float m2 = 0.f;
      for (int c = lane; c < cols; c += 64) {
        const float d = r[c] - mean;
        m2 += d * d;
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) m2 += __shfl_xor(m2, off);
      const int m = m0 + row;
      if (lane == 0 && m < M) {
        part_mean[static_cast<int64_t>(nb_i) * g.co_total + g.co_off + m] = mean;
        part_m2[static_cast<int64_t>(nb_i) * g.co_total + g.co_off + m] = m2;
      }
    }
  }
}

template <int MODE, int CFG>
void launch_cfg(const float* a, const float* b, const float* xm, float* out, float* pmean,
                float* pm2, const Geo& g, int M, int N, int K, int splits, int64_t split_stride,
                bool accumulate, int64_t a_bytes, int64_t b_bytes, hipStream_t stream,
                const PhaseSet& ps = PhaseSet{}, bool pre_a = false) {
  using C = Cfg<CFG>;
  const int mb = (M + C::BM - 1) / C::BM, nb = (N + C::BN - 1) / C::BN;
  int k_chunk = (K + splits - 1) / splits;
  k_chunk = (k_chunk + kBK - 1) / kBK * kBK;  // (the plan's split count: whole BK steps)
  const int zs = (K + k_chunk - 1) / k_chunk;
  const bool plain = g.taps == 1 && g.sh == 1 && g.sw == 1 && g.ph == 0 && g.pw == 0 &&
                     g.oh == 0 && g.ow == 0;
  const dim3 grid(mb * nb, zs, ps.count > 0 ? ps.count : 1), block(C::kThreads);
  auto go = [&](auto plain_c, auto pre_c) {
    hipLaunchKernelGGL((conv_gemm_kernel<MODE, CFG, decltype(plain_c)::value,
                                         decltype(pre_c)::value>),
                       grid, block, 0, stream, a, b, xm, out, pmean, pm2, g, M, N, K, k_chunk,
                       split_stride, accumulate ? 1 : 0, a_bytes, b_bytes, ps);
  };
  using T = std::true_type;
  using F = std::false_type;
  if constexpr (C::EMU && MODE != kWgrad) {
    if (pre_a) {
      if (plain) go(T{}, T{}); else go(F{}, T{});
      return;
    }
  }
  if (plain) go(T{}, F{}); else go(F{}, F{});
}

// A operand of a forward / backward-data GEMM split into bf16 planes once (see
// launch_conv_gemm_presplit): one thread per (row, k octet), split1 as the GEMM kernels
// would split it (bit-identical products).
__global__ __launch_bounds__(256) void conv_gemm_presplit_kernel(const float* __restrict__ w,
                                                                 bf16x8* __restrict__ out,
                                                                 int M, int K, int ko, int taps,
                                                                 int transposed) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (idx >= static_cast<int64_t>(M) * ko) return;
  const int row = static_cast<int>(idx / ko), j = static_cast<int>(idx - static_cast<int64_t>(row) * ko);
  bf16x8 hi, mid, lo;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = 8 * j + e;
    float v = 0.f;
    if (k < K) {
      if (transposed) {  // A[ci = row][co * T + t] = W[co][ci][t]
        const int co = k / taps, t = k - co * taps;
        v = w[(static_cast<int64_t>(co) * M + row) * taps + t];
      } else {
        v = w[static_cast<int64_t>(row) * K + k];
      }
    }
    __bf16 h, m, l;
    split1(v, h, m, l);
    hi[e] = h;
    mid[e] = m;
    lo[e] = l;
  }
  out[3 * idx] = hi;
  out[3 * idx + 1] = mid;
  out[3 * idx + 2] = lo;
}

// Sum of the split partials: ws[s][plane][c][hw] -> out[plane][c_off + c][hw] (c_total
// channels), times the ReLU mask (x_mask, indexed like out) when given, plus the
// previous contents of out when accumulating.  A workgroup covers 64 quads (or 64
// elements) with its 4 waves each summing every 4th split through 4 independent
// accumulators (16 loads in flight per lane), then the waves combine through LDS: the
// weight gradient's 30-60-way splits no longer walk a serial chain of dependent loads
// per element (measured 12 us for 62 x 64 KiB partials with one lane per element).
template <bool kVec>
__global__ __launch_bounds__(256) void split_reduce_kernel(
    const float* __restrict__ ws, int splits, int64_t stride, float* __restrict__ out,
    const float* __restrict__ mask, int accumulate, int64_t total, int64_t c, int64_t hw,
    int64_t c_total, int64_t c_off) {
  constexpr int kE = kVec ? 4 : 1;
  typedef float V __attribute__((ext_vector_type(kE)));
  __shared__ V part[3][64];
  const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int64_t items = total / kE;
  const int64_t q = static_cast<int64_t>(blockIdx.x) * 64 + lane;
  const bool ok = q < items;
  const V* src = reinterpret_cast<const V*>(ws) + (ok ? q : 0);
  const int64_t vstride = stride / kE;
  V acc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) acc[u] = V(0.f);
  int sp = grp;
  for (; sp + 12 < splits; sp += 16) {
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] += src[(sp + 4 * u) * vstride];
  }
  for (; sp < splits; sp += 4) acc[0] += src[sp * vstride];
  V v = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  if (grp > 0) part[grp - 1][lane] = v;
  __syncthreads();
  if (grp != 0 || !ok) return;
  v += part[0][lane] + part[1][lane] + part[2][lane];
  const int64_t i = q * kE;
  const int64_t pl = i / (c * hw), r = i - pl * c * hw;
  const int64_t o = (pl * c_total + c_off) * hw + r;
  V* dst = reinterpret_cast<V*>(out + o);
  if (mask) {
    const V m = *reinterpret_cast<const V*>(mask + o);
#pragma unroll
    for (int e = 0; e < kE; ++e) v[e] = m[e] > 0.f ? v[e] : 0.f;
  }
  if (accumulate) v += *dst;
  *dst = v;
}

void launch_split_reduce(const float* ws, int splits, int64_t stride, float* out,
                         const float* mask, bool accumulate, int64_t planes, int64_t c,
                         int64_t hw, int64_t c_total, int64_t c_off, hipStream_t stream) {
  const int64_t total = planes * c * hw;
  if (total == 0) return;
  // quads never straddle a channel plane when hw % 4 == 0, and a single dense output
  // (backward-data / weight-gradient partials: planes 1, hw 1) is one flat array
  const bool flat = planes == 1 && c_off == 0 && c_total == c;
  const bool vec = ((hw & 3) == 0 || (flat && (total & 3) == 0)) && (stride & 3) == 0;
  const int64_t items = vec ? total / 4 : total;
  const unsigned blocks = static_cast<unsigned>((items + 63) / 64);
  if (vec)
    hipLaunchKernelGGL(split_reduce_kernel<true>, dim3(blocks), dim3(256), 0, stream, ws, splits,
                       stride, out, mask, accumulate ? 1 : 0, total, c, hw, c_total, c_off);
  else
    hipLaunchKernelGGL(split_reduce_kernel<false>, dim3(blocks), dim3(256), 0, stream, ws,
                       splits, stride, out, mask, accumulate ? 1 : 0, total, c, hw, c_total,
                       c_off);
}

// Forward split reduction fused with the BatchNorm statistics pass: one wave per (image,
// channel) plane of this convolution sums the split partials ws[s][img][ch][p] in split
// order, stores the plane into z[img][c_off + ch], and writes the plane's mean and centred
// M2 to pm / pm2[img][c_off + ch] (per-image partials, like launch_bn_stats): one launch
// where split_reduce + bn_stats took two.  kPer > 0: the plane (<= 64 * kPer pixels) stays
// in registers for the M2 pass; kPer = 0: each lane re-reads the pixels it stored.
template <int kPer>
__global__ __launch_bounds__(256) void split_reduce_stats_kernel(
    const float* __restrict__ ws, int splits, int64_t stride, float* __restrict__ z,
    float* __restrict__ pm, float* __restrict__ pm2, int64_t planes, int c, int hw, int c_total,
    int c_off) {
  const int lane = threadIdx.x & 63;
  const int64_t plane = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (plane >= planes) return;
  const int64_t img = plane / c;
  const int ch = static_cast<int>(plane - img * c);
  const float* src = ws + plane * hw;
  float* dst = z + (img * c_total + c_off + ch) * hw;
  float sum = 0.f;
  float v[kPer > 0 ? kPer : 1];
  if constexpr (kPer > 0) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) v[i] = 0.f;
    for (int s = 0; s < splits; ++s) {
      const float* sp = src + s * stride;
#pragma unroll
      for (int i = 0; i < kPer; ++i) {
        const int p = lane + 64 * i;
        if (p < hw) v[i] += sp[p];
      }
    }
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int p = lane + 64 * i;
      if (p < hw) {
        dst[p] = v[i];
        sum += v[i];
      }
    }
  } else {
    for (int p = lane; p < hw; p += 64) {
      float a0 = 0.f, a1 = 0.f;
      int s = 0;
      for (; s + 1 < splits; s += 2) {
        a0 += src[s * stride + p];
        a1 += src[(s + 1) * stride + p];
      }
      if (s < splits) a0 += src[s * stride + p];
      const float t = a0 + a1;
      dst[p] = t;
      sum += t;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off);
  const float mean = sum / static_cast<float>(hw);
  float m2 = 0.f;
  if constexpr (kPer > 0) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int p = lane + 64 * i;
      if (p < hw) {
        const float d = v[i] - mean;
        m2 += d * d;
      }
    }
  } else {
    for (int p = lane; p < hw; p += 64) {  // this lane's own stores: program-order reads
      const float d = dst[p] - mean;
      m2 += d * d;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m2 += __shfl_xor(m2, off);
  if (lane == 0) {
    pm[img * c_total + c_off + ch] = mean;
    pm2[img * c_total + c_off + ch] = m2;
  }
}

// Planes of <= 64 pixels (AmoebaNet's 7^2): one wave per plane spent its life on one
// chain of `splits` dependent loads (58 us per call for 40 k planes at micro-batch 40 in
// the stage-6 trace, profiles/r4/rocprof/).  Here a wave takes 4 planes and loads two splits
// of all of them before adding -- 8 loads in flight -- summing each plane in split order
// (bitwise the sums of the kernel above), then the four planes' statistics.
__global__ __launch_bounds__(256) void split_reduce_stats_small_kernel(
    const float* __restrict__ ws, int splits, int64_t stride, float* __restrict__ z,
    float* __restrict__ pm, float* __restrict__ pm2, int64_t planes, int c, int hw, int c_total,
    int c_off) {
  constexpr int P = 4;
  const int lane = threadIdx.x & 63;
  const int64_t p0 = (static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6)) * P;
  if (p0 >= planes) return;
  bool ok[P];
#pragma unroll
  for (int k = 0; k < P; ++k) ok[k] = lane < hw && p0 + k < planes;
  float v[P];
#pragma unroll
  for (int k = 0; k < P; ++k) v[k] = 0.f;
  const float* src = ws + p0 * hw + lane;
  int s = 0;
  for (; s + 1 < splits; s += 2) {
    float a[P], b[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
      a[k] = ok[k] ? src[s * stride + k * hw] : 0.f;
      b[k] = ok[k] ? src[(s + 1) * stride + k * hw] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < P; ++k) v[k] = (v[k] + a[k]) + b[k];
  }
  if (s < splits) {
#pragma unroll
    for (int k = 0; k < P; ++k) v[k] += ok[k] ? src[s * stride + k * hw] : 0.f;
  }
  float sum[P], m2[P], mean[P];
#pragma unroll
  for (int k = 0; k < P; ++k) sum[k] = ok[k] ? v[k] : 0.f;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
#pragma unroll
    for (int k = 0; k < P; ++k) sum[k] += __shfl_xor(sum[k], off);
#pragma unroll
  for (int k = 0; k < P; ++k) {
    mean[k] = sum[k] / static_cast<float>(hw);
    const float d = v[k] - mean[k];
    m2[k] = ok[k] ? d * d : 0.f;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
#pragma unroll
    for (int k = 0; k < P; ++k) m2[k] += __shfl_xor(m2[k], off);
#pragma unroll
  for (int k = 0; k < P; ++k) {
    if (p0 + k >= planes) break;
    const int64_t plane = p0 + k;
    const int64_t img = plane / c;
    const int ch = static_cast<int>(plane - img * c);
    if (ok[k]) z[(img * c_total + c_off + ch) * hw + lane] = v[k];
    if (lane == 0) {
      pm[img * c_total + c_off + ch] = mean[k];
      pm2[img * c_total + c_off + ch] = m2[k];
    }
  }
}

void launch_split_reduce_stats(const float* ws, int splits, int64_t stride, float* z, float* pm,
                               float* pm2, int64_t n, int c, int hw, int c_total, int c_off,
                               hipStream_t stream) {
  const int64_t planes = n * c;
  if (planes == 0 || hw == 0) return;
  const dim3 grid(static_cast<unsigned>((planes + 3) / 4)), block(256);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, block, 0, stream, ws, splits, stride, z, pm, pm2, planes, c, hw,
                       c_total, c_off);
  };
  if (hw <= 64) {
    hipLaunchKernelGGL(split_reduce_stats_small_kernel,
                       dim3(static_cast<unsigned>((planes + 15) / 16)), block, 0, stream, ws,
                       splits, stride, z, pm, pm2, planes, c, hw, c_total, c_off);
  } else if (hw <= 256) go(split_reduce_stats_kernel<4>);
  else if (hw <= 1024) go(split_reduce_stats_kernel<16>);
  else go(split_reduce_stats_kernel<0>);
}

// Deferred weight gradients (launch_conv_gemm_wgrad_slab): grad[i] (+)= sum_s slab[s][i] for a
// table of parameters in one launch, splits summed in order (bitwise reproducible).  Each
// workgroup covers 1024 floats of one entry; the entry is found from the prefix of block
// counts in the (by-value) table.
struct SlabTable {
  const float* slab[kSlabFlushMax];
  float* grad[kSlabFlushMax];
  int64_t numel[kSlabFlushMax];
  int splits[kSlabFlushMax];
  int accumulate[kSlabFlushMax];
  int block_end[kSlabFlushMax];  // exclusive prefix of workgroups per entry
  int count;
};

__global__ __launch_bounds__(256) void slab_flush_kernel(SlabTable t) {
  int e = 0;
  while (e + 1 < t.count && static_cast<int>(blockIdx.x) >= t.block_end[e]) ++e;
  const int first_block = e == 0 ? 0 : t.block_end[e - 1];
  const int64_t numel = t.numel[e];
  const int64_t base = static_cast<int64_t>(blockIdx.x - first_block) * 1024 + 4 * threadIdx.x;
  const float* slab = t.slab[e];
  float* grad = t.grad[e];
  const int splits = t.splits[e];
  if ((numel & 3) == 0) {
    if (base >= numel) return;
    floatx4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
    int s = 0;
    for (; s + 1 < splits; s += 2) {
      a0 += *reinterpret_cast<const floatx4*>(slab + s * numel + base);
      a1 += *reinterpret_cast<const floatx4*>(slab + (s + 1) * numel + base);
    }
    if (s < splits) a0 += *reinterpret_cast<const floatx4*>(slab + s * numel + base);
    floatx4 v = a0 + a1;
    if (t.accumulate[e]) v += *reinterpret_cast<const floatx4*>(grad + base);
    *reinterpret_cast<floatx4*>(grad + base) = v;
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t i = base + k;
      if (i >= numel) break;
      float a = 0.f;
      for (int s = 0; s < splits; ++s) a += slab[s * numel + i];
      grad[i] = t.accumulate[e] ? grad[i] + a : a;
    }
  }
}

Geo make_geo(const ConvGemmGeo& cg) {
  // TGPIPE_CG_SPREAD=0: element-gathered columns as adjacent quads (the round-2 mapping)
  static const int spread = env_int("TGPIPE_CG_SPREAD", 1) != 0 ? 1 : 0;
  Geo g{cg.n, cg.ci, cg.h, cg.w, cg.co, cg.ho, cg.wo, cg.co_total, cg.co_off, cg.kh, cg.kw,
        cg.kh * cg.kw, cg.sh, cg.sw, cg.ph, cg.pw, cg.oh, cg.ow, cg.relu ? 1 : 0, 0,
        cg.a_t ? 1 : 0, spread, {}, {}, {}, {}, {},
        cg.phase ? 1 : 0, cg.zh, cg.zw, cg.dy0, cg.dx0, cg.fill ? 1 : 0};
  g.fd_taps = make_fastdiv(g.taps);
  g.fd_kw = make_fastdiv(g.kw);
  g.fd_hwo = make_fastdiv(g.ho * g.wo);
  g.fd_wo = make_fastdiv(g.wo);
  g.fd_hwi = make_fastdiv(g.h * g.w);
  return g;
}

void gemm_dims(int mode, const Geo& g, int& M, int& N, int& K) {
  if (mode == kFwd) {
    M = g.co; N = g.n * g.ho * g.wo; K = g.ci * g.taps;
  } else if (mode == kBwdData) {
    M = g.ci; N = g.n * (g.scatter ? g.ho * g.wo : g.h * g.w); K = g.co * g.taps;
  } else {
    M = g.co; N = g.ci * g.taps; K = g.n * g.ho * g.wo;
  }
}

// Block width (rows = columns) of a tile configuration, and the runtime -> template dispatch.
int cfg_width(int cfg) {
  return cfg == 0 || cfg == 3 || cfg == 6 || cfg == 7 || cfg == 11 ? 64 : 128;
}

template <typename F>
void with_cfg(int cfg, F&& f) {
  switch (cfg) {
    case 1: f(std::integral_constant<int, 1>{}); break;
    case 2: f(std::integral_constant<int, 2>{}); break;
    case 3: f(std::integral_constant<int, 3>{}); break;
    case 4: f(std::integral_constant<int, 4>{}); break;
    case 5: f(std::integral_constant<int, 5>{}); break;
    case 6: f(std::integral_constant<int, 6>{}); break;
    case 7: f(std::integral_constant<int, 7>{}); break;
    case 8: f(std::integral_constant<int, 8>{}); break;
    case 9: f(std::integral_constant<int, 9>{}); break;
    case 10: f(std::integral_constant<int, 10>{}); break;
    case 11: f(std::integral_constant<int, 11>{}); break;
    default: f(std::integral_constant<int, 0>{}); break;
  }
}

// TGPIPE_CG_SINGLE=1: plans naming CFG 9 (the double-buffered 8-wave split-bf16 tile) run
// CFG 10, its single-buffered twin at two workgroups per CU (same tile, same products).
int run_cfg(int cfg) {
  static const bool single = env_int("TGPIPE_CG_SINGLE", 0) != 0;
  return cfg == 9 && single ? 10 : cfg;
}

// TGPIPE_CG_EMU=0: the split-bf16 configurations are never candidates (exact f32 MFMA only;
// a plan naming one falls back to the heuristic).
bool emu_enabled() {
  static const bool on = env_int("TGPIPE_CG_EMU", 1) != 0;
  return on;
}

bool scatter_bwd(const ConvGemmGeo& cg) {
  return cg.phase || (cg.kh == 1 && cg.kw == 1 && (cg.sh > 1 || cg.sw > 1));
}

}  // namespace

int env_int(const char* name, int fallback) {
  const char* v = std::getenv(name);
  return v != nullptr && *v != 0 ? std::atoi(v) : fallback;
}

bool conv_gemm_emu_cfg(int cfg) { return cfg >= kFirstEmuCfg && cfg < kConvGemmCfgs; }

void launch_conv_gemm_presplit(const float* w, void* out, int M, int K, int taps,
                               bool transposed, hipStream_t stream) {
  const int ko = (K + 7) / 8;
  const int64_t total = static_cast<int64_t>(M) * ko;
  if (total == 0) return;
  hipLaunchKernelGGL(conv_gemm_presplit_kernel, dim3(static_cast<unsigned>((total + 255) / 256)),
                     dim3(256), 0, stream, w, static_cast<bf16x8*>(out), M, K, ko,
                     std::max(1, taps), transposed ? 1 : 0);
}

bool conv_gemm_phased(const ConvGemmGeo& g) {
  return !g.phase && (g.kh > 1 || g.kw > 1) && (g.sh > 1 || g.sw > 1) && g.oh == 0 &&
         g.ow == 0;
}

// Residue (a, b) of the input pixel modulo the stride: the taps th = th0 + sh*i with
// th0 = (a + ph) mod sh meet it (y + ph - th divisible by sh), reading dZ row
// (y + ph - th) / sh = yy + dy0 - i for y = sh*yy + a, dy0 = (a + ph - th0) / sh.
std::vector<ConvGemmPhase> conv_gemm_phases(const ConvGemmGeo& g) {
  std::vector<ConvGemmPhase> out;
  for (int a = 0; a < g.sh && a < g.h; ++a) {
    const int th0 = (a + g.ph) % g.sh;
    if (th0 >= g.kh) continue;
    for (int b = 0; b < g.sw && b < g.w; ++b) {
      const int tw0 = (b + g.pw) % g.sw;
      if (tw0 >= g.kw) continue;
      ConvGemmPhase p{g, th0, tw0};
      ConvGemmGeo& q = p.geo;
      q.phase = true;
      q.kh = (g.kh - th0 + g.sh - 1) / g.sh;
      q.kw = (g.kw - tw0 + g.sw - 1) / g.sw;
      q.ho = (g.h - a + g.sh - 1) / g.sh;  // this phase's pixel grid
      q.wo = (g.w - b + g.sw - 1) / g.sw;
      q.zh = g.ho;
      q.zw = g.wo;
      q.dy0 = (a + g.ph - th0) / g.sh;
      q.dx0 = (b + g.pw - tw0) / g.sw;
      q.ph = q.pw = 0;  // destination pixel (sh*y + oh, sw*x + ow) in the epilogue
      q.oh = a;
      q.ow = b;
      q.a_t = true;
      out.push_back(p);
    }
  }
  return out;
}

ConvGemmPlan conv_gemm_plan(int mode, const ConvGemmGeo& cg) {
  Geo g = make_geo(cg);
  g.scatter = mode == kBwdData && scatter_bwd(cg);
  int M, N, K;
  gemm_dims(mode, g, M, N, K);
  ConvGemmPlan plan;
  // Workgroups per launch to aim for: the 128 x 128 kernel runs 2 per CU (LDS), the
  // 64 x 64 one 4; fewer leave SIMDs with a single wave that cannot hide its own
  // global-load latency, so small grids split the reduction (>= 4 stages per split).
  static const int fill_big = env_int("TGPIPE_CG_FILL_BIG", 200);
  static const int fill_small = env_int("TGPIPE_CG_FILL_SMALL", 200);
  static const int target_small = env_int("TGPIPE_CG_TARGET_SMALL", 400);
  static const int target_wgrad = env_int("TGPIPE_CG_TARGET_WGRAD", 512);
  const int64_t big = static_cast<int64_t>((M + 127) / 128) * ((N + 127) / 128);
  const int64_t small = static_cast<int64_t>((M + 63) / 64) * ((N + 63) / 64);
  const int64_t max_split = std::max<int64_t>(1, K / (4 * kBK));
  if (mode == kWgrad) {
    // few output tiles, long reduction: split until ~512 workgroups
    plan.cfg = big >= 64 ? 1 : 0;
    const int64_t tiles = plan.cfg ? big : small;
    plan.splits = static_cast<int>(
        std::min<int64_t>((target_wgrad + tiles - 1) / tiles, max_split));
  } else {
    static const int bigsplit_k = env_int("TGPIPE_CG_BIGSPLIT_MINK", 1 << 30);
    static const int target_big = env_int("TGPIPE_CG_TARGET_BIG", 256);
    if (big < fill_big && K >= bigsplit_k) {
      // long reduction over a small output: 8-wave 128 x 128 tiles, split reduction
      plan.cfg = 1;
      plan.splits = static_cast<int>(std::min<int64_t>((target_big + big - 1) / big, max_split));
    } else {
      plan.cfg = big >= fill_big ? 1 : 0;
      const int64_t tiles = plan.cfg ? big : small;
      const int64_t fill = plan.cfg ? fill_big : fill_small;
      plan.splits = tiles >= fill ? 1
                    : static_cast<int>(std::min<int64_t>((target_small + tiles - 1) / tiles,
                                                         max_split));
    }
  }
  if (plan.splits < 1 || g.scatter) plan.splits = 1;
  // The split-bf16 tiles of the same shapes won 628 of the 709 measured plans
  // (tuned/conv_gemm_mi355x.txt): shapes missing from the table take them too -- 7 for 0,
  // and for 1 the single-buffered 10 (two workgroups per CU; profiles/KERNELS.md "Round 6").
  if (emu_enabled()) plan.cfg = plan.cfg == 1 ? 10 : 7;
  // the launch rounds each split to whole stages: report the number it really runs
  int k_chunk = (K + plan.splits - 1) / plan.splits;
  k_chunk = (k_chunk + kBK - 1) / kBK * kBK;
  plan.splits = std::max(1, (K + k_chunk - 1) / k_chunk);
  plan.col_width = cfg_width(plan.cfg);
  plan.col_blocks = static_cast<int>((N + plan.col_width - 1) / plan.col_width);
  plan.scatter = g.scatter;
  return plan;
}

std::vector<ConvGemmPlan> conv_gemm_candidates(int mode, const ConvGemmGeo& cg) {
  Geo g = make_geo(cg);
  g.scatter = mode == kBwdData && scatter_bwd(cg);
  int M, N, K;
  gemm_dims(mode, g, M, N, K);
  std::vector<ConvGemmPlan> out;
  const int max_split = std::max(1, K / (4 * kBK));
  const int cfgs = emu_enabled() ? kConvGemmCfgs : kFirstEmuCfg;
  for (int cfg = 0; cfg < cfgs; ++cfg) {
    const int wd = cfg_width(cfg);
    const int64_t tiles = static_cast<int64_t>((M + wd - 1) / wd) * ((N + wd - 1) / wd);
    int last = 0;
    for (int s : {1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 64, 128, 256, 512, 1024}) {
      if (s > 1 && (s > max_split || g.scatter || tiles * s > 8192)) break;
      int k_chunk = (K + s - 1) / s;
      k_chunk = (k_chunk + kBK - 1) / kBK * kBK;
      const int real = std::max(1, (K + k_chunk - 1) / k_chunk);
      if (real == last) continue;
      last = real;
      ConvGemmPlan p;
      p.cfg = cfg;
      p.splits = real;
      p.col_width = wd;
      p.col_blocks = static_cast<int>((N + p.col_width - 1) / p.col_width);
      p.scatter = g.scatter;
      out.push_back(p);
    }
  }
  return out;
}

int64_t conv_gemm_workspace(int mode, const ConvGemmGeo& cg, const ConvGemmPlan& plan) {
  if (plan.splits <= 1) return 0;
  Geo g = make_geo(cg);
  int M, N, K;
  gemm_dims(mode, g, M, N, K);
  // one output-shaped slice per split (forward: this convolution's channels only)
  return static_cast<int64_t>(plan.splits) * M * N;
}

void launch_conv_gemm(int mode, const float* a, const float* b, const float* x_mask, float* out,
                      float* part_mean, float* part_m2, const ConvGemmGeo& cg,
                      const ConvGemmPlan& plan, bool accumulate, float* ws, int64_t a_bytes,
                      int64_t b_bytes, hipStream_t stream) {
  Geo g = make_geo(cg);
  g.scatter = plan.scatter || cg.phase ? 1 : 0;
  int M, N, K;
  gemm_dims(mode, g, M, N, K);
  if (M == 0 || N == 0) return;
  const bool split = plan.splits > 1;
  const int64_t stride = split ? static_cast<int64_t>(M) * N : 0;
  float* dst = out;
  Geo gk = g;
  if (split) {
    // the GEMM writes raw partial sums into ws; split_reduce applies the channel slice,
    // the ReLU mask and the accumulation
    dst = ws;
    if (mode == kFwd) {
      gk.co_total = g.co;
      gk.co_off = 0;
    } else if (mode == kBwdData) {
      gk.relu = 0;
    }
  }
  float* pm = split ? nullptr : part_mean;
  float* pm2 = split ? nullptr : part_m2;
  const bool acc = accumulate && !split;
  if (cg.a_split && (mode == kWgrad || !conv_gemm_emu_cfg(plan.cfg) || cg.phase))
    throw std::runtime_error("conv_gemm: a pre-split A needs a split-bf16 forward / "
                             "backward-data plan");
  auto go = [&](auto mode_c, auto cfg_c, float* p1, float* p2, const float* mask) {
    launch_cfg<decltype(mode_c)::value, decltype(cfg_c)::value>(
        a, b, mask, dst, p1, p2, gk, M, N, K, plan.splits, stride, acc, a_bytes, b_bytes,
        stream, PhaseSet{}, cg.a_split);
  };
  using F = std::integral_constant<int, kFwd>;
  using D = std::integral_constant<int, kBwdData>;
  using W = std::integral_constant<int, kWgrad>;
  auto by_cfg = [&](auto mode_c, float* p1, float* p2, const float* mask) {
    with_cfg(run_cfg(plan.cfg), [&](auto cfg_c) { go(mode_c, cfg_c, p1, p2, mask); });
  };
  if (mode == kFwd)
    by_cfg(F{}, pm, pm2, x_mask);
  else if (mode == kBwdData)
    by_cfg(D{}, nullptr, nullptr, x_mask);
  else
    by_cfg(W{}, nullptr, nullptr, nullptr);
  if (!split) return;
  if (mode == kFwd && part_mean != nullptr) {
    // split forward with statistics: reduction and per-image BatchNorm partials in one pass
    launch_split_reduce_stats(ws, plan.splits, stride, out, part_mean, part_m2, g.n, g.co,
                              g.ho * g.wo, g.co_total, g.co_off, stream);
    return;
  }
  // out[dst(i)] = (accumulate ? out : 0) + mask * sum_s ws[s][i]
  int64_t planes, c, hw, c_total = 0, c_off = 0;
  if (mode == kFwd) {
    planes = g.n; c = g.co; hw = static_cast<int64_t>(g.ho) * g.wo;
    c_total = g.co_total; c_off = g.co_off;
  } else if (mode == kBwdData) {
    planes = 1; c = static_cast<int64_t>(M) * N; hw = 1; c_total = c;
  } else {
    planes = 1; c = static_cast<int64_t>(M) * N; hw = 1; c_total = c;
  }
  launch_split_reduce(ws, plan.splits, stride, out, mode == kBwdData && g.relu ? x_mask : nullptr,
                      accumulate, planes, c, hw, c_total, c_off, stream);
}

void launch_conv_gemm_partials(const float* a, const float* b, float* ws, const ConvGemmGeo& cg,
                               const ConvGemmPlan& plan, int64_t a_bytes, int64_t b_bytes,
                               hipStream_t stream) {
  Geo g = make_geo(cg);
  int M, N, K;
  gemm_dims(kFwd, g, M, N, K);
  if (M == 0 || N == 0) return;
  if (plan.splits <= 1 || cg.phase)
    throw std::runtime_error("conv_gemm: partials need a split forward plan");
  if (cg.a_split && !conv_gemm_emu_cfg(plan.cfg))
    throw std::runtime_error("conv_gemm: a pre-split A needs a split-bf16 plan");
  g.co_total = g.co;  // (each split's slice holds this convolution's channels only)
  g.co_off = 0;
  const int64_t stride = static_cast<int64_t>(M) * N;
  with_cfg(run_cfg(plan.cfg), [&](auto cfg_c) {
    launch_cfg<kFwd, decltype(cfg_c)::value>(a, b, nullptr, ws, nullptr, nullptr, g, M, N, K,
                                             plan.splits, stride, false, a_bytes, b_bytes,
                                             stream, PhaseSet{}, cg.a_split);
  });
}

void launch_conv_gemm_wgrad_slab(const float* a, const float* b, float* slab,
                                 const ConvGemmGeo& cg, const ConvGemmPlan& plan, bool accumulate,
                                 int64_t a_bytes, int64_t b_bytes, hipStream_t stream) {
  Geo g = make_geo(cg);
  int M, N, K;
  gemm_dims(kWgrad, g, M, N, K);
  if (M == 0 || N == 0) return;
  const int64_t stride = static_cast<int64_t>(M) * N;
  // every split block read-modify-writes its own slice: no reduction pass
  auto go = [&](auto cfg_c) {
    launch_cfg<kWgrad, decltype(cfg_c)::value>(a, b, nullptr, slab, nullptr, nullptr, g, M, N, K,
                                               plan.splits, stride, accumulate, a_bytes, b_bytes,
                                               stream);
  };
  with_cfg(run_cfg(plan.cfg), go);
}

void launch_conv_gemm_phases(const float* a, const int64_t* a_off, const float* b,
                             const float* x_mask, float* out, const ConvGemmPhase* phases,
                             int count, const ConvGemmPlan& plan, bool accumulate,
                             int64_t a_bytes, int64_t b_bytes, hipStream_t stream) {
  if (count <= 0) return;
  PhaseSet ps{};
  ps.count = count;
  int N = 0, K = 0;
  for (int p = 0; p < count; ++p) {
    const ConvGemmGeo& q = phases[p].geo;
    ps.kh[p] = q.kh;
    ps.kw[p] = q.kw;
    ps.ho[p] = q.ho;
    ps.wo[p] = q.wo;
    ps.dy0[p] = q.dy0;
    ps.dx0[p] = q.dx0;
    ps.oh[p] = q.oh;
    ps.ow[p] = q.ow;
    ps.a_off[p] = a_off[p];
    ps.a_bytes[p] = (p + 1 < count ? a_off[p + 1] : a_bytes / 4) * 4 - a_off[p] * 4;
    ps.fd_taps[p] = make_fastdiv(q.kh * q.kw);
    ps.fd_kw[p] = make_fastdiv(q.kw);
    ps.fd_hwo[p] = make_fastdiv(q.ho * q.wo);
    ps.fd_wo[p] = make_fastdiv(q.wo);
    N = std::max(N, q.n * q.ho * q.wo);
    K = std::max(K, q.co * q.kh * q.kw);
  }
  Geo g = make_geo(phases[0].geo);
  g.scatter = 1;
  const int M = g.ci;
  auto go = [&](auto cfg_c) {
    launch_cfg<kBwdData, decltype(cfg_c)::value>(a, b, x_mask, out, nullptr, nullptr, g, M, N, K,
                                                 1, 0, accumulate, a_bytes, b_bytes, stream, ps);
  };
  with_cfg(run_cfg(plan.cfg), go);
}

void launch_slab_flush(const SlabFlushEntry* entries, int count, hipStream_t stream) {
  for (int first = 0; first < count; first += kSlabFlushMax) {
    SlabTable t{};
    t.count = std::min(kSlabFlushMax, count - first);
    int blocks = 0;
    for (int k = 0; k < t.count; ++k) {
      const SlabFlushEntry& e = entries[first + k];
      t.slab[k] = e.slab;
      t.grad[k] = e.grad;
      t.numel[k] = e.numel;
      t.splits[k] = e.splits;
      t.accumulate[k] = e.accumulate ? 1 : 0;
      blocks += static_cast<int>((e.numel + 1023) / 1024);
      t.block_end[k] = blocks;
    }
    if (blocks > 0)
      hipLaunchKernelGGL(slab_flush_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                         stream, t);
  }
}

}  // namespace tgpipe
