// Host-side launchers of the framework's HIP kernels (gfx950 / CDNA4).
// Pure HIP (no ATen) so that kernels.hip compiles in seconds; the ATen
// bindings in bindings.cpp validate shapes/dtypes before calling these.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace tgpipe {

// RNG ops take an optional device-resident Philox state ``rng`` (int64 [2]: seed, base
// offset; nullptr = use ``seed`` / ``offset``): with it the seed is rng[0] and the offset
// rng[1] + offset, read by the kernel when it runs (graph replays, parallel/segments.py).
//
// Fused Dropout2d(p) -> InstanceNorm2d(eps, affine=False) -> LeakyReLU(slope) over
// planes x[P, S] (P = N*C, S = H*W).  Saves per-plane mean (of x), rstd (of the
// dropped-out input) and the dropout scale (0 or 1/(1-p)).
void launch_dna_forward(const float* x, float* y, float* mean, float* rstd, float* scale,
                        int64_t planes, int64_t s, float p, float eps, float slope,
                        uint64_t seed, uint64_t offset, bool dropout, const int64_t* rng,
                        hipStream_t stream);

void launch_dna_backward(const float* dy, const float* x, const float* mean, const float* rstd,
                         const float* scale, float* dx, int64_t planes, int64_t s, float slope,
                         hipStream_t stream);

// Elementwise inverted dropout with explicit Philox (seed, offset); the mask is
// regenerated in backward instead of stored.
void launch_dropout(const float* x, float* y, int64_t n, float p, uint64_t seed, uint64_t offset,
                    const int64_t* rng, hipStream_t stream);

// Uniform [0,1) Philox draws (tests / reference checks).
void launch_philox_uniform(float* out, int64_t n, uint64_t seed, uint64_t offset,
                           const int64_t* rng, hipStream_t stream);

// Spin for `ns` nanoseconds of wall time (s_memrealtime, 100 MHz) — race tests.
void launch_spin(uint64_t ns, hipStream_t stream);

// Multi-tensor pack/unpack: copy `count` byte segments between separate buffers
// and one contiguous buffer in a single launch (inter-stage message packing).
struct Segment {
  const void* src;
  void* dst;
  int64_t bytes;
};
constexpr int kMaxSegments = 16;
void launch_segments_copy(const Segment* segs, int count, hipStream_t stream);

// Winograd F(2x2,3x3) convolution (3x3, stride 1, pad 1, fp32 NCHW) on f32 MFMA.
// Transformed weights: U[Rp][Op][16], Rp = wino_pad_reduction(R), Op = wino_pad_output(O).
// flip = false: w is [O][R][3][3] (forward).  flip = true: w is [R][O][3][3] and the
// kernel is rotated 180 degrees (backward-data: O = input channels, R = output channels).
int64_t wino_pad_reduction(int64_t r);
int64_t wino_pad_output(int64_t o);
void launch_wino_weight(const float* w, float* u, int64_t out_channels, int64_t red_channels,
                        bool flip, hipStream_t stream);
// Launch plan: block-tile variant (0: 64 channels x 32 tiles, 1: 32 x 64, 2: 64 x 64
// double-buffered, one workgroup per CU) and the
// number of reduction splits (> 1 needs a workspace of `workspace` floats).
struct WinoPlan {
  int variant = 0;
  int splits = 1;
  int64_t workspace = 0;
};
WinoPlan wino_plan(int64_t n, int64_t red_channels, int64_t h, int64_t w, int64_t out_channels,
                   int variant, int splits);
// y[N][O][H][W] = conv3x3(x[N][R][H][W]) (+ bias[O] if non-null).
void launch_wino_conv(const float* x, const float* u, const float* bias, float* y, float* ws,
                      int64_t n, int64_t red_channels, int64_t h, int64_t w, int64_t out_channels,
                      const WinoPlan& plan, hipStream_t stream);

// Winograd F(4x4,3x3) (winograd_f4.hip): same convolution, 36 MFMA multiplies per 16
// output pixels.  Transformed weights U4[Rp4/4][Op4/16][4][16][36] (Rp4 = multiple of 4,
// Op4 = multiple of 64).  Variant 4: 64 output channels x 32 tiles per 8-wave workgroup
// (one per CU); variant 5: 32 x 32 per 4-wave workgroup (two per CU); 6 / 7: the same with
// the weight slab by LDS-DMA; 14 / 15: non-fused (input-transform pass, then a GEMM with
// both operands by LDS-DMA; the plan's workspace then includes V); 8-10: timing
// ablations; 12: 6 with 16-byte patch rows; -1: auto (5).
// wino4_supported(): input < 1 GiB etc.
int64_t wino4_pad_reduction(int64_t r);
int64_t wino4_pad_output(int64_t o);
bool wino4_supported(int64_t n, int64_t r, int64_t h, int64_t w, int64_t o);
void launch_wino4_weight(const float* w, float* u, int64_t out_channels, int64_t red_channels,
                         bool flip, hipStream_t stream);
WinoPlan wino4_plan(int64_t n, int64_t red_channels, int64_t h, int64_t w, int64_t out_channels,
                    int variant, int splits);
void launch_wino4_conv(const float* x, const float* u, const float* bias, float* y, float* ws,
                       int64_t n, int64_t red_channels, int64_t h, int64_t w, int64_t out_channels,
                       const WinoPlan& plan, hipStream_t stream);

// Batched-GEMM Winograd F(4x4, 3x3) / F(2x2, 3x3) (winograd_f4.hip): input-transform pass, 36 / 16 independent
// MFMA GEMMs with 128 x bn output tiles, output-transform pass (also sums split-K slabs).
struct BgPlan {
  int kind = 4;           // 4: F(4x4) (36 positions), 2: F(2x2) (16 positions)
  int waves = 8;          // GEMM tile height 32 * waves: 4 (128 rows) or 8 (256 rows)
  int bn = 64;            // GEMM tile width (tiles): 48-128 (4 waves), 64-144 (8 waves)
  int sub = 1;            // 16-deep reduction steps per pipeline stage (1 or 2)
  int splits = 1;         // split-K slabs
  bool emu = false;       // split-bf16 operands on the bf16 matrix pipes (bn 64 / 96 / 128)
  int64_t mp = 0, np = 0, ksteps = 0;
  int64_t workspace = 0;  // floats: V + split slabs of M
};
// Whether `emu` (-1: the process default, TGPIPE_BG_EMU, on unless =0) asks for the
// split-bf16 batched GEMM.
bool bg_emu(int emu);
int bg_pick_bn(int64_t tiles, int kind, bool emu = false);
BgPlan bg_plan(int64_t n, int64_t red_channels, int64_t h, int64_t w, int64_t out_channels,
               int bn, int splits, int kind, int waves, int sub, int emu = -1);
// weights in the GEMM's operand layout U[36 or 16][2 ceil(R/32)][round(O, 256)][16] (f32),
// or the split-bf16 image of the same values (1.5x the bytes)
int64_t bg_weight_numel(int64_t out_channels, int64_t red_channels, int kind, int emu = -1);
void launch_bg_weight(const float* w, float* a, int64_t out_channels, int64_t red_channels,
                      bool flip, int kind, hipStream_t stream, int emu = -1);
// pm / pm2 (optional, [groups][out_channels] each, groups = ceil(n / ipg)): the output pass
// also leaves the BatchNorm (mean, M2) partials of y per (image group, channel), count
// ipg * h * w (bn_stats_kernel's role); ipg from bg_stats_ipg.
int bg_stats_ipg(int64_t n, int64_t h, int64_t w, int kind);
void launch_bg_conv(const float* x, const float* a, const float* bias, float* y, float* ws,
                    int64_t n, int64_t red_channels, int64_t h, int64_t w, int64_t out_channels,
                    const BgPlan& plan, hipStream_t stream, float* pm = nullptr,
                    float* pm2 = nullptr, int ipg = 0);


// F(4x4,3x3) weight gradient (winograd_f4.hip): dw[K][C][3][3], 36 MFMA multiplies per
// 16 output pixels of each (k, c) pair; 64 k x 32 c per 8-wave workgroup, tiles split
// over `splits` workgroups (> 1 needs a workspace of splits*K*C*9 floats).
bool wino4_wgrad_supported(int64_t n, int64_t c, int64_t k, int64_t h, int64_t w);
int wino4_wgrad_splits(int64_t n, int64_t c, int64_t k, int64_t h, int64_t w);
// variant 2: the split-bf16 batched-GEMM weight gradient (its own split count / workspace)
int wino4_wgrad_emu_splits(int64_t n, int64_t c, int64_t k, int64_t h, int64_t w);
int64_t wino4_wgrad_emu_workspace(int64_t n, int64_t c, int64_t k, int64_t h, int64_t w,
                                  int splits);
void launch_wino4_wgrad_emu(const float* x, const float* dy, float* dw, float* ws, int64_t n,
                            int64_t c, int64_t k, int64_t h, int64_t w, int splits, bool accum,
                            hipStream_t stream);
// variant 0: fused (patch / gradient-tile staging inside the GEMM kernel); 1: non-fused
// (transform passes into the GEMM's LDS image order, then an LDS-DMA GEMM).  The workspace
// holds the split-K partials (splits > 1) and, for variant 1, the transformed operands.
int64_t wino4_wgrad_workspace(int64_t n, int64_t c, int64_t k, int64_t h, int64_t w, int splits,
                              int variant);
// accum: add into dw (an existing gradient) instead of overwriting it.
void launch_wino4_wgrad(const float* x, const float* dy, float* dw, float* ws, int64_t n,
                        int64_t c, int64_t k, int64_t h, int64_t w, int splits, int variant,
                        bool accum, hipStream_t stream);

// Weight gradient of the same convolution: dw[K][C][3][3] from x[N][C][H][W] and
// dy[N][K][H][W]; `splits` > 1 needs a workspace of splits*K*C*9 floats.
// variant 0: 64 x 32 (c x k) blocks, two workgroups per CU; variant 2: 64 x 64 blocks,
// one 8-wave workgroup per CU, double-buffered LDS (the forward variant 2 structure).
int wino_wgrad_splits(int64_t n, int64_t c, int64_t k, int64_t h, int64_t w, int variant);
void launch_wino_wgrad(const float* x, const float* dy, float* dw, float* ws, int64_t n,
                       int64_t c, int64_t k, int64_t h, int64_t w, int splits, int variant,
                       bool accum, hipStream_t stream);

// ---- AmoebaNet cell operations (conv_gemm.hip, batchnorm.hip) -----------------------------

// Implicit-GEMM convolution, NCHW fp32: 1x1 with any stride / offset, any kh x kw at
// stride 1 (AmoebaNet's 1x1 / 1x7 / 7x1, U-Net's 3-channel input and 1x1 output convs).
struct ConvGemmGeo {
  int n, ci, h, w;       // input
  int co, ho, wo;        // output of this convolution
  int co_total, co_off;  // its channel slice inside the (concatenated) output Z
  int kh, kw, sh, sw, ph, pw;
  int oh, ow;            // extra input offset (FactorizedReduce's shifted branch)
  bool relu;             // ReLU on the input (its mask in backward-data)
  bool a_t = false;      // backward-data: `a` is W transposed, [ci][co*kh*kw] row-major
  // backward-data of one stride phase of a strided k x k convolution (conv_gemm_phases):
  // ho x wo = the phase's pixel grid (input pixels (sh*y + oh, sw*x + ow)), kh x kw its
  // taps, zh x zw the dZ plane, tap (i, j) reading dZ[y + dy0 - i][x + dx0 - j]
  bool phase = false;
  int zh = 0, zw = 0, dy0 = 0, dx0 = 0;
  // strided 1x1 backward-data (stride 2, no padding / offset, even width): also write the
  // zeros of the other three pixels of each 2x2 block, so dX needs no memset first
  bool fill = false;
  // forward / backward-data on a split-bf16 tile config (conv_gemm_emu_cfg): `a` is the A
  // operand pre-split into bf16 planes ([M][ceil(K/8)][hi, mid, lo][8], conv_gemm_presplit),
  // a_bytes its size -- the kernel stages it without splitting
  bool a_split = false;
};
// Sub-pixel decomposition of a strided convolution's backward-data: input pixels of one
// residue (a, b) modulo the stride receive exactly the taps th = th0 + sh*i, tw = tw0 + sw*j,
// so each phase is a dense stride-1 GEMM (no stride holes), its results scattered back.
// Phases without taps (kernel smaller than the stride) are left out: their pixels are 0.
struct ConvGemmPhase {
  ConvGemmGeo geo;  // a = the weight transposed [ci][co][kh][kw] sliced to [:, :, th0::sh, tw0::sw]
  int th0, tw0;
};
bool conv_gemm_phased(const ConvGemmGeo& g);
// Every phase of one backward-data in one launch (up to kConvGemmMaxPhases; grid.z = phase):
// `a` holds the phases' weight slices back to back, phase p's starting a_off[p] floats in;
// one reduction split.
constexpr int kConvGemmMaxPhases = 4;
struct ConvGemmPlan;
void launch_conv_gemm_phases(const float* a, const int64_t* a_off, const float* b,
                             const float* x_mask, float* out, const ConvGemmPhase* phases,
                             int count, const ConvGemmPlan& plan, bool accumulate,
                             int64_t a_bytes, int64_t b_bytes, hipStream_t stream);
// Integer environment setting (conv_gemm.hip): `fallback` when unset or empty.
int env_int(const char* name, int fallback);
std::vector<ConvGemmPhase> conv_gemm_phases(const ConvGemmGeo& g);
// mode 0: forward  Z[:, co_off:co_off+co] = conv(relu(X)); a = W[co][ci*kh*kw], b = X;
//         part_mean / part_m2 (may be null): BatchNorm statistics partials of each output
//         channel, per column block ([col_blocks][co_total]) when the plan does not split
//         the reduction, per image ([n][co_total], like launch_bn_stats) when it does (the
//         split reduction computes them in the same pass).
// mode 1: backward-data  dX (+)= relu'(X) * conv^T(dZ); a = W (untransposed), b = dZ,
//         x_mask = X (relu mask); `accumulate` adds to dX (several convolutions of one X).
//         dX must be zeroed when the plan scatters (stride holes).
// mode 2: weight gradient  dW[co][ci*kh*kw] = dZ * relu(X); a = dZ, b = X.
// splits > 1 needs a workspace of conv_gemm_workspace() floats.
struct ConvGemmPlan {
  int cfg = 1;           // tiles: 0 = 64 x 64 (4 waves), 1 = 128 x 128 (8 waves),
                         // 2 = 128 x 128 (4 waves of 2 x 2 MFMA tiles); 3 / 4 / 5 / 6 = 0 / 1 /
                         // 2 / 0 with 4 / 2 / 2 / 2 BK steps per pipeline stage
  int splits = 1;        // reduction splits (grid.y), > 1: workspace slices + split_reduce
  int col_width = 128;   // forward: columns per statistics block
  int col_blocks = 0;    // forward: statistics blocks
  bool scatter = false;  // backward-data over output / phase pixels, results scattered
};
ConvGemmPlan conv_gemm_plan(int mode, const ConvGemmGeo& g);
// Every launch shape worth timing (tile size x reduction splits) for the autotuner.
std::vector<ConvGemmPlan> conv_gemm_candidates(int mode, const ConvGemmGeo& g);
int64_t conv_gemm_workspace(int mode, const ConvGemmGeo& g, const ConvGemmPlan& plan);
void launch_conv_gemm(int mode, const float* a, const float* b, const float* x_mask, float* out,
                      float* part_mean, float* part_m2, const ConvGemmGeo& g,
                      const ConvGemmPlan& plan, bool accumulate, float* ws, int64_t a_bytes,
                      int64_t b_bytes, hipStream_t stream);
// Weight gradient of a split plan (splits > 1) into a per-parameter slab of `splits` weight-
// sized slices that persists across the micro-batches of a step: split s stores
// (accumulate = false) or adds (true) its partial into slice s, with no reduction pass;
// launch_slab_flush sums the slices into the gradient once per step.
// Whether a plan's tile config runs on the split-bf16 MFMA (and so can take a pre-split A).
bool conv_gemm_emu_cfg(int cfg);
// The A operand of a forward / backward-data GEMM (M x K row-major: W[co][ci*T], or with
// `transposed` A[ci][co*T + t] = W[co][ci][t], T = taps) split into three bf16 planes,
// [M][ceil(K/8)][3][8] (k octets, zero past K): 6 bytes per element, into `out`
// (M * ceil(K/8) * 24 bf16).
void launch_conv_gemm_presplit(const float* w, void* out, int M, int K, int taps,
                               bool transposed, hipStream_t stream);
void launch_conv_gemm_wgrad_slab(const float* a, const float* b, float* slab,
                                 const ConvGemmGeo& g, const ConvGemmPlan& plan, bool accumulate,
                                 int64_t a_bytes, int64_t b_bytes, hipStream_t stream);
// The GEMM of a split forward plan (plan.splits > 1) alone: partial sums of split s into
// ws[s][n][co][ho*wo] (conv_gemm_workspace floats), no reduction, no statistics.
void launch_conv_gemm_partials(const float* a, const float* b, float* ws, const ConvGemmGeo& g,
                               const ConvGemmPlan& plan, int64_t a_bytes, int64_t b_bytes,
                               hipStream_t stream);
constexpr int kSlabFlushMax = 24;  // table entries per flush launch (kernel argument bytes)
struct SlabFlushEntry {
  const float* slab;
  float* grad;
  int64_t numel;
  int splits;
  bool accumulate;
};
// grad (+)= sum_s slab[s] for every entry (ceil(count / kSlabFlushMax) launches).
void launch_slab_flush(const SlabFlushEntry* entries, int count, hipStream_t stream);

// (mean, M2) partials of z[n][c][s] per (image, channel): part_*[n][c] (width s).
void launch_bn_stats(const float* z, float* part_mean, float* part_m2, int64_t n, int64_t c,
                     int64_t s, hipStream_t stream);

// BatchNorm (training) around the convolutions.  Statistics partials of `blocks` column
// blocks of `width` columns (`total` columns per channel) are merged with Chan's formula
// in fp64 into mean / invstd; the running statistics get the EMA with factor `momentum`
// (unbiased variance) when running_mean is non-null, and `tracked` (BatchNorm's
// num_batches_tracked, may be null) is incremented in the same launch.  `acc` (may be
// null): DeferredBatchNorm's fp64 [3][C] (count, mean, M2) accumulators, Chan-merged.
// `zero2c` (may be null): a [2][C] buffer zeroed by the same launch (the backward's sums).
void launch_bn_finalize(const float* part_mean, const float* part_m2, int blocks, int width,
                        int64_t total, int64_t c, float eps, double momentum, float* mean,
                        float* invstd, float* running_mean, float* running_var, int64_t* tracked,
                        double* acc, float* zero2c, hipStream_t stream);
// DeferredBatchNorm commit from the fp64 accumulators; zeroes them.
void launch_dbn_commit64(double* acc, float* running_mean, float* running_var, int64_t c,
                         double momentum, hipStream_t stream);
// y[n][c][p] = (z - mean) * invstd * gamma + beta (+ add[n][c][p]), planes of s pixels.
void launch_bn_apply(const float* z, const float* mean, const float* invstd, const float* gamma,
                     const float* beta, const float* add, float* y, int64_t n, int64_t c,
                     int64_t s, hipStream_t stream);
// Backward: sums[2][C] (zeroed, e.g. by the forward's finalize) += (sum dy,
// sum dy*(z-mean)); then
// dz = gamma*invstd*(dy - sum_dy/M - (z-mean)*invstd^2*sum_dyz/M), dgamma, dbeta.
// BatchNorm finalize (as launch_bn_finalize) fused with the normalising pass (as
// launch_bn_apply): one launch of (channel, image range) workgroups.
// A grouped convolution (one GEMM over the concatenated weights of several convolutions
// reading the same input) feeding one BatchNorm per convolution: part p covers channels
// [c_end[p-1], c_end[p]) of z / mean / invstd and has its own parameters, running
// statistics and output y_p [n][c_p][s] (forward) / gradient dy_p (image stride dy_img[p];
// null = no gradient) and parameter gradients (backward).  count = 0: not grouped.
constexpr int kBnPartsMax = 3;
struct BnParts {
  int count;
  int c_end[kBnPartsMax];
  const float* gamma[kBnPartsMax];
  const float* beta[kBnPartsMax];
  float* rm[kBnPartsMax];
  float* rv[kBnPartsMax];
  int64_t* tracked[kBnPartsMax];
  float* y[kBnPartsMax];
  const float* dy[kBnPartsMax];
  int64_t dy_img[kBnPartsMax];
  float* dgamma[kBnPartsMax];
  float* dbeta[kBnPartsMax];
  int acc_gamma[kBnPartsMax];
  int acc_beta[kBnPartsMax];
};
void launch_bn_finalize_apply(const float* part_mean, const float* part_m2, int blocks,
                              int width, int64_t n, int64_t c, int64_t s, float eps,
                              double momentum, float* mean, float* invstd, float* running_mean,
                              float* running_var, int64_t* tracked, double* acc, float* zero2c,
                              const float* z, const float* gamma, const float* beta,
                              const float* add, float* y, hipStream_t stream, bool relu = false,
                              const BnParts* parts = nullptr);
// A split-K forward's partials (ws[split][n][c][s], launch_conv_gemm_partials) summed into z
// and its BatchNorm finalized and applied in one launch of per-channel workgroups (the
// arguments as launch_bn_finalize_apply's); for planes of s <= 64 pixels and n * s <= 4096
// (split_bn_small_ok; TGPIPE_SPLIT_BN=0: never).
bool split_bn_small_ok(int64_t n, int64_t s);
void launch_split_bn_small(const float* ws, int splits, int64_t stride, float* z, int64_t n,
                           int64_t c, int64_t s, float eps, double momentum, float* mean,
                           float* invstd, float* running_mean, float* running_var,
                           int64_t* tracked, double* acc, float* zero2c, const float* gamma,
                           const float* beta, const float* add, float* y, hipStream_t stream,
                           bool relu = false, const BnParts* parts = nullptr);
// Backward of a grouped BatchNorm (one workgroup per channel, both passes): dz [n][c][s].
bool bn_backward_parts_ok(int64_t n, int64_t c, int64_t s);
void launch_bn_backward_parts(const BnParts& parts, const float* z, const float* mean,
                              const float* invstd, float* dz, int64_t n, int64_t c, int64_t s,
                              hipStream_t stream);
// relu_out: the forward applied a ReLU after the normalisation (launch_bn_finalize_apply's
// `relu`); dy is that ReLU's output gradient and its mask is re-derived from z (needs beta).
// ymask / gout (ResNet's residual join relu(bn(z) + identity), relu_out false): dy is masked
// by ymask > 0 (the join's output, z's layout) inside the kernel and the masked gradient
// written to gout -- only where bn_backward_one_pass(n, c, s, dy_img) holds.
bool bn_backward_one_pass(int64_t n, int64_t c, int64_t s, int64_t dy_img);
void launch_bn_backward(const float* dy, const float* z, const float* mean, const float* invstd,
                        const float* gamma, float* sums, float* dz, float* dgamma, float* dbeta,
                        bool acc_gamma, bool acc_beta, int64_t n, int64_t c, int64_t s,
                        int64_t dy_img, hipStream_t stream,  // dy_img: dy's image stride
                        bool relu_out = false, const float* beta = nullptr,
                        const float* ymask = nullptr, float* gout = nullptr);

// 3x3 average pool, padding 1, count_include_pad = False, stride 1 / 2 (pool.hip):
// y = pool(x) (+ add) over `planes` = N*C planes of h x w; backward gathers dx.
void launch_avgpool3_forward(const float* x, const float* add, float* y, int64_t planes, int h,
                             int w, int stride, hipStream_t stream);
// dy may be a channel slice: plane (img, ch) at dy + img * dy_img + ch * ho * wo (only
// when avgpool3_backward_strided_ok(h, w); otherwise dy must be dense)
bool avgpool3_backward_strided_ok(int h, int w);
void launch_avgpool3_backward(const float* dy, float* dx, int64_t images, int64_t channels,
                              int h, int w, int stride, int64_t dy_img, hipStream_t stream);

// U-Net resolution changes (unet_ops.hip).  up2x_cat: out[n][c1+c2][2h][2w] =
// cat(nearest 2x upsample of x[n][c1][h][w], skip[n][c2][2h][2w]); up2x_backward: dx = 2x2
// block sums of dy's first c channels (image stride dy_img, elements); maxpool 2x2 / stride 2
// without indices (the backward re-finds the argmax from x; dx is pre-zeroed by the caller
// when h or w is odd).
void launch_up2x_cat(const float* x, const float* skip, float* out, int64_t n, int c1, int c2,
                     int h, int w, hipStream_t stream);
void launch_up2x_backward(const float* dy, float* dx, int64_t n, int c, int h, int w,
                          int64_t dy_img, hipStream_t stream);
// y = relu(a + b) over `total` floats (ResNet's residual join; 16-byte aligned tensors).
void launch_add_relu(const float* a, const float* b, float* y, int64_t total,
                     hipStream_t stream);
// add (nullable): y = maxpool(x) + add.  dy: image stride dy_img (channel slices).
void launch_maxpool2x2_forward(const float* x, const float* add, float* y, int64_t planes, int h,
                               int w, hipStream_t stream);
void launch_maxpool2x2_backward(const float* x, const float* dy, float* dx, int64_t planes,
                                int channels, int h, int w, int64_t dy_img, hipStream_t stream);

}  // namespace tgpipe
