// ATen bindings of the fused ReLU -> Conv -> BatchNorm(train) operation of AmoebaNet-D
// cells (conv_gemm.hip, batchnorm.hip).  One call runs the whole forward or backward of
// the operation, so the host issues one op per cell operation instead of ~10 ATen ops.
//
// A "part" is one convolution writing a channel slice of the concatenated output Z
// (FactorizedReduce = two parts reading the same input, the second shifted by one
// pixel); geometry per part: {kh, kw, sh, sw, ph, pw, oh, ow}.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>

#include <atomic>
#include <cstdlib>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <tuple>
#include <vector>

#include "kernels.h"

namespace tgpipe {
namespace {

constexpr int64_t kMaxBytes = 0x7ffffff0;  // buffer-resource offsets (conv_gemm.hip)

hipStream_t cur_stream(const at::Tensor& t) {
  return at::hip::getCurrentHIPStream(t.device().index()).stream();
}

void launch_one(int mode, const float* a, const float* b, const float* mask, float* out,
                float* pm, float* pm2, const ConvGemmGeo& g, const ConvGemmPlan& plan,
                bool accumulate, int64_t a_bytes, int64_t b_bytes, const at::Tensor& like) {
  const int64_t ws_size = conv_gemm_workspace(mode, g, plan);
  at::Tensor ws;
  if (ws_size > 0) ws = at::empty({ws_size}, like.options());
  launch_conv_gemm(mode, a, b, mask, out, pm, pm2, g, plan, accumulate,
                   ws_size > 0 ? ws.data_ptr<float>() : nullptr, a_bytes, b_bytes,
                   cur_stream(like));
}

// Measured launch plans per (mode, device, geometry), like MIOpen's find step: the first
// launch of a shape times every candidate (tile size x reduction splits) on the current
// stream and keeps the fastest.  TGPIPE_CG_TUNE=0 uses the static heuristic instead;
// stream captures never tune; an accumulating launch times its candidates on a scratch
// output (`out_numel` floats) so the real output is untouched.
// Keyed by geometry only: every GPU of a process is the same gfx950 part.  The table can
// be exported / imported as text (conv_gemm_plans_export/import): the package ships the
// plans measured on an MI355X for its benchmark models, so a fresh process skips the find.
using PlanKey = std::tuple<int, int, int, int, int, int, int, int, int, int, int, int, int, int,
                           int>;
std::mutex plan_mutex;
std::map<PlanKey, ConvGemmPlan> plan_cache;
std::atomic<int> forced_cfg{-1};
std::atomic<int> forced_splits{1};

// Test / profiling hook: run every implicit-GEMM launch with tile config `cfg` and (at
// most) `splits` reduction splits; cfg -1 = tuned plans.
void conv_gemm_force_cfg(int64_t cfg, int64_t splits) {
  forced_cfg.store(static_cast<int>(cfg));
  forced_splits.store(static_cast<int>(splits));
}

// The weight a forward / backward-data GEMM's A operand comes from, for a pre-split A:
// `t` row-major [M][K] (transposed = false) or W[co][ci][T] read transposed.
struct ASource {
  const at::Tensor* t = nullptr;
  bool transposed = false;
};
void run_gemm(int mode, const float* a, const float* b, const float* mask, float* out,
              float* pm, float* pm2, const ConvGemmGeo& g, const ConvGemmPlan& plan,
              bool accumulate, int64_t a_bytes, int64_t b_bytes, const at::Tensor& like,
              ASource src = {}, float* partials = nullptr);

ConvGemmPlan tuned_plan_raw(int mode, const float* a, const float* b, const float* mask,
                            float* out, float* pm, float* pm2, const ConvGemmGeo& g,
                            bool accumulate, int64_t a_bytes, int64_t b_bytes,
                            const at::Tensor& like, int64_t out_numel, ASource src) {
  // Timing trials only when asked for (TGPIPE_CG_TUNE=1: benchmarks/tune_plans.py, the
  // offline tuner): a training step never synchronises the host to time candidates, and
  // every rank of a pipeline picks the same plan for the same shape.  A shape missing from
  // the shipped table (torchgpipe_amd/tuned/conv_gemm_mi355x.txt) runs the heuristic.
  static const bool tune = [] {
    const char* v = std::getenv("TGPIPE_CG_TUNE");
    return v != nullptr && std::string(v) == "1";
  }();
  const int forced = forced_cfg.load();
  if (forced >= 0) {  // test hook: that tile config's candidate with the most splits <= N
    ConvGemmPlan pick = conv_gemm_plan(mode, g);
    bool found = false;
    for (const auto& cand : conv_gemm_candidates(mode, g))
      if (cand.cfg == forced && cand.splits <= std::max(1, forced_splits.load()) &&
          (!found || cand.splits > pick.splits)) {
        pick = cand;
        found = true;
      }
    return pick;
  }
  const hipStream_t stream = cur_stream(like);
  const PlanKey key{mode, g.n, g.ci, g.h, g.w, g.co, g.kh, g.kw, g.sh, g.sw, g.ph, g.pw, g.oh,
                    g.ow, g.co_total};
  std::lock_guard<std::mutex> lock(plan_mutex);
  auto hit = plan_cache.find(key);
  if (hit != plan_cache.end()) {
    // (a stride phase's key could name a plain strided geometry too: its plan must
    // scatter and cannot split)
    if (!g.phase) return hit->second;
    ConvGemmPlan p = hit->second;
    p.scatter = true;
    p.splits = 1;
    return p;
  }
  // (the heuristic only on a miss: every launch of a launch-bound stage asks)
  const ConvGemmPlan heuristic = conv_gemm_plan(mode, g);
  if (!tune) return heuristic;
  // A stream capture (hipGraph) records launches, it cannot time them: a shape first met
  // inside a capture runs the heuristic plan (warm-up steps before capturing tune it).
  hipStreamCaptureStatus capture = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &capture) != hipSuccess ||
      capture != hipStreamCaptureStatusNone)
    return heuristic;
  at::Tensor scratch;
  if (accumulate) {
    scratch = at::empty({out_numel}, like.options());
    out = scratch.data_ptr<float>();
    pm = pm2 = nullptr;
  }
  hipEvent_t t0, t1;
  hipEventCreate(&t0);
  hipEventCreate(&t1);
  ConvGemmPlan best = heuristic;
  float best_ms = -1.f;
  for (const auto& cand : conv_gemm_candidates(mode, g)) {
    float ms = 0.f;
    for (int rep = 0; rep < 2; ++rep) {  // first run: warm-up (code object, caches)
      hipEventRecord(t0, stream);
      // (as the launch will run: split-bf16 candidates on the pre-split weights)
      run_gemm(mode, a, b, mask, out, pm, pm2, g, cand, false, a_bytes, b_bytes, like, src);
      hipEventRecord(t1, stream);
      hipEventSynchronize(t1);
      hipEventElapsedTime(&ms, t0, t1);
    }
    if (best_ms < 0.f || ms < best_ms) {
      best_ms = ms;
      best = cand;
    }
  }
  hipEventDestroy(t0);
  hipEventDestroy(t1);
  plan_cache[key] = best;
  return best;
}

// TGPIPE_CG_SPLIT_CAP=N (profiling knob): forward / backward-data plans split the reduction
// at most N ways (same tile config), so a stage whose cells already run several GEMMs
// side by side on their streams can trade the split-reduction passes for a less full
// single-kernel grid.  The plans were timed one kernel at a time.
ConvGemmPlan tuned_plan(int mode, const float* a, const float* b, const float* mask, float* out,
                        float* pm, float* pm2, const ConvGemmGeo& g, bool accumulate,
                        int64_t a_bytes, int64_t b_bytes, const at::Tensor& like,
                        int64_t out_numel, ASource src = {}) {
  static const int cap = env_int("TGPIPE_CG_SPLIT_CAP", 0);
  ConvGemmPlan p = tuned_plan_raw(mode, a, b, mask, out, pm, pm2, g, accumulate, a_bytes,
                                  b_bytes, like, out_numel, src);
  if (cap <= 0 || mode == 2 || p.splits <= cap) return p;
  ConvGemmPlan pick = p;
  bool found = false;
  for (const auto& cand : conv_gemm_candidates(mode, g))
    if (cand.cfg == p.cfg && cand.splits <= cap && (!found || cand.splits > pick.splits)) {
      pick = cand;
      found = true;
    }
  return found ? pick : p;
}

// One line per plan: "mode n ci h w co kh kw sh sw ph pw oh ow co_total cfg splits".
std::string conv_gemm_plans_export() {
  std::lock_guard<std::mutex> lock(plan_mutex);
  std::ostringstream out;
  for (const auto& kv : plan_cache) {
    const auto& k = kv.first;
    out << std::get<0>(k) << ' ' << std::get<1>(k) << ' ' << std::get<2>(k) << ' '
        << std::get<3>(k) << ' ' << std::get<4>(k) << ' ' << std::get<5>(k) << ' '
        << std::get<6>(k) << ' ' << std::get<7>(k) << ' ' << std::get<8>(k) << ' '
        << std::get<9>(k) << ' ' << std::get<10>(k) << ' ' << std::get<11>(k) << ' '
        << std::get<12>(k) << ' ' << std::get<13>(k) << ' ' << std::get<14>(k) << ' '
        << kv.second.cfg << ' ' << kv.second.splits << '\n';
  }
  return out.str();
}

// Adds the plans of `text` that are still valid launch shapes for this build (a plan must
// equal one of conv_gemm_candidates for its geometry); plans already measured win.
// Returns the number of plans taken.
int64_t conv_gemm_plans_import(const std::string& text) {
  std::istringstream in(text);
  std::string line;
  int64_t taken = 0;
  std::lock_guard<std::mutex> lock(plan_mutex);
  while (std::getline(in, line)) {
    std::istringstream ls(line);
    int v[17];
    int got = 0;
    while (got < 17 && (ls >> v[got])) ++got;
    if (got != 17 || v[0] < 0 || v[0] > 2) continue;
    ConvGemmGeo g;
    g.n = v[1];
    g.ci = v[2];
    g.h = v[3];
    g.w = v[4];
    g.co = v[5];
    g.kh = v[6];
    g.kw = v[7];
    g.sh = v[8];
    g.sw = v[9];
    g.ph = v[10];
    g.pw = v[11];
    g.oh = v[12];
    g.ow = v[13];
    g.co_total = v[14];
    if (g.n <= 0 || g.ci <= 0 || g.h <= 0 || g.w <= 0 || g.co <= 0 || g.kh <= 0 || g.kw <= 0 ||
        g.sh <= 0 || g.sw <= 0 || g.ph < 0 || g.pw < 0 || g.co_total < g.co)
      continue;
    g.ho = (g.h + 2 * g.ph - g.kh) / g.sh + 1;
    g.wo = (g.w + 2 * g.pw - g.kw) / g.sw + 1;
    if (g.ho <= 0 || g.wo <= 0) continue;
    const PlanKey key{v[0], g.n, g.ci, g.h, g.w, g.co, g.kh, g.kw, g.sh, g.sw, g.ph, g.pw, g.oh,
                      g.ow, g.co_total};
    if (plan_cache.count(key)) continue;
    for (const auto& cand : conv_gemm_candidates(v[0], g)) {
      if (cand.cfg == v[15] && cand.splits == v[16]) {
        plan_cache[key] = cand;
        ++taken;
        break;
      }
    }
  }
  return taken;
}

// ---- pre-split A operands -------------------------------------------------------------------
// A split-bf16 plan (conv_gemm.hip, tile configs 7-9) splits every A element into three bf16
// planes as it stages them -- the same weights again in every column block of every
// micro-batch, half of the kernel's split arithmetic.  Here the weights of forward /
// backward-data GEMMs are split once per weight version instead ([M][ceil(K/8)][3][8] bf16,
// 1.5x the weight's bytes) and the kernel loads the planes.  Entries are keyed by the
// source tensor's storage, held by weak reference (a dead weight's entry is dropped), and
// re-derived when its version counter moves or a new training step starts (updates through
// `.data` move no version counter): lazily by the next launch (readers on other
// streams wait for that derive's event), or in place for a whole stage by
// conv_gemm_presplit_refresh (PipelineStage's step start, ops/conv.py
// refresh_step_caches) -- which is what keeps a captured hipGraph, that baked the buffer in,
// reading the current weights.  Inside a capture a stale or missing entry leaves that launch
// on the in-kernel split (the cache is not written, and a derive per replay would cost a
// graph node per launch).  TGPIPE_CG_PRESPLIT_MB: the bytes all entries may hold (default
// 2048; 0 = off); a pipeline stage's first, measuring step and the memory-lean cache mode
// set it to 0 (ops/conv.py hold_cache / size_cache_budget).
struct PreDims {
  int M = 0, K = 0, taps = 1;
  bool transposed = false;
  bool operator==(const PreDims& o) const {
    return M == o.M && K == o.K && taps == o.taps && transposed == o.transposed;
  }
};
using WeakImpl = c10::weak_intrusive_ptr<c10::TensorImpl, c10::UndefinedTensorImpl>;
struct PreSplit {
  PreSplit(WeakImpl s, PreDims dims) : src(std::move(s)), d(dims) {}
  WeakImpl src;
  PreDims d;
  int64_t version = -1;
  int64_t step = -1;  // the training step it was derived in (conv_gemm_presplit_step)
  at::Tensor split;
  hipEvent_t ready = nullptr;
  hipStream_t stream = nullptr;  // derived lazily on this stream (null: ordered by the caller)
};
using PreKey = std::tuple<const void*, bool, int>;
std::mutex pre_mutex;
std::map<PreKey, PreSplit> pre_cache;
int64_t pre_bytes = 0;
std::atomic<int64_t> pre_budget{-1};
// The current training step (ops/conv.py new_step).  An update through `param.data`
// (copy_, EMA swaps) moves no version counter, so an entry is fresh only for the version
// AND the step it was derived in: the first launch (or the step-start refresh) of every
// step re-derives it, like the Winograd transform caches keyed on ops/conv.py _STEP.
std::atomic<int64_t> pre_step{0};

int64_t presplit_budget() {
  int64_t b = pre_budget.load();
  if (b < 0) {
    b = static_cast<int64_t>(std::max(0, env_int("TGPIPE_CG_PRESPLIT_MB", 2048))) << 20;
    pre_budget.store(b);
  }
  return b;
}

int64_t presplit_numel(int M, int K) { return static_cast<int64_t>(M) * ((K + 7) / 8) * 24; }

void presplit_derive(const at::Tensor& src, at::Tensor& out, const PreDims& d,
                     hipStream_t stream) {
  launch_conv_gemm_presplit(src.data_ptr<float>(), out.data_ptr(), d.M, d.K, d.taps,
                            d.transposed, stream);
}

void presplit_erase(std::map<PreKey, PreSplit>::iterator it) {
  pre_bytes -= it->second.split.numel() * 2;
  if (it->second.ready != nullptr) hipEventDestroy(it->second.ready);
  pre_cache.erase(it);
}

// The pre-split A of `src` (row-major [M][K], or with `transposed` W[co][ci][T] read as
// A[ci][co*T + t]) for a launch on the current stream, or undefined (no budget).
at::Tensor presplit_of(const at::Tensor& src, bool transposed, int M, int K, int taps,
                       const at::Tensor& like) {
  const int64_t budget = presplit_budget();
  const int64_t numel = presplit_numel(M, K);
  if (budget <= 0 || numel * 2 > kMaxBytes || !src.is_contiguous() ||
      src.scalar_type() != at::kFloat || src.numel() != static_cast<int64_t>(M) * K)
    return {};
  const hipStream_t stream = cur_stream(like);
  hipStreamCaptureStatus capture = hipStreamCaptureStatusNone;
  const bool capturing = hipStreamIsCapturing(stream, &capture) == hipSuccess &&
                         capture != hipStreamCaptureStatusNone;
  const int64_t version = static_cast<int64_t>(src._version());
  const PreKey key{src.data_ptr(), transposed, src.device().index()};
  const PreDims probe{M, K, taps, transposed};
  std::lock_guard<std::mutex> lock(pre_mutex);
  auto it = pre_cache.find(key);
  if (it != pre_cache.end()) {
    PreSplit& e = it->second;
    auto alive = e.src.lock();
    const bool same = alive.get() == src.unsafeGetTensorImpl() && e.d == probe;
    const int64_t step = pre_step.load();
    if (same && e.version == version && e.step == step) {
      if (e.stream != nullptr && e.stream != stream && !capturing)
        hipStreamWaitEvent(stream, e.ready, 0);
      return e.split;
    }
    if (capturing) return {};  // (see above)
    if (same) {  // stale: in place, on this stream
      presplit_derive(src, e.split, e.d, stream);
      e.version = version;
      e.step = step;
      hipEventRecord(e.ready, stream);
      e.stream = stream;
      return e.split;
    }
    presplit_erase(it);  // another tensor at the same address (or a reshaped use)
  }
  if (capturing) return {};
  // drop the entries of dead tensors before charging the budget
  for (auto j = pre_cache.begin(); j != pre_cache.end();) {
    auto nxt = std::next(j);
    if (j->second.src.expired()) presplit_erase(j);
    j = nxt;
  }
  if (pre_bytes + numel * 2 > budget) return {};
  PreSplit e(WeakImpl(src.getIntrusivePtr()), probe);
  e.version = version;
  e.step = pre_step.load();
  e.split = at::empty({numel}, like.options().dtype(at::kBFloat16));
  presplit_derive(src, e.split, e.d, stream);
  hipEventCreateWithFlags(&e.ready, hipEventDisableTiming);
  hipEventRecord(e.ready, stream);
  e.stream = stream;
  pre_bytes += numel * 2;
  at::Tensor out = e.split;
  pre_cache.emplace(key, std::move(e));
  return out;
}

// The step-start refresh of one stage (ops/conv.py refresh_step_caches): the entries derived
// from `sources` (the stage's parameters and its transposed / concatenated weights) are
// re-derived in place on the device's current stream when stale -- and every one of them
// when that stream is capturing: a whole-step graph (parallel/graph.py) captures this
// refresh and the optimizer, and its replays must re-derive even the entries that were
// fresh at the capture.  Other stages' entries are left alone; dead ones are dropped.
// Returns the entries refreshed or checked.
int64_t conv_gemm_presplit_refresh(at::TensorList sources) {
  std::lock_guard<std::mutex> lock(pre_mutex);
  for (auto it = pre_cache.begin(); it != pre_cache.end();) {
    auto nxt = std::next(it);
    if (it->second.src.expired()) presplit_erase(it);
    it = nxt;
  }
  int64_t count = 0;
  for (const at::Tensor& t : sources) {
    if (!t.defined() || !t.is_cuda()) continue;
    for (const bool transposed : {false, true}) {
      auto it = pre_cache.find(PreKey{t.data_ptr(), transposed, t.device().index()});
      if (it == pre_cache.end()) continue;
      PreSplit& e = it->second;
      auto alive = e.src.lock();
      if (!alive) {
        presplit_erase(it);
        continue;
      }
      const at::Tensor src(alive);
      c10::hip::HIPGuardMasqueradingAsCUDA guard(src.device());
      const hipStream_t stream = cur_stream(src);
      hipStreamCaptureStatus capture = hipStreamCaptureStatusNone;
      const bool capturing = hipStreamIsCapturing(stream, &capture) == hipSuccess &&
                             capture != hipStreamCaptureStatusNone;
      const int64_t version = static_cast<int64_t>(src._version());
      const int64_t step = pre_step.load();
      if (capturing || version != e.version || step != e.step) {
        presplit_derive(src, e.split, e.d, stream);
        e.version = version;
        e.step = step;
      }
      e.stream = nullptr;  // ordered before the step by the caller
      ++count;
    }
  }
  return count;
}

// A new training step: every entry is re-derived before its next use.
void conv_gemm_presplit_step(int64_t step) { pre_step.store(step); }

// Set the pre-split budget (MiB; 0 = off, < 0 = the environment's) and, with `clear`, drop
// every entry (test / benchmark hook).  Returns the bytes the entries held.
int64_t conv_gemm_presplit(int64_t budget_mb, bool clear) {
  std::lock_guard<std::mutex> lock(pre_mutex);
  const int64_t held = pre_bytes;
  if (clear)
    while (!pre_cache.empty()) presplit_erase(pre_cache.begin());
  pre_budget.store(budget_mb < 0 ? -1 : budget_mb << 20);
  return held;
}

// One implicit-GEMM launch with its split-reduction workspace (a pre-split A when the plan
// is a split-bf16 one and `src` names the A operand's weight).  `partials` (split forward
// plans): the GEMM alone, its split partials left in that workspace
// (launch_conv_gemm_partials) for the caller's own reduction.
void run_gemm(int mode, const float* a, const float* b, const float* mask, float* out,
              float* pm, float* pm2, const ConvGemmGeo& g, const ConvGemmPlan& plan,
              bool accumulate, int64_t a_bytes, int64_t b_bytes, const at::Tensor& like,
              ASource src, float* partials) {
  ConvGemmGeo gs = g;
  at::Tensor split;
  if (src.t != nullptr && mode != 2 && conv_gemm_emu_cfg(plan.cfg) && !g.phase) {
    const int taps = g.kh * g.kw;
    const int M = mode == 0 ? g.co : g.ci;
    const int K = (mode == 0 ? g.ci : g.co) * taps;
    split = presplit_of(*src.t, src.transposed, M, K, taps, like);
    if (split.defined()) {
      gs.a_split = true;
      a = static_cast<const float*>(split.data_ptr());
      a_bytes = split.numel() * 2;
    }
  }
  if (partials != nullptr) {
    TORCH_CHECK(mode == 0, "split partials: forward only");
    launch_conv_gemm_partials(a, b, partials, gs, plan, a_bytes, b_bytes, cur_stream(like));
    return;
  }
  launch_one(mode, a, b, mask, out, pm, pm2, gs, plan, accumulate, a_bytes, b_bytes, like);
}

// Whether a backward-data into `dx` leaves pixels unwritten (stride holes of a strided 1x1,
// or stride phases no tap reaches): such a dx starts zeroed.
bool dx_needs_zero(const ConvGemmGeo& g) {
  if (conv_gemm_phased(g))
    return conv_gemm_phases(g).size() <
           static_cast<size_t>(std::min(g.sh, g.h) * std::min(g.sw, g.w));
  return conv_gemm_plan(1, g).scatter;
}

// A strided 1x1 backward-data that writes its stride holes' zeros itself (ConvGemmGeo::fill:
// stride 2, no padding / offset, even width), so its dX is allocated without a memset and
// written in whole 2x2 blocks.  TGPIPE_CG_FILL=0: the memset + scattered stores instead.
bool dx_fillable(const ConvGemmGeo& g) {
  static const bool on = env_int("TGPIPE_CG_FILL", 1) != 0;
  return on && !g.phase && g.kh == 1 && g.kw == 1 && g.sh == 2 && g.sw == 2 && g.ph == 0 &&
         g.pw == 0 && g.oh == 0 && g.ow == 0 && g.w % 2 == 0 && g.ho == (g.h + 1) / 2 &&
         g.wo == g.w / 2;
}

// Backward-data of one convolution into `dx` (accumulating onto it when asked) with the
// transposed weight `wt` ([ci][co][kh][kw]) as the A operand.  A strided k x k convolution
// runs as one GEMM per stride phase (conv_gemm_phases: the sub-pixel decomposition, no
// stride holes walked) on that phase's slice of the weight's taps.
void backward_data_into(const at::Tensor& wt, const at::Tensor& dz, const at::Tensor& x,
                        at::Tensor& dx, ConvGemmGeo g, bool accumulate) {
  g.a_t = true;
  if (conv_gemm_phased(g)) {
    const std::vector<ConvGemmPhase> phases = conv_gemm_phases(g);
    static const bool batched = env_int("TGPIPE_CG_PHASE_BATCH", 1) != 0;
    if (batched && phases.size() > 1 && phases.size() <= kConvGemmMaxPhases) {
      // one launch for all phases (each is a small grid alone: 124 workgroups per phase on
      // AmoebaNet's 14^2 reduction-cell shape), their weight slices back to back
      std::vector<at::Tensor> slices;
      std::vector<int64_t> offs;
      int64_t off = 0;
      size_t big = 0;
      for (size_t p = 0; p < phases.size(); ++p) {
        slices.push_back(wt.slice(2, phases[p].th0, c10::nullopt, g.sh)
                             .slice(3, phases[p].tw0, c10::nullopt, g.sw)
                             .reshape({-1}));
        offs.push_back(off);
        off += slices.back().numel();
        if (phases[p].geo.kh * phases[p].geo.kw > phases[big].geo.kh * phases[big].geo.kw) big = p;
      }
      const at::Tensor wp = at::cat(slices);
      // the tile config of the phase with the longest reduction (no split: phases scatter)
      const ConvGemmPlan plan =
          tuned_plan(1, wp.data_ptr<float>() + offs[big], dz.data_ptr<float>(),
                     x.data_ptr<float>(), dx.data_ptr<float>(), nullptr, nullptr,
                     phases[big].geo, accumulate, slices[big].numel() * 4, dz.numel() * 4, x,
                     x.numel());
      launch_conv_gemm_phases(wp.data_ptr<float>(), offs.data(), dz.data_ptr<float>(),
                              x.data_ptr<float>(), dx.data_ptr<float>(), phases.data(),
                              static_cast<int>(phases.size()), plan, accumulate,
                              wp.numel() * 4, dz.numel() * 4, cur_stream(x));
      return;
    }
    for (const auto& ph : phases) {
      const at::Tensor wp = wt.slice(2, ph.th0, c10::nullopt, g.sh)
                                .slice(3, ph.tw0, c10::nullopt, g.sw)
                                .contiguous();
      const ConvGemmPlan plan =
          tuned_plan(1, wp.data_ptr<float>(), dz.data_ptr<float>(), x.data_ptr<float>(),
                     dx.data_ptr<float>(), nullptr, nullptr, ph.geo, accumulate,
                     wp.numel() * 4, dz.numel() * 4, x, x.numel());
      run_gemm(1, wp.data_ptr<float>(), dz.data_ptr<float>(), x.data_ptr<float>(),
               dx.data_ptr<float>(), nullptr, nullptr, ph.geo, plan, accumulate,
               wp.numel() * 4, dz.numel() * 4, x);
    }
    return;
  }
  const ConvGemmPlan plan =
      tuned_plan(1, wt.data_ptr<float>(), dz.data_ptr<float>(), x.data_ptr<float>(),
                 dx.data_ptr<float>(), nullptr, nullptr, g, accumulate, wt.numel() * 4,
                 dz.numel() * 4, x, x.numel(), ASource{&wt, false});
  run_gemm(1, wt.data_ptr<float>(), dz.data_ptr<float>(), x.data_ptr<float>(),
           dx.data_ptr<float>(), nullptr, nullptr, g, plan, accumulate, wt.numel() * 4,
           dz.numel() * 4, x, ASource{&wt, false});
}

// A channel slice of a dense NCHW tensor (e.g. the gradient of one input of a
// concatenation): dense within each image, any image stride.  Returns that stride, or 0.
int64_t image_stride_if_channel_slice(const at::Tensor& t) {
  if (t.dim() != 4 || t.scalar_type() != at::kFloat || !t.is_cuda()) return 0;
  const int64_t c = t.size(1), h = t.size(2), w = t.size(3);
  if (t.stride(3) != 1 || t.stride(2) != w || t.stride(1) != h * w) return 0;
  if (t.size(0) > 1 && t.stride(0) < c * h * w) return 0;
  if ((reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) != 0) return 0;  // float4 loads
  if ((t.stride(0) & 3) != 0) return 0;
  return t.size(0) > 1 ? t.stride(0) : c * h * w;
}

void check_f32(const at::Tensor& t, const char* name, const at::Tensor& like) {
  TORCH_CHECK(t.is_cuda() && t.device() == like.device(), name, " must be on ", like.device());
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(t.numel() * 4 <= kMaxBytes, name, " is too large (< 2 GiB per tensor)");
}

const float* opt_ptr(const c10::optional<at::Tensor>& t, const char* name, const at::Tensor& like,
                     int64_t numel) {
  if (!t.has_value() || !t->defined()) return nullptr;
  check_f32(*t, name, like);
  TORCH_CHECK(t->numel() == numel, name, " must have ", numel, " elements");
  return t->data_ptr<float>();
}

struct Parts {
  std::vector<ConvGemmGeo> geo;
  int64_t co_total = 0, ho = 0, wo = 0;
};

Parts make_parts(const at::Tensor& x, at::TensorList weights, at::IntArrayRef geo, bool relu) {
  TORCH_CHECK(x.dim() == 4, "x must be NCHW");
  TORCH_CHECK(!weights.empty() && geo.size() == weights.size() * 8,
              "need 8 geometry values {kh, kw, sh, sw, ph, pw, oh, ow} per weight");
  Parts p;
  const int64_t n = x.size(0), ci = x.size(1), h = x.size(2), w = x.size(3);
  for (size_t i = 0; i < weights.size(); ++i) {
    const auto& wt = weights[i];
    check_f32(wt, "weight", x);
    const int64_t* g = geo.data() + 8 * i;
    const int64_t kh = g[0], kw = g[1], sh = g[2], sw = g[3], ph = g[4], pw = g[5];
    TORCH_CHECK(wt.dim() == 4 && wt.size(1) == ci && wt.size(2) == kh && wt.size(3) == kw,
                "weight must be [Co][Ci][kh][kw] matching x and the geometry");
    TORCH_CHECK(sh >= 1 && sw >= 1 && ph >= 0 && pw >= 0 && g[6] >= 0 && g[7] >= 0,
                "bad stride / padding / offset");
    const int64_t ho = (h + 2 * ph - kh) / sh + 1, wo = (w + 2 * pw - kw) / sw + 1;
    TORCH_CHECK(ho > 0 && wo > 0, "empty output");
    if (i == 0) {
      p.ho = ho;
      p.wo = wo;
    }
    TORCH_CHECK(ho == p.ho && wo == p.wo, "all parts must produce the same output plane");
    ConvGemmGeo c;
    c.n = static_cast<int>(n);
    c.ci = static_cast<int>(ci);
    c.h = static_cast<int>(h);
    c.w = static_cast<int>(w);
    c.co = static_cast<int>(wt.size(0));
    c.ho = static_cast<int>(ho);
    c.wo = static_cast<int>(wo);
    c.co_off = static_cast<int>(p.co_total);
    c.kh = static_cast<int>(kh);
    c.kw = static_cast<int>(kw);
    c.sh = static_cast<int>(sh);
    c.sw = static_cast<int>(sw);
    c.ph = static_cast<int>(ph);
    c.pw = static_cast<int>(pw);
    c.oh = static_cast<int>(g[6]);
    c.ow = static_cast<int>(g[7]);
    c.relu = relu;
    p.geo.push_back(c);
    p.co_total += wt.size(0);
  }
  for (auto& c : p.geo) c.co_total = static_cast<int>(p.co_total);
  TORCH_CHECK(n * p.co_total * p.ho * p.wo * 4 <= kMaxBytes, "output too large");
  return p;
}

// One allocation for a BatchNorm's small outputs -- sums [2][C] (the backward's reduction
// buffer), mean [C], invstd [C], each starting on a 16-byte boundary -- followed by `extra`
// scratch floats (the statistics partials): allocations are host time on the launch-bound
// stages (ResNet-101 at 22-image micro-batches runs ~15 k of these ops per step).  The views
// share one storage, so the partials live as long as the saved statistics (a few MB).
struct StatBlock {
  at::Tensor sums, mean, invstd;
  float* extra;
};

StatBlock stat_block(const at::Tensor& like, int64_t c, int64_t extra) {
  const int64_t seg = (c + 3) / 4 * 4;
  auto all = at::empty({4 * seg + extra}, like.options());
  StatBlock b;
  b.sums = all.narrow(0, 0, 2 * c).view({2, c});
  b.mean = all.narrow(0, 2 * seg, c);
  b.invstd = all.narrow(0, 3 * seg, c);
  b.extra = all.data_ptr<float>() + 4 * seg;
  return b;
}

// Forward (training): returns {y, z, mean, invstd} with z the convolution output and
// mean / invstd its batch statistics (saved for the backward).
std::vector<at::Tensor> convbn_forward(const at::Tensor& x_in, at::TensorList weights,
                                       at::IntArrayRef geo, bool relu,
                                       const c10::optional<at::Tensor>& gamma,
                                       const c10::optional<at::Tensor>& beta,
                                       const c10::optional<at::Tensor>& running_mean,
                                       const c10::optional<at::Tensor>& running_var,
                                       const c10::optional<at::Tensor>& num_batches_tracked,
                                       double momentum, double eps,
                                       const c10::optional<at::Tensor>& add, bool relu_out) {
  auto x = x_in.contiguous();
  check_f32(x, "x", x);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Parts p = make_parts(x, weights, geo, relu);
  const int64_t n = x.size(0), c = p.co_total, s = p.ho * p.wo, cols = n * s;
  const auto stream = cur_stream(x);
  auto z = at::empty({n, c, p.ho, p.wo}, x.options());
  std::vector<ConvGemmPlan> plans;
  bool split = false;
  for (size_t i = 0; i < p.geo.size(); ++i) {
    // (tuning candidates write z without statistics; the real launches follow)
    plans.push_back(tuned_plan(0, weights[i].data_ptr<float>(), x.data_ptr<float>(), nullptr,
                               z.data_ptr<float>(), nullptr, nullptr, p.geo[i], false,
                               weights[i].numel() * 4, x.numel() * 4, x, z.numel(),
                               ASource{&weights[i], false}));
    split = split || plans.back().splits > 1;
  }
  // statistics partials: from the GEMM epilogue (all parts share one column tiling), or
  // per (image, channel) when a reduction is split -- from the split reduction itself for a
  // single convolution, from a separate pass for several
  for (const auto& pl : plans)
    split = split || pl.col_width != plans[0].col_width;
  const bool fused_stats = split && p.geo.size() == 1;
  const float* rm = opt_ptr(running_mean, "running_mean", x, c);
  const float* rv = opt_ptr(running_var, "running_var", x, c);
  TORCH_CHECK((rm == nullptr) == (rv == nullptr), "running_mean and running_var go together");
  int64_t* tracked = nullptr;
  if (num_batches_tracked.has_value() && num_batches_tracked->defined()) {
    TORCH_CHECK(num_batches_tracked->device() == x.device() &&
                    num_batches_tracked->scalar_type() == at::kLong &&
                    num_batches_tracked->numel() == 1,
                "num_batches_tracked must be a 1-element int64 tensor on the input's device");
    tracked = num_batches_tracked->data_ptr<int64_t>();
  }
  const float* ga = opt_ptr(gamma, "gamma", x, c);
  const float* be = opt_ptr(beta, "beta", x, c);
  const float* ad = nullptr;
  at::Tensor add_c;
  if (add.has_value() && add->defined()) {
    add_c = add->contiguous();
    check_f32(add_c, "add", x);
    TORCH_CHECK(add_c.sizes() == z.sizes(), "add must have the output's shape");
    ad = add_c.data_ptr<float>();
  }
  // relu_out with a node sum: relu(bn(z) + add) (ResNet's residual join); the caller masks
  // the gradient with the saved output (the backward's re-derived mask cannot see `add`)
  auto y = at::empty_like(z);
  const bool small = fused_stats && split_bn_small_ok(n, s);
  const int width = split ? static_cast<int>(s) : plans[0].col_width;
  const int blocks = split ? static_cast<int>(n) : plans[0].col_blocks;
  // mean / invstd / the backward's sums and the statistics partials: one allocation
  StatBlock st = stat_block(x, c, small ? 0 : 2 * static_cast<int64_t>(blocks) * c);
  auto mean = st.mean, invstd = st.invstd, sums = st.sums;  // (sums: zeroed by the finalize)
  if (small) {
    // small planes: the split partials reduced, normalised and their statistics taken by
    // one per-channel launch (launch_split_bn_small) instead of two
    const ConvGemmPlan& pl = plans[0];
    auto ws = at::empty({conv_gemm_workspace(0, p.geo[0], pl)}, x.options());
    run_gemm(0, weights[0].data_ptr<float>(), x.data_ptr<float>(), nullptr, nullptr, nullptr,
             nullptr, p.geo[0], pl, false, weights[0].numel() * 4, x.numel() * 4, x,
             ASource{&weights[0], false}, ws.data_ptr<float>());
    launch_split_bn_small(ws.data_ptr<float>(), pl.splits, c * cols, z.data_ptr<float>(), n, c,
                          s, static_cast<float>(eps), momentum, mean.data_ptr<float>(),
                          invstd.data_ptr<float>(), const_cast<float*>(rm),
                          const_cast<float*>(rv), tracked, nullptr, sums.data_ptr<float>(), ga,
                          be, ad, y.data_ptr<float>(), stream, relu_out);
    return {y, z, mean, invstd, sums};
  }
  // the two halves by pointer: part[k] would be an aten::select per use (host time of a
  // launch-bound stage, profiles/r5/host_profile.md)
  float* const part0 = st.extra;
  float* const part1 = part0 + static_cast<int64_t>(blocks) * c;
  const bool epilogue_stats = !split || fused_stats;
  for (size_t i = 0; i < p.geo.size(); ++i) {
    const auto wt = weights[i];
    const ConvGemmPlan& pl = plans[i];
    run_gemm(0, wt.data_ptr<float>(), x.data_ptr<float>(), nullptr, z.data_ptr<float>(),
             epilogue_stats ? part0 : nullptr,
             epilogue_stats ? part1 : nullptr, p.geo[i], pl, false,
             wt.numel() * 4, x.numel() * 4, x, ASource{&weights[i], false});
  }
  if (split && !fused_stats)
    launch_bn_stats(z.data_ptr<float>(), part0, part1, n,
                    c, s, stream);
  launch_bn_finalize_apply(part0, part1, blocks, width, n,
                           c, s, static_cast<float>(eps), momentum, mean.data_ptr<float>(),
                           invstd.data_ptr<float>(), const_cast<float*>(rm),
                           const_cast<float*>(rv), tracked, nullptr, sums.data_ptr<float>(),
                           z.data_ptr<float>(), ga, be, ad, y.data_ptr<float>(), stream, relu_out);
  return {y, z, mean, invstd, sums};
}

// Backward: returns {dx (undefined unless need_dx), dgamma, dbeta, dw_0, dw_1, ...}.
// `sums` is the forward's zeroed [2][C] buffer (consumed).  `accum` is empty or holds one
// optional entry per parameter gradient {dgamma, dbeta, dw_0, ...}: a given tensor (the
// parameter's .grad across micro-batches) is accumulated into in place and returned.
// One part's weight gradient: dw (+)= dz x relu(X) taps (accumulating into `into` when given).
//
// `slab` (optional, ops/gradacc.py deferred weight gradients): when the plan splits the
// reduction, the split partials go into this per-parameter buffer of `splits` weight-sized
// slices instead of a workspace + reduction pass -- stored when `slab_first` (the step's
// first use; the slab is resized to fit), added otherwise -- and the slab itself is
// returned; wgrad_slab_flush sums its slices into .grad at the end of the step.  A later
// call whose plan splits differently reduces into the slab's first slice.
at::Tensor wgrad_part(const at::Tensor& dz, const at::Tensor& x, const at::Tensor& weight,
                      const ConvGemmGeo& g, const at::Tensor& into,
                      c10::optional<at::Tensor> slab = c10::nullopt, bool slab_first = false) {
  const bool acc = into.defined();
  auto dw = acc ? into : at::empty_like(weight);
  const ConvGemmPlan plan =
      tuned_plan(2, dz.data_ptr<float>(), x.data_ptr<float>(), nullptr, dw.data_ptr<float>(),
                 nullptr, nullptr, g, acc, dz.numel() * 4, x.numel() * 4, x, dw.numel());
  if (slab.has_value() && slab->defined() && plan.splits > 1) {
    at::Tensor sb = *slab;
    TORCH_CHECK(sb.is_cuda() && sb.device() == x.device() && sb.scalar_type() == at::kFloat &&
                    sb.dim() == 1,
                "slab must be a 1-D float32 tensor on the input's device");
    const int64_t need = static_cast<int64_t>(plan.splits) * weight.numel();
    TORCH_CHECK(need * 4 <= kMaxBytes, "slab too large");
    if (slab_first) {
      if (sb.numel() != need) sb.resize_({need});
    }
    if (slab_first || sb.numel() == need) {
      launch_conv_gemm_wgrad_slab(dz.data_ptr<float>(), x.data_ptr<float>(), sb.data_ptr<float>(),
                                  g, plan, !slab_first, dz.numel() * 4, x.numel() * 4,
                                  cur_stream(x));
    } else {
      TORCH_CHECK(sb.numel() >= weight.numel() && sb.numel() % weight.numel() == 0,
                  "slab does not hold whole weight-sized slices");
      run_gemm(2, dz.data_ptr<float>(), x.data_ptr<float>(), nullptr, sb.data_ptr<float>(),
               nullptr, nullptr, g, plan, true, dz.numel() * 4, x.numel() * 4, x);
    }
    return sb;
  }
  run_gemm(2, dz.data_ptr<float>(), x.data_ptr<float>(), nullptr, dw.data_ptr<float>(), nullptr,
           nullptr, g, plan, acc, dz.numel() * 4, x.numel() * 4, x);
  return dw;
}

c10::optional<at::Tensor> slab_of(const c10::List<c10::optional<at::Tensor>>& slabs, size_t i) {
  if (i >= slabs.size()) return c10::nullopt;
  return slabs.get(i);
}

bool first_of(at::IntArrayRef slab_first, size_t i) {
  return i < slab_first.size() && slab_first[i] != 0;
}

// End of a step with deferred weight gradients: grads[i] (+)= sum of slabs[i]'s slices
// (accumulate[i]: add to the existing gradient), for every parameter in one launch per
// kSlabFlushMax entries.
void wgrad_slab_flush(at::TensorList slabs, at::TensorList grads, at::IntArrayRef accumulate) {
  TORCH_CHECK(slabs.size() == grads.size() && grads.size() == accumulate.size(),
              "slabs, grads and accumulate must have one entry per parameter");
  if (slabs.empty()) return;
  c10::hip::HIPGuardMasqueradingAsCUDA guard(grads[0].device());
  std::vector<SlabFlushEntry> entries;
  for (size_t i = 0; i < slabs.size(); ++i) {
    const auto& g = grads[i];
    const auto& sb = slabs[i];
    check_f32(g, "grad", grads[0]);
    check_f32(sb, "slab", grads[0]);
    TORCH_CHECK(g.numel() > 0 && sb.numel() % g.numel() == 0 && sb.numel() >= g.numel(),
                "slab must hold whole gradient-sized slices");
    entries.push_back({sb.data_ptr<float>(), g.data_ptr<float>(), g.numel(),
                       static_cast<int>(sb.numel() / g.numel()), accumulate[i] != 0});
  }
  launch_slab_flush(entries.data(), static_cast<int>(entries.size()), cur_stream(grads[0]));
}

// Backward-data of a single-part operation on the library convolution (MIOpen, through
// ATen) + the ReLU mask, for the geometries where that measured faster than the implicit
// GEMM: the strided convolutions of reduction cells (the GEMM walks every stride hole:
// 206 vs 43 us for 32 ch 3x3 s2 at 112^2) and some deep 7x7 / 28x28 planes
// (profiles/r3/convbn_bench_n20_spread.json).  Decided per geometry by the shipped table
// (torchgpipe_amd/tuned/lib_dgrad_mi355x.txt, measured by benchmarks/tune_plans.py); with
// TGPIPE_CG_TUNE=1 a geometry missing from it is timed both ways on its first eager call.
// Otherwise (and inside a stream capture, or with TGPIPE_LIB_DGRAD=0) the implicit GEMM.
std::mutex lib_mutex;
std::map<PlanKey, bool> lib_dgrad_cache;
std::atomic<int> forced_lib{-1};

// Test hook: -1 = measured choice, 0 = always the implicit GEMM, 1 = always the library.
void lib_dgrad_force(int64_t mode) { forced_lib.store(static_cast<int>(mode)); }

bool lib_dgrad_eligible(const ConvGemmGeo& g) {
  static const bool on = [] {
    const char* v = std::getenv("TGPIPE_LIB_DGRAD");
    return v == nullptr || std::string(v) != "0";
  }();
  const int forced = forced_lib.load();
  if (forced == 0 || (forced < 0 && (!on || forced_cfg.load() >= 0))) return false;
  if (g.oh != 0 || g.ow != 0 || g.co != g.co_total) return false;
  // small operands stay native without a trial: the library's per-call overhead loses
  // there, and a tiny 1x1 shape's library call faulted on the GPU box (miopenStatus-
  // InternalError after an illegal address, r3ag)
  const int64_t x_numel = static_cast<int64_t>(g.n) * g.ci * g.h * g.w;
  return forced == 1 || (x_numel >= (int64_t{1} << 17) && g.ci >= 32 && g.co >= 32);
}

at::Tensor lib_dgrad(const at::Tensor& dz, const at::Tensor& x, const at::Tensor& w,
                     const ConvGemmGeo& g) {
  const int64_t stride[2] = {g.sh, g.sw}, pad[2] = {g.ph, g.pw}, one[2] = {1, 1},
                zero[2] = {0, 0};
  auto dxr = std::get<0>(at::convolution_backward(dz, x, w, c10::nullopt, stride, pad, one,
                                                  false, zero, 1, {true, false, false}));
  return g.relu ? at::threshold_backward(dxr, x, 0) : dxr;
}

template <typename Ours, typename Lib>
bool lib_dgrad_chosen(const ConvGemmGeo& g, const at::Tensor& like, Ours&& ours, Lib&& lib) {
  const PlanKey key{1, g.n, g.ci, g.h, g.w, g.co, g.kh, g.kw, g.sh, g.sw, g.ph, g.pw, g.oh,
                    g.ow, g.co_total};
  if (forced_lib.load() == 1) return true;
  static const bool tune = [] {
    const char* v = std::getenv("TGPIPE_CG_TUNE");
    return v != nullptr && std::string(v) == "1";
  }();
  std::lock_guard<std::mutex> lock(lib_mutex);
  auto hit = lib_dgrad_cache.find(key);
  if (hit != lib_dgrad_cache.end()) return hit->second;
  if (!tune) return false;
  const hipStream_t stream = cur_stream(like);
  hipStreamCaptureStatus capture = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &capture) != hipSuccess ||
      capture != hipStreamCaptureStatusNone)
    return false;
  hipEvent_t t0, t1;
  hipEventCreate(&t0);
  hipEventCreate(&t1);
  auto time = [&](auto&& fn) {
    float ms = 0.f, best = -1.f;
    for (int rep = 0; rep < 3; ++rep) {  // first run: warm-up (plans, MIOpen's find step)
      hipEventRecord(t0, stream);
      fn();
      hipEventRecord(t1, stream);
      hipEventSynchronize(t1);
      hipEventElapsedTime(&ms, t0, t1);
      if (rep > 0 && (best < 0.f || ms < best)) best = ms;
    }
    return best;
  };
  const float ours_ms = time(ours);
  const float lib_ms = time(lib);
  hipEventDestroy(t0);
  hipEventDestroy(t1);
  const bool pick = lib_ms < 0.95f * ours_ms;  // ties stay on the native kernel
  lib_dgrad_cache[key] = pick;
  return pick;
}

// Seed the backward-data choice with a saved table (lib_dgrad_export's format); entries
// already decided in this process are kept.  Returns the lines taken.
int64_t lib_dgrad_import(const std::string& text) {
  std::istringstream in(text);
  std::string line;
  int64_t taken = 0;
  std::lock_guard<std::mutex> lock(lib_mutex);
  while (std::getline(in, line)) {
    std::istringstream ls(line);
    int v[11];
    int got = 0;
    while (got < 11 && (ls >> v[got])) ++got;
    if (got != 11) continue;
    bool ok = true;
    for (int i = 0; i < 11; ++i) ok = ok && v[i] >= (i >= 9 ? 0 : 1);
    if (!ok) continue;
    const PlanKey key{1, v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8], v[9], v[10], 0,
                      0, v[4]};
    if (lib_dgrad_cache.emplace(key, true).second) ++taken;
  }
  return taken;
}

// Geometries whose backward-data runs on the library convolution: "n ci h w co kh kw sh sw
// ph pw" per line.
std::string lib_dgrad_export() {
  std::lock_guard<std::mutex> lock(lib_mutex);
  std::ostringstream out;
  for (const auto& kv : lib_dgrad_cache) {
    if (!kv.second) continue;
    const auto& k = kv.first;
    out << std::get<1>(k) << ' ' << std::get<2>(k) << ' ' << std::get<3>(k) << ' '
        << std::get<4>(k) << ' ' << std::get<5>(k) << ' ' << std::get<6>(k) << ' '
        << std::get<7>(k) << ' ' << std::get<8>(k) << ' ' << std::get<9>(k) << ' '
        << std::get<10>(k) << ' ' << std::get<11>(k) << '\n';
  }
  return out.str();
}

std::vector<at::Tensor> convbn_backward(const at::Tensor& dy_in, const at::Tensor& x_in,
                                        const at::Tensor& z, const at::Tensor& mean,
                                        const at::Tensor& invstd, at::Tensor& sums,
                                        const c10::optional<at::Tensor>& gamma,
                                        at::TensorList weights, at::IntArrayRef geo, bool relu,
                                        bool need_dx,
                                        const c10::List<c10::optional<at::Tensor>>& accum,
                                        at::TensorList weights_t, bool defer_wgrad,
                                        const c10::List<c10::optional<at::Tensor>>& slabs,
                                        at::IntArrayRef slab_first,
                                        const c10::optional<at::Tensor>& beta, bool relu_out,
                                        const c10::optional<at::Tensor>& dx_into,
                                        const c10::optional<at::Tensor>& y_mask,
                                        const c10::optional<at::Tensor>& dy_masked) {
  auto x = x_in.contiguous();
  // dy is read in place when it is a channel slice (a concatenated cell output's gradient)
  int64_t dy_img = image_stride_if_channel_slice(dy_in);
  auto dy = dy_img > 0 ? dy_in : dy_in.contiguous();
  // y_mask (the residual join relu(bn(z) + add)'s output): dy is the join's output gradient;
  // masked by y > 0 into dy_masked (the add's gradient too) -- inside the BatchNorm backward
  // where its one-pass kernel runs, by threshold_backward before it otherwise
  const bool out_mask = y_mask.has_value() && y_mask->defined();
  const float* ymask_ptr = nullptr;
  float* gout_ptr = nullptr;
  if (out_mask) {
    TORCH_CHECK(!relu_out, "y_mask and relu_out exclude each other");
    TORCH_CHECK(dy_masked.has_value() && dy_masked->defined() && dy_masked->is_contiguous() &&
                    dy_masked->sizes() == z.sizes() && y_mask->is_contiguous() &&
                    y_mask->sizes() == z.sizes(),
                "y_mask needs a contiguous dy_masked output, both of z's shape");
    check_f32(*y_mask, "y_mask", x_in);
    check_f32(*dy_masked, "dy_masked", x_in);
    // (dy read through its image stride; y / dy_masked in z's contiguous layout)
    const int64_t zs = z.size(2) * z.size(3);
    if (bn_backward_one_pass(z.size(0), z.size(1), zs, dy_img > 0 ? dy_img : z.size(1) * zs)) {
      ymask_ptr = y_mask->data_ptr<float>();
      gout_ptr = dy_masked->data_ptr<float>();
    } else {
      at::Tensor masked = *dy_masked;  // (a handle to the caller's buffer)
      at::threshold_backward_out(masked, dy, *y_mask, 0);
      dy = masked;
      dy_img = 0;
    }
  }
  if (dy_img == 0) {
    check_f32(dy, "dy", x);
  } else {
    TORCH_CHECK(dy.device() == x.device(), "dy must be on ", x.device());
  }
  check_f32(x, "x", x);
  check_f32(z, "z", x);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Parts p = make_parts(x, weights, geo, relu);
  const int64_t n = x.size(0), c = p.co_total, s = p.ho * p.wo;
  TORCH_CHECK(dy.sizes() == z.sizes() && z.size(1) == c && z.size(2) == p.ho,
              "dy / z do not match the operation's output");
  check_f32(mean, "mean", x);
  check_f32(invstd, "invstd", x);
  TORCH_CHECK(mean.numel() == c && invstd.numel() == c, "statistics must have C elements");
  const auto stream = cur_stream(x);
  const float* ga = opt_ptr(gamma, "gamma", x, c);
  check_f32(sums, "sums", x);
  TORCH_CHECK(sums.numel() == 2 * c, "sums must be the forward's [2][C] buffer");
  const size_t n_grads = 2 + p.geo.size();
  TORCH_CHECK(accum.empty() || accum.size() == n_grads,
              "accum must be empty or hold {dgamma, dbeta, dw...}");
  std::vector<at::Tensor> into(n_grads);
  for (size_t i = 0; i < accum.size(); ++i) {
    const c10::optional<at::Tensor> t = accum.get(i);
    if (!t.has_value() || !t->defined()) continue;
    check_f32(*t, "accumulated gradient", x);
    TORCH_CHECK(t->numel() == (i < 2 ? c : weights[i - 2].numel()),
                "accumulated gradient has the wrong size");
    into[i] = *t;
  }
  auto dz = at::empty_like(z);
  auto dgamma = into[0].defined() ? into[0] : at::empty({c}, x.options());
  auto dbeta = into[1].defined() ? into[1] : at::empty({c}, x.options());
  launch_bn_backward(dy.data_ptr<float>(), z.data_ptr<float>(), mean.data_ptr<float>(),
                     invstd.data_ptr<float>(), ga, sums.data_ptr<float>(), dz.data_ptr<float>(),
                     dgamma.data_ptr<float>(), dbeta.data_ptr<float>(), into[0].defined(),
                     into[1].defined(), n, c, s, dy_img, stream, relu_out,
                     opt_ptr(beta, "beta", x, c), ymask_ptr, gout_ptr);
  std::vector<at::Tensor> out;
  at::Tensor dx;
  // `dx_into`: a gradient of the same input from another consumer (ResNet's identity path,
  // ops/fusion.py): the backward-data GEMM accumulates onto it instead of autograd adding
  // the two afterwards
  const bool has_into = dx_into.has_value() && dx_into->defined();
  if (has_into) {
    check_f32(*dx_into, "dx_into", x);
    TORCH_CHECK(dx_into->sizes() == x.sizes(), "dx_into must have the input's shape");
  }
  auto ours_into = [&](bool use_into) -> at::Tensor {
    bool zero = false;
    for (const auto& g : p.geo) zero = zero || dx_needs_zero(g);
    // (the first part writing every pixel, holes included: no memset for the others)
    const bool fill = !use_into && dx_fillable(p.geo[0]);
    zero = zero && !fill;
    at::Tensor d = use_into ? *dx_into
                            : (zero ? at::zeros_like(x) : at::empty_like(x));  // stride holes
    zero = zero || use_into;  // (from here: accumulate onto d)
    // the backward-data A operand is W^T: one small transpose per weight, then the
    // GEMM streams K-contiguous rows instead of gathering a column per element
    // (`weights_t`: the caller's per-step cached transposes, ops/conv.py _TransformCache)
    std::vector<at::Tensor> wts;
    TORCH_CHECK(weights_t.empty() || weights_t.size() == p.geo.size(),
                "weights_t must be empty or hold one transposed weight per weight");
    for (size_t i = 0; i < p.geo.size(); ++i) {
      if (weights_t.empty()) {
        wts.push_back(weights[i].transpose(0, 1).contiguous());
      } else {
        check_f32(weights_t[i], "weights_t", x);
        TORCH_CHECK(weights_t[i].dim() == 4 && weights_t[i].size(0) == weights[i].size(1) &&
                        weights_t[i].size(1) == weights[i].size(0) &&
                        weights_t[i].numel() == weights[i].numel(),
                    "weights_t[i] must be weights[i] transposed to [ci][co][kh][kw]");
        wts.push_back(weights_t[i]);
      }
    }
    for (size_t i = 0; i < p.geo.size(); ++i) {
      ConvGemmGeo gi = p.geo[i];
      gi.fill = i == 0 && fill;
      backward_data_into(wts[i], dz, x, d, gi, i > 0 || zero);
    }
    return d;
  };
  if (need_dx) {
    auto ours = [&]() { return ours_into(false); };  // (timing trials never touch dx_into)
    const bool lib = p.geo.size() == 1 && lib_dgrad_eligible(p.geo[0]) &&
                     lib_dgrad_chosen(p.geo[0], x, ours, [&] {
                       return lib_dgrad(dz, x, weights[0], p.geo[0]);
                     });
    if (lib) {
      dx = lib_dgrad(dz, x, weights[0], p.geo[0]);
      if (has_into) dx = dx_into->add_(dx);
    } else {
      dx = ours_into(has_into);
    }
  }
  out.push_back(dx);
  out.push_back(dgamma);
  out.push_back(dbeta);
  if (defer_wgrad) {  // the caller runs convbn_wgrad (e.g. on a weight-gradient stream)
    out.push_back(dz);
    return out;
  }
  for (size_t i = 0; i < p.geo.size(); ++i) {
    const bool acc = into[2 + i].defined();
    out.push_back(wgrad_part(dz, x, weights[i], p.geo[i], acc ? into[2 + i] : at::Tensor(),
                             slab_of(slabs, i), first_of(slab_first, i)));
  }
  return out;
}

// ---- grouped convolutions (AmoebaNet normal cells) ----------------------------------------
// Several ReLU -> 1x1 Conv -> BatchNorm operations reading the same input (a normal cell's
// node 0 feeds three) as ONE implicit-GEMM convolution over their concatenated weights
// (`w_cat` [sum co_p][ci], cached per step by the caller), one statistics + finalize +
// normalise pass writing each operation's own output, and in the backward one BatchNorm
// pass, one backward-data GEMM (`w_cat_t`) and one weight-gradient GEMM per operation.

BnParts make_bn_parts(at::IntArrayRef channels, const c10::List<c10::optional<at::Tensor>>& gammas,
                      const c10::List<c10::optional<at::Tensor>>& betas, const at::Tensor& like,
                      int64_t c_total) {
  TORCH_CHECK(channels.size() >= 1 && static_cast<int>(channels.size()) <= kBnPartsMax,
              "1 to ", kBnPartsMax, " grouped operations");
  TORCH_CHECK(gammas.size() == channels.size() && betas.size() == channels.size(),
              "one gamma / beta per grouped operation");
  BnParts pt{};
  pt.count = static_cast<int>(channels.size());
  int64_t end = 0;
  for (size_t i = 0; i < channels.size(); ++i) {
    end += channels[i];
    pt.c_end[i] = static_cast<int>(end);
    pt.gamma[i] = opt_ptr(gammas.get(i), "gamma", like, channels[i]);
    pt.beta[i] = opt_ptr(betas.get(i), "beta", like, channels[i]);
  }
  TORCH_CHECK(end == c_total, "grouped channel counts must add up to the weight's rows");
  return pt;
}

std::vector<at::Tensor> convbn_group_forward(
    const at::Tensor& x_in, const at::Tensor& w_cat, at::IntArrayRef geo, bool relu,
    at::IntArrayRef channels, const c10::List<c10::optional<at::Tensor>>& gammas,
    const c10::List<c10::optional<at::Tensor>>& betas,
    const c10::List<c10::optional<at::Tensor>>& running_means,
    const c10::List<c10::optional<at::Tensor>>& running_vars,
    const c10::List<c10::optional<at::Tensor>>& tracked, double momentum, double eps) {
  auto x = x_in.contiguous();
  check_f32(x, "x", x);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Parts p = make_parts(x, {w_cat}, geo, relu);
  const int64_t n = x.size(0), c = p.co_total, s = p.ho * p.wo;
  const auto stream = cur_stream(x);
  BnParts pt = make_bn_parts(channels, gammas, betas, x, c);
  TORCH_CHECK(running_means.size() == channels.size() && running_vars.size() == channels.size() &&
                  tracked.size() == channels.size(),
              "one running_mean / running_var / num_batches_tracked per grouped operation");
  std::vector<at::Tensor> out;
  for (size_t i = 0; i < channels.size(); ++i) {
    pt.rm[i] = const_cast<float*>(opt_ptr(running_means.get(i), "running_mean", x, channels[i]));
    pt.rv[i] = const_cast<float*>(opt_ptr(running_vars.get(i), "running_var", x, channels[i]));
    TORCH_CHECK((pt.rm[i] == nullptr) == (pt.rv[i] == nullptr),
                "running_mean and running_var go together");
    const c10::optional<at::Tensor> t = tracked.get(i);
    if (t.has_value() && t->defined()) {
      TORCH_CHECK(t->device() == x.device() && t->scalar_type() == at::kLong && t->numel() == 1,
                  "num_batches_tracked must be a 1-element int64 tensor on the input's device");
      pt.tracked[i] = t->data_ptr<int64_t>();
    }
    out.push_back(at::empty({n, channels[i], p.ho, p.wo}, x.options()));
    pt.y[i] = out.back().data_ptr<float>();
  }
  auto z = at::empty({n, c, p.ho, p.wo}, x.options());
  const ConvGemmPlan plan =
      tuned_plan(0, w_cat.data_ptr<float>(), x.data_ptr<float>(), nullptr, z.data_ptr<float>(),
                 nullptr, nullptr, p.geo[0], false, w_cat.numel() * 4, x.numel() * 4, x,
                 z.numel(), ASource{&w_cat, false});
  const bool split = plan.splits > 1;
  auto mean = at::empty({c}, x.options());
  auto invstd = at::empty({c}, x.options());
  if (split && split_bn_small_ok(n, s)) {  // (as convbn_forward)
    auto ws = at::empty({conv_gemm_workspace(0, p.geo[0], plan)}, x.options());
    run_gemm(0, w_cat.data_ptr<float>(), x.data_ptr<float>(), nullptr, nullptr, nullptr,
             nullptr, p.geo[0], plan, false, w_cat.numel() * 4, x.numel() * 4, x,
             ASource{&w_cat, false}, ws.data_ptr<float>());
    launch_split_bn_small(ws.data_ptr<float>(), plan.splits, c * n * s, z.data_ptr<float>(), n,
                          c, s, static_cast<float>(eps), momentum, mean.data_ptr<float>(),
                          invstd.data_ptr<float>(), nullptr, nullptr, nullptr, nullptr, nullptr,
                          nullptr, nullptr, nullptr, nullptr, stream, false, &pt);
    out.push_back(z);
    out.push_back(mean);
    out.push_back(invstd);
    return out;
  }
  const int width = split ? static_cast<int>(s) : plan.col_width;
  const int blocks = split ? static_cast<int>(n) : plan.col_blocks;
  auto part = at::empty({2, blocks, c}, x.options());
  // the two halves by pointer: part[k] would be an aten::select per use (host time of a
  // launch-bound stage, profiles/r5/host_profile.md)
  float* const part0 = part.data_ptr<float>();
  float* const part1 = part0 + static_cast<int64_t>(blocks) * c;
  run_gemm(0, w_cat.data_ptr<float>(), x.data_ptr<float>(), nullptr, z.data_ptr<float>(),
           part0, part1, p.geo[0], plan, false,
           w_cat.numel() * 4, x.numel() * 4, x, ASource{&w_cat, false});
  launch_bn_finalize_apply(part0, part1, blocks, width, n,
                           c, s, static_cast<float>(eps), momentum, mean.data_ptr<float>(),
                           invstd.data_ptr<float>(), nullptr, nullptr, nullptr, nullptr, nullptr,
                           z.data_ptr<float>(), nullptr, nullptr, nullptr, nullptr, stream, false,
                           &pt);
  out.push_back(z);
  out.push_back(mean);
  out.push_back(invstd);
  return out;
}

bool convbn_group_backward_ok(int64_t n, int64_t c, int64_t hw) {
  return bn_backward_parts_ok(n, c, hw);
}

// Returns {dx (undefined unless need_dx), dgamma_0, dbeta_0, ..., dw_0, ...}; `accum` holds
// per operation {dgamma, dbeta, dw} (.grad to accumulate into, or none), `slabs` /
// `slab_first` one entry per weight (ops/gradacc.py deferred weight gradients).
std::vector<at::Tensor> convbn_group_backward(
    const c10::List<c10::optional<at::Tensor>>& dys, const at::Tensor& x_in, const at::Tensor& z,
    const at::Tensor& mean, const at::Tensor& invstd, at::TensorList weights,
    const at::Tensor& w_cat_t, at::IntArrayRef geo, bool relu, bool need_dx,
    at::IntArrayRef channels, const c10::List<c10::optional<at::Tensor>>& gammas,
    const c10::List<c10::optional<at::Tensor>>& accum,
    const c10::List<c10::optional<at::Tensor>>& slabs, at::IntArrayRef slab_first) {
  auto x = x_in.contiguous();
  check_f32(x, "x", x);
  check_f32(z, "z", x);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int64_t n = x.size(0), c = z.size(1), s = z.size(2) * z.size(3);
  TORCH_CHECK(bn_backward_parts_ok(n, c, s), "grouped backward: channels too large");
  const size_t np = channels.size();
  TORCH_CHECK(weights.size() == np && dys.size() == np, "one weight and dy per operation");
  TORCH_CHECK(accum.size() == 3 * np, "accum must hold {dgamma, dbeta, dw} per operation");
  c10::List<c10::optional<at::Tensor>> no_beta;
  for (size_t i = 0; i < np; ++i) no_beta.push_back(c10::nullopt);
  BnParts pt = make_bn_parts(channels, gammas, no_beta, x, c);
  std::vector<at::Tensor> keep;  // contiguous dys, parameter gradients
  std::vector<at::Tensor> dgb;
  for (size_t i = 0; i < np; ++i) {
    const c10::optional<at::Tensor> d = dys.get(i);
    if (d.has_value() && d->defined()) {
      int64_t img = image_stride_if_channel_slice(*d);
      at::Tensor dd = img > 0 ? *d : d->contiguous();
      if (img == 0) {
        check_f32(dd, "dy", x);
        img = channels[i] * s;
      }
      TORCH_CHECK(dd.dim() == 4 && dd.size(0) == n && dd.size(1) == channels[i] &&
                      dd.size(2) * dd.size(3) == s,
                  "dy of a grouped operation has the wrong shape");
      keep.push_back(dd);
      pt.dy[i] = dd.data_ptr<float>();
      pt.dy_img[i] = img;
    }
    for (int k = 0; k < 2; ++k) {
      const c10::optional<at::Tensor> a = accum.get(3 * i + k);
      at::Tensor g;
      if (a.has_value() && a->defined()) {
        check_f32(*a, "accumulated gradient", x);
        TORCH_CHECK(a->numel() == channels[i], "accumulated BatchNorm gradient size");
        g = *a;
        (k == 0 ? pt.acc_gamma : pt.acc_beta)[i] = 1;
      } else {
        g = at::empty({channels[i]}, x.options());
      }
      (k == 0 ? pt.dgamma : pt.dbeta)[i] = g.data_ptr<float>();
      dgb.push_back(g);
    }
  }
  auto dz = at::empty_like(z);
  launch_bn_backward_parts(pt, z.data_ptr<float>(), mean.data_ptr<float>(),
                           invstd.data_ptr<float>(), dz.data_ptr<float>(), n, c, s, cur_stream(x));
  std::vector<at::Tensor> out;
  Parts pc = make_parts(x, {weights[0]}, geo, relu);  // input geometry of the 1x1 convolutions
  at::Tensor dx;
  if (need_dx) {
    check_f32(w_cat_t, "w_cat_t", x);
    TORCH_CHECK(w_cat_t.size(0) == x.size(1) && w_cat_t.numel() == c * x.size(1),
                "w_cat_t must be the concatenated weights transposed to [ci][sum co]");
    ConvGemmGeo g = pc.geo[0];
    g.co = static_cast<int>(c);
    g.co_total = static_cast<int>(c);
    g.co_off = 0;
    g.fill = dx_fillable(g);
    const bool zero = dx_needs_zero(g) && !g.fill;
    dx = zero ? at::zeros_like(x) : at::empty_like(x);
    backward_data_into(w_cat_t, dz, x, dx, g, zero);
  }
  out.push_back(dx);
  for (auto& g : dgb) out.push_back(g);
  int64_t off = 0;
  for (size_t i = 0; i < np; ++i) {
    check_f32(weights[i], "weight", x);
    TORCH_CHECK(weights[i].size(0) == channels[i] && weights[i].size(1) == x.size(1) &&
                    weights[i].numel() == channels[i] * x.size(1),
                "grouped operations must be 1x1 convolutions of the input");
    ConvGemmGeo g = pc.geo[0];
    g.co = static_cast<int>(channels[i]);
    g.co_total = static_cast<int>(c);
    g.co_off = static_cast<int>(off);
    off += channels[i];
    const c10::optional<at::Tensor> a = accum.get(3 * i + 2);
    out.push_back(wgrad_part(dz, x, weights[i], g,
                             a.has_value() && a->defined() ? *a : at::Tensor(), slab_of(slabs, i),
                             first_of(slab_first, i)));
  }
  return out;
}

// Weight gradients of a fused op from its BatchNorm-backward output dz (convbn_backward
// with defer_wgrad), on the current stream: dW_i (+)= dz[:, part i] x relu(X) taps.
std::vector<at::Tensor> convbn_wgrad(const at::Tensor& dz, const at::Tensor& x_in,
                                     at::TensorList weights, at::IntArrayRef geo, bool relu,
                                     const c10::List<c10::optional<at::Tensor>>& accum,
                                     const c10::List<c10::optional<at::Tensor>>& slabs,
                                     at::IntArrayRef slab_first) {
  auto x = x_in.contiguous();
  check_f32(x, "x", x);
  check_f32(dz, "dz", x);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Parts p = make_parts(x, weights, geo, relu);
  TORCH_CHECK(dz.dim() == 4 && dz.size(0) == x.size(0) && dz.size(1) == p.co_total &&
                  dz.size(2) == p.ho && dz.size(3) == p.wo,
              "dz does not match the operation's output");
  TORCH_CHECK(accum.empty() || accum.size() == p.geo.size(),
              "accum must be empty or hold one gradient per weight");
  std::vector<at::Tensor> out;
  for (size_t i = 0; i < p.geo.size(); ++i) {
    at::Tensor into;
    if (!accum.empty()) {
      const c10::optional<at::Tensor> t = accum.get(i);
      if (t.has_value() && t->defined()) {
        check_f32(*t, "accumulated gradient", x);
        TORCH_CHECK(t->numel() == weights[i].numel(), "accumulated gradient has the wrong size");
        into = *t;
      }
    }
    out.push_back(wgrad_part(dz, x, weights[i], p.geo[i], into, slab_of(slabs, i),
                             first_of(slab_first, i)));
  }
  return out;
}

// Benchmark hook (benchmarks/convgemm_sweep.py): device time of every candidate plan of one
// convolution's GEMM `mode` (0 fwd, 1 bwd-data, 2 wgrad), `reps` back-to-back launches each
// (kernel + split reduction) between two events.  Returns [cfg, splits, microseconds]*.
std::vector<double> conv_gemm_sweep(int64_t mode, const at::Tensor& x_in,
                                    const at::Tensor& weight, at::IntArrayRef geo, int64_t reps) {
  auto x = x_in.contiguous();
  check_f32(x, "x", x);
  TORCH_CHECK(mode >= 0 && mode <= 2 && reps > 0, "mode 0-2, reps > 0");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Parts p = make_parts(x, {weight}, geo, false);
  ConvGemmGeo& g = p.geo[0];
  const at::Tensor wt_t = weight.transpose(0, 1).contiguous();
  auto z = at::randn({x.size(0), p.co_total, p.ho, p.wo}, x.options());
  auto dx = at::empty_like(x);
  auto dw = at::empty_like(weight);
  const float *a, *b;
  float* out;
  int64_t a_bytes, b_bytes;
  if (mode == 0) {
    a = weight.data_ptr<float>(); b = x.data_ptr<float>(); out = z.data_ptr<float>();
    a_bytes = weight.numel() * 4; b_bytes = x.numel() * 4;
  } else if (mode == 1) {
    a = wt_t.data_ptr<float>(); b = z.data_ptr<float>(); out = dx.data_ptr<float>();
    a_bytes = weight.numel() * 4; b_bytes = z.numel() * 4;
    g.a_t = true;
  } else {
    a = z.data_ptr<float>(); b = x.data_ptr<float>(); out = dw.data_ptr<float>();
    a_bytes = z.numel() * 4; b_bytes = x.numel() * 4;
  }
  const hipStream_t stream = cur_stream(x);
  hipEvent_t t0, t1;
  hipEventCreate(&t0);
  hipEventCreate(&t1);
  std::vector<double> res;
  for (const auto& cand : conv_gemm_candidates(static_cast<int>(mode), g)) {
    launch_one(static_cast<int>(mode), a, b, nullptr, out, nullptr, nullptr, g, cand,
               cand.scatter, a_bytes, b_bytes, x);  // warm-up
    hipEventRecord(t0, stream);
    for (int64_t r = 0; r < reps; ++r)
      launch_one(static_cast<int>(mode), a, b, nullptr, out, nullptr, nullptr, g, cand,
                 cand.scatter, a_bytes, b_bytes, x);
    hipEventRecord(t1, stream);
    hipEventSynchronize(t1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, t0, t1);
    res.push_back(cand.cfg);
    res.push_back(cand.splits);
    res.push_back(1000.0 * ms / static_cast<double>(reps));
  }
  hipEventDestroy(t0);
  hipEventDestroy(t1);
  return res;
}

// Plain convolution (no BatchNorm) through the same kernels: forward / backward-data /
// weight-gradient, e.g. U-Net's final 1x1 segmentation convolution.
at::Tensor conv_gemm_forward(const at::Tensor& x_in, const at::Tensor& weight,
                             at::IntArrayRef geo, bool relu) {
  auto x = x_in.contiguous();
  check_f32(x, "x", x);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Parts p = make_parts(x, {weight}, geo, relu);
  auto z = at::empty({x.size(0), p.co_total, p.ho, p.wo}, x.options());
  const ConvGemmPlan plan =
      tuned_plan(0, weight.data_ptr<float>(), x.data_ptr<float>(), nullptr, z.data_ptr<float>(),
                 nullptr, nullptr, p.geo[0], false, weight.numel() * 4, x.numel() * 4, x,
                 z.numel(), ASource{&weight, false});
  run_gemm(0, weight.data_ptr<float>(), x.data_ptr<float>(), nullptr, z.data_ptr<float>(),
           nullptr, nullptr, p.geo[0], plan, false, weight.numel() * 4, x.numel() * 4, x,
           ASource{&weight, false});
  return z;
}

at::Tensor conv_gemm_backward_data(const at::Tensor& dz_in, const at::Tensor& x_in,
                                   const at::Tensor& weight, at::IntArrayRef geo, bool relu,
                                   const c10::optional<at::Tensor>& weight_t) {
  auto x = x_in.contiguous();
  auto dz = dz_in.contiguous();
  check_f32(x, "x", x);
  check_f32(dz, "dz", x);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Parts p = make_parts(x, {weight}, geo, relu);
  TORCH_CHECK(dz.size(1) == p.co_total && dz.size(2) == p.ho && dz.size(3) == p.wo,
              "dz does not match the convolution's output");
  ConvGemmGeo g0 = p.geo[0];
  g0.fill = dx_fillable(g0);
  const bool zero = dx_needs_zero(g0) && !g0.fill;
  auto dx = zero ? at::zeros_like(x) : at::empty_like(x);
  at::Tensor wt;  // A = W^T (see convbn_backward)
  if (weight_t.has_value() && weight_t->defined()) {
    check_f32(*weight_t, "weight_t", x);
    TORCH_CHECK(weight_t->dim() == 4 && weight_t->size(0) == weight.size(1) &&
                    weight_t->size(1) == weight.size(0) && weight_t->numel() == weight.numel(),
                "weight_t must be the weight transposed to [ci][co][kh][kw]");
    wt = *weight_t;
  } else {
    wt = weight.transpose(0, 1).contiguous();
  }
  backward_data_into(wt, dz, x, dx, g0, zero);
  return dx;
}

// `accum` (optional): accumulate into this tensor (the weight's .grad) and return it.
at::Tensor conv_gemm_backward_weight(const at::Tensor& dz_in, const at::Tensor& x_in,
                                     const at::Tensor& weight, at::IntArrayRef geo, bool relu,
                                     const c10::optional<at::Tensor>& accum,
                                     const c10::optional<at::Tensor>& slab, bool slab_first) {
  auto x = x_in.contiguous();
  auto dz = dz_in.contiguous();
  check_f32(x, "x", x);
  check_f32(dz, "dz", x);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  Parts p = make_parts(x, {weight}, geo, relu);
  TORCH_CHECK(dz.size(1) == p.co_total && dz.size(2) == p.ho && dz.size(3) == p.wo,
              "dz does not match the convolution's output");
  const bool acc = accum.has_value() && accum->defined();
  if (acc) {
    check_f32(*accum, "accum", x);
    TORCH_CHECK(accum->numel() == weight.numel(), "accum must have the weight's size");
  }
  return wgrad_part(dz, x, weight, p.geo[0], acc ? *accum : at::Tensor(), slab, slab_first);
}

// BatchNorm (training) of x[N][C][*] with micro-batch statistics, for DeferredBatchNorm:
// statistics partials per (image, channel), Chan/fp64 finalize (folded into the fp64
// accumulators `acc` [3][C] when given), one normalising pass.  Returns {y, mean, invstd}.
//
// Plain BatchNorm2d training (ops/fusion.py): running_mean / running_var (EMA with
// `momentum`, unbiased variance) and num_batches_tracked are updated by the finalize when
// given; `relu` applies a ReLU after the normalisation (its backward: bn_train_backward
// with relu).
std::vector<at::Tensor> bn_train_forward(const at::Tensor& x_in,
                                         const c10::optional<at::Tensor>& gamma,
                                         const c10::optional<at::Tensor>& beta,
                                         const c10::optional<at::Tensor>& acc, double eps,
                                         const c10::optional<at::Tensor>& running_mean,
                                         const c10::optional<at::Tensor>& running_var,
                                         const c10::optional<at::Tensor>& num_batches_tracked,
                                         double momentum, bool relu,
                                         const c10::optional<at::Tensor>& part,
                                         int64_t part_images) {
  auto x = x_in.contiguous();
  check_f32(x, "x", x);
  TORCH_CHECK(x.dim() >= 2, "x must be [N][C][*]");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int64_t n = x.size(0), c = x.size(1), s = n * c == 0 ? 0 : x.numel() / (n * c);
  const auto stream = cur_stream(x);
  // `part`: x's (mean, M2) partials left by its producer ([2][groups][C], `part_images`
  // images per group: bg_conv's `stats`) -- no statistics pass here
  const bool given = part.has_value() && part->defined();
  int64_t groups = n, width = s;
  if (given) {
    check_f32(*part, "part", x);
    TORCH_CHECK(part_images > 0, "part needs part_images > 0");
    groups = (n + part_images - 1) / part_images;
    width = part_images * s;
    TORCH_CHECK(part->numel() == 2 * groups * c, "part must be [2][ceil(n / part_images)][C]");
  }
  // the statistics outputs and the partials in one allocation (stat_block): a launch-bound
  // stage pays host time per allocation
  StatBlock st = stat_block(x, c, given ? 0 : 2 * n * c);
  float* const part0 = given ? part->data_ptr<float>() : st.extra;
  float* const part1 = part0 + groups * c;
  auto mean = st.mean, invstd = st.invstd;
  auto y = at::empty_like(x);
  if (x.numel() == 0) return {y, mean.zero_(), invstd.fill_(1.f), at::zeros({2, c}, x.options())};
  double* accp = nullptr;
  if (acc.has_value() && acc->defined()) {
    TORCH_CHECK(acc->device() == x.device() && acc->scalar_type() == at::kDouble &&
                    acc->is_contiguous() && acc->numel() == 3 * c,
                "acc must be a contiguous float64 [3][C] tensor on the input's device");
    accp = acc->data_ptr<double>();
  }
  const float* rm = opt_ptr(running_mean, "running_mean", x, c);
  const float* rv = opt_ptr(running_var, "running_var", x, c);
  TORCH_CHECK((rm == nullptr) == (rv == nullptr), "running_mean and running_var go together");
  int64_t* tracked = nullptr;
  if (num_batches_tracked.has_value() && num_batches_tracked->defined()) {
    TORCH_CHECK(num_batches_tracked->device() == x.device() &&
                    num_batches_tracked->scalar_type() == at::kLong &&
                    num_batches_tracked->numel() == 1,
                "num_batches_tracked must be a 1-element int64 tensor on the input's device");
    tracked = num_batches_tracked->data_ptr<int64_t>();
  }
  if (!given) launch_bn_stats(x.data_ptr<float>(), part0, part1, n, c, s, stream);
  auto sums = st.sums;  // zeroed by the finalize, for the backward
  launch_bn_finalize_apply(part0, part1,
                           static_cast<int>(groups), static_cast<int>(width), n, c, s,
                           static_cast<float>(eps), rm != nullptr ? momentum : 0.0,
                           mean.data_ptr<float>(), invstd.data_ptr<float>(),
                           const_cast<float*>(rm), const_cast<float*>(rv), tracked, accp,
                           sums.data_ptr<float>(), x.data_ptr<float>(),
                           opt_ptr(gamma, "gamma", x, c), opt_ptr(beta, "beta", x, c), nullptr,
                           y.data_ptr<float>(), stream, relu);
  return {y, mean, invstd, sums};
}

// Backward of bn_train_forward: {dx, dgamma, dbeta}.
std::vector<at::Tensor> bn_train_backward(const at::Tensor& dy_in, const at::Tensor& x_in,
                                          const at::Tensor& mean, const at::Tensor& invstd,
                                          at::Tensor& sums,
                                          const c10::optional<at::Tensor>& gamma,
                                          const c10::optional<at::Tensor>& beta, bool relu,
                                          const c10::optional<at::Tensor>& accum_gamma,
                                          const c10::optional<at::Tensor>& accum_beta) {
  auto x = x_in.contiguous();
  auto dy = dy_in.contiguous();
  check_f32(x, "x", x);
  check_f32(dy, "dy", x);
  TORCH_CHECK(dy.sizes() == x.sizes(), "dy must have x's shape");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int64_t n = x.size(0), c = x.size(1), s = n * c == 0 ? 0 : x.numel() / (n * c);
  check_f32(sums, "sums", x);
  TORCH_CHECK(sums.numel() == 2 * c, "sums must be the forward's [2][C] buffer");
  auto dx = at::empty_like(x);
  // gradient-accumulation fusion (ops/gradacc.py): the affine gradients added straight into
  // the parameters' existing .grad instead of returned for autograd's add
  const bool acc_g = accum_gamma.has_value() && accum_gamma->defined();
  const bool acc_b = accum_beta.has_value() && accum_beta->defined();
  auto dgamma = acc_g ? *accum_gamma : at::empty({c}, x.options());
  auto dbeta = acc_b ? *accum_beta : at::empty({c}, x.options());
  if (acc_g) check_f32(dgamma, "accum_gamma", x);
  if (acc_b) check_f32(dbeta, "accum_beta", x);
  TORCH_CHECK(dgamma.numel() == c && dbeta.numel() == c && dgamma.is_contiguous() &&
                  dbeta.is_contiguous(),
              "the affine gradients are contiguous [C]");
  launch_bn_backward(dy.data_ptr<float>(), x.data_ptr<float>(), mean.data_ptr<float>(),
                     invstd.data_ptr<float>(), opt_ptr(gamma, "gamma", x, c),
                     sums.data_ptr<float>(), dx.data_ptr<float>(), dgamma.data_ptr<float>(),
                     dbeta.data_ptr<float>(), acc_g, acc_b, n, c, s, 0, cur_stream(x), relu,
                     opt_ptr(beta, "beta", x, c));
  return {dx, dgamma, dbeta};
}

void dbn_commit64(at::Tensor& acc, at::Tensor& running_mean, at::Tensor& running_var,
                  double momentum) {
  TORCH_CHECK(acc.is_cuda() && acc.scalar_type() == at::kDouble && acc.is_contiguous(),
              "acc must be a contiguous float64 GPU tensor");
  const int64_t c = running_mean.numel();
  check_f32(running_mean, "running_mean", running_mean);
  check_f32(running_var, "running_var", running_mean);
  TORCH_CHECK(acc.numel() == 3 * c && running_var.numel() == c, "acc must be [3][C]");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(acc.device());
  launch_dbn_commit64(acc.data_ptr<double>(), running_mean.data_ptr<float>(),
                      running_var.data_ptr<float>(), c, momentum, cur_stream(running_mean));
}

// AmoebaNet's 3x3 average pools (pool.hip): y = pool(x) (+ add).
at::Tensor avgpool3_forward(const at::Tensor& x_in, int64_t stride,
                            const c10::optional<at::Tensor>& add) {
  auto x = x_in.contiguous();
  check_f32(x, "x", x);
  TORCH_CHECK(x.dim() == 4 && (stride == 1 || stride == 2), "x must be NCHW, stride 1 or 2");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const int64_t h = x.size(2), w = x.size(3);
  auto y = at::empty({x.size(0), x.size(1), (h - 1) / stride + 1, (w - 1) / stride + 1},
                     x.options());
  const float* ad = nullptr;
  at::Tensor add_c;
  if (add.has_value() && add->defined()) {
    add_c = add->contiguous();
    check_f32(add_c, "add", x);
    TORCH_CHECK(add_c.sizes() == y.sizes(), "add must have the pooled shape");
    ad = add_c.data_ptr<float>();
  }
  if (y.numel() > 0)
    launch_avgpool3_forward(x.data_ptr<float>(), ad, y.data_ptr<float>(), x.size(0) * x.size(1),
                            static_cast<int>(h), static_cast<int>(w), static_cast<int>(stride),
                            cur_stream(x));
  return y;
}

at::Tensor avgpool3_backward(const at::Tensor& dy_in, int64_t h, int64_t w, int64_t stride) {
  TORCH_CHECK(dy_in.dim() == 4 && dy_in.size(2) == (h - 1) / stride + 1 &&
                  dy_in.size(3) == (w - 1) / stride + 1,
              "dy does not match the pooled shape");
  // a channel slice (gradient of one input of a concatenation) is read in place
  int64_t dy_img = avgpool3_backward_strided_ok(static_cast<int>(h), static_cast<int>(w))
                       ? image_stride_if_channel_slice(dy_in) : 0;
  auto dy = dy_img > 0 ? dy_in : dy_in.contiguous();
  if (dy_img == 0) check_f32(dy, "dy", dy);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  auto dx = at::empty({dy.size(0), dy.size(1), h, w}, dy.options());
  if (dx.numel() > 0)
    launch_avgpool3_backward(dy.data_ptr<float>(), dx.data_ptr<float>(), dy.size(0), dy.size(1),
                             static_cast<int>(h), static_cast<int>(w), static_cast<int>(stride),
                             dy_img, cur_stream(dy));
  return dx;
}

// U-Net decoder: cat(upsample2x(x), skip) and its backward for x (unet_ops.hip).
at::Tensor add_relu_forward(const at::Tensor& a_in, const at::Tensor& b_in) {
  auto a = a_in.contiguous();
  auto b = b_in.contiguous();
  check_f32(a, "a", a);
  check_f32(b, "b", a);
  TORCH_CHECK(a.sizes() == b.sizes(), "a and b must have one shape");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(a.device());
  auto y = at::empty_like(a);
  launch_add_relu(a.data_ptr<float>(), b.data_ptr<float>(), y.data_ptr<float>(), a.numel(),
                  cur_stream(a));
  return y;
}

at::Tensor up2x_cat_forward(const at::Tensor& x_in, const at::Tensor& skip_in) {
  auto x = x_in.contiguous();
  auto skip = skip_in.contiguous();
  check_f32(x, "x", x);
  check_f32(skip, "skip", x);
  TORCH_CHECK(x.dim() == 4 && skip.dim() == 4 && skip.size(0) == x.size(0) &&
                  skip.size(2) == 2 * x.size(2) && skip.size(3) == 2 * x.size(3),
              "skip must be [N][C2][2H][2W] for x [N][C1][H][W]");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto out = at::empty({x.size(0), x.size(1) + skip.size(1), skip.size(2), skip.size(3)},
                       x.options());
  check_f32(out, "output", x);
  launch_up2x_cat(x.data_ptr<float>(), skip.data_ptr<float>(), out.data_ptr<float>(), x.size(0),
                  static_cast<int>(x.size(1)), static_cast<int>(skip.size(1)),
                  static_cast<int>(x.size(2)), static_cast<int>(x.size(3)), cur_stream(x));
  return out;
}

// dx = 2x2 block sums of dy[:, :c] (dy: the concatenation's gradient or its channel slice).
at::Tensor up2x_backward(const at::Tensor& dy_in, int64_t c) {
  TORCH_CHECK(dy_in.dim() == 4 && dy_in.size(1) >= c && dy_in.size(2) % 2 == 0 &&
                  dy_in.size(3) % 2 == 0, "dy must be [N][>=C][2H][2W]");
  auto dy = dy_in.narrow(1, 0, c);
  int64_t dy_img = image_stride_if_channel_slice(dy);
  if (dy_img == 0) {
    dy = dy.contiguous();
    dy_img = c * dy.size(2) * dy.size(3);
  }
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kFloat, "dy must be float32 on the GPU");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  const int64_t h = dy.size(2) / 2, w = dy.size(3) / 2;
  auto dx = at::empty({dy.size(0), c, h, w}, dy.options());
  launch_up2x_backward(dy.data_ptr<float>(), dx.data_ptr<float>(), dy.size(0),
                       static_cast<int>(c), static_cast<int>(h), static_cast<int>(w), dy_img,
                       cur_stream(dy));
  return dx;
}

at::Tensor maxpool2x2_forward(const at::Tensor& x_in, const c10::optional<at::Tensor>& add) {
  auto x = x_in.contiguous();
  check_f32(x, "x", x);
  TORCH_CHECK(x.dim() == 4, "x must be NCHW");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto y = at::empty({x.size(0), x.size(1), x.size(2) / 2, x.size(3) / 2}, x.options());
  const float* ad = nullptr;
  at::Tensor add_c;
  if (add.has_value() && add->defined()) {
    add_c = add->contiguous();
    check_f32(add_c, "add", x);
    TORCH_CHECK(add_c.sizes() == y.sizes(), "add must have the pooled shape");
    ad = add_c.data_ptr<float>();
  }
  launch_maxpool2x2_forward(x.data_ptr<float>(), ad, y.data_ptr<float>(), x.size(0) * x.size(1),
                            static_cast<int>(x.size(2)), static_cast<int>(x.size(3)),
                            cur_stream(x));
  return y;
}

at::Tensor maxpool2x2_backward(const at::Tensor& x_in, const at::Tensor& dy_in) {
  auto x = x_in.contiguous();
  check_f32(x, "x", x);
  TORCH_CHECK(x.dim() == 4 && dy_in.dim() == 4 && dy_in.size(2) == x.size(2) / 2 &&
                  dy_in.size(3) == x.size(3) / 2 && dy_in.size(1) == x.size(1) &&
                  dy_in.size(0) == x.size(0),
              "dy must be the pooled shape of x");
  TORCH_CHECK(dy_in.scalar_type() == at::kFloat && dy_in.device() == x.device(),
              "dy must be fp32 on x's device");
  // a channel slice (gradient of one input of a concatenation) is read in place
  const int64_t dy_img = image_stride_if_channel_slice(dy_in);
  auto dy = dy_img > 0 ? dy_in : dy_in.contiguous();
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const bool odd = (x.size(2) & 1) || (x.size(3) & 1);
  auto dx = odd ? at::zeros_like(x) : at::empty_like(x);
  const int64_t c = x.size(1);
  launch_maxpool2x2_backward(x.data_ptr<float>(), dy.data_ptr<float>(), dx.data_ptr<float>(),
                             x.size(0) * c, static_cast<int>(c), static_cast<int>(x.size(2)),
                             static_cast<int>(x.size(3)),
                             dy_img > 0 ? dy_img : c * dy.size(2) * dy.size(3), cur_stream(x));
  return dx;
}

}  // namespace
}  // namespace tgpipe

TORCH_LIBRARY_FRAGMENT(tgpipe, m) {
  m.def("up2x_cat_forward(Tensor x, Tensor skip) -> Tensor");
  m.def("add_relu_forward(Tensor a, Tensor b) -> Tensor");
  m.def("up2x_backward(Tensor dy, int c) -> Tensor");
  m.def("maxpool2x2_forward(Tensor x, Tensor? add=None) -> Tensor");
  m.def("maxpool2x2_backward(Tensor x, Tensor dy) -> Tensor");
  m.def("avgpool3_forward(Tensor x, int stride, Tensor? add) -> Tensor");
  m.def("avgpool3_backward(Tensor dy, int h, int w, int stride) -> Tensor");
  m.def("bn_train_forward(Tensor x, Tensor? gamma, Tensor? beta, Tensor(a!)? acc, float eps, "
        "Tensor(b!)? running_mean=None, Tensor(c!)? running_var=None, "
        "Tensor(d!)? num_batches_tracked=None, float momentum=0.0, bool relu=False, "
        "Tensor? part=None, int part_images=0) -> Tensor[]");
  m.def("bn_train_backward(Tensor dy, Tensor x, Tensor mean, Tensor invstd, Tensor(a!) sums, "
        "Tensor? gamma, Tensor? beta=None, bool relu=False, Tensor(b!)? accum_gamma=None, "
        "Tensor(c!)? accum_beta=None) -> Tensor[]");
  m.def("dbn_commit64(Tensor(a!) acc, Tensor(b!) running_mean, Tensor(c!) running_var, "
        "float momentum) -> ()");
  m.def("convbn_forward(Tensor x, Tensor[] weights, int[] geo, bool relu, Tensor? gamma, "
        "Tensor? beta, Tensor(a!)? running_mean, Tensor(b!)? running_var, "
        "Tensor(c!)? num_batches_tracked, float momentum, float eps, Tensor? add, "
        "bool relu_out=False) -> Tensor[]");
  m.def("convbn_backward(Tensor dy, Tensor x, Tensor z, Tensor mean, Tensor invstd, "
        "Tensor(a!) sums, Tensor? gamma, Tensor[] weights, int[] geo, bool relu, bool need_dx, "
        "Tensor?[] accum, Tensor[] weights_t, bool defer_wgrad, Tensor?[] slabs, "
        "int[] slab_first, Tensor? beta=None, bool relu_out=False, Tensor? dx_into=None, "
        "Tensor? y_mask=None, Tensor(b!)? dy_masked=None) -> Tensor[]");
  m.def("convbn_group_forward(Tensor x, Tensor w_cat, int[] geo, bool relu, int[] channels, "
        "Tensor?[] gammas, Tensor?[] betas, Tensor?[] running_means, Tensor?[] running_vars, "
        "Tensor?[] tracked, float momentum, float eps) -> Tensor[]");
  m.def("convbn_group_backward(Tensor?[] dys, Tensor x, Tensor z, Tensor mean, Tensor invstd, "
        "Tensor[] weights, Tensor w_cat_t, int[] geo, bool relu, bool need_dx, int[] channels, "
        "Tensor?[] gammas, Tensor?[] accum, Tensor?[] slabs, int[] slab_first) -> Tensor[]");
  m.def("convbn_group_backward_ok(int n, int c, int hw) -> bool",
        &tgpipe::convbn_group_backward_ok);
  m.def("convbn_wgrad(Tensor dz, Tensor x, Tensor[] weights, int[] geo, bool relu, "
        "Tensor?[] accum, Tensor?[] slabs, int[] slab_first) -> Tensor[]");
  m.def("wgrad_slab_flush(Tensor[] slabs, Tensor(a!)[] grads, int[] accumulate) -> ()");
  m.def("conv_gemm_forward(Tensor x, Tensor weight, int[] geo, bool relu) -> Tensor");
  m.def("conv_gemm_plans_export() -> str", &tgpipe::conv_gemm_plans_export);
  m.def("lib_dgrad_export() -> str", &tgpipe::lib_dgrad_export);
  m.def("lib_dgrad_import(str text) -> int", &tgpipe::lib_dgrad_import);
  m.def("lib_dgrad_force(int mode) -> ()", &tgpipe::lib_dgrad_force);
  m.def("conv_gemm_force_cfg(int cfg, int splits=1) -> ()", &tgpipe::conv_gemm_force_cfg);
  m.def("conv_gemm_presplit(int budget_mb, bool clear=True) -> int", &tgpipe::conv_gemm_presplit);
  m.def("conv_gemm_presplit_refresh(Tensor[] sources) -> int",
        &tgpipe::conv_gemm_presplit_refresh);
  m.def("conv_gemm_presplit_step(int step) -> ()", &tgpipe::conv_gemm_presplit_step);
  m.def("conv_gemm_sweep(int mode, Tensor x, Tensor weight, int[] geo, int reps) -> float[]");
  m.def("conv_gemm_plans_import(str text) -> int", &tgpipe::conv_gemm_plans_import);
  m.def("conv_gemm_backward_data(Tensor dz, Tensor x, Tensor weight, int[] geo, bool relu, "
        "Tensor? weight_t=None) -> Tensor");
  m.def("conv_gemm_backward_weight(Tensor dz, Tensor x, Tensor weight, int[] geo, bool relu, "
        "Tensor? accum=None, Tensor? slab=None, bool slab_first=False) -> Tensor");
}

TORCH_LIBRARY_IMPL(tgpipe, CUDA, m) {
  m.impl("convbn_forward", &tgpipe::convbn_forward);
  m.impl("convbn_backward", &tgpipe::convbn_backward);
  m.impl("convbn_wgrad", &tgpipe::convbn_wgrad);
  m.impl("convbn_group_forward", &tgpipe::convbn_group_forward);
  m.impl("convbn_group_backward", &tgpipe::convbn_group_backward);
  m.impl("wgrad_slab_flush", &tgpipe::wgrad_slab_flush);
  m.impl("conv_gemm_forward", &tgpipe::conv_gemm_forward);
  m.impl("conv_gemm_sweep", &tgpipe::conv_gemm_sweep);
  m.impl("conv_gemm_backward_data", &tgpipe::conv_gemm_backward_data);
  m.impl("conv_gemm_backward_weight", &tgpipe::conv_gemm_backward_weight);
  m.impl("bn_train_forward", &tgpipe::bn_train_forward);
  m.impl("bn_train_backward", &tgpipe::bn_train_backward);
  m.impl("dbn_commit64", &tgpipe::dbn_commit64);
  m.impl("avgpool3_forward", &tgpipe::avgpool3_forward);
  m.impl("avgpool3_backward", &tgpipe::avgpool3_backward);
  m.impl("up2x_cat_forward", &tgpipe::up2x_cat_forward);
  m.impl("add_relu_forward", &tgpipe::add_relu_forward);
  m.impl("up2x_backward", &tgpipe::up2x_backward);
  m.impl("maxpool2x2_forward", &tgpipe::maxpool2x2_forward);
  m.impl("maxpool2x2_backward", &tgpipe::maxpool2x2_backward);
}
