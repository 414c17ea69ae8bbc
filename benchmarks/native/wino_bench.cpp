// Standalone timing harness for the Winograd forward kernels (no PyTorch): builds
// against csrc/winograd.hip so compile-time experiments (-D flags) can be compared in
// one GPU session.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I torchgpipe_amd/csrc \
//       benchmarks/native/wino_bench.cpp torchgpipe_amd/csrc/winograd.hip -o wino_bench
//   ./wino_bench <variant> N C K H [iters]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "kernels.h"

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 6) {
    std::fprintf(stderr, "usage: %s variant N C K H [iters]\n", argv[0]);
    return 2;
  }
  const int variant = std::atoi(argv[1]);
  const int64_t n = std::atoll(argv[2]), c = std::atoll(argv[3]), k = std::atoll(argv[4]),
                h = std::atoll(argv[5]);
  const int iters = argc > 6 ? std::atoi(argv[6]) : 20;
  const int64_t w = h;
  std::vector<float> hx(n * c * h * w), hw(k * c * 9);
  unsigned s = 1;
  for (auto& v : hx) v = ((s = s * 1664525u + 1013904223u) >> 8) * (1.f / 16777216.f) - 0.5f;
  for (auto& v : hw) v = ((s = s * 1664525u + 1013904223u) >> 8) * (1.f / 16777216.f) - 0.5f;
  float *x, *wt, *u, *y, *ws = nullptr;
  CHECK(hipMalloc(&x, hx.size() * 4));
  CHECK(hipMalloc(&wt, hw.size() * 4));
  CHECK(hipMalloc(&u, tgpipe::wino_pad_reduction(c) * tgpipe::wino_pad_output(k) * 16 * 4));
  CHECK(hipMalloc(&y, n * k * h * w * 4));
  CHECK(hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(wt, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
  tgpipe::launch_wino_weight(wt, u, k, c, false, nullptr);
  const tgpipe::WinoPlan plan = tgpipe::wino_plan(n, c, h, w, k, variant, 0);
  if (plan.workspace) CHECK(hipMalloc(&ws, plan.workspace * 4));
  for (int i = 0; i < 3; ++i) tgpipe::launch_wino_conv(x, u, nullptr, y, ws, n, c, h, w, k, plan, nullptr);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  CHECK(hipEventRecord(a, nullptr));
  for (int i = 0; i < iters; ++i)
    tgpipe::launch_wino_conv(x, u, nullptr, y, ws, n, c, h, w, k, plan, nullptr);
  CHECK(hipEventRecord(b, nullptr));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  ms /= iters;
  // checksum of a few outputs against a direct convolution on the host
  std::vector<float> hy(n * k * h * w);
  CHECK(hipMemcpy(hy.data(), y, hy.size() * 4, hipMemcpyDeviceToHost));
  double maxerr = 0, maxref = 0;
  for (int t = 0; t < 64; ++t) {
    const int64_t idx = (static_cast<int64_t>(t) * 2654435761u) % hy.size();
    const int64_t ni = idx / (k * h * w), ki = (idx / (h * w)) % k, yi = (idx / w) % h, xi = idx % w;
    double ref = 0;
    for (int64_t ci = 0; ci < c; ++ci)
      for (int dy = 0; dy < 3; ++dy)
        for (int dx = 0; dx < 3; ++dx) {
          const int64_t yy = yi + dy - 1, xx = xi + dx - 1;
          if (yy < 0 || yy >= h || xx < 0 || xx >= w) continue;
          ref += double(hx[((ni * c + ci) * h + yy) * w + xx]) * hw[((ki * c + ci) * 3 + dy) * 3 + dx];
        }
    maxerr = std::max(maxerr, std::abs(ref - hy[idx]));
    maxref = std::max(maxref, std::abs(ref));
  }
  const double tf = 2.0 * n * k * c * 9 * h * w / (ms * 1e9);
  std::printf("{\"variant\": %d, \"shape\": [%ld, %ld, %ld, %ld], \"splits\": %d, \"ms\": %.4f, "
              "\"direct_tflops\": %.1f, \"rel_err\": %.2e}\n",
              plan.variant, (long)n, (long)c, (long)k, (long)h, plan.splits, ms, tf,
              maxerr / (maxref + 1e-30));
  return 0;
}
