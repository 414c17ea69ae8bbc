"""1x1 stride-1 convolutions as plain GEMMs: the implicit-GEMM kernels (csrc/conv_gemm.hip)
vs the library GEMM (torch.matmul -> hipBLASLt / rocBLAS) at ResNet-101 pipeline-1 shapes
(micro-batch 110) and AmoebaNet n1m32 shapes (micro-batch 20): forward, backward-data and
weight gradient, device time per call.

    python benchmarks/diag/gemm_lib_probe.py
"""
import json

import torch

SHAPES = [  # n, ci, co, hw
    (110, 64, 256, 56), (110, 256, 64, 56), (110, 128, 512, 28), (110, 512, 128, 28),
    (110, 256, 1024, 14), (110, 1024, 256, 14), (110, 512, 2048, 7), (110, 2048, 512, 7),
    (20, 1024, 1024, 7), (20, 4096, 1024, 7), (20, 256, 256, 28), (20, 1024, 256, 28),
]


def timed(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return round(a.elapsed_time(b) * 1000 / iters, 1)


def main() -> None:
    ops = torch.ops.tgpipe
    import torchgpipe_amd.ops._ext as ext
    ext.require(torch.empty(0, device='cuda'))
    geo = [1, 1, 1, 1, 0, 0, 0, 0]
    for n, ci, co, hw in SHAPES:
        x = torch.randn(n, ci, hw, hw, device='cuda')
        w = torch.randn(co, ci, 1, 1, device='cuda') / ci ** 0.5
        dz = torch.randn(n, co, hw, hw, device='cuda')
        w2 = w.view(co, ci)
        xv, dzv = x.view(n, ci, hw * hw), dz.view(n, co, hw * hw)
        gflop = 2 * n * ci * co * hw * hw / 1e9
        row = {'n': n, 'ci': ci, 'co': co, 'hw': hw, 'gflop': round(gflop, 2),
               'ours_fwd': timed(lambda: ops.conv_gemm_forward(x, w, geo, False)),
               'lib_fwd': timed(lambda: torch.matmul(w2, xv)),
               'ours_dgrad': timed(lambda: ops.conv_gemm_backward_data(dz, x, w, geo, False)),
               'lib_dgrad': timed(lambda: torch.matmul(w2.t(), dzv)),
               'ours_wgrad': timed(lambda: ops.conv_gemm_backward_weight(dz, x, w, geo, False)),
               'lib_wgrad': timed(lambda: torch.bmm(dzv, xv.transpose(1, 2)).sum(0))}
        ref = torch.matmul(w2, xv)
        got = ops.conv_gemm_forward(x, w, geo, False).view(n, co, -1)
        row['fwd_rel'] = ((got - ref).norm() / ref.norm()).item()
        for k in ('fwd', 'dgrad', 'wgrad'):
            row[k + '_lib_tflops'] = round(gflop / row['lib_' + k] * 1e3, 1)
            row[k + '_ours_tflops'] = round(gflop / row['ours_' + k] * 1e3, 1)
        print(json.dumps(row), flush=True)


if __name__ == '__main__':
    main()
