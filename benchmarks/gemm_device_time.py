"""Device-only time of the AmoebaNet implicit-GEMM convolutions (hipGraph-timed).

Timing back-to-back eager calls measures the host when a kernel is short (~10-20 us of
Python, allocation and launch per call); here `iters` calls are captured into one hipGraph
and the replays are timed, so only device time remains.  For each shape: this package's
forward / backward-data / weight-gradient, MIOpen (F.conv2d / convolution_backward) and,
for 1x1 shapes, hipBLASLt's batched GEMM of the same product (W @ X[n]).

    python benchmarks/gemm_device_time.py [out.json]
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # n, c, h, co, kh, kw
    (20, 1024, 7, 1024, 1, 1), (20, 4096, 7, 1024, 1, 1), (20, 2048, 14, 512, 1, 1),
    (20, 1024, 28, 256, 1, 1), (20, 512, 14, 512, 1, 1), (20, 256, 28, 256, 1, 1),
    (20, 64, 28, 64, 1, 7), (20, 128, 14, 128, 7, 1), (20, 256, 7, 256, 1, 7),
]


def graph_time(fn, iters: int = 20, reps: int = 5) -> float:
    """Median microseconds per call of ``fn`` replayed from a captured hipGraph."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    times = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        e.synchronize()
        times.append(1000.0 * s.elapsed_time(e) / iters)
    return sorted(times)[len(times) // 2]


def main() -> None:
    from torchgpipe_amd.ops import _ext
    ops = _ext.require()
    rows = []
    for n, c, h, co, kh, kw in SHAPES:
        x = torch.randn(n, c, h, h, device='cuda')
        wt = torch.randn(co, c, kh, kw, device='cuda') * 0.05
        pad = ((kh - 1) // 2, (kw - 1) // 2)
        geo = [kh, kw, 1, 1, pad[0], pad[1], 0, 0]
        z = ops.conv_gemm_forward(x, wt, geo, True)
        dz = torch.randn_like(z)
        gflop = 2.0 * n * co * c * kh * kw * h * h / 1e9
        row = {'shape': [n, c, h, co, kh, kw], 'gflop': round(gflop, 3)}
        row['tgpipe_us'] = {
            'fwd': graph_time(lambda: ops.conv_gemm_forward(x, wt, geo, True)),
            'bwd': graph_time(lambda: ops.conv_gemm_backward_data(dz, x, wt, geo, True)),
            'wgrad': graph_time(lambda: ops.conv_gemm_backward_weight(dz, x, wt, geo, True)),
        }
        row['miopen_us'] = {
            'fwd': graph_time(lambda: F.conv2d(x, wt, padding=pad)),
            'bwd': graph_time(lambda: torch.ops.aten.convolution_backward(
                dz, x, wt, None, [1, 1], list(pad), [1, 1], False, [0, 0], 1,
                [True, False, False])),
            'wgrad': graph_time(lambda: torch.ops.aten.convolution_backward(
                dz, x, wt, None, [1, 1], list(pad), [1, 1], False, [0, 0], 1,
                [False, True, False])),
        }
        if kh == 1 and kw == 1:
            w2 = wt.view(co, c)
            xv = x.view(n, c, h * h)
            dzv = dz.view(n, co, h * h)
            row['hipblaslt_us'] = {
                'fwd': graph_time(lambda: torch.matmul(w2, xv)),
                'bwd': graph_time(lambda: torch.matmul(w2.t(), dzv)),
                'wgrad': graph_time(lambda: torch.einsum('nop,ncp->oc', dzv, xv)),
            }
        for k in [k for k in row if k.endswith('_us')]:
            row[k] = {m: round(v, 2) for m, v in row[k].items()}
        row['tgpipe_tflops'] = {m: round(gflop / v * 1e3, 1)
                                for m, v in row['tgpipe_us'].items()}
        rows.append(row)
        print(json.dumps(row), flush=True)
    if len(sys.argv) > 1:
        json.dump(rows, open(sys.argv[1], 'w'), indent=1)


if __name__ == '__main__':
    main()
