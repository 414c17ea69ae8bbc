"""Capture AmoebaNet-D(18,256) training steps with N-stream cells (debug, one GPU).

``--mode step``: the whole step as one hipGraph (StepGraph, big-stack thread);
``--mode cells``: per-micro-batch graphs (PipelineStage(graph_cells=True)).
Prints the DAG size (kernel nodes of the captured step when known) and the step time.
Run under ``python -X faulthandler`` so a crash names its Python frame.
"""
import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

p = argparse.ArgumentParser()
p.add_argument('--streams', type=int, default=3)
p.add_argument('--chunks', type=int, default=32)
p.add_argument('--micro', type=int, default=20)
p.add_argument('--layers', type=int, default=18)
p.add_argument('--filters', type=int, default=256)
p.add_argument('--mode', choices=['step', 'cells'], default='step')
p.add_argument('--steps', type=int, default=3)
args = p.parse_args()
os.environ['TGPIPE_CAPTURE_CELL_STREAMS'] = str(args.streams)

from torchgpipe_amd.models import amoebanetd  # noqa: E402
from torchgpipe_amd.models.amoebanet import set_cell_streams  # noqa: E402
from torchgpipe_amd.parallel import PipelineStage, StepGraph  # noqa: E402

dev = torch.device('cuda', 0)
torch.manual_seed(0)
model = amoebanetd(num_classes=1000, num_layers=args.layers, num_filters=args.filters)
stage = PipelineStage(model, [len(model)], device=dev, chunks=args.chunks,
                      graph_cells=args.mode == 'cells')
set_cell_streams(stage.partition, args.streams)
opt = torch.optim.SGD(stage.parameters(), lr=0.1)
batch = args.chunks * args.micro
x = torch.rand(batch, 3, 224, 224, device=dev)
t = torch.randint(1000, (batch,), device=dev)
print(f'mode={args.mode} streams={args.streams} chunks={args.chunks} micro={args.micro}',
      flush=True)
if args.mode == 'step':
    graph = StepGraph(stage, F.cross_entropy, opt, warmup=1)

    def step():
        graph.step(x, t)
else:
    def step():
        stage.train_step(x, t, F.cross_entropy)
        opt.step()
        opt.zero_grad(set_to_none=True)

for k in range(args.steps + 2):
    t0 = time.perf_counter()
    step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    phase = ('captured' if graph.captured else 'eager') if args.mode == 'step' \
        else stage.graph_phase
    print(f'step {k}: {phase} {1000 * dt:.1f} ms ({batch / dt:.1f} samples/s)', flush=True)
print('ok', flush=True)
