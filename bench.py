#!/usr/bin/env python
"""Headline benchmark: U-Net(5,64) GPipe training throughput, plus AmoebaNet-D(18,256).

Metric (BASELINE.json): samples/sec of a full SGD training step (forward,
backward with checkpoint recomputation, optimizer step) at 1/2/4/8 pipeline
partitions, using the reference's experiment tables
(``benchmarks/unet-speed/main.py:23-68``, ``benchmarks/amoebanetd-speed/main.py:35-96``):

    N=1  U-Net pipeline-1  B=80,  chunks=2,  balance [241]
    N=2  U-Net pipeline-2  B=512, chunks=32, balance [104, 137]
    N=4  U-Net pipeline-4  B=512, chunks=16, balance [30, 66, 84, 61]
    N=8  U-Net pipeline-8  B=640, chunks=40, balance [16, 27, 31, 44, 22, 57, 27, 17]

The top-level ``value`` is the U-Net headline: the reference balance on the plain eager
engine.  After it, every run also times (``--sections``), in this order:

* ``baseline``: the reference's speed-up denominator, U-Net(5,64) *without* GPipe
  (plain model, B=40, no checkpointing) on rank 0's GPU, so ``speedup_vs_baseline``
  is measured on the same box as the headline;
* ``gpipe`` (N=1): the headline experiment through the public single-process ``GPipe``
  API (the reference's own benchmark path), ``vs_pipeline_stage`` its ratio;
* ``amoebanet``: AmoebaNet-D(18,256), n{N}m32 at the reference balance (n1m32, B=640
  at N=1), and at N=2 the reference's own denominator n2m1 (B=96, ``always``);
* ``resnet``: ResNet-101 pipeline-1 (B=220, m=2) at N=1, BASELINE.json's config #2
  (pipeline-2, chunks=32, ``always``) at N=2, the reference's pipeline-4 / -8 (B=5632,
  m=256 / B=5400, m=150) at N=4 / 8, and the reference's ResNet denominator (no GPipe,
  B=118) on rank 0's GPU;
* at N > 1, the opt-in engine variants, each under its own key: ``tuned`` (the
  MI355X-tuned balances of U-Net and AmoebaNet), ``striped`` (N >= 3: the headline with
  multi-path transfers) and ``amoebanet_graph_cells`` (captured cells);
* for N > 1, one extra *diagnostic* step (not timed) in which every rank measures
  how long its streams waited for activations / gradients (``per_rank``).

One process per GPU (``torch.distributed.run``), RCCL point-to-point between
stages; fp32 like the reference.  Rank 0 prints the JSON record right after the headline
and re-prints it, augmented, after every section (each line complete; the last one the
most complete), so a late section that fails cannot lose the headline.

    python bench.py --gpus 1 --steps 5 --warmup 2
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        bench.py --gpus 8
"""
import argparse
import datetime
import gc
import json
import os
import sys
import time
from typing import Any, Callable, Dict, List, Optional

# Hardware queues of a multi-rank run: every stream a rank queues work on -- compute,
# lanes, AmoebaNet cell streams, relay routes -- and one stream per RCCL communicator
# (parallel/stage.py stream_census, HW_QUEUES; tests/test_stream_census.py checks the
# 8-rank pipelines, multi-path transfers included, against it).  HIP's default is 4:
# streams beyond that share a queue, whose work then runs in order, so a spinning RCCL
# receive could hold up unrelated compute.  Set before the HIP runtime initialises (first
# CUDA call); 32 is the most this pool's runtime is given.
HW_QUEUES = 32
if int(os.environ.get('WORLD_SIZE', '1')) > 1:
    os.environ.setdefault('GPU_MAX_HW_QUEUES', str(HW_QUEUES))

import torch
import torch.distributed as dist
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

# Reference (Tesla P40) throughputs of the same experiments, BASELINE.md §1/§2.
# Batch / chunks / reference balance are the reference's experiment tables.
# ``tuned`` balances for MI355X: the stage times of benchmarks/stage_harness.py (reference and
# earlier tuned balances) spread over their layers by the per-layer profile
# (profiles/unet_layer_profile_f4w.json) and min-max partitioned by
# scripts/balance_from_harness.py.  p2 from round 3; p4 / p8 re-derived on the round-4 tree
# (profiles/r4/final/stage_harness_unet_p{4,8}_tuned{,2}.json): measured max stage p2 522 /
# p4 235 / p8 176 ms against 537 / 283 / 240 for the reference balances
# (profiles/r4/speedup_prediction.md).
UNET_EXPERIMENTS = {
    1: dict(name='pipeline-1', batch=80, chunks=2, balance=[241], tuned=[241], ref=24.456),
    2: dict(name='pipeline-2', batch=512, chunks=32, balance=[104, 137], tuned=[100, 141],
            ref=35.502),
    4: dict(name='pipeline-4', batch=512, chunks=16, balance=[30, 66, 84, 61],
            tuned=[38, 55, 74, 74], ref=67.042),
    8: dict(name='pipeline-8', batch=640, chunks=40, balance=[16, 27, 31, 44, 22, 57, 27, 17],
            tuned=[18, 26, 27, 30, 22, 44, 40, 34], ref=88.497),
}
# the reference's speed-up denominator: U-Net without GPipe, one GPU
UNET_BASELINE = dict(name='baseline', batch=40, ref=28.500)
# AmoebaNet tuned balances: n4 from round 3 (every layer timed as its own stage at
# micro-batch 40, min-max partitioned: profiles/r3/speedup_prediction.md); n2 / n8 searched
# in round 5 with the step simulator at 100 GB/s links (scripts/r5/tune_transfer.py) and
# measured stage by stage (profiles/r5/harness/*_search.json): n2 [10, 14] predicts 1.784x
# over n2m1 where round 3's [11, 13] predicts 1.679x, n8 4.991x vs 4.956x.
AMOEBA_EXPERIMENTS = {
    1: dict(name='n1m32', batch=640, chunks=32, balance=[24], tuned=[24], ref=None),
    2: dict(name='n2m32', batch=1280, chunks=32, balance=[9, 15], tuned=[10, 14], ref=47.386),
    4: dict(name='n4m32', batch=1152, chunks=32, balance=[3, 6, 7, 8], tuned=[5, 6, 6, 7],
            ref=72.412),
    8: dict(name='n8m32', batch=1280, chunks=32, balance=[2, 2, 2, 3, 3, 4, 4, 4],
            tuned=[2, 2, 3, 3, 3, 3, 3, 5], ref=132.413),
}
# the reference's AmoebaNet speed-up denominator (benchmarks/amoebanetd-speed/main.py:39-45)
AMOEBA_N2M1 = dict(name='n2m1', batch=96, chunks=1, balance=[7, 17], ref=26.733)
# ResNet-101 (benchmarks/resnet101-speed/main.py:22-67): pipeline-1 as in
# the reference; at N=2 BASELINE.json's config #2, pipeline-2 at the reference balance with
# chunks=32 and 'always'.  The reference ran B=25000 as m=1667 micro-batches of 15 images,
# a P40 sizing: 15-image micro-batches leave an MI355X's GEMMs underfed (the stages run at
# half of pipeline-1's per-image speed, profiles/r4/speedup_prediction.md), so the 32
# micro-batches here hold pipeline-1's 110 images each (B = 3520).
# pipeline-2 is therefore not the reference's p2 configuration and carries no P40 number
# (``ref=None``; BASELINE.md's 135.539 is for B=25000, m=1667).  Pipeline-4 / -8 are the
# reference's own (B=5632, m=256 / B=5400, m=150: 22 / 36 images per micro-batch).
RESNET_EXPERIMENTS = {
    1: dict(name='pipeline-1', batch=220, chunks=2, balance=[370], checkpoint='except_last',
            ref=81.796),
    2: dict(name='pipeline-2 (BASELINE config #2: chunks=32, always, 110-image micro-batches)',
            batch=3520, chunks=32, balance=[135, 235], checkpoint='always', ref=None),
    4: dict(name='pipeline-4', batch=5632, chunks=256, balance=[44, 92, 124, 110],
            checkpoint='except_last', ref=265.958),
    8: dict(name='pipeline-8', batch=5400, chunks=150,
            balance=[26, 22, 33, 44, 44, 66, 66, 69], checkpoint='except_last', ref=411.662),
}
# the reference's ResNet speed-up denominator: ResNet-101 without GPipe, one GPU
RESNET_BASELINE = dict(name='baseline', batch=118, ref=95.862)


def parse() -> argparse.Namespace:
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawTextHelpFormatter)
    p.add_argument('--gpus', type=int, default=int(os.environ.get('WORLD_SIZE', '1')))
    p.add_argument('--steps', type=int, default=5)
    p.add_argument('--warmup', type=int, default=2)
    p.add_argument('--model', choices=['unet', 'amoebanet', 'resnet'], default='unet')
    p.add_argument('--checkpoint', choices=['always', 'except_last', 'never'], default=None,
                   help='override the experiment checkpoint mode (default: reference mode)')
    p.add_argument('--batch', type=int, default=None, help='override the global batch')
    p.add_argument('--chunks', type=int, default=None, help='override the micro-batch count')
    p.add_argument('--unfused', action='store_true', help='use the unfused PyTorch U-Net cells')
    p.add_argument('--balance', default='ref',
                   help="'ref' (the reference's experiment table, default), 'tuned' "
                        "(MI355X-measured) or a comma-separated list")
    p.add_argument('--also-tuned', choices=['auto', 'yes', 'no'], default='auto',
                   help="after the headline timing, time the MI355X-tuned balance too and "
                        "report it as the 'tuned' field (auto: when N > 1 and it differs)")
    p.add_argument('--sections', default='auto',
                   help="comma-separated extra timings after the headline, in this order: "
                        "'baseline' (U-Net without GPipe, B=40, rank 0), 'gpipe' (N=1: the "
                        "headline through single-process GPipe), 'amoebanet' (AmoebaNet-D "
                        "n{N}m32 and, at N=2, n2m1), 'resnet' (ResNet-101 pipeline-{N} and its "
                        "no-GPipe baseline), then at N > 1 the MI355X-tuned balances "
                        "(--also-tuned), 'striped' (N >= 3: the headline with multi-path "
                        "transfers) and 'graph_cells' (AmoebaNet with captured cells); "
                        "'auto' = all that apply when the headline is U-Net; 'none'.  The JSON "
                        'record is printed after the headline and re-printed after each section')
    p.add_argument('--section-steps', type=int, default=None,
                   help='timed steps of each extra section (default: --steps)')
    p.add_argument('--probe', choices=['auto', 'on', 'off'], default='auto',
                   help='one extra untimed step in which every rank measures its receive '
                        'waits (auto: N > 1)')
    p.add_argument('--timeout', type=float, default=120.0,
                   help='seconds any pipeline wait may take before the run fails (RCCL '
                        'watchdog and gloo waits): a dead or stuck rank ends the job')
    p.add_argument('--cudnn-benchmark', action='store_true',
                   help='MIOpen exhaustive find (slow first step, cached afterwards)')
    p.add_argument('--backend', choices=['auto', 'gloo'], default='auto',
                   help="tensor transport: 'auto' = RCCL on GPUs (gloo on CPU); 'gloo' stages "
                        "messages through host memory and lets several ranks share one GPU "
                        "(functional rehearsal only, not a valid measurement)")
    p.add_argument('--tiny', action='store_true',
                   help='tiny models of the same families (CI smoke test of this script only)')
    p.add_argument('--channels-last', action='store_true',
                   help='NHWC activations and weights (MIOpen NHWC kernels; AmoebaNet)')
    p.add_argument('--cell-streams', choices=['auto', 'on', 'off'], default='auto',
                   help="AmoebaNet: run each cell's independent nodes on several HIP streams "
                        '(TGPIPE_CELL_STREAMS, default 3; auto: on)')
    p.add_argument('--overlap-recompute', choices=['auto', 'on', 'off'], default='auto',
                   help="recompute the next micro-batch on a second stream during this one's "
                        'backward (PipelineStage(overlap_recompute=True); auto: on for '
                        'U-Net, and for ResNet-101 at N=1)')
    p.add_argument('--overlap-forward', choices=['auto', 'on', 'off'], default='auto',
                   help='alternate the forward micro-batches of a partition between two '
                        'streams (BatchNorm statistics slotted and folded in order; auto: on '
                        'for U-Net, and for ResNet-101 at N=1)')
    p.add_argument('--graph-cells', choices=['auto', 'on', 'off'], default='auto',
                   help='replay each micro-batch of a stage as captured hipGraphs, transfers '
                        'issued between them (PipelineStage(graph_cells=True), '
                        'parallel/segments.py; '
                        'auto: on for one-GPU AmoebaNet)')
    p.add_argument('--stripes', choices=['auto', 'on', 'off'], default='auto',
                   help='multi-path transfers in the headline: messages of at least '
                        '--stripe-mb also travel through up to 3 idle ranks over otherwise '
                        'unused links (PipelineStage(stripes=...), parallel/stripes.py; '
                        'planned from the first step, so the warm-up runs until the plan '
                        "exists; auto: off -- the 'striped' section times them at N >= 3)")
    p.add_argument('--stripe-mb', type=float, default=16.0,
                   help='smallest striped message, MB')
    p.add_argument('--profile-steps', type=int, default=0,
                   help='after timing, run N more steps under torch.profiler (rank 0)')
    return p.parse_args()


def even_balance(layers: int, parts: int) -> list:
    base, extra = divmod(layers, parts)
    return [base + (1 if i < extra else 0) for i in range(parts)]


def choice(value: str, auto: bool) -> bool:
    return {'on': True, 'off': False}.get(value, auto)


class Bench:
    """One bench job: process-group setup, model builders and the timing loops."""

    def __init__(self, args: argparse.Namespace) -> None:
        self.args = args
        self.world = int(os.environ.get('WORLD_SIZE', '1'))
        self.rank = int(os.environ.get('RANK', '0'))
        local_rank = int(os.environ.get('LOCAL_RANK', '0'))
        if self.world != args.gpus:
            raise SystemExit(f'--gpus {args.gpus} but WORLD_SIZE={self.world}: '
                             'launch one rank per GPU')
        self.gpu = torch.cuda.is_available()
        self.rehearsal = args.backend == 'gloo' and self.gpu and self.world > 1
        if self.gpu and not self.rehearsal and local_rank >= torch.cuda.device_count():
            raise SystemExit(f'LOCAL_RANK {local_rank} but only {torch.cuda.device_count()} GPUs')
        self.device = (torch.device('cuda', local_rank % torch.cuda.device_count()) if self.gpu
                       else torch.device('cpu'))
        if self.gpu:
            torch.cuda.set_device(self.device)
            torch.backends.cudnn.benchmark = args.cudnn_benchmark
        self.ctrl = None
        if self.world > 1:
            # Lazy RCCL init: each pipeline link (peer pair) then gets its own
            # communicator and stream on first use.
            backend = 'nccl' if self.gpu and not self.rehearsal else 'gloo'
            timeout = datetime.timedelta(seconds=args.timeout)
            dist.init_process_group(backend, rank=self.rank, world_size=self.world,
                                    timeout=timeout)
            self.ctrl = (dist.group.WORLD if backend == 'gloo'
                         else dist.new_group(backend='gloo', timeout=timeout))

    def log(self, msg: str) -> None:
        if self.rank == 0:
            print(f'[bench] {msg}', file=sys.stderr, flush=True)

    def sync(self) -> None:
        if self.world > 1:
            dist.barrier()
        if self.gpu:
            torch.cuda.synchronize(self.device)

    def ctrl_barrier(self) -> None:
        if self.world > 1:
            dist.barrier(group=self.ctrl)

    # -- models -----------------------------------------------------------------------------

    def build(self, kind: str, meta: bool = True) -> torch.nn.Sequential:
        from torchgpipe_amd.models import amoebanetd, resnet101, unet
        args = self.args
        ctx = torch.device('meta') if meta else torch.device(self.device)
        # Built on the meta device for pipelines: each rank materialises (random-initialises)
        # only its own partition inside PipelineStage.
        with ctx:
            if kind == 'unet':
                if args.tiny:
                    return unet(depth=2, num_convs=1, base_channels=4, input_channels=3,
                                output_channels=1, fused=not args.unfused)
                return unet(depth=5, num_convs=5, base_channels=64, input_channels=3,
                            output_channels=1, fused=not args.unfused)
            if kind == 'resnet':
                if args.tiny:
                    from torchgpipe_amd.models.resnet import build_resnet
                    return build_resnet([1, 1, 1, 1], num_classes=10)
                return resnet101(num_classes=1000)
            if args.tiny:
                return amoebanetd(num_classes=10, num_layers=3, num_filters=8)
            return amoebanetd(num_classes=1000, num_layers=18, num_filters=256)

    def data(self, kind: str, batch: int, first: bool, last: bool):
        gen = torch.Generator(device=self.device).manual_seed(0)
        if kind == 'unet':
            shape = (3, 192, 192)
            x = torch.rand(batch, *shape, device=self.device, generator=gen) if first else None
            t = torch.ones(batch, 1, 192, 192, device=self.device) if last else None
            return x, t, F.binary_cross_entropy_with_logits, shape
        shape = (3, 224, 224)
        x = torch.rand(batch, *shape, device=self.device, generator=gen) if first else None
        t = (torch.randint(10 if self.args.tiny else 1000, (batch,), device=self.device,
                           generator=gen) if last else None)
        if x is not None and self.args.channels_last:
            x = x.contiguous(memory_format=torch.channels_last)
        return x, t, F.cross_entropy, shape

    # -- timing -----------------------------------------------------------------------------

    def timed(self, step: Callable[[], None], steps: int, warmup: int, tag: str,
              settle: Optional[Callable[[], bool]] = None) -> Dict[str, float]:
        """``warmup`` untimed steps (plus any until ``settle()``), then ``steps`` timed steps
        bracketed by a barrier and a device sync; elapsed = MAX over ranks."""
        t0 = time.time()
        first_s = 0.0
        for k in range(warmup):
            step()
            self.sync()
            if k == 0:
                first_s = time.time() - t0
            self.log(f'{tag} warmup step {k + 1}/{warmup} done at {time.time() - t0:.1f}s')
        while settle is not None and not settle():  # e.g. a hipGraph capture: untimed
            step()
            self.sync()
        warm_s = time.time() - t0
        self.sync()
        start = time.perf_counter()
        for _ in range(steps):
            step()
        self.sync()
        elapsed = time.perf_counter() - start
        if self.world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device=self.device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        self.log(f'{tag}: {steps} steps in {elapsed:.3f}s')
        return {'elapsed': elapsed, 'warm_s': warm_s, 'first_step_s': first_s}

    def pipeline(self, kind: str, exp: Dict[str, Any], balance: List[int], checkpoint: str,
                 steps: int, tag: str, probe: bool = False, stripes: Optional[bool] = None,
                 graph_cells: Optional[bool] = None) -> Dict[str, Any]:
        """Build the PipelineStage for ``balance``, warm up, time ``steps`` SGD steps."""
        from torchgpipe_amd.parallel import PipelineStage
        from torchgpipe_amd.parallel.stage import signature_of
        args = self.args
        batch, chunks = exp['batch'], exp['chunks']
        unet = kind == 'unet'
        # Intra-rank stream concurrency: U-Net alternates forward micro-batches between two
        # lanes and recomputes the next micro-batch beside the current backward; AmoebaNet
        # runs each cell's independent branches on two streams (its recompute lane cost 19 %
        # on one GPU: profiles/r2/bench_amoeba_s13.md).  Multi-rank runs keep them: sends
        # leave from the lane that computed them and backward passes are ordered across
        # lanes (parallel/stage.py), parity-tested on shared-GPU gloo rehearsals.
        # (ResNet-101 p1: 1459 vs 1411 samples/s with the recompute lane,
        # profiles/r4/resnet_p1_engine.md)
        # ResNet-101: lanes at pipeline-1 (110-image micro-batches: 1741-1754 -> 1781-1785
        # samples/s), none at N > 1, where its 15-36-image stages are host-bound and the
        # lanes' extra host work costs the bottleneck stage 2-5 % (p4 stage 3 1656 vs 1745 ms,
        # p8 stage 7 833 vs 850; profiles/r6/resnet_lanes/)
        lanes = self.gpu and (kind == 'unet' or (kind == 'resnet' and self.world == 1))
        overlap = choice(args.overlap_recompute, lanes)
        overlap_fwd = choice(args.overlap_forward, lanes)
        cell_streams = kind == 'amoebanet' and choice(args.cell_streams, self.gpu)
        # captured cells (parallel/segments.py): one GPU, AmoebaNet -- three-stream cells in
        # per-pass captures, 392.0 vs 389.4 samples/s for the two-stream whole-step graph
        # (profiles/r4/amoeba_n1_graph_modes.md).  Multi-rank runs stay eager by default: in
        # one-GPU stage emulation the captured stages ran within 0-2.5 % of the eager ones
        # (U-Net p8 stages 134.3 / 267.3 / 191.6 vs 133.8 / 268.6 / 194.2 ms, AmoebaNet
        # n8m32 stage 6 494.1 vs 506.6 ms: profiles/r4/stage_harness_*_ref_{eager,
        # graph_cells}.jsonl), which does not pay for running RCCL receives into captured
        # graphs' buffers before any multi-GPU node has (--graph-cells on to opt in).
        if graph_cells is None:
            graph_cells = choice(args.graph_cells, self.world == 1 and kind == 'amoebanet')
        graph_cells = graph_cells and self.gpu
        # multi-path transfers (parallel/stripes.py): U-Net p8's 226 MB skip and AmoebaNet
        # n8's 321 MB boundary outrun one xGMI link (profiles/r5/speedup_prediction.md);
        # opt-in (the 'striped' section times them at N >= 3) until a multi-GPU node has
        # run their RCCL relay chains
        if stripes is None:
            stripes = choice(args.stripes, False)
        stage = PipelineStage(self.build(kind), balance, device=self.device, chunks=chunks,
                              checkpoint=checkpoint, timeout=args.timeout,
                              overlap_recompute=overlap, overlap_forward=overlap_fwd,
                              graph_cells=graph_cells,
                              stripes=max(1, int(args.stripe_mb * 1e6)) if stripes else None)
        if args.channels_last and not unet:
            stage.partition.to(memory_format=torch.channels_last)
        if cell_streams:
            from torchgpipe_amd.models.amoebanet import DEFAULT_CELL_STREAMS, set_cell_streams
            set_cell_streams(stage.partition, True)
            cell_streams = DEFAULT_CELL_STREAMS  # streams per cell (TGPIPE_CELL_STREAMS)
        # (a partition may hold no parameters at all -- pooling-only stages of a small model
        # split eight ways -- and SGD refuses an empty list: nothing to update there)
        params = list(stage.parameters())
        optimizer = torch.optim.SGD(params, lr=0.1) if params else None
        x, target, loss_fn, shape = self.data(kind, batch, stage.is_first, stage.is_last)
        signature = signature_of(torch.empty(batch, *shape, device='meta'))

        def step() -> None:
            stage.train_step(x, target, loss_fn, signature=signature)
            if optimizer is not None:
                optimizer.step()
                optimizer.zero_grad(set_to_none=True)

        if self.gpu:
            torch.cuda.reset_peak_memory_stats(self.device)
        settle = None
        if graph_cells:
            settle = lambda: stage._segments is not None and stage._segments.captured  # noqa: E731
        elif stripes:  # the step that plans the stripes (and opens relay links) is untimed
            settle = lambda: stage.stripes_ready  # noqa: E731
        res: Dict[str, Any] = self.timed(step, steps, args.warmup, tag, settle=settle)
        res.update(batch=batch, chunks=chunks, balance=list(balance), checkpoint=checkpoint,
                   steps=steps, overlap_recompute=overlap, cell_streams=int(cell_streams),
                   overlap_forward=overlap_fwd, graph_cells=graph_cells,
                   striped_routes=stage.striped_routes)
        if probe:
            # one untimed diagnostic step: per-rank receive waits and busy time
            mine = stage.probe_step(step)
            mine['rank'] = self.rank
            gathered: List[Any] = [None] * self.world
            if self.world > 1:
                dist.all_gather_object(gathered, mine, group=self.ctrl)
            else:
                gathered = [mine]
            res['per_rank'] = gathered
        if args.profile_steps and self.rank == 0 and tag == 'headline':
            from torch.profiler import ProfilerActivity, profile
            acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if self.gpu else [])
            with profile(activities=acts) as prof:
                for _ in range(args.profile_steps):
                    step()
                self.sync()
            print(prof.key_averages().table(
                sort_by='cuda_time_total' if self.gpu else 'cpu_time_total', row_limit=30),
                file=sys.stderr)
        res['mem'] = torch.cuda.max_memory_allocated(self.device) / 2 ** 30 if self.gpu else 0.0
        del stage, optimizer, x, target, step, settle
        self.release()
        return res

    def gpipe_api(self, exp: Dict[str, Any], balance: List[int], checkpoint: str,
                  steps: int) -> Dict[str, Any]:
        """The U-Net experiment through the public single-process ``GPipe`` API on this
        rank's GPU (the reference's speed benchmark path, ``benchmarks/unet-speed/main.py:
        37-67``): ``model(x)``, the loss on the gathered output, ``loss.backward()``, SGD."""
        from torchgpipe_amd import GPipe
        batch, chunks = exp['batch'], exp['chunks']
        # the headline's forward lanes where the headline has them (--overlap-forward)
        lanes = choice(self.args.overlap_forward, self.gpu)
        model = GPipe(self.build('unet'), balance=balance, devices=[self.device] * len(balance),
                      chunks=chunks, checkpoint=checkpoint, overlap_forward=lanes)
        optimizer = torch.optim.SGD(model.parameters(), lr=0.1)
        x, target, loss_fn, _ = self.data('unet', batch, True, True)

        def step() -> None:
            loss = loss_fn(model(x), target)
            loss.backward()
            optimizer.step()
            optimizer.zero_grad(set_to_none=True)

        world, self.world = self.world, 1  # one process drives it: no collective
        try:
            res: Dict[str, Any] = self.timed(step, steps, self.args.warmup, 'gpipe')
        finally:
            self.world = world
        res.update(batch=batch, chunks=chunks, balance=list(balance), checkpoint=checkpoint,
                   steps=steps, overlap_forward=lanes)
        model._workers.close()  # (its device thread, before the next section's stage)
        from torchgpipe_amd.ops.conv import clear_winograd_caches
        clear_winograd_caches(model)
        del model, optimizer, x, target, step
        self.release()
        return res

    def release(self) -> None:
        """Free what a finished timing held before the next one is built: autograd graphs
        and captured graphs in reference cycles, and with them their Winograd transform
        caches, which would otherwise still count against the next stage's cache budget."""
        gc.collect()
        if self.gpu:
            from torchgpipe_amd.ops.conv import cache_bytes
            torch.cuda.synchronize(self.device)
            torch.cuda.empty_cache()
            held = cache_bytes()
            if held:
                self.log(f'{held / 2 ** 20:.0f} MiB of transform caches still held')

    def plain(self, kind: str, batch: int, steps: int, tag: str) -> Optional[Dict[str, Any]]:
        """The model without GPipe (no micro-batches, no checkpointing) on rank 0's GPU,
        SGD like the pipelines: the reference's ``baseline`` experiment.  Other ranks wait."""
        res = None
        self.ctrl_barrier()
        if self.rank == 0:
            from torchgpipe_amd.ops.conv import new_step
            model = self.build(kind, meta=False)
            optimizer = torch.optim.SGD(model.parameters(), lr=0.1)
            x, target, loss_fn, _ = self.data(kind, batch, True, True)

            def step() -> None:
                new_step()
                loss = loss_fn(model(x), target)
                loss.backward()
                optimizer.step()
                optimizer.zero_grad(set_to_none=True)

            world, self.world = self.world, 1  # rank 0 alone: no collective in its timing
            try:
                res = self.timed(step, steps, self.args.warmup, tag)
            finally:
                self.world = world
            res.update(batch=batch, steps=steps)
            del model, optimizer, x, target, step
            self.release()
        self.ctrl_barrier()
        return res


def summary(res: Dict[str, Any], ref: Optional[float]) -> Dict[str, Any]:
    value = res['batch'] * res['steps'] / res['elapsed']
    out = {'value': round(value, 3), 'ms_per_step': round(1000 * res['elapsed'] / res['steps'], 3),
           'steps': res['steps'], 'batch': res['batch']}
    if 'chunks' in res:
        out.update(chunks=res['chunks'], balance=res['balance'], checkpoint=res['checkpoint'])
    out['vs_p40'] = round(value / ref, 3) if ref else None
    return out


def main() -> None:
    args = parse()
    # stdout carries the JSON lines (rank 0).  Libraries print to fd 1 from native code
    # (gloo's "[Gloo] Rank r is connected to ..." banner, RCCL info): point fd 1 at stderr
    # for the whole run and keep a private handle on the real stdout for the result.
    sys.stdout.flush()
    result_out = os.fdopen(os.dup(1), 'w')
    os.dup2(2, 1)
    b = Bench(args)
    world = b.world

    kind = args.model
    n_layers = len(b.build(kind))
    table = UNET_EXPERIMENTS if kind == 'unet' else AMOEBA_EXPERIMENTS
    if kind == 'unet':
        exp = dict(table.get(world) or dict(name=f'pipeline-{world}', batch=80 * world,
                                            chunks=4 * world,
                                            balance=even_balance(n_layers, world), ref=None))
        checkpoint = 'except_last'
        model_name = 'U-Net(5,64)'
        in_shape = '3x192x192'
    elif kind == 'resnet':
        exp = dict(RESNET_EXPERIMENTS.get(world) or dict(
            name=f'pipeline-{world}', batch=240 * world, chunks=32,
            balance=even_balance(n_layers, world), checkpoint='always', ref=None))
        checkpoint = exp['checkpoint']
        model_name = 'ResNet-101'
        in_shape = '3x224x224'
    else:
        exp = dict(table.get(world) or dict(name=f'n{world}m32', batch=160 * world, chunks=32,
                                            balance=even_balance(n_layers, world), ref=None))
        checkpoint = 'except_last' if exp['chunks'] > 1 else 'always'
        model_name = 'AmoebaNet-D(18,256)'
        in_shape = '3x224x224'
    if args.tiny:
        exp['balance'] = exp['tuned'] = even_balance(n_layers, world)
        if kind == 'resnet':
            exp.update(batch=4, chunks=2)
    if args.checkpoint:
        checkpoint = args.checkpoint
    if args.batch:
        exp['batch'] = args.batch
    if args.chunks:
        exp['chunks'] = args.chunks
    tuned_balance = list(exp.get('tuned', exp['balance']))
    if args.balance == 'tuned':
        exp['balance'] = tuned_balance
    elif args.balance != 'ref':
        exp['balance'] = [int(v) for v in args.balance.split(',')]
    batch, chunks, balance = exp['batch'], exp['chunks'], list(exp['balance'])
    probe = choice(args.probe, world > 1)

    # wall seconds of every timed section (warm-up, capture and diagnostics included), so a
    # multi-GPU run's budget can be checked section by section
    section_s: Dict[str, float] = {}
    t_sec = time.time()

    def lap(name: str) -> None:
        nonlocal t_sec
        section_s[name] = round(time.time() - t_sec, 1)
        b.log(f'section {name}: {section_s[name]} s')
        t_sec = time.time()

    record: Dict[str, Any] = {}

    def emit() -> None:
        """Rank 0 prints the record as it stands: right after the headline, then again,
        augmented, after every section -- a later section that fails or hangs cannot take
        the lines already printed with it.  Each line is a complete record; the last one
        printed is the most complete."""
        if b.rank == 0:
            record['section_s'] = dict(section_s)
            print(json.dumps(record), file=result_out, flush=True)

    # 1. the headline: the reference balance on the plain eager engine (no multi-path
    #    transfers, no captured cells at N > 1 -- those have their own sections below)
    main_run = b.pipeline(kind, exp, balance, checkpoint, args.steps, 'headline', probe=probe)
    lap('headline')
    elapsed = main_run['elapsed']
    samples_per_s = batch * args.steps / elapsed
    ref = None if args.tiny else exp.get('ref')
    if args.tiny:
        model_name += ' TINY smoke-test variant (not a measurement)'
    record.update({
        'metric': f'{model_name} GPipe training throughput (samples/sec)',
        'value': round(samples_per_s, 3),
        'unit': 'samples/sec',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(1000 * elapsed / args.steps, 3),
        'higher_is_better': True,
        'scaling': 'strong',
        'vs_baseline': round(samples_per_s / ref, 3) if ref else None,
        'dtype': 'fp32',
        'data': 'synthetic (torch.rand inputs, constant targets), random-init weights',
        'config': {
            'model': model_name,
            'experiment': exp['name'],
            'global_batch': batch,
            'seq_len': None,
            'input': in_shape,
            'chunks': chunks,
            'balance': balance,
            'balance_source': args.balance,
            'checkpoint': checkpoint,
            'parallelism': f'pp{world}',
            'transport': 'gloo-host-staged (rehearsal)' if b.rehearsal else
                         ('rccl' if b.gpu and world > 1 else 'none'),
            'fused_cells': kind == 'unet' and not args.unfused,
            'baseline_samples_per_sec_p40': ref,
            'rank0_peak_mem_gib': round(main_run['mem'], 2),
            'warmup_s': round(main_run['warm_s'], 1),
            'first_step_s': round(main_run['first_step_s'], 2),
            'timeout_s': args.timeout,
            'cell_streams': main_run['cell_streams'],
            'overlap_recompute': main_run['overlap_recompute'],
            'overlap_forward': main_run['overlap_forward'],
            'graph_cells': main_run['graph_cells'],
            'striped_routes': main_run['striped_routes'],
            'hw_queues': os.environ.get('GPU_MAX_HW_QUEUES'),
        },
        'tuned': None,
    })
    if 'per_rank' in main_run:
        record['per_rank'] = main_run['per_rank']
    emit()

    if args.sections == 'auto':
        sections = set()
        if kind == 'unet':
            sections = {'baseline', 'amoebanet'}
            if world in RESNET_EXPERIMENTS:
                sections.add('resnet')
            if world == 1:
                sections.add('gpipe')
            if world >= 3:
                sections.add('striped')
            if world > 1:
                sections.add('graph_cells')
    elif args.sections == 'none':
        sections = set()
    else:
        sections = set(args.sections.split(','))
    sec_steps = args.section_steps or args.steps
    # the opt-in engine variants at N > 1 (striped transfers, captured cells, tuned
    # balances): fewer timed steps, they are comparisons against the sections above
    extra_steps = min(sec_steps, 10)

    if 'baseline' in sections and kind == 'unet':
        bl = b.plain('unet', 4 if args.tiny else UNET_BASELINE['batch'], sec_steps, 'baseline')
        if bl is not None:
            baseline = summary(bl, None if args.tiny else UNET_BASELINE['ref'])
            baseline['experiment'] = 'baseline (no GPipe, rank 0 GPU)'
            # same-box speed-up over the reference's own denominator (no GPipe, B=40)
            record['baseline_samples_per_sec'] = baseline['value']
            record['speedup_vs_baseline'] = round(samples_per_s / baseline['value'], 3)
            record['baseline'] = baseline
        lap('baseline')
        emit()

    if 'gpipe' in sections and kind == 'unet' and world == 1:
        # the reference's own API on its own benchmark path: single-process GPipe
        gr = b.gpipe_api(exp, balance, checkpoint, sec_steps)
        g = summary(gr, None if args.tiny else exp.get('ref'))
        g['experiment'] = (f"{exp['name']} through GPipe(balance={balance}, chunks={chunks}, "
                           f"overlap_forward={gr['overlap_forward']})")
        g['vs_pipeline_stage'] = round(g['value'] / samples_per_s, 3)
        record['gpipe'] = g
        lap('gpipe')
        emit()

    a_layers = None
    aexp: Dict[str, Any] = {}
    if ('amoebanet' in sections or 'graph_cells' in sections) and kind == 'unet':
        a_layers = len(b.build('amoebanet'))
        aexp = dict(AMOEBA_EXPERIMENTS.get(world) or dict(
            name=f'n{world}m32', batch=160 * world, chunks=32,
            balance=even_balance(a_layers, world), ref=None))
        if args.tiny:
            aexp.update(batch=4, chunks=2, balance=even_balance(a_layers, world))
    a_ckpt = 'except_last' if aexp.get('chunks', 2) > 1 else 'always'

    if 'amoebanet' in sections and kind == 'unet':
        assert a_layers is not None
        ar = b.pipeline('amoebanet', aexp, aexp['balance'], a_ckpt, sec_steps, 'amoebanet')
        amoeba = summary(ar, None if args.tiny else aexp['ref'])
        amoeba['experiment'] = aexp['name']
        amoeba['cell_streams'] = ar['cell_streams']
        amoeba['graph_cells'] = ar['graph_cells']
        amoeba['striped_routes'] = ar['striped_routes']
        record['amoebanet'] = amoeba
        if world == 2:
            d = dict(AMOEBA_N2M1)
            if args.tiny:
                d.update(batch=4, balance=even_balance(a_layers, 2))
            dr = b.pipeline('amoebanet', d, d['balance'], 'always', sec_steps, 'amoebanet-n2m1')
            amoeba['n2m1'] = summary(dr, None if args.tiny else d['ref'])
            amoeba['speedup_vs_n2m1'] = round(amoeba['value'] / amoeba['n2m1']['value'], 3)
        lap('amoebanet')
        emit()

    if 'resnet' in sections and kind == 'unet' and world in RESNET_EXPERIMENTS:
        rexp = dict(RESNET_EXPERIMENTS[world])
        if args.tiny:
            r_layers = len(b.build('resnet'))
            rexp.update(batch=4, chunks=2, balance=even_balance(r_layers, world))
        rr = b.pipeline('resnet', rexp, rexp['balance'], rexp['checkpoint'], sec_steps, 'resnet')
        resnet = summary(rr, None if args.tiny else rexp['ref'])
        resnet['experiment'] = rexp['name']
        resnet['graph_cells'] = rr['graph_cells']
        resnet['striped_routes'] = rr['striped_routes']
        record['resnet101'] = resnet
        rb = b.plain('resnet', 4 if args.tiny else RESNET_BASELINE['batch'], sec_steps,
                     'resnet-baseline')
        if rb is not None:
            resnet['baseline'] = summary(rb, None if args.tiny else RESNET_BASELINE['ref'])
            resnet['speedup_vs_baseline'] = round(resnet['value'] / resnet['baseline']['value'],
                                                  3)
        lap('resnet')
        emit()

    # The opt-in engine variants (tuned balances, multi-path transfers, captured cells) come
    # last.  At N > 1 a variant that raises on every rank (a planner error, a PipelineTimeout
    # of its own transfers) is recorded under its key and ends the optional sections; the
    # lines already printed keep the headline and the sections before it.
    failed: List[str] = []

    def optional(name: str, fn: Callable[[], None]) -> None:
        if failed:
            return
        if world == 1:
            fn()
            return
        try:
            if os.environ.get('TGPIPE_BENCH_FAIL') == name:  # (tests/test_bench_script.py)
                raise RuntimeError(f'{name}: failure injected by TGPIPE_BENCH_FAIL')
            fn()
        except Exception as e:  # noqa: BLE001 - recorded, then the run winds down
            import traceback
            traceback.print_exc()
            failed.append(name)
            record[name] = {'error': f'{type(e).__name__}: {e}'[:500]}
            lap(name)
            emit()

    also = args.also_tuned == 'yes' or (args.also_tuned == 'auto' and world > 1
                                         and args.balance == 'ref' and tuned_balance != balance)

    def tuned_section() -> None:
        t = b.pipeline(kind, exp, tuned_balance, checkpoint, extra_steps, 'tuned')
        record['tuned'] = {'balance': tuned_balance,
                           'value': round(batch * extra_steps / t['elapsed'], 3),
                           'ms_per_step': round(1000 * t['elapsed'] / extra_steps, 3),
                           'steps': extra_steps}
        if 'amoebanet' in record and world > 1 and not args.tiny:
            a_tuned = list(aexp.get('tuned', aexp['balance']))
            if a_tuned != list(aexp['balance']):
                # the MI355X-searched balance too (AMOEBA_EXPERIMENTS 'tuned')
                at = b.pipeline('amoebanet', aexp, a_tuned, a_ckpt, extra_steps,
                                'amoebanet-tuned')
                record['amoebanet']['tuned'] = {
                    'balance': a_tuned,
                    'value': round(aexp['batch'] * extra_steps / at['elapsed'], 3),
                    'ms_per_step': round(1000 * at['elapsed'] / extra_steps, 3),
                    'steps': extra_steps}
        lap('tuned')
        emit()

    def striped_section() -> None:
        # multi-path transfers (parallel/stripes.py) on the headline configuration: opt-in
        # until a multi-GPU node has run their RCCL relay chains
        sr = b.pipeline(kind, exp, balance, checkpoint, extra_steps, 'striped', stripes=True)
        st = summary(sr, None if args.tiny else exp.get('ref'))
        st['striped_routes'] = sr['striped_routes']
        st['stripe_mb'] = args.stripe_mb
        record['striped'] = st
        lap('striped')
        emit()

    def graph_cells_section() -> None:
        # captured cells at N > 1 (parallel/segments.py: RCCL receives into the captured
        # graphs' persistent buffers) on the AmoebaNet experiment, opt-in like the stripes
        gc_run = b.pipeline('amoebanet', aexp, aexp['balance'], a_ckpt, extra_steps,
                            'amoebanet-graph-cells', graph_cells=True)
        gcs = summary(gc_run, None if args.tiny else aexp['ref'])
        gcs['experiment'] = aexp['name']
        gcs['graph_cells'] = gc_run['graph_cells']
        record['amoebanet_graph_cells'] = gcs
        lap('graph_cells')
        emit()

    if also:
        optional('tuned', tuned_section)
    if 'striped' in sections and world >= 3:
        optional('striped', striped_section)
    if 'graph_cells' in sections and kind == 'unet' and world > 1:
        optional('amoebanet_graph_cells', graph_cells_section)

    if world > 1:
        if failed:
            # the communicators may be mid-exchange: no barrier, no orderly teardown
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(0)
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
