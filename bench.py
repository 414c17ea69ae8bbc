#!/usr/bin/env python
"""Headline benchmark: U-Net(5,64) (or AmoebaNet-D(18,256)) GPipe training throughput.

Metric (BASELINE.json): samples/sec of a full SGD training step (forward,
backward with checkpoint recomputation, optimizer step) of U-Net(5,64) on
3×192×192 synthetic images at 1/2/4/8 pipeline partitions, using the
reference's experiment tables (``benchmarks/unet-speed/main.py:23-68``):

    N=1  pipeline-1  B=80,  chunks=2,  balance [241]
    N=2  pipeline-2  B=512, chunks=32, balance [104, 137]
    N=4  pipeline-4  B=512, chunks=16, balance [30, 66, 84, 61]
    N=8  pipeline-8  B=640, chunks=40, balance [16, 27, 31, 44, 22, 57, 27, 17]

One process per GPU (``torch.distributed.run``), RCCL point-to-point between
stages; fp32 like the reference.  Rank 0 prints one JSON line.

    python bench.py --gpus 1 --steps 5 --warmup 2
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        bench.py --gpus 8
"""
import argparse
import datetime
import json
import os
import sys
import time

if int(os.environ.get('WORLD_SIZE', '1')) > 1:
    # One HIP hardware queue per stream: a rank runs its compute stream plus one RCCL
    # stream per pipeline link (up to 6 on U-Net p8 with long skips).  With HIP's
    # default of 4 queues, streams beyond that share a queue and their kernels
    # serialise, so a spinning RCCL receive could hold up unrelated work.  Set before
    # the HIP runtime initialises (first CUDA call).
    os.environ.setdefault('GPU_MAX_HW_QUEUES', '8')

import torch
import torch.distributed as dist
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

# Reference (Tesla P40) throughputs of the same experiments, BASELINE.md §1/§2.
# Batch / chunks / reference balance are the reference's experiment tables.
# ``tuned`` balances were re-derived for MI355X with the Winograd F(4x4) MFMA kernels
# (fused and non-fused): candidates from the per-layer device times
# (profiles/unet_layer_profile_m1.json, benchmarks/layer_profile.py), then rounds of
# benchmarks/stage_harness.py measurements fed back through
# scripts/balance_from_harness.py (profiles/stage_harness_nf_p{2,4,8}.json): measured max
# stage p8 206 ms, p4 283 ms, p2 643 ms (the reference's P40 balances measured a 613 ms
# max stage at p8 with the earlier kernels).
UNET_EXPERIMENTS = {
    1: dict(name='pipeline-1', batch=80, chunks=2, balance=[241], tuned=[241], ref=24.456),
    2: dict(name='pipeline-2', batch=512, chunks=32, balance=[104, 137], tuned=[102, 139],
            ref=35.502),
    4: dict(name='pipeline-4', batch=512, chunks=16, balance=[30, 66, 84, 61],
            tuned=[45, 55, 59, 82], ref=67.042),
    8: dict(name='pipeline-8', batch=640, chunks=40, balance=[16, 27, 31, 44, 22, 57, 27, 17],
            tuned=[22, 23, 26, 30, 22, 37, 43, 38], ref=88.497),
}
# AmoebaNet tuned balances: profiles/amoebanet_layer_profile.json (micro-batch 40) through
# the same simulator (n2 535 vs 492, n4 851 vs 814, n8 1539 vs 1503 simulated samples/s).
AMOEBA_EXPERIMENTS = {
    1: dict(name='n1m32', batch=640, chunks=32, balance=[24], tuned=[24], ref=None),
    2: dict(name='n2m32', batch=1280, chunks=32, balance=[9, 15], tuned=[10, 14], ref=47.386),
    4: dict(name='n4m32', batch=1152, chunks=32, balance=[3, 6, 7, 8], tuned=[5, 5, 6, 8],
            ref=72.412),
    8: dict(name='n8m32', batch=1280, chunks=32, balance=[2, 2, 2, 3, 3, 4, 4, 4],
            tuned=[2, 2, 3, 3, 3, 3, 4, 4], ref=132.413),
}


def parse() -> argparse.Namespace:
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawTextHelpFormatter)
    p.add_argument('--gpus', type=int, default=int(os.environ.get('WORLD_SIZE', '1')))
    p.add_argument('--steps', type=int, default=5)
    p.add_argument('--warmup', type=int, default=2)
    p.add_argument('--model', choices=['unet', 'amoebanet'], default='unet')
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
    p.add_argument('--timeout', type=float, default=300.0,
                   help='seconds any pipeline wait may take before the run fails (RCCL '
                        'watchdog and gloo waits): a dead or stuck rank ends the job')
    p.add_argument('--cudnn-benchmark', action='store_true',
                   help='MIOpen exhaustive find (slow first step, cached afterwards)')
    p.add_argument('--backend', choices=['auto', 'gloo'], default='auto',
                   help="tensor transport: 'auto' = RCCL on GPUs (gloo on CPU); 'gloo' stages "
                        "messages through host memory and lets several ranks share one GPU "
                        "(functional rehearsal only, not a valid measurement)")
    p.add_argument('--tiny', action='store_true',
                   help='tiny model of the same family (CI smoke test of this script only)')
    p.add_argument('--channels-last', action='store_true',
                   help='NHWC activations and weights (MIOpen NHWC kernels; AmoebaNet)')
    p.add_argument('--graph', action='store_true',
                   help='one-GPU runs: capture the whole step (forward, backward, SGD) into a '
                        'hipGraph after the warm-up and replay it (RNG-free models only: '
                        'AmoebaNet; parallel/graph.py)')
    p.add_argument('--cell-streams', choices=['auto', 'on', 'off'], default='auto',
                   help="AmoebaNet: run each cell's independent nodes on two HIP streams "
                        '(auto: on for one-GPU runs)')
    p.add_argument('--overlap-recompute', choices=['auto', 'on', 'off'], default='auto',
                   help="recompute the next micro-batch on a second stream during this one's "
                        'backward (PipelineStage(overlap_recompute=True); auto: on for '
                        'one-GPU U-Net runs)')
    p.add_argument('--overlap-forward', choices=['auto', 'on', 'off'], default='auto',
                   help='alternate the forward micro-batches of a one-rank stateless partition '
                        '(no running statistics: U-Net) between two streams (auto: on for '
                        'one-GPU U-Net runs)')
    p.add_argument('--wgrad-stream', choices=['auto', 'on', 'off'], default='auto',
                   help='run the fused ops\' weight-gradient GEMMs on a side stream '
                        '(PipelineStage(wgrad_stream=True); auto: off)')
    p.add_argument('--profile-steps', type=int, default=0,
                   help='after timing, run N more steps under torch.profiler (rank 0)')
    return p.parse_args()


def even_balance(layers: int, parts: int) -> list:
    base, extra = divmod(layers, parts)
    return [base + (1 if i < extra else 0) for i in range(parts)]


def main() -> None:
    args = parse()
    # stdout carries exactly one JSON line (rank 0).  Libraries print to fd 1
    # from native code (gloo's "[Gloo] Rank r is connected to ..." banner, RCCL
    # info): point fd 1 at stderr for the whole run and keep a private handle
    # on the real stdout for the result.
    sys.stdout.flush()
    result_out = os.fdopen(os.dup(1), 'w')
    os.dup2(2, 1)
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        raise SystemExit(f'--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU')

    gpu = torch.cuda.is_available()
    rehearsal = args.backend == 'gloo' and gpu and world > 1
    if gpu and not rehearsal and local_rank >= torch.cuda.device_count():
        raise SystemExit(f'LOCAL_RANK {local_rank} but only {torch.cuda.device_count()} GPUs')
    device = (torch.device('cuda', local_rank % torch.cuda.device_count()) if gpu
              else torch.device('cpu'))
    if gpu:
        torch.cuda.set_device(device)
        torch.backends.cudnn.benchmark = args.cudnn_benchmark
    if world > 1:
        # Lazy RCCL init: each pipeline link (peer pair) then gets its own
        # communicator and stream on first use.
        backend = 'nccl' if gpu and not rehearsal else 'gloo'
        dist.init_process_group(backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=args.timeout))

    from torchgpipe_amd.models import amoebanetd, unet
    from torchgpipe_amd.parallel import PipelineStage

    table = UNET_EXPERIMENTS if args.model == 'unet' else AMOEBA_EXPERIMENTS

    def build_model() -> torch.nn.Sequential:
        # Built on the meta device: each rank materialises (random-initialises) only
        # its own partition inside PipelineStage.
        with torch.device('meta'):
            if args.model == 'unet':
                if args.tiny:
                    return unet(depth=2, num_convs=1, base_channels=4, input_channels=3,
                                output_channels=1, fused=not args.unfused)
                return unet(depth=5, num_convs=5, base_channels=64, input_channels=3,
                            output_channels=1, fused=not args.unfused)
            if args.tiny:
                return amoebanetd(num_classes=10, num_layers=3, num_filters=8)
            return amoebanetd(num_classes=1000, num_layers=18, num_filters=256)

    n_layers = len(build_model())
    if args.model == 'unet':
        exp = dict(table.get(world) or dict(name=f'pipeline-{world}', batch=80 * world,
                                            chunks=4 * world,
                                            balance=even_balance(n_layers, world), ref=None))
        in_shape = (3, 192, 192)
        checkpoint = 'except_last'
        model_name = 'U-Net(5,64)'
    else:
        exp = dict(table.get(world) or dict(name=f'n{world}m32', batch=160 * world, chunks=32,
                                            balance=even_balance(n_layers, world), ref=None))
        in_shape = (3, 224, 224)
        checkpoint = 'except_last' if exp['chunks'] > 1 else 'always'
        model_name = 'AmoebaNet-D(18,256)'
    if args.tiny:
        exp['balance'] = exp['tuned'] = even_balance(n_layers, world)
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
    # Intra-rank stream concurrency (measured on one GPU; multi-rank runs keep the
    # one-stream schedule that the RCCL rehearsals exercised)
    # (auto: U-Net only -- AmoebaNet's two-stream cells already fill the CUs, and the extra
    # recompute lane cost it 19 %: profiles/r2/bench_amoeba_s13.md)
    overlap = {'on': True, 'off': False}.get(args.overlap_recompute,
                                             world == 1 and gpu and args.model == 'unet')
    cell_streams = args.model == 'amoebanet' and {'on': True, 'off': False}.get(
        args.cell_streams, world == 1 and gpu)
    # (auto: off -- with the two-stream cells it measured 280.3 vs 328.6 samples/s on one box,
    # profiles/r2/bench_amoeba_s13.md)
    wgrad_stream = {'on': True, 'off': False}.get(args.wgrad_stream, False)
    overlap_fwd = {'on': True, 'off': False}.get(args.overlap_forward,
                                                 world == 1 and gpu and args.model == 'unet')

    def sync() -> None:
        if world > 1:
            dist.barrier()
        if gpu:
            torch.cuda.synchronize(device)

    def measure(balance: list, tag: str) -> dict:
        """Build the stage for ``balance``, warm up, time ``--steps`` full SGD steps."""
        stage = PipelineStage(build_model(), balance, device=device, chunks=chunks,
                              checkpoint=checkpoint, timeout=args.timeout,
                              overlap_recompute=overlap, overlap_forward=overlap_fwd,
                              wgrad_stream=wgrad_stream)
        if args.channels_last:
            stage.partition.to(memory_format=torch.channels_last)
        if cell_streams:
            from torchgpipe_amd.models.amoebanet import set_cell_streams
            set_cell_streams(stage.partition, True)
        optimizer = torch.optim.SGD(stage.parameters(), lr=0.1)

        gen = torch.Generator(device=device).manual_seed(0)
        x = torch.rand(batch, *in_shape, device=device, generator=gen) if stage.is_first else None
        if x is not None and args.channels_last:
            x = x.contiguous(memory_format=torch.channels_last)
        if args.model == 'unet':
            target = torch.ones(batch, 1, 192, 192, device=device) if stage.is_last else None
            loss_fn = F.binary_cross_entropy_with_logits
        else:
            target = (torch.randint(10 if args.tiny else 1000, (batch,), device=device,
                                    generator=gen) if stage.is_last else None)
            loss_fn = F.cross_entropy
        from torchgpipe_amd.parallel.stage import signature_of
        signature = signature_of(torch.empty(batch, *in_shape, device='meta'))

        graph = None
        if args.graph:
            if world != 1:
                raise SystemExit('--graph captures one-rank runs only')
            from torchgpipe_amd.parallel import StepGraph
            graph = StepGraph(stage, loss_fn, optimizer, warmup=max(1, args.warmup - 1))

        def step() -> None:
            if graph is not None:
                graph.step(x, target)  # type: ignore[arg-type]
                return
            stage.train_step(x, target, loss_fn, signature=signature)
            optimizer.step()
            optimizer.zero_grad(set_to_none=True)

        if gpu:
            torch.cuda.reset_peak_memory_stats(device)
        t0 = time.time()
        first_s = 0.0
        for k in range(args.warmup):
            step()
            sync()
            if k == 0:
                first_s = time.time() - t0
            if rank == 0:
                print(f'[bench] {tag} warmup step {k + 1}/{args.warmup} done at '
                      f'{time.time() - t0:.1f}s', file=sys.stderr, flush=True)
        while graph is not None and not graph.captured:  # the capture stays untimed
            step()
            sync()
        warm_s = time.time() - t0

        sync()
        start = time.perf_counter()
        for _ in range(args.steps):
            step()
        sync()
        elapsed = time.perf_counter() - start

        if world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())

        if args.profile_steps and rank == 0 and tag == 'headline':
            from torch.profiler import ProfilerActivity, profile
            acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if gpu else [])
            with profile(activities=acts) as prof:
                for _ in range(args.profile_steps):
                    step()
                sync()
            print(prof.key_averages().table(
                sort_by='cuda_time_total' if gpu else 'cpu_time_total', row_limit=30),
                file=sys.stderr)
        mem = torch.cuda.max_memory_allocated(device) / 2 ** 30 if gpu else 0.0
        del stage, optimizer, x, target
        if gpu:
            torch.cuda.empty_cache()
        return {'elapsed': elapsed, 'warm_s': warm_s, 'first_step_s': first_s, 'mem': mem}

    main_run = measure(balance, 'headline')
    elapsed, warm_s = main_run['elapsed'], main_run['warm_s']
    tuned = None
    also = args.also_tuned == 'yes' or (args.also_tuned == 'auto' and world > 1
                                         and args.balance == 'ref' and tuned_balance != balance)
    if also:
        t = measure(tuned_balance, 'tuned')
        tuned = {'balance': tuned_balance,
                 'value': round(batch * args.steps / t['elapsed'], 3),
                 'ms_per_step': round(1000 * t['elapsed'] / args.steps, 3)}

    samples_per_s = batch * args.steps / elapsed
    if rank == 0:
        ref = None if args.tiny else exp.get('ref')
        if args.tiny:
            model_name += ' TINY smoke-test variant (not a measurement)'
        mem = main_run['mem']
        print(json.dumps({
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
                'input': 'x'.join(map(str, in_shape)),
                'chunks': chunks,
                'balance': balance,
                'balance_source': args.balance,
                'checkpoint': checkpoint,
                'parallelism': f'pp{world}',
                'transport': 'gloo-host-staged (rehearsal)' if rehearsal else
                             ('rccl' if gpu and world > 1 else 'none'),
                'fused_cells': args.model == 'unet' and not args.unfused,
                'baseline_samples_per_sec_p40': ref,
                'rank0_peak_mem_gib': round(mem, 2),
                'warmup_s': round(warm_s, 1),
                'first_step_s': round(main_run['first_step_s'], 2),
                'timeout_s': args.timeout,
                'hipgraph': bool(args.graph),
                'cell_streams': cell_streams,
                'overlap_recompute': overlap,
                'wgrad_stream': wgrad_stream,
                'overlap_forward': overlap_fwd,
            },
            'tuned': tuned,
        }), file=result_out, flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
