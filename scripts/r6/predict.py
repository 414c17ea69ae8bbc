"""Speed-up predictions from stage-harness runs at attainable xGMI rates (round 6).

Round 5's ``scripts/r5/predict.py`` headlined 100 GB/s per link and direction, above what
one xGMI link moves (~153 GB/s counting both directions, ~77 GB/s per direction at peak;
RCCL point-to-point gets less).  This version:

* simulates at **64 and 50 GB/s per direction** (and free links);
* plans multi-path transfers with the engine's own, now direction-aware, planner
  (``parallel/stripes.py``: a detour may run against the direction of a busy pipeline
  link, since a GPipe step's forward and gradient transfers happen in two phases);
* charges every GPU for the RCCL kernels it runs -- as a sender, a receiver, and a relay
  (twice: in and out) -- as a share of its compute time: the kernel runs for the transfer
  time on ``RCCL_CUS`` of the 256 CUs, and moves its bytes through HBM
  (``HBM_GBPS``), both serialised onto the stage's cells (pessimistic: HBM and CUs are
  not wholly taken);
* prints, per directed link, the bytes per step and the fraction of the step it is busy.

Every stage ran alone on one GPU through the real engine (``benchmarks/stage_harness.py``:
device ms per step and the bytes the stage sends per micro-batch).  The pipeline is
``torchgpipe_amd.balance.simulate.step_time`` with each stage as one pseudo-layer
(forward F, backward 2F per micro-batch, recomputation before the gradient arrives).

    python scripts/r6/predict.py --unet-baseline 753.9 --resnet-baseline 1703.4 \\
        --stripes 16 profiles/r5/harness_final/*.json
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from torchgpipe_amd.balance.simulate import step_time  # noqa: E402
from torchgpipe_amd.parallel import stripes  # noqa: E402

REF = {'unet_p2': 1.246, 'unet_p4': 2.352, 'unet_p8': 3.105,
       'amoeba_n2m32': 1.773, 'amoeba_n4m32': 2.709, 'amoeba_n8m32': 4.953,
       'resnet_p2': 1.414, 'resnet_p4': 2.774, 'resnet_p8': 4.294}
LINKS = (64.0, 50.0)  # GB/s per direction and link, effective
RCCL_CUS = 4          # CUs an RCCL point-to-point kernel occupies while it moves data
HBM_GBPS = 5000.0     # HBM rate of an RCCL kernel's reads / writes
SUB = 4


def load(path):
    with open(path) as f:
        d = json.load(f)
    return d['args'], d['stages']


def routes_of(stages):
    """[(src, dst, kind, bytes per micro-batch)] of the forward messages."""
    out = []
    for j, s in enumerate(stages):
        for key, nbytes in s.get('sent_bytes', {}).items():
            kind, dst = key.split('->')
            out.append((j, int(dst), kind, int(nbytes)))
    return out


def plan_of(stages, min_mb, max_relays=3):
    sends = {j: [] for j in range(len(stages))}
    for src, dst, kind, nbytes in routes_of(stages):
        sends[src].append(stripes.Send(dst, kind, nbytes))
        sends[dst].append(stripes.Send(src, 'g' + kind, nbytes))
    return stripes.plan(sends, list(range(len(stages))), int(min_mb * 1e6), max_relays, SUB)


def rccl_ms(nbytes, gbps, hbm_passes):
    """Stage time an RCCL kernel moving ``nbytes`` costs its GPU (ms)."""
    link = gbps or LINKS[0]
    return nbytes * (RCCL_CUS / 256 / (link * 1e6) + hbm_passes / (HBM_GBPS * 1e6))


def simulate(args, stages, gbps, plan=None, links_out=None):
    n, m = len(stages), args['chunks']
    stop = {'always': m, 'except_last': m - 1, 'never': 0}[args.get('checkpoint',
                                                                  'except_last')]
    fwd = [s['device_ms'] / (3 * m + stop) for s in stages]
    bwd = [2 * f for f in fwd]
    routes, jobs = plan if plan is not None else ({}, {})
    w0 = (SUB + 1) / SUB
    share = {r: w0 / (w0 + len(rl)) for r, rl in routes.items()}
    # RCCL kernels: sender reads, receiver writes (one HBM pass each), relay both (two);
    # forward messages in the forward cells, their gradients in the backward cells
    extra = [0.0] * n
    for src, dst, _, nbytes in routes_of(stages):
        extra[src] += rccl_ms(nbytes, gbps, 1)
        extra[dst] += rccl_ms(nbytes, gbps, 1)
    for r, js in jobs.items():
        extra[r] += sum(rccl_ms(sum(j.forward), gbps, 2) for j in js)
    if gbps is not None:
        fwd = [f + e for f, e in zip(fwd, extra)]
        bwd = [b + e for b, e in zip(bwd, extra)]
    out_bytes = [0.0] * n
    skips = []
    for src, dst, kind, nbytes in routes_of(stages):
        b = nbytes * share.get((src, dst), 1.0)
        if kind == 'act':
            out_bytes[src] = b
        else:
            skips.append((src, dst, b))
    t = step_time(fwd, bwd, [1] * n, m, 'except_last' if stop == m - 1 else
                  ('always' if stop == m else 'never'), out_bytes, skips, gbps)
    if links_out is not None and gbps is not None:
        # per forward route: MB per micro-batch, the direct link's ms per micro-batch at
        # this rate (its share when striped), and the sending stage's forward cell (ms) --
        # a ratio above 1 makes the route, not the stage, set the pace of the forward
        # phase (gradients take the mirrored links during backward cells 3x as long)
        for src, dst, kind, nbytes in routes_of(stages):
            ms = nbytes * share.get((src, dst), 1.0) / (gbps * 1e6)
            links_out.append((src, dst, kind, nbytes, routes.get((src, dst), []), ms,
                              fwd[src]))
    return t


def main():
    p = argparse.ArgumentParser()
    p.add_argument('files', nargs='+')
    p.add_argument('--unet-baseline', type=float, required=True)
    p.add_argument('--resnet-baseline', type=float, default=None)
    p.add_argument('--stripes', type=float, default=16.0,
                   help='multi-path transfers of messages >= this many MB')
    p.add_argument('--links', action='store_true', help='per directed link byte tables')
    a = p.parse_args()
    runs = {}
    for f in a.files:
        name = os.path.basename(f).replace('stage_harness_', '').replace('.json', '')
        runs[name.replace('_ref', '')] = load(f)
    denom = {'unet': a.unet_baseline, 'resnet': a.resnet_baseline}
    if 'amoeba_n2m1' in runs:
        args, st = runs['amoeba_n2m1']
        denom['amoeba'] = args['batch'] / (sum(s['device_ms'] for s in st) / 1e3)
        print(f"AmoebaNet n2m1 (denominator): stages "
              f"{' / '.join(str(s['device_ms']) for s in st)} ms -> {denom['amoeba']:.1f} "
              'samples/s\n')
    cols = ['free links'] + [f'{g:.0f} GB/s' for g in LINKS] + \
        [f'striped {g:.0f} GB/s' for g in LINKS]
    print('| experiment | stage device ms | ' + ' | '.join(cols) + ' | reference |')
    print('|---|---|' + '---:|' * (len(cols) + 1))
    link_tables = []
    for name, (args, st) in sorted(runs.items()):
        if name == 'amoeba_n2m1':
            continue
        batch = args['batch']
        d = denom.get(name.split('_')[0])
        plan = plan_of(st, a.stripes)
        cells = [batch / (simulate(args, st, None) / 1e3)]
        cells += [batch / (simulate(args, st, g) / 1e3) for g in LINKS]
        striped = []
        for g in LINKS:
            lt = []
            cells.append(batch / (simulate(args, st, g, plan, lt) / 1e3))
            striped.append(lt)
        plain = []
        t_plain = simulate(args, st, LINKS[0], None, plain)
        t_striped = simulate(args, st, LINKS[0], plan)
        link_tables.append((name, args['balance'], plan[0], plain, striped[0], args['chunks'],
                            t_plain, t_striped))
        fmt = [f'{c / d:.3f}' if d else f'{c:.1f}/s' for c in cells]
        stages = ' / '.join('%.1f' % s['device_ms'] for s in st)
        print(f"| {name} B {batch} m {args['chunks']} {args['balance']} | {stages} | " +
              ' | '.join(fmt) + f" | {REF.get(name, '')} |")
    if not a.links:
        return
    g = LINKS[0]
    for name, bal, routes, plain, striped, m, t_plain, t_striped in link_tables:
        if len(bal) < 2:
            continue
        print(f'\n#### {name} {bal}: forward routes at {g:.0f} GB/s')
        print('| route | kind | MB / micro-batch | direct: link ms | striped: relays | '
              'striped: link ms | sender forward cell ms | link / cell (direct, striped) |')
        print('|---|---|---:|---:|---|---:|---:|---:|')
        for (src, dst, kind, nb, _, ms, cell), (_, _, _, _, rl, sms, _) in zip(plain, striped):
            print(f'| {src}->{dst} | {kind} | {nb / 1e6:.0f} | {ms:.2f} | {rl or "-"} | '
                  f'{sms:.2f} | {cell:.2f} | {ms / cell:.2f}, {sms / cell:.2f} |')
        print(f'\n{name} {bal}: per directed link at {g:.0f} GB/s, bytes per step (forward '
              'messages one way, their gradients the mirrored way) and the share of the '
              'simulated step the link is busy')
        print('| link | direct GB / step | direct busy | striped GB / step | striped busy |')
        print('|---|---:|---:|---:|---:|')
        for a_, b_, direct, strip in link_bytes(plain, routes, m):
            print(f'| {a_}->{b_} | {direct / 1e9:.2f} | {direct / (g * 1e6) / t_plain:.2f} | '
                  f'{strip / 1e9:.2f} | {strip / (g * 1e6) / t_striped:.2f} |')


def link_bytes(plain, routes, m):
    """[(a, b, direct bytes, striped bytes)] per directed link and step: every forward
    route's bytes per micro-batch x m on its link(s), the gradients on the mirrored ones;
    striped, the direct link keeps its ``w0 / (w0 + relays)`` share and each relay hop
    (src -> r, r -> dst) carries ``1 / (w0 + relays)``."""
    w0 = (SUB + 1) / SUB
    direct, striped = {}, {}

    def add(table, a_, b_, nbytes):
        table[(a_, b_)] = table.get((a_, b_), 0.0) + nbytes
        table[(b_, a_)] = table.get((b_, a_), 0.0) + nbytes  # the gradients, mirrored

    for src, dst, _, nb, _, _, _ in plain:
        add(direct, src, dst, nb * m)
        rl = routes.get((src, dst), [])
        share = w0 / (w0 + len(rl))
        add(striped, src, dst, nb * m * share)
        for r in rl:
            add(striped, src, r, nb * m * (1 - share) / len(rl))
            add(striped, r, dst, nb * m * (1 - share) / len(rl))
    links = sorted(set(direct) | set(striped))
    return [(a_, b_, direct.get((a_, b_), 0.0), striped.get((a_, b_), 0.0))
            for a_, b_ in links]


if __name__ == '__main__':
    main()
