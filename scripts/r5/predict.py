"""Speed-up predictions from stage-harness runs, with and without link transfers.

Every stage of an experiment ran alone on one GPU through the real engine
(``benchmarks/stage_harness.py``: device ms per step and the bytes each stage sends per
micro-batch).  Two predictions per experiment:

* ``max-stage``: max stage device time x (m + n - 1) / m (the GPipe bubble, free links);
* ``sim``: :func:`torchgpipe_amd.balance.simulate.step_time` with each stage as one
  pseudo-layer -- forward F_j and backward B_j = 2 F_j per micro-batch, F_j from the stage's
  device time (m F + (recomputed cells) F + m B), checkpoint mode, the boundary activation
  bytes on each j -> j+1 link and every cross-stage skip on its own direct link (both ways
  for the gradients) -- at free links and at the stated per-link bandwidths.

``--stripes MB``: two more columns, the ``sim`` at each bandwidth with multi-path transfers
(``parallel/stripes.py``): the engine's own planner picks relays from these sends (messages
of at least MB megabytes), and a striped route's direct link then carries its direct share
``w0 / (w0 + R)`` of the bytes (R relays, ``w0 = 1.25``); the detours run on links nothing
else uses, so the direct share bounds the route.

Denominators: U-Net / ResNet over their no-GPipe baselines (same tree, bench.py sections),
AmoebaNet over n2m1 (its two stages back to back, m = 1).

    python scripts/r5/predict.py --unet-baseline 712 --resnet-baseline 1640 \\
        profiles/r5/harness/*.json
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
LINKS = (100.0, 50.0)  # GB/s per direction and link, effective


def load(path):
    with open(path) as f:
        d = json.load(f)
    return d['args'], d['stages']


def striped_shares(stages, min_mb, max_relays=3, sub=4):
    """{(src, dst): share of the route's bytes left on its direct link} from the planner."""
    sends = {j: [] for j in range(len(stages))}
    for j, s in enumerate(stages):
        for key, nbytes in s.get('sent_bytes', {}).items():
            kind, dst = key.split('->')
            sends[j].append(stripes.Send(int(dst), kind, int(nbytes)))
            sends[int(dst)].append(stripes.Send(j, 'g' + kind, int(nbytes)))
    routes, _ = stripes.plan(sends, list(range(len(stages))), int(min_mb * 1e6), max_relays,
                             sub)
    w0 = (sub + 1) / sub
    return {r: w0 / (w0 + len(relays)) for r, relays in routes.items()}


def simulate(args, stages, gbps, shares=None):
    n, m = len(stages), args['chunks']
    stop = {'always': m, 'except_last': m - 1, 'never': 0}[args.get('checkpoint',
                                                                  'except_last')]
    fwd = [s['device_ms'] / (3 * m + stop) for s in stages]
    bwd = [2 * f for f in fwd]
    shares = shares or {}
    out_bytes = [float(s.get('sent_bytes', {}).get(f'act->{j + 1}', 0))
                 * shares.get((j, j + 1), 1.0) for j, s in enumerate(stages)]
    skips = []
    for j, s in enumerate(stages):
        for key, nbytes in s.get('sent_bytes', {}).items():
            kind, dst = key.split('->')
            if kind == 'skip':
                skips.append((j, int(dst), float(nbytes) * shares.get((j, int(dst)), 1.0)))
    return step_time(fwd, bwd, [1] * n, m, 'except_last' if stop == m - 1 else
                     ('always' if stop == m else 'never'), out_bytes, skips, gbps)


def main():
    p = argparse.ArgumentParser()
    p.add_argument('files', nargs='+')
    p.add_argument('--unet-baseline', type=float, required=True)
    p.add_argument('--resnet-baseline', type=float, default=None)
    p.add_argument('--stripes', type=float, default=None,
                   help='also simulate multi-path transfers of messages >= this many MB')
    a = p.parse_args()
    runs = {}
    for f in a.files:
        name = os.path.basename(f).replace('stage_harness_', '').replace('.json', '')
        name = name.replace('_ref', '')
        runs[name] = load(f)
    denom = {'unet': a.unet_baseline, 'resnet': a.resnet_baseline}
    if 'amoeba_n2m1' in runs:
        args, st = runs['amoeba_n2m1']
        denom['amoeba'] = args['batch'] / (sum(s['device_ms'] for s in st) / 1e3)
        print(f"AmoebaNet n2m1 (denominator): stages "
              f"{' / '.join(str(s['device_ms']) for s in st)} ms -> {denom['amoeba']:.1f} "
              'samples/s\n')
    cols = ' | '.join(f'sim {g:.0f} GB/s' for g in LINKS)
    if a.stripes is not None:
        cols += ' | ' + ' | '.join(f'striped {g:.0f} GB/s' for g in LINKS)
    print(f'| experiment | stage device ms | max-stage speed-up | sim free links | {cols} |'
          ' reference |')
    extra = len(LINKS) if a.stripes is not None else 0
    print('|---|---|---:|---:|' + '---:|' * (len(LINKS) + extra) + '---:|')
    for name, (args, st) in sorted(runs.items()):
        if name == 'amoeba_n2m1':
            continue
        n, m, batch = len(st), args['chunks'], args['batch']
        d = denom.get(name.split('_')[0])
        mx = max(s['device_ms'] for s in st)
        cells = [batch / (mx * (m + n - 1) / m / 1e3)]
        cells += [batch / (simulate(args, st, g) / 1e3) for g in (None,) + LINKS]
        if a.stripes is not None:
            shares = striped_shares(st, a.stripes)
            cells += [batch / (simulate(args, st, g, shares) / 1e3) for g in LINKS]
        fmt = [f'{c / d:.3f}' if d else f'{c:.1f}/s' for c in cells]
        stages = ' / '.join('%.1f' % s['device_ms'] for s in st)
        print(f"| {name} B {batch} m {m} {args['balance']} | {stages} | " + ' | '.join(fmt) +
              f" | {REF.get(name, '')} |")


if __name__ == '__main__':
    main()
