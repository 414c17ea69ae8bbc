"""Re-derive MI355X balances from a measured per-layer profile.

Reads ``benchmarks/layer_profile.py`` output, rebuilds the model's skip routes
(stash layer, pop layer, bytes per micro-batch) and runs the step simulator's
balance search (``torchgpipe_amd.balance.simulate.optimize``) for each
pipeline depth of the bench tables, printing simulated samples/s of the
reference balance and of the tuned one.

    python scripts/tune_balance.py --profile profiles/unet_layer_profile.json --model unet
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchgpipe_amd.balance.simulate import optimize, step_time  # noqa: E402
from torchgpipe_amd.models import amoebanetd, unet  # noqa: E402
from torchgpipe_amd.skip.skippable import Skippable  # noqa: E402


def skip_routes(model, out_bytes):
    stash, routes = {}, []
    for idx, layer in enumerate(model.children()):
        if isinstance(layer, Skippable):
            for key in layer.stashable():
                stash[key] = idx
            for key in layer.poppable():
                s = stash[key]
                routes.append((s, idx, float(out_bytes[s])))
    return routes


def calibrate(fwd, bwd, m, paths):
    """Per-layer times scaled so every stage measured by the stage harness at this
    micro-batch count matches its measured device time (forward + recompute + backward
    of all micro-batches); layers no harness covers keep their profiled times."""
    fwd, bwd = list(fwd), list(bwd)
    for path in paths:
        run = json.load(open(path))
        if run['args']['chunks'] != m:
            continue
        ck = run['args'].get('checkpoint', 'except_last')
        for st in run['stages']:
            lo, hi = st['layers']
            f, b = sum(fwd[lo:hi]), sum(bwd[lo:hi])
            recompute = f * (m - 1 if ck == 'except_last' else m if ck == 'always' else 0)
            predicted = (f + b) * m + recompute
            scale = st['device_ms'] / predicted
            for i in range(lo, hi):
                fwd[i] *= scale
                bwd[i] *= scale
    return fwd, bwd


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument('--profile', required=True)
    p.add_argument('--model', choices=['unet', 'amoebanet'], default='unet')
    p.add_argument('--link-gbps', type=float, default=60.0)
    p.add_argument('--calibrate', nargs='*', default=[],
                   help='benchmarks/stage_harness.py outputs: scale the layers of each '
                        'measured stage by measured / profiled stage time before searching')
    args = p.parse_args()
    import bench
    prof = json.load(open(args.profile))
    if args.model == 'unet':
        model, table = unet(), bench.UNET_EXPERIMENTS
    else:
        model, table = amoebanetd(1000, 18, 256), bench.AMOEBA_EXPERIMENTS
    for n, exp in sorted(table.items()):
        if n == 1:
            continue
        m = exp['chunks']
        mb = exp['batch'] // m
        key = str(mb) if str(mb) in prof['profiles'] else min(
            prof['profiles'], key=lambda k: abs(int(k) - mb))
        pr = prof['profiles'][key]
        scale = mb / int(key)
        fwd = [f * scale for f in pr['fwd_ms']]
        bwd = [b * scale for b in pr['bwd_ms']]
        ob = [b * scale for b in pr['out_bytes']]
        skips = skip_routes(model, ob)
        fwd, bwd = calibrate(fwd, bwd, m, args.calibrate)
        kw = dict(out_bytes=ob, skips=skips, link_gbps=args.link_gbps)
        ck = 'except_last' if m > 1 else 'always'
        t_ref = step_time(fwd, bwd, exp['balance'], m, ck, **kw)
        t_old = step_time(fwd, bwd, exp['tuned'], m, ck, **kw)
        best, t_best = optimize(fwd, bwd, n, m, ck, start=exp['tuned'], **kw)
        print(json.dumps({'n': n, 'm': m, 'mb_profile': key,
                          'ref': [exp['balance'], round(exp['batch'] / t_ref * 1e3, 1)],
                          'old_tuned': [exp['tuned'], round(exp['batch'] / t_old * 1e3, 1)],
                          'new': [best, round(exp['batch'] / t_best * 1e3, 1)]}))


if __name__ == '__main__':
    main()
