"""Transfer-aware balances: search partitions with the step simulator at a link bandwidth.

Per-layer costs come from a stage-harness run at the reference balance (its stage device
times, spread over each stage's layers in proportion to a per-layer profile:
``scripts/balance_from_harness.py``); per micro-batch each layer runs F forward and 2F
backward (recomputed where checkpointed), sends its output when it ends a stage, and every
cross-stage skip travels on its own link (``torchgpipe_amd.balance.simulate``).  Prints the
reference balance, the balance given with ``--current`` and the searched one, each
simulated at free links and at ``--gbps``.

    python scripts/r5/tune_transfer.py --model unet \\
        --profile profiles/unet_layer_profile_f4w.json \\
        --harness profiles/r5/harness/stage_harness_unet_p8.json --gbps 100 \\
        --current 18 26 27 30 22 44 40 34
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'scripts'))

from balance_from_harness import calibrated_costs  # noqa: E402
from torchgpipe_amd.balance.simulate import optimize, step_time  # noqa: E402


def skip_routes(model_name: str, out_bytes):
    """(stash layer, pop layer, bytes) of every skip: one-layer partitions of the model."""
    if model_name != 'unet':
        return []
    import torch
    from torchgpipe_amd.models import unet
    from torchgpipe_amd.skip.layout import inspect_skip_layout
    with torch.device('meta'):
        model = unet(depth=5, num_convs=5, base_channels=64)
    parts = [torch.nn.Sequential(m) for m in model]
    layout = inspect_skip_layout(parts)
    return [(s, p, float(out_bytes[s])) for (s, p) in layout.by_ns_name.values()]


def main() -> None:
    p = argparse.ArgumentParser(description=__doc__,
                                formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument('--model', choices=['unet', 'amoebanet'], required=True)
    p.add_argument('--profile', required=True)
    p.add_argument('--profile-micro', default=None, help='micro-batch key of the profile')
    p.add_argument('--harness', required=True)
    p.add_argument('--gbps', type=float, default=100.0)
    p.add_argument('--current', type=int, nargs='*', default=None)
    a = p.parse_args()
    run = json.load(open(a.harness))
    args = run['args']
    m, batch, n = args['chunks'], args['batch'], len(args['balance'])
    mb = -(-batch // m)
    prof_all = json.load(open(a.profile))['profiles']
    key = a.profile_micro or min(prof_all, key=lambda k: abs(int(k) - mb))
    prof = prof_all[key]
    weights = [2 * f + b for f, b in zip(prof['fwd_ms'], prof['bwd_ms'])]
    cost = calibrated_costs(weights, [run])  # per layer, ms per step
    ckpt = args.get('checkpoint', 'except_last')
    stop = {'always': m, 'except_last': m - 1, 'never': 0}[ckpt]
    fwd = [c / (3 * m + stop) for c in cost]
    bwd = [2 * f for f in fwd]
    scale = mb / int(key)
    out_bytes = [b * scale for b in prof['out_bytes']]
    skips = skip_routes(a.model, out_bytes)

    def show(name, bal):
        free = step_time(fwd, bwd, bal, m, ckpt, out_bytes, skips, None)
        link = step_time(fwd, bwd, bal, m, ckpt, out_bytes, skips, a.gbps)
        print(json.dumps({'balance': name, 'layers': list(bal), 'sim_ms_free': round(free, 1),
                          f'sim_ms_{a.gbps:g}GBps': round(link, 1),
                          'samples_per_s': round(batch / link * 1e3, 1)}))

    show('reference', args['balance'])
    if a.current:
        show('current tuned', a.current)
    best, _ = optimize(fwd, bwd, n, m, ckpt, out_bytes, skips, a.gbps, start=args['balance'])
    if a.current:
        alt, _ = optimize(fwd, bwd, n, m, ckpt, out_bytes, skips, a.gbps, start=a.current)
        if step_time(fwd, bwd, alt, m, ckpt, out_bytes, skips, a.gbps) < \
                step_time(fwd, bwd, best, m, ckpt, out_bytes, skips, a.gbps):
            best = alt
    show('searched', best)


if __name__ == '__main__':
    main()
