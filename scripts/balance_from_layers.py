"""MI355X balances from a per-layer stage-harness profile.

``benchmarks/stage_harness.py --balance 1 1 ... 1`` times every layer as its own stage
(forward + recompute + backward of all micro-batches, device ms).  This picks, for each
pipeline depth, the contiguous partition with the least maximum stage (then least sum of
squares: ``balance.blockpartition.solve_splits``) and predicts samples/s with the GPipe
fill/drain bubble, max stage x (m + n - 1) / m -- the same model as
``profiles/r3/speedup_prediction.md``; per-layer sums ignore cross-layer effects.

    python scripts/balance_from_layers.py profile.json --parts 2 4 8 --batch 1280 --chunks 32
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchgpipe_amd.balance.blockpartition import solve_splits  # noqa: E402


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument('profile')
    p.add_argument('--parts', type=int, nargs='+', default=[2, 4, 8])
    p.add_argument('--batch', type=int, nargs='+', required=True,
                   help='global batch per depth (one value, or one per --parts entry)')
    p.add_argument('--chunks', type=int, required=True)
    p.add_argument('--scale', type=float, default=1.0,
                   help='multiply the profiled times (a profile taken with fewer micro-batches)')
    p.add_argument('--ref', type=str, nargs='*', default=[],
                   help="reference balances to price too, e.g. '2,2,2,3,3,4,4,4'")
    a = p.parse_args()
    stages = json.load(open(a.profile))['stages']
    layers = [s['device_ms'] * a.scale for s in sorted(stages, key=lambda s: s['layers'][0])]
    batches = a.batch if len(a.batch) == len(a.parts) else a.batch * len(a.parts)
    refs = {len(b.split(',')): [int(v) for v in b.split(',')] for b in a.ref}
    m = a.chunks
    out = []
    for k, batch in zip(a.parts, batches):
        rows = {'tuned': solve_splits(layers, k)}
        if k in refs:
            rows['ref'] = refs[k]
        for name, bal in rows.items():
            assert sum(bal) == len(layers), (name, bal)
            sums, i = [], 0
            for size in bal:
                sums.append(round(sum(layers[i:i + size]), 1))
                i += size
            t = max(sums) * (m + k - 1) / m
            row = {'parts': k, 'balance_source': name, 'balance': bal, 'stage_ms': sums,
                   'max_stage_ms': max(sums), 'predicted_samples_per_sec':
                   round(batch / (t / 1000), 1)}
            out.append(row)
            print(json.dumps(row))
    return None


if __name__ == '__main__':
    main()
