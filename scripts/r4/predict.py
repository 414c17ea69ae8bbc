"""Reference-balance speed-up predictions from stage-harness runs (one GPU per stage).

Prediction = max stage device ms x (m + n - 1) / m (GPipe fill/drain; transfers excluded),
samples/s = B / that; U-Net over the no-GPipe baseline (same tree, bench.py's `baseline`),
AmoebaNet over n2m1 (its two stages run back to back: m = 1).

    python scripts/r4/predict.py --unet-baseline 710.5 profiles/r4/stage_harness_*_ref.json
"""
import argparse
import json
import os

REF = {'unet_p2': 1.246, 'unet_p4': 2.352, 'unet_p8': 3.105,
       'amoeba_n2m32': 1.773, 'amoeba_n4m32': 2.709, 'amoeba_n8m32': 4.953,
       'resnet_p2': 1.414}


def load(path):
    with open(path) as f:
        d = json.load(f)
    a = d['args']
    stages = [s['device_ms'] for s in d['stages']]
    host = [s['host_ms'] for s in d['stages']]
    return a, stages, host


def main():
    p = argparse.ArgumentParser()
    p.add_argument('files', nargs='+')
    p.add_argument('--unet-baseline', type=float, required=True)
    p.add_argument('--resnet-baseline', type=float, default=None)
    args = p.parse_args()
    runs = {}
    for f in args.files:
        name = os.path.basename(f).replace('stage_harness_', '').replace('_ref.json', '')
        runs[name] = load(f)
    denom = {'unet': args.unet_baseline, 'resnet': args.resnet_baseline}
    if 'amoeba_n2m1' in runs:
        a, st, _ = runs['amoeba_n2m1']
        denom['amoeba'] = a['batch'] / (sum(st) / 1e3)
        print(f"amoeba n2m1: stages {st} -> {denom['amoeba']:.1f} samples/s")
    print('| experiment | stage device ms | max | predicted samples/s | speed-up | reference |'
          ' host/device (max stage) |')
    print('|---|---|---:|---:|---:|---:|---:|')
    for name, (a, st, host) in sorted(runs.items()):
        if name == 'amoeba_n2m1':
            continue
        n, m = len(st), a['chunks']
        k = max(range(n), key=lambda i: st[i])
        step = st[k] * (m + n - 1) / m
        sps = a['batch'] / (step / 1e3)
        d = denom.get(name.split('_')[0])
        sp = f'{sps / d:.3f}' if d else 'n/a'
        print(f"| {name} B {a['batch']} m {m} {a['balance']} | "
              f"{' / '.join(f'{s:.1f}' for s in st)} | {st[k]:.1f} | {sps:.1f} | {sp} | "
              f"{REF.get(name, REF.get(name[:9], ''))} | {host[k] / st[k]:.2f} |")


if __name__ == '__main__':
    main()
