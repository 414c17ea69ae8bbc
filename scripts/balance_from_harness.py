"""Min-max balance from measured stage times (benchmarks/stage_harness.py outputs).

Every harness run measures the device time of whole stages; their boundaries give
points of the cumulative per-layer cost curve.  Between two known points the cost is
spread over the layers in proportion to a layer profile (benchmarks/layer_profile.py:
forward + recompute + backward), and the balance minimising the largest stage is found
by dynamic programming over that calibrated curve.

    python scripts/balance_from_harness.py --profile profiles/unet_layer_profile_f4w.json \\
        --partitions 8 gpurun_out/stage_p8_a.json gpurun_out/stage_p8_b.json
"""
import argparse
import json
from typing import Dict, List, Sequence, Tuple


def calibrated_costs(weights: Sequence[float], runs: Sequence[dict]) -> List[float]:
    points: Dict[int, float] = {0: 0.0}
    for run in runs:
        total = 0.0
        for st in run['stages']:
            total += st['device_ms']
            points[st['layers'][1]] = total
    keys = sorted(points)
    if keys[-1] != len(weights):
        raise ValueError('harness runs must cover every layer')
    cost = [0.0] * len(weights)
    for a, b in zip(keys, keys[1:]):
        seg, tot = points[b] - points[a], sum(weights[a:b])
        for i in range(a, b):
            cost[i] = seg * weights[i] / tot if tot > 0 else seg / (b - a)
    return cost


def min_max_partition(cost: Sequence[float], n: int) -> Tuple[List[int], List[float]]:
    pre = [0.0]
    for c in cost:
        pre.append(pre[-1] + c)
    length = len(cost)
    inf = float('inf')
    best = [[inf] * (length + 1) for _ in range(n + 1)]
    arg = [[0] * (length + 1) for _ in range(n + 1)]
    best[0][0] = 0.0
    for k in range(1, n + 1):
        for j in range(k, length + 1):
            for i in range(k - 1, j):
                v = max(best[k - 1][i], pre[j] - pre[i])
                if v < best[k][j]:
                    best[k][j], arg[k][j] = v, i
    balance, j = [], length
    for k in range(n, 0, -1):
        i = arg[k][j]
        balance.append(j - i)
        j = i
    balance.reverse()
    stages, b = [], 0
    for x in balance:
        stages.append(pre[b + x] - pre[b])
        b += x
    return balance, stages


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument('--profile', required=True)
    p.add_argument('--micro-batch', default='16')
    p.add_argument('--partitions', type=int, required=True)
    p.add_argument('runs', nargs='+')
    a = p.parse_args()
    prof = json.load(open(a.profile))['profiles'][a.micro_batch]
    weights = [2 * f + b for f, b in zip(prof['fwd_ms'], prof['bwd_ms'])]
    cost = calibrated_costs(weights, [json.load(open(r)) for r in a.runs])
    balance, stages = min_max_partition(cost, a.partitions)
    print(json.dumps({'balance': balance, 'predicted_stage_ms': [round(s, 1) for s in stages]}))


if __name__ == '__main__':
    main()
