"""Summarise a rocprofv3 rocpd database (kernel trace) of a bench.py run.

Kernels of the timed steps only: step boundaries are the SGD optimizer's
``multi_tensor_apply`` launches (one burst per step); the first ``--skip``
bursts (warm-up steps, incl. MIOpen's find-mode trials) are dropped.

    python scripts/rocpd_summary.py gpurun_out/prof/run_results.db --skip 2 \\
        --csv profiles/x_kernel_stats.csv --md profiles/x_summary.md
"""
import argparse
import collections
import csv
import sqlite3

GROUPS = [
    ('tgpipe Winograd F(4,3) conv fwd/bwd-data on MFMA (HIP)',
     ('f4_conv_kernel', 'f4_split_reduce', 'f4_gemm_kernel', 'f4_input_transform')),
    ('tgpipe Winograd weight transform (HIP)', ('wino_weight_kernel', 'f4_weight_kernel')),
    ('tgpipe Winograd F(2,3) conv fwd/bwd-data on MFMA (HIP)',
     ('wino_conv', 'wino_split_reduce')),
    ('tgpipe Winograd weight gradient on MFMA (HIP)', ('wino_wgrad', 'f4_wgrad', 'f4_wg_')),
    ('tgpipe Winograd weight transform (HIP)', ('wino_weight_kernel',)),
    ('tgpipe fused Dropout2d+InstanceNorm+LeakyReLU (HIP)', ('dna_forward', 'dna_backward')),
    ('tgpipe other (HIP)', ('tgpipe::',)),
    ('MIOpen winograd', ('Winograd', 'Sp3AsmConv', 'winograd')),
    ('MIOpen igemm (wrw/fwd/bwd conv)', ('igemm',)),
    ('MIOpen other conv', ('miopen', 'MIOpen', 'naive_conv', 'conv')),
    ('layout transposes', ('transpose',)),
]


def group_of(name: str) -> str:
    for label, keys in GROUPS:
        if any(k in name for k in keys):
            return label
    return 'other ATen / runtime'


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument('db')
    p.add_argument('--skip', type=int, default=2, help='warm-up steps to drop')
    p.add_argument('--csv', default=None)
    p.add_argument('--md', default=None)
    p.add_argument('--title', default='rocprofv3 kernel trace')
    p.add_argument('--whole', type=int, default=0,
                   help='no optimizer bursts (e.g. benchmarks/stage_harness.py): the whole '
                        'trace counts as this many steps')
    args = p.parse_args()
    con = sqlite3.connect(args.db)
    rows = con.execute('select name, start, end from kernels order by start').fetchall()
    # optimizer bursts = step ends
    ends, last = [], None
    for i, (name, start, end) in enumerate(rows):
        if 'multi_tensor_apply' in name:
            if last is None or i - last > 1:
                ends.append(end)
            else:
                ends[-1] = end
            last = i
    if args.whole:
        ends, args.skip = [max(e for _, _, e in rows)], 0
    steps = args.whole or len(ends) - args.skip
    t0 = ends[args.skip - 1] if args.skip > 0 else rows[0][1]
    timed = [(n, s, e) for n, s, e in rows if s >= t0 and e <= ends[-1]]
    per = collections.defaultdict(lambda: [0, 0])
    for n, s, e in timed:
        per[n][0] += 1
        per[n][1] += e - s
    total = sum(v[1] for v in per.values())
    span = ends[-1] - t0
    # device idle: gaps between the end of everything launched so far and the next start
    idle, big, horizon = 0, 0, t0
    for _, s, e in timed:
        if s > horizon:
            idle += s - horizon
            big += (s - horizon) > 50_000
        horizon = max(horizon, e)
    ordered = sorted(per.items(), key=lambda kv: -kv[1][1])
    if args.csv:
        with open(args.csv, 'w', newline='') as f:
            w = csv.writer(f)
            w.writerow(['Name', 'Calls', 'TotalDurationNs', 'AverageNs', 'Percentage'])
            for n, (c, d) in ordered:
                w.writerow([n, c, d, round(d / c, 1), round(100 * d / total, 3)])
    groups = collections.defaultdict(int)
    for n, (c, d) in per.items():
        groups[group_of(n)] += d
    lines = [f'# {args.title}', '',
             f'{steps} timed steps; kernel time {total / 1e6:.1f} ms '
             f'({total / 1e6 / steps:.1f} ms/step); wall span {span / 1e6 / steps:.1f} ms/step; '
             f'device idle {idle / 1e6 / steps:.1f} ms/step ({big / steps:.0f} gaps > 50 us '
             f'per step).',
             '', '| group | ms/step | share |', '|---|---:|---:|']
    for g, d in sorted(groups.items(), key=lambda kv: -kv[1]):
        lines.append(f'| {g} | {d / 1e6 / steps:.1f} | {100 * d / total:.1f}% |')
    lines += ['', '| top kernels | calls/step | ms/step | share |', '|---|---:|---:|---:|']
    for n, (c, d) in ordered[:15]:
        short = n if len(n) < 90 else n[:87] + '...'
        lines.append(f'| `{short}` | {c / steps:.0f} | {d / 1e6 / steps:.2f} | '
                     f'{100 * d / total:.1f}% |')
    text = '\n'.join(lines) + '\n'
    print(text)
    if args.md:
        with open(args.md, 'w') as f:
            f.write(text)


if __name__ == '__main__':
    main()
