"""Summarise a rocprofv3 rocpd database (kernel dispatches): per-kernel totals and GPU busy
time (union of kernel intervals across streams) inside a time window.

    python scripts/r4/rocpd_summary.py run_results.db --last-ms 1011 --steps 2
"""
import argparse
import re
import sqlite3
from collections import defaultdict


def family(name):
    n = name.replace('(anonymous namespace)::', '')
    n = re.sub(r'\(.*', '', n)
    n = re.sub(r'^void ', '', n)
    return n[:90]


def main():
    p = argparse.ArgumentParser()
    p.add_argument('db')
    p.add_argument('--last-ms', type=float, required=True, help='window: the last N ms')
    p.add_argument('--steps', type=int, default=1, help='steps inside the window')
    p.add_argument('--top', type=int, default=25)
    a = p.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    rows = cur.execute('select name, start, end from kernels order by start').fetchall()
    end = max(r[2] for r in rows)
    lo = end - a.last_ms * 1e6
    rows = [r for r in rows if r[1] >= lo]
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for name, s, e in rows:
        tot[family(name)] += (e - s) / 1e6
        cnt[family(name)] += 1
    busy, cur_s, cur_e = 0.0, None, None
    for _, s, e in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = (end - rows[0][1]) / 1e6
    ksum = sum(tot.values())
    print(f'window {span:.1f} ms, {len(rows)} kernels ({len(rows) / a.steps:.0f} per step), '
          f'busy (union) {busy / 1e6:.1f} ms = {busy / 1e6 / span:.3f}, '
          f'kernel time sum {ksum:.1f} ms (concurrency {ksum / (busy / 1e6):.2f})')
    print('| kernel | ms per step | share of kernel time | launches per step |')
    print('|---|---:|---:|---:|')
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:a.top]:
        print(f'| `{k}` | {v / a.steps:.1f} | {v / ksum:.3f} | {cnt[k] / a.steps:.0f} |')


if __name__ == '__main__':
    main()
