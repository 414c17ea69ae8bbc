"""Largest GPU idle gaps of a rocprofv3 kernel trace (rocpd database) in the last window:
the kernels before and after each gap.

    python scripts/r6/gaps.py run_results.db --last-ms 278 --top 25
"""
import argparse
import sqlite3
from collections import Counter


def main():
    p = argparse.ArgumentParser()
    p.add_argument('db')
    p.add_argument('--last-ms', type=float, required=True)
    p.add_argument('--top', type=int, default=25)
    a = p.parse_args()
    rows = sqlite3.connect(a.db).cursor().execute(
        'select name, start, end from kernels order by start').fetchall()
    end = max(r[2] for r in rows)
    rows = [r for r in rows if r[1] >= end - a.last_ms * 1e6]
    gaps = []
    cur_end, cur_name = rows[0][2], rows[0][0]
    for name, s, e in rows[1:]:
        if s > cur_end:
            gaps.append(((s - cur_end) / 1e3, cur_name[:70], name[:70]))
        if e > cur_end:
            cur_end, cur_name = e, name
    total = sum(g[0] for g in gaps)
    print(f'{len(gaps)} gaps, {total / 1e3:.1f} ms idle in {a.last_ms:.1f} ms')
    hist = Counter()
    for g, _, _ in gaps:
        hist['<5us' if g < 5 else '<20us' if g < 20 else '<100us' if g < 100 else '>=100us'] += g
    print({k: round(v / 1e3, 2) for k, v in hist.items()}, '(ms idle by gap size)')
    for g, before, after in sorted(gaps, reverse=True)[:a.top]:
        print(f'{g:9.1f} us  after {before}  ->  {after}')


if __name__ == '__main__':
    main()
