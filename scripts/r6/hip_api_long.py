"""Longest HIP API calls of a rocprofv3 --hip-trace database in the last window (host-side
blocking calls: synchronisations, allocations, copies).

    python scripts/r6/hip_api_long.py run_results.db --last-ms 280 --top 25
"""
import argparse
import sqlite3
from collections import defaultdict


def main():
    p = argparse.ArgumentParser()
    p.add_argument('db')
    p.add_argument('--last-ms', type=float, required=True)
    p.add_argument('--top', type=int, default=25)
    a = p.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    tables = [r[0] for r in cur.execute("select name from sqlite_master where type in "
                                        "('table', 'view')").fetchall()]
    print('tables:', [t for t in tables if 'region' in t or 'api' in t or 'hip' in t][:12])
    src = 'regions' if 'regions' in tables else None
    if src is None:
        return
    cols = [r[1] for r in cur.execute(f'pragma table_info({src})').fetchall()]
    print('columns:', cols)
    rows = cur.execute(f'select name, start, end from {src}').fetchall()
    end = max(r[2] for r in rows)
    rows = [r for r in rows if r[1] >= end - a.last_ms * 1e6]
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for name, s, e in rows:
        tot[name] += (e - s) / 1e3
        cnt[name] += 1
    print('total us per API (top):')
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:15]:
        print(f'  {v:10.1f} us  {cnt[k]:7d} calls  {k}')
    print('longest calls:')
    for name, s, e in sorted(rows, key=lambda r: r[1] - r[2])[:a.top]:
        print(f'  {(e - s) / 1e3:9.1f} us  {name}')


if __name__ == '__main__':
    main()
