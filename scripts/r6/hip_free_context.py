"""What runs around the HIP API hipFree calls of a rocprofv3 --hip-trace database: the API
calls just before / after each of the longest ones, and the kernels dispatched next.

    python scripts/r6/hip_free_context.py run_results.db --last-ms 280
"""
import argparse
import sqlite3


def main():
    p = argparse.ArgumentParser()
    p.add_argument('db')
    p.add_argument('--last-ms', type=float, required=True)
    p.add_argument('--name', default='hipFree')
    a = p.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    cols = [r[1] for r in cur.execute('pragma table_info(regions)').fetchall()]
    kcols = [r[1] for r in cur.execute('pragma table_info(kernels)').fetchall()]
    print('regions columns:', cols)
    print('kernels columns:', kcols)
    regs = cur.execute('select name, start, end from regions order by start').fetchall()
    end = max(r[2] for r in regs)
    lo = end - a.last_ms * 1e6
    regs = [r for r in regs if r[1] >= lo]
    kerns = cur.execute('select name, start from kernels order by start').fetchall()
    frees = sorted([i for i, r in enumerate(regs) if r[0] == a.name],
                   key=lambda i: regs[i][1] - regs[i][2])[:6]
    for i in frees:
        print(f'--- {a.name} {(regs[i][2] - regs[i][1]) / 1e3:.1f} us')
        for j in range(max(0, i - 6), min(len(regs), i + 4)):
            mark = '*' if j == i else ' '
            print(f'   {mark} {regs[j][0]} {(regs[j][2] - regs[j][1]) / 1e3:.1f}')
        nxt = [k[0][:80] for k in kerns if k[1] > regs[i][2]][:3]
        print('   next kernels:', nxt)
    names = {}
    for r in regs:
        names[r[0]] = names.get(r[0], 0) + 1
    print('api counts:', sorted(names.items(), key=lambda kv: -kv[1])[:30])


if __name__ == '__main__':
    main()
