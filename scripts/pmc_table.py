"""Aggregate rocprofv3 --pmc CSV output per kernel (mean over dispatches).

    python scripts/pmc_table.py gpurun_out/pmc/p1_*/run_counter_collection.csv --kernel wino_conv
"""
import argparse
import collections
import csv


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument('files', nargs='+')
    p.add_argument('--kernel', default='wino')
    a = p.parse_args()
    for path in a.files:
        acc = collections.defaultdict(list)
        meta = {}
        for r in csv.DictReader(open(path)):
            if a.kernel not in r['Kernel_Name']:
                continue
            acc[r['Counter_Name']].append(float(r['Counter_Value']))
            meta = {k: r[k] for k in ('Grid_Size', 'VGPR_Count', 'Accum_VGPR_Count',
                                      'LDS_Block_Size')}
            meta['ns'] = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
        print(path, meta)
        for k, v in sorted(acc.items()):
            print(f'  {k:28s} {sum(v) / len(v):16.0f}  (n={len(v)})')


if __name__ == '__main__':
    main()
