"""Per-kernel PMC summary of rocprofv3 --pmc CSVs (counter_collection): MFMA busy =
SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), wait share =
SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES, LDS bank conflicts per dispatch.

    python scripts/r4/pmc_summary.py profiles/r4/pmc/*.csv
"""
import collections
import csv
import os
import sys

print('| probe | kernel | dispatches | MFMA busy | wait / wave cycles |'
      ' LDS bank conflicts per dispatch |')
print('|---|---|---:|---:|---:|---:|')
for path in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0]
        k = k.replace('void ', '')
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
        disp[k].add(r.get('Dispatch_Id', r.get('Correlation_Id', '')))
    for k, v in agg.items():
        if 'conv_gemm' not in k:
            continue
        n = max(1, len(disp[k]))
        g = v['GRBM_GUI_ACTIVE']
        busy = v['SQ_VALU_MFMA_BUSY_CYCLES'] / (g / 8 * 1024) if g else 0.0
        wait = v['SQ_WAIT_INST_ANY'] / v['SQ_WAVE_CYCLES'] if v['SQ_WAVE_CYCLES'] else 0.0
        print(f'| {os.path.basename(path)} | `{k}` | {n} | {busy:.3f} | {wait:.2f} | '
              f'{v["SQ_LDS_BANK_CONFLICT"] / n:.0f} |')
