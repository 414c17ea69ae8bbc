"""Per-kernel PMC table of rocprofv3 --pmc runs (counter_collection CSVs): counters summed
over a kernel's dispatches, plus derived MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES /
(GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) and per-wave-cycle shares.

    python scripts/r5/pmc_table.py gpurun_out/r5b/*/run_counter_collection.csv
"""
import collections
import csv
import sys


def main() -> None:
    for path in sys.argv[1:]:
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        disp = collections.defaultdict(set)
        for r in csv.DictReader(open(path)):
            k = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0]
            k = k.replace('void ', '').replace('tgpipe::', '')
            agg[k][r['Counter_Name']] += float(r['Counter_Value'])
            disp[k].add(r.get('Dispatch_Id', r.get('Correlation_Id', '')))
        for k, v in agg.items():
            if 'conv_gemm' not in k and 'gemm' not in k and 'f4_' not in k:
                continue
            n = max(1, len(disp[k]))
            g = v.get('GRBM_GUI_ACTIVE', 0.0)
            wc = v.get('SQ_WAVE_CYCLES', 0.0)
            out = {'dispatches': n}
            if g and 'SQ_VALU_MFMA_BUSY_CYCLES' in v:
                out['mfma_busy'] = round(v['SQ_VALU_MFMA_BUSY_CYCLES'] / (g / 8 * 1024), 3)
            for c in ('SQ_WAIT_INST_ANY', 'SQ_WAIT_ANY', 'SQ_WAIT_INST_LDS', 'SQ_ACTIVE_INST_VALU',
                      'SQ_ACTIVE_INST_LDS', 'SQ_ACTIVE_INST_ANY', 'SQ_VALU_MFMA_COEXEC_CYCLES'):
                if c in v and wc:
                    out[c.replace('SQ_', '').lower() + '/wave_cyc'] = round(v[c] / wc, 3)
            for c in ('SQ_INSTS_VALU', 'SQ_INSTS_LDS', 'SQ_LDS_BANK_CONFLICT', 'SQ_LDS_IDX_ACTIVE',
                      'SQ_WAVES'):
                if c in v:
                    out[c.replace('SQ_', '').lower() + '/disp'] = round(v[c] / n)
            if 'SQ_LDS_BANK_CONFLICT' in v and v.get('SQ_LDS_IDX_ACTIVE'):
                out['lds_conflict_share'] = round(
                    v['SQ_LDS_BANK_CONFLICT'] / v['SQ_LDS_IDX_ACTIVE'], 3)
            print(path.split('/')[-2], k[:48], out)


if __name__ == '__main__':
    main()
