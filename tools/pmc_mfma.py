"""MFMA-busy evidence per kernel from a rocprofv3 --pmc pass.

The pass (one run, counters within the gfx950 slot limits: 8 SQ, 2 GRBM):
    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY \
        SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d DIR -- python3 bench.py ...
This script averages every counter per dispatch of each (kernel, grid) and derives
    mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs x 4 SIMDs)
the share of the dispatch's active cycles in which an average SIMD's matrix pipe was busy
(GRBM_GUI_ACTIVE is summed over the 8 XCDs: MI355X_MICROARCH.md "DVFS give-back";
SQ_VALU_MFMA_BUSY_CYCLES counts cycles, 16 per v_mfma_f32_16x16x32_f16: § Per-instruction
cycle constants), and the clock the dispatch ran at, GRBM_GUI_ACTIVE / 8 / duration, where
the kernel trace of the same run gives the duration.
usage: python tools/pmc_mfma.py DIR OUT.json [label=name-prefix ...]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS = 256 * 4


def short(n):
    n = n.replace('void ', '').replace('(anonymous namespace)::', '')
    return n.split('(')[0]


def load(src):
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in glob.glob(f'{src}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            k = f'{short(r["Kernel_Name"])}|{r["Grid_Size"]}'
            acc[k][r['Counter_Name']] += float(r['Counter_Value'])
            disp[k].add((f, r['Dispatch_Id']))
    out = {}
    for k, cs in acc.items():
        n = len(disp[k])
        row = {c: v / n for c, v in cs.items()}
        row['dispatches'] = n
        gui = row.get('GRBM_GUI_ACTIVE')
        if gui and 'SQ_VALU_MFMA_BUSY_CYCLES' in row:
            row['mfma_busy'] = round(row['SQ_VALU_MFMA_BUSY_CYCLES'] / (gui / 8 * SIMDS), 4)
        if 'SQ_WAVE_CYCLES' in row and row['SQ_WAVE_CYCLES'] > 0:
            for c in ('SQ_WAIT_ANY', 'SQ_ACTIVE_INST_ANY'):
                if c in row:
                    row[c.lower() + '_share'] = round(row[c] / row['SQ_WAVE_CYCLES'], 4)
        out[k] = row
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    labels = dict(a.split('=', 1) for a in sys.argv[3:])
    ks = load(src)
    doc = {'what': __doc__.split('\n\n')[0], 'source_dir': src, 'kernels': ks}
    if labels:  # friendly names: the heaviest dispatch group whose key starts with the prefix
        named = {}
        for name, pref in labels.items():
            hit = [(k, v) for k, v in ks.items() if k.startswith(pref)]
            if hit:
                k, v = max(hit, key=lambda kv: kv[1].get('GRBM_GUI_ACTIVE', 0))
                named[name] = {'kernel': k, **{c: v[c] for c in v if c in (
                    'mfma_busy', 'SQ_VALU_MFMA_BUSY_CYCLES', 'GRBM_GUI_ACTIVE', 'dispatches',
                    'sq_wait_any_share', 'sq_active_inst_any_share')}}
        doc['named'] = named
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    json.dump(doc, open(dst, 'w'), indent=1, sort_keys=True)
    for k, v in sorted(ks.items(), key=lambda kv: -kv[1].get('GRBM_GUI_ACTIVE', 0))[:25]:
        print(f'{k[:90]:90s} busy {v.get("mfma_busy", float("nan")):7.3f}  gui {v.get("GRBM_GUI_ACTIVE", 0):12.0f}')


if __name__ == '__main__':
    main()
