"""Average PMC counters per dispatch of attention_h3_kernel under gpurun_out/apmc.
usage: python tools/attn_pmc_summary.py [dir]"""
import csv, glob, sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/apmc'
tot = defaultdict(float); disp = defaultdict(set)
for f in glob.glob(f'{root}/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'attention_h3' not in r['Kernel_Name']:
            continue
        tot[r['Counter_Name']] += float(r['Counter_Value'])
        disp[r['Counter_Name']].add(r['Dispatch_Id'])
for k in sorted(tot):
    print(f'   {k:28s} {tot[k] / max(1, len(disp[k])):16.4g}')
