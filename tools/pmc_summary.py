"""Average PMC counters per dispatch of the conv_gemm kernels under a pmc_gemm.sh output
directory.  usage: python tools/pmc_summary.py gpurun_out/pmc_<shape>"""
import csv, glob, os, sys
from collections import defaultdict

root = sys.argv[1]
for var in sorted(os.listdir(root)):
    d = os.path.join(root, var)
    if not os.path.isdir(d):
        continue
    tot = defaultdict(float); disp = defaultdict(set)
    for f in glob.glob(f'{d}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if 'conv_gemm' not in r['Kernel_Name']:
                continue
            tot[r['Counter_Name']] += float(r['Counter_Value'])
            disp[r['Counter_Name']].add(r['Dispatch_Id'])
    print(f'== {var}')
    for k in sorted(tot):
        print(f'   {k:28s} {tot[k] / max(1, len(disp[k])):16.4g}')
