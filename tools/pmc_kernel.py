"""Average PMC counters per dispatch of the kernels whose name contains a substring, over
every counter_collection.csv under a directory.  usage: python tools/pmc_kernel.py DIR SUBSTR"""
import collections
import csv
import glob
import sys

tot, disp = collections.defaultdict(float), collections.defaultdict(set)
for f in glob.glob(f'{sys.argv[1]}/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if sys.argv[2] in r['Kernel_Name']:
            tot[r['Counter_Name']] += float(r['Counter_Value'])
            disp[r['Counter_Name']].add((f, r['Dispatch_Id']))
for k in sorted(tot):
    print(f'{k:28s} {tot[k] / len(disp[k]):16.4g}')
