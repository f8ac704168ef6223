"""Condense a tools/profile_round.sh output directory into committed evidence:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats summary (copied)
  profiles/<tag>_pmc_traffic.json   per-kernel average HBM bytes per launch from the
                                    FETCH_SIZE / WRITE_SIZE passes (gfx950 correction:
                                    FETCH_SIZE x 2, MI355X_MICROARCH.md § HBM)
usage: python tools/summarize_prof.py gpurun_out/prof_<tag> <tag>"""
import csv, glob, json, os, shutil, sys
from collections import defaultdict

src, tag = sys.argv[1], sys.argv[2]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(ROOT, 'profiles')
stats = glob.glob(f'{src}/trace/**/*kernel_stats.csv', recursive=True)
if stats:
    shutil.copy(stats[0], os.path.join(dst, f'{tag}_kernel_stats.csv'))


def short(n):
    n = n.replace('void ', '').replace('(anonymous namespace)::', '')
    return n.split('(')[0]


def pmc(sub, counter):
    acc, cnt = defaultdict(float), defaultdict(int)
    for f in glob.glob(f'{src}/{sub}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if r['Counter_Name'] != counter:
                continue
            k = short(r['Kernel_Name'])
            acc[k] += float(r['Counter_Value'])
            cnt[k] += 1
    return {k: acc[k] / cnt[k] for k in acc}


fetch, write = pmc('fetch', 'FETCH_SIZE'), pmc('write', 'WRITE_SIZE')
out = {}
for k in sorted(set(fetch) | set(write)):
    f = fetch.get(k)
    w = write.get(k)
    out[k] = {'fetch_size_kb_raw': f, 'read_bytes_corrected': None if f is None else f * 1024 * 2,
              'write_bytes': None if w is None else w * 1024,
              'hbm_bytes_per_launch': (f * 1024 * 2 if f else 0) + (w * 1024 if w else 0)}
json.dump({'source': src, 'units': 'FETCH_SIZE / WRITE_SIZE are KB (rocprofv3 derived); '
           'read bytes = FETCH_SIZE x 1024 x 2 (gfx950: 128-B requests tallied at 64 B)',
           'kernels': out}, open(os.path.join(dst, f'{tag}_pmc_traffic.json'), 'w'), indent=1)
print(f'{len(out)} kernels')
for k, v in sorted(out.items(), key=lambda kv: -kv[1]['hbm_bytes_per_launch'])[:15]:
    print(f'{v["hbm_bytes_per_launch"] / 1e6:10.1f} MB  {k[:110]}')
