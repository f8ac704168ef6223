"""Condense rocprofv3 output directories into committed evidence:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats summary (copied)
  profiles/<tag>_pmc_traffic.json   per-kernel average HBM bytes per launch from the
                                    FETCH_SIZE / WRITE_SIZE passes (gfx950 correction:
                                    FETCH_SIZE x 2, MI355X_MICROARCH.md § HBM)
usage: python tools/summarize_prof.py gpurun_out/prof_<tag> <tag>     (tools/profile_round.sh
       layout: <dir>/trace, <dir>/fetch, <dir>/write)
       python tools/summarize_prof.py --stats DIR [--fetch DIR --write DIR] <tag>"""
import argparse
import csv
import glob
import json
import os
import shutil
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DST = os.path.join(ROOT, 'profiles')


def short(n):
    n = n.replace('void ', '').replace('(anonymous namespace)::', '')
    return n.split('(')[0]


def pmc(src, counter, by_grid=False):
    """average counter value per dispatch, keyed by kernel name (by_grid: 'name|grid size',
    which tells apart the shapes one kernel runs)"""
    acc, disp = defaultdict(float), defaultdict(set)
    for f in glob.glob(f'{src}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if r['Counter_Name'] != counter:
                continue
            k = short(r['Kernel_Name'])
            if by_grid:
                k = f'{k}|{r["Grid_Size"]}'
            acc[k] += float(r['Counter_Value'])
            disp[k].add((f, r['Dispatch_Id']))
    return {k: acc[k] / len(disp[k]) for k in acc}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('src', nargs='?', help='profile_round.sh directory (trace / fetch / write)')
    ap.add_argument('tag')
    ap.add_argument('--stats')
    ap.add_argument('--fetch')
    ap.add_argument('--write')
    a = ap.parse_args()
    stats_dir = a.stats or (a.src and f'{a.src}/trace')
    fetch_dir = a.fetch or (a.src and f'{a.src}/fetch')
    write_dir = a.write or (a.src and f'{a.src}/write')
    if stats_dir:
        stats = glob.glob(f'{stats_dir}/**/*kernel_stats.csv', recursive=True)
        if stats:
            shutil.copy(stats[0], os.path.join(DST, f'{a.tag}_kernel_stats.csv'))
            print('stats ->', f'profiles/{a.tag}_kernel_stats.csv')
    if not (fetch_dir and write_dir and os.path.isdir(fetch_dir) and os.path.isdir(write_dir)):
        return
    def table(fetch, write):
        out = {}
        for k in sorted(set(fetch) | set(write)):
            f = fetch.get(k)
            w = write.get(k)
            out[k] = {'fetch_size_kb_raw': f, 'read_bytes_corrected': None if f is None else f * 1024 * 2,
                      'write_bytes': None if w is None else w * 1024,
                      'hbm_bytes_per_launch': (f * 1024 * 2 if f else 0) + (w * 1024 if w else 0)}
        return out
    out = table(pmc(fetch_dir, 'FETCH_SIZE'), pmc(write_dir, 'WRITE_SIZE'))
    out_grid = table(pmc(fetch_dir, 'FETCH_SIZE', True), pmc(write_dir, 'WRITE_SIZE', True))
    json.dump({'source': [fetch_dir, write_dir],
               'units': 'FETCH_SIZE / WRITE_SIZE are KB (rocprofv3 derived); read bytes = '
                        'FETCH_SIZE x 1024 x 2 (gfx950: 128-B requests tallied at 64 B)',
               'kernels': out, 'kernels_by_grid': out_grid},
              open(os.path.join(DST, f'{a.tag}_pmc_traffic.json'), 'w'), indent=1)
    print(f'{len(out)} kernels -> profiles/{a.tag}_pmc_traffic.json')
    for k, v in sorted(out.items(), key=lambda kv: -kv[1]['hbm_bytes_per_launch'])[:15]:
        print(f'{v["hbm_bytes_per_launch"] / 1e6:10.1f} MB  {k[:110]}')


if __name__ == '__main__':
    main()
