"""Average PMC counters (and durations) per dispatch of the kernels matching a name filter,
from rocprofv3's sqlite output (run_results.db files under a directory).
usage: python tools/pmc_db.py <dir> [name_substring]"""
import glob
import sqlite3
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ''
    for db in sorted(glob.glob(f'{root}/**/*.db', recursive=True)):
        c = sqlite3.connect(db)
        tot, disp = defaultdict(float), defaultdict(set)
        try:
            rows = c.execute('select k.name, p.counter_name, p.counter_value, p.dispatch_id from pmc_events p '
                             'join kernels k on k.dispatch_id = p.dispatch_id').fetchall()
        except sqlite3.Error:
            rows = []
        for name, cn, cv, d in rows:
            if filt in name:
                tot[cn] += cv
                disp[cn].add(d)
        durs = [r[1] for r in c.execute('select name, duration from kernels').fetchall() if filt in r[0]]
        print(f'== {db}  ({len(durs)} dispatches, avg {sum(durs) / max(1, len(durs)) / 1e3:.1f} us)')
        for k in sorted(tot):
            print(f'   {k:28s} {tot[k] / max(1, len(disp[k])):16.6g}')


if __name__ == '__main__':
    main()
