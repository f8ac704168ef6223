"""Summarise a rocprofv3 --kernel-trace CSV: per-kernel totals and the timeline of the last
generate() step (start offset, duration, overlap).  usage: python tools/timeline.py <dir>
[marker]: with a marker (a kernel-name substring launched once per step, e.g.
duration_counts_kernel for FastPitch) the window between its last two launches is shown
instead of the ForwardTacotron LSTM-based step."""
import csv, glob, sys
from collections import defaultdict

path = sorted(glob.glob(f'{sys.argv[1]}/**/*kernel_trace.csv', recursive=True))[-1]
rows = list(csv.DictReader(open(path)))
for r in rows:
    r['s'] = int(r['Start_Timestamp']); r['e'] = int(r['End_Timestamp'])
rows.sort(key=lambda r: r['s'])
name = lambda r: r['Kernel_Name'].replace('void ', '').replace('(anonymous namespace)::', '').split('(')[0][:70]
# steps: the LSTM kernel marks each generate(); take the window between the last two
if len(sys.argv) > 2:
    marks = [i for i, r in enumerate(rows) if sys.argv[2] in r['Kernel_Name']]
    a, b = marks[-2], marks[-1]
    t0 = rows[a]['s']
    print(f'window between the last two {sys.argv[2]}: {b - a} kernels, '
          f'wall {(rows[b]["s"] - t0) / 1e6:.3f} ms')
    tot = defaultdict(float)
    for r in rows[a:b]:
        tot[name(r)] += (r['e'] - r['s']) / 1e3
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:25]:
        print(f'   {v:9.1f} us  {k}')
    for r in rows[a:b]:
        print(f'   {(r["s"] - t0) / 1e3:9.1f} us  +{(r["e"] - r["s"]) / 1e3:8.1f} us  q{r.get("Queue_Id", "?"):>3}  {name(r)}')
    sys.exit(0)
marks = [i for i, r in enumerate(rows) if 'rnn_bidir_kernel<1' in r['Kernel_Name']]
if len(marks) >= 2:
    # one whole step: from the first embedding after an LSTM to the first embedding after the
    # next LSTM.  With three or more LSTMs the second-to-last step (bench.py's last traced
    # pass is the eager per-kernel probe, followed by the prenet-bank timing calls)
    i0, i1 = (marks[-3], marks[-2]) if len(marks) >= 3 else (marks[-2], None)
    starts = [i for i in range(i0 + 1, len(rows)) if 'embedding' in rows[i]['Kernel_Name']]
    a = starts[0] if starts else i0 + 1
    ends = [i for i in range(i1 + 1, len(rows)) if 'embedding' in rows[i]['Kernel_Name']] if i1 else []
    b = ends[0] if ends else len(rows)
    t0 = rows[a]['s']
    print(f'step: {len(rows[a:b])} kernels, wall {(max(r["e"] for r in rows[a:b]) - t0) / 1e6:.3f} ms')
    busy = 0; last = t0
    for r in rows[a:b]:
        s, e = max(r['s'], last), r['e']
        if e > s: busy += e - s
        last = max(last, e)
    print(f'   device busy (union) {busy / 1e6:.3f} ms')
    for r in rows[a:b]:
        print(f'   {(r["s"] - t0) / 1e3:9.1f} us  +{(r["e"] - r["s"]) / 1e3:8.1f} us  q{r.get("Queue_Id", "?"):>3}  {name(r)}')
