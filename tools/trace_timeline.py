"""One generate() step from a rocprofv3 --kernel-trace CSV as a timeline: every kernel's start
offset, duration and queue, the busy union (time with at least one kernel running) and the
gaps, so the critical path of a step can be read off.  A step is the window between two
consecutive starts of the MARKER kernel (default: the decoder LSTM's rnn_bidir_kernel<1, 512>);
the window after the last marker but one is used (steady state).
usage: python tools/trace_timeline.py TRACE.csv [marker-substring] [step-index from the end]"""
import csv
import sys


def short(n):
    n = n.replace('void ', '').replace('(anonymous namespace)::', '')
    return n.split('(')[0][:64]


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else 'rnn_bidir_kernel<1, 512'
    back = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Queue_Id'],
                     r['Kernel_Name'], r['Grid_Size_X'], r['Workgroup_Size_X']))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if marker in r[3]]
    if len(marks) < back + 1:
        sys.exit(f'fewer than {back + 1} marker kernels')
    # the window: the marker's previous phoneme phase .. next step's phoneme phase: from the end
    # of the marker (back + 1) to the end of the marker (back) — one whole step in steady state
    i0, i1 = marks[-back - 1], marks[-back]
    t_lo, t_hi = rows[i0][1], rows[i1][1]
    win = [r for r in rows if r[0] >= t_lo and r[0] < t_hi]
    busy, last_end, gaps = 0, t_lo, []
    for s, e, *_ in win:
        if s > last_end:
            gaps.append((last_end - t_lo, s - last_end))
        busy += max(0, e - max(s, last_end))
        last_end = max(last_end, e)
    span = t_hi - t_lo
    print(f'window {span / 1e3:.1f} us, busy union {busy / 1e3:.1f} us, idle {(span - busy) / 1e3:.1f} us '
          f'in {len(gaps)} gaps, {len(win)} kernels')
    for s, e, q, name, g, wg in win:
        print(f'{(s - t_lo) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q:>2} grid {int(g) // int(wg):>6}  {short(name)}')
    big = sorted(gaps, key=lambda x: -x[1])[:10]
    print('largest gaps (offset us, length us):', [(round(a / 1e3, 1), round(b / 1e3, 1)) for a, b in big])


if __name__ == '__main__':
    main()
