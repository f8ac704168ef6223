"""Interleaved A/B of bench.py variants in one box session, keeping every child's evidence.

    python tools/ab_bench.py --rounds 3 --log gpurun_out/ab.jsonl \
        --variant base: --variant halves0:FTMI_BANK_HALVES=0 -- --config c2 --steps 50

A variant is NAME:VAR=VAL,VAR=VAL (empty after the colon: the default environment;
FTMI_LIB=<path> selects another build).  Each round runs every variant once, in order, as a
child `python bench.py <bench args> --no-cpu-baseline` under its own time limit.  Every
child's command, environment overrides, exit code, wall time and the tails of its stdout and
stderr go to the JSONL log whatever happens, and a child that fails — non-zero exit, or no
JSON line on stdout — is reported with its exit code and stderr tail, and ends the A/B (a
GPU fault or abort must not be followed by more GPU work).  Replaces the round-1..3 shell
A/B loops, which discarded the children's stderr (the empty c3 legs of a round-3 A/B could
not be told apart from a script error afterwards)."""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def parse_variant(spec: str):
    name, _, rest = spec.partition(':')
    env = {}
    for kv in filter(None, rest.split(',')):
        k, _, v = kv.partition('=')
        env[k] = v
    return name, env


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--variant', action='append', required=True)
    ap.add_argument('--log', default=os.path.join(ROOT, 'gpurun_out', 'ab_bench.jsonl'))
    ap.add_argument('--timeout', type=int, default=300)
    ap.add_argument('--key', default='ms_per_step', help='bench line field to report')
    ap.add_argument('bench_args', nargs=argparse.REMAINDER)
    a = ap.parse_args()
    args = [x for x in a.bench_args if x != '--']
    if '--no-cpu-baseline' not in args:
        args.append('--no-cpu-baseline')
    variants = [parse_variant(v) for v in a.variant]
    os.makedirs(os.path.dirname(a.log), exist_ok=True)
    cmd = [sys.executable, '-u', os.path.join(ROOT, 'bench.py'), *args]
    results = {n: [] for n, _ in variants}
    with open(a.log, 'a') as log:
        for r in range(a.rounds):
            for name, env in variants:
                t0 = time.time()
                try:
                    p = subprocess.run(cmd, env={**os.environ, **env}, capture_output=True,
                                       text=True, timeout=a.timeout, cwd=ROOT)
                    rc, out, err = p.returncode, p.stdout, p.stderr
                except subprocess.TimeoutExpired as e:
                    rc = 'timeout'
                    out = (e.stdout or b'').decode() if isinstance(e.stdout, bytes) else (e.stdout or '')
                    err = (e.stderr or b'').decode() if isinstance(e.stderr, bytes) else (e.stderr or '')
                line = None
                for s in reversed(out.strip().splitlines()):
                    if s.startswith('{'):
                        try:
                            line = json.loads(s)
                            break
                        except json.JSONDecodeError:
                            pass
                rec = {'round': r, 'variant': name, 'env': env, 'cmd': cmd, 'rc': rc,
                       'wall_s': round(time.time() - t0, 2), 'stdout_tail': out[-2000:],
                       'stderr_tail': err[-4000:], 'line': line}
                log.write(json.dumps(rec) + '\n')
                log.flush()
                if rc != 0 or line is None:
                    print(f'{name} (round {r}) FAILED: rc={rc}, '
                          f'{"no JSON line on stdout" if line is None else ""}\n'
                          f'cmd: {" ".join(cmd)}\nenv: {env}\n--- stderr tail ---\n{err[-3000:]}',
                          flush=True)
                    sys.exit(1)
                v = line.get(a.key)
                results[name].append(v)
                print(f'round {r} {name:16s} {a.key} {v}', flush=True)
    for name, vs in results.items():
        print(f'{name:16s} min {min(vs)} all {vs}')


if __name__ == '__main__':
    main()
