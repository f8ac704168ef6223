"""Device L-BFGS-B NNLS (csrc/nnls.hip) vs scipy and vs the numpy restatement
(tools/lbfgsb_np.py), GPU run:
    python tools/nnls_diag.py [rand]          per iteration (maxiter = 1, 2, ...)
    python tools/nnls_diag.py state IT [rand]  the state before FREEV / SUBSM / EVAL of
                                               iteration IT against the restatement's"""
import json
import sys
from pathlib import Path

import numpy as np
import scipy.optimize
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / 'tools'))
from oracle import dsp_oracle as D  # noqa: E402
from forwardtacotron_amd import dsp as G  # noqa: E402
import lbfgsb_np  # noqa: E402

PH = {'EVAL': 1, 'CAUCHY': 2, 'WALK': 3, 'FREEV': 4, 'FORMK': 5, 'SUBSM': 6}


def regions(n_pad, m, groups):
    """csrc/nnls.hip carve(): name -> byte offset"""
    al = lambda b: (b + 255) // 256 * 256  # noqa: E731
    ns = 6 * ((m + 7) // 8 * 8) + 16
    sizes = [('st', 376)] + [(k, 8 * n_pad) for k in ('X0', 'X1', 'G0', 'G1', 'Z', 'DD', 'R')] + [
        ('WS', 8 * n_pad * m), ('WY', 8 * n_pad * m), ('BKEY', 8 * n_pad), ('BIDX', 4 * n_pad),
        ('CHG', 4 * n_pad), ('IW', n_pad), ('PF', n_pad)] + [(k, 8 * m * m) for k in ('SY', 'SS', 'WT')] + [
        (k, 8 * 4 * m * m) for k in ('WN1', 'WN')] + [(k, 8 * 2 * m) for k in ('P', 'C', 'WA', 'WV', 'V', 'WBP')] + [
        ('NEWROW', 8 * 4 * m), ('PART', 8 * groups * ns), ('DELTA', 8 * 6 * m * m)]
    off, o = {}, 0
    for k, sz in sizes:
        off[k] = o
        o += al(sz)
    return off


DBL = ['f', 'fold', 'sbgnrm', 'theta', 'f1', 'f2', 'f2_org', 'dtm', 'tsum', 'tj', 'stp', 'dtd', 'dnorm',
       'stpmx', 'gd', 'gdold', 'rr', 'dr', 'alpha']
INT = ['phase', 'it', 'col', 'iupdat', 'updatd', 'pending', 'nbreak', 'nfree_c', 'bnded', 'kpassed',
       'nfree', 'nenter', 'nleave', 'iword', 'ibd', 'ifun', 'ls_brackt', 'ls_stage', 'cur', 'status',
       'nfev', 'nskip', 'nseg', 'walk_done', 'bk_count', 'backtrack']


def decode(dbg, nb, nc):
    ws = dbg['ws'].cpu().numpy()
    off = regions(dbg['n_pad'], dbg['m'], dbg['groups'])
    n = nb * nc
    st = {k: float(np.frombuffer(ws[8 * i:8 * i + 8].tobytes(), np.float64)[0]) for i, k in enumerate(DBL)}
    st.update({k: int(np.frombuffer(ws[264 + 4 * i:268 + 4 * i].tobytes(), np.int32)[0]) for i, k in enumerate(INT)})
    vec = lambda k: np.frombuffer(ws[off[k]:off[k] + 8 * n].tobytes(), np.float64).reshape(nc, nb).T.ravel()  # noqa: E731
    small = lambda k, cnt: np.frombuffer(ws[off[k]:off[k] + 8 * cnt].tobytes(), np.float64)  # noqa: E731
    iw = np.frombuffer(ws[off['IW']:off['IW'] + n].tobytes(), np.int8).reshape(nc, nb).T.ravel()
    cur = st['cur']
    x, g = vec(f'X{cur}'), vec(f'G{cur}')
    return st, dict(x=x, g=g, Z=vec('Z'), R=vec('R'), IW=iw, P=small('P', 2 * st['col']),
                    C=small('C', 2 * st['col']), WA=small('WA', 2 * st['col']), WV=small('WV', 2 * st['col']))


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb else 1.0)


def main():
    cfg = json.loads((ROOT / 'tests/golden/dsp_config.json').read_text())
    dsp = G.DSP.from_config(cfg)
    plan = dsp.plan()
    args = sys.argv[1:]
    mel = np.load(ROOT / 'tests/golden/ref_test_mel.npy')
    if 'rand' in args:
        mel = (np.random.RandomState(5).randn(80, 24) * 2 - 3).astype(np.float32)
        args.remove('rand')
    A = D.mel_filters(22050, 1024, 80, 0, 8000)
    M = np.exp(mel).astype(np.float32)
    x0 = np.clip(np.linalg.lstsq(A, M, rcond=None)[0], 0, None)
    md = torch.from_numpy(np.ascontiguousarray(M)).cuda()[None]  # numpy's exp, as the reference
    nb, nc = 513, mel.shape[1]
    if args and args[0] == 'state':
        it = int(args[1])
        snap = {it: {}}
        lbfgsb_np.lbfgsb(A, M, x0, snap=snap)
        ref = snap[it]
        for ph in ('FREEV', 'SUBSM', 'EVAL'):
            dbg = {'stop': 16 * it + PH[ph]}
            G._nnls_lbfgsb(plan, md, None, False, debug=dbg)
            st, v = decode(dbg, nb, nc)
            print(f'--- before {ph} (it {it}): state', {k: st[k] for k in ('it', 'col', 'nfree', 'nenter', 'nleave', 'nbreak', 'kpassed', 'walk_done', 'nfev', 'theta', 'tsum', 'dtm', 'stp', 'f')}, flush=True)
            if ph == 'FREEV':
                iwd = v['IW']
                xcp = np.where(iwd == 1, 0.0, np.where(iwd == 0, v['x'] - st['tsum'] * v['g'], v['x']))
                print(f'  xcp rel {rel(xcp, ref["xcp"]):.3e}  iwhere mismatches {(iwd != ref["iwhere"]).sum()}  '
                      f'nbreak ref {ref["nbreak"]}  tsum ref {ref["tsum"]:.16e} dev {st["tsum"]:.16e}')
                print(f'  c rel {rel(v["C"], ref["c"]):.3e}  p rel {rel(v["P"], ref["p"]):.3e}  theta ref {ref["theta"]!r} dev {st["theta"]!r}')
            if ph == 'SUBSM' and 'r' in ref:
                print(f'  r rel {rel(v["R"], ref["r"]):.3e}  wa rel {rel(v["WA"], ref["wa"]):.3e}')
                wvs = lbfgsb_np._solve_upper(ref['wn_f'], np.concatenate([-lbfgsb_np._solve_upper_T(ref['wn_f'], ref['wv_raw'])[:st['col']], lbfgsb_np._solve_upper_T(ref['wn_f'], ref['wv_raw'])[st['col']:]]))
                print(f'  wv (solved) rel {rel(v["WV"], wvs):.3e}  dev {v["WV"]}  ref {wvs}')
            if ph == 'EVAL':
                print(f'  z rel {rel(v["Z"], ref["z"]):.3e}')
        return
    import time
    its = [1, 2, 3, 5, 10, 20, 31, 33, 40, 60, 15000] if 'rand' in sys.argv else list(range(1, 10)) + [15000]
    for k in its:
        xs, f, d = scipy.optimize.fmin_l_bfgs_b(D._nnls_obj, x0, args=(x0.shape, A, M),
                                                bounds=[(0, None)] * x0.size, m=A.shape[1], maxiter=k)
        info = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        S = G._nnls_lbfgsb(plan, md, None, False, maxiter=k, info=info)[0].cpu().numpy().T
        dt = time.perf_counter() - t0
        ref = xs.reshape(x0.shape)
        print(f'maxiter {k}: rel {rel(S, ref):.3e}  scipy nit {d["nit"]} nfev {d["funcalls"]} f {f:.10e} | '
              f'device {info[0]}  {dt * 1e3:.1f} ms', flush=True)


if __name__ == '__main__':
    main()
