"""Griffin-Lim iteration timing at BASELINE sizes (GPU): the fused one-launch iteration
(ftmi_griffinlim_iter) against the three-kernel path (FTMI_GL_FUSED=0), HIP events over a
32-iteration griffinlim_from_stft, and the NNLS (both solvers) on the same batch.
    python tools/gl_bench.py [B] [F]     (default c5: 64 x 1400)"""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from forwardtacotron_amd import dsp as G  # noqa: E402


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e))
    return best


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    F = int(sys.argv[2]) if len(sys.argv) > 2 else 1400
    cfg = json.loads((ROOT / 'tests/golden/dsp_config.json').read_text())
    dsp = G.DSP.from_config(cfg)
    plan = dsp.plan()
    g = torch.Generator(device='cuda')
    g.manual_seed(0)
    S = torch.rand(B, F, plan.nb, device='cuda', generator=g) * 2
    u = torch.rand(B, F, plan.nb, dtype=torch.float64, device='cuda', generator=g)
    ang = torch.polar(torch.ones_like(u), u * 6.283185307179586).to(torch.complex64)
    out = {'B': B, 'F': F}
    if os.environ.get('GL_BENCH_PROF'):
        # profiling run: the fused iteration only (rocprofv3 --pmc)
        for _ in range(3):
            G.griffinlim_from_stft(plan, S, ang, 8)
        torch.cuda.synchronize()
        print(json.dumps(out), flush=True)
        return
    for fused in ('1', '0'):
        os.environ['FTMI_GL_FUSED'] = fused
        ms = timed(lambda: G.griffinlim_from_stft(plan, S, ang, 32))
        out['gl32_ms_fused' if fused == '1' else 'gl32_ms_unfused'] = round(ms, 3)
    os.environ['FTMI_GL_FUSED'] = '1'
    bytes_iter = 36.0 * S.numel()
    out['iter_ms_fused'] = round(out['gl32_ms_fused'] / 33, 4)  # 32 iterations + the final istft
    out['hbm_frac_fused'] = round(bytes_iter / (out['iter_ms_fused'] / 1e3) / 8e12, 4)
    a = G.griffinlim_from_stft(plan, S, ang, 4)
    os.environ['FTMI_GL_FUSED'] = '0'
    b = G.griffinlim_from_stft(plan, S, ang, 4)
    os.environ['FTMI_GL_FUSED'] = '1'
    out['fused_vs_unfused_max_abs'] = float((a - b).abs().max())
    out['fused_vs_unfused_peak'] = float(b.abs().max())
    # the NNLS on a speech-like batch
    mel = torch.log(torch.clamp(torch.rand(B, plan.n_mels, F, device='cuda', generator=g), min=1e-5))
    out['nnls_fista_ms'] = round(timed(lambda: G.mel_to_stft(plan, mel, method='fista'), 2), 3)
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
