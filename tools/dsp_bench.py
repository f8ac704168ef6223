"""Throughput of the audio path (utils/dsp.py on HIP) at c3 shapes: wav_to_mel and the
Griffin-Lim vocoder (mel_to_stft NNLS + 32 fast-GL iterations) for a batch of 64
utterances of T_mel frames; the librosa-0.7.2 numpy oracle on one utterance is the CPU
reference point.  usage: python tools/dsp_bench.py [--batch 64 --frames 1368]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forwardtacotron_amd import dsp as G  # noqa: E402
from forwardtacotron_amd.probe import KernelProbe  # noqa: E402
from forwardtacotron_amd.synthetic import default_config  # noqa: E402


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=64)
    ap.add_argument('--frames', type=int, default=1368)
    ap.add_argument('--cpu-frames', type=int, default=200)
    a = ap.parse_args()
    dsp = G.DSP.from_config(default_config())
    plan = dsp.plan()
    B, F = a.batch, a.frames
    L = 256 * (F - 1)
    rng = np.random.RandomState(0)
    t = np.arange(L) / 22050.0
    wav = (0.3 * np.sin(2 * np.pi * 180 * t)[None] + 0.05 * rng.randn(B, L)).astype(np.float32)
    y = torch.from_numpy(wav).cuda()
    res = {}
    with KernelProbe() as pr:
        dt, mel = timed(lambda: G.mel_spectrogram(plan, y))
    res['wav_to_mel'] = {'frames_per_s': round(B * mel.shape[2] / dt, 1), 'ms': round(dt * 1e3, 3),
                         'kernels': {k: round(v['avg_ms'], 4) for k, v in pr.summary().items()}}
    with KernelProbe() as pr:
        dt, (w, n) = timed(lambda: dsp.griffinlim_batch(mel, n_iter=32), reps=1)
    res['griffinlim'] = {'frames_per_s': round(B * F / dt, 1), 'ms': round(dt * 1e3, 3),
                         'kernels': {k: {'n': v['launches'], 'avg_ms': round(v['avg_ms'], 4),
                                         'GB/s': round(v['bytes'] / (v['avg_ms'] / 1e3) / 1e9, 1)}
                                     for k, v in pr.summary().items()}}
    # CPU reference point: the librosa 0.7.2 restatement (numpy / scipy) on one utterance
    from oracle import dsp_oracle as D
    m1 = mel[0, :, :a.cpu_frames].cpu().numpy()
    ang = D.random_angles((513, a.cpu_frames), 0)
    t0 = time.perf_counter()
    D.griffinlim(m1, ang)
    dc = time.perf_counter() - t0
    t0 = time.perf_counter()
    D.wav_to_mel(wav[0, :256 * (a.cpu_frames - 1)])
    dm = time.perf_counter() - t0
    res['cpu_oracle'] = {'griffinlim_frames_per_s': round(a.cpu_frames / dc, 1),
                         'wav_to_mel_frames_per_s': round(a.cpu_frames / dm, 1),
                         'sample': f'one utterance of {a.cpu_frames} frames, oracle/dsp_oracle.py'}
    res['config'] = {'batch': B, 'frames': F, 'n_fft': 1024, 'hop': 256, 'n_mels': 80,
                     'gl_iters': 32, 'nnls_iters': dsp.nnls_iters}
    print(json.dumps(res))


if __name__ == '__main__':
    main()
