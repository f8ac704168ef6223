"""The FastPitch c5 mel-decoder contractions (B 64, T 1400, d_model 256, d_fft 1024) timed
one by one on each GEMM kernel the dispatcher can pick: the slab kernel (default), the x6b
kernel (FTMI_GEMM_SLAB_MIN above the shape's MACs) and the slab kernel's 512/768-thread
forms.  usage (GPU box): python tools/fp_gemm_ab.py [rounds]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forwardtacotron_amd import ops  # noqa: E402

B, T, D, F = 64, 1400, 256, 1024
SHAPES = {  # name: (Cin, N, k, relu, residual)
    'qkv': (D, 3 * D, 1, False, False),
    'out_proj': (D, D, 1, False, True),
    'conv1': (D, F, 9, True, False),
    'conv2': (F, D, 1, False, True),
}


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    torch.manual_seed(0)
    M = B * T
    for _ in range(rounds):
        for name, (cin, n, k, relu, res) in SHAPES.items():
            x = torch.randn(B, T, cin, device='cuda')
            w = torch.randn(n, k * cin, device='cuda') / (k * cin) ** 0.5
            bias = torch.randn(n, device='cuda') * 0.1
            r = torch.randn(B, T, n, device='cuda') if res else None
            w3 = ops.presplit_for(w)
            fn = lambda: ops.conv1d(x, w, k, k // 2, bias=bias, relu=relu, residual=r, w_split=w3)  # noqa
            fl = 2.0 * M * n * k * cin
            by = 4.0 * (M * cin + M * n * (2 if res else 1))
            line = []
            for tag, env in (('slab', {}), ('x6b', {'FTMI_GEMM_SLAB_MIN': str(10 ** 15)})):
                for kk, v in env.items():
                    os.environ[kk] = v
                t = timed(fn)
                for kk in env:
                    del os.environ[kk]
                line.append(f'{tag} {t:7.1f} us {fl / t / 1e6:6.1f} TF {by / t / 1e3:6.0f} GB/s')
            if k == 1:  # the row-panel launch, with norm for the N = d outputs
                wf = ops.split_weights_f16(w, frag=True)
                ln = (torch.ones(n, device='cuda'), torch.zeros(n, device='cuda'), 1e-5) \
                    if n == D else None
                t = timed(lambda: ops.panel_proj(x, wf, n, bias=bias, residual=r, ln=ln))
                line.append(f'panel{"+ln" if ln else ""} {t:7.1f} us {fl / t / 1e6:6.1f} TF '
                            f'{by / t / 1e3:6.0f} GB/s')
                if ln:
                    t = timed(lambda: ops.layernorm(r, ln[0], ln[1], 1e-5))
                    line.append(f'(layernorm alone {t:5.1f} us)')
            print(f'{name:9s} ' + ' | '.join(line), flush=True)


if __name__ == '__main__':
    main()
