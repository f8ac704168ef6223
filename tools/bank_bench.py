"""c2 prenet bank (B = 1, T = 120, K = 16, Cin = Cout = 256) on the channel-split bank
schedules: the one-launch channel-halves kernel (default; halves-image: reading the
stream-order weight image), group pairs per block or
quarter-balanced waves (FTMI_BANK_QB=1), each finished by the finish launch or in-kernel by
each tile's last split block (FTMI_BANK_LAST=1).  HIP events over back-to-back calls ('warm': the weight planes stay
Infinity-Cache resident, as in a generate() loop) and per call behind a 512 MiB overwrite
('cold'); max |d| against the first variant.  Run under rocprofv3 --kernel-trace --stats
for the kernel durations.  usage: python tools/bank_bench.py [T] [reps] [variant ...]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forwardtacotron_amd import ops  # noqa: E402
from forwardtacotron_amd.common_layers import pack_conv  # noqa: E402

VARIANTS = {'halves': {'FTMI_BANK_HALVES': '1'},
            'halves-image': {'FTMI_BANK_HALVES': '1'},  # + the stream-order weight image
            'pairs+finish': {'FTMI_BANK_HALVES': '0', 'FTMI_BANK_QB': '0', 'FTMI_BANK_LAST': '0'},
            'pairs+last': {'FTMI_BANK_HALVES': '0', 'FTMI_BANK_QB': '0', 'FTMI_BANK_LAST': '1'},
            'qb+finish': {'FTMI_BANK_HALVES': '0', 'FTMI_BANK_QB': '1', 'FTMI_BANK_LAST': '0'},
            'qb+last': {'FTMI_BANK_HALVES': '0', 'FTMI_BANK_QB': '1', 'FTMI_BANK_LAST': '1'}}


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 120
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    names = sys.argv[3:] or list(VARIANTS)
    rng = np.random.Generator(np.random.PCG64(0))
    B, C, K = 1, 256, 16
    x = torch.from_numpy(rng.normal(0, 1, (B, T, C)).astype(np.float32)).cuda()
    ws = [rng.normal(0, 1 / np.sqrt(C * k), (C, C, k)).astype(np.float32) for k in range(1, K + 1)]
    wp = torch.cat([pack_conv(torch.from_numpy(w)).reshape(-1) for w in ws]).cuda()
    w3 = ops.split_bank_weights(wp, K, C, C, 2)
    img = ops.bank_halves_image(w3, K, C, C)
    sc = torch.from_numpy(rng.uniform(0.5, 1.5, K * C).astype(np.float32)).cuda()
    sh = torch.from_numpy(rng.normal(0, 0.1, K * C).astype(np.float32)).cuda()
    nbytes = 4.0 * (B * T * C + C * C * K * (K + 1) / 2 + B * T * K * C)
    flush = torch.empty(512 << 20, dtype=torch.uint8, device='cuda')
    ref = None
    for name in names:
        os.environ.update(VARIANTS[name])
        wi = img if name.endswith('-image') else None
        fn = lambda: ops.conv_bank(x, wp, K, C, sc, sh, mma=2, w_split=w3, w_image=wi)  # noqa: E731
        for _ in range(5):
            y = fn()
        torch.cuda.synchronize()
        got = y.cpu().numpy()
        ref = got if ref is None else ref
        d = float(np.abs(got - ref).max())
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        warm = a.elapsed_time(b) / reps
        # the same calls replayed from a HIP graph: device time without the host's
        # per-call issue cost (ctypes + argument packing)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        graph = a.elapsed_time(b) / reps
        cold = 0.0
        for _ in range(10):
            flush.fill_(1)
            a.record()
            fn()
            b.record()
            torch.cuda.synchronize()
            cold += a.elapsed_time(b) / 10
        print(f'{name:13s} T={T}: warm {warm * 1e3:6.1f} us ({nbytes / warm / 1e6:6.0f} GB/s, '
              f'{nbytes / warm / 1e6 / 8000:.1%} of HBM) | graph {graph * 1e3:6.1f} us '
              f'({nbytes / graph / 1e6 / 8000:.1%}) | cold {cold * 1e3:6.1f} us '
              f'({nbytes / cold / 1e6:6.0f} GB/s) | max|d| vs {names[0]} {d:.2e}', flush=True)


if __name__ == '__main__':
    main()
