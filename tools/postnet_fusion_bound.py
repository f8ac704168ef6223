"""Measured bound on fusing the c3 postnet bank with proj1: what the
717 MB intermediate (the pooled bank output, f16x3 split rows, B 64 x T_mel 1368 x 2048
channels) costs the two kernels that write and read it.  In the diagnostic library
(FTMI_SLAB_DIAG, results invalid when set, read per launch):
  bank  (conv_bank_walk_kernel)  0 = as shipped, 8 = no epilogue stores (the intermediate
        is never written: what a fused kernel that keeps it on chip would not pay)
  proj1 (conv_gemm_slab_kernel)  0 = as shipped, 4 = no global loads in the main loop (the
        operand, AND its weights, never fetched: more than a fusion could save)
The sum of the two savings bounds what ANY bank -> proj1 fusion can gain (it still has to
do both kernels' MFMAs, staging and epilogues).  HIP events around 20 back-to-back calls,
5 interleaved rounds, median per call.
usage: FTMI_LIB=forwardtacotron_amd/libftmi_diag.so python tools/postnet_fusion_bound.py"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forwardtacotron_amd import ops  # noqa: E402


def timed(fn, n=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


def main():
    B, T, Cin, K, C = 64, 1368, 80, 8, 256
    g = torch.Generator().manual_seed(0)
    x = torch.randn(B, T, Cin, generator=g).cuda()
    w = (torch.randn(C * Cin * K * (K + 1) // 2, generator=g) * 0.05).cuda()
    sc = torch.rand(K * C, generator=g).cuda() + 0.5
    sh = torch.randn(K * C, generator=g).cuda() * 0.1
    w3 = ops.split_bank_weights(w, K, Cin, C, 2)
    wp = (torch.randn(C, 3 * K * C, generator=g) * 0.02).cuda()
    wp3 = ops.presplit_for(wp, 2)
    bank = lambda: ops.conv_bank(x, w, K, C, sc, sh, mma=2, w_split=w3, pool=True, split_out=True)  # noqa: E731
    inter = bank()
    proj1 = lambda: ops.conv1d(inter, wp, 3, 1, relu=True, w_split=wp3, mma=2, x_split=True)  # noqa: E731
    cases = [('bank', bank, '0'), ('bank', bank, '8'), ('proj1', proj1, '0'), ('proj1', proj1, '4')]
    res = {f'{n}:{d}': [] for n, _, d in cases}
    for _ in range(5):
        for n, fn, d in cases:
            os.environ['FTMI_SLAB_DIAG'] = d
            res[f'{n}:{d}'].append(timed(fn))
    os.environ['FTMI_SLAB_DIAG'] = '0'
    med = {k: round(statistics.median(v), 4) for k, v in res.items()}
    save_bank = med['bank:0'] - med['bank:8']
    save_proj = med['proj1:0'] - med['proj1:4']
    out = {'ms': med, 'intermediate_bytes': inter.numel() * inter.element_size(),
           'bank_store_cost_ms': round(save_bank, 4), 'proj1_operand_fetch_cost_ms': round(save_proj, 4),
           'fusion_gain_bound_ms': round(save_bank + save_proj, 4),
           'target_ms': 0.2}
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
