"""Time the narrow (N = 80) postnet GEMMs of c3 — lin (1024 -> 80), post_proj (512 -> 80),
proj2 (256 -> 80, k 3) — on the current build; prints ms per call."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

from forwardtacotron_amd import ops  # noqa: E402

torch.manual_seed(0)
B, T = 64, 1368
for name, Cin, k in (('lin', 1024, 1), ('post_proj', 512, 1), ('proj2', 256, 3)):
    x = torch.randn(B, T, Cin, device='cuda')
    w = torch.randn(80, k * Cin, device='cuda') * 0.03
    w3 = ops.presplit_for(w)
    fn = lambda: ops.conv1d(x, w, k, k // 2, w_split=w3)
    y, _ = fn()
    ref = torch.nn.functional.conv1d(x.transpose(1, 2), w.view(80, k, Cin).permute(0, 2, 1),
                                     padding=k // 2).transpose(1, 2)
    err = (y - ref).abs().max().item()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(20):
        fn()
    e.record()
    torch.cuda.synchronize()
    print(f'{name:10s} {s.elapsed_time(e) / 20:.4f} ms  max|err| {err:.2e}', flush=True)
