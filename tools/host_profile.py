"""Host-side cost of one generate() call at c3 (or c2): cProfile of a few calls after warm-up,
with the device kept ahead (no sync inside the profiled region except generate()'s own), so the
Python / ctypes time per launch on the phoneme phase's critical chain shows.
usage: python tools/host_profile.py [c3|c2] (GPU box)"""
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from forwardtacotron_amd.forward_tacotron import ForwardTacotron  # noqa: E402
from forwardtacotron_amd.synthetic import default_config, synthetic_state_dict, synthetic_tokens  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else 'c3'
    B, tmin, tmax = (64, 50, 200) if cfg == 'c3' else (1, 120, 120)
    dev = torch.device('cuda')
    model = ForwardTacotron.from_config(default_config())
    sd = synthetic_state_dict(model, seed=0, model='forward_tacotron')
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model = model.to(dev).eval()
    x = torch.from_numpy(synthetic_tokens(B, tmax, seed=0, min_len=tmin)).to(dev)
    for _ in range(3):
        model.generate(x)
    torch.cuda.synchronize()
    n = 5
    t0 = time.perf_counter()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        model.generate(x)
    pr.disable()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    s = io.StringIO()
    st = pstats.Stats(pr, stream=s)
    st.sort_stats('tottime').print_stats(30)
    st.sort_stats('cumulative').print_stats(45)
    print(f'{cfg}: {dt * 1e3:.3f} ms per call (wall, profiled)')
    print(s.getvalue())


if __name__ == '__main__':
    main()
