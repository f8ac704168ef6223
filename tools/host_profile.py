"""Host-side cost of one generate() on the c3 workload: wall time per phase and the Python
functions that dominate the launch path (cProfile).  Run on the GPU box."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from forwardtacotron_amd.synthetic import default_config, synthetic_state_dict, synthetic_tokens  # noqa: E402
from forwardtacotron_amd.forward_tacotron import ForwardTacotron  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    model = ForwardTacotron.from_config(default_config())
    sd = synthetic_state_dict(model, seed=0, model='forward_tacotron')
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model = model.to(dev).eval()
    x = torch.from_numpy(synthetic_tokens(64, 200, seed=0, min_len=50)).to(dev)
    for _ in range(3):
        model.generate(x)
    torch.cuda.synchronize()
    # host issue time of the whole call vs device completion
    t0 = time.perf_counter()
    model.generate(x)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f'generate: host returns after {1e3 * (t1 - t0):.3f} ms, device done after '
          f'{1e3 * (t2 - t0):.3f} ms')
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(5):
        model.generate(x)
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats('tottime').print_stats(35)
    st.sort_stats('cumulative').print_stats(45)


if __name__ == '__main__':
    main()
