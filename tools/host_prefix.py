"""Host time from generate() entry to the first launches of the prenet chain at c3 (the
step-start window in which the device idles), per call, without a profiler."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from forwardtacotron_amd import ops  # noqa: E402
from forwardtacotron_amd.synthetic import default_config, synthetic_state_dict, synthetic_tokens  # noqa: E402
from forwardtacotron_amd.forward_tacotron import ForwardTacotron  # noqa: E402

marks = []


def wrap(name):
    f = getattr(ops, name)

    def g(*a, **k):
        marks.append((name + '>', time.perf_counter()))
        r = f(*a, **k)
        marks.append((name + '<', time.perf_counter()))
        return r
    setattr(ops, name, g)


for n in ('embedding', 'conv_bank', 'conv1d', 'run_checked', 'status_word'):
    wrap(n)
dev = torch.device('cuda', 0)
model = ForwardTacotron.from_config(default_config())
sd = synthetic_state_dict(model, seed=0, model='forward_tacotron')
model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
model = model.to(dev).eval()
x = torch.from_numpy(synthetic_tokens(64, 200, seed=0, min_len=50)).to(dev)
for _ in range(3):
    model.generate(x)
torch.cuda.synchronize()
for rep in range(3):
    marks.clear()
    t0 = time.perf_counter()
    model.generate(x)
    t1 = time.perf_counter()
    seen = {}
    for name, t in marks:
        if name not in seen:
            seen[name] = t
    print(f'call {rep}: total {1e3 * (t1 - t0):.3f} ms; first marks (us from entry): ' +
          ', '.join(f'{k} {1e6 * (v - t0):.0f}' for k, v in sorted(seen.items(), key=lambda kv: kv[1])))
