"""Griffin-Lim of one c2-length mel (821 frames) as gen_forward.py's griffinlim vocoder runs
it (numpy in, numpy wav out), a few times: for rocprofv3 kernel traces."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from forwardtacotron_amd.dsp import DSP  # noqa: E402
from forwardtacotron_amd.synthetic import default_config  # noqa: E402

dsp = DSP.from_config(default_config())
mel = (np.random.RandomState(0).randn(80, 821) - 4).astype(np.float32)
for i in range(5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    wav = dsp.griffinlim(mel)
    print(f'{(time.perf_counter() - t0) * 1e3:.2f} ms', flush=True)
