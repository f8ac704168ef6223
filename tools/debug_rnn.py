"""Debug: GRU recurrence step 1 vs hypotheses (run on the GPU box)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from forwardtacotron_amd import ops, _lib
from oracle import ft_oracle as O

rng = np.random.Generator(np.random.PCG64(5))
H, B, T = int(sys.argv[1]) if len(sys.argv) > 1 else 64, 1, 3
G = 3
w_hh = rng.normal(0, 1 / np.sqrt(H), (2, G * H, H)).astype(np.float32)
b_hh = rng.normal(0, 0.1, (2 * G * H,)).astype(np.float32)
xp = rng.normal(0, 1, (B, T, 2 * G * H)).astype(np.float32)
y = ops.rnn_bidir(0, torch.from_numpy(xp).cuda(), H, torch.from_numpy(w_hh).cuda(),
                  torch.from_numpy(b_hh).cuda(), check=True)
y = y.cpu().numpy()

def sig(x): return 1 / (1 + np.exp(-x))
def step(h, gx, W, bh):
    gh = W @ h + bh
    r = sig(gx[:H] + gh[:H]); z = sig(gx[H:2*H] + gh[H:2*H]); n = np.tanh(gx[2*H:] + r * gh[2*H:])
    return n + z * (h - n)
h0 = step(np.zeros(H, np.float32), xp[0, 0, :G*H], w_hh[0], b_hh[:G*H])
print('t0 err', np.abs(y[0, 0, :H] - h0).max())
h1 = step(h0, xp[0, 1, :G*H], w_hh[0], b_hh[:G*H])
print('t1 correct err', np.abs(y[0, 1, :H] - h1).max())
print('t1 if h_prev=0 err', np.abs(y[0, 1, :H] - step(np.zeros(H, np.float32), xp[0, 1, :G*H], w_hh[0], b_hh[:G*H])).max())
print('t1 if W transposed-blocks err', np.abs(y[0, 1, :H] - step(h0, xp[0, 1, :G*H], w_hh[0].reshape(G, H, H).transpose(0, 2, 1).reshape(G*H, H), b_hh[:G*H])).max())
# recover the effective recurrent contribution from r/z/n is hard; print a few values
print('got', y[0, 1, :8]); print('want', h1[:8])
