"""Ground-truth-aligned (GTA) mel export: the caller of the teacher-forced `forward()` path
(`train_forward.py:33-50`, create_gta_features) and the batch format it consumes
(`utils/dataset.py:282-315`, collate_tts).

A GTA batch is the reference's collate_tts dict: phoneme ids right-padded with 0, mels
(n_mels, T) right-padded with -11.5129 to max(mel_len) + 1 rounded up to a multiple of r,
durations / pitch / energy (per phoneme) zero-padded to the longest id sequence.  The
teacher-forced pass runs on the HIP path (ForwardTacotron.forward: packed LSTM over the
given durations); each item's mel_post is cropped to its mel_len and written as
`{item_id}.npy` (np.save, allow_pickle=False), exactly what the reference writes.
"""
from __future__ import annotations

import itertools
from pathlib import Path
from typing import Dict, Iterable, List, Union

import numpy as np
import torch

PAD_MEL = -11.5129


def pad1d(x: np.ndarray, max_len: int) -> np.ndarray:
    """`utils/dataset.py:276-277`: zero right-padding of a 1-d array."""
    x = np.asarray(x)
    return np.concatenate([x, np.zeros(max_len - len(x), dtype=x.dtype)])


def pad2d(x: np.ndarray, max_len: int) -> np.ndarray:
    """`utils/dataset.py:280-281`: right-pad the time axis of (C, T) with -11.5129."""
    x = np.asarray(x)
    out = np.full((x.shape[0], max_len), PAD_MEL, dtype=x.dtype)
    out[:, :x.shape[-1]] = x
    return out


def collate_tts(batch: List[Dict[str, object]], r: int) -> Dict[str, object]:
    """`utils/dataset.py:284-315`.  Items: {'x': ids, 'mel': (n_mels, T), 'item_id',
    'x_len', 'mel_len', and optionally 'dur', 'pitch', 'energy' (per phoneme)}."""
    x_len = torch.tensor([b['x_len'] for b in batch])
    max_x_len = int(max(x_len))
    text = torch.tensor(np.stack([pad1d(b['x'], max_x_len) for b in batch])).long()
    spec_lens = [b['mel_len'] for b in batch]
    max_spec_len = max(spec_lens) + 1
    if max_spec_len % r != 0:
        max_spec_len += r - max_spec_len % r
    mel = torch.tensor(np.stack([pad2d(b['mel'], max_spec_len) for b in batch]))
    out = {'x': text, 'mel': mel, 'item_id': [b['item_id'] for b in batch], 'x_len': x_len,
           'mel_len': torch.tensor(spec_lens), 'dur': None, 'pitch': None, 'energy': None}
    for k in ('dur', 'pitch', 'energy'):
        if k in batch[0]:
            out[k] = torch.tensor(np.stack([pad1d(np.asarray(b[k])[:max_x_len], max_x_len)
                                            for b in batch])).float()
    return out


def to_device(batch: Dict[str, object], device) -> Dict[str, object]:
    """`trainer/common.py` to_device: tensors to the device, everything else unchanged."""
    return {k: (v.to(device) if isinstance(v, torch.Tensor) else v) for k, v in batch.items()}


def create_gta_features(model, train_set: Iterable[Dict[str, object]],
                        val_set: Iterable[Dict[str, object]],
                        save_path: Union[str, Path]) -> int:
    """`train_forward.py:33-50`: teacher-forced forward() over every batch of both sets,
    mel_post[:, :mel_len] of each item saved as {item_id}.npy.  Returns the item count."""
    model.eval()
    device = next(model.parameters()).device
    save_path = Path(save_path)
    n = 0
    for batch in itertools.chain(train_set, val_set):
        batch = to_device(batch, device)
        with torch.no_grad():
            pred = model(batch)
        gta = pred['mel_post'].cpu().numpy()
        for j, item_id in enumerate(batch['item_id']):
            mel = gta[j][:, :int(batch['mel_len'][j])]
            np.save(str(save_path / f'{item_id}.npy'), mel, allow_pickle=False)
            n += 1
    return n
