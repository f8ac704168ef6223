"""Checkpoint format and model factory of the reference (`utils/checkpoints.py:12-40`).

Checkpoints are the reference's `torch.save({'model': state_dict, 'optim': ..., 'config':
yaml dict})` files; the state_dict keys of forwardtacotron_amd.ForwardTacotron are
identical, so reference checkpoints load unchanged (and ours load in the reference).
Loading uses `weights_only=True` (no unpickling of arbitrary objects).
"""
from pathlib import Path
from typing import Any, Dict, Optional

import torch

from .forward_tacotron import ForwardTacotron


def save_checkpoint(model: torch.nn.Module, optim: Optional[torch.optim.Optimizer],
                    config: Dict[str, Any], path: Path) -> None:
    """`utils/checkpoints.py:12-18`."""
    torch.save({'model': model.state_dict(),
                'optim': optim.state_dict() if optim is not None else {},
                'config': config}, str(path))


def restore_checkpoint(model: torch.nn.Module, optim: Optional[torch.optim.Optimizer],
                       path: Path, device: torch.device) -> None:
    """`utils/checkpoints.py:21-29`."""
    path = Path(path)
    if path.is_file():
        checkpoint = torch.load(path, map_location=device, weights_only=True)
        model.load_state_dict(checkpoint['model'])
        if optim is not None and checkpoint.get('optim'):
            optim.load_state_dict(checkpoint['optim'])
        print(f'Restored model with step {model.get_step()}\n')


def init_tts_model(config: Dict[str, Any]) -> ForwardTacotron:
    """`utils/checkpoints.py:32-40`."""
    model_type = config.get('tts_model', 'forward_tacotron')
    if model_type == 'forward_tacotron':
        return ForwardTacotron.from_config(config)
    if model_type == 'fast_pitch':
        from .fast_pitch import FastPitch
        return FastPitch.from_config(config)
    raise ValueError(f'Model type not supported: {model_type}')
