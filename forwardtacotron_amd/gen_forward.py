"""Drop-in counterpart of the reference CLI `gen_forward.py:40-136`, from phonemes / token
ids onward (the text frontend — `utils/text/cleaners.py`: unidecode, inflect, espeak via
phonemizer — is absent from this image, so raw English text is refused with that reason).

    python -m forwardtacotron_amd.gen_forward --checkpoint ckpt.pt \\
        [--input_phonemes "həloʊ wɜːld" | --input_tokens 12,40,7 | --sentences file] \\
        [--alpha 1.0] [--amp 1.0] {griffinlim,melgan,hifigan,wavernn}
        [--voc_checkpoint voc.pt | --voc_synthetic] [--target 11000] [--overlap 550]

Per sentence, exactly like the reference loop (`gen_forward.py:106-134`): tokens (B = 1) ->
`generate(x, alpha, pitch_function=lambda x: x * amp, energy_function=lambda x: x)` on the
HIP path -> `mel_post.cpu()` -> the vocoder's output file in model_outputs/:
  griffinlim  {name}.wav  DSP.griffinlim (HIP NNLS + Griffin-Lim) -> DSP.save_wav (16-bit PCM)
  melgan      {name}.mel  torch.save of the (1, n_mels, T) mel tensor
  hifigan     {name}.npy  np.save(..., allow_pickle=False) of the same array
  wavernn     {name}.wav  WaveRNN.generate(mels, batched=True, target, overlap, mu_law of the
              vocoder's dsp config) on the HIP sample loop -> DSP.save_wav (`:78-80, :125-131`)
with name = f'{i}_forward_{tts_k}k_alpha{alpha}_amp{amp}_{vocoder}' (`:113`).  --synthetic /
--voc_synthetic run the synthetic weights (tests / benchmarks without a checkpoint).
"""
from __future__ import annotations

import argparse
from pathlib import Path
from typing import List, Optional, Sequence

import numpy as np
import torch

VOCODERS = ('griffinlim', 'wavernn', 'melgan', 'hifigan')


def load_tts_model(checkpoint_path: str):
    """`gen_forward.py:19-27` (weights_only load: nothing in the file is executed)."""
    from .checkpoints import init_tts_model
    print(f'Loading tts checkpoint {checkpoint_path}')
    checkpoint = torch.load(checkpoint_path, map_location=torch.device('cpu'), weights_only=True)
    config = checkpoint['config']
    tts_model = init_tts_model(config)
    tts_model.load_state_dict(checkpoint['model'])
    print(f'Initialized tts model: {tts_model}')
    print(f'Restored model with step {tts_model.get_step()}')
    return tts_model, config


def synthetic_tts_model(kind: str = 'forward_tacotron'):
    from .checkpoints import init_tts_model
    from .synthetic import default_config, load_synthetic
    config = default_config()
    config['tts_model'] = kind
    model = init_tts_model(config)
    load_synthetic(model, 0, kind)
    return model, config


def wav_name(i: int, tts_k: int, alpha: float, amp: float, vocoder: str) -> str:
    """`gen_forward.py:113`."""
    return f'{i}_forward_{tts_k}k_alpha{alpha}_amp{amp}_{vocoder}'


def load_wavernn(checkpoint_path: str):
    """`gen_forward.py:30-37` (weights_only load)."""
    from .wavernn import WaveRNN
    print(f'Loading voc checkpoint {checkpoint_path}')
    checkpoint = torch.load(checkpoint_path, map_location=torch.device('cpu'), weights_only=True)
    config = checkpoint['config']
    voc_model = WaveRNN.from_config(config)
    voc_model.load_state_dict(checkpoint['model'])
    print(f'Loaded model with step {voc_model.get_step()}')
    return voc_model, config


def synthetic_wavernn():
    from .synthetic import default_config, load_synthetic
    from .wavernn import WaveRNN
    config = default_config()
    return load_synthetic(WaveRNN.from_config(config), 0, 'wavernn'), config


def write_output(m: torch.Tensor, name: str, vocoder: str, out_path: Path, dsp=None, voc=None,
                 target: int = 11000, overlap: int = 550) -> Path:
    """`gen_forward.py:120-134` for one sentence: m is the host (1, n_mels, T) mel_post;
    voc = (WaveRNN model, its DSP) for the wavernn vocoder."""
    if vocoder == 'melgan':
        p = out_path / f'{name}.mel'
        torch.save(m, p)
    elif vocoder == 'hifigan':
        p = out_path / f'{name}.npy'
        np.save(p, m.numpy(), allow_pickle=False)
    elif vocoder == 'wavernn':
        p = out_path / f'{name}.wav'
        voc_model, voc_dsp = voc
        wav = voc_model.generate(mels=m, batched=True, target=target, overlap=overlap,
                                 mu_law=voc_dsp.mu_law)
        dsp.save_wav(wav, p)
    elif vocoder == 'griffinlim':
        p = out_path / f'{name}.wav'
        wav = dsp.griffinlim(m.squeeze().numpy())
        dsp.save_wav(wav, p)
    else:
        raise ValueError(f'unsupported vocoder {vocoder!r}')
    return p


def read_inputs(args) -> List[List[int]]:
    """Token id lists, one per sentence."""
    from .text.tokenizer import Tokenizer
    tok = Tokenizer()
    if args.input_tokens:
        return [[int(v) for v in args.input_tokens.split(',') if v.strip()]]
    if args.input_phonemes:
        return [tok(args.input_phonemes)]
    if args.input_text:
        raise SystemExit('--input_text needs the reference text frontend (utils/text/cleaners.py: '
                         'unidecode + phonemizer/espeak), absent here: pass --input_phonemes or '
                         '--input_tokens')
    path = Path(args.sentences)
    with open(path, 'r', encoding='utf-8') as f:  # gen_forward.py:93-94 (phonemised lines)
        return [tok(line.strip()) for line in f if line.strip()]


def main(argv: Optional[Sequence[str]] = None) -> List[Path]:
    parser = argparse.ArgumentParser(description='TTS Generator (MI355X HIP path)')
    parser.add_argument('--input_text', '-i', default=None, type=str)
    parser.add_argument('--input_phonemes', default=None, type=str,
                        help='phonemised sentence (what the reference cleaner produces)')
    parser.add_argument('--input_tokens', default=None, type=str, help='comma-separated token ids')
    parser.add_argument('--sentences', default='sentences.txt',
                        help='file of phonemised sentences, one per line')
    parser.add_argument('--checkpoint', type=str, default=None)
    parser.add_argument('--synthetic', action='store_true', help='synthetic weights, no checkpoint')
    parser.add_argument('--alpha', type=float, default=1.)
    parser.add_argument('--amp', type=float, default=1.)
    parser.add_argument('--out', default='model_outputs')
    parser.add_argument('vocoder', choices=VOCODERS)
    # the reference's `wavernn` sub-command options (gen_forward.py:54-57)
    parser.add_argument('--voc_checkpoint', type=str, default=None,
                        help='[string/path] Load in different WaveRNN weights')
    parser.add_argument('--voc_synthetic', action='store_true', help='synthetic WaveRNN weights')
    parser.add_argument('--overlap', '-o', default=550, type=int, help='[int] number of crossover samples')
    parser.add_argument('--target', '-t', default=11_000, type=int,
                        help='[int] number of samples in each batch index')
    args = parser.parse_args(argv)
    if args.checkpoint:
        tts_model, config = load_tts_model(args.checkpoint)
    elif args.synthetic:
        tts_model, config = synthetic_tts_model()
    else:
        raise SystemExit('--checkpoint (or --synthetic) is required')
    from .dsp import DSP
    dsp = DSP.from_config(config)
    voc = None
    if args.vocoder == 'wavernn':
        if args.voc_checkpoint:
            voc_model, voc_config = load_wavernn(args.voc_checkpoint)
        elif args.voc_synthetic:
            voc_model, voc_config = synthetic_wavernn()
        else:
            raise SystemExit('wavernn: --voc_checkpoint (or --voc_synthetic) is required')
        voc = (voc_model, DSP.from_config(voc_config))
    out_path = Path(args.out)
    out_path.mkdir(parents=True, exist_ok=True)
    if not torch.cuda.is_available():
        raise SystemExit('the HIP path needs a GPU (there is no CPU fallback)')
    device = torch.device('cuda')
    tts_model.to(device)
    tts_model.eval()
    if voc is not None:
        voc[0].to(device)
    tts_k = tts_model.get_step() // 1000
    texts = read_inputs(args)
    pitch_function = lambda x: x * args.amp  # noqa: E731  (gen_forward.py:103)
    energy_function = lambda x: x  # noqa: E731  (gen_forward.py:104)
    written = []
    for i, ids in enumerate(texts, 1):
        print(f'\n| Generating {i}/{len(texts)}')
        x = torch.as_tensor(ids, dtype=torch.long, device=device).unsqueeze(0)
        name = wav_name(i, tts_k, args.alpha, args.amp, args.vocoder)
        gen = tts_model.generate(x=x, alpha=args.alpha, pitch_function=pitch_function,
                                 energy_function=energy_function)
        m = gen['mel_post'].cpu()
        written.append(write_output(m, name, args.vocoder, out_path, dsp, voc, args.target,
                                    args.overlap))
    print('\n\nDone.\n')
    return written


if __name__ == '__main__':
    main()
