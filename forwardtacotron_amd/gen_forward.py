"""Drop-in counterpart of the reference CLI `gen_forward.py:40-136`, from phonemes / token
ids onward (the text frontend — `utils/text/cleaners.py`: unidecode, inflect, espeak via
phonemizer — is absent from this image, so raw English text is refused with that reason).

    python -m forwardtacotron_amd.gen_forward [--checkpoint ckpt.pt | --config config.yaml] \\
        [--input_phonemes "həloʊ wɜːld" | --input_tokens 12,40,7 | --sentences file] \\
        [--alpha 1.0] [--amp 1.0] {griffinlim,melgan,hifigan,wavernn}
    python -m forwardtacotron_amd.gen_forward ... wavernn \\
        [--voc_checkpoint voc.pt | --voc_synthetic] [--target 11000] [--overlap 550]

Without --checkpoint the checkpoint is found from --config like the reference
(`gen_forward.py:68-72`: checkpoints/{tts_model_id}.forward/latest_model.pt).

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
                 target: int = 11000, overlap: int = 550, mel_dev=None) -> Path:
    """`gen_forward.py:120-134` for one sentence: m is the host (1, n_mels, T) mel_post;
    voc = (WaveRNN model, its DSP) for the wavernn vocoder; mel_dev: the same mel still on
    the device (griffinlim then starts from it instead of copying m back)."""
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
        wav = (dsp.griffinlim(m.squeeze().numpy()) if mel_dev is None
               else dsp.griffinlim(mel_dev.reshape(mel_dev.shape[-2:])).cpu().numpy())
        dsp.save_wav(wav, p)
    else:
        raise ValueError(f'unsupported vocoder {vocoder!r}')
    return p


RAW_TEXT_HINT = ('needs the reference text frontend (utils/text/cleaners.py: unidecode + '
                 'phonemizer/espeak), absent here: pass --input_phonemes, --input_tokens or a '
                 '--sentences file of phonemised lines')


def _looks_raw(line: str) -> bool:
    """Uppercase ASCII letters or digits never occur in the cleaner's phonemised output
    (espeak IPA is lower case, numbers are spelled out): such a line is raw text."""
    return any(('A' <= c <= 'Z') or c.isdigit() for c in line)


def _maybe_raw(line: str) -> bool:
    """A line of lowercase ASCII only (no IPA symbol, no stress mark) passes _looks_raw but
    may be raw English ('hello world' is made of phoneme-set symbols too); espeak's output
    nearly always carries a stress mark or a non-ASCII vowel, so such a line gets a warning."""
    return all(ord(c) < 128 for c in line)


def read_inputs(args) -> List[List[int]]:
    """Token id lists, one per sentence.  Phonemised input only: the reference cleans raw
    text first (`gen_forward.py:86,109`), which needs espeak.  Lines that are certainly raw
    text (uppercase letters or digits) are refused with that reason; lowercase ASCII-only
    lines cannot be told apart from phonemes by their symbols and are tokenised with a
    warning."""
    from .text.symbols import phonemes
    from .text.tokenizer import Tokenizer
    tok = Tokenizer()
    if args.input_tokens:
        return [[int(v) for v in args.input_tokens.split(',') if v.strip()]]
    if args.input_phonemes:
        return [tok(args.input_phonemes)]
    if args.input_text:
        raise SystemExit('--input_text ' + RAW_TEXT_HINT)
    # the reference reads sentences.txt (raw text, gen_forward.py:92-94); here a file of
    # phonemised lines (--sentences, default the reference's file name)
    path = Path(args.sentences)
    with open(path, 'r', encoding='utf-8') as f:
        lines = [line.strip() for line in f if line.strip()]
    known = set(phonemes)
    for i, line in enumerate(lines, 1):
        if _looks_raw(line):
            raise SystemExit(f'{path}:{i} looks like raw text ({line[:40]!r}); it ' + RAW_TEXT_HINT)
        if _maybe_raw(line):
            print(f'warning: {path}:{i}: no IPA symbol or stress mark ({line[:40]!r}); if this '
                  'is raw text it ' + RAW_TEXT_HINT)
        skipped = sorted(set(line) - known)
        if skipped:  # the reference Tokenizer drops them too (utils/text/tokenizer.py)
            print(f'warning: {path}:{i}: symbols outside the phoneme set skipped: {skipped}')
    return [tok(line) for line in lines]


def checkpoint_from_config(config_path: str) -> Path:
    """`gen_forward.py:68-72`: without --checkpoint, the latest forward checkpoint of the
    config's tts_model_id — Paths(...).forward_checkpoints / 'latest_model.pt', i.e.
    checkpoints/{tts_model_id}.forward/latest_model.pt under the directory the CLI runs from
    (the reference resolves it under its repository root, where it is run from).  The config
    is read with yaml.safe_load (the reference: FullLoader)."""
    import yaml
    with open(config_path, 'r', encoding='utf-8') as f:
        config = yaml.safe_load(f)
    return Path.cwd() / 'checkpoints' / f"{config['tts_model_id']}.forward" / 'latest_model.pt'


def build_parser() -> argparse.ArgumentParser:
    """The reference's grammar (`gen_forward.py:43-61`): top-level options, then the vocoder
    as a sub-command; `wavernn` takes --overlap / --target / --voc_checkpoint.  Additions:
    phonemised / token input, --synthetic / --voc_synthetic weights, --out."""
    parser = argparse.ArgumentParser(description='TTS Generator (MI355X HIP path)')
    parser.add_argument('--input_text', '-i', default=None, type=str,
                        help='[string] raw text (refused: needs the espeak text frontend)')
    parser.add_argument('--input_phonemes', default=None, type=str,
                        help='phonemised sentence (what the reference cleaner produces)')
    parser.add_argument('--input_tokens', default=None, type=str, help='comma-separated token ids')
    parser.add_argument('--sentences', default='sentences.txt',
                        help='file of PHONEMISED sentences, one per line (raw text is refused)')
    parser.add_argument('--checkpoint', type=str, default=None,
                        help='[string/path] path to .pt model file.')
    parser.add_argument('--config', metavar='FILE', default='config.yaml',
                        help='The config containing all hyperparams. Only used if no checkpoint is set.')
    parser.add_argument('--synthetic', action='store_true', help='synthetic weights, no checkpoint')
    parser.add_argument('--alpha', type=float, default=1.)
    parser.add_argument('--amp', type=float, default=1.)
    parser.add_argument('--out', default='model_outputs')
    subparsers = parser.add_subparsers(dest='vocoder')
    wr_parser = subparsers.add_parser('wavernn')
    wr_parser.add_argument('--overlap', '-o', default=550, type=int,
                           help='[int] number of crossover samples')
    wr_parser.add_argument('--target', '-t', default=11_000, type=int,
                           help='[int] number of samples in each batch index')
    wr_parser.add_argument('--voc_checkpoint', type=str,
                           help='[string/path] Load in different WaveRNN weights')
    wr_parser.add_argument('--voc_synthetic', action='store_true', help='synthetic WaveRNN weights')
    for name in ('griffinlim', 'melgan', 'hifigan'):
        subparsers.add_parser(name)
    return parser


def main(argv: Optional[Sequence[str]] = None) -> List[Path]:
    args = build_parser().parse_args(argv)
    if args.vocoder not in VOCODERS:  # gen_forward.py:65-66
        raise SystemExit("Please provide a valid vocoder! Choices: ['griffinlim', 'wavernn', "
                         "'melgan', 'hifigan']")
    if args.synthetic:
        tts_model, config = synthetic_tts_model()
    else:
        checkpoint = args.checkpoint or checkpoint_from_config(args.config)
        tts_model, config = load_tts_model(str(checkpoint))
    from .dsp import DSP
    dsp = DSP.from_config(config)
    voc = None
    if args.vocoder == 'wavernn':
        if args.voc_synthetic:
            voc_model, voc_config = synthetic_wavernn()
        elif args.voc_checkpoint:
            voc_model, voc_config = load_wavernn(args.voc_checkpoint)
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
    # gen_forward.py:103-104, the same plain lambdas: generate() replays the phoneme phase
    # from its split graph and runs them eagerly in between (forward_tacotron._phoneme_graph)
    pitch_function = lambda x: x * args.amp  # noqa: E731
    energy_function = lambda x: x  # noqa: E731
    from .host_io import PinnedD2H
    d2h = PinnedD2H(device, depth=1)  # pinned D2H: the drop-in for .cpu() (gen_forward.py:120)
    written = []
    for i, ids in enumerate(texts, 1):
        print(f'\n| Generating {i}/{len(texts)}')
        x = torch.as_tensor(ids, dtype=torch.long, device=device).unsqueeze(0)
        name = wav_name(i, tts_k, args.alpha, args.amp, args.vocoder)
        gen = tts_model.generate(x=x, alpha=args.alpha, pitch_function=pitch_function,
                                 energy_function=energy_function)
        m = d2h.fetch(gen['mel_post'])
        written.append(write_output(m, name, args.vocoder, out_path, dsp, voc,
                                    getattr(args, 'target', 11000), getattr(args, 'overlap', 550),
                                    mel_dev=gen['mel_post']))
    print('\n\nDone.\n')
    return written


if __name__ == '__main__':
    main()
