"""Phoneme token space of the reference (`utils/text/symbols.py:8-25`).

The ids are the drop-in contract: id 0 is the pad symbol ``_`` and
``len(phonemes) == 135`` is the ``num_chars`` that
``ForwardTacotron.from_config`` injects (`models/forward_tacotron.py:341`).
"""

_pad = '_'
_punctuation = '!\'(),.:;? '
_special = '-'
_vowels = 'iyɨʉɯuɪʏʊeøɘəɵɤoɛœɜɞʌɔæɐaɶɑɒᵻ'
_non_pulmonic_consonants = 'ʘɓǀɗǃʄǂɠǁʛ'
_pulmonic_consonants = 'pbtdʈɖcɟkɡqɢʔɴŋɲɳnɱmʙrʀⱱɾɽɸβfvθðszʃʒʂʐçʝxɣχʁħʕhɦɬɮʋɹɻjɰlɭʎʟ'
_suprasegmentals = 'ˈˌːˑ'
_other_symbols = 'ʍwɥʜʢʡɕʑɺɧ'
_diacritics = 'ɚ˞ɫ'
_extra_phons = ['g', 'ɝ', '̃', '̍', '̥', '̩', '̯', '͡']

phonemes = list(_pad + _punctuation + _special + _vowels + _non_pulmonic_consonants
                + _pulmonic_consonants + _suprasegmentals + _other_symbols
                + _diacritics) + _extra_phons
phonemes_set = set(phonemes)
