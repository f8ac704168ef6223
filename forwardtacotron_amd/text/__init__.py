from .symbols import phonemes, phonemes_set  # noqa: F401
from .tokenizer import Tokenizer  # noqa: F401
