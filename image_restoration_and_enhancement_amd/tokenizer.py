"""Prompt -> CLIP token ids (77, BOS 49406, EOS/pad 49407).

The reference tokenizes inside diffusers' `encode_prompt` with transformers' CLIPTokenizer
loaded from `<model_dir>/tokenizer/` (vocab.json + merges.txt,
`outputs/models/*/best/tokenizer/tokenizer_config.json`), padding="max_length", max_length=77,
truncation=True.  This module uses the same tokenizer when a model directory with tokenizer
files is available.  Without one (random-weight benchmarking on a box with no model files),
the reference's own default prompts (`src/inference.py:86-91`, `app.py:99`) and the empty
negative prompt resolve from the table below, which holds exactly the ids CLIPTokenizer
produces for them (pinned by tests/test_tokenizer.py against the reference vocabulary).
"""
from __future__ import annotations

from pathlib import Path
from typing import List, Optional

import numpy as np

BOS, EOS = 49406, 49407
MAX_LEN = 77

KNOWN_PROMPTS = {
    "clean high quality photo, no noise, sharp details":
        [49406, 3772, 1400, 3027, 1125, 267, 871, 9307, 267, 8157, 2353, 49407],
    "high quality, detailed, sharp": [49406, 1400, 3027, 267, 12609, 267, 8157, 49407],
    "vibrant realistic natural colors, colorful, high quality photo, detailed, full color, rich colors":
        [49406, 14270, 16157, 3288, 5389, 267, 11444, 267, 1400, 3027, 1125, 267, 12609, 267, 1476, 3140, 267,
         4021, 5389, 49407],
    "high quality detailed photo": [49406, 1400, 3027, 12609, 1125, 49407],
    "high quality detailed photo, realistic": [49406, 1400, 3027, 12609, 1125, 267, 16157, 49407],
    "": [49406, 49407],
}


class PromptTokenizer:
    def __init__(self, tokenizer_dir: Optional[str | Path] = None):
        self._tok = None
        if tokenizer_dir is not None and (Path(tokenizer_dir) / "vocab.json").exists():
            from transformers import CLIPTokenizer
            self._tok = CLIPTokenizer.from_pretrained(str(tokenizer_dir))

    def __call__(self, prompt: str) -> np.ndarray:
        if self._tok is not None:
            ids = self._tok(prompt, padding="max_length", max_length=MAX_LEN, truncation=True).input_ids
            return np.asarray(ids, dtype=np.int64)
        if prompt not in KNOWN_PROMPTS:
            raise ValueError("no tokenizer files available (model_dir/tokenizer/vocab.json) and the prompt is not "
                             "one of the reference's default prompts")
        ids: List[int] = list(KNOWN_PROMPTS[prompt])
        return np.asarray(ids + [EOS] * (MAX_LEN - len(ids)), dtype=np.int64)
