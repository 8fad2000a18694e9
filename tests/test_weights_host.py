"""CPU tests: weight-file selection of a saved component directory follows diffusers' from_pretrained rules
(every *.safetensors was merged, so .fp16 / .non_ema variants could silently win)."""
import json

import pytest
import torch
from safetensors.torch import save_file

from image_restoration_and_enhancement_amd import weights as W


def _save(path, val):
    save_file({"a.weight": torch.full((2, 2), float(val))}, str(path))


def test_plain_file_wins_over_variants(tmp_path):
    _save(tmp_path / "diffusion_pytorch_model.safetensors", 1)
    _save(tmp_path / "diffusion_pytorch_model.fp16.safetensors", 2)
    _save(tmp_path / "diffusion_pytorch_model.non_ema.safetensors", 3)
    assert W.load_component_dir(tmp_path)["a.weight"][0, 0] == 1
    assert W.load_component_dir(tmp_path, variant="fp16")["a.weight"][0, 0] == 2


def test_variants_only_is_an_error(tmp_path):
    _save(tmp_path / "diffusion_pytorch_model.non_ema.safetensors", 3)
    with pytest.raises(FileNotFoundError, match="non_ema"):
        W.load_component_dir(tmp_path)


def test_sharded_index_and_text_encoder_name(tmp_path):
    save_file({"x": torch.ones(1)}, str(tmp_path / "model-00001-of-00002.safetensors"))
    save_file({"y": torch.zeros(1)}, str(tmp_path / "model-00002-of-00002.safetensors"))
    save_file({"z": torch.zeros(1)}, str(tmp_path / "stray.safetensors"))
    (tmp_path / "model.safetensors.index.json").write_text(json.dumps(
        {"weight_map": {"x": "model-00001-of-00002.safetensors", "y": "model-00002-of-00002.safetensors"}}))
    assert set(W.load_component_dir(tmp_path)) == {"x", "y"}
