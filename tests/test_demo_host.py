"""CPU checks of the demo-fixture goldens (tests/golden/demo_<case>.npz, tests/golden/make_golden_demo.py).

The fixture files under tests/golden/demo/ are the reference's own `data/demo/images` / `data/demo/mask` files; each
golden records their sha256, the weights fingerprint and the executed timestep grid.  One small case (sr1, 15x10
latents, 17 evals) is re-run through the oracle here to pin that the committed golden is what the oracle produces."""
import hashlib
from pathlib import Path

import numpy as np
import pytest
import torch
from PIL import Image

from oracle import pipeline_ref as PR
from tests import models_common as MC

GOLDEN = Path(__file__).resolve().parent / "golden"
DEMO = GOLDEN / "demo"
REFERENCE_DEMO = Path("/root/reference/data/demo")


@pytest.mark.parametrize("name", list(MC.DEMO_CASES))
def test_demo_golden_matches_fixture(name):
    task, img_f, mask_f = MC.DEMO_CASES[name]
    g = np.load(GOLDEN / f"demo_{name}.npz")
    assert str(g["sha_image"]) == hashlib.sha256((DEMO / img_f).read_bytes()).hexdigest()
    if mask_f:
        assert str(g["sha_mask"]) == hashlib.sha256((DEMO / mask_f).read_bytes()).hexdigest()
    im = Image.open(DEMO / img_f)
    h, w = (512, 512) if task == "inpaint" else (im.height - im.height % 8, im.width - im.width % 8)
    assert g["image"].shape == (h, w, 3) and g["decoded16"].shape == (h, w, 3)
    assert g["latents"].shape == (4, h // 8, w // 8)
    assert "x".join(map(str, (w // 8, h // 8))) == MC.DEMO_LATENTS[name]
    _, strength, steps, _ = PR.TASKS[task]
    sched = PR.make_scheduler("ddim" if task == "inpaint" else "pndm")
    sched.set_timesteps(steps)
    ts, _ = PR.get_timesteps(sched, steps, strength)
    assert g["timesteps"].tolist() == [int(t) for t in ts]


@pytest.mark.skipif(not REFERENCE_DEMO.exists(), reason="reference checkout absent (GPU box)")
def test_demo_fixtures_are_the_reference_files():
    for task, img_f, mask_f in MC.DEMO_CASES.values():
        for sub, f in (("images", img_f), ("mask", mask_f)):
            if f:
                assert (DEMO / f).read_bytes() == (REFERENCE_DEMO / sub / f).read_bytes(), f


def test_demo_golden_reproduced_by_oracle():
    """sr1 (125x83 -> 120x80, latents 15x10, 17 PNDM evals, no CFG) through the oracle again: the same uint8 image
    (within 1 level: CPU thread-count reassociation) and latents within 1e-5 relative."""
    g = np.load(GOLDEN / "demo_sr1.npz")
    pc, sd = MC.state_dicts("denoise")
    assert np.array_equal(MC.weight_fingerprint(sd["unet"]), g["fp_unet"])
    prompt, strength, steps, guidance = PR.TASKS["sr"]
    img = Image.open(DEMO / MC.DEMO_CASES["sr1"][1]).convert("RGB")
    with torch.no_grad():
        r = PR.img2img_ref(MC.oracle_models("denoise"), img, MC.prompt_ids(prompt), None, strength, steps, guidance,
                           42, "pndm")
    assert r.timesteps == g["timesteps"].tolist()
    d = np.abs(np.asarray(r.image).astype(int) - g["image"].astype(int))
    assert d.max() <= 1
    lat = r.latents[0].float().numpy()
    assert np.abs(lat - g["latents"]).max() <= 1e-5 * np.abs(g["latents"]).max()
