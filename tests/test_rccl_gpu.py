"""The engine's own RCCL path through the C ABI (SURVEY.md §8b `irx_weights_bcast`).

A one-GPU box can only host a world of one RCCL rank (RCCL refuses two ranks on one device), so this checks
that the communicator initialises on the box, that an in-place broadcast from the root leaves the root's bytes
intact, and that `dist.broadcast_models` — the call bench.py makes on every rank — moves the bound blobs of
real models with irx_weights_bcast.  The N > 1 rendezvous logic is covered on CPU (tests/test_dist.py)."""
import ctypes as C

import pytest
import torch

from image_restoration_and_enhancement_amd import _lib as L
from image_restoration_and_enhancement_amd import dist as D
from image_restoration_and_enhancement_amd.configs import PipelineConfig
from image_restoration_and_enhancement_amd.engine import CLIPText, VAE
from tests import models_common as MC

pytestmark = pytest.mark.gpu


def test_rccl_world_of_one(device):
    assert L.call("irx_rccl_available") == 1
    comm = D.rccl_comm(0, 1)
    try:
        buf = torch.randint(0, 256, (3 << 20,), dtype=torch.uint8, device=device)
        ref = buf.clone()
        s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        L.call("irx_rccl_broadcast", comm, C.c_void_p(buf.data_ptr()), buf.numel(), 0, s)
        torch.cuda.synchronize()
        assert torch.equal(buf, ref)
        # a model's bound blob, in place
        pc, sd = MC.state_dicts("denoise")
        clip = CLIPText(pc.clip, "bf16", device)
        clip.load_state_dict(sd["clip"])
        before = clip.blob.clone()
        L.call("irx_weights_bcast", clip.h, comm, 0, s)
        torch.cuda.synchronize()
        assert torch.equal(clip.blob, before)
    finally:
        L.call("irx_rccl_comm_destroy", comm)


def test_weights_bcast_requires_bound_blob(device):
    pc = PipelineConfig.default("denoise")
    vae = VAE(pc.vae, "bf16", device)
    comm = D.rccl_comm(0, 1)
    try:
        with pytest.raises(L.IrxError, match="no weight blob"):
            L.call("irx_weights_bcast", vae.h, comm, 0, None)
    finally:
        L.call("irx_rccl_comm_destroy", comm)
