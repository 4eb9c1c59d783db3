"""Checkpoint boundary: the reference's {'model': state_dict} files load
strictly into the product diffusion through the tensor-only loader, and the sampling plan is
rebuilt from the loaded weights."""
import os

import pytest
import torch

from conftest import build_release_diffusion, golden, release_inputs
from skeletondiffusion_amd import checkpoint as C


def _perturbed(d):
    with torch.no_grad():
        for p in d.parameters():
            p.add_(0.01)
    return d


def test_save_load_round_trip_strict(tmp_path):
    z = golden("release_h36m16_T10")
    src = build_release_diffusion(z)
    dst = _perturbed(build_release_diffusion(z))
    path = tmp_path / "checkpoint_7_val_ade=-0.5.pt"
    C.save_diffusion_checkpoint(src, str(path), epoch=7, note="synthetic")
    ckpt = C.load_diffusion_checkpoint(dst, str(path))
    assert ckpt["epoch"] == 7 and ckpt["note"] == "synthetic"
    a, b = src.state_dict(), dst.state_dict()
    assert a.keys() == b.keys() and len(a) == 137  # the release Denoiser's key set
    for k in a:
        assert torch.equal(a[k], b[k]), k


def test_bare_state_dict_and_missing_keys(tmp_path):
    z = golden("release_h36m16_T10")
    src = build_release_diffusion(z)
    path = tmp_path / "bare.pt"
    torch.save(src.state_dict(), path)
    dst = _perturbed(build_release_diffusion(z))
    C.load_diffusion_checkpoint(dst, str(path))
    assert torch.equal(dst.model.final_glin.weight, src.model.final_glin.weight)
    sd = src.state_dict()
    sd.pop("model.final_glin.bias")
    torch.save({"model": sd}, path)
    with pytest.raises(RuntimeError, match="Missing key"):
        C.load_diffusion_checkpoint(build_release_diffusion(z), str(path))
    C.load_diffusion_checkpoint(build_release_diffusion(z), str(path), strict=False)


def test_refuses_pickled_objects(tmp_path):
    """Only tensors and plain containers load: an arbitrary pickled object is refused."""
    import argparse

    path = tmp_path / "obj.pt"
    torch.save({"model": {}, "obj": argparse.Namespace(a=1)}, path)
    with pytest.raises(Exception, match="[Ww]eights only load failed"):
        C.load_model_checkpoint(str(path))


def test_latest_model_path(tmp_path):
    for name in ("checkpoint_3_val_ade=-0.61.pt", "checkpoint_12_val_ade=-0.55.pt", "checkpoint_9.pt", "other.pt"):
        (tmp_path / name).write_bytes(b"")
    assert os.path.basename(C.get_latest_model_path(str(tmp_path))) == "checkpoint_12_val_ade=-0.55.pt"
    with pytest.raises(FileNotFoundError):
        C.get_latest_model_path(str(tmp_path / ".."))  # no checkpoint_* there


@pytest.mark.gpu
def test_loaded_checkpoint_drives_the_sampler(tmp_path, cuda):
    """A checkpoint loaded into a differently initialised diffusion samples bitwise like the
    diffusion that saved it (the plan is rebuilt from the loaded weights)."""
    z = golden("release_h36m16_T10")
    src = build_release_diffusion(z, cuda)
    dst = _perturbed(build_release_diffusion(z, cuda))
    xcs = release_inputs(z)[0].to(cuda)
    before = dst.sample(batch_size=8, x_cond=xcs, seed=3)[0].clone()
    path = tmp_path / "checkpoint_1.pt"
    C.save_diffusion_checkpoint(src, str(path), epoch=1)
    C.load_diffusion_checkpoint(dst, str(path), map_location=cuda)
    a = src.sample(batch_size=8, x_cond=xcs, seed=3)[0]
    b = dst.sample(batch_size=8, x_cond=xcs, seed=3)[0]
    torch.cuda.synchronize()
    assert torch.equal(a, b) and not torch.equal(a, before)
