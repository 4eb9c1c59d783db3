"""On-device evaluation metrics (skeletondiffusion_amd.metrics) against the reference's own
src/metrics/multimodal.py outputs (tests/golden/metrics.npz, made by gen_golden.py) and the
oracle's restatement.  Tolerance: relative 1e-5 (fp32 sums over up to 1536 features, fixed order
on the device, cdist / float64 on the host)."""
import numpy as np
import pytest
import torch

import oracle as O
from conftest import golden
from skeletondiffusion_amd import synthetic

RTOL = 1e-5


def _inputs():
    lat = torch.from_numpy(synthetic.normal((3, 50, 16, 96), seed=31)) * 0.3
    motion = torch.from_numpy(synthetic.normal((2, 7, 20, 16, 3), seed=32))
    target = torch.from_numpy(synthetic.normal((2, 20, 16, 3), seed=33))
    return lat, motion, target


def _close(a, b):
    a = np.asarray(a.cpu() if torch.is_tensor(a) else a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    assert np.all(np.abs(a - b) <= RTOL * np.abs(b) + 1e-6), (a, b)


def test_oracle_metrics_match_reference():
    z = golden("metrics")
    lat, motion, target = _inputs()
    _close(O.metric_lat_apd(lat), z["lat_apd"])
    _close(O.metric_apd(lat.unsqueeze(2)), z["lat_apd_l2"])
    _close(O.metric_apd(motion), z["apd"])
    _close(O.metric_apd(motion, 5, 15), z["apd_t5_15"])
    _close(O.metric_ade(target, motion), z["ade"])
    _close(O.metric_ade(target, motion, 5, 15), z["ade_t5_15"])
    _close(O.metric_ade(target, motion, last_only=True), z["fde"])
    _close(O.metric_ade(target, motion, reduction="none"), z["ade_per_sample"])
    _close(O.metric_ade(target, motion, reduction="none", last_only=True), z["fde_per_sample"])


def test_metrics_refuse_cpu_tensors():
    from skeletondiffusion_amd import metrics
    from skeletondiffusion_amd._lib import SkelDiffError

    with pytest.raises(SkelDiffError):
        metrics.lat_apd(torch.zeros(2, 3, 4))


@pytest.mark.gpu
def test_device_metrics_match_reference(cuda):
    from skeletondiffusion_amd import metrics as M

    z = golden("metrics")
    lat, motion, target = (t.to(cuda) for t in _inputs())
    _close(M.lat_apd(lat), z["lat_apd"])
    _close(M.apd(lat.unsqueeze(2)), z["lat_apd_l2"])
    _close(M.apd(motion), z["apd"])
    _close(M.apd(motion, t0=5, t=15), z["apd_t5_15"])
    _close(M.ade(target, motion), z["ade"])
    _close(M.ade(target, motion, t0=5, t=15), z["ade_t5_15"])
    _close(M.fde(target, motion), z["fde"])
    _close(M.ade(target, motion, reduction="none"), z["ade_per_sample"])
    _close(M.fde(target, motion, reduction="none"), z["fde_per_sample"])


@pytest.mark.gpu
def test_device_metrics_deterministic_and_edges(cuda):
    from skeletondiffusion_amd import metrics as M
    from skeletondiffusion_amd._lib import SkelDiffError

    g = torch.Generator(device=cuda).manual_seed(5)
    lat = torch.randn(4, 64, 16, 96, device=cuda, generator=g)   # 64 samples: the maximum
    a, b = M.lat_apd(lat), M.lat_apd(lat)
    assert torch.equal(a, b)
    _close(a, O.metric_lat_apd(lat.cpu()).numpy())
    one = torch.randn(3, 1, 5, 7, device=cuda, generator=g)
    assert torch.equal(M.apd(one).cpu(), torch.zeros(3, dtype=torch.int64))   # multimodal.py:19-20
    _close(M.ade(one[:, 0], one), np.zeros(3))
    with pytest.raises(SkelDiffError):
        M.lat_apd(torch.randn(2, 65, 8, device=cuda))
    empty = torch.zeros(0, 50, 16, 96, device=cuda)
    assert M.lat_apd(empty).shape == (0,)


@pytest.mark.gpu
def test_lat_apd_of_sampled_futures(cuda):
    """The metric on the sampler's own output: 2 sequences x 50 futures of the release Denoiser."""
    from conftest import build_release_diffusion, release_inputs
    from skeletondiffusion_amd import metrics as M

    z = golden("release_h36m16_T10")
    d = build_release_diffusion(z, cuda)
    xcs = torch.from_numpy(synthetic.uniform((2, 16, 96), 41)).to(cuda)
    img, _ = d.sample(batch_size=100, x_cond=xcs)
    lat = img.view(2, 50, 16, 96)
    _close(M.lat_apd(lat), O.metric_lat_apd(lat.cpu()).numpy())
    _close(M.apd(lat.unsqueeze(2)), O.metric_apd(lat.unsqueeze(2).cpu()).numpy())


def _mm_inputs():
    """tests/golden/gen_golden.py:mm_inputs (3 sequences, 3 / 1 / 2 multimodal ground truths)."""
    motion = torch.from_numpy(synthetic.normal((3, 7, 20, 16, 3), seed=34))
    gts = torch.from_numpy(synthetic.normal((4, 20, 16, 3), seed=35))
    target = torch.from_numpy(synthetic.normal((3, 20, 16, 3), seed=36))
    return motion, [gts[:3], gts[3:4], gts[1:3]], target


def test_oracle_mm_metrics_match_reference():
    z = golden("metrics")
    motion, mm_gt, _ = _mm_inputs()
    _close(O.metric_mmade(motion, mm_gt), z["mmade"])
    _close(O.metric_mmade(motion, mm_gt, last_only=True), z["mmfde"])
    _close(O.metric_mmade(motion, mm_gt, 5, 15), z["mmade_t5_15"])
    assert bool(z["mm_empty_raises"])  # the reference raises for a sequence without ground truths


@pytest.mark.gpu
def test_device_mm_metrics_match_reference(cuda):
    from skeletondiffusion_amd import _lib
    from skeletondiffusion_amd import metrics as M

    z = golden("metrics")
    motion, mm_gt, target = _mm_inputs()
    motion, target = motion.to(cuda), target.to(cuda)
    mm_gt = [g.to(cuda) for g in mm_gt]
    _close(M.mmade(target, motion, mm_gt), z["mmade"])
    _close(M.mmfde(target, motion, mm_gt), z["mmfde"])
    _close(M.mmade(target, motion, mm_gt, t0=5, t=15), z["mmade_t5_15"])
    with pytest.raises(RuntimeError):
        M.mmade(target, motion, [mm_gt[0], mm_gt[1], mm_gt[2][:0]])
    # the C ABI itself: a sequence without ground truths -> NaN; nseq == 0 is a no-op
    p = motion.reshape(3, 7, 20, 48).contiguous()
    g = torch.cat([mm_gt[0], mm_gt[1]]).reshape(4, 20, 48).contiguous()
    off = torch.tensor([0, 3, 4, 4], dtype=torch.int64, device=cuda)
    seq = torch.tensor([0, 0, 0, 1], dtype=torch.int64, device=cuda)
    pa, out = torch.empty(4, device=cuda), torch.empty(3, device=cuda)
    L = _lib.lib()
    assert L.sd_mm_ade_fde(p.data_ptr(), g.data_ptr(), seq.data_ptr(), 4, off.data_ptr(), 3, 7, 20, 48,
                           pa.data_ptr(), None, out.data_ptr(), None, 0) == 0
    torch.cuda.synchronize()
    _close(out[:2], z["mmade"][:2])
    assert torch.isnan(out[2])
    assert L.sd_mm_ade_fde(None, None, None, 0, None, 0, 7, 20, 48, None, None, None, None, 0) == 0
