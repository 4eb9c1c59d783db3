"""Best-of-k training relaxation (reference src/core/trainer.py:182-222):
the oracle restatement against the reference-generated fixture (tests/golden/best_of_k.npz,
gen_golden.py:gen_best_of_k: the release Denoiser's p_losses with n_train_samples = k, the
reference AutoEncoder's decode + loss, the trainer's min/gather selection), and on the GPU the HIP
path -- sd_gru_decode, sd_pose_loss, sd_best_of_k and its backward -- against the same fixture and
against torch's gather autograd."""
import numpy as np
import pytest
import torch

import oracle as O
from conftest import build_release_diffusion, golden

AE_KW = dict(num_nodes=16, encoder_hidden_size=96, decoder_hidden_size=96, latent_size=96, input_size=3,
             z_activation="tanh", enc_num_layers=1, output_size=3, recurrent_arch_enc="StaticGraphGRU",
             recurrent_arch_decoder="StaticGraphGRU", if_consider_hip=False)


def test_oracle_pose_loss_and_selection_match_reference():
    z = golden("best_of_k")
    pred, tgt = torch.from_numpy(z["pose_pred"]), torch.from_numpy(z["pose_target"])
    np.testing.assert_allclose(O.pose_loss(pred, tgt, False).numpy(), z["pose_l1"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(O.pose_loss(pred, tgt, True).numpy(), z["pose_mse"], rtol=1e-6, atol=1e-7)
    k = int(z["k"])
    dec = torch.from_numpy(z["decoded"])
    sim = O.pose_loss(dec, torch.from_numpy(z["fut"]), False)
    np.testing.assert_allclose(sim.numpy(), z["sim"], rtol=1e-6, atol=1e-8)
    loss = torch.from_numpy(z["loss"])
    sel, idx = O.best_of_k(loss, k, sim)
    np.testing.assert_array_equal(idx.numpy(), z["idx"])
    np.testing.assert_array_equal(sel.numpy(), z["sel"])
    _, idx_l = O.best_of_k(loss, k)
    np.testing.assert_array_equal(idx_l.numpy(), z["idx_latent"])
    assert abs(float((sel * torch.from_numpy(z["weight"])).mean()) - float(z["final"])) < 1e-7


def _autoencoder(device):
    from skeletondiffusion_amd import synthetic
    from skeletondiffusion_amd.core.network.autoencoder import AutoEncoder
    from skeletondiffusion_amd.skeletons import skeleton

    _, _, _, types = skeleton("h36m16")
    m = AutoEncoder(node_types=torch.from_numpy(types), **AE_KW).eval()
    synthetic.fill_module_(m, 4321)
    return m.to(device)


def _to_metric_space(kpts, box=1.5):
    """The release task's skeleton (SkeletonRescalePose, if_consider_hip False, pose_box_size 1.5;
    reference rescalepose.py:29-39 via base.py:69-86): the pose scaled back out of the unit box."""
    return kpts * box


def test_metric_space_selection_matches_reference():
    """metric_space (trainer.py:193-198, 213-214) restated on the fixture's decoded samples against
    tests/golden/best_of_k_metric.npz (gen_golden.py:gen_best_of_k_metric, the reference skeleton)."""
    z, m = golden("best_of_k"), golden("best_of_k_metric")
    assert float(m["pose_box_size"]) == 1.5
    k = int(z["k"])
    out_c = _to_metric_space(torch.from_numpy(z["decoded"])).flatten(start_dim=3)
    fut_c = _to_metric_space(torch.from_numpy(z["fut"])).unsqueeze(1).flatten(start_dim=3).repeat_interleave(k, 1)
    np.testing.assert_array_equal(out_c.numpy(), m["out_c"])
    np.testing.assert_array_equal(fut_c.numpy(), m["fut_c"])
    sim = torch.linalg.norm(out_c - fut_c, dim=-1).mean(dim=-1)
    np.testing.assert_allclose(sim.numpy(), m["sim"], rtol=1e-6, atol=1e-8)
    sel, idx = O.best_of_k(torch.from_numpy(z["loss"]), k, sim.reshape(-1))
    np.testing.assert_array_equal(idx.numpy(), m["idx"])
    np.testing.assert_array_equal(sel.numpy(), m["sel"])


@pytest.mark.gpu
@pytest.mark.parametrize("space", ["input_space", "metric_space", "latent_space"])
def test_hip_best_of_k_matches_reference(space, cuda):
    """p_losses(n_train_samples=k) on the HIP training kernels, the HIP decoder, sd_pose_loss /
    sd_ade_fde and sd_best_of_k: the selected indices equal the reference's, the selected losses and
    the trainer's scalar within 1e-5, and the gradient reaches only the selected samples' rows."""
    from skeletondiffusion_amd.core import best_of_k as B

    z = golden("best_of_k")
    m = golden("best_of_k_metric")
    d = build_release_diffusion(golden("release_h36m16_T10"), cuda)
    d.train()
    ae = _autoencoder(cuda)
    k, ph = int(z["k"]), int(z["ph"])
    dev = lambda n: torch.from_numpy(z[n]).to(cuda)  # noqa: E731
    dev_m = lambda n: torch.from_numpy(m[n]).to(cuda)  # noqa: E731
    data, x_cond, t, noise, past, fut = (dev(n) for n in ("data", "x_cond", "t", "noise", "past", "fut"))
    loss, w, samples = d.p_losses(data, t, noise=noise, x_cond=x_cond, n_train_samples=k)
    assert float((loss - dev("loss")).abs().max()) < 1e-5
    out_c, fut_c = B.to_comparison_space_train(samples.detach(), diff_input=data, past_seq=past, autoencoder=ae,
                                               fut_seq=fut, space=space, x_cond=x_cond, prediction_horizon=ph,
                                               transform_to_metric_space=_to_metric_space)
    sel, idx = B.get_ksimilarity_loss(loss, out_c, fut_c, similarity_space=space, autoencoder=ae)
    want = {"input_space": z["idx"], "metric_space": m["idx"], "latent_space": z["idx_latent"]}[space]
    np.testing.assert_array_equal(idx.cpu().numpy(), want)
    ref_sel = torch.gather(dev("loss").view(3, -1), 1, torch.from_numpy(want).to(cuda).unsqueeze(1)).squeeze(1)
    assert float((sel - ref_sel).abs().max()) < 1e-5
    if space == "input_space":
        assert float((out_c - dev("decoded")).abs().max()) < 1e-4
        final = (sel * w).mean()
        assert abs(float(final) - float(z["final"])) < 1e-5
    if space == "metric_space":
        assert float((out_c - dev_m("out_c")).abs().max()) < 1.5e-4  # the decoder's 1e-4, scaled by the box
        sim = B._metrics.ade(fut_c[:, 0], out_c, reduction="none")
        assert float((sim - dev_m("sim")).abs().max()) < 1e-4
    g = torch.autograd.grad(sel.sum(), samples, retain_graph=False)[0]
    torch.cuda.synchronize()
    rows = torch.arange(3, device=cuda) * k + idx
    mask = torch.zeros(3 * k, dtype=torch.bool, device=cuda)
    mask[rows] = True
    assert float(g[~mask].abs().max()) == 0.0 and float(g[mask].abs().max()) > 0.0


@pytest.mark.gpu
def test_best_of_k_kernel_semantics(cuda):
    """sd_best_of_k against torch.min(dim).indices + gather on ties (first minimum), NaNs (first NaN)
    and k = 1, and its backward against gather's autograd; sd_pose_loss against the oracle at
    ragged sizes."""
    from skeletondiffusion_amd import training

    g = torch.Generator().manual_seed(3)
    for nseq, k in ((1, 1), (5, 7), (300, 50), (2, 64)):
        loss = torch.rand(nseq * k, generator=g)
        sim = torch.rand(nseq * k, generator=g)
        if k > 2:
            sim.view(nseq, k)[0, 1] = sim.view(nseq, k)[0, 2] = -1.0  # tie: the first wins
        if nseq > 1 and k > 3:
            sim.view(nseq, k)[1, 3] = float("nan")  # torch.min propagates the first NaN
        lg = loss.to(cuda).requires_grad_(True)
        sel, idx = training.best_of_k(lg, k, sim.to(cuda))
        ref_sel, ref_idx = O.best_of_k(loss, k, sim)
        np.testing.assert_array_equal(idx.cpu().numpy(), ref_idx.numpy())
        np.testing.assert_array_equal(sel.detach().cpu().numpy(), ref_sel.numpy())
        up = torch.rand(nseq, generator=g)
        sel.backward(up.to(cuda))
        lr = loss.clone().requires_grad_(True)
        O.best_of_k(lr, k, sim)[0].backward(up)
        np.testing.assert_array_equal(lg.grad.cpu().numpy(), lr.grad.numpy())
    for shape in ((3, 5, 7, 21, 3), (1, 50, 120, 16, 3), (2, 1, 1, 1, 1)):
        pred = torch.randn(shape, generator=g)
        tgt = torch.randn((shape[0],) + shape[2:], generator=g)
        for mse in (False, True):
            got = training.pose_loss(pred.to(cuda), tgt.to(cuda), mse).cpu()
            np.testing.assert_allclose(got.numpy(), O.pose_loss(pred, tgt, mse).numpy(), rtol=1e-5, atol=1e-6)
