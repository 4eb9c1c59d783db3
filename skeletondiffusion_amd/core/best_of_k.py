"""The reference Trainer's best-of-k training relaxation (src/core/trainer.py:182-244) on the device.

`train_pick_best_sample_among_k = k > 1`: `NonisotropicGaussianDiffusion.forward(data, x_cond,
n_train_samples=k)` draws k noisy copies of every training sequence (p_losses' repeat_interleave,
base.py:264-268), and the loss of each sequence is the diffusion loss of the copy whose sample is
closest to the ground truth in `similarity_space`:
  latent_space -- the diffusion loss itself;
  input_space  -- AutoEncoder.loss(reduction='none') of the decoded samples against the future
                  (`sd_gru_decode` + `sd_pose_loss`);
  metric_space -- the ADE of the decoded samples in metric space (`sd_ade_fde` per_sample_ade).
The Trainer itself (ignite engine, EMA, optimiser loop) stays out of scope; these are
its three methods as functions of the state they read, with the reference's signatures, shapes and
return values.  Every step after `model(...)` runs on HIP kernels: the Mahalanobis loss
(training.MahalanobisLossFunction), the decoder, the similarity and the selection with its
gradient (training.BestOfKFunction).
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

from .. import metrics as _metrics
from .. import training as _training

SPACES = ("input_space", "metric_space", "latent_space")


def decode_diffusion_sample(samples, obs, autoencoder, x_cond=None, prediction_horizon=None):
    """trainer.py:278-287: decode the (b * k) sampled latents from each sequence's observed past
    (repeated k times) -> (out (b, k, ph, J, F), samples (b, k, J, D))."""
    x_t = obs.repeat_interleave(samples.shape[0] // obs.shape[0], dim=0)
    out = autoencoder.decode(x_t, samples, x_cond, prediction_horizon)
    out = out.view(obs.shape[0], -1, *out.shape[1:])
    return out, samples.view(obs.shape[0], -1, *samples.shape[1:])


def to_comparison_space_train(samples, diff_input, past_seq, autoencoder, fut_seq, space="latent_space", x_cond=None,
                              prediction_horizon=None, transform_to_metric_space: Optional[Callable] = None):
    """trainer.py:182-205 -> (out_comparespace, fut_seq_comparespace) of equal shape."""
    assert space in SPACES, f"Similarity space must be one of {SPACES} but is {space}"
    num_samples = samples.shape[0] // past_seq.shape[0]
    if x_cond is not None:
        x_cond = x_cond.repeat_interleave(num_samples, dim=0)
    if space in ("input_space", "metric_space"):
        ph = prediction_horizon if prediction_horizon is not None else fut_seq.shape[1]
        out, _ = decode_diffusion_sample(samples, past_seq, autoencoder, x_cond=x_cond, prediction_horizon=ph)
    if space == "input_space":
        out_c = out
        fut_c = fut_seq.unsqueeze(1).repeat_interleave(num_samples, dim=1)
    elif space == "metric_space":
        if transform_to_metric_space is None:
            raise ValueError("metric_space needs the skeleton's transform_to_metric_space")
        out_c = transform_to_metric_space(out).flatten(start_dim=3)
        fut_c = transform_to_metric_space(fut_seq).unsqueeze(1).flatten(start_dim=3).repeat_interleave(num_samples,
                                                                                                         dim=1)
    else:
        out_c = samples.view(diff_input.shape[0], -1, *samples.shape[1:])
        fut_c = diff_input.unsqueeze(1).repeat_interleave(num_samples, dim=1)
    assert out_c.shape == fut_c.shape
    return out_c, fut_c


def get_ksimilarity_loss(diffusion_loss, out_comparespace, fut_seq_comparespace, similarity_space="latent_space",
                         autoencoder=None, **kwargs):
    """trainer.py:207-222 -> (loss (b,), closest2gt_idx (b,)).  The similarity target is one future
    per sequence (the reference repeats it k times; the first copy is read)."""
    assert similarity_space in SPACES, f"Similarity space must be one of {SPACES} but is {similarity_space}"
    b = out_comparespace.shape[0]
    k = diffusion_loss.numel() // b
    with torch.no_grad():
        if similarity_space == "input_space":
            mse = autoencoder.loss_pose_type == "mse"
            assert mse or autoencoder.loss_pose_type in ("l1", "L1"), "Not implemnted"
            sim = _training.pose_loss(out_comparespace, fut_seq_comparespace[:, 0], mse)
        elif similarity_space == "metric_space":
            # ||out - fut|| over the flattened (J * 3) features, mean over frames: the per-sample ADE
            sim = _metrics.ade(fut_seq_comparespace[:, 0], out_comparespace, reduction="none")
        else:
            sim = None  # the diffusion loss itself
    loss, idx = _training.best_of_k(diffusion_loss.reshape(-1), k, sim)
    assert len(loss.shape) == 1 and loss.shape[0] == b
    return loss, idx


def pick_best_loss(model, data, x_cond, k: int, similarity_space="latent_space", autoencoder=None, past_seq=None,
                   fut_seq=None, prediction_horizon=None, transform_to_metric_space=None):
    """Trainer.loss (trainer.py:224-234) with train_pick_best_sample_among_k = k: the scalar the
    optimiser steps on.  Returns (loss, closest2gt_idx or None)."""
    loss, diff_weights, samples = model(data, x_cond=x_cond, n_train_samples=k)
    idx = None
    if k > 1:
        out_c, fut_c = to_comparison_space_train(samples, diff_input=data, past_seq=past_seq, autoencoder=autoencoder,
                                                 fut_seq=fut_seq, space=similarity_space, x_cond=x_cond,
                                                 prediction_horizon=prediction_horizon,
                                                 transform_to_metric_space=transform_to_metric_space)
        sim_loss, idx = get_ksimilarity_loss(loss, out_c, fut_c, similarity_space=similarity_space,
                                             autoencoder=autoencoder)
    else:
        sim_loss = loss
    return (sim_loss * diff_weights).mean(), idx
