"""Sigma_N construction from a joint correlation matrix (reference
src/core/diffusion/utils.py:3-86).  Host-side by design: the eigendecomposition fixes U, and at
J=51 (AMASS-MANO) the spectrum has degenerate eigenspaces, so U must come from exactly this
LAPACK `eigh(UPLO='L')` call (or from a checkpoint), never from a device solver
(hard part ii)."""
from __future__ import annotations

import torch


def dim_null_space(matrix: torch.Tensor) -> torch.Tensor:
    assert matrix.shape[-1] == matrix.shape[-2], "Matrix must be square"
    return torch.sum(torch.linalg.eigh(matrix)[0].abs() < 0.7e-7)


def is_positive_def(matrix: torch.Tensor) -> torch.Tensor:
    assert torch.allclose(matrix.transpose(-1, -2), matrix), "Matrix must be symmetric"
    ev = torch.linalg.eigvals(matrix)
    ok = (torch.real(ev) > 0).all()
    if ok:
        assert torch.isreal(ev).all(), "Eigenvalues must be real"
    return ok


def make_positive_definite(matrix: torch.Tensor, epsilon: float = 1e-6, if_submin: bool = False):
    ev = torch.linalg.eigvals(matrix)
    if is_positive_def(matrix):
        return matrix
    ev = torch.real(ev)
    shift = (ev.abs().max() + epsilon) if not if_submin else (-ev.min() + epsilon)
    out = matrix + torch.eye(matrix.shape[0], device=matrix.device) * shift
    assert dim_null_space(out) == 0
    return out


def normalize_cov(Sigma_N, Lambda_N, U, if_sigma_n_scale=True, sigma_n_scale="spectral", **kwargs):
    N = Sigma_N.shape[0]
    assert Lambda_N.shape == (N,)
    assert U.shape == (N, N)
    if if_sigma_n_scale:
        if sigma_n_scale == "spectral":
            scale = Lambda_N.max()
        elif sigma_n_scale == "frob":
            scale = Lambda_N.sum() / N
        else:
            raise AssertionError("Not implemented")
        Lambda_N = Lambda_N / scale
        Sigma_N = Sigma_N / scale
        recon = U @ torch.diag(Lambda_N) @ U.mT
        assert torch.isclose(Sigma_N, recon, atol=1e-06).all(), "Sigma_N must be equal to U @ Lambda_N @ U.t()"
    assert (Lambda_N > 0.7e-7).all(), f"Lambda_N must be positive definite: {Lambda_N}"
    assert is_positive_def(Sigma_N), "Sigma_N must be positive definite"
    return Sigma_N, Lambda_N


def get_cov_from_corr(correlation_matrix: torch.Tensor, if_sigma_n_scale=True, sigma_n_scale="spectral",
                      if_run_as_isotropic=False, diffusion_covariance_type="skeleton-diffusion", **kwargs):
    """-> (Sigma_N, Lambda_N, U).  Extra kwargs are accepted and ignored, as in the reference."""
    N = correlation_matrix.shape[0]
    dev = correlation_matrix.device
    if if_run_as_isotropic:
        if diffusion_covariance_type == "skeleton-diffusion":
            return torch.zeros_like(correlation_matrix), torch.ones(N, device=dev), torch.eye(N, device=dev)
        if diffusion_covariance_type == "anisotropic":
            return torch.eye(N, device=dev), torch.ones(N, device=dev), torch.eye(N, device=dev)
        return torch.zeros_like(correlation_matrix), torch.zeros(N, device=dev), torch.eye(N, device=dev)
    Sigma_N = make_positive_definite(correlation_matrix)
    Lambda_N, U = torch.linalg.eigh(Sigma_N, UPLO="L")
    Sigma_N, Lambda_N = normalize_cov(Sigma_N=Sigma_N, Lambda_N=Lambda_N, U=U,
                                      if_sigma_n_scale=if_sigma_n_scale, sigma_n_scale=sigma_n_scale)
    return Sigma_N, Lambda_N, U
