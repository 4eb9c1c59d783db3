"""The C-ABI library loads and exports every symbol include/skeldiff.h declares (no GPU work),
and its host-side argument validation behaves (no device call happens on these paths)."""
import ctypes
import os
import re

from conftest import REPO
from skeletondiffusion_amd import _lib

HEADER = os.path.join(REPO, "include", "skeldiff.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sd_[a-z_0-9]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert declared_symbols() == sorted(_lib.EXPORTED)


def test_library_exports_every_declared_symbol():
    lib = _lib.lib()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.sd_abi_version() == _lib.SD_ABI_VERSION == 4
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "skeldiff.h")).read()
    assert re.search(r"#define SD_ABI_VERSION (\d+)", hdr).group(1) == str(_lib.SD_ABI_VERSION)


def test_invalid_desc_is_rejected_on_host():
    lib = _lib.lib()
    d = _lib.SDPlanDesc()
    d.num_nodes = 65  # > 64
    d.latent_dim = 96
    d.out_dim = 96
    d.depth = 1
    d.timesteps = 10
    h = ctypes.c_void_p()
    rc = lib.sd_plan_create(ctypes.byref(h), ctypes.byref(d))
    assert rc == -1 and b"num_nodes" in lib.sd_last_error()
    d.num_nodes = 16
    d.self_condition = 1
    assert lib.sd_plan_create(ctypes.byref(h), ctypes.byref(d)) == -1
    assert b"self_condition" in lib.sd_last_error()


def test_plan_registry_uses_reference_state_dict_keys():
    """The plan's tensor registry (host-only, no device memory yet) lists exactly the
    reference's Denoiser keys plus the posterior buffers the sampler needs."""
    import torch

    import oracle as O

    lib = _lib.lib()
    nt = torch.tensor([0, 1, 2, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 7, 8, 9])
    d = _lib.SDPlanDesc(num_nodes=16, latent_dim=96, cond_dim=96, out_dim=96, depth=4, attn_heads=8,
                        attn_dim_head=32, use_attention=1, self_condition=0, learn_influence=1,
                        num_node_types=10, timesteps=100, isotropic=0, activation=0, sinusoidal_theta=10000.0)
    arr = (ctypes.c_int64 * 16)(*nt.tolist())
    d.node_types = ctypes.cast(arr, ctypes.POINTER(ctypes.c_int64))
    h = ctypes.c_void_p()
    assert lib.sd_plan_create(ctypes.byref(h), ctypes.byref(d)) == 0
    try:
        names = {lib.sd_plan_tensor_name(h, i).decode(): lib.sd_plan_tensor_numel(h, i)
                 for i in range(lib.sd_plan_num_tensors(h))}
        expect = {k: int(torch.Size(s).numel()) for k, s, _ in O.denoiser_param_shapes(O.release_config(16, nt))}
        expect.update({"posterior_mean_coef1_x0": 100 * 256, "posterior_mean_coef2_xt": 100 * 256,
                       "Lambda_posterior_log_variance_clipped": 100 * 16, "U": 256})
        assert names == expect
        assert lib.sd_plan_kernels_per_step(h) == 1 + 8 * 2 + 7 * 3 + 3 + 1 + 1
    finally:
        lib.sd_plan_destroy(h)


def test_plan_options_validated_on_host():
    """sd_plan_set_option / sd_plan_get_option are host-side plan state (no device call): every
    SD_OPT_* range is checked, including the split route's tiled value 3 (DESIGN.md §4d'')."""
    lib = _lib.lib()
    d = _lib.SDPlanDesc(num_nodes=16, latent_dim=96, cond_dim=96, out_dim=96, depth=1, attn_heads=8,
                        attn_dim_head=32, use_attention=1, self_condition=0, learn_influence=1,
                        num_node_types=10, timesteps=10, isotropic=0, activation=0, sinusoidal_theta=10000.0)
    arr = (ctypes.c_int64 * 16)(0, 1, 2, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 7, 8, 9)
    d.node_types = ctypes.cast(arr, ctypes.POINTER(ctypes.c_int64))
    h = ctypes.c_void_p()
    assert lib.sd_plan_create(ctypes.byref(h), ctypes.byref(d)) == 0, lib.sd_last_error()
    try:
        v = ctypes.c_int64()
        for value in (0, 1, 2, 3, 4):
            assert lib.sd_plan_set_option(h, _lib.SD_OPT_SPLIT_ROUTE, value) == 0
            assert lib.sd_plan_get_option(h, _lib.SD_OPT_SPLIT_ROUTE, ctypes.byref(v)) == 0 and v.value == value
        for value in (5, 6, 7):  # 5 / 6: the measured-slower routes ABI 3 removed
            assert lib.sd_plan_set_option(h, _lib.SD_OPT_SPLIT_ROUTE, value) == -1
            assert b"split route" in lib.sd_last_error()
        assert lib.sd_plan_set_option(h, _lib.SD_OPT_ROW_CHAINS, -1) == -1
        assert lib.sd_plan_set_option(h, _lib.SD_OPT_ROW_CHAINS, 0) == 0  # auto
        assert lib.sd_plan_set_option(h, _lib.SD_OPT_ROW_CHAINS, 8) == 0
        assert lib.sd_plan_set_option(h, _lib.SD_OPT_GL4_STAGING, 3) == -1
        assert lib.sd_plan_set_option(h, 99, 0) == -1
        for value in (2, 3, 4):  # 2 / 3: the pipelined forms ABI 3 removed
            assert lib.sd_plan_set_option(h, _lib.SD_OPT_UPDATE_KERNEL, value) == -1
        assert lib.sd_plan_set_option(h, _lib.SD_OPT_UPDATE_KERNEL, 0) == 0
        assert lib.sd_plan_set_option(h, _lib.SD_OPT_UPDATE_KERNEL, 1) == 0
        assert lib.sd_plan_get_option(h, _lib.SD_OPT_UPDATE_KERNEL, ctypes.byref(v)) == 0 and v.value == 1
        assert lib.sd_plan_set_option(h, _lib.SD_OPT_UPDATE_KERNEL, 0) == 0
        for opt, ok, bad in ((_lib.SD_OPT_V5_MIX, (1,), (2,)), (_lib.SD_OPT_ATTENTION, (2, 3), (1, 4))):
            assert lib.sd_plan_get_option(h, opt, ctypes.byref(v)) == 0 and v.value == 0
            for x in ok:
                assert lib.sd_plan_set_option(h, opt, x) == 0
                assert lib.sd_plan_get_option(h, opt, ctypes.byref(v)) == 0 and v.value == x
            for x in bad:  # SD_OPT_ATTENTION 1: the tail form ABI 3 removed
                assert lib.sd_plan_set_option(h, opt, x) == -1
            assert lib.sd_plan_set_option(h, opt, 0) == 0
        # SD_OPT_LAST_CHAINS: read-only, 0 before the plan's first sampling call
        assert lib.sd_plan_get_option(h, _lib.SD_OPT_LAST_CHAINS, ctypes.byref(v)) == 0 and v.value == 0
        assert lib.sd_plan_set_option(h, _lib.SD_OPT_LAST_CHAINS, 1) == -1
        assert b"read-only" in lib.sd_last_error()
        assert lib.sd_plan_get_option(h, _lib.SD_OPT_LAST_ROUTE, ctypes.byref(v)) == 0 and v.value == 0
        assert lib.sd_plan_set_option(h, _lib.SD_OPT_LAST_ROUTE, 1) == -1
    finally:
        lib.sd_plan_destroy(h)


def test_layernorm_plan_registry_and_limits():
    """norm_type 'layer' (ABI 4): each Block's LayerNorm(J) affine joins the registry under the
    reference keys; J outside the v4 mixing epilogue's 16 / 17 / 21 and the exact-f32 variants are
    refused on the host by name."""
    import dataclasses
    import torch

    import oracle as O

    lib = _lib.lib()
    nt = [0, 1, 2, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 7, 8, 9]
    arr = (ctypes.c_int64 * 16)(*nt)
    d = _lib.SDPlanDesc(num_nodes=16, latent_dim=96, cond_dim=96, out_dim=96, depth=4, attn_heads=8,
                        attn_dim_head=32, use_attention=1, self_condition=0, learn_influence=1,
                        num_node_types=10, timesteps=10, isotropic=0, activation=0, sinusoidal_theta=10000.0,
                        norm_type=1)
    d.node_types = ctypes.cast(arr, ctypes.POINTER(ctypes.c_int64))
    h = ctypes.c_void_p()
    assert lib.sd_plan_create(ctypes.byref(h), ctypes.byref(d)) == 0, lib.sd_last_error()
    try:
        names = {lib.sd_plan_tensor_name(h, i).decode(): lib.sd_plan_tensor_numel(h, i)
                 for i in range(lib.sd_plan_num_tensors(h))}
        cfg = dataclasses.replace(O.release_config(16, torch.tensor(nt)), norm_type="layer")
        expect = {k: int(torch.Size(s).numel()) for k, s, _ in O.denoiser_param_shapes(cfg)}
        ln = {k for k in expect if ".norm.norm." in k}
        assert len(ln) == 2 * 2 * 9  # (block1, block2) x (weight, bias) x 9 ResnetBlocks
        assert ln <= set(names) and all(names[k] == 16 for k in ln)
        assert lib.sd_plan_set_option(h, _lib.SD_OPT_KERNEL_VARIANT, 3) == -1
        assert b"norm_type" in lib.sd_last_error()
        assert lib.sd_plan_set_option(h, _lib.SD_OPT_KERNEL_VARIANT, 4) == 0
    finally:
        lib.sd_plan_destroy(h)
    d.num_nodes, d.num_node_types = 51, 0
    assert lib.sd_plan_create(ctypes.byref(h), ctypes.byref(d)) == -1
    assert b"norm_type" in lib.sd_last_error()
    d.num_nodes, d.norm_type = 16, 2
    assert lib.sd_plan_create(ctypes.byref(h), ctypes.byref(d)) == -1
