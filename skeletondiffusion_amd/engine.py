"""SamplingEngine: binds a (Nonisotropic|Isotropic)GaussianDiffusion module to a libskeldiff plan.

* The plan is built from the module's own state_dict (the reference key names), so a checkpoint
  loaded with `load_state_dict` (reference src/utils/load.py:11-17) is what runs.
* The plan is rebuilt automatically when any parameter/buffer changes (tracked through torch's
  per-tensor version counters and storage pointers), e.g. after an optimizer step.
* Workspaces are cached per (device, rows).  All launches go to torch's current HIP stream.
* There is no CPU path: a module on the CPU, or a missing library, raises SkelDiffError.
"""
from __future__ import annotations

import ctypes
import threading
from typing import Optional, Tuple

import torch

from . import _lib
from . import ops  # noqa: F401  (registers torch.ops.skeldiff.sample_loop)
from ._lib import SkelDiffError, check, ptr


def _stream(dev: torch.device) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


class SamplingEngine:
    def __init__(self, diffusion):
        self.diff = diffusion
        self._plan = None
        self._key = None
        self._device = None
        self._ws = {}  # (device, rows, stream) -> workspace
        self._ws_lock = threading.Lock()
        self._graph = False
        self._precision = 0
        self._options = {}  # sd_plan_set_option values, re-applied when the plan is rebuilt

    # ---------------------------------------------------------------------------------------
    def __del__(self):
        try:
            if self._plan is not None:
                _lib.lib().sd_plan_destroy(self._plan)
        except Exception:
            pass

    def _device_of_module(self) -> torch.device:
        dev = self.diff.betas.device
        if dev.type != "cuda":
            raise SkelDiffError(
                "skeletondiffusion_amd samples on the MI355X HIP engine only: move the diffusion module to "
                "a ROCm device first (e.g. diffusion.to('cuda')); there is no CPU sampling path")
        return dev

    def _fingerprint(self):
        return tuple((t.data_ptr(), t._version) for t in self.diff.state_dict(keep_vars=True).values()
                     if torch.is_tensor(t))

    def _desc(self):
        m = self.diff.model
        d = _lib.SDPlanDesc()
        unsupported = []
        if getattr(m, "learned_time_embedding", False):
            unsupported.append("learned/random sinusoidal time embedding")
        if getattr(m, "learned_variance", False):
            unsupported.append("learned_variance")
        if m.self_condition:
            unsupported.append("self_condition")
        norm_types = {"none": 0, "layer": 1}
        norm = m.graph_kwargs.get("norm_type", "none")
        if norm not in norm_types:
            unsupported.append(f"norm_type {norm!r}")
        objectives = {"pred_x0": 0, "pred_noise": 1, "pred_v": 2}
        iso = not hasattr(self.diff, "posterior_mean_coef1_x0")
        if self.diff.objective not in objectives or (self.diff.objective != "pred_x0" and not iso):
            unsupported.append(f"objective {self.diff.objective!r} on the nonisotropic sampler (pred_x0 only; the "
                               "isotropic sampler also takes pred_noise / pred_v)")
        if unsupported:
            raise SkelDiffError("sampling engine does not support: " + ", ".join(unsupported))
        d.num_nodes = m.channels
        d.latent_dim = self.diff.seq_length
        d.cond_dim = m.cond_dim
        d.out_dim = m.out_dim
        d.depth = m.depth
        d.attn_heads = m.attn_heads
        d.attn_dim_head = m.attn_dim_head
        d.use_attention = int(bool(m.use_attention))
        d.self_condition = 0
        d.learn_influence = int(bool(m.learn_influence))
        nt = m.node_types
        self._node_types = None
        if nt is not None:
            arr = (ctypes.c_int64 * m.channels)(*[int(v) for v in torch.as_tensor(nt).tolist()])
            self._node_types = arr
            d.num_node_types = int(torch.as_tensor(nt).max()) + 1
            d.node_types = ctypes.cast(arr, ctypes.POINTER(ctypes.c_int64))
        else:
            d.num_node_types = 0
        d.timesteps = self.diff.num_timesteps
        d.isotropic = int(not hasattr(self.diff, "posterior_mean_coef1_x0"))
        d.activation = 1 if self.diff.diffusion_activation == "tanh" else 0
        d.sinusoidal_theta = float(m.sinusoidal_pos_emb_theta)
        d.objective = objectives.get(self.diff.objective, 0)
        d.norm_type = norm_types.get(norm, 0)  # 'layer': Block LayerNorm over nodes (J = 16 / 17 / 21)
        return d

    PRECISIONS = {"f32": 0, "half": 1, "bf16": 2}

    def set_precision(self, precision: str) -> None:
        """Arithmetic of the graph-linear launches: "f32" (default; f32-accurate split-f16
        products), "half" (one f16 product per multiply-add, f32 accumulate) or "bf16" (bf16
        products, bf16 latents and residual-stream activations in HBM, f32 posterior update;
        BASELINE config 5).  See sd_plan_set_precision."""
        if precision not in self.PRECISIONS:
            raise SkelDiffError(f"precision must be one of {sorted(self.PRECISIONS)}, got {precision!r}")
        mode = self.PRECISIONS[precision]
        if self.diff.betas.device.type == "cuda":  # validate now (builds the plan if needed)
            check(_lib.lib().sd_plan_set_precision(self.plan(), mode))
        self._precision = mode

    OPTIONS = {"kernel_variant": _lib.SD_OPT_KERNEL_VARIANT, "gl4_tile": _lib.SD_OPT_GL4_TILE,
               "row_chains": _lib.SD_OPT_ROW_CHAINS, "gl4_staging": _lib.SD_OPT_GL4_STAGING,
               "split_route": _lib.SD_OPT_SPLIT_ROUTE, "last_chains": _lib.SD_OPT_LAST_CHAINS,
               "last_route": _lib.SD_OPT_LAST_ROUTE, "update_kernel": _lib.SD_OPT_UPDATE_KERNEL,
               "v5_mix": _lib.SD_OPT_V5_MIX, "attention": _lib.SD_OPT_ATTENTION}
    READ_ONLY = ("last_chains", "last_route")
    # The split-f16 graph-linear tiles need |x| < 65504.  A wave whose operands leave that range
    # recomputes its tiles on exact-f32 MFMA inside the kernel (sd_graph_linear_v4.hip:
    # exact_tile_f32; every f16-product kernel: the split routes' GEMM phases and the one-kernel
    # tiles) and sets SD_STATUS_F16_RANGE in the workspace status word for information (status());
    # sample() needs no host check, no re-run and no warning: in f32 mode its latents are
    # f32-accurate for any finite input.

    def set_option(self, name: str, value: int) -> None:
        """Per-plan kernel option (sd_plan_set_option): "kernel_variant" (0 auto, 1..5),
        "gl4_tile" (<waves><row tiles><col tiles>, 0 auto), "row_chains" (1..8), "gl4_staging"
        (0 LDS-DMA, 1 register-staged), "split_route" (0 auto, 1 never, 2 k_gl4y, 3 k_gl4t, 4 k_gl4t
        except to_qkv + attention), "update_kernel" (0 matrix cores, 1 element-per-thread),
        "attention" (0 auto, 2 to_qkv mixing in the attention kernel, 3 separate mixing pass),
        "v5_mix" (0 matrix cores, 1 VALU);
        get_option("last_chains") reads the row chains the last sample_loop ran.  Kept across plan rebuilds;
        other engines (plans) in the process are unaffected."""
        if name not in self.OPTIONS or name in self.READ_ONLY:
            raise SkelDiffError(f"unknown or read-only option {name!r}; one of "
                                f"{sorted(set(self.OPTIONS) - set(self.READ_ONLY))}")
        if self._plan is not None:
            check(_lib.lib().sd_plan_set_option(self._plan, self.OPTIONS[name], int(value)))
        self._options[name] = int(value)

    def get_option(self, name: str) -> int:
        v = ctypes.c_int64()
        check(_lib.lib().sd_plan_get_option(self.plan(), self.OPTIONS[name], ctypes.byref(v)))
        return int(v.value)

    @property
    def precision(self) -> str:
        return {v: k for k, v in self.PRECISIONS.items()}[self._precision]

    def plan(self):
        dev = self._device_of_module()
        key = (dev, self._fingerprint())
        if self._plan is not None and key == self._key:
            return self._plan
        L = _lib.lib()
        if self._plan is not None:
            torch.cuda.synchronize(dev)
            L.sd_plan_destroy(self._plan)
            self._plan = None
        desc = self._desc()
        handle = ctypes.c_void_p()
        with torch.cuda.device(dev):
            check(L.sd_plan_create(ctypes.byref(handle), ctypes.byref(desc)))
            sd = self.diff.state_dict()
            stream = _stream(dev)
            keep = []
            try:
                for i in range(L.sd_plan_num_tensors(handle)):
                    name = L.sd_plan_tensor_name(handle, i).decode()
                    if name not in sd:
                        raise SkelDiffError(f"state_dict has no tensor {name!r} required by the sampling engine")
                    t = sd[name].detach().to(device=dev, dtype=torch.float32).contiguous()
                    keep.append(t)
                    check(L.sd_plan_set_tensor(handle, name.encode(), ptr(t), t.numel(), stream))
                check(L.sd_plan_finalize(handle, stream))
                check(L.sd_plan_set_precision(handle, self._precision))
                for name, value in self._options.items():
                    check(L.sd_plan_set_option(handle, self.OPTIONS[name], value))
            except Exception:
                L.sd_plan_destroy(handle)
                raise
        self._plan, self._key, self._device = handle, key, dev
        return handle

    def workspace(self, rows: int) -> Tuple[torch.Tensor, int]:
        """The workspace of `rows` rows for torch's current stream.  A workspace belongs to one
        stream at a time (include/skeldiff.h), so concurrent callers on different streams each
        get their own; it is allocated on that stream (caching-allocator ordering)."""
        plan = self.plan()
        nbytes = int(_lib.lib().sd_workspace_bytes(plan, rows))
        stream = _stream(self._device)
        k = (self._device, rows, stream)
        with self._ws_lock:
            ws = self._ws.get(k)
            if ws is None or ws.numel() < nbytes:
                if len(self._ws) >= 8:  # bounded: drop the oldest
                    self._ws.pop(next(iter(self._ws)))
                ws = torch.empty(nbytes, dtype=torch.uint8, device=self._device)
                self._ws[k] = ws
        return ws, nbytes

    # ---------------------------------------------------------------------------------------
    def _f32(self, t: Optional[torch.Tensor], shape=None) -> Optional[torch.Tensor]:
        if t is None:
            return None
        t = t.to(device=self._device, dtype=torch.float32).contiguous()
        if shape is not None and tuple(t.shape) != tuple(shape):
            raise SkelDiffError(f"expected shape {tuple(shape)}, got {tuple(t.shape)}")
        return t

    def _cond(self, x_cond, rows):
        m = self.diff.model
        if m.cond_dim == 0 or not self.diff.condition:
            return None, 1
        if x_cond is None:
            raise SkelDiffError("x_cond is required (diffusion_conditioning=True)")
        x_cond = self._f32(x_cond)
        bc = x_cond.shape[0]
        if bc == 0 or rows % bc:
            raise SkelDiffError(f"x_cond rows ({bc}) must divide the batch ({rows}) (base.py:246-248)")
        return x_cond, rows // bc

    def denoiser_forward(self, x: torch.Tensor, t: int, x_cond=None) -> torch.Tensor:
        plan = self.plan()
        J, D = self.diff.channels, self.diff.seq_length
        x = self._f32(x)
        rows = x.shape[0]
        if tuple(x.shape[1:]) != (J, D):
            raise SkelDiffError(f"x must be (B, {J}, {D})")
        xc, rep = self._cond(x_cond, rows)
        out = torch.empty((rows, J, self.diff.model.out_dim), device=self._device, dtype=torch.float32)
        ws, nb = self.workspace(rows)
        check(_lib.lib().sd_denoiser_forward(plan, ptr(x), ptr(xc), rep, int(t), ptr(out), rows, ptr(ws), nb,
                                             _stream(self._device)))
        return out

    def denoiser_trace(self, x: torch.Tensor, t: int, x_cond=None):
        """-> (x0, [block outputs]) -- sd_denoiser_trace: init_lin, per layer the ResnetBlock and
        attention (Identity for the last) outputs, final_res_block; each (B, J, D + cond_dim)."""
        plan = self.plan()
        J, D = self.diff.channels, self.diff.seq_length
        x = self._f32(x)
        rows = x.shape[0]
        xc, rep = self._cond(x_cond, rows)
        m = self.diff.model
        H = m.dim + m.cond_dim
        acts = [torch.empty((rows, J, H), device=self._device) for _ in range(2 + 4 * m.depth)]
        arr = (ctypes.c_void_p * len(acts))(*[a.data_ptr() for a in acts])
        out = torch.empty((rows, J, m.out_dim), device=self._device, dtype=torch.float32)
        ws, nb = self.workspace(rows)
        check(_lib.lib().sd_denoiser_trace(plan, ptr(x), ptr(xc), rep, int(t), ptr(out), rows, ptr(ws), nb, arr,
                                           len(acts), _stream(self._device)))
        return out, acts

    def p_sample(self, x, t: int, x_cond=None, eps=None, clip: bool = True):
        plan = self.plan()
        x = self._f32(x)
        rows = x.shape[0]
        x0_raw = self.denoiser_forward(x, t, x_cond)
        out = torch.empty_like(x)
        mean = torch.empty_like(x)
        eps = self._f32(eps, x.shape) if (eps is not None and t > 0) else None
        noise_used = torch.empty_like(x) if t > 0 else None
        L = _lib.lib()
        JD = x.shape[1] * x.shape[2]
        if eps is None and t > 0:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        else:
            seed = 0
        flags = 0 if clip else _lib.SD_FLAG_NO_CLIP
        check(L.sd_p_sample_update(plan, ptr(x0_raw), ptr(x), ptr(eps), JD, seed, 0, int(t), ptr(out),
                                   ptr(mean), JD, ptr(noise_used), JD, rows, flags, _stream(self._device)))
        x0 = self.start_from_output(x, t, x0_raw)
        if clip:
            x0.clamp_(-1.0, 1.0)
        return out, x0, (noise_used if t > 0 else 0.0), mean

    def start_from_output(self, x, t: int, out):
        """x0 from the Denoiser output per objective, as model_predictions forms it (base.py:219-241):
        activation, then predict_start_from_noise / _from_v for the isotropic pred_noise / pred_v
        (isotropic.py:48-52, 66-70); the update kernels do the same arithmetic before their clamp."""
        x0 = torch.tanh(out) if self.diff.diffusion_activation == "tanh" else out
        obj = self.diff.objective
        if obj == "pred_noise":
            x0 = self.diff.sqrt_recip_alphas_cumprod[t] * x - self.diff.sqrt_recipm1_alphas_cumprod[t] * x0
        elif obj == "pred_v":
            x0 = self.diff.sqrt_alphas_cumprod[t] * x - self.diff.sqrt_one_minus_alphas_cumprod[t] * x0
        return x0

    def sample_loop(self, rows: int, x_cond=None, start_noise=None, sampling_noise=None,
                    record=(False, False), seed: Optional[int] = None, row0: int = 0,
                    graph: Optional[bool] = None, out: Optional[torch.Tensor] = None,
                    keep_start: bool = True, clip: bool = True):
        """-> (img, start_noise, noise_t, mean_t, imgs).  Unrequested records are None.
        `out` (rows, J, D) fp32 may be passed to reuse an output buffer (keeps a captured
        hipGraph valid across calls).  clip=False: x0 is not clamped (clip_denoised=False)."""
        plan = self.plan()
        J, D, T = self.diff.channels, self.diff.seq_length, self.diff.num_timesteps
        dev = self._device
        flags = 0
        start = self._f32(start_noise, (rows, J, D))
        samp = self._f32(sampling_noise, (rows, T - 1, J, D)) if sampling_noise is not None else None
        if start is None:
            flags |= _lib.SD_FLAG_DEVICE_START
        if samp is None:
            flags |= _lib.SD_FLAG_DEVICE_NOISE
        if graph if graph is not None else self._graph:
            flags |= _lib.SD_FLAG_GRAPH
        if not clip:
            flags |= _lib.SD_FLAG_NO_CLIP
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if (flags & (_lib.SD_FLAG_DEVICE_START |
                                                                             _lib.SD_FLAG_DEVICE_NOISE)) else 0
        xc, rep = self._cond(x_cond, rows)
        rec_noise, rec_img = record
        if out is None:
            out = torch.empty((rows, J, D), device=dev, dtype=torch.float32)
        elif out.shape != (rows, J, D) or out.dtype != torch.float32 or not out.is_contiguous() or out.device != dev:
            raise SkelDiffError("out must be a contiguous fp32 (rows, J, D) tensor on the module's device")
        tm1 = max(T - 1, 0)
        mean_t = torch.empty((rows, tm1, J, D), device=dev) if rec_noise and not rec_img else None
        noise_t = torch.empty((rows, tm1, J, D), device=dev) if rec_noise else None
        imgs = torch.empty((rows, tm1, J, D), device=dev) if rec_img else None
        start_out = torch.empty((rows, J, D), device=dev) if (start is None and keep_start) else None
        ws, _ = self.workspace(rows)
        # through the torch.library op skeldiff::sample_loop (ops.py): shape / dtype / device
        # validation against the plan, then sd_sample_loop on torch's current stream
        # the op's schema int is signed int64: a uint64 seed >= 2^63 travels as its two's
        # complement and the op masks it back to uint64 (ops.py)
        seed = int(seed) & (2 ** 64 - 1)
        seed_i64 = seed - 2 ** 64 if seed >= 2 ** 63 else seed
        torch.ops.skeldiff.sample_loop(plan.value, xc, rep, start, samp, seed_i64, int(row0), out, noise_t, mean_t,
                                       imgs, start_out, ws, flags)
        start_ret = start.clone() if start is not None else start_out
        return out, start_ret, noise_t, mean_t, imgs

    def status(self, rows: int) -> int:
        """Flags of the last sample_loop / denoiser_forward on the `rows`-row workspace
        (sd_workspace_status; synchronises the current stream): SD_STATUS_F16_RANGE = an
        activation left the f16 range of the f16 products and its tiles were recomputed on
        exact-f32 MFMA in the kernel (informational: in f32 mode the results are f32-accurate
        either way; half mode's in-range tiles stay one f16 product)."""
        ws, nb = self.workspace(rows)
        v = ctypes.c_uint32()
        check(_lib.lib().sd_workspace_status(self.plan(), ptr(ws), nb, ctypes.byref(v), _stream(self._device)))
        return int(v.value)

    def enable_graph(self, on: bool = True):
        """Capture whole sample() chains in hipGraphs (cached per shape/pointer set)."""
        self._graph = on
