"""FlowUniPCMultistepScheduler for the MI355X sampler.

Same API and numerics as the reference scheduler
(cosmos_predict2/_src/predict2/models/fm_solvers_unipc.py: set_timesteps :150-219, step :630-713):
the schedule and every scalar coefficient are computed on the host with fp32 0-dim CPU tensors in
the reference's operation order (bit-exact), and the elementwise update of one step
(convert_model_output + corrector + predictor) runs as ONE fused HIP kernel (cp25_unipc_step) over
the latent, in place, with the solver history kept in HBM.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np
import torch

from . import _native

_ONE = torch.tensor(1.0, dtype=torch.float32)


def _lambda(sigma: torch.Tensor) -> torch.Tensor:
    alpha = 1 - sigma
    return torch.log(alpha) - torch.log(sigma)


class FlowUniPCMultistepScheduler:
    """UniPC (bh2, predict_x0, flow prediction, solver_order 2, lower_order_final)."""

    def __init__(self, num_train_timesteps: int = 1000, solver_order: int = 2, shift: float = 1.0):
        if solver_order != 2:
            raise NotImplementedError("the fused update implements solver_order=2 (the reference default)")
        self.num_train_timesteps = num_train_timesteps
        self.solver_order = solver_order
        alphas = np.linspace(1, 1 / num_train_timesteps, num_train_timesteps)[::-1].copy()
        s = torch.from_numpy(1.0 - alphas).to(torch.float32)
        s = shift * s / (1 + (shift - 1) * s)
        self.sigma_max = s[0].item()
        self.sigma_min = s[-1].item()
        self.config_shift = shift
        self.timesteps: Optional[torch.Tensor] = None
        self.sigmas: Optional[torch.Tensor] = None
        self.num_inference_steps: Optional[int] = None
        self._reset_state()

    # ------------------------------------------------------------------ schedule
    def set_timesteps(self, num_inference_steps: int, device=None, shift: Optional[float] = None,
                      use_kerras_sigma: bool = False) -> None:
        if use_kerras_sigma:
            smax, smin, rho = 200, 0.01, 7
            ramp = np.arange(num_inference_steps + 1) / num_inference_steps
            lo, hi = smin ** (1 / rho), smax ** (1 / rho)
            sig = (hi + ramp * (lo - hi)) ** rho
            sig = sig / (1 + sig)
        else:
            sig = np.linspace(self.sigma_max, self.sigma_min, num_inference_steps + 1).copy()[:-1]
            sh = self.config_shift if shift is None else shift
            sig = sh * sig / (1 + (sh - 1) * sig)
        self.timesteps = torch.from_numpy(sig * self.num_train_timesteps).to(device=device, dtype=torch.int64)
        self.sigmas = torch.from_numpy(np.concatenate([sig, [0]]).astype(np.float32))  # stays on the CPU
        self.num_inference_steps = len(self.timesteps)
        self._reset_state()

    def _reset_state(self):
        self.lower_order_nums = 0
        self.this_order = None
        self._step_index: Optional[int] = None
        self._have_last = False
        self._buf = None  # (x, m0, m1, last) device fp32 buffers

    @property
    def step_index(self):
        return self._step_index

    # ------------------------------------------------------------------ scalar coefficients
    def _bh(self, i_t: int, i_s0: int, i_prev: int, order: int):
        sg = self.sigmas
        sigma_t, sigma_s0 = sg[i_t], sg[i_s0]
        alpha_t = 1 - sigma_t
        lam_s0 = _lambda(sigma_s0)
        h = _lambda(sigma_t) - lam_s0
        rks: List = []
        if order == 2:
            rks.append((_lambda(sg[i_prev]) - lam_s0) / h)
        rks_t = torch.tensor([float(r) for r in rks] + [1.0], dtype=torch.float32)
        hh = -h
        h_phi_1 = torch.expm1(hh)
        h_phi_k = h_phi_1 / hh - 1
        fact = 1
        B_h = torch.expm1(hh)
        R, b = [], []
        for i in range(1, order + 1):
            R.append(torch.pow(rks_t, i - 1))
            b.append(h_phi_k * fact / B_h)
            fact *= i + 1
            h_phi_k = h_phi_k / hh - 1 / fact
        return {
            "a": (sigma_t / sigma_s0).item(),
            "b": (alpha_t * h_phi_1).item(),
            "c": (alpha_t * B_h).item(),
            "inv_rk": (_ONE / rks[0]).item() if order == 2 else 0.0,
            "R": torch.stack(R),
            "bvec": torch.tensor([float(x) for x in b], dtype=torch.float32),
        }

    def _params(self) -> _native.UniPCParams:
        k = self._step_index
        P = _native.UniPCParams()
        P.sigma = self.sigmas[k].item()
        use_corr = k > 0 and self._have_last
        P.use_corr = int(use_corr)
        P.order_c = 1
        if use_corr:
            oc = self.this_order
            c = self._bh(k, k - 1, k - 2, oc)
            rhos = torch.tensor([0.5], dtype=torch.float32) if oc == 1 else torch.linalg.solve(c["R"], c["bvec"])
            P.order_c = oc
            P.c_a, P.c_b, P.c_c, P.c_inv_rk = c["a"], c["b"], c["c"], c["inv_rk"]
            P.c_rho0 = rhos[0].item()
            P.c_rho_last = rhos[-1].item()
        order = min(self.solver_order, len(self.timesteps) - k)
        order = min(order, self.lower_order_nums + 1)
        p = self._bh(k + 1, k, k - 1, order)
        P.order_p = order
        P.p_a, P.p_b, P.p_c, P.p_inv_rk = p["a"], p["b"], p["c"], p["inv_rk"]
        P.p_rho0 = 0.5
        return P, order

    # ------------------------------------------------------------------ stepping
    def begin(self, sample: torch.Tensor) -> torch.Tensor:
        """Adopt `sample` as the running state (fp32, contiguous, in HBM); returns the state tensor
        that step_() updates in place."""
        x = sample.detach().to(torch.float32).contiguous().clone()
        z = torch.zeros_like(x)
        self._buf = (x, z, z.clone(), z.clone())
        return x

    def _init_step_index(self, timestep) -> None:
        t = timestep.to(self.timesteps.device) if isinstance(timestep, torch.Tensor) else timestep
        idx = (self.timesteps == t).nonzero()
        self._step_index = idx[1 if len(idx) > 1 else 0].item()

    def step_(self, v: torch.Tensor, timestep) -> torch.Tensor:
        """Fused in-place step on the state from begin(); v = velocity prediction (same numel)."""
        if self.num_inference_steps is None:
            raise ValueError("Number of inference steps is 'None', you need to run 'set_timesteps' first")
        if self._buf is None:
            raise ValueError("call begin(sample) before step_()")
        if self._step_index is None:
            self._init_step_index(timestep)
        P, order = self._params()
        x, m0, m1, last = self._buf
        _native.unipc_step(x, v.reshape(x.shape) if v.is_contiguous() else v.contiguous().reshape(x.shape),
                           m0, m1, last, P)
        self._have_last = True
        self.this_order = order
        if self.lower_order_nums < self.solver_order:
            self.lower_order_nums += 1
        self._step_index += 1
        return x

    def step(self, model_output: torch.Tensor, timestep, sample: torch.Tensor, return_dict: bool = True,
             generator=None):
        """Reference-compatible step(): returns prev_sample (a new tensor)."""
        if self._buf is None or self._buf[0].data_ptr() != sample.data_ptr():
            if self._buf is None:
                self.begin(sample)
            else:
                self._buf[0].copy_(sample.reshape(self._buf[0].shape))
        out = self.step_(model_output.float(), timestep).clone().reshape(sample.shape)
        if not return_dict:
            return (out, None)
        return {"prev_sample": out}
