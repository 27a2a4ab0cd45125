"""UniPC (bh2, flow prediction, predict_x0) restatement — TEST INFRASTRUCTURE (see oracle/__init__.py).

Follows cosmos_predict2/_src/predict2/models/fm_solvers_unipc.py:
  schedule            :100-122 (train sigmas), set_timesteps :150-219
  convert_model_output:266-318
  predictor           :337-464 (multistep_uni_p_bh_update)
  corrector           :466-601 (multistep_uni_c_bh_update)
  step                :630-713
Scalar math uses fp32 0-dim CPU tensors exactly as the reference does (its sigmas live on the CPU,
:120/:219), so coefficients are bit-identical. Elementwise tensor math mirrors the reference's op
order; a CUDA tensor divided by a CPU scalar is a multiply by its fp32 reciprocal in PyTorch's CUDA
backend (aten/src/ATen/native/cuda/BinaryDivTrueKernel.cu), which `_div_scalar` restates.
"""
from __future__ import annotations

import numpy as np
import torch

NUM_TRAIN_TIMESTEPS = 1000


def train_sigmas(shift: float = 1.0) -> torch.Tensor:
    """fm_solvers_unipc.py:100-108 (use_dynamic_shifting=False)."""
    alphas = np.linspace(1, 1 / NUM_TRAIN_TIMESTEPS, NUM_TRAIN_TIMESTEPS)[::-1].copy()
    s = torch.from_numpy(1.0 - alphas).to(torch.float32)
    return shift * s / (1 + (shift - 1) * s)


def schedule(num_steps: int, shift: float = 5.0, use_karras: bool = False):
    """set_timesteps (:150-219) -> (timesteps int64 [N], sigmas fp32 [N+1])."""
    if use_karras:
        # EDM / Karras sigmas mapped to the flow time sigma/(1+sigma) (:170-179)
        smax, smin, rho = 200, 0.01, 7
        ramp = np.arange(num_steps + 1) / num_steps
        lo, hi = smin ** (1 / rho), smax ** (1 / rho)
        sig = (hi + ramp * (lo - hi)) ** rho
        sig = sig / (1 + sig)
    else:
        base = train_sigmas(1.0)  # the model builds the scheduler with shift=1 (text2world_model_rectified_flow.py:144-146)
        sig = np.linspace(base[0].item(), base[-1].item(), num_steps + 1).copy()[:-1]
        sig = shift * sig / (1 + (shift - 1) * sig)
    timesteps = torch.from_numpy(sig * NUM_TRAIN_TIMESTEPS).to(torch.int64)
    sigmas = torch.from_numpy(np.concatenate([sig, [0]]).astype(np.float32))
    return timesteps, sigmas


def _lam(sigma: torch.Tensor) -> torch.Tensor:
    # alpha = 1 - sigma ; lambda = log(alpha) - log(sigma)   (:259-260, :393-394)
    return torch.log(1 - sigma) - torch.log(sigma)


def _div_scalar(t: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    return t * (torch.tensor(1.0, dtype=torch.float32) / s)


def _coeffs(sigmas, i_t, i_s0, i_prev, order):
    """Shared scalar part of predictor/corrector: returns dict of fp32 0-dim tensors."""
    sigma_t, sigma_s0 = sigmas[i_t], sigmas[i_s0]
    alpha_t = 1 - sigma_t
    lambda_t, lambda_s0 = _lam(sigma_t), _lam(sigma_s0)
    h = lambda_t - lambda_s0
    rks = []
    for i_si in i_prev[: order - 1]:
        rks.append((_lam(sigmas[i_si]) - lambda_s0) / h)
    rk_list = rks + [1.0]
    rks_t = torch.tensor([float(r) for r in rk_list], dtype=torch.float32)
    hh = -h
    h_phi_1 = torch.expm1(hh)
    h_phi_k = h_phi_1 / hh - 1
    fact = 1
    B_h = torch.expm1(hh)  # bh2
    R, b = [], []
    for i in range(1, order + 1):
        R.append(torch.pow(rks_t, i - 1))
        b.append(h_phi_k * fact / B_h)
        fact *= i + 1
        h_phi_k = h_phi_k / hh - 1 / fact
    R = torch.stack(R)
    b = torch.tensor([float(x) for x in b], dtype=torch.float32)
    return dict(sigma_t=sigma_t, sigma_s0=sigma_s0, alpha_t=alpha_t, h_phi_1=h_phi_1, B_h=B_h, R=R, b=b, rks=rks)


class UniPC:
    """Stateful restatement of FlowUniPCMultistepScheduler (solver_order=2, bh2, lower_order_final)."""

    def __init__(self, num_steps: int, shift: float = 5.0, use_karras: bool = False, solver_order: int = 2):
        self.timesteps, self.sigmas = schedule(num_steps, shift, use_karras)
        self.order = solver_order
        self.outputs = [None] * solver_order  # converted model outputs, oldest first
        self.lower_order_nums = 0
        self.last_sample = None
        self.step_index = None
        self.this_order = None

    def _init_index(self, t):
        idx = (self.timesteps == t).nonzero()
        self.step_index = idx[1 if len(idx) > 1 else 0].item()  # :603-628

    def coefficients(self):
        """Scalar coefficients the next step() will use (for the fused device kernel)."""
        k = self.step_index
        out = {"sigma": self.sigmas[k]}
        use_corr = k > 0 and self.last_sample is not None
        out["use_corr"] = use_corr
        if use_corr:
            oc = self.this_order
            c = _coeffs(self.sigmas, k, k - 1, [k - 2], oc)
            out["corr"] = (oc, c, self._rhos_c(oc, c))
        n_after = min(self.lower_order_nums + 1, self.order)
        op = min(min(self.order, len(self.timesteps) - k), n_after)
        c = _coeffs(self.sigmas, k + 1, k, [k - 1], op)
        out["pred"] = (op, c, torch.tensor([0.5], dtype=torch.float32) if op == 2 else None)
        return out

    @staticmethod
    def _rhos_c(order, c):
        if order == 1:
            return torch.tensor([0.5], dtype=torch.float32)
        return torch.linalg.solve(c["R"], c["b"]).to(torch.float32)

    def step(self, v: torch.Tensor, t, sample: torch.Tensor) -> torch.Tensor:
        """step(model_output, timestep, sample) -> prev_sample (:630-713), fp32 tensors."""
        if self.step_index is None:
            self._init_index(t)
        k = self.step_index
        use_corr = k > 0 and self.last_sample is not None
        x0 = sample - self.sigmas[k] * v  # convert_model_output (:307-308)
        if use_corr:
            sample = self._corrector(x0, self.last_sample, sample, self.this_order)
        self.outputs = self.outputs[1:] + [x0]
        this_order = min(self.order, len(self.timesteps) - k)  # lower_order_final (:689-690)
        self.this_order = min(this_order, self.lower_order_nums + 1)
        self.last_sample = sample
        out = self._predictor(sample, self.this_order)
        if self.lower_order_nums < self.order:
            self.lower_order_nums += 1
        self.step_index += 1
        return out

    def _predictor(self, x, order):
        k = self.step_index
        m0 = self.outputs[-1]
        c = _coeffs(self.sigmas, k + 1, k, [k - 1], order)
        xt_ = (c["sigma_t"] / c["sigma_s0"]) * x - (c["alpha_t"] * c["h_phi_1"]) * m0
        if order == 2:
            d1 = _div_scalar(self.outputs[-2] - m0, c["rks"][0])
            pred = torch.tensor([0.5], dtype=torch.float32)[0] * d1
            return xt_ - (c["alpha_t"] * c["B_h"]) * pred
        return xt_ - (c["alpha_t"] * c["B_h"]) * 0

    def _corrector(self, model_t, last, this_sample, order):
        k = self.step_index
        m0 = self.outputs[-1]
        c = _coeffs(self.sigmas, k, k - 1, [k - 2], order)
        rhos = self._rhos_c(order, c)
        xt_ = (c["sigma_t"] / c["sigma_s0"]) * last - (c["alpha_t"] * c["h_phi_1"]) * m0
        d1t = model_t - m0
        if order == 2:
            d1 = _div_scalar(self.outputs[-2] - m0, c["rks"][0])
            s = rhos[0] * d1 + rhos[-1] * d1t
        else:
            s = 0 + rhos[-1] * d1t
        return xt_ - (c["alpha_t"] * c["B_h"]) * s
