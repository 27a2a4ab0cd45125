"""A/B aid, not the product: one MinimalV1LVGDiT instance's block projections on the library GEMMs (hipBLASLt bf16
through F.linear, torch._scaled_mm for the fp8 option), with the MLP GELU and the gated residuals in the elementwise
kernels: the round-2 path the hand-written GEMMs replaced. The package has no library GEMM on any
path; this patches the net's projection methods, for timing comparisons only.

    sys.path.insert(0, "tools"); from library_gemm_net import use_library_gemms; use_library_gemms(net)
"""
import types

import torch
import torch.nn.functional as F

from cosmos_predict2 import _native as N


def use_library_gemms(net) -> None:
    def _own(self, x, w):  # no hand-written bf16 GEMM: every projection goes through _linear below
        return False

    def _own_fp8(self, w):
        return False

    def _linear(self, x, w, key, gelu_in=False):
        if isinstance(x, tuple) or self.linear_precision == "fp8":
            q, s = x if isinstance(x, tuple) else N.quant_fp8_rows(x, gelu=gelu_in)
            w8, ws = self._fp8_weight(key, w)
            return torch._scaled_mm(q, w8.t(), scale_a=s, scale_b=ws, out_dtype=torch.bfloat16)
        if gelu_in:
            N.gelu_(x)
        y = F.linear(x, w)
        if key.endswith("mlp.layer1"):  # the product fuses this GELU into its GEMM's epilogue
            N.gelu_(y)
        return y

    net._own = types.MethodType(_own, net)
    net._own_fp8 = types.MethodType(_own_fp8, net)
    net._linear = types.MethodType(_linear, net)
