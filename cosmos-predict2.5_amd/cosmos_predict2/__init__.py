"""MI355X-native cosmos-predict2.5 sampler (DiT + Wan2.1 VAE + UniPC) behind the reference's
`cosmos_predict2.inference` / `cosmos_predict2.config` API. Kernels: libcp25.so (include/cp25.h)."""

__version__ = "0.1.0"
