"""Drop-in `metrics` package (reference metrics/): the FID leg on the HIP kernels."""
