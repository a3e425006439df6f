"""FID (reference metrics/FID/): InceptionV3 pool_3 features on the HIP conv
kernels, activation statistics on the GPU, Frechet distance on the host."""
