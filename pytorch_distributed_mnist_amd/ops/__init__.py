"""Host wrappers for the gfx950 HIP kernels (``csrc/kernels``) — shape-checked before launch."""
