"""Algorithm families (the reference's JDF algorithm layer, re-designed as
stream programs of batched tile kernels)."""
