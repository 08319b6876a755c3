from distributed_training_amd.compat.colossalai import HybridAdam  # noqa: F401
