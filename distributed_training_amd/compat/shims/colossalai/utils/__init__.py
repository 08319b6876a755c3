from distributed_training_amd.compat.colossalai import get_current_device  # noqa: F401
