from distributed_training_amd.compat.deepspeed import get_accelerator  # noqa: F401
