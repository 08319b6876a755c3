from distributed_training_amd.compat.colossalai import DistCoordinator  # noqa: F401
