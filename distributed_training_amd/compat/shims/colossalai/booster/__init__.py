from distributed_training_amd.compat.colossalai import Booster  # noqa: F401
