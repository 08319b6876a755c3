from distributed_training_amd.compat.colossalai import _DPPluginBase as DPPluginBase  # noqa: F401
