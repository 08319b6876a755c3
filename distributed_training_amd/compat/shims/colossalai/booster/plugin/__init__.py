from distributed_training_amd.compat.colossalai import GeminiPlugin, LowLevelZeroPlugin, TorchDDPPlugin  # noqa: F401
