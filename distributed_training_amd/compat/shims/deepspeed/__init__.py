"""`deepspeed` name -> libgsync (distributed_training_amd.compat.deepspeed)."""
from distributed_training_amd.compat.deepspeed import (  # noqa: F401
    DeepSpeedEngine, WarmupLR, add_config_arguments, get_accelerator, init_distributed, initialize)
