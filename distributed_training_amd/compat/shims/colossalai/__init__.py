"""`colossalai` name -> libgsync (distributed_training_amd.compat.colossalai)."""
from distributed_training_amd.compat.colossalai import launch_from_torch  # noqa: F401
