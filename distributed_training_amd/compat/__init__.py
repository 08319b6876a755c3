"""API shims for the reference's DeepSpeed and ColossalAI trainers.

Put ``distributed_training_amd/compat/shims`` on PYTHONPATH and the reference
scripts' ``import deepspeed`` / ``import colossalai`` resolve to these
libgsync-backed implementations."""
