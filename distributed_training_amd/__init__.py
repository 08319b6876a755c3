"""distributed_training_amd — MI355X-native data-parallel gradient-synchronisation
engine (libgsync) behind the reference's DDP / DeepSpeed / ColossalAI wrappers.

Public surface:
  DistributedDataParallel   drop-in for torch.nn.parallel.DistributedDataParallel
  FusedSGD / FusedAdam / FusedAdamW / clip_grad_norm_
  Communicator              libgsync-owned RCCL communicator
  CapturedStep              the whole training step recorded into one hipGraph
  compat.deepspeed / compat.colossalai   API shims for the other two trainers
"""
from . import _lib  # noqa: F401
from .comm import Communicator, destroy_communicators, get_communicator  # noqa: F401
from .ddp import DDP, DistributedDataParallel, GradBucket, compute_bucket_assignment_by_size  # noqa: F401
from .graphs import CapturedStep  # noqa: F401
from .flatten import copy_flat_to, flatten_dense_tensors, unflatten_dense_tensors  # noqa: F401
from .multi_tensor import TensorListPlan  # noqa: F401
from .optim import FusedAdam, FusedAdamW, FusedSGD, clip_grad_norm_  # noqa: F401

__version__ = "0.1.0"
