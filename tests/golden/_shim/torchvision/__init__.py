"""Minimal local stand-in for torchvision (absent in this image) so that the
reference's trainer module R:resnet/pytorch_ddp/ddp_train.py can be imported to
run its own train_epoch (:52-75) when generating golden vectors.  Only the
names the reference touches at import/call time are provided; models come
from distributed_training_amd.resnet (torchvision-0.15-equivalent)."""
from . import datasets, models, transforms  # noqa: F401
