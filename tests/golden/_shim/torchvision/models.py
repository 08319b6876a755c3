from distributed_training_amd.resnet import resnet18, resnet50, resnet152  # noqa: F401
