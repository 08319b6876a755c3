class _T:
    def __init__(self, *a, **k):
        pass

    def __call__(self, x):
        return x


Compose = Pad = RandomHorizontalFlip = RandomCrop = ToTensor = Normalize = _T
