class CIFAR10:  # never constructed by the golden generator (needs network)
    def __init__(self, *a, **k):
        raise RuntimeError("CIFAR10 download is unavailable offline")
