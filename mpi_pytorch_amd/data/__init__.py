from .loader import DevicePrefetcher, SyntheticSource, IMAGENET_MEAN, IMAGENET_STD  # noqa: F401
