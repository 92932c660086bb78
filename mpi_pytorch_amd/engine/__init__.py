from .step import (TrainStep, build_model, build_training, loss_fn,  # noqa: F401
                   reserve_device_memory, steps_without_gc)
