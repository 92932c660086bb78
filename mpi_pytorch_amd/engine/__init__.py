from .step import TrainStep, build_model, build_training, loss_fn, steps_without_gc  # noqa: F401
