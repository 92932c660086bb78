from .logging import init_logger, get_logger, MetricsWriter  # noqa: F401
