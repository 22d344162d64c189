"""Platform utilities: config, logging, metrics, tracing, service discovery."""
from .config import Config, load_config  # noqa: F401
from .log import Logger, get_logger  # noqa: F401
