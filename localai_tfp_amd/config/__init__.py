"""Configuration: application flags (app_config), per-model YAML (model_config), registry
(loader) and GGUF-driven defaults (guesser)."""
from .app_config import ApplicationConfig  # noqa: F401
from .loader import ModelConfigLoader  # noqa: F401
from .model_config import ModelConfig  # noqa: F401
