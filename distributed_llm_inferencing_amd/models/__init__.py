from .configs import ModelConfig, get_config, list_models  # noqa: F401
from .model import TransformerLM  # noqa: F401
