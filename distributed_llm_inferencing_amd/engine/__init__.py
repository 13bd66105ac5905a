"""Engine layer: scheduler, paged KV cache, hipGraph runner, LLMEngine (lazy exports)."""
from .sequence import SamplingParams, RequestOutput  # noqa: F401


def __getattr__(name):
    if name == "LLMEngine":
        from .llm_engine import LLMEngine
        return LLMEngine
    raise AttributeError(name)
