"""Process-wide configuration read from environment variables.

Keeps every environment variable name the reference reads, with the same
semantics, and adds the MI355X-specific knobs of SURVEY.md §5.6:

reference (master, ``master/master/settings.py:8-101``):
    SECRET_KEY, DEBUG, REDIS_HOST, REDIS_PORT, REDIS_DB, MODEL_CACHE_DIR
reference (worker, ``worker/app.py:19-30``):
    MODEL_CACHE_DIR, USE_GPU, AUTH_ENABLED, AUTH_KEY

new:
    NUM_GPUS, PIPELINE_STAGES, DP_REPLICAS, DISPATCH_WORKERS, QUEUE_BACKEND (inproc|sqlite|redis),
    TRANSPORT (rccl|gloo|loopback), MAX_NEW_TOKENS, KV_CACHE_FRACTION,
    MASTER_DB, MAX_BATCH, DLI_FAULT (fault-injection spec, see utils/faults.py)
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from pathlib import Path

REPO_ROOT = Path(__file__).resolve().parent.parent
PKG_ROOT = Path(__file__).resolve().parent


def _env_bool(name: str, default: str = "0") -> bool:
    return os.environ.get(name, default).strip().lower() in ("1", "true", "yes", "on")


def _env_int(name: str, default: int) -> int:
    try:
        return int(os.environ.get(name, str(default)))
    except ValueError:
        return default


def _env_float(name: str, default: float) -> float:
    try:
        return float(os.environ.get(name, str(default)))
    except ValueError:
        return default


@dataclass
class Settings:
    # --- reference names (same defaults where they make sense off-Docker) ---
    secret_key: str = "dli-insecure-key-for-development-only"
    debug: bool = False
    redis_host: str = "redis"
    redis_port: int = 6379
    redis_db: int = 0
    model_cache_dir: str = str(REPO_ROOT / "model_cache")
    use_gpu: bool = False
    auth_enabled: bool = False
    auth_key: str = ""
    # --- new knobs ---
    num_gpus: int = 1
    pipeline_stages: int = 1
    dp_replicas: int = 1
    queue_backend: str = "inproc"
    transport: str = "rccl"
    max_new_tokens: int = 0          # 0 -> use the reference's max_length=100 rule
    max_length: int = 100            # reference default, prompt included (views.py:351)
    kv_cache_fraction: float = 0.85
    master_db: str = str(REPO_ROOT / "db.sqlite3")
    max_batch: int = 256
    # master dispatcher threads = requests in flight to workers (each blocks on one HTTP
    # call); a worker batches concurrent requests, so this bounds its decode batch
    dispatch_workers: int = 256
    log_dir: str = str(REPO_ROOT / "logs")
    fault: str = ""
    extra: dict = field(default_factory=dict)

    @classmethod
    def from_env(cls) -> "Settings":
        s = cls()
        s.secret_key = os.environ.get("SECRET_KEY", s.secret_key)
        s.debug = _env_bool("DEBUG", "0")
        s.redis_host = os.environ.get("REDIS_HOST", s.redis_host)
        s.redis_port = _env_int("REDIS_PORT", s.redis_port)
        s.redis_db = _env_int("REDIS_DB", s.redis_db)
        s.model_cache_dir = os.environ.get("MODEL_CACHE_DIR", s.model_cache_dir)
        s.use_gpu = _env_bool("USE_GPU", "0")
        s.auth_enabled = _env_bool("AUTH_ENABLED", "0")
        s.auth_key = os.environ.get("AUTH_KEY", "")
        s.num_gpus = _env_int("NUM_GPUS", s.num_gpus)
        s.pipeline_stages = _env_int("PIPELINE_STAGES", s.pipeline_stages)
        s.dp_replicas = _env_int("DP_REPLICAS", s.dp_replicas)
        s.queue_backend = os.environ.get("QUEUE_BACKEND", s.queue_backend)
        s.transport = os.environ.get("TRANSPORT", s.transport)
        s.max_new_tokens = _env_int("MAX_NEW_TOKENS", s.max_new_tokens)
        s.kv_cache_fraction = _env_float("KV_CACHE_FRACTION", s.kv_cache_fraction)
        s.master_db = os.environ.get("MASTER_DB", s.master_db)
        s.max_batch = _env_int("MAX_BATCH", s.max_batch)
        s.dispatch_workers = _env_int("DISPATCH_WORKERS", s.dispatch_workers)
        s.log_dir = os.environ.get("DLI_LOG_DIR", s.log_dir)
        s.fault = os.environ.get("DLI_FAULT", "")
        return s


def get_settings() -> Settings:
    """Fresh read of the environment (cheap; lets tests monkeypatch env)."""
    return Settings.from_env()
