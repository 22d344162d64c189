"""Service discovery (the reference's ``triton-core/dynamics``).

``dyn('rabbitmq')`` returns the broker endpoint (lib/main.js:14,46,49). The upstream
implementation is not vendored; it is INFERRED to be env / Kubernetes-DNS driven. Lookup
order here: ``<SERVICE>_URL`` env, ``<SERVICE>_ENDPOINT`` env, Kubernetes service env
(``<SERVICE>_SERVICE_HOST``/``_PORT``), then a localhost default.
"""
from __future__ import annotations

import os
from typing import Mapping, Optional

DEFAULTS = {
    "rabbitmq": "amqp://guest:guest@127.0.0.1:5672/",
    "minio": "http://127.0.0.1:9000",
}
SCHEMES = {"rabbitmq": "amqp", "minio": "http"}


def dyn(service: str, env: Optional[Mapping[str, str]] = None) -> str:
    env = os.environ if env is None else env
    key = service.upper().replace("-", "_")
    for suffix in ("_URL", "_ENDPOINT"):
        v = env.get(key + suffix)
        if v:
            return v
    host = env.get(key + "_SERVICE_HOST")
    if host:
        port = env.get(key + "_SERVICE_PORT", "5672" if service == "rabbitmq" else "80")
        scheme = SCHEMES.get(service, "http")
        if scheme == "amqp":
            return f"amqp://guest:guest@{host}:{port}/"
        return f"{scheme}://{host}:{port}"
    return DEFAULTS.get(service, f"http://127.0.0.1/{service}")
