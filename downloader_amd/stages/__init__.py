"""Plugin stage pipeline (reference lib/main.js:28-32,98-115).

Stages are resolved by name. Built-ins: ``download``, ``process``, ``upload``. A custom stage
is any ``"package.module:factory"`` string in ``config.stages``; its factory must be
``async (config, services) -> Stage`` and the loader enforces that the result is callable
(the reference's ``typeof fn !== 'function'`` check, lib/main.js:107-110).
"""
from __future__ import annotations

import importlib
from typing import Awaitable, Callable, Dict, List, Tuple

from .base import Services, Stage

Factory = Callable[..., Awaitable[Stage]]

BUILTIN = {
    "download": "downloader_amd.stages.download:factory",
    "process": "downloader_amd.stages.process:factory",
    "upload": "downloader_amd.stages.upload:factory",
}


class InvalidStage(Exception):
    pass


def resolve(name: str) -> Factory:
    target = BUILTIN.get(name, name)
    if ":" not in target:
        raise InvalidStage(f"Invalid stage '{name}': unknown stage")
    mod, attr = target.split(":", 1)
    return getattr(importlib.import_module(mod), attr)


async def build_stages(names: List[str], cfg, services: Services) -> List[Tuple[str, Stage]]:
    out: List[Tuple[str, Stage]] = []
    for name in names:
        fn = await resolve(name)(cfg, services)
        if not callable(fn):
            raise InvalidStage(f"Invalid stage '{name}' return value was not a function")
        out.append((name.split(":")[-1] if name not in BUILTIN else name, fn))
    return out


REGISTRY: Dict[str, str] = BUILTIN
