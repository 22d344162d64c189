"""Forward-proxy selection for HTTP *sources* (the reference's ``request@2`` semantics).

The reference downloads ``http``/``https`` media with ``request(url)`` (lib/download.js:160),
which honours the proxy environment by default: ``HTTP_PROXY``/``http_proxy`` for ``http:``
URLs, ``HTTPS_PROXY``/``https_proxy`` (falling back to the HTTP variables) for ``https:``, and
``NO_PROXY``/``no_proxy`` - a comma list of host names, domain suffixes (``.example.com`` or
``example.com``), optional ``:port``, or ``*`` for "never". Only that path uses a proxy:
minio-js (S3), webtorrent's simple-get (``.torrent`` fetches, webseeds, trackers) do not.

Deviation: in ``env`` mode loopback hosts (``localhost``, ``127.*``, ``::1``) are never
proxied (request@2 would proxy them unless listed in NO_PROXY).

``download.http_proxy`` picks the behaviour: ``env`` (default, as the reference), ``""``
(never) or an explicit ``http://[user:pass@]host:port`` URL for every source request.
Plain-http sources go to the proxy in absolute form (``GET http://host/path``) on the native
transport, so the stream relay still splices origin -> S3; https sources open a CONNECT
tunnel on the native transport and run TLS inside it (``HttpConn.connect_tunnel``).
"""
from __future__ import annotations

import base64
import os
from dataclasses import dataclass
from typing import Mapping, Optional
from urllib.parse import unquote, urlsplit


@dataclass(frozen=True)
class Proxy:
    url: str            # as configured (aiohttp takes it as is)
    host: str
    port: int
    auth: str = ""      # Proxy-Authorization value ("Basic ...") or ""

    @classmethod
    def parse(cls, url: str) -> "Proxy":
        if "://" not in url:
            url = "http://" + url                 # request accepts bare host:port too
        u = urlsplit(url)
        if u.scheme != "http" or not u.hostname:
            raise ValueError(f"unsupported proxy URL {url!r} (http://host:port expected)")
        auth = ""
        if u.username is not None:
            cred = f"{unquote(u.username)}:{unquote(u.password or '')}".encode()
            auth = "Basic " + base64.b64encode(cred).decode()
        clean = f"http://{u.hostname}:{u.port or 80}"
        return cls(url if auth else clean, u.hostname, u.port or 80, auth)


def _no_proxy(host: str, port: int, spec: str) -> bool:
    spec = spec.strip()
    if not spec:
        return False
    if spec == "*":
        return True
    host = host.lower()
    for item in spec.split(","):
        item = item.strip().lower()
        if not item:
            continue
        iport = None
        if item.count(":") == 1:
            item, _, p = item.partition(":")
            try:
                iport = int(p)
            except ValueError:
                continue
        if iport is not None and iport != port:
            continue
        dom = item.lstrip(".")
        if host == dom or host.endswith("." + dom):
            return True
    return False


def _loopback(host: str) -> bool:
    return host in ("localhost", "::1") or host.startswith("127.")


def proxy_from_env(url: str, env: Optional[Mapping[str, str]] = None) -> Optional[Proxy]:
    env = os.environ if env is None else env
    u = urlsplit(url)
    if _loopback((u.hostname or "").lower()):
        return None          # deliberate deviation from request@2: loopback never proxied
    port = u.port or (443 if u.scheme == "https" else 80)
    if _no_proxy(u.hostname or "", port, env.get("NO_PROXY", env.get("no_proxy", ""))):
        return None
    if u.scheme == "https":
        raw = (env.get("HTTPS_PROXY") or env.get("https_proxy") or env.get("HTTP_PROXY")
               or env.get("http_proxy"))
    elif u.scheme == "http":
        raw = env.get("HTTP_PROXY") or env.get("http_proxy")
    else:
        return None
    if not raw:
        return None
    try:
        return Proxy.parse(raw)
    except ValueError:
        return None


class ProxyConfig:
    """Per-URL proxy choice for source fetches (see module docstring)."""

    def __init__(self, setting: str = "env", env: Optional[Mapping[str, str]] = None):
        self.setting = (setting or "").strip()
        self.env = env
        self._fixed = None
        if self.setting and self.setting != "env":
            self._fixed = Proxy.parse(self.setting)

    def for_url(self, url: str) -> Optional[Proxy]:
        if not self.setting:
            return None
        if self._fixed is not None:
            return self._fixed
        return proxy_from_env(url, self.env)

    @property
    def active(self) -> bool:
        return bool(self.setting)


NO_PROXY = ProxyConfig("")
