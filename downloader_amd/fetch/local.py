"""``file://`` source (reference ``methods.file``, lib/download.js:177-189).

Gated by ``ALLOW_FILE_URLS=true`` (config ``download.allow_file_urls``). The file is copied to
``<dir>/<name><ext>`` - in-kernel (``copy_file_range`` / ``sendfile`` via ``shutil``), never
through Python buffers.
"""
from __future__ import annotations

import os
import shutil
from urllib.parse import unquote, urlsplit


class FileUrlsNotAllowed(Exception):
    def __init__(self) -> None:
        super().__init__("File URLs are not allowed.")


def file_uri_to_path(uri: str) -> str:
    """``file-uri-to-path``: ``file:///a/b%20c`` -> ``/a/b c``; ``file://host/x`` -> ``//host/x``."""
    u = urlsplit(uri)
    if u.scheme != "file":
        raise ValueError(f"not a file URI: {uri}")
    host = u.netloc
    path = unquote(u.path)
    if host and host != "localhost":
        return "//" + host + path
    return path


def copy_file(src: str, dst: str) -> int:
    try:
        return _copy_range(src, dst)
    except OSError:
        shutil.copyfile(src, dst)
        return os.path.getsize(dst)


def _copy_range(src: str, dst: str) -> int:
    with open(src, "rb") as fi, open(dst, "wb") as fo:
        size = os.fstat(fi.fileno()).st_size
        done = 0
        while done < size:
            n = os.copy_file_range(fi.fileno(), fo.fileno(), size - done)
            if n == 0:
                break
            done += n
        if done != size:
            raise OSError("short copy")
        return done


def target_path(uri: str, download_dir: str) -> str:
    src = file_uri_to_path(uri)
    return os.path.join(download_dir, os.path.basename(src))
