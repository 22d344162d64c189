"""S3 staging layout: object keys and the done marker.

Reference contract:
  * bucket ``triton-staging`` (lib/main.js:120, lib/upload.js:29-30)
  * object key ``path.join(mediaId, 'original/', base64(basename(file)))`` (lib/upload.js:43-45)
  * done marker ``path.join(mediaId, 'original/', 'done')`` with body ``"true"`` (lib/upload.js:55)

``path.join`` is Node's POSIX join, which normalises the result: repeated slashes collapse,
``.``/``..`` segments resolve and a trailing slash is kept. Standard base64 may contain ``/``
(and ``//``), so the normalisation is observable in the key and is
reproduced exactly here.
"""
from __future__ import annotations

import base64
import hashlib
import mimetypes
import os

STAGING_BUCKET = "triton-staging"
DONE_BODY = b"true"


def node_normalize(p: str) -> str:
    """POSIX ``path.normalize`` with Node semantics."""
    if p == "":
        return "."
    absolute = p.startswith("/")
    trailing = p.endswith("/")
    out: list[str] = []
    for seg in p.split("/"):
        if seg == "" or seg == ".":
            continue
        if seg == "..":
            if out and out[-1] != "..":
                out.pop()
            elif not absolute:
                out.append("..")
            continue
        out.append(seg)
    s = "/".join(out)
    if not s and not absolute:
        s = "."
    if s and trailing:
        s += "/"
    return ("/" + s) if absolute else s


def node_join(*parts: str) -> str:
    """POSIX ``path.join`` with Node semantics (empty segments dropped, then normalised)."""
    joined = "/".join(p for p in parts if p)
    return node_normalize(joined) if joined else "."


def b64_name(basename: str) -> str:
    """Standard-alphabet base64 of the UTF-8 basename (``Buffer.from(s).toString('base64')``)."""
    return base64.b64encode(basename.encode("utf-8")).decode("ascii")


def object_key(media_id: str, file_path: str) -> str:
    """``<id>/original/<b64(basename)>`` exactly as lib/upload.js:43-44 builds it."""
    return node_join(media_id, "original/", b64_name(os.path.basename(file_path)))


def done_key(media_id: str) -> str:
    return node_join(media_id, "original/", "done")


def originals_prefix(media_id: str) -> str:
    """Prefix of every staged original of a job (``object_key`` without the name)."""
    return node_join(media_id, "original/")


def journal_prefix(media_id: str) -> str:
    """Prefix of a job's relay resume journals (``relay_journal_key``)."""
    return node_join(media_id, ".stager/")


def relay_journal_key(media_id: str, file_path: str) -> str:
    """Resume journal of a streamed relay (``S3Client.relay_object(journal=)``): outside
    ``<id>/original/`` so nothing that lists the staged originals ever sees it."""
    return node_join(media_id, ".stager/", "relay-" + hashlib.sha1(
        os.path.basename(file_path).encode("utf-8")).hexdigest() + ".json")


# mime-db types of the media the selector keeps (lib/process.js:15-20): minio-js 7's
# fPutObject looks the Content-Type up from the file name with mime-types (yarn.lock:2162).
_MEDIA_TYPES = {".mkv": "video/x-matroska", ".mp4": "video/mp4", ".mov": "video/quicktime",
                ".webm": "video/webm"}
DEFAULT_CONTENT_TYPE = "application/octet-stream"


def content_type(file_path: str) -> str:
    """Content-Type minio-js would send for ``file_path`` (by extension, lower-cased)."""
    ext = os.path.splitext(file_path)[1].lower()
    if ext in _MEDIA_TYPES:
        return _MEDIA_TYPES[ext]
    return mimetypes.guess_type("x" + ext)[0] or DEFAULT_CONTENT_TYPE if ext else \
        DEFAULT_CONTENT_TYPE
